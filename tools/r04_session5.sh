#!/bin/bash
# Round 4: the driver's bench command after the timed-region prologue change (x3)
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/r04e
export TMPDIR=/tmp
O=gpurun_out/r04e
for i in 1 2 3; do
  timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/driver_$i.json 2> $O/driver_$i.err || exit $?
  python3 -c "import json; d=json.loads(open('$O/driver_$i.json').read().strip().splitlines()[-1]); print(round(d['value']/1e9,3), 'G q/s', d['timing']['itemised'])"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_driver -o run --output-format csv -- python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/driver_prof.json 2> $O/driver_prof.err || exit $?
python3 tools/driver_timeline.py $O/prof_driver $O/driver_prof.json $O/driver_timeline.json || exit $?
rm -rf $O/prof_driver
