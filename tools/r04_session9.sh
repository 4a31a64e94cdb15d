#!/bin/bash
# Round 4: first-touch A/B of the evidence batches on the driver's command
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/r04j
export TMPDIR=/tmp
O=gpurun_out/r04j
for v in touch notouch w64 touch notouch w64; do
  case $v in touch) a="--warmup 5";; notouch) a="--warmup 5 --no-touch";; w64) a="--warmup 64 --no-touch";; esac
  timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 $a --no-cpu-baseline > $O/d_$v.json 2> $O/d_$v.err || exit $?
  python3 -c "import json; d=json.loads(open('$O/d_$v.json').read().strip().splitlines()[-1]); print('$v', round(d['value']/1e9,3), 'G q/s', d['timing']['itemised'])"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $O/dp.json 2> $O/dp.err || exit $?
python3 tools/driver_timeline.py $O/prof $O/dp.json $O/timeline.json | cut -c1-700 || exit $?
rm -rf $O/prof
