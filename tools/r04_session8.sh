#!/bin/bash
# Round 4: is the timed-region kernel slow-down a kernel-argument placement
# effect?  The driver's command with HIP_FORCE_DEV_KERNARG unset / 1 / 0
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/r04i
export TMPDIR=/tmp
O=gpurun_out/r04i
for v in unset 1 0 unset 1 0; do
  if [ $v = unset ]; then envs=""; else envs="HIP_FORCE_DEV_KERNARG=$v"; fi
  env $envs timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $O/d_$v.json 2> $O/d_$v.err || exit $?
  python3 -c "import json; d=json.loads(open('$O/d_$v.json').read().strip().splitlines()[-1]); print('$v', round(d['value']/1e9,3), 'G q/s', d['timing']['itemised'])"
done
for v in unset 1; do
  if [ $v = unset ]; then envs=""; else envs="HIP_FORCE_DEV_KERNARG=$v"; fi
  env $envs timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_$v -o run --output-format csv -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $O/dp_$v.json 2> $O/dp_$v.err || exit $?
  python3 tools/driver_timeline.py $O/prof_$v $O/dp_$v.json $O/timeline_$v.json | cut -c1-700 || exit $?
  rm -rf $O/prof_$v
done
