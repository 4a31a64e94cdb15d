#!/bin/bash
# Round 4: prespin A/B on the driver's command (same box, alternating, x4)
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/r04r
export TMPDIR=/tmp
O=gpurun_out/r04r
for r in 1 2 3 4; do
  for v in spin nospin; do
    a=""; [ $v = nospin ] && a="--no-prespin"
    timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline $a > $O/d_${v}_$r.json 2> $O/d_$v.err || exit $?
    python3 -c "import json; d=json.loads(open('$O/d_${v}_$r.json').read().strip().splitlines()[-1]); print('$v', round(d['value']/1e9,3), d['timing']['itemised'][:120])"
  done
done
