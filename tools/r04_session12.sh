#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/r04m
export TMPDIR=/tmp
O=gpurun_out/r04m
for a in "--no-fold --skip-other" "--gather --skip-other"; do
  timeout -k 10 300 python3 bench.py --sharded --steps 200 --warmup 20 $a > $O/s.json 2> $O/s.err || exit $?
  python3 -c "import json; d=json.loads(open('$O/s.json').read().strip().splitlines()[-1]); print('$a', d['value_kind'], round(d['value']/1e9,3), 'G q/s', d['timing'])"
done
