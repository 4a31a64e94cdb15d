#!/bin/bash
# Round 4: the full GPU suite + smoke + default bench, as the driver runs them
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/r04h
export TMPDIR=/tmp
O=gpurun_out/r04h
timeout -k 10 1500 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
tail -4 $O/pytest_gpu.log
grep -c PASSED $O/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
tail -1 $O/smoke.log
timeout -k 10 300 python3 bench.py > $O/bench_default.json 2> $O/bench_default.err || exit $?
python3 -c "import json; d=json.loads(open('$O/bench_default.json').read().strip().splitlines()[-1]); print(round(d['value']/1e9,3), 'G q/s', d['timing']['itemised'])"
