#!/bin/bash
# Round 4, final tree: the full GPU suite, smoke, the driver's bench command
# (x3), the default bench, and the configs[2] / [3] / [4] benches
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/${OUT:-r04z}
export TMPDIR=/tmp
O=gpurun_out/${OUT:-r04z}
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
tail -2 $O/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
tail -1 $O/smoke.log
for i in 1 2 3; do
  timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/driver_$i.json 2> $O/driver_$i.err || exit $?
  python3 -c "import json; d=json.loads(open('$O/driver_$i.json').read().strip().splitlines()[-1]); print(round(d['value']/1e9,3), 'G q/s', d['timing']['itemised'])"
done
timeout -k 10 300 python3 bench.py > $O/bench_default.json 2> $O/bench_default.err || exit $?
python3 -c "import json; d=json.loads(open('$O/bench_default.json').read().strip().splitlines()[-1]); print('default', round(d['value']/1e9,3), 'G q/s', d['roofline']['avg_us'], 'us', d['roofline']['frac'])"
timeout -k 10 300 python3 tools/bench_alarm.py > $O/alarm.log 2>&1 || exit $?
grep '^{' $O/alarm.log
timeout -k 10 600 python3 tools/bench_cont.py > $O/cont.log 2>&1 || exit $?
grep '^{' $O/cont.log | cut -c1-300
timeout -k 10 600 python3 tools/bench_grid.py > $O/grid.log 2>&1 || exit $?
grep '^{' $O/grid.log | cut -c1-300
