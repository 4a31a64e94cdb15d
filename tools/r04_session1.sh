#!/bin/bash
# Round 4, first GPU session: parity of the column-staged kernel (k_query_cols),
# configs[2] A/B cols vs fast (same box, two rounds), then the driver's exact
# bench command plain / under rocprofv3.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/r04
export TMPDIR=/tmp
O=gpurun_out/r04
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_api.py tests/test_gpu_direct.py -m gpu -x -q --timeout 300 --timeout-method thread -k "not x99" > $O/pytest_parity.log 2>&1; rc=$?
tail -5 $O/pytest_parity.log
[ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  timeout -k 10 300 python tools/bench_alarm.py > $O/alarm_cols_$r.log 2>&1 || exit $?
  tail -2 $O/alarm_cols_$r.log
  CBN_NO_COLS=1 timeout -k 10 300 python tools/bench_alarm.py > $O/alarm_fast_$r.log 2>&1 || exit $?
  tail -2 $O/alarm_fast_$r.log
done
timeout -k 10 300 python tools/bench_grid.py > $O/grid_cols.log 2>&1 || exit $?
tail -2 $O/grid_cols.log
CBN_NO_COLS=1 timeout -k 10 300 python tools/bench_grid.py > $O/grid_fast.log 2>&1 || exit $?
tail -2 $O/grid_fast.log
timeout -k 10 120 ./tools/probes/valu_rate > $O/valu_rate.txt 2>&1 || exit $?
cat $O/valu_rate.txt
timeout -k 10 600 bash tools/ab_param.sh "base:base:" "unpk:unpk:" > $O/ab_param.txt 2>&1 || exit $?
cat $O/ab_param.txt
bash tools/r04_driver_cmd.sh
