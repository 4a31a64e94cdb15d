#!/bin/bash
# Round 4: configs[2] cols kernel with software-pipelined offsets -- parity
# (alarm + grid + random DAG table cases), bench (x2), stamps
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/r04g
export TMPDIR=/tmp
O=gpurun_out/r04g
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log
[ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  timeout -k 10 300 python3 tools/bench_alarm.py > $O/alarm_$r.log 2>&1 || exit $?
  grep '^{' $O/alarm_$r.log
done
timeout -k 10 300 python3 tools/bench_chain16.py > $O/chain16.log 2>&1 || exit $?
grep '^{' $O/chain16.log
ALARM=1 timeout -k 10 300 python3 tools/stamp_probe.py > $O/stamps_cols.txt 2>&1 || exit $?
head -14 $O/stamps_cols.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_alarm -o run --output-format csv -- python3 tools/bench_alarm.py > $O/prof_alarm.log 2>&1 || exit $?
find $O/prof_alarm -name "*kernel_stats.csv" -exec cp {} $O/alarm_kernel_stats.csv \;
find $O/prof_alarm -name "*kernel_trace.csv" -exec cp {} $O/alarm_kernel_trace.csv \;
rm -rf $O/prof_alarm
grep k_query $O/alarm_kernel_stats.csv
