#!/bin/bash
# Round 4: k_param_query part swizzle A/B + k_query_cols compact records
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/r04q
export TMPDIR=/tmp
O=gpurun_out/r04q
timeout -k 10 900 python -u -m pytest tests/test_gpu_param.py tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log
[ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  timeout -k 10 300 python3 tools/bench_alarm.py > $O/alarm_$r.log 2>&1 || exit $?
  grep '^{' $O/alarm_$r.log | cut -c1-120
done
ALARM=1 timeout -k 10 300 python3 tools/stamp_probe.py > $O/stamps_cols.txt 2>&1 || exit $?
sed -n 2,12p $O/stamps_cols.txt
timeout -k 10 900 bash tools/ab_param.sh "swz:base:" "nosw:nosw:" > $O/ab.txt 2>&1 || exit $?
cat $O/ab.txt
