#!/bin/bash
# Round 4: k_query_cols with scalar (readlane) records and LDS/global row
# paths vs the previous library (libcbn_amd_old.so, tools/build_variant.sh
# old), same box: parity first, then alternating configs[2] / chain16 benches
set -u
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/r04c
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_api.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -2 $O/pytest.log
[ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for v in ${VARIANTS:-new old}; do
    if [ $v = new ]; then e="CBN_X=0"; else e="CBN_LIB_PATH=continuousbayesiannetwork_amd/libcbn_amd_$v.so"; fi
    env $e timeout -k 10 300 python3 tools/bench_alarm.py > $O/alarm_${v}_$r.log 2>&1 || exit $?
    grep '^{' $O/alarm_${v}_$r.log | python3 -c "import sys,json; [print('alarm $v $r', d['target'], d['us_per_call'], d['plan_flags']) for d in map(json.loads, sys.stdin)]"
    env $e timeout -k 10 300 python3 tools/bench_chain16.py > $O/c16_${v}_$r.log 2>&1 || exit $?
    grep '^{' $O/c16_${v}_$r.log | cut -c1-160 | sed "s/^/c16 $v $r /"
  done
done
