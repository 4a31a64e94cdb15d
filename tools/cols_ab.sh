#!/bin/bash
# configs[2] (k_query_cols) A/B: the in-tree library (base), base with
# CBN_COLS_NO_SPLIT=1 (under CBN_DIAG), and libcbn_amd_old.so; X35 / X36
# (tools/bench_alarm.py) and the N = 16 chain (tools/bench_chain16.py), two
# rounds; GPU parity of the base library first
set -u
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/${OUT:-cols_ab}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_api.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; tail -2 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for v in base nosplit old; do
    case $v in base) e="CBN_X=0";; nosplit) e="CBN_DIAG=1 CBN_COLS_NO_SPLIT=1";; old) e="CBN_LIB_PATH=$PWD/continuousbayesiannetwork_amd/libcbn_amd_old.so";; esac
    for b in alarm chain16; do
      env $e timeout -k 10 600 python3 tools/bench_$b.py > $O/${b}_${v}_$r.log 2>&1 || exit $?
      grep '^{' $O/${b}_${v}_$r.log | python3 -c "import sys,json; [print('$v r$r $b', d.get('target', d.get('queries')), d.get('queries'), d['us_per_call'], d.get('plan_flags')) for d in map(json.loads, sys.stdin)]"
    done
  done
done
