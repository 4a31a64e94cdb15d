#!/bin/bash
# Round 5: k_query_slots with the survivor chain (base) vs without (libcbn_amd_slots1.so)
# vs k_query_fast (CBN_NO_SLOTS=1 under CBN_DIAG); grid parity first
set -u
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/${OUT:-r05o}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_direct.py tests/test_gpu_api.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; tail -2 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for v in chain slots1 fast; do
    case $v in chain) e="CBN_X=0";; slots1) e="CBN_LIB_PATH=$PWD/continuousbayesiannetwork_amd/libcbn_amd_slots1.so";; fast) e="CBN_DIAG=1 CBN_NO_SLOTS=1";; esac
    env $e timeout -k 10 600 python3 tools/bench_grid.py --headline > $O/grid_${v}_$r.log 2>&1 || exit $?
    grep '^{' $O/grid_${v}_$r.log | python3 -c "import sys,json; [print('$v r$r', d['queries'], d['us_per_call'], d['plan_flags'], d['nonzero_frac']) for d in map(json.loads, sys.stdin)]"
  done
done
