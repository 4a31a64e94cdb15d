#!/bin/bash
# Round 5: k_query_slots raw-launch grid (1 or 2 blocks per CU of words/grid, CBN_SLOTS_BPC under CBN_DIAG) vs k_query_fast
set -u
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/${OUT:-r05m}; mkdir -p $O; export TMPDIR=/tmp
for r in 1 2; do
  for v in bpc1 bpc2 fast; do
    case $v in bpc1) e="CBN_X=0";; bpc2) e="CBN_DIAG=1 CBN_SLOTS_BPC=2";; fast) e="CBN_DIAG=1 CBN_NO_SLOTS=1";; esac
    env $e timeout -k 10 600 python3 tools/bench_grid.py --headline > $O/grid_${v}_$r.log 2>&1 || exit $?
    grep '^{' $O/grid_${v}_$r.log | python3 -c "import sys,json; [print('$v r$r', d['queries'], d['us_per_call'], d['plan_flags'], d['nonzero_frac']) for d in map(json.loads, sys.stdin)]"
  done
done
