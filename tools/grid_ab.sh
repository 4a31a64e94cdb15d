#!/bin/bash
# configs[4] grid A/B of library variants: tools/grid_ab.sh name1 name2 ...
# ("base" = the default library, else continuousbayesiannetwork_amd/libcbn_amd_<name>.so);
# grid / golden GPU parity of the default library first, then two rounds of
# tools/bench_grid.py --headline per variant (65 536 and 262 144 queries)
set -u
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/${OUT:-grid_ab}; mkdir -p $O; export TMPDIR=/tmp
if [ -z "${NO_PYTEST:-}" ]; then
  timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_direct.py tests/test_gpu_api.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; tail -2 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
fi
for r in 1 2; do
  for v in "$@"; do
    if [ $v = base ]; then lib=$PWD/continuousbayesiannetwork_amd/libcbn_amd.so; else lib=$PWD/continuousbayesiannetwork_amd/libcbn_amd_$v.so; fi
    CBN_LIB_PATH=$lib timeout -k 10 600 python3 tools/bench_grid.py --headline > $O/grid_${v}_$r.log 2>&1 || exit $?
    grep '^{' $O/grid_${v}_$r.log | python3 -c "import sys,json; [print('$v r$r', d['queries'], d['us_per_call'], d['plan_flags'], d['nonzero_frac'], d.get('pdf_sha256', '')[:12]) for d in map(json.loads, sys.stdin)]"
  done
done
