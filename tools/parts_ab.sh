set -u
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/r05j; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_param.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; tail -2 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for v in 3 4 6; do
    CBN_DIAG=1 CBN_PARAM_PARTS=$v timeout -k 10 300 python3 tools/bench_cont.py --est lr --queries 131072 1048576 > $O/parts_${v}_$r.log 2>&1 || exit $?
    grep '^{' $O/parts_${v}_$r.log | python3 -c "import sys,json; [print('parts $v r$r', d['queries'], d['us_per_call'], d['pdf_sha256']) for d in map(json.loads, sys.stdin)]"
  done
  CBN_LIB_PATH=$PWD/continuousbayesiannetwork_amd/libcbn_amd_pold.so timeout -k 10 300 python3 tools/bench_cont.py --est lr --queries 131072 1048576 > $O/pold_$r.log 2>&1 || exit $?
  grep '^{' $O/pold_$r.log | python3 -c "import sys,json; [print('pold r$r', d['queries'], d['us_per_call'], d['pdf_sha256']) for d in map(json.loads, sys.stdin)]"
done
