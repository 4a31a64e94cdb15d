#!/bin/bash
# Round 4: linear weights carried by the prefetched factor header (PHead::lw)
# -- parametric GPU tests, then same-box A/B against the previous library
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/r04o
export TMPDIR=/tmp
O=gpurun_out/r04o
timeout -k 10 900 python -u -m pytest tests/test_gpu_param.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 900 bash tools/ab_param.sh "new:base:" "old:old:" > $O/ab.txt 2>&1 || exit $?
cat $O/ab.txt
