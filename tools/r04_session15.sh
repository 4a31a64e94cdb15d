#!/bin/bash
# Round 4: wave -> factor-part swizzle in k_param_query -- param GPU tests,
# same-box A/B against the unswizzled build (CBN_NO_PART_SWIZZLE)
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/r04p
export TMPDIR=/tmp
O=gpurun_out/r04p
timeout -k 10 900 python -u -m pytest tests/test_gpu_param.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 900 bash tools/ab_param.sh "swz:base:" "nosw:nosw:" > $O/ab.txt 2>&1 || exit $?
cat $O/ab.txt
