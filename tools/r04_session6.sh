#!/bin/bash
# Round 4: phase stamps of the configs[2] kernel, k_query_cols vs k_query_fast
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/r04f
export TMPDIR=/tmp
O=gpurun_out/r04f
ALARM=1 timeout -k 10 300 python3 tools/stamp_probe.py > $O/stamps_cols.txt 2>&1 || exit $?
cat $O/stamps_cols.txt
ALARM=1 CBN_NO_COLS=1 timeout -k 10 300 python3 tools/stamp_probe.py > $O/stamps_fast.txt 2>&1 || exit $?
cat $O/stamps_fast.txt
