#!/bin/bash
# phase stamps of the fused kernel, paired vs padded table layout
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 300 python tools/stamp_probe.py > gpurun_out/stamps_paired.log 2>&1 || exit $?
CBN_NO_PAIRED=1 timeout -k 10 300 python tools/stamp_probe.py > gpurun_out/stamps_nopaired.log 2>&1 || exit $?
