#!/bin/bash
# phase stamps of the fused kernel, paired vs padded table layout
set -u
export CBN_DIAG=1  # diagnostic CBN_* switches count only under CBN_DIAG=1 (round 5)
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 300 python tools/stamp_probe.py > gpurun_out/stamps_paired.log 2>&1 || exit $?
CBN_NO_PAIRED=1 timeout -k 10 300 python tools/stamp_probe.py > gpurun_out/stamps_nopaired.log 2>&1 || exit $?
