#!/bin/bash
# Headline-kernel diagnostics on the GPU box: launch-ramp probe, per-wave phase
# stamps (libcbn_amd_stamps.so) and the phase-ablation builds' kernel times.
# Build first (here, on the CPU): tools/build_variant.sh stamps -DCBN_STAMPS,
# tools/build_variant.sh abl_<X> -DCBN_ABL_<X> ..., hipcc tools/probes/ramp.hip.
set -u
export CBN_DIAG=1  # diagnostic CBN_* switches count only under CBN_DIAG=1 (round 5)
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 tools/probes/ramp > gpurun_out/diag_ramp.log 2>&1 || exit $?
cat gpurun_out/diag_ramp.log
timeout -k 10 300 python tools/stamp_probe.py > gpurun_out/diag_stamps.log 2>&1 || exit $?
cat gpurun_out/diag_stamps.log
bash tools/ablate_prof.sh
