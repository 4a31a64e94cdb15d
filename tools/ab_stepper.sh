#!/bin/bash
# Same-box A/B of the sharded step (tools/comm_probe.py steady-state rounds):
# folded scales vs the separate batched scale (new: 1 block/CU, 8 float4 per
# thread in flight; old: 4 blocks/CU, one float4 per thread)
set -u
export CBN_DIAG=1  # diagnostic CBN_* switches count only under CBN_DIAG=1 (round 5)
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export MASTER_ADDR=127.0.0.1 MASTER_PORT=29533
L=$PWD/continuousbayesiannetwork_amd
for round in 1 2; do
  timeout -k 10 300 python tools/comm_probe.py fold=True > gpurun_out/abst_fold.log 2>&1 || exit $?
  grep "round [3-5]" gpurun_out/abst_fold.log | sed 's/^/fold  /'
  timeout -k 10 300 python tools/comm_probe.py fold=False > gpurun_out/abst_new.log 2>&1 || exit $?
  grep "round [3-5]" gpurun_out/abst_new.log | sed 's/^/scale-new  /'
  CBN_LIB_PATH=$L/libcbn_amd_scaleold.so CBN_SCALE_BLOCKS_PER_CU=4 timeout -k 10 300 python tools/comm_probe.py fold=False > gpurun_out/abst_old.log 2>&1 || exit $?
  grep "round [3-5]" gpurun_out/abst_old.log | sed 's/^/scale-old  /'
done
