#!/bin/bash
# SQ counters of the headline kernel (one rocprofv3 --pmc pass per group)
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=${TAG:-sq}
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY --kernel-trace -d gpurun_out/pmc_${tag}1 -o run --output-format csv -- python3 bench.py --steps 40 --warmup 4 --no-cpu-baseline > gpurun_out/pmc_${tag}1.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_BUSY_CYCLES SQ_ACTIVE_INST_LDS SQ_INSTS_SMEM --kernel-trace -d gpurun_out/pmc_${tag}2 -o run --output-format csv -- python3 bench.py --steps 40 --warmup 4 --no-cpu-baseline > gpurun_out/pmc_${tag}2.log 2>&1 || exit $?
