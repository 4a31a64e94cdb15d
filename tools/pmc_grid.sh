#!/bin/bash
# PMC of the configs[4] grid kernel (tools/bench_grid.py --profile: 65 536
# queries, 10 calls), one rocprofv3 --pmc pass per counter group; then
# tools/pmc_table.py over the passes.  OUT= subdirectory of gpurun_out.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/${OUT:-pmc_grid}; mkdir -p $O; export TMPDIR=/tmp
i=0
for counters in \
  "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY" \
  "SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_BUSY_CYCLES SQ_ACTIVE_INST_LDS SQ_INSTS_SMEM SQ_WAVES" \
  "TCC_HIT_sum TCC_MISS_sum" \
  "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum"; do
  i=$((i + 1))
  timeout -s KILL 120 rocprofv3 --pmc $counters -d $O/p$i -o run --output-format csv -- python3 tools/bench_grid.py --profile > $O/p$i.log 2>&1 || exit $?
done
python3 tools/pmc_table.py $O/p1 $O/p2 $O/p3 $O/p4 | tee $O/pmc_table.txt
rm -rf $O/p1 $O/p2 $O/p3 $O/p4  # the per-dispatch CSVs exceed what gpurun copies back
