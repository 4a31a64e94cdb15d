# Counters for the parametric query kernel (tools/prof_param.py), one --pmc pass
# each, summarised on the box (raw traces of the training kernels are large).
set -u
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out
ARGS=${PROF_ARGS:-}
K='--kernel-include-regex k_param'
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/pp_stats -o run --output-format csv -- python3 tools/prof_param.py $ARGS > gpurun_out/pp_stats.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 $K --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU -d /tmp/pp_pmc1 -o run --output-format csv -- python3 tools/prof_param.py $ARGS > gpurun_out/pp_pmc1.log 2>&1 || exit 2
timeout -s KILL 120 rocprofv3 $K --pmc SQ_INSTS_VMEM SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_SALU SQ_ACTIVE_INST_LDS SQ_INSTS_LDS SQ_ACTIVE_INST_MISC -d /tmp/pp_pmc2 -o run --output-format csv -- python3 tools/prof_param.py $ARGS > gpurun_out/pp_pmc2.log 2>&1 || exit 3
python3 tools/pmc_summary.py --kernel k_param_query --out gpurun_out/pp_summary.json /tmp/pp_stats /tmp/pp_pmc1 /tmp/pp_pmc2
