#!/bin/bash
# Round 4: configs[2] after the k_query_cols record change -- rocprofv3 kernel
# trace + stats, one SQ PMC pass, for the current library and the previous one
# (libcbn_amd_old.so: tools/build_variant.sh old, built from the tree before
# that change)
set -u
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/r04p
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_alarm -o run --output-format csv -- python3 tools/bench_alarm.py > $O/prof_alarm.log 2>&1 || exit $?
grep '^{' $O/prof_alarm.log | cut -c1-100
find $O/prof_alarm -name "*kernel_stats.csv" -exec cp {} $O/alarm_kernel_stats.csv \;
grep -h "k_query" $O/alarm_kernel_stats.csv | cut -c1-60,200-400
for v in new old; do
  if [ $v = new ]; then e="CBN_X=0"; else e="CBN_LIB_PATH=continuousbayesiannetwork_amd/libcbn_amd_old.so"; fi
  env $e timeout -s KILL 120 rocprofv3 --pmc SQ_WAIT_INST_ANY SQ_INSTS_VMEM SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_ANY SQ_BUSY_CYCLES SQ_INSTS_SALU --kernel-trace -d $O/pmc_sq_$v -o run --output-format csv -- python3 tools/bench_alarm.py > $O/pmc_sq_$v.log 2>&1 || exit $?
  python3 tools/pmc_summary.py --kernel k_query_cols --out $O/pmc_cols_$v.json $O/pmc_sq_$v || exit $?
  rm -rf $O/pmc_sq_$v
done
head -40 $O/pmc_cols_new.json
head -40 $O/pmc_cols_old.json
rm -rf $O/prof_alarm
echo done
