#!/bin/bash
# Round 4, second GPU session: host-step diagnostics,
# configs[2] k_query_cols under rocprofv3 (kernel trace + PMC passes, VERDICT
# item 4), the N = 16 (L = 2) cols/fast A/B, the VALU issue-rate probe.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/r04b
export TMPDIR=/tmp
O=gpurun_out/r04b
timeout -k 10 300 python3 tools/host_steps.py 5 20 > $O/host_steps.txt 2>&1 || exit $?
cat $O/host_steps.txt | cut -c1-600
timeout -k 10 120 ./tools/probes/valu_rate > $O/valu_rate.txt 2>&1 || exit $?
cat $O/valu_rate.txt
for r in 1 2; do
  timeout -k 10 300 python3 tools/bench_chain16.py > $O/chain16_cols_$r.log 2>&1 || exit $?
  CBN_NO_COLS=1 timeout -k 10 300 python3 tools/bench_chain16.py > $O/chain16_fast_$r.log 2>&1 || exit $?
  echo cols; grep '^{' $O/chain16_cols_$r.log; echo fast; grep '^{' $O/chain16_fast_$r.log
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_alarm -o run --output-format csv -- python3 tools/bench_alarm.py > $O/prof_alarm.log 2>&1 || exit $?
grep '^{' $O/prof_alarm.log
find $O/prof_alarm -name "*kernel_stats.csv" -exec grep -h "k_query" {} \;
timeout -s KILL 120 rocprofv3 --pmc SQ_WAIT_INST_ANY SQ_INSTS_VMEM SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_ANY SQ_BUSY_CYCLES SQ_INSTS_SALU --kernel-trace -d $O/pmc_alarm_sq -o run --output-format csv -- python3 tools/bench_alarm.py > $O/pmc_alarm_sq.log 2>&1 || exit $?
CBN_NO_COLS=1 timeout -s KILL 120 rocprofv3 --pmc SQ_WAIT_INST_ANY SQ_INSTS_VMEM SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_ANY SQ_BUSY_CYCLES SQ_INSTS_SALU --kernel-trace -d $O/pmc_alarm_sq_fast -o run --output-format csv -- python3 tools/bench_alarm.py > $O/pmc_alarm_sq_fast.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-trace -d $O/pmc_alarm_tcc -o run --output-format csv -- python3 tools/bench_alarm.py > $O/pmc_alarm_tcc.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $O/pmc_alarm_fetch -o run --output-format csv -- python3 tools/bench_alarm.py > $O/pmc_alarm_fetch.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $O/pmc_alarm_write -o run --output-format csv -- python3 tools/bench_alarm.py > $O/pmc_alarm_write.log 2>&1 || exit $?
python3 tools/pmc_summary.py --kernel k_query_cols --out $O/pmc_alarm_cols.json $O/pmc_alarm_sq $O/pmc_alarm_tcc $O/pmc_alarm_fetch $O/pmc_alarm_write || exit $?
python3 tools/pmc_summary.py --kernel k_query_fast --out $O/pmc_alarm_fast.json $O/pmc_alarm_sq_fast || exit $?
cat $O/pmc_alarm_cols.json $O/pmc_alarm_fast.json | head -80
find $O/prof_alarm -name "*kernel_stats.csv" -exec cp {} $O/alarm_kernel_stats.csv \;
rm -rf $O/pmc_alarm_sq $O/pmc_alarm_sq_fast $O/pmc_alarm_tcc $O/pmc_alarm_fetch $O/pmc_alarm_write $O/prof_alarm
echo done
