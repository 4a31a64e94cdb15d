#!/bin/bash
# One parameterised GPU session (round 6: also absorbs the one-off A/B,
# profiling and PMC scripts of rounds 1-5).  Run on the GPU box through gpurun:
#
#   OUT=r06a tools/session.sh pytest smoke driver3 bench alarm cont grid
#
# Steps (in the order given; the session stops at the first failure, so a
# fault or time limit ends it and nothing more touches the GPU):
#   pytest        the GPU suite (PYTEST_K / PYTEST_FILES narrow it; PYTEST_X= runs past failures)
#   smoke         __graft_entry__.smoke()
#   driverN       the driver's bench command (--gpus 1 --steps 20 --warmup 5), N times
#   bench         python bench.py (default: 200 steps, the CPU baseline)
#   sharded       bench.py --sharded --no-cpu-baseline (the N>1 step over a one-rank communicator)
#   alarm|cont|grid|chain16|direct   tools/bench_<name>.py (configs[2] / [3] / [4], N = 16 chain,
#                 direct plans; BENCH_ARGS passes arguments)
#   prof          rocprofv3 --kernel-trace --stats of the driver's command
#   fetch|write   one rocprofv3 --pmc FETCH_SIZE (WRITE_SIZE) pass of bench.py --steps 40 (HBM traffic)
#   summary       tools/profile_summary.py over prof / fetch / write -> profiles/$TAG_*
#   pmcNAME       one rocprofv3 --pmc pass of the driver's command with the counters in $PMC_NAME
#   profcfg       rocprofv3 --kernel-trace --stats of tools/bench_{alarm,cont,grid}.py ($CONFIGS)
#   pmcgrid       the configs[4] kernel's SQ / TCC / TCP counters, four passes, tools/pmc_table.py
#   pmcparam      the parametric query kernel's SQ counters (tools/prof_param.py $PROF_ARGS)
#   stamps        tools/stamp_probe.py (per-wave phase stamps; needs libcbn_amd_stamps.so)
#   ab            same-box A/B on tools/bench_$AB_BENCH.py (default grid), two rounds, over the
#                 arms in AB_ARMS: "name:ENV=V,ENV2=V" (environment knobs) or "name:lib=<variant>"
#                 (continuousbayesiannetwork_amd/libcbn_amd_<variant>.so, built by
#                 tools/build_variant.sh); "base" = the in-tree library, no knobs
# Diagnostic kernel-selection variables (CBN_NO_STAGED, ...) and CBN_LIB_PATH
# count only under CBN_DIAG=1 (include/cbn_amd.h cbn_diag_enabled;
# _native.lib_path); the ab / stamps steps set it themselves.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/${OUT:-session}
mkdir -p "$O"
line() {  # summary of a bench JSON line
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d.get('roofline') or {}; print(sys.argv[2], round(d['value']/1e9,3), 'G q/s', round(d['ms_per_step']*1e3,2), 'us/step', r.get('avg_us'), 'us/launch', r.get('frac'), (d.get('timing') or {}).get('itemised',''))" "$1" "$2"
}
kstats() {  # our kernels' rows of a rocprofv3 kernel_stats CSV
  python3 - "$1" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    name = r["Name"].replace("void (anonymous namespace)::", "")
    if name.startswith("k_"):
        print(name.split("(")[0][:70], r["Calls"], round(float(r["AverageNs"]) / 1000, 2), "us avg",
              round(float(r["MinNs"]) / 1000, 2), "us min")
PY
}
for step in "$@"; do
  case $step in
    pytest)
      timeout -k 10 1100 python -u -m pytest ${PYTEST_FILES:-tests} -m gpu ${PYTEST_X--x} -q --timeout 300 --timeout-method thread \
        ${PYTEST_K:+-k "$PYTEST_K"} > $O/pytest_gpu.log 2>&1; rc=$?
      tail -3 $O/pytest_gpu.log
      [ $rc -eq 0 ] || exit $rc ;;
    smoke)
      timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
      tail -1 $O/smoke.log ;;
    driver*)
      n=${step#driver}; n=${n:-1}
      for i in $(seq 1 $n); do
        timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/driver_$i.json 2> $O/driver_$i.err || exit $?
        line $O/driver_$i.json "driver $i"
      done ;;
    bench)
      timeout -k 10 300 python3 bench.py > $O/bench_default.json 2> $O/bench_default.err || exit $?
      line $O/bench_default.json default ;;
    sharded)
      timeout -k 10 300 python3 bench.py --sharded --no-cpu-baseline > $O/bench_sharded.json 2> $O/bench_sharded.err || exit $?
      line $O/bench_sharded.json sharded ;;
    alarm|cont|grid|chain16|direct)
      timeout -k 10 600 python3 tools/bench_$step.py ${BENCH_ARGS:-} > $O/$step.log 2>&1 || exit $?
      grep '^{' $O/$step.log | cut -c1-400 ;;
    prof)
      timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --gpus 1 \
        --steps 20 --warmup 5 > $O/prof_bench.json 2> $O/prof_bench.err || exit $?
      rm -f $O/prof/run_kernel_trace.csv
      kstats $O/prof/run_kernel_stats.csv ;;
    fetch|write)
      c=FETCH_SIZE; [ $step = write ] && c=WRITE_SIZE
      timeout -s KILL 120 rocprofv3 --pmc $c --kernel-trace -d $O/pmc_$step -o run --output-format csv -- python3 bench.py \
        --steps 40 --warmup 4 --no-cpu-baseline > $O/pmc_$step.json 2> $O/pmc_$step.err || exit $? ;;
    summary)
      timeout -k 10 120 python3 tools/profile_summary.py --tag "${TAG:-r06}" --prof $O/prof --fetch $O/pmc_fetch \
        --write $O/pmc_write --warmup 5 --steps 20 --command "rocprofv3 --kernel-trace --stats -- python3 bench.py --gpus 1 --steps 20 --warmup 5 (PMC: separate --pmc FETCH_SIZE / WRITE_SIZE passes, --steps 40)" \
        > $O/summary.log 2>&1 || exit $?
      cp profiles/${TAG:-r06}_summary.json profiles/${TAG:-r06}_kernel_stats.csv $O/  # (gpurun copies gpurun_out back)
      tail -5 $O/summary.log ;;
    pmc*)
      name=${step#pmc}
      case $name in
        grid)
          i=0
          for counters in \
            "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY" \
            "SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_BUSY_CYCLES SQ_ACTIVE_INST_LDS SQ_INSTS_SMEM SQ_WAVES" \
            "TCC_HIT_sum TCC_MISS_sum" \
            "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum"; do
            i=$((i + 1))
            timeout -s KILL 120 rocprofv3 --pmc $counters -d $O/pg$i -o run --output-format csv -- python3 tools/bench_grid.py \
              --profile > $O/pg$i.log 2>&1 || exit $?
          done
          python3 tools/pmc_table.py $O/pg1 $O/pg2 $O/pg3 $O/pg4 | tee $O/pmc_grid_table.txt
          rm -rf $O/pg1 $O/pg2 $O/pg3 $O/pg4 ;;  # the per-dispatch CSVs exceed what gpurun copies back
        param)
          K='--kernel-include-regex k_param'
          timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/pp_stats -o run --output-format csv -- python3 \
            tools/prof_param.py ${PROF_ARGS:-} > $O/pp_stats.log 2>&1 || exit $?
          timeout -s KILL 120 rocprofv3 $K --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVE_CYCLES \
            SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU -d /tmp/pp_pmc1 -o run --output-format csv -- python3 \
            tools/prof_param.py ${PROF_ARGS:-} > $O/pp_pmc1.log 2>&1 || exit $?
          timeout -s KILL 120 rocprofv3 $K --pmc SQ_INSTS_VMEM SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_SCA \
            SQ_INST_CYCLES_SALU SQ_ACTIVE_INST_LDS SQ_INSTS_LDS SQ_ACTIVE_INST_MISC -d /tmp/pp_pmc2 -o run \
            --output-format csv -- python3 tools/prof_param.py ${PROF_ARGS:-} > $O/pp_pmc2.log 2>&1 || exit $?
          python3 tools/pmc_summary.py --kernel k_param_query --out $O/pmc_param.json /tmp/pp_stats /tmp/pp_pmc1 /tmp/pp_pmc2 ;;
        *)
          var=PMC_$name; counters=${!var}
          timeout -s KILL 120 rocprofv3 --pmc $counters -d $O/pmc_$name -o run -- python3 bench.py --gpus 1 --steps 20 \
            --warmup 5 --no-cpu-baseline > $O/pmc_$name.json 2> $O/pmc_$name.err || exit $?
          find $O/pmc_$name -name "*counter_collection.csv" | head -2 ;;
      esac ;;
    profcfg)
      for n in ${CONFIGS:-alarm cont grid}; do
        args=""; [ $n = grid ] && args="--profile"
        timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof_$n -o run --output-format csv -- python3 \
          tools/bench_$n.py $args > $O/prof_$n.log 2>&1 || exit $?
        rm -f $O/prof_$n/run_kernel_trace.csv
        echo "== $n"; kstats $O/prof_$n/run_kernel_stats.csv
      done ;;
    ab)  # same-box A/B, two rounds
      for r in 1 2; do
        for spec in ${AB_ARMS:-base}; do
          IFS=: read -r v knobs <<< "$spec"
          envs="CBN_DIAG=1"
          case $knobs in
            lib=*) envs="$envs CBN_LIB_PATH=$PWD/continuousbayesiannetwork_amd/libcbn_amd_${knobs#lib=}.so" ;;
            ?*) envs="$envs ${knobs//,/ }" ;;
          esac
          env $envs timeout -k 10 600 python3 tools/bench_${AB_BENCH:-grid}.py ${BENCH_ARGS:-} > $O/ab_${v}_$r.log 2>&1 || exit $?
          grep '^{' $O/ab_${v}_$r.log | cut -c1-300 | sed "s/^/$v $r /"
        done
      done ;;
    stamps)
      CBN_DIAG=1 timeout -k 10 300 python3 tools/stamp_probe.py > $O/stamps.log 2>&1 || exit $?
      tail -20 $O/stamps.log ;;
    *) echo "session.sh: unknown step $step" >&2; exit 2 ;;
  esac
done
