#!/bin/bash
# One parameterised GPU session (replaces round 4's 25 one-off
# tools/r04_*.sh scripts).  Run on the GPU box through gpurun:
#
#   OUT=r05a tools/session.sh pytest smoke driver3 bench alarm cont grid
#
# Steps (in the order given; the session stops at the first failure, so a
# fault or time limit ends it and nothing more touches the GPU):
#   pytest        the GPU suite (PYTEST_K / PYTEST_FILES narrow it)
#   smoke         __graft_entry__.smoke()
#   driverN       the driver's bench command (--gpus 1 --steps 20 --warmup 5), N times
#   bench         python bench.py (default: 200 steps, the CPU baseline)
#   sharded       bench.py --sharded --no-cpu-baseline (the N>1 step over a one-rank communicator)
#   alarm|cont|grid|chain16|direct   tools/bench_<name>.py (configs[2] / [3] / [4], N = 16 chain, direct plans)
#   prof          rocprofv3 --kernel-trace --stats of the driver's command
#   pmcNAME       one rocprofv3 --pmc pass of the driver's command with the counters in $PMC_NAME
#   stamps        tools/stamp_probe.py (per-wave phase stamps, configs[1])
#   ab            A/B of library variants (AB_LIBS="base old", libcbn_amd_<name>.so built by
#                 tools/build_variant.sh) on tools/bench_$AB_BENCH.py (default grid), two rounds
# Diagnostic kernel-selection variables (CBN_NO_STAGED, ...) need CBN_DIAG=1
# in the environment of the session (include/cbn_amd.h, cbn_diag_enabled).
set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/${OUT:-session}
mkdir -p "$O"
line() {  # summary of a bench JSON line
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d.get('roofline') or {}; print(sys.argv[2], round(d['value']/1e9,3), 'G q/s', round(d['ms_per_step']*1e3,2), 'us/step', r.get('avg_us'), 'us/launch', r.get('frac'), (d.get('timing') or {}).get('itemised',''))" "$1" "$2"
}
for step in "$@"; do
  case $step in
    pytest)
      timeout -k 10 1100 python -u -m pytest ${PYTEST_FILES:-tests} -m gpu -x -q --timeout 300 --timeout-method thread \
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
      timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 bench.py --gpus 1 --steps 20 \
        --warmup 5 > $O/prof_bench.json 2> $O/prof_bench.err || exit $?
      find $O/prof -name "*kernel_stats.csv" | head -2 ;;
    pmc*)
      name=${step#pmc}; var=PMC_$name; counters=${!var}
      timeout -s KILL 120 rocprofv3 --pmc $counters -d $O/pmc_$name -o run -- python3 bench.py --gpus 1 --steps 20 \
        --warmup 5 --no-cpu-baseline > $O/pmc_$name.json 2> $O/pmc_$name.err || exit $?
      find $O/pmc_$name -name "*counter_collection.csv" | head -2 ;;
    ab)  # same-box A/B of library variants on tools/bench_$AB_BENCH.py, two rounds (base = the in-tree library)
      for r in 1 2; do
        for v in ${AB_LIBS:-base old}; do
          if [ $v = base ]; then lib=$PWD/continuousbayesiannetwork_amd/libcbn_amd.so
          else lib=$PWD/continuousbayesiannetwork_amd/libcbn_amd_$v.so; fi
          CBN_LIB_PATH=$lib timeout -k 10 600 python3 tools/bench_${AB_BENCH:-grid}.py ${BENCH_ARGS:-} \
            > $O/ab_${v}_$r.log 2>&1 || exit $?
          grep '^{' $O/ab_${v}_$r.log | cut -c1-300 | sed "s/^/$v $r /"
        done
      done ;;
    stamps)
      timeout -k 10 300 python3 tools/stamp_probe.py > $O/stamps.log 2>&1 || exit $?
      tail -20 $O/stamps.log ;;
    *) echo "session.sh: unknown step $step" >&2; exit 2 ;;
  esac
done
