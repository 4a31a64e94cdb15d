#!/bin/bash
# GPU-box session runner: each step under its own timeout; stops at the first
# fault-like exit (abort/segv/timeout/kill) so nothing else touches the GPU.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out
mkdir -p "$OUT"
export TMPDIR=/tmp
step() {
  local name=$1 t=$2; shift 2
  echo "== $name ($(date +%T))"
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"
  tail -n 15 "$OUT/$name.log"
  case $rc in
    0|1|5) return 0 ;;
    *) echo "fatal rc=$rc in $name: stopping the session"; exit "$rc" ;;
  esac
}
for s in "$@"; do
  case $s in
    pytest) step pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread ;;
    smoke) step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) step bench 600 python bench.py ;;
    benchfast) step bench 600 python bench.py --no-cpu-baseline ;;
    benchcold) step bench_cold 600 python bench.py --no-cpu-baseline --rebuild-tables ;;
    prof) step rocprof_stats 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- python3 bench.py --no-cpu-baseline ;;
    pmc) step pmc_fetch 600 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d "$OUT/pmc_fetch" -o run --output-format csv -- python3 bench.py --steps 40 --warmup 4 --no-cpu-baseline &&
         step pmc_write 600 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d "$OUT/pmc_write" -o run --output-format csv -- python3 bench.py --steps 40 --warmup 4 --no-cpu-baseline ;;
    summary) step summary 120 python tools/profile_summary.py --tag "${TAG:-r01}" --command "rocprofv3 --kernel-trace --stats -- python3 bench.py --no-cpu-baseline (PMC: separate --pmc FETCH_SIZE / WRITE_SIZE passes, --steps 40)" ;;
    stepper) step pytest_stepper 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "stepper or raw_launch" --timeout 120 --timeout-method thread ;;
    probe) step shard_probe 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29517 tools/shard_step_probe.py ;;
    benchsharded) step bench_sharded 300 python bench.py --no-cpu-baseline --sharded ;;
    profsharded) step rocprof_sharded 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof_sharded" -o run --output-format csv -- python3 bench.py --no-cpu-baseline --sharded ;;
    bench2) step bench_n2 600 python bench.py --gpus 2 --no-cpu-baseline ;;
    benchserial) step bench_serial 300 python bench.py --no-cpu-baseline --sharded --serial-exchange ;;
    torchrun1) step bench_torchrun1 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29518 bench.py --gpus 1 --no-cpu-baseline ;;
    param) step pytest_param 400 python -u -m pytest tests/test_gpu_param.py -m gpu -x -q --timeout 120 --timeout-method thread ;;
    cont) step bench_cont 400 python tools/bench_cont.py ;;
    alarm) step bench_alarm 400 python tools/bench_alarm.py ;;
    direct) step bench_direct 400 python tools/bench_direct.py ;;
    newtests) step pytest_new 400 python -u -m pytest tests/test_gpu_api.py tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "redrawn or rebinds or stepper" ;;
    grid) step bench_grid 600 python tools/bench_grid.py ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
echo "session done"
