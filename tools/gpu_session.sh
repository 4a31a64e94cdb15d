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
    pytest) step pytest_gpu 900 python -m pytest tests -m gpu -x -q ;;
    smoke) step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) step bench 600 python bench.py ;;
    benchfast) step bench 600 python bench.py --no-cpu-baseline ;;
    benchcold) step bench_cold 600 python bench.py --no-cpu-baseline --rebuild-tables ;;
    prof) step rocprof_stats 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- python3 bench.py --no-cpu-baseline ;;
    pmc) step pmc_fetch 600 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d "$OUT/pmc_fetch" -o run --output-format csv -- python3 bench.py --steps 40 --warmup 4 --no-cpu-baseline &&
         step pmc_write 600 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d "$OUT/pmc_write" -o run --output-format csv -- python3 bench.py --steps 40 --warmup 4 --no-cpu-baseline ;;
    summary) step summary 120 python tools/profile_summary.py --tag "${TAG:-r01}" --command "rocprofv3 --kernel-trace --stats -- python3 bench.py --no-cpu-baseline (PMC: separate --pmc FETCH_SIZE / WRITE_SIZE passes, --steps 40)" ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
echo "session done"
