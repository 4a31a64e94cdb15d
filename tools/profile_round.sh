#!/bin/bash
# Round profile session: the headline (fused N = 1) and the sharded step
# (--sharded, N = 1 over a one-rank communicator), each with a
# --kernel-trace --stats run and separate FETCH_SIZE / WRITE_SIZE PMC passes,
# condensed into profiles/<TAG>_*.  Usage: TAG=r03 tools/profile_round.sh
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r03}
run() {  # name seconds cmd...
  local name=$1 t=$2; shift 2
  echo "== $name ($(date +%T))"
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"; tail -n 3 "gpurun_out/$name.log"
  [ $rc -eq 0 ] || exit $rc
}
run prof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --no-cpu-baseline
run pmc_fetch 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/pmc_fetch -o run --output-format csv -- python3 bench.py --steps 40 --warmup 4 --no-cpu-baseline
run pmc_write 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d gpurun_out/pmc_write -o run --output-format csv -- python3 bench.py --steps 40 --warmup 4 --no-cpu-baseline
run summary 120 python tools/profile_summary.py --tag $TAG --command "rocprofv3 --kernel-trace --stats -- python3 bench.py --no-cpu-baseline (PMC: separate --pmc FETCH_SIZE / WRITE_SIZE passes, --steps 40)"
run prof_sh 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_sh -o run --output-format csv -- python3 bench.py --no-cpu-baseline --sharded
run pmc_sh_fetch 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/pmc_sh_fetch -o run --output-format csv -- python3 bench.py --steps 200 --warmup 4 --no-cpu-baseline --sharded --skip-other
run pmc_sh_write 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d gpurun_out/pmc_sh_write -o run --output-format csv -- python3 bench.py --steps 200 --warmup 4 --no-cpu-baseline --sharded --skip-other
run summary_sh 120 python tools/profile_summary.py --tag ${TAG}_sharded --prof gpurun_out/prof_sh --fetch gpurun_out/pmc_sh_fetch --write gpurun_out/pmc_sh_write --command "rocprofv3 --kernel-trace --stats -- python3 bench.py --no-cpu-baseline --sharded (PMC: separate --pmc FETCH_SIZE / WRITE_SIZE passes, --steps 200 --warmup 4 --skip-other: 204 raw launches, the first 16 without a fold)"
run bench_final 600 python bench.py
run bench_sharded_final 300 python bench.py --sharded --no-cpu-baseline
echo "session done"
