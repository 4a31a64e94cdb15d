#!/bin/bash
# Round 4, fourth GPU session: the X99 free-parent pin, the driver's exact
# command under rocprofv3 (itemised timeline), the headline profile + PMC
# traffic refresh (profiles/r04_*).
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/r04d
export TMPDIR=/tmp
O=gpurun_out/r04d
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k "free_parent" > $O/pytest_fp.log 2>&1; rc=$?
tail -3 $O/pytest_fp.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_driver -o run --output-format csv -- python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/driver_prof.json 2> $O/driver_prof.err || exit $?
python3 tools/driver_timeline.py $O/prof_driver $O/driver_prof.json $O/driver_timeline.json || exit $?
find $O/prof_driver -name "*kernel_stats.csv" -exec cp {} $O/driver_kernel_stats.csv \;
rm -rf $O/prof_driver
for i in 1 2; do
  timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/driver_$i.json 2> $O/driver_$i.err || exit $?
  python3 -c "import json; d=json.loads(open('$O/driver_$i.json').read().strip().splitlines()[-1]); print(round(d['value']/1e9,3), 'G q/s', d['timing']['itemised'])"
done
run() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; tail -n 2 "gpurun_out/$name.log"; [ $rc -eq 0 ] || exit $rc; }
run prof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --no-cpu-baseline
run pmc_fetch 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/pmc_fetch -o run --output-format csv -- python3 bench.py --steps 40 --warmup 4 --no-cpu-baseline
run pmc_write 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d gpurun_out/pmc_write -o run --output-format csv -- python3 bench.py --steps 40 --warmup 4 --no-cpu-baseline
run summary 120 python tools/profile_summary.py --tag r04 --command "rocprofv3 --kernel-trace --stats -- python3 bench.py --no-cpu-baseline (PMC: separate --pmc FETCH_SIZE / WRITE_SIZE passes, --steps 40)"
cp profiles/r04_kernel_stats.csv profiles/r04_summary.json $O/
rm -rf gpurun_out/prof gpurun_out/pmc_fetch gpurun_out/pmc_write
