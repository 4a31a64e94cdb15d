#!/bin/bash
# A/B of library variants on the headline bench: tools/ab_libs.sh name1 name2 ...
# (name "base" = the default library; else continuousbayesiannetwork_amd/libcbn_amd_<name>.so);
# kernel-only rocprof average of k_query_staged<2> per variant + the bench's HIP-event
# launch time (no profiler), two rounds
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for round in 1 2; do
for v in "$@"; do
  if [ $v = base ]; then lib=$PWD/continuousbayesiannetwork_amd/libcbn_amd.so; else lib=$PWD/continuousbayesiannetwork_amd/libcbn_amd_$v.so; fi
  CBN_LIB_PATH=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/ab_$v -o run --output-format csv -- python3 bench.py --no-cpu-baseline --steps 200 > gpurun_out/ab_$v.log 2>&1 || exit $?
  python - <<PY
import csv, glob
f = sorted(glob.glob("gpurun_out/ab_$v/**/*kernel_stats.csv", recursive=True))[0]
for r in csv.DictReader(open(f)):
    if "k_query_staged<2>" in r["Name"]:
        print("$v", "avg", round(float(r["AverageNs"]) / 1000, 2), "us  min", round(float(r["MinNs"]) / 1000, 2))
PY
  rm -rf gpurun_out/ab_$v
  CBN_LIB_PATH=$lib timeout -k 10 300 python bench.py --no-cpu-baseline --steps 400 > gpurun_out/abb_$v.log 2>&1 || exit $?
  python -c "import json; d=json.loads(open('gpurun_out/abb_$v.log').read().strip().splitlines()[-1]); print('$v', 'bench', round(d['value']/1e9, 3), 'G q/s', d['roofline']['avg_us'], 'us/launch (HIP events)')"
done
done
