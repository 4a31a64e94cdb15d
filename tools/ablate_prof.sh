#!/bin/bash
# kernel-only durations (rocprofv3 --kernel-trace --stats) of the phase-ablation builds
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in base NOPROD NOBAR NOSTAGE NODMA ALL; do
  if [ $v = base ]; then lib=$PWD/continuousbayesiannetwork_amd/libcbn_amd.so; else lib=$PWD/continuousbayesiannetwork_amd/libcbn_amd_abl_$v.so; fi
  CBN_LIB_PATH=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/ablp_$v -o run --output-format csv -- python3 bench.py --no-cpu-baseline --steps 200 > gpurun_out/ablp_$v.log 2>&1 || exit $?
  python - <<PY
import csv, glob
f = sorted(glob.glob("gpurun_out/ablp_$v/**/*kernel_stats.csv", recursive=True))[0]
for r in csv.DictReader(open(f)):
    if "k_query_staged<2>" in r["Name"]:
        print("$v", "avg", round(float(r["AverageNs"]) / 1000, 2), "us  min", round(float(r["MinNs"]) / 1000, 2))
PY
done
