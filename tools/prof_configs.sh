#!/bin/bash
# rocprofv3 --kernel-trace --stats of the secondary configs' bench scripts
# (configs[2] alarm, configs[3] cont, configs[4] grid --profile), one run each
# (CONFIGS="alarm cont grid" by default); the kernel_stats CSVs land in
# gpurun_out/$OUT/<name>/
set -u
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/${OUT:-prof_configs}; mkdir -p $O; export TMPDIR=/tmp
for n in ${CONFIGS:-alarm cont grid}; do
  args=""; [ $n = grid ] && args="--profile"
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/$n -o run --output-format csv -- python3 tools/bench_$n.py $args > $O/$n.log 2>&1 || exit $?
  rm -f $O/$n/run_kernel_trace.csv
  python3 - "$O/$n/run_kernel_stats.csv" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    name = r["Name"].replace("void (anonymous namespace)::", "")
    if name.startswith("k_"):
        print(name.split("(")[0][:70], r["Calls"], round(float(r["AverageNs"]) / 1000, 2), "us avg", round(float(r["MinNs"]) / 1000, 2), "us min")
PY
done
