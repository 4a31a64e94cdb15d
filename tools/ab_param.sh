#!/bin/bash
# A/B of library variants / launch knobs on the parametric bench (configs[3]):
# tools/ab_param.sh "name:lib:ENV=V ..." ...   (lib "base" = the default library,
# else continuousbayesiannetwork_amd/libcbn_amd_<lib>.so), two rounds
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for round in 1 2; do
for spec in "$@"; do
  IFS=: read -r name lib envs <<< "$spec"
  if [ "$lib" = base ]; then p=$PWD/continuousbayesiannetwork_amd/libcbn_amd.so; else p=$PWD/continuousbayesiannetwork_amd/libcbn_amd_$lib.so; fi
  env CBN_LIB_PATH=$p $envs timeout -k 10 300 python tools/bench_cont.py > gpurun_out/abp_$name.log 2>&1 || exit $?
  python - "$name" <<'PY'
import json, sys
rows = [json.loads(l) for l in open(f"gpurun_out/abp_{sys.argv[1]}.log") if l.startswith("{")]
print(sys.argv[1], "  ".join(f"{r['estimator'][:2]}@{r['queries']}: {r['us_per_call']}" for r in rows), flush=True)
PY
done
done
