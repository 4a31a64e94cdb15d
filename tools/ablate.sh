#!/bin/bash
# phase ablation of the staged fused kernel: bench with diagnostic builds that
# skip one phase each (outputs are wrong by construction; timing only)
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
for v in base NOPROD NOBAR NOSTAGE NODMA ALL; do
  if [ $v = base ]; then unset CBN_LIB_PATH; else export CBN_LIB_PATH=$PWD/continuousbayesiannetwork_amd/libcbn_amd_abl_$v.so; fi
  timeout -k 10 300 python bench.py --no-cpu-baseline --steps 400 > gpurun_out/abl_$v.log 2>&1 || exit $?
  python -c "import json; d=json.loads(open('gpurun_out/abl_$v.log').read().strip().splitlines()[-1]); print('$v', round(d['ms_per_step']*1e3,2), 'us/step', d['roofline']['avg_us'], 'us/launch')"
done
