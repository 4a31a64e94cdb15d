#!/bin/bash
# Sharded-step A/B of the batched scale's grid (CBN_SCALE_BLOCKS_PER_CU):
# tools/ab_scale.sh 1 2 4 ...  -> bench.py --sharded (N = 1 over a one-rank RCCL
# communicator), two rounds, per-step time and the raw launch's HIP-event time
set -u
export CBN_DIAG=1  # diagnostic CBN_* switches count only under CBN_DIAG=1 (round 5)
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
for round in 1 2; do
for v in "$@"; do
  CBN_SCALE_BLOCKS_PER_CU=$v timeout -k 10 300 python bench.py --sharded --no-cpu-baseline --steps 400 > gpurun_out/abs_$v.log 2>&1 || exit $?
  python -c "
import json; d=json.loads(open('gpurun_out/abs_$v.log').read().strip().splitlines()[-1])
print('blocks/CU $v', round(d['value']/1e9, 3), 'G q/s', round(d['ms_per_step']*1e3, 2), 'us/step; raw launch', d['roofline']['avg_us'], 'us; gathered', round(d.get('value_gathered', 0)/1e9, 3))"
done
done
