#!/bin/bash
# Sharded-step A/B: folded scales (default) vs the separate batched scale
# (--no-fold), bench.py --sharded (N = 1 over a one-rank RCCL communicator),
# two rounds; then a kernel trace of the folded run.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for round in 1 2; do
for v in fold nofold; do
  extra=""; [ $v = nofold ] && extra="--no-fold"
  timeout -k 10 300 python bench.py --sharded --no-cpu-baseline --steps 400 $extra > gpurun_out/abf_$v.log 2>&1 || exit $?
  python -c "
import json; d=json.loads(open('gpurun_out/abf_$v.log').read().strip().splitlines()[-1])
print('$v', round(d['value']/1e9, 3), 'G q/s', round(d['ms_per_step']*1e3, 2), 'us/step; raw launch', d['roofline']['avg_us'], 'us; step', d['sharded_step']['avg_us'], 'us')"
done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_fold -o run --output-format csv -- python3 bench.py --sharded --no-cpu-baseline --steps 200 > gpurun_out/prof_fold.log 2>&1 || exit $?
