#!/bin/bash
# A/B of the paired LDS table layout (CBN_NO_PAIRED=1 = padded rows) + LDS PMC of both
set -u
export CBN_DIAG=1  # diagnostic CBN_* switches count only under CBN_DIAG=1 (round 5)
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in paired nopaired; do
  if [ $v = nopaired ]; then export CBN_NO_PAIRED=1; else unset CBN_NO_PAIRED; fi
  timeout -k 10 300 python bench.py --no-cpu-baseline --steps 400 > gpurun_out/ab_$v.log 2>&1 || exit $?
  python -c "import json,sys; d=json.loads(open('gpurun_out/ab_$v.log').read().strip().splitlines()[-1]); print('$v', d['value']/1e9, d['ms_per_step']*1e3, d['roofline']['avg_us'])"
  timeout -k 10 300 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAVES --kernel-trace -d gpurun_out/pmc_$v -o run --output-format csv -- python3 bench.py --steps 40 --warmup 4 --no-cpu-baseline > gpurun_out/pmc_$v.log 2>&1 || exit $?
done
