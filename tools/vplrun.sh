#!/bin/bash
# A/B of the fast kernel's float4 chunks per lane (CBN_FAST_VPL) + phase stamps.
set -e
export CBN_DIAG=1  # diagnostic CBN_* switches count only under CBN_DIAG=1 (round 5)
cd "${GRAFT_REPO_ROOT:-.}"
for v in 1 2; do
  echo "VPL=$v"; CBN_FAST_VPL=$v timeout -k 10 300 python bench.py --no-cpu-baseline --steps 100 2>&1 | grep value | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['roofline']['avg_us'], d['roofline']['max_pass_us'], d.get('value_rebuild_tables'))"
done
CBN_FAST_VPL=2 timeout -k 10 300 python tools/stamp_probe.py
