#!/bin/bash
# Round 4: configs[2] with one float4 per lane (CBN_FAST_VPL=1: 2 lanes per
# query, twice the waves) against the default (2 float4 per lane), same box,
# two rounds each
set -u
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/r04v
mkdir -p $O
export TMPDIR=/tmp
for r in 1 2; do
  for v in default vpl1; do
    if [ $v = vpl1 ]; then e="CBN_FAST_VPL=1"; else e="CBN_X=0"; fi
    env $e timeout -k 10 300 python3 tools/bench_alarm.py > $O/${v}_$r.log 2>&1 || exit $?
    grep '^{' $O/${v}_$r.log | python3 -c "import sys,json; [print('$v', '$r', d['target'], d['us_per_call'], d['plan_flags'], d['fused_capacity']) for d in map(json.loads, sys.stdin)]"
  done
done
