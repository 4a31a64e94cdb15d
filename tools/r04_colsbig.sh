#!/bin/bash
# Round 4: diagnostic k_query_cols for plans of up to 128 factors and any lanes
# per query (libcbn_amd_big.so: tools/build_variant.sh big -DCBN_COLS_BIG) on
# the configs[4] grid (L = 8) and configs[2], against the default library
set -u
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/r04g
mkdir -p $O
export TMPDIR=/tmp
B="CBN_LIB_PATH=continuousbayesiannetwork_amd/libcbn_amd_big.so"
env $B timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "grid or alarm or config2 or config4" --timeout 300 --timeout-method thread > $O/pytest_big.log 2>&1; rc=$?
tail -2 $O/pytest_big.log
[ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for v in new big; do
    if [ $v = big ]; then e="$B"; else e="CBN_X=0"; fi
    env $e timeout -k 10 600 python3 tools/bench_grid.py > $O/grid_${v}_$r.log 2>&1 || exit $?
    grep '^{' $O/grid_${v}_$r.log | python3 -c "import sys,json; [print('grid $v $r', d['queries'], d['us_per_call'], d.get('plan_flags')) for d in map(json.loads, sys.stdin)]"
    env $e timeout -k 10 300 python3 tools/bench_alarm.py > $O/alarm_${v}_$r.log 2>&1 || exit $?
    grep '^{' $O/alarm_${v}_$r.log | python3 -c "import sys,json; [print('alarm $v $r', d['target'], d['us_per_call'], d['plan_flags']) for d in map(json.loads, sys.stdin)]"
  done
done
