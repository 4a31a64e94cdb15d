#!/bin/bash
# Round 4: stepper hot path -- API/stepper GPU tests, the one-rank sharded bench
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/r04l
export TMPDIR=/tmp
O=gpurun_out/r04l
timeout -k 10 900 python -u -m pytest tests/test_gpu_api.py tests/test_gpu_direct.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "stepper or sharded or fold or raw" > $O/pytest_st.log 2>&1; rc=$?
tail -3 $O/pytest_st.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 bench.py --sharded --steps 100 --warmup 10 --no-fold > $O/sharded_ring.json 2> $O/sharded_ring.err || exit $?
python3 -c "import json; d=json.loads(open('$O/sharded_ring.json').read().strip().splitlines()[-1]); print(d['value_kind'], round(d['value']/1e9,3), 'G q/s; other', {k: v for k, v in d.items() if k.startswith('value_')}, d['timing'])"
timeout -k 10 300 python3 bench.py --sharded --gather --steps 100 --warmup 10 > $O/sharded_gather.json 2> $O/sharded_gather.err || exit $?
python3 -c "import json; d=json.loads(open('$O/sharded_gather.json').read().strip().splitlines()[-1]); print(d['value_kind'], round(d['value']/1e9,3), 'G q/s; other', {k: v for k, v in d.items() if k.startswith('value_')}, d['timing'])"
