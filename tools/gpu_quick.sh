#!/bin/bash
# quick GPU iteration: parity subset, bench, stamps
set -u
export CBN_DIAG=1  # diagnostic CBN_* switches count only under CBN_DIAG=1 (round 5)
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/quick_pytest.log 2>&1; rc=$?
tail -3 gpurun_out/quick_pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 400 > gpurun_out/quick_bench.log 2>&1 || exit $?
python -c "import json; d=json.loads(open('gpurun_out/quick_bench.log').read().strip().splitlines()[-1]); print('bench', d['value']/1e9, 'G q/s', d['ms_per_step']*1e3, 'us/step', d['roofline']['avg_us'], 'us/launch')"
CBN_NO_STAGED=1 timeout -k 10 300 python bench.py --no-cpu-baseline --steps 400 > gpurun_out/quick_bench_nostaged.log 2>&1 || exit $?
python -c "import json; d=json.loads(open('gpurun_out/quick_bench_nostaged.log').read().strip().splitlines()[-1]); print('nostaged', d['value']/1e9, 'G q/s', d['ms_per_step']*1e3, 'us/step', d['roofline']['avg_us'], 'us/launch')"
timeout -k 10 300 python tools/stamp_probe.py > gpurun_out/quick_stamps.log 2>&1 || exit $?
cat gpurun_out/quick_stamps.log
