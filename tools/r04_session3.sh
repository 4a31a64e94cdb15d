#!/bin/bash
# Round 4, third GPU session: the native Runner host path -- GPU parity/API
# tests, host-step diagnostics, the driver's bench command x2, steps 200.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/r04c
export TMPDIR=/tmp
O=gpurun_out/r04c
timeout -k 10 900 python -u -m pytest tests/test_gpu_api.py tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k "not x99" > $O/pytest.log 2>&1; rc=$?
tail -5 $O/pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 tools/host_steps.py 5 20 > $O/host_steps.txt 2>&1 || exit $?
cut -c1-400 $O/host_steps.txt
for i in 1 2 3; do
  timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/driver_$i.json 2> $O/driver_$i.err || exit $?
  python3 -c "import json; d=json.loads(open('$O/driver_$i.json').read().strip().splitlines()[-1]); print(round(d['value']/1e9,3), 'G q/s', d['ms_per_step']*1e3, 'us/step', d['timing']['itemised'])"
done
timeout -k 10 300 python3 bench.py --gpus 1 --steps 200 --warmup 20 --no-cpu-baseline > $O/steps200.json 2> $O/steps200.err || exit $?
python3 -c "import json; d=json.loads(open('$O/steps200.json').read().strip().splitlines()[-1]); print(round(d['value']/1e9,3), 'G q/s', d['ms_per_step']*1e3, 'us/step', d['timing']['itemised'])"
