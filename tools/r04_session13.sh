#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/r04n
export TMPDIR=/tmp
O=gpurun_out/r04n
timeout -k 10 300 python3 tools/host_steps.py 5 20 > $O/host_steps.txt 2>&1 || exit $?
python3 -c "
import json
for l in open('$O/host_steps.txt'):
    if l.startswith('{'):
        d=json.loads(l); print(d['variant'], 'first', d['steps_us'][0], 'rest', round(sum(d['steps_us'][1:])/19,2), 'wall', d['wall_us_per_step'], 'region', d['region_us_per_step'])
"
