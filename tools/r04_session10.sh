#!/bin/bash
# Round 4: the one-rank sharded bench paths (rank-local and gathered) and the
# driver's command after the start-event change
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/r04k
export TMPDIR=/tmp
O=gpurun_out/r04k
timeout -k 10 300 python3 bench.py --sharded --steps 100 --warmup 10 > $O/sharded.json 2> $O/sharded.err || exit $?
tail -1 $O/sharded.json | cut -c1-1500
timeout -k 10 300 python3 bench.py --sharded --gather --steps 100 --warmup 10 > $O/sharded_gather.json 2> $O/sharded_gather.err || exit $?
tail -1 $O/sharded_gather.json | cut -c1-600
for i in 1 2 3; do
  timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/d_$i.json 2> $O/d_$i.err || exit $?
  python3 -c "import json; d=json.loads(open('$O/d_$i.json').read().strip().splitlines()[-1]); print(round(d['value']/1e9,3), 'G q/s', d['timing']['itemised'])"
done
