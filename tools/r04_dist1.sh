#!/bin/bash
# Round 4: the torch.distributed branches of bench.py at world size 1 (the
# driver's launch form with one rank): default, the gathered step, the
# rank-local step, fold off -- each one JSON line, checked for value_kind
set -u
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/r04d
mkdir -p $O
export TMPDIR=/tmp
run() {
  local name=$1; shift
  timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
    --master-port 29531 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline "$@" > $O/$name.json 2> $O/$name.err || exit $?
  python3 -c "import json; d=json.loads(open('$O/$name.json').read().strip().splitlines()[-1]); print('$name', round(d['value']/1e9,3), 'G q/s', d.get('value_kind'), d['config'].get('parallelism'))"
}
run plain
run sharded_gather --sharded --gather
run sharded_local --sharded
run sharded_nofold --sharded --no-fold
