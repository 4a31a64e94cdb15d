"""Diagnostic: host enqueue cost and wall time of the sharded step's pieces
on configs[1] (65 536 queries per rank).  Run under torch.distributed.run;
the exchange is forced even at world size 1 so a one-GPU box exercises the
RCCL path:

  serial     raw launch -> all_reduce(MAX) of the block max words -> scale
  pipelined  raw launch on the compute stream; all_reduce + scale on a comm
             stream, so step i's exchange overlaps step i+1's raw launch
"""
import os
import sys
import time

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

from continuousbayesiannetwork_amd import BayesianNetwork  # noqa: E402
from continuousbayesiannetwork_amd.distributed import ShardedStepper  # noqa: E402
from helpers import chain_data, make_bn, sample_evidence  # noqa: E402

local = int(os.environ.get("LOCAL_RANK", "0"))
dev = torch.device("cuda", local)
torch.cuda.set_device(dev)
dist.init_process_group("nccl", device_id=dev)
rank, world = dist.get_rank(), dist.get_world_size()


def report(name, fn, K):
    for _ in range(20):
        fn()
    torch.cuda.synchronize()
    dist.barrier()
    t0 = time.perf_counter()
    for _ in range(K):
        fn()
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    if rank == 0:
        print(f"world={world} {name}: enqueue {(t1 - t0) / K * 1e6:.2f} us/step, wall {(t2 - t0) / K * 1e6:.2f} us/step",
              flush=True)


w = torch.zeros(256, dtype=torch.int32, device=dev)
report("all_reduce(1 KB)", lambda: dist.all_reduce(w, op=dist.ReduceOp.MAX), 2000)

data, cols, edges = chain_data(20, 32, 200_000, 3, stay=0.8)
bn = make_bn(BayesianNetwork, edges, cols, data, device=dev)
names = [c for c in cols if c != "X19"]
ev = {k: torch.tensor(v, device=dev) for k, v in sample_evidence(data, cols, names, 65536, 1000 + rank).items()}
report("fused infer (no exchange)", lambda: bn.infer("X19", ev, N_max=32), 2000)


report("raw launch alone (infer_raw)", lambda: bn.engine.infer_raw("X19", ev, 32), 2000)


def serial():
    rows, _, words, scale = bn.engine.infer_raw("X19", ev, 32)
    dist.all_reduce(words, op=dist.ReduceOp.MAX)
    scale(rows, words)


report("serial raw + all_reduce + scale", serial, 2000)

st0 = ShardedStepper(bn, "X19", 32)
report("pipelined ShardedStepper.step, no exchange", lambda: st0.step(ev), 2000)
st0.close()
st1 = ShardedStepper(bn, "X19", 32, exchange_every=1, force_exchange=True)
report("pipelined ShardedStepper.step, exchange every step", lambda: st1.step(ev), 2000)
st1.close()
for fold in (False, True):
    st2 = ShardedStepper(bn, "X19", 32, force_exchange=True, exchange_every=8, fold=fold)
    report(f"pipelined ShardedStepper.step, groups of 8, fold={fold}", lambda: st2.step(ev), 2000)
    st2.close()
st = ShardedStepper(bn, "X19", 32, force_exchange=True, fold=False)
report("pipelined ShardedStepper.step", lambda: st.step(ev), 2000)
flags = bn.engine.raw_flags(st._fp.plan)
report("native Stepper.step called directly", lambda: st._c.step(ev, None, flags, None), 2000)
if rank == 0:
    names = ["gather+alloc", "raw launch", "exchange share + return"]
    print("  native step phases (us):", {k: round(v, 2) for k, v in zip(names, st._c.host_timing())}, flush=True)
st.close()
dist.destroy_process_group()
