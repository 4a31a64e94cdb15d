"""Diagnostic: host cost of one torch.distributed all_reduce of the 4-byte max
word (the sharded step's only exchange) and of the whole sharded step.
Run under torch.distributed.run (any world size, one rank per GPU)."""
import os
import sys
import time

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

local = int(os.environ.get("LOCAL_RANK", "0"))
torch.cuda.set_device(local)
dist.init_process_group("nccl", device_id=torch.device("cuda", local))
rank, world = dist.get_rank(), dist.get_world_size()
w = torch.zeros(1, dtype=torch.int32, device="cuda")
for _ in range(50):
    dist.all_reduce(w, op=dist.ReduceOp.MAX)
torch.cuda.synchronize()
K = 2000
t0 = time.perf_counter()
for _ in range(K):
    dist.all_reduce(w, op=dist.ReduceOp.MAX)
t1 = time.perf_counter()
torch.cuda.synchronize()
t2 = time.perf_counter()
if rank == 0:
    print(f"world={world} all_reduce(4 B): enqueue {(t1 - t0) / K * 1e6:.2f} us/call, "
          f"wall {(t2 - t0) / K * 1e6:.2f} us/call", flush=True)

from continuousbayesiannetwork_amd import BayesianNetwork  # noqa: E402
from continuousbayesiannetwork_amd.distributed import sharded_infer  # noqa: E402
from helpers import chain_data, make_bn, sample_evidence  # noqa: E402

data, cols, edges = chain_data(20, 32, 200_000, 3, stay=0.8)
bn = make_bn(BayesianNetwork, edges, cols, data, device=torch.device("cuda", local))
names = [c for c in cols if c != "X19"]
ev = {k: torch.tensor(v, device="cuda") for k, v in sample_evidence(data, cols, names, 65536, 1000 + rank).items()}
for _ in range(20):
    sharded_infer(bn, "X19", ev, N_max=32)
torch.cuda.synchronize()
dist.barrier()
K = 500
t0 = time.perf_counter()
for _ in range(K):
    sharded_infer(bn, "X19", ev, N_max=32)
t1 = time.perf_counter()
torch.cuda.synchronize()
t2 = time.perf_counter()
if rank == 0:
    print(f"world={world} sharded step (raw + all_reduce + scale): enqueue {(t1 - t0) / K * 1e6:.2f} us/call, "
          f"wall {(t2 - t0) / K * 1e6:.2f} us/call", flush=True)
dist.destroy_process_group()
