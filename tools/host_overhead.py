"""Diagnostic: host cost of one cached-plan infer call vs the GPU time per call
(bench workload: chain20 d32, 65 536 queries).  Prints enqueue us/call (no
sync inside the loop) and wall us/call (sync at the end)."""
import os
import random
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from continuousbayesiannetwork_amd import BayesianNetwork  # noqa: E402
from helpers import chain_data, make_bn, sample_evidence  # noqa: E402

dev = torch.device("cuda:0")
data, cols, edges = chain_data(20, 32, 200_000, 3, stay=0.8)
bn = make_bn(BayesianNetwork, edges, cols, data, device=dev)
names = [c for c in cols if c != "X19"]
ev = {k: torch.tensor(v, device=dev) for k, v in sample_evidence(data, cols, names, 65536, 1000).items()}
random.seed(0)
for _ in range(50):
    bn.infer("X19", ev, N_max=32)
torch.cuda.synchronize()
for K in (200, 2000):
    t0 = time.perf_counter()
    for _ in range(K):
        bn.infer("X19", ev, N_max=32)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f"K={K}: enqueue {(t1 - t0) / K * 1e6:.2f} us/call, wall {(t2 - t0) / K * 1e6:.2f} us/call")
fp = next(iter(bn.engine._fast.values()))
print("native host path:", fp.host)
