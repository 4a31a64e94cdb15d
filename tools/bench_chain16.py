"""A/B helper (round 4): the reference's default N_max = 16 on a 20-node
chain with d = 16 (two lanes per query: L = 2), evidence on X0..X18, 65 536
and 262 144 queries -- k_query_cols vs k_query_fast (CBN_NO_COLS=1).  One
JSON line per batch size: us per call (HIP events over 100 calls)."""
import json
import os
import random
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from continuousbayesiannetwork_amd import BayesianNetwork  # noqa: E402
from helpers import chain_data, make_bn, sample_evidence  # noqa: E402

dev = torch.device("cuda:0")
data, cols, edges = chain_data(20, 16, 200_000, 5, stay=0.8)
names = cols[:-1]
bn = make_bn(BayesianNetwork, edges, cols, data, device=dev)
for Q in (65536, 262144):
    batches = [{k: torch.tensor(v, device=dev) for k, v in sample_evidence(data, cols, names, Q, s).items()}
               for s in range(4)]
    random.seed(0)
    for b in batches:
        bn.infer("X19", b, N_max=16)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for i in range(100):
        bn.infer("X19", batches[i % 4], N_max=16)
    e1.record()
    torch.cuda.synchronize()
    plan = next(iter(bn.engine._plans.values()))
    lib = bn.engine._fast[("X19", tuple(batches[0].keys()), 16)].lib
    print(json.dumps(dict(queries=Q, us_per_call=round(e0.elapsed_time(e1) * 10, 2),
                          plan_flags=int(lib.cbn_plan_flags(plan.handle)))), flush=True)
