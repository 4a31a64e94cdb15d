"""Diagnostic: host enqueue time and wall time per sharded step, folded vs
separate scale, in one process and in a chosen order (argv: sequence of
'fold' / 'nofold' / 'fused'); world size 1 over a one-rank RCCL communicator."""
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

dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
data, cols, edges = chain_data(20, 32, 200_000, 3, stay=0.8)
bn = make_bn(BayesianNetwork, edges, cols, data, device=dev)
names = [c for c in cols if c != "X19"]
evs = [{k: torch.tensor(v, device=dev) for k, v in sample_evidence(data, cols, names, 65536, 1000 + i).items()}
       for i in range(int(os.environ.get("NB", "8")))]


def report(name, fn, K=2000):
    for i in range(40):
        fn(evs[i % len(evs)])
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(K):
        fn(evs[i % len(evs)])
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f"{name}: enqueue {(t1 - t0) / K * 1e6:.2f} us/step, wall {(t2 - t0) / K * 1e6:.2f} us/step", flush=True)


for what in sys.argv[1:]:
    if what == "fused":
        report("fused infer", lambda e: bn.infer("X19", e, N_max=32))
        continue
    st = ShardedStepper(bn, "X19", 32, force_exchange=True, exchange_every=8, fold=(what == "fold"))

    def step(e):
        st.step(e)

    report(f"stepper {what}", step)
    st.wait()
    torch.cuda.synchronize()
    st.close()
