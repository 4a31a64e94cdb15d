"""Diagnostic: does a freshly created RCCL communicator slow the sharded step
(host enqueue / wall per step) and for how long?  One stepper, several rounds
of K steps; first without an exchange (no communicator), then with one."""
import os
import sys
import time

import torch

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
       for i in range(16)]
K = 500


def rounds(name, st, n=6):
    t_start = time.perf_counter()
    for r in range(n):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(K):
            st.step(evs[i % len(evs)])
        t1 = time.perf_counter()
        st.wait()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        print(f"{name} round {r} (t={t0 - t_start:.3f} s): enqueue {(t1 - t0) / K * 1e6:.2f} us, "
              f"wall {(t2 - t0) / K * 1e6:.2f} us per step", flush=True)


only = sys.argv[1] if len(sys.argv) > 1 else None
if only is None:
    for fold in (True, False):
        st = ShardedStepper(bn, "X19", 32, force_exchange=False, exchange_every=8, fold=fold)
        rounds(f"no comm, fold={fold}", st, 3)
        st.close()
for fold in (True, False):
    if only not in (None, f"fold={fold}"):
        continue
    st = ShardedStepper(bn, "X19", 32, force_exchange=True, exchange_every=8, fold=fold)
    rounds(f"comm, fold={fold}", st)
    st.close()
