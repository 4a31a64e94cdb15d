"""Diagnostic: the folding raw launch in isolation -- a Python loop of
cbn_plan_run_fold calls (each folding the rows of the launch R steps back)
over a ring of R row buffers, vs plain raw launches; wall per step."""
import ctypes
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

from continuousbayesiannetwork_amd import BayesianNetwork, _native  # noqa: E402
from helpers import chain_data, make_bn, sample_evidence  # noqa: E402

dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
data, cols, edges = chain_data(20, 32, 200_000, 3, stay=0.8)
bn = make_bn(BayesianNetwork, edges, cols, data, device=dev)
names = [c for c in cols if c != "X19"]
evs = [{k: torch.tensor(v, device=dev) for k, v in sample_evidence(data, cols, names, 65536, 1000 + i).items()}
       for i in range(16)]
bn.infer("X19", evs[0], N_max=32)
fp = bn.engine.raw_fast_path("X19", evs[0], 32)
plan = fp.plan
lib = _native.load()
ptrs = [(ctypes.c_void_p * len(fp.slot_keys))(*[e[k].data_ptr() for k in fp.slot_keys]) for e in evs]
W = fp.words.numel()
s = _native.stream_ptr(dev)
K = 2000


def run(R, fold):
    rows = [torch.empty((65536, 32), device=dev) for _ in range(R)]
    words = [torch.zeros(W, dtype=torch.int32, device=dev) for _ in range(R)]
    for rep in range(2):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(K):
            j = i % R
            jf = (i + 1) % R  # the oldest buffer: launched R - 1 steps ago
            if fold and i >= R:
                rc = lib.cbn_plan_run_fold(plan.handle, 65536, ptrs[i % 16], len(fp.slot_keys), words[j].data_ptr(),
                                           rows[j].data_ptr(), rows[jf].data_ptr(), rows[jf].numel(),
                                           words[jf].data_ptr(), W, 0, s)
            else:
                rc = lib.cbn_plan_run(plan.handle, 65536, ptrs[i % 16], len(fp.slot_keys), words[j].data_ptr(),
                                      rows[j].data_ptr(), _native.CBN_RUN_RAW, s)
            assert rc == 0
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        print(f"R={R:3d} fold={fold}: enqueue {(t1 - t0) / K * 1e6:6.2f} wall {(t2 - t0) / K * 1e6:6.2f} us/step",
              flush=True)


for R in (2, 24):
    run(R, False)
    run(R, True)
