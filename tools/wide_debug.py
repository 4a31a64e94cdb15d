"""Diagnostic (round 6): width-1 vs [Q, N] evidence calls on one engine."""
import os
import random
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]
from continuousbayesiannetwork_amd import BayesianNetwork  # noqa: E402
from helpers import make_bn  # noqa: E402
from oracle.ref_infer import OracleBN  # noqa: E402
from test_gpu_direct import _wide_net  # noqa: E402

dev = torch.device("cuda:0")
data, cols, edges = _wide_net()
N, Q = 4, 3000
rng = np.random.default_rng(N * 7 + Q)
cw = rng.integers(0, 4, (Q, N)).astype(np.float32)
cw[::17, 0] = 9.0
ora = OracleBN(edges, cols, data)


def run(bn, ev, tag):
    random.seed(12)
    ref, _ = ora.infer("E", ev, N)
    random.seed(12)
    pdf, _ = bn.infer("E", {k: torch.tensor(v, device=dev) for k, v in ev.items()}, N_max=N)
    p = pdf.cpu().numpy()
    print(tag, "nan", int(np.isnan(p).sum()), "max", float(np.nanmax(p)) if np.isfinite(p).any() else None,
          "maxdiff", float(np.nanmax(np.abs(p - ref))), "plans", len(bn.engine._plans), len(bn.engine._wide_plans),
          flush=True)


for order in (("w1", "wide", "w1"), ("wide", "w1")):
    bn = make_bn(BayesianNetwork, edges, cols, data, device=dev)
    for o in order:
        run(bn, {"C": cw[:, :1].copy()} if o == "w1" else {"C": cw}, o)
    print("---")
