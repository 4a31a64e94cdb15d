"""Host side of one direct-plan case of tools/bench_direct.py (argv[1]: wide16
(default), continuous, hicard): cProfile of 20 infer calls.  Run it under
rocprofv3 --kernel-trace --stats for the kernel side."""
import cProfile
import os
import pstats
import random
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from continuousbayesiannetwork_amd import BayesianNetwork  # noqa: E402
from helpers import continuous_free_data, hicard_data, make_bn, sample_evidence, wide_data  # noqa: E402

case = sys.argv[1] if len(sys.argv) > 1 else "wide16"
dev = torch.device("cuda:0")
if case == "continuous":
    data, cols, edges = continuous_free_data(200_000, 37)
    target, ev_names, N = "X3", ["X0", "X1"], 8
elif case == "hicard":
    data, cols, edges = hicard_data(200_000, 33)
    target, ev_names, N = "E", cols[:4], 40
else:
    data, cols, edges = wide_data(200_000, 8, k=16)
    target, ev_names, N = "Y", cols[:16], 3
bn = make_bn(BayesianNetwork, edges, cols, data, device=dev)
b = {k: torch.tensor(v, device=dev) for k, v in sample_evidence(data, cols, ev_names, 65536, 0).items()}
for _ in range(3):
    random.seed(0)
    bn.infer(target, b, N_max=N)
torch.cuda.synchronize()
pr = cProfile.Profile()
pr.enable()
for _ in range(20):
    random.seed(0)
    bn.infer(target, b, N_max=N)
torch.cuda.synchronize()
pr.disable()
pstats.Stats(pr).sort_stats("cumulative").print_stats(25)
