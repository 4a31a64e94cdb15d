"""Direct plans (csrc/cbn_direct.hip) at batch scale: BruteForce networks the
table path cannot take -- a 40-level child of 4 parents (hashed CPD), a
continuous network with a free parent (hashed), a 16-parent node (dense CPD,
> 8 parents).  65 536 queries; writes gpurun_out/bench_direct.json."""
import json
import os
import random
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from continuousbayesiannetwork_amd import BayesianNetwork  # noqa: E402
from helpers import continuous_free_data, hicard_data, make_bn, sample_evidence, wide_data  # noqa: E402


def run(name, data, cols, edges, target, ev_names, N, Q=65536, K=20):
    dev = torch.device("cuda:0")
    bn = make_bn(BayesianNetwork, edges, cols, data, device=dev)
    batches = [{k: torch.tensor(v, device=dev) for k, v in sample_evidence(data, cols, ev_names, Q, s).items()}
               for s in range(2)]
    random.seed(0)
    for b in batches:
        bn.infer(target, b, N_max=N)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for i in range(K):
        random.seed(0)
        bn.infer(target, batches[i % 2], N_max=N)
    e1.record()
    torch.cuda.synchronize()
    t = e0.elapsed_time(e1) / 1e3 / K
    est = bn.nodes_obj[target].estimator
    r = dict(case=name, queries=Q, N=N, us_per_call=round(t * 1e6, 1), queries_per_s=round(Q / t, 1),
             hashed=bool(est.sparse), cpd_cells=est.n_cells(), unique_rows=int(est.mle_tensor.shape[0]))
    print(json.dumps(r), flush=True)
    return r


def main():
    out = []
    data, cols, edges = hicard_data(200_000, 33)
    out.append(run("hicard40: E | R0..R3 (40 levels), all observed", data, cols, edges, "E", cols[:4], 40))
    out.append(run("hicard40: E | R0..R3, R1 free", data, cols, edges, "E", ["R0", "R2", "R3"], 8))
    data, cols, edges = continuous_free_data(200_000, 37)
    out.append(run("continuous: X3 | X0, X1 (~1500 values), X2 free", data, cols, edges, "X3", ["X0", "X1"], 8))
    data, cols, edges = wide_data(200_000, 8, k=16)
    out.append(run("wide16: Y | P0..P15, all observed", data, cols, edges, "Y", cols[:16], 3))
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    with open(os.path.join(ROOT, "gpurun_out", "bench_direct.json"), "w") as fh:
        json.dump(out, fh, indent=1)


if __name__ == "__main__":
    main()
