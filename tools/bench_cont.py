"""BASELINE configs[3] on one GPU: 50-node mixed continuous/discrete DAG
(in-degree <= 3, 20-level discrete columns, unit-scaled), LinearRegression and
NeuralNetwork (hidden [16], tanh -- cbn/conf/parameter_learning/
neural_network.yaml) CPDs, evidence on the 49 non-target nodes, N_max = 16.
Batches: 131 072 queries (one GPU's share of the 1 048 576-query, 8-GPU
config) and the whole 1 048 576 on one GPU (--est lr|nn|both, --queries ...;
pdf_sha256 fingerprints the first batch's rows for same-bits A/Bs).

The parametric kernel is VALU-bound (one density -- one exp -- per query x
factor x sample column), so next to queries/s it reports density evaluations
per second and their share of the gfx950 transcendental issue peak (v_exp_f32:
8 cycles per wave instruction per SIMD -> 256 CUs x 4 SIMDs x 64 lanes / 8 cyc
x 2.4 GHz = 19.7 T/s).  Writes gpurun_out/bench_cont.json."""
import json
import os
import random
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from continuousbayesiannetwork_amd import BayesianNetwork  # noqa: E402
from helpers import make_bn, mixed_dag_data, param_config, sample_evidence  # noqa: E402

EXP_PEAK = 256 * 4 * 64 / 8 * 2.4e9  # v_exp_f32 issue peak, /s


def main():
    import argparse
    import hashlib

    ap = argparse.ArgumentParser()
    ap.add_argument("--est", choices=["lr", "nn", "both"], default="both")
    ap.add_argument("--queries", type=int, nargs="*", default=[131072, 1048576])
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    N = 16
    data, cols, edges = mixed_dag_data(50_000, 7, unit=True)
    target, names = cols[-1], cols[:-1]
    out = {"workload": "mixed DAG 50 nodes (25 continuous, 25 20-level discrete, unit-scaled), in-degree <= 3, "
                       f"{len(edges)} edges, evidence on 49 nodes, N_max={N}", "runs": []}
    torch.manual_seed(0)
    ests = [("linear_regression", None), ("neural_network", {"hidden_dims": [16], "activation": "tanh"})]
    ests = ests[:1] if a.est == "lr" else ests[1:] if a.est == "nn" else ests
    for est, model in ests:
        t0 = time.time()
        bn = make_bn(BayesianNetwork, edges, cols, data, device=dev, estimator=est,
                     config=param_config(est, n_epochs=50, model=model))
        fit_s = time.time() - t0
        for Q in a.queries:
            batches = [{k: torch.tensor(v, device=dev) for k, v in sample_evidence(data, cols, names, Q, s).items()}
                       for s in range(2)]
            random.seed(0)
            for b in batches:
                pdf, _ = bn.infer(target, b, N_max=N)
            torch.cuda.synchronize()
            p = pdf.cpu().numpy()
            K = 20 if Q > 200000 else 50
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for i in range(K):
                bn.infer(target, batches[i % 2], N_max=N)
            e1.record()
            torch.cuda.synchronize()
            t = e0.elapsed_time(e1) / 1e3 / K
            plan = next(iter(bn.engine._plans.values()))
            nq = sum(1 for f in plan.factors if f.kind == 2)
            dens = Q * nq * N / t
            r = dict(estimator=est, model=model, queries=Q, factors=len(plan.factors), query_factors=nq,
                     us_per_call=round(t * 1e6, 1), queries_per_s=round(Q / t, 1),
                     density_evals_per_s=round(dens, 1), exp_issue_frac=round(dens / EXP_PEAK, 4),
                     nonzero_frac=round(float((p > 0).mean()), 4), fit_s=round(fit_s, 1),
                     pdf_sha256=hashlib.sha256(p.tobytes()).hexdigest()[:16])
            out["runs"].append(r)
            print(json.dumps(r), flush=True)
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    with open(os.path.join(ROOT, "gpurun_out", "bench_cont.json"), "w") as fh:
        json.dump(out, fh, indent=1)


if __name__ == "__main__":
    main()
