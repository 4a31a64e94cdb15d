"""Profiling driver for the parametric query kernel (configs[3] shape):
K calls of BayesianNetwork.infer on the 50-node mixed DAG, LinearRegression
(or --nn: NeuralNetwork [16] tanh), Q queries, N_max 16.  Run under
rocprofv3 (--kernel-trace --stats, or one --pmc pass at a time)."""
import argparse
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from continuousbayesiannetwork_amd import BayesianNetwork  # noqa: E402
from helpers import make_bn, mixed_dag_data, param_config, sample_evidence  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--nn", action="store_true")
    ap.add_argument("--queries", type=int, default=1048576)
    ap.add_argument("--calls", type=int, default=10)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    data, cols, edges = mixed_dag_data(50_000, 7, unit=True)
    est = "neural_network" if a.nn else "linear_regression"
    model = {"hidden_dims": [16], "activation": "tanh"} if a.nn else None
    bn = make_bn(BayesianNetwork, edges, cols, data, device=dev, estimator=est,
                 config=param_config(est, n_epochs=5, model=model))
    ev = {k: torch.tensor(v, device=dev) for k, v in sample_evidence(data, cols, cols[:-1], a.queries, 1).items()}
    for _ in range(a.calls):
        bn.infer(cols[-1], ev, N_max=16)
    torch.cuda.synchronize()
    print("done", flush=True)


if __name__ == "__main__":
    main()
