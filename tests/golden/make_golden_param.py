"""Golden vectors for the PARAMETRIC estimators, produced by running the
REFERENCE itself (run here, in the container that has /root/reference):

    python tests/golden/make_golden_param.py

Networks are fitted by the reference's own LinearRegression /
LogisticRegression / NeuralNetwork (cbn/parameter_learning/*.py, a short Adam
run: the training result only has to be *some* fitted model), then
``BayesianNetwork.infer`` (cbn/base/bayesian_network.py:208-305) is called on
seeded evidence.  Each fixture stores the data, the evidence, the fitted
parameters of every node (nn.Linear weights/biases + log_sigma / log_scale)
and the reference's outputs, so the tests can load the same parameters into
the framework under test and into the oracle.  The reference package's
``cbn/parameter_learning/__init__.py`` imports gpytorch (absent here), so the
package is assembled from the reference's own estimator modules without
executing that ``__init__``.  No reference source is copied.
"""
from __future__ import annotations

import importlib.util
import json
import os
import random
import sys
import types

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference"

MODULES = {
    "linear_regression": ("linear_regression", "LinearRegression"),
    "logistic_regression": ("logistIc_regression", "LogisticRegression"),
    "neural_network": ("neural_network", "NeuralNetwork"),
}


def _load_reference():
    sys.path.insert(0, REF)

    def load(name, path):
        spec = importlib.util.spec_from_file_location(name, path)
        m = importlib.util.module_from_spec(spec)
        sys.modules[name] = m
        spec.loader.exec_module(m)
        return m

    import cbn  # noqa: F401  (empty package __init__)

    pl = types.ModuleType("cbn.parameter_learning")
    pl.__path__ = [REF + "/cbn/parameter_learning"]
    sys.modules["cbn.parameter_learning"] = pl
    load("cbn.parameter_learning.utils", REF + "/cbn/parameter_learning/utils.py")
    pl.ESTIMATORS = {}
    for key, (mod, cls) in MODULES.items():
        m = load("cbn.parameter_learning." + mod, f"{REF}/cbn/parameter_learning/{mod}.py")
        pl.ESTIMATORS[key] = getattr(m, cls)
    from cbn.base.bayesian_network import BayesianNetwork

    return BayesianNetwork


# ----------------------------------------------------------------- data -----
def chain_cont(n, S, seed):
    """Continuous Gaussian chain X0 -> ... -> X{n-1}."""
    rng = np.random.default_rng(seed)
    X = np.zeros((S, n), np.float32)
    X[:, 0] = rng.normal(0, 1, S)
    for i in range(1, n):
        X[:, i] = 0.8 * X[:, i - 1] + rng.normal(0, 0.6, S)
    cols = [f"X{i}" for i in range(n)]
    return np.round(X, 3).astype(np.float32), cols, [(f"X{i}", f"X{i+1}") for i in range(n - 1)]


def mixed_multi(S, seed):
    """A (discrete 3), B (continuous) -> C (continuous); A -> D (discrete 3);
    C, D -> E (continuous)."""
    rng = np.random.default_rng(seed)
    A = rng.integers(0, 3, S).astype(np.float32)
    B = rng.normal(0, 1, S).astype(np.float32)
    C = 0.5 * A + 0.7 * B + rng.normal(0, 0.5, S)
    D = ((A + rng.choice(3, S, p=[0.7, 0.2, 0.1])) % 3).astype(np.float32)
    E = 0.6 * C - 0.4 * D + rng.normal(0, 0.5, S)
    X = np.stack([A, B, C, D, E], 1)
    cols = ["A", "B", "C", "D", "E"]
    edges = [("A", "C"), ("B", "C"), ("C", "E"), ("D", "E"), ("A", "D")]
    return np.round(X, 3).astype(np.float32), cols, edges


def sample_evidence(data, cols, names, Q, seed):
    rng = np.random.default_rng(seed)
    rows = rng.integers(0, data.shape[0], Q)
    return {nm: data[rows, cols.index(nm)].astype(np.float32).reshape(Q, 1) for nm in names}


CASES = [
    dict(name="lr_chain5_all", est="linear_regression", data=("chain", 5, 300, 21), target="X4",
         ev=["X0", "X1", "X2", "X3"], Q=48, N=8),
    dict(name="lr_chain5_sparse", est="linear_regression", data=("chain", 5, 300, 22), target="X4",
         ev=["X1", "X3"], Q=32, N=6),
    dict(name="lr_multi_partial", est="linear_regression", data=("multi", 400, 23), target="E",
         ev=["C", "A"], Q=24, N=6, seed=5),
    dict(name="lr_chain4_noevidence", est="linear_regression", data=("chain", 4, 200, 24), target="X3",
         ev=[], Q=1, N=5),
    dict(name="nn_multi_all", est="neural_network", data=("multi", 400, 25), target="E",
         ev=["A", "B", "C", "D"], Q=40, N=5, model={"hidden_dims": [16], "activation": "tanh"}),
    dict(name="nn_multi_partial_deep_relu", est="neural_network", data=("multi", 400, 26), target="E",
         ev=["C", "A"], Q=16, N=4, seed=9, model={"hidden_dims": [8, 6], "activation": "relu"}),
    dict(name="nn_chain5_sigmoid", est="neural_network", data=("chain", 5, 300, 27), target="X4",
         ev=["X3", "X1"], Q=24, N=6, model={"hidden_dims": [12], "activation": "sigmoid"}),
    dict(name="nn_root_target", est="neural_network", data=("multi", 300, 28), target="A",
         ev=[], Q=1, N=3, model={"hidden_dims": [16], "activation": "tanh"}),
    dict(name="nn_multi_deep_elu", est="neural_network", data=("multi", 400, 31), target="E",
         ev=["C", "A"], Q=16, N=4, seed=11, model={"hidden_dims": [8, 6], "activation": "elu"}, unit=True),
    dict(name="nn_chain5_gelu", est="neural_network", data=("chain", 5, 300, 32), target="X4",
         ev=["X3"], Q=20, N=5, model={"hidden_dims": [10], "activation": "gelu"}),
    dict(name="nn_multi_leakyrelu", est="neural_network", data=("multi", 400, 33), target="E",
         ev=["A", "B", "C", "D"], Q=24, N=4, model={"hidden_dims": [16], "activation": "leakyrelu"}, unit=True),
    dict(name="logreg_multi", est="logistic_regression", data=("multi", 400, 29), target="E",
         ev=["C", "D"], Q=32, N=5),
    dict(name="logreg_multi_partial", est="logistic_regression", data=("multi", 400, 30), target="C",
         ev=["A"], Q=20, N=4, seed=3),
    # BASELINE configs[3] shape: 50-node mixed continuous / 20-level discrete DAG
    # (tests/helpers.mixed_dag_data, unit-scaled), evidence on the 49 non-target nodes
    dict(name="lr_mixed50_config3", est="linear_regression", data=("mixed50", 2000, 41), target="X49",
         ev=[f"X{i}" for i in range(49)], Q=32, N=16),
    dict(name="nn_mixed50_config3", est="neural_network", data=("mixed50", 2000, 42), target="X49",
         ev=[f"X{i}" for i in range(49)], Q=32, N=16, model={"hidden_dims": [16], "activation": "tanh"}),
]


def make_data(spec, unit=False):
    """``unit``: min-max scale every column into [0, 1] -- the NeuralNetwork /
    LogisticRegression estimators train a BCE-with-logits loss, whose logits
    diverge on targets outside [0, 1] until exp(-(x - mu)) overflows and the
    reference's density turns NaN (kept as one edge case)."""
    if spec[0] == "mixed50":
        sys.path.insert(0, os.path.dirname(HERE))
        from helpers import mixed_dag_data

        return mixed_dag_data(spec[1], spec[2], n=50, unit=True)
    data, cols, edges = chain_cont(spec[1], spec[2], spec[3]) if spec[0] == "chain" else mixed_multi(spec[1], spec[2])
    if unit:
        lo, hi = data.min(0), data.max(0)
        data = np.round((data - lo) / (hi - lo), 3).astype(np.float32)
    return data, cols, edges


def _params(est):
    """nn.Linear layers + log scale of a fitted reference estimator."""
    import torch

    if hasattr(est, "nn_model"):
        lins = [m for m in est.nn_model if isinstance(m, torch.nn.Linear)]
        ls = est.log_scale
    else:
        lins = [est.linear_model]
        ls = est.log_sigma if hasattr(est, "log_sigma") else est.log_scale
    return [(l.weight.detach().numpy().astype(np.float32), l.bias.detach().numpy().astype(np.float32))
            for l in lins], float(ls.detach())


def main():
    import networkx as nx
    import pandas as pd
    import torch

    BayesianNetwork = _load_reference()
    only = set(sys.argv[1:])  # regenerate just these cases (default: all)
    manifest = []
    for i, c in enumerate(CASES):
        if only and c["name"] not in only:
            manifest.append(c["name"])
            continue
        torch.manual_seed(1000 + i)
        data, cols, edges = make_data(c["data"], c.get("unit", False))
        dag = nx.DiGraph()
        dag.add_nodes_from(cols)
        dag.add_edges_from(edges)
        df = pd.DataFrame(data, columns=cols)
        cfg = {"estimator_name": c["est"], "optimizer": {"name": "Adam", "params": {"lr": 0.05}},
               "train": {"n_epochs": 40}}
        if "model" in c:
            cfg["model"] = c["model"]
        bn = BayesianNetwork(dag, df, cfg, {"inference_obj": "exact"}, device="cpu")
        ev = sample_evidence(data, cols, c["ev"], c["Q"], seed=200 + i)
        ev_t = {k: torch.tensor(v) for k, v in ev.items()}
        random.seed(c.get("seed", 0))
        p, d = bn.infer(c["target"], ev_t, N_max=c["N"])
        out = dict(data=data, pdf=p.numpy().astype(np.float32), domain=d.numpy().astype(np.float32))
        meta_params = {}
        for n in cols:
            layers, ls = _params(bn.nodes_obj[n].estimator)
            for li, (W, b) in enumerate(layers):
                out[f"W_{n}_{li}"] = W
                out[f"b_{n}_{li}"] = b
            meta_params[n] = dict(n_layers=len(layers), log_scale=ls)
        for k, v in ev.items():
            out["ev_" + k] = v
        out["meta"] = np.array(json.dumps(dict(
            name=c["name"], estimator=c["est"], model=c.get("model", {}), columns=cols, edges=edges,
            target=c["target"], evidence=list(ev.keys()), N_max=c["N"], seed=c.get("seed", 0), unit=c.get("unit", False),
            params=meta_params)))
        np.savez_compressed(os.path.join(HERE, c["name"] + ".npz"), **out)
        manifest.append(c["name"])
        print(c["name"], out["pdf"].shape, float(out["pdf"].min()), flush=True)
    with open(os.path.join(HERE, "MANIFEST_param.json"), "w") as f:
        json.dump(dict(generator="tests/golden/make_golden_param.py",
                       reference="Giovannibriglia/ContinuousBayesianNetwork @ /root/reference",
                       cases=manifest), f, indent=1)


if __name__ == "__main__":
    main()
