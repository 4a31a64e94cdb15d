"""Full-batch golden vectors for BASELINE configs[3] (50-node mixed DAG,
LinearRegression and NeuralNetwork [16] tanh CPDs): the REFERENCE's
``BayesianNetwork.infer`` (cbn/base/bayesian_network.py:208-305) over one
GPU's share of the 1 048 576-query batch (131 072 queries), so the GPU test
compares a 4 096-row slice normalised by the max of the WHOLE batch at the
north-star tolerance.  Run here (the container with /root/reference):

    python tests/golden/make_golden_full_param.py

Each case takes the fitted parameters of the reference-generated fixture
``<base>.npz`` (tests/golden/make_golden_param.py: data, every node's
nn.Linear weights + log scale), builds the reference network on the same data
(a 1-epoch fit, then the fixture's parameters are written into every
estimator), and runs ONE ``infer`` over 131 072 queries drawn from the data
(seed 300).  Stored: the row indices (every 32nd row + the batch argmax row),
those rows of the output, the domain, digests of the inputs.  No reference
source is copied.
"""
from __future__ import annotations

import hashlib
import json
import os
import random
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.dirname(HERE))

CASES = {
    "lr_mixed50_config3_full": dict(base="lr_mixed50_config3", Q=131072, ev_seed=300, keep=32),
    "nn_mixed50_config3_full": dict(base="nn_mixed50_config3", Q=131072, ev_seed=301, keep=32),
}


def main():
    import contextlib
    import io

    import networkx as nx
    import pandas as pd
    import torch

    from golden_io import load_param_golden
    from helpers import sample_evidence
    from make_golden_param import _load_reference

    torch.set_num_threads(8)
    BN = _load_reference()
    only = set(sys.argv[1:])
    for name, c in CASES.items():
        if only and name not in only:
            continue
        g = load_param_golden(c["base"])
        m = g["meta"]
        data, cols = g["data"], m["columns"]
        dag = nx.DiGraph()
        dag.add_nodes_from(cols)
        dag.add_edges_from(m["edges"])
        cfg = {"estimator_name": m["estimator"], "optimizer": {"name": "Adam", "params": {"lr": 0.05}},
               "train": {"n_epochs": 1}}
        if m["model"]:
            cfg["model"] = m["model"]
        torch.manual_seed(0)
        with contextlib.redirect_stdout(io.StringIO()):
            bn = BN(dag, pd.DataFrame(data, columns=cols), cfg, {"inference_obj": "exact"}, device="cpu")
        with torch.no_grad():
            for n, (layers, ls) in g["params"].items():
                est = bn.nodes_obj[n].estimator
                lins = ([mm for mm in est.nn_model if isinstance(mm, torch.nn.Linear)] if hasattr(est, "nn_model")
                        else [est.linear_model])
                assert len(lins) == len(layers)
                for lin, (W, b) in zip(lins, layers):
                    lin.weight.copy_(torch.tensor(W))
                    lin.bias.copy_(torch.tensor(b))
                scale = est.log_scale if hasattr(est, "log_scale") else est.log_sigma
                scale.copy_(torch.tensor(ls, dtype=scale.dtype))
        names = [x for x in cols if x != m["target"]]
        ev = sample_evidence(data, cols, names, c["Q"], c["ev_seed"])
        random.seed(0)
        with torch.no_grad(), contextlib.redirect_stdout(io.StringIO()):
            pdf, dom = bn.infer(m["target"], {k: torch.tensor(v) for k, v in ev.items()}, N_max=m["N_max"])
        pdf = pdf.numpy().astype(np.float32)
        finite = np.where(np.isfinite(pdf), pdf, -np.inf)
        rstar = int(np.unravel_index(np.argmax(finite), pdf.shape)[0])
        keep = np.union1d(np.arange(0, c["Q"], c["keep"]), [rstar])
        h = hashlib.sha256()
        for k in sorted(ev):
            h.update(np.ascontiguousarray(ev[k]).tobytes())
        meta = dict(name=name, base=c["base"], generator="tests/golden/make_golden_full_param.py", Q=c["Q"],
                    ev_seed=c["ev_seed"], target=m["target"], N_max=m["N_max"], argmax_row=rstar,
                    evidence_sha256=h.hexdigest(), max=float(np.nanmax(pdf)),
                    nan_rows=int(np.isnan(pdf).any(1).sum()),
                    reference="Giovannibriglia/ContinuousBayesianNetwork @ /root/reference, BayesianNetwork.infer")
        np.savez_compressed(os.path.join(HERE, name + ".npz"), rows=keep.astype(np.int64), pdf=pdf[keep],
                            domain=dom.numpy().astype(np.float32), meta=np.array(json.dumps(meta)))
        print(name, keep.size, "rows, argmax row", rstar, "nan rows", meta["nan_rows"], flush=True)


if __name__ == "__main__":
    main()
