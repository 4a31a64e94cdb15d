"""Generate golden input/output vectors by running the REFERENCE itself.

Run here (the container that has /root/reference), never on the GPU box:

    python tests/golden/make_golden.py

It imports the reference's own modules from /root/reference and calls
``BayesianNetwork.infer`` (cbn/base/bayesian_network.py:208-305) on small
seeded networks fitted with the BruteForce estimator
(cbn/parameter_learning/brute_force.py).  The reference package's
``cbn/parameter_learning/__init__.py`` imports the GP estimator, whose
third-party dependency (gpytorch ~=1.14, requirements.txt) is not installed in
this image; the package is therefore assembled from the reference's own
brute_force.py module without executing that ``__init__`` (the GP estimator is
not on the inference path).  No reference source is copied: only the
inputs/outputs land in ``tests/golden/*.npz``.
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
    bf = load("cbn.parameter_learning.brute_force", REF + "/cbn/parameter_learning/brute_force.py")
    pl.ESTIMATORS = {"brute_force": bf.BruteForce}
    from cbn.base.bayesian_network import BayesianNetwork

    return BayesianNetwork


# ----------------------------------------------------------------- data -----
def chain_data(n, d, S, seed, values=None):
    rng = np.random.default_rng(seed)
    X = np.zeros((S, n), np.int64)
    X[:, 0] = rng.integers(0, d, S)
    for i in range(1, n):
        X[:, i] = (X[:, i - 1] + rng.choice(3, S, p=[0.6, 0.3, 0.1])) % d
    vals = np.arange(d, dtype=np.float32) if values is None else np.asarray(values, np.float32)
    cols = [f"X{i}" for i in range(n)]
    edges = [(f"X{i}", f"X{i+1}") for i in range(n - 1)]
    return vals[X], cols, edges


def multi_data(S, seed):
    """A, B -> C ; C, D -> E ; A -> D ; d = 3 with non-integer values."""
    rng = np.random.default_rng(seed)
    A = rng.integers(0, 3, S)
    B = rng.integers(0, 3, S)
    C = (A + B + rng.integers(0, 2, S)) % 3
    D = (A + rng.choice(3, S, p=[0.7, 0.2, 0.1])) % 3
    E = (C * D + rng.integers(0, 2, S)) % 3
    vals = np.array([-1.5, 0.25, 2.0], np.float32)
    X = np.stack([A, B, C, D, E], 1)
    cols = ["A", "B", "C", "D", "E"]
    edges = [("A", "C"), ("B", "C"), ("C", "E"), ("D", "E"), ("A", "D")]
    return vals[X], cols, edges


def sample_evidence(data, cols, names, Q, seed, missing_frac=0.0, missing_value=7.5):
    rng = np.random.default_rng(seed)
    rows = rng.integers(0, data.shape[0], Q)
    ev = {}
    for nm in names:
        v = data[rows, cols.index(nm)].astype(np.float32).reshape(Q, 1)
        if missing_frac > 0:
            m = rng.random(Q) < missing_frac
            v[m, 0] = missing_value
        ev[nm] = v
    return ev


CASES = [
    # name, data-fn, target, evidence names, Q, N_max, rnd seed, extra
    dict(name="chain5_d4_q1024_parent", data=("chain", 5, 4, 3000, 1), target="X4",
         ev=["X3"], Q=1024, N=4),
    dict(name="chain5_d4_all_evidence", data=("chain", 5, 4, 3000, 2), target="X4",
         ev=["X0", "X1", "X2", "X3"], Q=64, N=4),
    dict(name="chain5_d4_noevidence", data=("chain", 5, 4, 3000, 3), target="X4",
         ev=[], Q=1, N=4),
    dict(name="chain5_d4_subsample", data=("chain", 5, 4, 3000, 4), target="X4",
         ev=["X3", "X1"], Q=32, N=3),
    dict(name="chain5_d4_oversample", data=("chain", 5, 4, 3000, 5), target="X4",
         ev=["X3"], Q=16, N=6, seed=123),
    dict(name="chain6_d5_float_values", data=("chain", 6, 5, 4000, 6, [0.1, 0.7, 1.3, 2.9, 11.0]),
         target="X5", ev=["X4", "X2"], Q=48, N=5),
    dict(name="multi_partial", data=("multi", 2000, 7), target="E",
         ev=["C", "A"], Q=20, N=3),
    dict(name="multi_all_parents", data=("multi", 2000, 8), target="E",
         ev=["C", "D", "A", "B"], Q=40, N=3),
    dict(name="multi_missing_values", data=("multi", 2000, 9), target="E",
         ev=["C", "D"], Q=40, N=3, missing=0.25),
    dict(name="multi_target_C_oversample", data=("multi", 2000, 10), target="C",
         ev=["A", "B"], Q=12, N=5, seed=7),
    dict(name="root_target_q1", data=("chain", 4, 3, 500, 11), target="X0",
         ev=[], Q=1, N=3),
    dict(name="err_evidence_none", data=("chain", 4, 3, 500, 13), target="X3",
         ev=[], Q=1, N=3, evidence_none=True, expect_error=True),
    dict(name="err_target_parent_free", data=("chain", 5, 4, 500, 12), target="X4",
         ev=["X1"], Q=8, N=4, expect_error=True),
    # BASELINE configs[1] shape (the headline network) at a reference-friendly batch
    dict(name="chain20_d32_config1", data=("chain_stay", 20, 32, 20000, 21, 0.8), target="X19",
         ev=[f"X{i}" for i in range(19)], Q=256, N=32, ev_seed=201),
    # configs[2] shape: alarm-like 37-node DAG, in-degree <= 4, d = 8 (tests/helpers.py)
    dict(name="alarm37_d8_config2", data=("alarm", 20000, 22), target="X36",
         ev=[f"X{i}" for i in range(36)], Q=96, N=8, ev_seed=202),
    dict(name="alarm37_d8_partial", data=("alarm", 20000, 23), target="X35",
         ev=[f"X{i}" for i in range(0, 35, 2)], Q=12, N=8, ev_seed=203),
    # configs[4] shape at a size where the 25-factor product stays finite: 5 x 5 grid, d = 4
    dict(name="grid5_d4_config4", data=("grid", 20000, 24, 5, 4), target="X24",
         ev=[f"X{i}" for i in range(24)], Q=64, N=4, ev_seed=204),
    # direct plans (csrc/cbn_direct.hip): > 8 parents, hashed CPDs of
    # high-cardinality and continuous columns
    dict(name="wide10_free2", data=("wide", 4000, 31, 10), target="Y",
         ev=[f"P{i}" for i in range(8)], Q=40, N=2, ev_seed=301),
    dict(name="wide12_all", data=("wide", 4000, 32, 12), target="Y",
         ev=[f"P{i}" for i in range(12)], Q=40, N=3, ev_seed=302),
    dict(name="hicard40_all", data=("hicard", 20000, 33), target="E",
         ev=["R0", "R1", "R2", "R3"], Q=64, N=16, ev_seed=303, seed=5),
    dict(name="hicard40_free1", data=("hicard", 20000, 34), target="E",
         ev=["R0", "R2", "R3"], Q=24, N=4, ev_seed=304, seed=6, missing=0.1),
    dict(name="cont4_all", data=("cont", 8000, 35), target="X3",
         ev=["X0", "X1", "X2"], Q=48, N=16, ev_seed=305, seed=7),
    dict(name="cont4_free1", data=("cont", 8000, 36), target="X3",
         ev=["X0", "X1"], Q=24, N=6, ev_seed=306, seed=8),
    dict(name="cont4_free_support", data=("cont_free", 20000, 37), target="X3",
         ev=["X0", "X1"], Q=24, N=8, ev_seed=307, seed=9),
    # evidence columns that are not [Q, 1] (round 5): width = {variable: k},
    # column j of a widened variable drawn with ev_seed + 1000 j.  The
    # reference copies a fully observed node's columns into [Q, 1] slots
    # (node.py:233-234) and expands a partially observed node's to [Q, N]
    # (:246-248): RuntimeError unless k = 1 (or k = N for the expand)
    dict(name="err_width2_chain", data=("chain", 5, 4, 3000, 41), target="X4",
         ev=["X0", "X1", "X2", "X3"], Q=16, N=4, ev_seed=401, expect_error=True,
         width={"X0": 2, "X1": 2, "X2": 2, "X3": 2}),
    dict(name="err_width2_last_slot", data=("chain", 5, 4, 3000, 42), target="X4",
         ev=["X0", "X1", "X2", "X3"], Q=16, N=4, ev_seed=402, expect_error=True, width={"X3": 2}),
    dict(name="err_width2_strict_parent", data=("multi", 2000, 43), target="E",
         ev=["C", "A"], Q=12, N=3, ev_seed=403, expect_error=True, width={"A": 2}),
    dict(name="err_width2_partial", data=("multi", 2000, 44), target="E",
         ev=["C"], Q=12, N=3, ev_seed=404, expect_error=True, width={"C": 2}),
    dict(name="err_width0", data=("chain", 5, 4, 3000, 45), target="X4",
         ev=["X3"], Q=16, N=4, ev_seed=405, expect_error=True, width={"X3": 0}),
    # ... and k = N through the expand only: the reference reads the column as
    # N per-sample values of the observed parent (a per-query free parent);
    # the HIP engine raises NotImplementedError for it (Parity),
    # the oracle reproduces the values
    dict(name="multi_widthN_partial", data=("multi", 2000, 46), target="E",
         ev=["C"], Q=12, N=3, ev_seed=406, width={"C": 3}),
]


def make_data(spec):
    if spec[0] == "chain":
        vals = spec[5] if len(spec) > 5 else None
        return chain_data(spec[1], spec[2], spec[3], spec[4], vals)
    if spec[0] in ("alarm", "grid", "chain_stay", "wide", "hicard", "cont", "cont_free"):
        sys.path.insert(0, os.path.dirname(HERE))
        from helpers import (alarm_like_data, continuous_data, continuous_free_data, grid_data, hicard_data,
                             wide_data)
        from helpers import chain_data as chain_stay

        if spec[0] == "wide":
            return wide_data(spec[1], spec[2], k=spec[3])
        if spec[0] == "hicard":
            return hicard_data(spec[1], spec[2])
        if spec[0] == "cont":
            return continuous_data(spec[1], spec[2])
        if spec[0] == "cont_free":
            return continuous_free_data(spec[1], spec[2])

        if spec[0] == "chain_stay":  # bench.py's generator: X_i = X_{i-1} w.p. stay, else uniform
            return chain_stay(spec[1], spec[2], spec[3], spec[4], stay=spec[5])
        if spec[0] == "alarm":
            return alarm_like_data(spec[1], spec[2])
        return grid_data(spec[1], spec[2], side=spec[3], d=spec[4], keep=0.9)
    return multi_data(spec[1], spec[2])


def main():
    import networkx as nx
    import pandas as pd
    import torch

    BayesianNetwork = _load_reference()
    only = set(sys.argv[1:])  # regenerate just these cases (default: all)
    manifest = []
    for c in CASES:
        if only and c["name"] not in only:
            manifest.append(c["name"])
            continue
        data, cols, edges = make_data(c["data"])
        dag = nx.DiGraph()
        dag.add_nodes_from(cols)
        dag.add_edges_from(edges)
        df = pd.DataFrame(data, columns=cols)
        bn = BayesianNetwork(dag, df, {"estimator_name": "brute_force"},
                             {"inference_obj": "exact"}, device="cpu")
        ev = sample_evidence(data, cols, c["ev"], c["Q"], seed=c.get("ev_seed", 100 + len(manifest)),
                             missing_frac=c.get("missing", 0.0))
        for v, k in c.get("width", {}).items():
            ev[v] = np.concatenate([sample_evidence(data, cols, [v], c["Q"], seed=c["ev_seed"] + 1000 * j)[v]
                                    for j in range(k)], 1) if k > 0 else np.zeros((c["Q"], 0), np.float32)
        ev_t = {k: torch.tensor(v) for k, v in ev.items()}
        if c.get("evidence_none"):
            ev_t = None
        seed = c.get("seed", 0)
        random.seed(seed)
        err = ""
        pdf = dom = np.zeros((0,), np.float32)
        try:
            p, d = bn.infer(c["target"], ev_t, N_max=c["N"])
            pdf, dom = p.numpy().astype(np.float32), d.numpy().astype(np.float32)
        except AssertionError as e:  # reference's shape assertion (bayesian_network.py:301)
            err = "AssertionError:" + str(e)
        except AttributeError as e:  # evidence=None (bayesian_network.py:193)
            err = "AttributeError:" + str(e)
        except RuntimeError as e:  # an evidence column that is not [Q, 1] (node.py:233-248)
            err = "RuntimeError:" + str(e)
        assert bool(err) == bool(c.get("expect_error", False)), (c["name"], err)
        out = dict(data=data.astype(np.float32), pdf=pdf, domain=dom,
                   meta=np.array(json.dumps(dict(
                       name=c["name"], columns=cols, edges=edges, target=c["target"],
                       evidence=list(ev.keys()), evidence_none=bool(c.get("evidence_none")), N_max=c["N"], seed=seed, error=err,
                       width=c.get("width", {})))))
        for k, v in ev.items():
            out["ev_" + k] = v
        np.savez_compressed(os.path.join(HERE, c["name"] + ".npz"), **out)
        manifest.append(c["name"])
        print(c["name"], pdf.shape, err)
    with open(os.path.join(HERE, "MANIFEST.json"), "w") as f:
        json.dump(dict(generator="tests/golden/make_golden.py",
                       reference="Giovannibriglia/ContinuousBayesianNetwork @ /root/reference",
                       cases=manifest), f, indent=1)


if __name__ == "__main__":
    main()
