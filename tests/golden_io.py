"""Shared loader for the golden fixtures written by tests/golden/make_golden.py."""
import glob
import json
import os

import numpy as np

GOLDEN_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def golden_names():
    with open(os.path.join(GOLDEN_DIR, "MANIFEST.json")) as f:
        return json.load(f)["cases"]


def load_golden(name):
    z = np.load(os.path.join(GOLDEN_DIR, name + ".npz"), allow_pickle=False)
    meta = json.loads(str(z["meta"]))
    ev = {k[3:]: z[k] for k in z.files if k.startswith("ev_")}
    return dict(meta=meta, data=z["data"], pdf=z["pdf"], domain=z["domain"], evidence=ev)


ERRORS = {"AttributeError": AttributeError, "AssertionError": AssertionError, "RuntimeError": RuntimeError}


def golden_error(meta):
    """(exception type, message) of a fixture whose reference run raised."""
    kind, _, msg = meta["error"].partition(":")
    return ERRORS[kind], msg


def width_n_only(meta):
    """A fixture whose evidence has [Q, N] columns that the reference reads
    through ``.expand(-1, N)`` only (node.py:246-248): N per-query sample
    values of that parent (the engine's wide direct plan, round 6)."""
    return not meta["error"] and any(k != 1 for k in meta.get("width", {}).values())


def param_golden_names():
    with open(os.path.join(GOLDEN_DIR, "MANIFEST_param.json")) as f:
        return json.load(f)["cases"]


def load_param_golden(name):
    """Fixture of tests/golden/make_golden_param.py: data, evidence, the
    reference's outputs and every node's fitted parameters
    (params[node] = ([(W, b), ...], log_scale))."""
    z = np.load(os.path.join(GOLDEN_DIR, name + ".npz"), allow_pickle=False)
    meta = json.loads(str(z["meta"]))
    ev = {k[3:]: z[k] for k in z.files if k.startswith("ev_")}
    params = {}
    for n, pm in meta["params"].items():
        layers = [(z[f"W_{n}_{i}"], z[f"b_{n}_{i}"]) for i in range(pm["n_layers"])]
        params[n] = (layers, pm["log_scale"])
    return dict(meta=meta, data=z["data"], pdf=z["pdf"], domain=z["domain"], evidence=ev, params=params)


FAMILY = {"linear_regression": "gauss", "logistic_regression": "logistic", "neural_network": "logistic"}


def oracle_estimators(g):
    """OracleParametric per node from a parametric fixture's parameters."""
    from oracle.ref_infer import OracleParametric

    m = g["meta"]
    act = m["model"].get("activation", "tanh") if m["estimator"] == "neural_network" else None
    return {n: OracleParametric(FAMILY[m["estimator"]], layers, ls, act=act,
                                root_bias_only=m["estimator"] == "linear_regression")
            for n, (layers, ls) in g["params"].items()}
