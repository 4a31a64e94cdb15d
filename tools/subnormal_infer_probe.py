"""Diagnostic for tests/test_gpu_param.py::test_subnormal_densities_in_infer:
print the worst raw-row mismatches against the oracle."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from continuousbayesiannetwork_amd import BayesianNetwork  # noqa: E402
from helpers import make_bn, param_config  # noqa: E402
from test_gpu_param import _oracle_from_bn, _set_linear  # noqa: E402


def main():
    gpu = torch.device("cuda:0")
    rng = np.random.default_rng(9)
    S = 3000
    x0 = np.round(rng.normal(0, 1, S), 2)
    x1 = np.round(x0 + rng.normal(0, 0.03, S), 2)
    data = np.stack([x0, x1], 1).astype(np.float32)
    cols, edges = ["X0", "X1"], [("X0", "X1")]
    bn = make_bn(BayesianNetwork, edges, cols, data, device=gpu, estimator="linear_regression",
                 config=param_config("linear_regression", n_epochs=5))
    _set_linear(bn.nodes_obj["X1"].estimator, [[1.0]], [0.0], float(np.log(0.03)), gpu)
    ora = _oracle_from_bn(bn, edges, cols, data, "linear_regression")
    ev = {"X0": (x0[rng.integers(0, S, 4000)] + rng.uniform(-0.2, 0.2, 4000)).astype(np.float32)[:, None]}
    rows, dom, words, scale = bn.engine.infer_raw("X1", {k: torch.tensor(v, device=gpu) for k, v in ev.items()}, 16)
    raw = rows.cpu().numpy().copy()
    ref, rdom = ora.infer_raw("X1", ev, 16)
    rel = np.abs(raw - ref) / np.maximum(np.abs(ref), 1e-45)
    bad = np.argwhere((np.abs(raw - ref) > 1e-5 * np.abs(ref) + 2.0 ** -148))
    print("n bad", len(bad), "domain", rdom[0])
    e = bn.nodes_obj["X1"].estimator
    print("scale/norm", e._scale_norm())
    for q, j in bad[:12]:
        print(f"q={q} j={j} x0={ev['X0'][q, 0]:.7f} s={rdom[0, j]:.4f} got={raw[q, j]:.7e} ref={ref[q, j]:.7e} rel={rel[q, j]:.2e}")


if __name__ == "__main__":
    main()
