"""Diagnostic: a deep NeuralNetwork (6 hidden ReLU layers of 8) on the
12-node mixed DAG -- HIP result vs the fp32 oracle vs an oracle whose mu is
evaluated in float64 (the 'ideal' network output), to tell a kernel error
from fp32 rounding noise amplified by the densities."""
import os
import random
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import oracle.ref_infer as R  # noqa: E402
from continuousbayesiannetwork_amd import BayesianNetwork  # noqa: E402
from helpers import make_bn, mixed_dag_data, param_config, sample_evidence  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    data, cols, edges = mixed_dag_data(3000, 4, n=12, unit=True)
    for model, evn in [({"hidden_dims": [8] * 6, "activation": "relu"}, "sparse"),
                       ({"hidden_dims": [8] * 6, "activation": "relu"}, "all"),
                       ({"hidden_dims": [16], "activation": "relu"}, "sparse")]:
        bn = make_bn(BayesianNetwork, edges, cols, data, device=dev, estimator="neural_network",
                     config=param_config("neural_network", n_epochs=25, model=model))

        def ora(f64):
            ests = {}
            for n in cols:
                e = bn.nodes_obj[n].estimator
                layers = [(l.weight.detach().cpu().numpy(), l.bias.detach().cpu().numpy()) for l in e._linears()]
                o = R.OracleParametric("logistic", layers, float(e._log_scale().detach().cpu()), act="relu")
                if f64:
                    def mu(q, o=o):
                        h = q.astype(np.float64)
                        for i, (W, b) in enumerate(o.layers):
                            h = h @ W.T.astype(np.float64) + b
                            if i < len(o.layers) - 1:
                                h = np.maximum(h, 0)
                        return h.astype(np.float32)
                    o.mu = mu
                ests[n] = o
            return R.OracleBN(edges, cols, data, estimators=ests)

        names = [c for c in cols if c != cols[-1]] if evn == "all" else [cols[-2], cols[5], cols[2]]
        ev = sample_evidence(data, cols, names, 700, 3)
        random.seed(4)
        a, _ = ora(False).infer(cols[-1], ev, 8)
        random.seed(4)
        b, _ = ora(True).infer(cols[-1], ev, 8)
        random.seed(4)
        g = bn.infer(cols[-1], {k: torch.tensor(v, device=dev) for k, v in ev.items()}, N_max=8)[0].cpu().numpy()
        m = b > 1e-7
        scales = [round(float(np.exp(bn.nodes_obj[n].estimator._log_scale().detach().cpu())), 4) for n in cols]
        print(model, evn, "scales", scales)
        print("  oracle32 vs ideal max rel", float((np.abs(a - b) / b)[m].max()),
              " hip vs ideal", float((np.abs(g - b) / b)[m].max()),
              " hip vs oracle32", float((np.abs(g - a) / np.maximum(a, 1e-30))[m].max()), flush=True)


if __name__ == "__main__":
    main()
