"""BASELINE configs[2]: ALARM-like 37-node DAG (in-degree <= 4, d=8), 262 144
batched queries on 1 GPU, evidence on every non-target node.  Prints one JSON
line (queries/s, us per call, effective GB/s over the algorithmic bytes:
4 B per evidence value + 4*N B per output row) and writes it to
gpurun_out/bench_alarm.json."""
import json
import os
import random
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from continuousbayesiannetwork_amd import BayesianNetwork  # noqa: E402
from helpers import alarm_like_data, make_bn, sample_evidence  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    data, cols, edges = alarm_like_data(200_000, 5)
    out = {"workload": "alarm-like 37 nodes / 46 edges, in-degree <= 4, d=8, N_max=8, evidence on 36 nodes",
           "targets": []}
    for target in ("X35", "X36"):
        names = [c for c in cols if c != target]
        Q = 262144
        batches = [{k: torch.tensor(v, device=dev) for k, v in sample_evidence(data, cols, names, Q, s).items()}
                   for s in range(4)]
        bn = make_bn(BayesianNetwork, edges, cols, data, device=dev)
        random.seed(0)
        for b in batches:
            bn.infer(target, b, N_max=8)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        K = 100
        e0.record()
        for i in range(K):
            bn.infer(target, batches[i % 4], N_max=8)
        e1.record()
        torch.cuda.synchronize()
        t = e0.elapsed_time(e1) / 1e3 / K
        byt = Q * (4 * len(names) + 4 * 8)
        plan = next(iter(bn.engine._plans.values()))
        lib = bn.engine._fast[(target, tuple(batches[0].keys()), 8)].lib
        out["targets"].append(dict(target=target, factors=len(plan.factors), queries=Q, us_per_call=round(t * 1e6, 2),
                                   queries_per_s=round(Q / t, 1), effective_GBps=round(byt / t / 1e9, 1),
                                   fused_capacity=int(lib.cbn_plan_fused_capacity(plan.handle)),
                                   plan_flags=int(lib.cbn_plan_flags(plan.handle)),
                                   ))
        print(json.dumps(out["targets"][-1]), flush=True)
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    with open(os.path.join(ROOT, "gpurun_out", "bench_alarm.json"), "w") as fh:
        json.dump(out, fh, indent=1)


if __name__ == "__main__":
    main()
