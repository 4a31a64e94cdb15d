"""Throughput vs batch size on the configs[1] network (chain20, d=32, N=32),
plus the PCIe-inclusive rate when evidence starts in (pinned) host memory and
the marginals go back to it.  Writes gpurun_out/batch_sweep.json (copied to
profiles/ by hand).

Per batch size: queries/s and effective GB/s (algorithmic bytes: 4 B per
evidence value read + 4*N B per output row written) with HIP events around
the timed loop on the launch stream.  Batches up to the fused capacity run as
one launch; larger ones as one raw compute pass + an in-place scale pass
(``--two-pass``-style max + write launches are also timed for comparison).
"""
import json
import os
import random
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from continuousbayesiannetwork_amd import BayesianNetwork  # noqa: E402
from helpers import chain_data, make_bn, sample_evidence  # noqa: E402


def timed(fn, k):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(k):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / 1e3 / k


def main():
    dev = torch.device("cuda:0")
    data, cols, edges = chain_data(20, 32, 200_000, 3, stay=0.8)
    bn = make_bn(BayesianNetwork, edges, cols, data, device=dev)
    names = [c for c in cols if c != "X19"]
    big = sample_evidence(data, cols, names, 1 << 22, 1000)
    random.seed(0)
    rows = []
    cap = None
    for q in [1024, 4096, 16384, 65536, 262144, 1 << 20, 1 << 22]:
        ev = {k: torch.tensor(v[:q], device=dev) for k, v in big.items()}
        bn.infer("X19", ev, N_max=32)
        if cap is None:
            cap = bn.engine.fused_capacity("X19", names, 32)
        k = max(5, min(200, (1 << 24) // q))
        t = timed(lambda: bn.infer("X19", ev, N_max=32), k)
        byt = q * (4 * len(names) + 4 * 32)
        bn.engine.fused = False  # max pass + write pass (both compute every product)
        bn.infer("X19", ev, N_max=32)
        t2 = timed(lambda: bn.infer("X19", ev, N_max=32), k)
        bn.engine.fused = True
        rows.append(dict(queries=q, path="fused" if q <= cap else "raw + scale", us_per_call=round(t * 1e6, 2),
                         queries_per_s=round(q / t, 1), effective_GBps=round(byt / t / 1e9, 1),
                         two_pass_us=round(t2 * 1e6, 2)))
        print(rows[-1], flush=True)
        del ev
    # PCIe-inclusive: evidence in pinned host memory -> device, marginals -> pinned host
    q = 65536
    hev = {k: torch.tensor(v[:q]).pin_memory() for k, v in big.items()}
    hout = torch.empty((q, 32), dtype=torch.float32).pin_memory()

    def pcie_step():
        ev = {k: v.to(dev, non_blocking=True) for k, v in hev.items()}
        pdf, _ = bn.infer("X19", ev, N_max=32)
        hout.copy_(pdf, non_blocking=True)

    t = timed(pcie_step, 100)
    pcie = dict(queries=q, us_per_call=round(t * 1e6, 2), queries_per_s=round(q / t, 1),
                note="19 evidence columns H2D (pinned) + infer + [Q,32] marginals D2H (pinned), one stream")
    print(pcie, flush=True)
    out = dict(workload="chain20_d32, target X19, evidence on X0..X18, N_max=32", fused_capacity=cap,
               sweep=rows, pcie_inclusive=pcie)
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    with open(os.path.join(ROOT, "gpurun_out", "batch_sweep.json"), "w") as fh:
        json.dump(out, fh, indent=1)


if __name__ == "__main__":
    main()
