"""Diagnostic (round 4): per-step host enqueue times of
the driver's bench sequence (configs[1], warmup W then K timed infer calls
on 64 rotating evidence batches) and the end-of-region synchronisation, for
a few host-side variants:
  base      -- bench.py's loop as is
  gcoff     -- gc disabled inside the timed region
  spin      -- poll the end event (busy) before torch.cuda.synchronize()
  prespin   -- the host polls the warmup's completion before the opening
               synchronize (it never sleeps in a blocking wait)
  busy      -- a spin kernel holds the stream before the timed steps (every
               launch then enqueues behind queued work: launch cost on a busy
               vs an idle queue)
Prints one JSON line per variant: per-step host us, region events us, sync us."""
import gc
import json
import os
import random
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from continuousbayesiannetwork_amd import BayesianNetwork  # noqa: E402
from helpers import chain_data, make_bn, sample_evidence  # noqa: E402


def main():
    W = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    K = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    dev = torch.device("cuda:0")
    data, cols, edges = chain_data(20, 32, 200_000, 3, stay=0.8)
    names = cols[:-1]
    ev_np = sample_evidence(data, cols, names, 65536, 1000)
    bn = make_bn(BayesianNetwork, edges, cols, data, device=dev)
    g = torch.Generator().manual_seed(7)
    base = {k: torch.tensor(v) for k, v in ev_np.items()}
    batches = []
    for b in range(64):
        perm = torch.randperm(65536, generator=g) if b else torch.arange(65536)
        batches.append({k: v[perm].contiguous().to(dev) for k, v in base.items()})
    it = [0]

    def step():
        ev = batches[it[0] % 64]
        it[0] += 1
        return bn.infer("X19", ev, N_max=32)

    random.seed(0)
    for variant in ("base", "prespin", "base", "prespin", "base", "prespin"):
        for _ in range(W):
            step()
        if variant == "prespin":  # poll the warmup's completion (the host never sleeps), then synchronize
            ew = torch.cuda.Event()
            ew.record()
            while not ew.query():
                pass
        torch.cuda.synchronize()
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        aff = os.sched_getaffinity(0)
        if variant == "pin":
            os.sched_setaffinity(0, {min(aff)})
        if variant == "gcoff":
            gc.disable()
        if variant == "busy":  # the launch queue starts non-empty: a ~300 us spin kernel ahead of the steps
            torch.cuda._sleep(600_000)
        ts = []
        ev0.record()
        t0 = time.perf_counter()
        for _ in range(K):
            step()
            ts.append(time.perf_counter())
        ev1.record()
        t1 = time.perf_counter()
        if variant == "spin":
            while not ev1.query():
                pass
        t2 = time.perf_counter()
        torch.cuda.synchronize()
        t3 = time.perf_counter()
        gc.enable()
        os.sched_setaffinity(0, aff)
        steps = [round((b - a) * 1e6, 2) for a, b in zip([t0] + ts[:-1], ts)]
        print(json.dumps(dict(variant=variant, W=W, K=K, steps_us=steps,
                              host_mean_us=round((ts[-1] - t0) / K * 1e6, 2),
                              region_us_per_step=round(ev0.elapsed_time(ev1) * 1e3 / K, 2),
                              spin_us=round((t2 - t1) * 1e6, 1), sync_us=round((t3 - t2) * 1e6, 1),
                              wall_us_per_step=round((t3 - t0) / K * 1e6, 2))), flush=True)


if __name__ == "__main__":
    main()
