"""Does the ~1.5 us per-launch excess of the first ~20-30 launches after an
idle GPU track the shader clock?  (DESIGN.md Measurements.)

Runs the driver's configs[1] pattern on the stamps build
(tools/build_variant.sh stamps -DCBN_STAMPS): 5 warm-up calls, a
synchronize and an idle gap, then 20 back-to-back calls (the timed region),
a synchronize, then 200 back-to-back calls.  For every launch of
k_query_staged<2>, block 0 / thread 0 records s_memtime (shader cycles) and
s_memrealtime (100 MHz) at entry and after its final stores (block 0 waits in
the grid barrier for every block, so that span is the launch's): duration =
realtime ticks x 10 ns, shader clock = cycles / duration.  Prints one JSON
line per phase and writes gpurun_out/clock_probe.json.

    CBN_LIB_PATH=continuousbayesiannetwork_amd/libcbn_amd_stamps.so python tools/clock_probe.py
"""
import ctypes
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import continuousbayesiannetwork_amd._native as nat  # noqa: E402

nat.LIB_PATH = os.environ.get("CBN_LIB_PATH", os.path.join(ROOT, "continuousbayesiannetwork_amd",
                                                           "libcbn_amd_stamps.so"))
from continuousbayesiannetwork_amd import BayesianNetwork  # noqa: E402
from helpers import chain_data, make_bn, sample_evidence  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    lib = nat.load()
    lib.cbn_debug_set_clock_buffer.argtypes = [ctypes.c_void_p]
    data, cols, edges = chain_data(20, 32, 200_000, 3, stay=0.8)
    target = "X19"
    names = [c for c in cols if c != target]
    bn = make_bn(BayesianNetwork, edges, cols, data, device=dev)
    base = {k: torch.tensor(v) for k, v in sample_evidence(data, cols, names, 65536, 1000).items()}
    g = torch.Generator().manual_seed(7)
    batches = [{k: v[torch.randperm(65536, generator=g) if b else torch.arange(65536)].contiguous().to(dev)
                for k, v in base.items()} for b in range(64)]
    ring = torch.zeros((4096, 4), dtype=torch.int64, device=dev)
    it = [0]

    def step():
        bn.infer(target, batches[it[0] % 64], N_max=32)
        it[0] += 1

    for _ in range(30):  # plan + tables + the runner path
        step()
    torch.cuda.synchronize()
    nat.check(lib.cbn_debug_set_clock_buffer(ctypes.c_void_p(ring.data_ptr())), "clock buffer")
    phases = []
    for _ in range(5):  # the driver's warm-up
        step()
    torch.cuda.synchronize()
    time.sleep(float(os.environ.get("IDLE_S", "0.002")))  # the idle gap before the timed region
    t0 = time.perf_counter()
    for _ in range(20):  # the driver's timed region
        step()
    torch.cuda.synchronize()
    t20 = time.perf_counter() - t0
    for _ in range(200):  # a long queued run
        step()
    torch.cuda.synchronize()
    n = 225
    r = ring[:n].cpu().numpy().astype(np.float64)
    cyc, ticks = r[:, 2] - r[:, 0], r[:, 3] - r[:, 1]
    us = ticks * 0.01
    ghz = cyc / (ticks * 10.0)
    gap = np.concatenate([[np.nan], (r[1:, 1] - r[:-1, 3]) * 0.01])  # idle between launches (block 0's view)
    out = {"launches": n, "timed_region_wall_us_per_step": round(t20 / 20 * 1e6, 2)}
    for name, sl in (("warmup_5", slice(0, 5)), ("timed_1_10", slice(5, 15)), ("timed_11_20", slice(15, 25)),
                     ("queued_1_30", slice(25, 55)), ("queued_31_200", slice(55, 225))):
        out[name] = dict(us=round(float(np.mean(us[sl])), 3), ghz=round(float(np.mean(ghz[sl])), 3),
                         gap_us=round(float(np.nanmean(gap[sl])), 3))
    out["per_launch"] = [dict(i=i, us=round(float(us[i]), 3), ghz=round(float(ghz[i]), 3),
                              gap_us=None if np.isnan(gap[i]) else round(float(gap[i]), 3)) for i in range(n)]
    out["corr_us_vs_ghz_first_60"] = round(float(np.corrcoef(us[5:65], ghz[5:65])[0, 1]), 3)
    print(json.dumps({k: v for k, v in out.items() if k != "per_launch"}), flush=True)
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    with open(os.path.join(ROOT, "gpurun_out", "clock_probe.json"), "w") as fh:
        json.dump(out, fh, indent=1)


if __name__ == "__main__":
    main()
