"""Diagnostic: per-step wall time of the fused infer and of the sharded
stepper (with and without an RCCL communicator), several rounds each, in one
process, in this order -- to see which one, and when, runs slow."""
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

from continuousbayesiannetwork_amd import BayesianNetwork  # noqa: E402
from continuousbayesiannetwork_amd.distributed import ShardedStepper  # noqa: E402
from helpers import chain_data, make_bn, sample_evidence  # noqa: E402

dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
data, cols, edges = chain_data(20, 32, 200_000, 3, stay=0.8)
bn = make_bn(BayesianNetwork, edges, cols, data, device=dev)
names = [c for c in cols if c != "X19"]
evs = [{k: torch.tensor(v, device=dev) for k, v in sample_evidence(data, cols, names, 65536, 1000 + i).items()}
       for i in range(int(os.environ.get("NB", "16")))]
K = 400
T0 = time.perf_counter()


def rounds(name, fn, after=None, n=3):
    for r in range(n):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(K):
            fn(evs[i % len(evs)])
        t1 = time.perf_counter()
        if after:
            after()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        print(f"t={t0 - T0:7.3f} {name} r{r}: enqueue {(t1 - t0) / K * 1e6:6.2f} wall {(t2 - t0) / K * 1e6:6.2f} us/step",
              flush=True)


_blk = None


def blocker(n_blocks):
    """A stand-in collective kernel on another stream once per group of 8 steps:
    n_blocks x 256 threads, 40 KB LDS each, ~25 us (tools/probes/blocker.hip)."""
    global _blk
    import ctypes

    if _blk is None:
        _blk = ctypes.CDLL(os.path.join(ROOT, "tools", "probes", "libblocker.so"))
        _blk.blocker_launch.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_longlong, ctypes.c_void_p]
    side = torch.cuda.Stream()
    count = [0]

    def hook():
        count[0] += 1
        if count[0] % 8 == 0:
            _blk.blocker_launch(n_blocks, 256, 40 * 1024, 25_000, ctypes.c_void_p(side.cuda_stream))
    return hook


def stepper(comm, fold, n_block=0, ring=0):
    st = ShardedStepper(bn, "X19", 32, force_exchange=comm, exchange_every=int(os.environ.get("G", "8")), fold=fold)
    hook = blocker(n_block) if n_block else None
    outs = [torch.empty((65536, 32), device=dev) for _ in range(ring)]
    k = [0]

    def step(e):
        if ring:
            k[0] += 1
            st.step(e, out=outs[k[0] % ring])
        else:
            st.step(e)
        if hook:
            hook()
    rounds(f"stepper comm={comm} fold={fold} blocker={n_block}", step, st.wait)
    st.close()


if os.environ.get("STREAM") == "1":  # a non-default current stream for everything
    torch.cuda.set_stream(torch.cuda.Stream())

for what in sys.argv[1:]:
    if what in ("pg_nccl", "pg_gloo"):  # a torch process group first, as bench.py has one
        import torch.distributed as dist

        for k, v in (("MASTER_ADDR", "127.0.0.1"), ("MASTER_PORT", "29541"), ("RANK", "0"), ("WORLD_SIZE", "1")):
            os.environ.setdefault(k, v)
        if what == "pg_nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group("gloo")
        print(f"t={time.perf_counter() - T0:7.3f} {what} initialised", flush=True)
        continue
    if what == "fused":
        rounds("fused", lambda e: bn.infer("X19", e, N_max=32))
    else:
        parts = what.split(",")
        stepper(parts[0] == "comm", parts[1] == "fold", int(parts[2]) if len(parts) > 2 else 0,
                int(parts[3]) if len(parts) > 3 else 0)
