"""Headline benchmark: BASELINE.json configs[1] -- 20-node discrete chain, d=32,
65 536 batched queries per GPU through ``BayesianNetwork.infer`` (the
reference's batched factor-product / mean-out / max-normalise loop,
bayesian_network.py:208-305) on the HIP engine.

One step = one ``infer`` call over one batch of 65 536 queries whose evidence
columns are already resident in HBM (target X19, evidence on X0..X18 -- the
reference's own benchmarking_df usage, every non-target column observed).
Each step runs both query passes over all queries (evidence -> domain index,
factor-row gather/product, global max, normalised write).  The factor tables
are plan constants (fitted CPDs x target x observed columns x N, independent
of evidence values) built once per plan; ``--rebuild-tables`` re-runs that
build every step, and the default run also reports that figure as
``value_rebuild_tables``.  N > 1 (``--gpus N`` starts N ranks itself through a
child ``torch.distributed.run`` unless it already runs under one): the batch
grows with N (weak scaling), each rank owns 65 536 queries and the ranks
exchange the global max with one RCCL all-reduce of the block max words
between the raw launch and the in-place scale, pipelined so a step's exchange
overlaps the next step's launch (distributed.ShardedStepper;
``--serial-exchange`` for the unpipelined step, ``--sharded`` runs that N>1
step at N=1 over a one-rank RCCL communicator).  At N > 1 ``value`` is
north_star's step: the shard's raw launch, the all-reduce + scale AND the RCCL
all-gather that reassembles the full [Q, N] marginal tensor on every rank
(``value_kind`` "gathered"); the step that leaves the tensor sharded is timed
after it as ``value_rank_local`` (``--rank-local`` swaps the two).  The line
carries DESIGN.md's ``projection`` for both at that N.  A rank that makes no
host progress for ``--watchdog`` seconds prints its step / ring state / last
collective and exits non-zero (distributed.Watchdog).

``timing`` itemises ms_per_step: host enqueue time per step, the GPU-side
event region, the same launches back-to-back with the queue held full (a
kernel duration independent of the host), and what lies outside the region
(first submit, final sync wake-up).

Prints ONE JSON line (rank 0).  Extra fields: ``roofline`` for the dominant
kernel -- the single-launch fused query kernel at N=1 (the write pass when the
two-launch path runs) -- timed with HIP events recorded by the library on the
launch stream inside the timed region; ``roofline.traffic`` = its per-launch
memory-side bytes from the committed rocprofv3 PMC summary of the same command
(profiles/<round>_summary.json, tools/profile_summary.py), null when absent;
``cpu_baseline`` = the CPU oracle (a restatement of the reference algorithm,
oracle/ref_infer.py) timed on a bounded sample on this host.
"""
from __future__ import annotations

import argparse
import json
import os
import random
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

from continuousbayesiannetwork_amd import BayesianNetwork  # noqa: E402
from continuousbayesiannetwork_amd.distributed import ShardedStepper, Watchdog  # noqa: E402
from helpers import chain_data, make_bn, sample_evidence  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: 8.0 TB/s spec
# xGMI: 7 links per GPU at ~153 GB/s each -- the figure of the task brief;
# the microarchitecture guide gives none, and whether 153 GB/s is per
# direction or both directions together is not stated.  Both readings are
# carried: the incoming peak is 7 x 153 if per direction, half
# of that if bidirectional.
XGMI_LINKS, XGMI_LINK_GBS = 7, 153.0
XGMI_PEAK_GBS = XGMI_LINKS * XGMI_LINK_GBS  # incoming, 153 GB/s per link per direction (assumed)
XGMI_PEAK_BIDIR_GBS = XGMI_PEAK_GBS / 2  # incoming, if 153 GB/s is the bidirectional per-link figure
LINK_ASSUMPTION = ("assumed: 7 xGMI links x 153 GB/s per GPU (task brief; not in MI355X_MICROARCH.md), taken as "
                   "per direction (incoming peak 1071 GB/s); '_if_bidirectional' fields take it as both directions "
                   "together (incoming 535.5 GB/s)")


def pmc_traffic(kernel: str):
    """Per-launch traffic (bytes) of ``kernel`` from the newest committed PMC
    summary (profiles/rNN_summary.json), with its source; (None, None) if none."""
    import glob

    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", "r*_summary.json")), reverse=True):
        try:
            with open(path) as fh:
                k = json.load(fh).get("kernels", {}).get(kernel, {})
        except (OSError, ValueError):
            continue
        if "traffic_bytes" in k:
            return k["traffic_bytes"], os.path.relpath(path, ROOT)
    return None, None


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--queries", type=int, default=65536, help="queries per GPU")
    ap.add_argument("--nodes", type=int, default=20)
    ap.add_argument("--card", type=int, default=32)
    ap.add_argument("--train-rows", type=int, default=200_000)
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="budget for the CPU oracle sample")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--batches", type=int, default=64,
                    help="distinct evidence batches cycled through (64 x 5 MB > the 256 MB Infinity Cache, so "
                         "evidence is read from HBM, not from a cache warmed by the previous step)")
    ap.add_argument("--no-touch", action="store_true",
                    help="do not read every evidence batch once on the device during setup (first-touch A/B)")
    ap.add_argument("--two-pass", action="store_true", help="force the two-launch (max, write) path")
    ap.add_argument("--sharded", action="store_true",
                    help="run the N>1 step (raw launch + RCCL all-reduce + scale, pipelined) even at N=1")
    ap.add_argument("--rank-local", action="store_true",
                    help="N>1: time the step WITHOUT the all-gather reassembly as `value` (each rank keeps its "
                         "normalised shard); by default `value` is north_star's step, with the RCCL all-gather of "
                         "the [Q, N] marginal tensor on every rank, and the rank-local step is timed after it "
                         "(value_rank_local)")
    ap.add_argument("--fold", action="store_true",
                    help="N>1 rank-local: fold each step's division into a later raw launch (cbn_plan_run_fold); "
                         "default only on a one-rank communicator (--sharded at N=1)")
    ap.add_argument("--watchdog", type=float, default=60.0,
                    help="N>1: seconds without host progress (a step, a wait, a barrier) after which a rank prints "
                         "its step index / ring state / last collective and exits non-zero")
    ap.add_argument("--serial-exchange", action="store_true",
                    help="N>1: no pipelining (each step's all-reduce + scale before the next raw launch)")
    ap.add_argument("--no-fold", action="store_true",
                    help="N>1 rank-local: a separate batched scale launch per group instead of each step's division "
                         "folded into a later raw launch (cbn_plan_run_fold)")
    ap.add_argument("--exchange-every", type=int, default=8,
                    help="N>1: steps per all-reduce + scale group (1..8)")
    ap.add_argument("--gather", action="store_true",
                    help="--sharded at N=1: time the step with the (one-rank) all-gather reassembly as `value`")
    ap.add_argument("--skip-other", action="store_true",
                    help="N>1: do not time the other reassembly choice after the headline step (profiling runs)")
    ap.add_argument("--rebuild-tables", action="store_true",
                    help="re-run k_build_tables in every step (the factor tables are plan constants; by default "
                         "they are built once per plan, as in serving)")
    return ap.parse_args(argv)


def free_port() -> int:
    import socket

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def rank_launch_command(gpus: int, argv, port: int, script: str = None):
    """The child command that runs this script as ``gpus`` ranks on one node
    (one process per GPU, torch.distributed.run, rendezvous on 127.0.0.1)."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={gpus}",
            "--master-addr=127.0.0.1", f"--master-port={port}", script or os.path.abspath(__file__), *argv]


def check_world(gpus: int, env) -> int:
    """World size this process runs in; --gpus and WORLD_SIZE must agree when
    both are given (a torch.distributed.run launch with a different rank count
    would time the wrong number of GPUs)."""
    w = env.get("WORLD_SIZE")
    if w is None:
        return 1
    if int(w) != gpus:
        raise SystemExit(f"bench.py: --gpus {gpus} but WORLD_SIZE={w} (launch with matching rank count)")
    return int(w)


def launch_ranks(a, argv, script: str = None) -> int:
    """``--gpus N > 1`` outside torch.distributed.run: start the N ranks as a
    CHILD process (never exec: nothing here has touched the GPU, and the
    parent only waits) and return its exit code (a rank that exits non-zero,
    e.g. on its watchdog, makes torch.distributed.run stop the others and
    return non-zero)."""
    import subprocess

    cmd = rank_launch_command(a.gpus, argv, free_port(), script=script)
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # dmabuf IPC (RCCL between the rank processes)
    print("bench.py: launching", " ".join(cmd), file=sys.stderr, flush=True)
    return subprocess.run(cmd, env=env).returncode


_ORACLE = None  # per-worker OracleBN of the CPU baseline pool


def _oracle_init(edges, cols, data):
    global _ORACLE
    from oracle.ref_infer import OracleBN

    _ORACLE = OracleBN(edges, cols, data)


def _oracle_ready(_):
    return _ORACLE is not None


def _oracle_chunk(args):
    target, sub, N = args
    return _ORACLE.infer_raw(target, sub, N)[0]


def host_cores() -> int:
    """CPU cores this process may use: its affinity set, capped by the
    OMP_NUM_THREADS share the GPU box sets (16 per GPU there)."""
    n = len(os.sched_getaffinity(0))
    omp = os.environ.get("OMP_NUM_THREADS")
    return max(1, min(n, int(omp))) if omp and omp.isdigit() else n


def cpu_baseline(data, cols, edges, ev_np, target, N, budget_s):
    """The oracle port timed on every host core: the query sample is split into
    one chunk per core (a fork pool -- created before anything touches the
    GPU), each worker runs the factor product of its chunk (the per-query work
    of bayesian_network.py:269-295), then the global-max division (:296) over
    the whole sample.  Worker setup (fitting the CPDs) is outside the timing."""
    import multiprocessing as mp

    cores = host_cores()
    with mp.get_context("fork").Pool(cores, initializer=_oracle_init, initargs=(edges, cols, data)) as pool:
        assert all(pool.map(_oracle_ready, range(cores), chunksize=1))
        q = 64 * cores
        t = 0.0
        while True:
            bounds = np.linspace(0, q, cores + 1).astype(int)
            jobs = [(target, {k: v[bounds[i]:bounds[i + 1]] for k, v in ev_np.items()}, N) for i in range(cores)]
            t0 = time.perf_counter()
            raw = np.concatenate(pool.map(_oracle_chunk, jobs, chunksize=1))
            _ = raw / raw.max()
            t = time.perf_counter() - t0
            if t > budget_s / 2 or q >= 65536:
                break
            q = min(65536, int(q * max(1.5, min(8.0, 0.8 * budget_s / max(t, 1e-3)))))
    return dict(value=q / t, unit="queries/s", cores=cores, kind="port",
                sample=f"oracle/ref_infer.py OracleBN factor products on the first {q} of the same queries, "
                       f"{cores} worker processes (numpy, one chunk each) + the global-max division; {t:.2f} s")


def step_modes(a, world: int) -> dict:
    """What the timed region measures (``value``) and what is timed after it.

    N > 1: north_star's configuration -- every rank runs its shard (one raw
    launch + the RCCL all-reduce(MAX) of the block max words + scale) AND the
    RCCL all-gather that reassembles the full [Q, N] marginal tensor on every
    rank -- is ``value``; the rank-local step (each rank keeps its normalised
    shard) is ``value_rank_local`` (``--rank-local`` swaps the two).  N = 1:
    the fused single launch (``--sharded``: the N>1 step over a one-rank
    communicator)."""
    sharded = world > 1 or a.sharded
    gather = (world > 1 and not a.rank_local) or (sharded and world == 1 and a.gather)
    fold = a.fold or (world == 1 and not a.no_fold)  # fold ring: one-rank only unless asked
    kind = ("gathered" if gather else "rank_local") if sharded else "single_process"
    other = ("rank_local" if gather else "gathered") if sharded and not a.skip_other else None
    if sharded:
        par = (f"query-shard x{world} + RCCL all-reduce(max) of the block max words"
               + (", serial" if a.serial_exchange else ", overlapped with the next step's launch")
               + (" + RCCL all-gather of the [Q, N] marginal tensor on every rank" if gather
                  else " (marginal tensor left sharded: no all-gather)"))
    else:
        par = f"query-shard x{world}"
    return dict(sharded=sharded, gather=gather, fold=fold, value_kind=kind, other_kind=other, parallelism=par)


def projection(world: int) -> dict:
    """DESIGN.md (Multi-GPU) bound on the gathered step: every rank receives
    (N-1) x 8.4 MB of rows per step over its 7 xGMI links and writes N x 8.4 MB
    of marginals -- a projection, not a measurement, under either reading of
    the link figure (LINK_ASSUMPTION)."""
    rows_b = 65536 * 32 * 4
    t_write = world * rows_b / (HBM_PEAK_GBS * 1e9)
    t_one = 10.3e-6
    t_ring = 16.7e-6  # step ring at N=1 (raw launch + batched scale + all-reduce): 15.7 us + ~1 us interference

    def gathered(peak_gbs):
        t_link = (world - 1) * rows_b / (peak_gbs * 1e9)
        return round(world * t_one / max(t_ring, t_link, t_write), 2)

    return {"gathered_x_vs_1gpu": gathered(XGMI_PEAK_GBS),
            "gathered_x_vs_1gpu_if_bidirectional": gathered(XGMI_PEAK_BIDIR_GBS),
            "rank_local_x_vs_1gpu": round(world * t_one / t_ring, 2) if world > 1 else 1.0,
            "link_assumption": LINK_ASSUMPTION,
            "status": "projection, not a measurement: no run with >= 2 GPUs has pinned these figures",
            "basis": "DESIGN.md Multi-GPU: gathered step >= max(16.7 us step-ring GPU time, (N-1) x 8.4 MB over "
                     "the incoming xGMI peak, N x 8.4 MB written at 8 TB/s); rank-local = the step ring (the folded "
                     "ring is one-rank only until a 2-GPU run pins it): 15.7 us per step measured at N=1 + ~1 us of "
                     "collective interference, vs the fused single-GPU 10.3 us"}


def multi_gpu_fields(gpus: int, world: int, rccl_ranks) -> dict:
    """The N > 1 self-checks of the JSON line: ``rccl_ranks`` = the ranks of
    the stepper's own RCCL communicator as ncclCommCount reports them (None
    when the step uses none), which must equal --gpus; plus the projection."""
    if rccl_ranks is not None and rccl_ranks != gpus:
        raise SystemExit(f"bench.py: --gpus {gpus} but the stepper's RCCL communicator has {rccl_ranks} ranks")
    out = {"rccl_ranks": rccl_ranks}
    if world > 1:
        out["projection"] = projection(world)
    return out


def reference_over_port():
    """Ratio of the reference's own CPU path to the oracle port at equal cores
    (profiles/r02_cpu_reference.json: 8 single-thread processes each), or None."""
    try:
        with open(os.path.join(ROOT, "profiles", "r02_cpu_reference.json")) as fh:
            d = json.load(fh)
        ref = max(r["queries_per_s"] for r in d["reference"] if r["threads"] * r["processes"] == 8)
        port = max(r["queries_per_s"] for r in d["port"] if r["processes"] == 8)
        return round(ref / port, 3)
    except (OSError, ValueError, KeyError):
        return None


def backlogged_launch_us(step, K: int, stream) -> float:
    """Average duration of K back-to-back steps with the launch queue full: the
    stream is first held by a spin kernel long enough for the host to enqueue
    all K steps, so the HIP events around them see no host gaps (a kernel
    duration, comparable with rocprofv3's, whatever the host's enqueue speed)."""
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
    ev[0].record(stream)
    torch.cuda._sleep(1_000_000)
    ev[1].record(stream)
    torch.cuda.synchronize()
    per_cycle_ms = ev[0].elapsed_time(ev[1]) / 1_000_000
    t0 = time.perf_counter()
    for _ in range(4):
        step()
    torch.cuda.synchronize()
    host_ms = (time.perf_counter() - t0) / 4 * 1e3
    torch.cuda._sleep(int(min(2e9, 3.0 * K * host_ms / max(per_cycle_ms, 1e-9) + 1e6)))
    ev[2].record(stream)
    for _ in range(K):
        step()
    ev[3].record(stream)
    torch.cuda.synchronize()
    return ev[2].elapsed_time(ev[3]) / K * 1e3


def main():
    a = parse()
    if a.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(a, sys.argv[1:]))  # N ranks as a child torch.distributed.run
    world = check_world(a.gpus, os.environ)
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    modes = step_modes(a, world)
    sharded, gather = modes["sharded"], modes["gather"]
    n, d, Q = a.nodes, a.card, a.queries
    target = f"X{n - 1}"
    data, cols, edges = chain_data(n, d, a.train_rows, 3, stay=0.8)
    names = [c for c in cols if c != target]
    ev_np = sample_evidence(data, cols, names, Q, seed=1000 + rank)
    cpu = None
    if rank == 0 and not sharded and not a.no_cpu_baseline:
        # first, while no process has touched the GPU: its worker pool forks
        cpu = cpu_baseline(data, cols, edges, ev_np, target, d, a.cpu_seconds)
    wd = None
    if sharded:
        torch.cuda.set_device(local)
        if "WORLD_SIZE" not in os.environ:  # --sharded outside torch.distributed.run: a one-rank group
            for k, v in (("MASTER_ADDR", "127.0.0.1"), ("MASTER_PORT", str(free_port())), ("RANK", "0"),
                         ("WORLD_SIZE", "1")):
                os.environ.setdefault(k, v)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        if world > 1:
            # bounded N>1 run: a rank stuck in a collective reports and exits
            wd = Watchdog(a.watchdog, what="(bench.py N>1)")
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)

    bn = make_bn(BayesianNetwork, edges, cols, data, device=dev)
    bn.engine.cache_tables = not a.rebuild_tables
    bn.engine.fused = not a.two_pass
    # B distinct batches: the first is ev_np; the others are row permutations of it
    g = torch.Generator().manual_seed(7 + rank)
    base = {k: torch.tensor(v) for k, v in ev_np.items()}
    batches = []
    for b in range(max(1, a.batches)):
        perm = torch.randperm(Q, generator=g) if b else torch.arange(Q)
        batches.append({k: v[perm].contiguous().to(dev) for k, v in base.items()})
    if not a.no_touch:
        # setup, untimed: read every uploaded column once on the device (the
        # inputs are resident in HBM AND mapped when the timed region starts;
        # a batch's first read otherwise pays its page-table walks inside a step)
        chk = torch.zeros((), device=dev)
        for ev in batches:
            for v in ev.values():
                chk += v.sum()
        torch.cuda.synchronize()
    it = [0]
    # N>1: one raw launch per step on the compute stream; the all-reduce(MAX)
    # of the block max words + the in-place scale (+ the all-gather) run on a
    # comm stream, once per --exchange-every steps (8) for all of them, so the
    # exchange overlaps the next steps' launches (distributed.ShardedStepper)
    stepper = ShardedStepper(bn, target, d, exchange_every=1 if a.serial_exchange else a.exchange_every,
                             force_exchange=sharded, gather=gather, fold=modes["fold"], watchdog=wd)
    if wd is not None:
        wd.describe = lambda: stepper.describe()

    def step():
        ev = batches[it[0] % len(batches)]
        it[0] += 1
        if sharded:
            rows = stepper.step(ev, total_rows=Q * world if stepper.gather else None)
            if a.serial_exchange:
                stepper.wait()
            return rows
        return bn.infer(target, ev, N_max=d)

    def barrier(what):
        if wd is not None:
            wd.beat(op=f"barrier ({what})")
            stepper.last_op = f"dist.barrier ({what})"
        dist.barrier()

    def timed_steps(K):
        """K steps between barriers + device syncs; max over ranks of the wall time."""
        if sharded:
            barrier("before the second timed region")
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(K):
            step()
        stepper.wait()
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        if sharded:  # outside the clock: the MAX over ranks below covers the slowest rank
            barrier("after the second timed region")
        dt = torch.tensor([t1 - t0], dtype=torch.float64, device=dev)
        if world > 1:
            dist.all_reduce(dt, op=dist.ReduceOp.MAX)
        return float(dt.item())

    if wd is not None:
        wd.arm(phase="warmup")
    K = a.steps
    stream = torch.cuda.current_stream(dev)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    random.seed(0)
    for _ in range(a.warmup):
        step()
    # everything the timed region needs is ready before its opening barrier +
    # synchronize, so the GPU goes idle only for that synchronize (a longer
    # idle gap before the first timed launch measurably slows the first
    # launches: profiles/r04_driver_cmd_timeline.json)
    fused = not sharded and not a.two_pass and bn.engine.fused_capacity(target, names, d) >= Q
    bn.engine.timing()  # drop warm-up timings (none on the fused path)
    stepper.wait()
    if wd is not None:
        wd.beat(phase="timed region")
    if sharded:
        barrier("before the timed region")
    torch.cuda.synchronize()
    # the library launches on torch's current stream: these events bracket
    # every launch (instrumentation, recorded before the host clock starts)
    ev0.record()
    t0 = time.perf_counter()
    per_step_events = not sharded and not fused
    for i in range(K):
        # two-launch path: HIP events recorded inside the library around the
        # passes of every 8th step (the sharded step and the fused launch are
        # timed over the region: per-step event records cost ~3 us per step)
        if per_step_events:
            bn.engine.timed = i % 8 == 7
        step()
    t_enq = time.perf_counter()  # host done enqueueing the K steps
    stepper.wait()
    ev1.record()
    torch.cuda.synchronize()
    t_sync = time.perf_counter()
    t1 = t_sync
    if sharded:
        # the closing barrier is outside the clock (a one-rank RCCL barrier
        # alone took 288 us, 1.4 us per step of a 200-step run): each rank
        # times its own K steps, collectives included, and the MAX over
        # ranks below is the slowest rank's
        barrier("after the timed region")
    bn.engine.timed = False
    dt = torch.tensor([t1 - t0], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(dt, op=dist.ReduceOp.MAX)
    sec = float(dt.item())
    ms_per_step = sec / K * 1e3
    value = Q * world * K / sec
    region_us = ev0.elapsed_time(ev1) * 1e3  # GPU-side: first event -> last event on the launch stream
    timing = {"host_enqueue_us_per_step": round((t_enq - t0) / K * 1e6, 3),
              "tail_us": round((t_sync - t_enq) * 1e6, 2),
              "region_events_us_per_step": round(region_us / K, 3),
              "outside_region_us": round((t_sync - t0) * 1e6 - region_us, 2)}
    if sharded:
        timing["barrier_us"] = round((time.perf_counter() - t_sync) * 1e6, 2)  # not in `value`
        c = getattr(stepper, "_c", None)
        if c is not None and hasattr(c, "host_timing"):  # the step ring's native phases (us per step)
            ht = c.host_timing()
            timing["stepper_host_us"] = {"gather_alloc": round(ht[0], 2), "launch_and_exchange": round(ht[1], 2)}

    roofline = None
    ntimed, tmax_ms, twrite_ms = bn.engine.timing() if not sharded else (0, 0.0, 0.0)
    bn.engine.check_status()
    if fused:
        # one launch per step: average launch duration = HIP-event time of the timed region / K
        ntimed, twrite_ms = K, region_us / K * 1e-3
        # the same launches with the queue kept full (no host gaps): a kernel duration
        kb = backlogged_launch_us(step, max(K, 100), stream)
        timing["backlogged_us_per_launch"] = round(kb, 3)
        timing["gpu_idle_us_per_step"] = round(region_us / K - kb, 3)
        timing["itemised"] = (f"{ms_per_step * 1e3:.2f} us/step = {kb:.2f} kernel (back-to-back) + "
                              f"{region_us / K - kb:.2f} GPU idle inside the event region (launch gaps: host "
                              f"enqueue {(t_enq - t0) / K * 1e6:.2f} us/step) + "
                              f"{((t_sync - t0) * 1e6 - region_us) / K:.2f} outside it (first submit + final "
                              f"sync wake-up, {(t_sync - t0) * 1e6 - region_us:.1f} us over {K} steps) + "
                              f"{(t1 - t_sync) * 1e6 / K:.2f} after the sync")
    if ntimed:
        tmax, twrite = tmax_ms * 1e-3, twrite_ms * 1e-3
        n_cols = len(names)  # evidence columns read per query
        bytes_q = Q * (4 * n_cols + 4 * d)  # evidence floats in + pdf row out
        from continuousbayesiannetwork_amd import _native

        plan = next(iter(bn.engine._plans.values()))
        pflags = _native.load().cbn_plan_flags(plan.handle)
        vpl = 2 if pflags & _native.CBN_PLAN_VPL2 else 1
        nptr = 128 if 4 * n <= 128 else 416  # kernel-argument pointer table sized to the plan (n factors)
        # the dominant kernel: fused single launch; beyond its capacity the raw
        # compute pass (then an HBM-bound scale); --two-pass: the write pass
        mode, what, t_dom = ((2, "single launch: both passes", twrite) if fused else
                             (1, "write pass", twrite) if a.two_pass else (3, "raw compute pass", tmax))
        kname = (f"k_query_staged<{mode}>" if pflags & _native.CBN_PLAN_STAGED
                 else f"k_query_fast<{vpl}, true, {mode}, {nptr}>")  # <MODE> / <VPL, LDS, MODE, NP>
        achieved = bytes_q / t_dom / 1e9
        traffic, tsrc = pmc_traffic(kname)
        roofline = dict(bound="hbm", achieved=round(achieved, 1), peak=HBM_PEAK_GBS, unit="GB/s",
                        frac=round(achieved / HBM_PEAK_GBS, 4), traffic=traffic, kernel=f"{kname} ({what})",
                        avg_us=round(t_dom * 1e6, 2), algorithmic_bytes_per_launch=bytes_q, timed_steps=ntimed)
        if tsrc:
            roofline["traffic_source"] = tsrc + " (2 x FETCH_SIZE + WRITE_SIZE per dispatch)"
        roofline["timing"] = ("HIP events on the launch stream around the whole timed region / K launches" if fused
                              else "HIP events around the launches of every 8th step (library-side)")
        if fused:
            kb = timing["backlogged_us_per_launch"] * 1e-6
            roofline["avg_us_backlogged"] = round(kb * 1e6, 2)
            roofline["frac_backlogged"] = round(bytes_q / kb / 1e9 / HBM_PEAK_GBS, 4)
        if not fused:
            roofline["first_launch_us"], roofline["second_launch_us"] = round(tmax * 1e6, 2), round(twrite * 1e6, 2)
    if sharded and gather and world > 1:
        # with the reassembly, each rank receives the other ranks' rows every
        # step over xGMI: (world - 1) x Q x 4N bytes -- the dominant transfer
        t_step = region_us / K * 1e-6
        bytes_in = (world - 1) * Q * 4 * d
        achieved = bytes_in / t_step / 1e9
        roofline = dict(bound="xgmi", achieved=round(achieved, 1), peak=XGMI_PEAK_GBS, unit="GB/s",
                        frac=round(achieved / XGMI_PEAK_GBS, 4), traffic=None,
                        peak_if_bidirectional=XGMI_PEAK_BIDIR_GBS,
                        frac_if_bidirectional=round(achieved / XGMI_PEAK_BIDIR_GBS, 4), peak_source=LINK_ASSUMPTION,
                        kernel="sharded step: raw launch + ncclAllReduce(MAX) + k_scale_batch + ncclAllGather of "
                               "the [Q, N] rows (per step)",
                        avg_us=round(t_step * 1e6, 2), algorithmic_bytes_per_launch=bytes_in, timed_steps=K,
                        timing="HIP events on rank 0's launch stream around the timed region / K steps; bytes = "
                               "rows received from the other ranks per step")
    elif sharded:
        # rank-local sharded step: ONE raw launch per step on the launch stream
        # (folded: it also divides an earlier step's rows by that step's
        # all-reduced max, cbn_plan_run_fold; else k_scale_batch per group on
        # the comm stream); algorithmic bytes of that launch = evidence in +
        # raw rows out + the rows read and written back by the division;
        # duration = HIP events on the launch stream around the timed region / K
        n_cols = len(names)
        bytes_step = Q * (4 * n_cols + 3 * 4 * d)
        t_step = region_us / K * 1e-6
        achieved = bytes_step / t_step / 1e9
        folded = getattr(stepper, "_folded", False)
        kname = "k_query_staged<3>"
        traffic, tsrc = pmc_traffic(kname)
        roofline = dict(bound="hbm", achieved=round(achieved, 1), peak=HBM_PEAK_GBS, unit="GB/s",
                        frac=round(achieved / HBM_PEAK_GBS, 4), traffic=traffic,
                        kernel=kname + (" (raw launch with an earlier step's scale folded in)" if folded
                                        else " (raw launch; k_scale_batch on the comm stream per group)"),
                        avg_us=round(t_step * 1e6, 2), algorithmic_bytes_per_launch=bytes_step, timed_steps=K,
                        timing="HIP events on the launch stream around the timed region / K steps")
        if tsrc:
            roofline["traffic_source"] = tsrc + " (2 x FETCH_SIZE + WRITE_SIZE per dispatch)"

    rccl_ranks = stepper.comm_ranks() if sharded else None  # before close(): the headline step's communicator
    other = None
    if modes["other_kind"] is not None:
        # the same step with the other reassembly choice: each rank keeping its
        # rows (value_rank_local) or, with --rank-local, the all-gather of the
        # full [Q, N] tensor on every rank (value_gathered)
        if wd is not None:
            wd.beat(phase="second timed region (" + modes["other_kind"] + ")")
        stepper.close()
        stepper = ShardedStepper(bn, target, d, exchange_every=1 if a.serial_exchange else a.exchange_every,
                                 force_exchange=True, gather=not gather, fold=modes["fold"], watchdog=wd)
        for _ in range(a.warmup):
            step()
        stepper.wait()
        other = Q * world * K / timed_steps(K)

    cold = None
    if not sharded and not a.rebuild_tables:
        bn.engine.cache_tables = False
        for _ in range(5):
            step()
        torch.cuda.synchronize()
        kc = max(10, K // 4)
        t0 = time.perf_counter()
        for _ in range(kc):
            step()
        torch.cuda.synchronize()
        cold = Q * kc / (time.perf_counter() - t0)
        bn.engine.cache_tables = True

    if rank == 0:
        if cpu is not None:
            r = reference_over_port()
            if r is not None:
                cpu["reference_over_port"] = r
                cpu["reference_over_port_source"] = ("profiles/r02_cpu_reference.json: the reference's own infer "
                                                     "vs this port, 8 single-thread processes each, same queries")
        line = {
            "metric": "marginal queries/sec + achieved HBM GB/s, 20-node d=32 DAG, 65k-batch VE",
            "value": round(value, 1), "unit": "queries/s", "n_gpus": world, "steps": K, "warmup": a.warmup,
            "ms_per_step": round(ms_per_step, 5), "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "f32", "data": "synthetic (seeded chain samples; BruteForce fit)",
            "config": {"workload": f"chain{n}_d{d}: BayesianNetwork.infer target {target}, evidence on the other "
                                   f"{n - 1} nodes, N_max={d}", "queries_per_gpu": Q, "global_batch": Q * world,
                       "parallelism": modes["parallelism"]},
            "value_kind": modes["value_kind"],
            "roofline": roofline, "cpu_baseline": cpu, "timing": timing,
            "tables": "rebuilt every step" if a.rebuild_tables else "built once per plan",
            "evidence_batches": len(batches),
        }
        line.update(multi_gpu_fields(a.gpus, world, rccl_ranks))
        if cold is not None:
            line["value_rebuild_tables"] = round(cold, 1)
        if other is not None:
            line["value_" + modes["other_kind"]] = round(other, 1)
        if cpu:
            line["speedup_vs_cpu_baseline"] = round(value / cpu["value"], 1)
            if cpu.get("reference_over_port"):
                line["speedup_vs_reference_cpu"] = round(value / (cpu["value"] * cpu["reference_over_port"]), 1)
        assert line["n_gpus"] == a.gpus, (line["n_gpus"], a.gpus)
        print(json.dumps(line), flush=True)
    if sharded:
        stepper.close()
        if wd is not None:
            wd.close()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
