"""Query-batch sharding over the GPUs of one node (one process per GPU, RCCL).

The reference's ``infer`` (bayesian_network.py:269-296) normalises the whole
batch by ONE global max, so a batch split over ranks has exactly one exchange
step between the two query passes: an all-reduce(MAX) of a single 4-byte word
(the float bits of the local max -- all values are >= 0, so integer order is
float order).  Re-assembling the marginal tensor on every rank is optional
(``gather=True``: all-gather of the [q_r, N] shards over xGMI); without it each
rank keeps the rows it owns.
"""
from __future__ import annotations

import os
import random
import sys
import threading
import time
from contextlib import contextmanager
from typing import Callable, Dict, Optional, Tuple

import torch
import torch.distributed as dist

from .base.parameter_learning import GENERATION

_RAW = 8  # CBN_RUN_RAW (include/cbn_amd.h)


class Watchdog:
    """Bound on a multi-rank run: a rank whose host makes no progress for
    ``bound_s`` seconds (a peer that stopped issuing steps leaves it blocked
    in a collective or a device wait) prints what it was doing and exits the
    process with ``code`` (``os._exit``: no re-exec, no retry, no cleanup that
    could block on the dead collective).  The launcher then sees a non-zero
    rank and returns non-zero.

    ``beat(**state)`` records progress (and what the rank is doing);
    ``describe`` (optional) adds live state -- a ShardedStepper's ring -- to
    the report.  The every-rank exchange this guards is the reference's one
    global max (bayesian_network.py:296): every rank must pair it each step.
    Blocking native waits release the GIL (csrc/host_fast.cpp), so the thread
    runs while the main thread is stuck in one."""

    def __init__(self, bound_s: float, what: str = "", describe: Optional[Callable[[], str]] = None,
                 code: int = 3, stream=None):
        self.bound = float(bound_s)
        self.what = what
        self.describe = describe
        self.code = code
        self.stream = stream if stream is not None else sys.stderr
        self.state: Dict[str, object] = {}
        self._last = time.monotonic()
        self._armed = False
        self._stop = threading.Event()
        self._thread = threading.Thread(target=self._run, name="cbn-watchdog", daemon=True)
        self._thread.start()

    def arm(self, **state):
        self.beat(**state)
        self._armed = True

    def disarm(self):
        self._armed = False

    def beat(self, **state):
        # copy-on-write: the watchdog thread's report() iterates whatever dict
        # it read, never one being resized under it
        if state:
            self.state = {**self.state, **state}
        self._last = time.monotonic()

    def close(self):
        self._armed = False
        self._stop.set()
        self._thread.join(timeout=5)

    def report(self) -> str:
        rank = os.environ.get("RANK", "?")
        world = os.environ.get("WORLD_SIZE", "?")
        parts = [f"[cbn watchdog] rank {rank}/{world}: no progress for {time.monotonic() - self._last:.1f} s "
                 f"(bound {self.bound:.1f} s) {self.what}".rstrip(),
                 "  state: " + ", ".join(f"{k}={v}" for k, v in dict(self.state).items())]
        if self.describe is not None:
            try:
                parts.append("  " + self.describe())
            except Exception as e:  # the report must not fail on a half-torn-down stepper
                parts.append(f"  (describe failed: {e!r})")
        return "\n".join(parts)

    def _run(self):
        tick = min(1.0, max(0.05, self.bound / 8))
        while not self._stop.wait(tick):
            if self._armed and time.monotonic() - self._last > self.bound:
                try:
                    print(self.report(), file=self.stream, flush=True)
                finally:
                    os._exit(self.code)


def shard_bounds(n: int, world: int, rank: int) -> Tuple[int, int]:
    """Contiguous, balanced [lo, hi) slice of n queries for ``rank``."""
    base, rem = divmod(n, world)
    lo = rank * base + min(rank, rem)
    return lo, lo + base + (1 if rank < rem else 0)


def shard_evidence(evidence: Dict[str, torch.Tensor], world: int, rank: int) -> Dict[str, torch.Tensor]:
    if not evidence:
        return evidence
    n = next(iter(evidence.values())).shape[0]
    lo, hi = shard_bounds(n, world, rank)
    return {k: v[lo:hi] for k, v in evidence.items()}


def normalise_across_ranks(local_max: Callable[[], torch.Tensor],
                           local_write: Callable[[torch.Tensor], torch.Tensor],
                           group=None, gather: bool = False, total_rows: Optional[int] = None) -> torch.Tensor:
    """Run pass 1 locally, all-reduce(MAX) the max word, run pass 2 locally.

    ``local_max()`` returns an int32 tensor [1] holding float bits;
    ``local_write(bits)`` returns this rank's [q_r, N] rows.
    """
    bits = local_max()
    if dist.is_initialized() and dist.get_world_size(group) > 1:
        dist.all_reduce(bits, op=dist.ReduceOp.MAX, group=group)
    out = local_write(bits)
    if not gather or not dist.is_initialized() or dist.get_world_size(group) == 1:
        return out
    return gather_rows(out, group, total_rows)


def gather_rows(out: torch.Tensor, group=None, total_rows: Optional[int] = None) -> torch.Tensor:
    """All-gather every rank's [q_r, N] rows (uneven q_r) into the full tensor, rank order."""
    world = dist.get_world_size(group)
    n = out.new_tensor([out.shape[0]], dtype=torch.int64)
    sizes = [torch.zeros_like(n) for _ in range(world)]
    dist.all_gather(sizes, n, group=group)
    sizes = [int(s.item()) for s in sizes]
    m = max(sizes)
    pad = out.new_zeros((m, out.shape[1]))
    pad[: out.shape[0]] = out
    parts = [torch.empty_like(pad) for _ in range(world)]
    dist.all_gather(parts, pad, group=group)
    full = torch.cat([p[:s] for p, s in zip(parts, sizes)], 0)
    if total_rows is not None:
        assert full.shape[0] == total_rows
    return full


@contextmanager
def shared_draws(group=None):
    """Every rank of ``group`` uses rank 0's sample_domain draws inside the
    block (node.py:302-333 pads a domain smaller than N with random.uniform
    values; a sharded call must use ONE set of them, as the single process
    does).  Rank 0 draws from its own ``random`` in the reference's order and
    broadcasts the values when the block ends (also on error, so no rank
    waits forever); every other rank receives them at its first draw and
    replays them, and checks it used exactly as many."""
    from .base import node as node_mod

    rank = dist.get_rank(group)
    src = dist.get_global_rank(group, 0) if group is not None else 0
    if node_mod._DRAWS[0] is not None:
        raise RuntimeError("shared_draws blocks do not nest")
    if rank == 0:
        rec = []

        def draw(n):
            v = [random.random() for _ in range(n)]
            rec.extend(v)
            return v

        node_mod._DRAWS[0] = draw
        try:
            yield
        finally:
            node_mod._DRAWS[0] = None
            dist.broadcast_object_list([rec], src=src, group=group)
        return
    st = {"vals": None, "pos": 0}

    def recv():
        obj = [None]
        dist.broadcast_object_list(obj, src=src, group=group)
        st["vals"] = obj[0]

    def draw(n):
        if st["vals"] is None:
            recv()
        v = st["vals"][st["pos"]:st["pos"] + n]
        if len(v) != n:
            raise RuntimeError("ranks disagree on the number of sample_domain draws of this call")
        st["pos"] += n
        return v

    node_mod._DRAWS[0] = draw
    try:
        yield
    finally:
        node_mod._DRAWS[0] = None
        if st["vals"] is None:
            recv()
    if st["pos"] != len(st["vals"]):
        raise RuntimeError("ranks disagree on the number of sample_domain draws of this call")


def sharded_infer(bn, target_node: str, evidence_shard: Dict[str, torch.Tensor], N_max: int = 16,
                  group=None, gather: bool = False, out: Optional[torch.Tensor] = None):
    """``BayesianNetwork.infer`` over a query batch sharded across ranks.

    Each rank passes its own rows of the evidence; the result equals the rows
    of the single-process ``infer`` on the concatenated batch.

    Fast-path plans: ONE launch per rank stores the unnormalised rows and the
    rank's max word, RCCL all-reduces the word (MAX), and an in-place scale
    launch divides by the global max.  Other plans: max pass, all-reduce,
    write pass.  Plans whose sample domains are redrawn on every call (N_max
    above a sampled variable's domain size) use rank 0's draws on every rank
    (``shared_draws``), so every rank's rows are those of the single process.
    """
    eng = bn.engine
    multi = dist.is_initialized() and dist.get_world_size(group) > 1
    if multi and eng.redraws(target_node, evidence_shard.keys(), N_max):
        with shared_draws(group):
            plan, fp = eng.call_plan(target_node, evidence_shard, N_max)
    else:
        plan, fp = eng.call_plan(target_node, evidence_shard, N_max)
    try:
        return _sharded_on_plan(eng, plan, fp, target_node, evidence_shard, N_max, group, gather, out, multi)
    finally:
        if not plan.deterministic and not plan.reusable:  # a plan rebuilt per call
            torch.cuda.current_stream().synchronize()
            plan.destroy()


def _sharded_on_plan(eng, plan, fp, target_node, evidence_shard, N_max, group, gather, out, multi):
    n = next(iter(evidence_shard.values())).shape[0] if evidence_shard else 1
    wide = set()
    if n == 0:  # no launch checks an empty shard's columns: raise the reference's shape errors here
        wide = eng.check_columns(plan, evidence_shard)  # ([Q, N] columns: the wide direct plan's raw launch)
    raw = eng.infer_raw(target_node, evidence_shard, N_max, out, fp=fp) if (fp is not None and n > 0) else None
    if raw is None and multi and fp is not None and (fp.words is not None or wide) and n == 0:
        # an empty shard on a raw-capable plan: no rows, zero max words -- the
        # same collectives as the other ranks
        rows = torch.empty((0, plan.n_samples), dtype=torch.float32, device=fp.device)
        bits = (torch.zeros(eng.wide_word_count(plan, wide, fp.device), dtype=torch.int32, device=fp.device)
                if wide else torch.zeros_like(fp.words))
        raw = (rows, plan.target_domain.unsqueeze(0).expand(0 if plan.target_observed else 1, -1), bits,
               lambda r, b: r)
    # the path must be the same on every rank (different collectives would hang):
    # take the raw path only where every rank can
    ok = torch.tensor([1 if raw is not None else 0], dtype=torch.int32)
    if multi:
        if dist.get_backend(group) == "nccl":
            ok = ok.to(torch.device("cuda", torch.cuda.current_device()))
        dist.all_reduce(ok, op=dist.ReduceOp.MIN, group=group)
    if int(ok.item()) == 1:
        rows, tdom, bits, scale = raw
        if multi:
            dist.all_reduce(bits, op=dist.ReduceOp.MAX, group=group)
        scale(rows, bits)
        if gather and multi:
            rows = gather_rows(rows, group)
        return rows, tdom
    # (a raw pass this rank launched that another rank cannot take is redone
    # two-pass below, stream-ordered after it)
    cols, nq, tdom, device = eng.prepare_plan(plan, evidence_shard)
    if out is None:
        out = torch.empty((nq, plan.n_samples), dtype=torch.float32, device=device)

    def local_max():
        return eng.query_max(plan, cols, nq, device)

    def local_write(bits):
        return eng.query_write(plan, cols, nq, bits, out, device)

    res = normalise_across_ranks(local_max, local_write, group=group, gather=gather)
    return res, tdom


class ShardedStepper:
    """Pipelined ``sharded_infer`` for a stream of query batches (serving /
    the multi-GPU bench): the exchange of a group of steps overlaps the next
    steps' raw launches.

    Per step, in ONE native host call (``_cbn_host.Stepper``), on the
    caller's (compute) stream: ONE raw launch (unnormalised rows + per-block
    max words into a ring slot).  Every ``exchange_every`` steps (G), on the
    stepper's comm stream: wait for the group's last launch, ONE
    ``ncclAllReduce(MAX)`` over the group's G x W words on our own RCCL
    communicator, ONE ``cbn_scale_batch`` launch dividing each step's rows by
    its own global max, and -- ``gather=True``, the north star's reassembly --
    each step's RCCL all-gather of the rank shards into the full [Q, N]
    marginal tensor over xGMI (in place: a rank's raw launch writes its rows at
    its offset of the full tensor; equal shards: ncclAllGather, uneven: one
    ncclBroadcast per rank in one group).  The per-exchange host costs are
    paid once per G steps and the RCCL latency hides behind the next group's
    launches.  (The same choreography in Python -- events, stream switch, c10d
    all_reduce, record_stream -- cost ~50 us of host time per step:
    tools/shard_step_probe.py.)  The ring/group bookkeeping is
    ``StepRing`` (csrc/host_fast.cpp), exercised on CPU by a world-size-2 gloo
    test through the same class (``_cbn_host.CpuStepRing``).

    A step's rows are final once its group has been exchanged: call
    ``wait()`` (exchanges a partial group; the current stream then waits for
    the comm stream) before reading them.  Results equal ``sharded_infer`` (and
    the single-process ``infer`` on the concatenated batch) bit for bit.
    Every rank calls ``step`` and ``wait`` the same number of times, in the
    same order (the exchanges are collectives); an empty shard is a valid step
    (zero max words, no rows), and evidence the native checks reject is
    converted and goes through the same ring, so no rank leaves the pipeline
    on its own.  Plans without a raw launch use the serial ``sharded_infer``.
    """

    def __init__(self, bn, target_node: str, N_max: int = 16, group=None, exchange_every: int = 4,
                 force_exchange: bool = False, gather: bool = False, fold: Optional[bool] = None,
                 watchdog: Optional[Watchdog] = None):
        self.bn, self.target, self.N_max, self.group = bn, target_node, N_max, group
        multi = dist.is_initialized() and dist.get_world_size(group) > 1
        # rank-local steps on staged plans: each step's division by its global
        # max runs inside a later raw launch (cbn_plan_run_fold, FoldStepper)
        # instead of a separate scale launch.  Default: only on a one-rank
        # communicator -- the fold ring's host hand-off has not yet run against
        # real peers on GPUs (tests/test_gpu_multi.py pins it when >= 2 GPUs
        # are visible), so with peers the separate batched scale is used
        self.fold = (not multi) if fold is None else fold
        # progress reporting for a bounded multi-rank run (bench.py)
        self.watchdog = watchdog
        self.n_steps = 0
        self.last_op = "none"
        # steps per exchange group: <= 8 for the separate batched scale (one
        # cbn_scale_batch per group), <= 32 when the scales are folded
        self.G_req = max(1, exchange_every)
        self.G = min(8, self.G_req)
        # force_exchange: all-reduce even at world size 1 (exercises RCCL on one GPU)
        multi = dist.is_initialized() and dist.get_world_size(group) > 1
        self.exchange = force_exchange or multi
        self.world = dist.get_world_size(group) if multi else 1
        self.rank = dist.get_rank(group) if multi else 0
        self.gather = gather
        self._c = None
        self._fp = None
        self._comm = 0
        self._serial = False
        self._folded = False
        self._epoch = None  # engine.epoch the native stepper's plan handle belongs to
        self._hot_counts = {}  # total_rows -> every rank's rows (gather=True step ring), for the hot path

    def _setup(self, evidence_shard) -> bool:
        import ctypes
        import os

        from . import _native

        eng = self.bn.engine
        fp = eng.raw_fast_path(self.target, evidence_shard, self.N_max)
        if fp is None:
            return False
        self._epoch = eng.epoch
        host = _native.load_host()
        if self.exchange and not self._comm:  # (kept across plan rebuilds)
            rccl = os.path.join(os.path.dirname(torch.__file__), "lib", "librccl.so")
            if dist.is_initialized():
                world, rank = dist.get_world_size(self.group), dist.get_rank(self.group)
                obj = [host.nccl_unique_id(rccl) if rank == 0 else None]
                src = dist.get_global_rank(self.group, 0) if self.group is not None else 0
                dist.broadcast_object_list(obj, src=src, group=self.group)
                uid = obj[0]
            else:
                world, rank, uid = 1, 0, host.nccl_unique_id(rccl)
            self._comm = host.nccl_comm_init(rccl, uid, world, rank, fp.device.index)
        plan = fp.plan
        lib = _native.load()
        scale_batch = ctypes.cast(lib.cbn_scale_batch, ctypes.c_void_p).value
        self._folded = (self.fold and not self.gather and int(fp.words.numel()) <= 256
                        and bool(lib.cbn_plan_flags(plan.handle) & _native.CBN_PLAN_STAGED))
        if self._folded:
            self.G = min(32, self.G_req)
            self._c = host.FoldStepper(ctypes.cast(lib.cbn_plan_run_fold, ctypes.c_void_p).value, scale_batch,
                                       plan.handle.value, fp.slot_keys, fp.first, fp.device.index, plan.n_samples,
                                       plan.target_observed, int(fp.words.numel()), self.G, self._comm)
        else:
            self._c = host.Stepper(fp.run_fn, scale_batch, plan.handle.value, fp.slot_keys, fp.first,
                                   fp.device.index, plan.n_samples, plan.target_observed, int(fp.words.numel()),
                                   self.G, self._comm, self.world, self.rank)
        self._fp = fp
        return True

    def _counts(self, n: int, total_rows: Optional[int]):
        if not self.gather:
            return None
        if total_rows is None:
            if self.world > 1:  # every rank's count must be known to size its all-gather: no guessing
                raise ValueError("ShardedStepper(gather=True).step needs total_rows (the whole batch, split by "
                                 "shard_bounds) when more than one rank takes part")
            return [n]
        return [shard_bounds(total_rows, self.world, r)[1] - shard_bounds(total_rows, self.world, r)[0]
                for r in range(self.world)]

    def step(self, evidence_shard: Dict[str, torch.Tensor], out: Optional[torch.Tensor] = None,
             total_rows: Optional[int] = None):
        """One step on this rank's shard.  ``gather=True``: returns the full
        [Q, N] tensor (Q = ``total_rows``, the whole batch split by
        ``shard_bounds``; None = equal shards), otherwise this rank's rows."""
        eng = self.bn.engine
        c = self._c
        self.n_steps += 1
        if self.watchdog is not None:
            self.watchdog.beat(step=self.n_steps)
        if c is not None and GENERATION[0] == eng._gen and eng.epoch == self._epoch:
            # hot path: one native call (folded ring, or the step ring with the
            # gather counts of this total_rows, cached)
            fp = self._fp
            if self._folded:
                res = c.step(evidence_shard, out, eng._flags(fp.plan) | _RAW)
            else:
                counts = self._hot_counts.get(total_rows, False) if self.gather else None
                if counts is False:
                    return self._step_slow(evidence_shard, out, total_rows)
                res = c.step(evidence_shard, out, eng._flags(fp.plan) | _RAW, counts)
            if type(res) is torch.Tensor:
                tdom = fp.tdom.get(res.shape[0])
                return res, (tdom if tdom is not None else self._tdom(fp, res.shape[0]))
            if res is not None:  # an error code: the step is enqueued (zero words), report it
                from . import _native

                _native.check(res, "cbn_plan_run_fold" if self._folded else "cbn_plan_run(raw)")
            # None: evidence the native checks reject -> the slow path converts (same ring)
        return self._step_slow(evidence_shard, out, total_rows)

    @staticmethod
    def _tdom(fp, m: int):
        plan = fp.plan
        t = fp.tdom[m] = plan.target_domain.unsqueeze(0).expand(m if plan.target_observed else 1, -1)
        return t

    def _step_slow(self, evidence_shard, out, total_rows):
        eng = self.bn.engine
        if GENERATION[0] != eng._gen:
            eng._check_generation()  # drops this network's plans if one of its estimators changed
        if self._c is not None and eng.epoch != self._epoch:
            # the plan the native stepper launches on was destroyed: finish what
            # was enqueued on it, then rebind to the rebuilt plan (every rank
            # refits alike, so every rank flushes here at the same step)
            self._c.synchronize()
            self._c = self._fp = None
        if self._c is None and not self._serial and not self._setup(evidence_shard):
            self._serial = True  # the plan has no raw launch / redraws its domains: every rank decides alike
        if self._serial:
            return sharded_infer(self.bn, self.target, evidence_shard, self.N_max, self.group, gather=self.gather,
                                 out=out)
        fp = self._fp
        n = next(iter(evidence_shard.values())).shape[0] if evidence_shard else 1
        flags = eng.raw_flags(fp.plan)
        counts = None if self._folded else self._counts(n, total_rows)
        if self.gather and not self._folded and (total_rows is not None or self.world == 1):
            # the counts depend on total_rows only (world 1: on n, so not cached)
            if total_rows is not None:
                self._hot_counts[total_rows] = counts

        def native_step(ev):
            return self._c.step(ev, out, flags) if self._folded else self._c.step(ev, out, flags, counts)

        res = native_step(evidence_shard)
        if res is None:  # dtype / device / layout the native checks reject: convert, same ring
            # (shape errors first, as the reference raises them; no step is
            # enqueued for a malformed batch)
            if eng.check_columns(fp.plan, evidence_shard):
                raise NotImplementedError(
                    "ShardedStepper takes [n_queries, 1] evidence columns; [n_queries, N_max] columns (per-query "
                    "sample values, node.py:246-248) go through sharded_infer")
            cols = {k: evidence_shard[k] for k in fp.slot_keys}
            conv = {k: v.to(device=fp.device, dtype=torch.float32).contiguous() for k, v in cols.items()}
            res = native_step(conv)
            if res is None:
                raise ValueError("ShardedStepper.step: evidence batch rejected (shape / target-unobserved batch > 1)")
        if type(res) is int:
            from . import _native

            _native.check(res, "cbn_plan_run(raw)")
        tdom = fp.tdom.get(res.shape[0])
        return res, (tdom if tdom is not None else self._tdom(fp, res.shape[0]))

    def comm_ranks(self) -> Optional[int]:
        """Ranks of the stepper's own RCCL communicator (ncclCommCount), None
        before the first step or when the step uses none."""
        if not self._comm:
            return None
        from . import _native

        return int(_native.load_host().nccl_comm_count(self._comm))

    def describe(self) -> str:
        """One line of ring state for a watchdog report."""
        c = self._c
        kind = "none" if c is None else ("fold ring" if self._folded else "step ring")
        ring = ""
        if c is not None:
            ring = f", native steps={c.steps()}, group={c.group()}"
            if self._folded:
                ring += f", unfinished={c.unfinished()}"
        return (f"stepper: {kind}, world={self.world}, rank={self.rank}, G={self.G}, gather={self.gather}, "
                f"serial={self._serial}, steps={self.n_steps}{ring}, last collective/wait={self.last_op}")

    def wait(self):
        """Make the current stream wait for every enqueued exchange + scale (+ gathers)."""
        if self._c is not None:
            self.last_op = f"wait() after step {self.n_steps} (flushes the partial group's all-reduce)"
            self._c.wait()
            if self.watchdog is not None:
                self.watchdog.beat(op="wait done")

    def synchronize(self):
        if self._c is not None:
            self.last_op = f"synchronize() after step {self.n_steps}"
            self._c.synchronize()

    def close(self):
        """Drain the comm stream and destroy the RCCL communicator (collective:
        every rank calls it)."""
        if self._c is not None:
            self._c.synchronize()
            self._c = None
        if self._comm:
            from . import _native

            _native.load_host().nccl_comm_destroy(self._comm)
            self._comm = 0
