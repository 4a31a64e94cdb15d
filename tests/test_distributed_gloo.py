"""World-size-2 gloo test of the sharded exchange (distributed.py): the
all-reduce(MAX) of the max word between the two query passes and the uneven
all-gather re-assembly.  The per-rank passes are played by the CPU oracle's
raw factor product, so this runs without a GPU."""
import os
import socket

import numpy as np
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from continuousbayesiannetwork_amd.distributed import normalise_across_ranks, shard_bounds, shard_evidence


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, Q, out_dir):
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root, os.path.join(root, "tests")]
    from helpers import chain_data, sample_evidence
    from oracle.ref_infer import OracleBN

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    data, cols, edges = chain_data(6, 4, 3000, 7, stay=0.6)
    ora = OracleBN(edges, cols, data)
    ev = {k: torch.tensor(v) for k, v in sample_evidence(data, cols, ["X4", "X2"], Q, 3).items()}
    mine = shard_evidence(ev, world, rank)
    raw, _ = ora.infer_raw("X5", {k: v.numpy() for k, v in mine.items()}, 4)
    raw_t = torch.tensor(raw)

    def local_max():
        return torch.tensor([np.float32(raw.max()).view(np.int32)], dtype=torch.int32)

    def local_write(bits):
        m = np.int32(bits.item()).view(np.float32)
        return raw_t / torch.tensor(m)

    full = normalise_across_ranks(local_max, local_write, gather=True, total_rows=Q)
    np.save(os.path.join(out_dir, f"r{rank}.npy"), full.numpy())
    dist.destroy_process_group()


def test_shard_bounds_cover_exactly():
    for n in (0, 1, 7, 64, 1001):
        for w in (1, 2, 3, 8):
            spans = [shard_bounds(n, w, r) for r in range(w)]
            assert spans[0][0] == 0 and spans[-1][1] == n
            assert all(a[1] == b[0] for a, b in zip(spans, spans[1:]))
            assert max(h - l for l, h in spans) - min(h - l for l, h in spans) <= 1


def test_two_rank_normalisation_matches_unsharded(tmp_path):
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root]
    from helpers import chain_data, sample_evidence
    from oracle.ref_infer import OracleBN

    Q = 301  # uneven shards
    mp.spawn(_worker, args=(2, _free_port(), Q, str(tmp_path)), nprocs=2, join=True)
    data, cols, edges = chain_data(6, 4, 3000, 7, stay=0.6)
    ref, _ = OracleBN(edges, cols, data).infer("X5", sample_evidence(data, cols, ["X4", "X2"], Q, 3), 4)
    for r in range(2):
        got = np.load(tmp_path / f"r{r}.npy")
        assert got.shape == ref.shape
        np.testing.assert_array_equal(got, ref)


class _RingOps:
    """CPU stand-in for the stepper's device side (csrc/host_fast.cpp HipOps):
    the raw launch is the oracle's unnormalised product, the exchange a gloo
    all-reduce(MAX), the scale a division, the gather an uneven all-gather.
    Every call is logged; the ring's stream-ordering protocol is checked here:
    a launch into a ring half whose words an earlier exchange read must come
    after a wait_done on that half, and each exchange covers exactly the
    launches of its group."""

    def __init__(self, G, W, ora, target, N):
        self.G, self.W, self.ora, self.target, self.N = G, W, ora, target, N
        self.words = torch.zeros((2 * G, W), dtype=torch.int32)
        self.dirty = [False, False]  # exchanged, not yet waited on by the compute side
        self.launched = [[], []]  # slot indices launched into each half since its last exchange
        self.log = []

    def launch(self, half, index, item):
        assert not self.dirty[half], f"launch into half {half} before wait_done"
        assert index == len(self.launched[half]), (index, self.launched[half])
        self.launched[half].append(index)
        w = self.words[half * self.G + index]
        w.zero_()
        ev = item["ev"]
        n = next(iter(ev.values())).shape[0]
        if n:
            raw, _ = self.ora.infer_raw(self.target, ev, self.N)
            item["rows"][:] = torch.tensor(raw)
            w[0] = int(np.float32(raw.max()).view(np.int32))
        self.log.append(("launch", half, index, item["step"]))
        return 0

    def exchange(self, half, nb):
        assert nb == len(self.launched[half]) and 1 <= nb <= self.G
        grp = self.words[half * self.G: half * self.G + nb]
        dist.all_reduce(grp, op=dist.ReduceOp.MAX)
        self.launched[half] = []
        self.log.append(("exchange", half, nb))
        return 0

    def scale(self, half, items):
        for b, it in enumerate(items):
            m = np.int32(int(self.words[half * self.G + b].max())).view(np.float32)
            it["rows"] /= torch.tensor(m)
        self.log.append(("scale", half, len(items)))
        return 0

    def gather(self, items):
        for it in items:
            if it.get("full") is None:
                continue
            counts = it["counts"]
            m = max(counts)
            pad = torch.zeros((m, self.N))
            pad[: it["rows"].shape[0]] = it["rows"]
            parts = [torch.empty_like(pad) for _ in counts]
            dist.all_gather(parts, pad)
            it["full"][:] = torch.cat([p[:c] for p, c in zip(parts, counts)])
        self.log.append(("gather", len(items)))
        return 0

    def handoff(self):
        self.log.append(("handoff",))

    def done(self, half):
        self.dirty[half] = True
        self.log.append(("done", half))

    def wait_done(self, half):
        self.dirty[half] = False
        self.log.append(("wait_done", half))

    def join(self):
        self.log.append(("join",))


SIZES = [301, 1, 64, 7, 128, 33, 2, 90]  # batch 1: rank 1's shard is empty; uneven splits


def _ring_worker(rank, world, port, G, gather, out_dir):
    import json
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root, os.path.join(root, "tests")]
    from helpers import chain_data, sample_evidence
    from oracle.ref_infer import OracleBN

    from continuousbayesiannetwork_amd import _native

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    data, cols, edges = chain_data(6, 4, 3000, 7, stay=0.6)
    ora = OracleBN(edges, cols, data)
    ops = _RingOps(G, 4, ora, "X5", 4)
    ring = _native.load_host().CpuStepRing(ops, G)
    items = []
    for k, Q in enumerate(SIZES):
        ev = sample_evidence(data, cols, ["X4", "X2"], Q, 40 + k)
        lo, hi = shard_bounds(Q, world, rank)
        mine = {c: v[lo:hi] for c, v in ev.items()}
        counts = [shard_bounds(Q, world, r)[1] - shard_bounds(Q, world, r)[0] for r in range(world)]
        full = torch.zeros((Q, 4)) if gather else None
        rows = full[lo:hi] if gather else torch.zeros((hi - lo, 4))
        it = dict(step=k, ev=mine, rows=rows, full=full, counts=counts)
        assert ring.step(it) == 0
        items.append(it)
        if k == 3:
            assert ring.wait() == 0  # mid-group: exchanges the partial group
    assert ring.wait() == 0
    for it in items:
        np.save(os.path.join(out_dir, f"r{rank}_s{it['step']}.npy"), (it["full"] if gather else it["rows"]).numpy())
    with open(os.path.join(out_dir, f"log{rank}.json"), "w") as fh:
        json.dump(ops.log, fh)
    dist.destroy_process_group()


def _ring_case(tmp_path, G, gather, world=2):
    import json
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root]
    from helpers import chain_data, sample_evidence
    from oracle.ref_infer import OracleBN

    mp.spawn(_ring_worker, args=(world, _free_port(), G, gather, str(tmp_path)), nprocs=world, join=True)
    data, cols, edges = chain_data(6, 4, 3000, 7, stay=0.6)
    ora = OracleBN(edges, cols, data)
    for k, Q in enumerate(SIZES):
        ref, _ = ora.infer("X5", sample_evidence(data, cols, ["X4", "X2"], Q, 40 + k), 4)
        for r in range(world):
            got = np.load(tmp_path / f"r{r}_s{k}.npy")
            lo, hi = shard_bounds(Q, world, r)
            np.testing.assert_array_equal(got, ref if gather else ref[lo:hi])
    logs = [json.load(open(tmp_path / f"log{r}.json")) for r in range(world)]
    # every rank issues the same collectives in the same order
    coll = [[e for e in lg if e[0] in ("exchange", "gather")] for lg in logs]
    assert all(c == coll[0] for c in coll[1:])
    # groups: full groups of G, a partial flush at the mid-stream wait() and at the end
    ex = [e[2] for e in coll[0] if e[0] == "exchange"]
    assert sum(ex) == len(SIZES) and max(ex) <= G
    assert ex[:2] == ([G, 4 - G] if G < 4 else [4])[:2]


def test_step_ring_two_ranks_rank_local(tmp_path):
    """csrc/host_fast.cpp StepRing (the ShardedStepper's group/ring bookkeeping)
    driven over gloo with the oracle as the device: groups of 3, a wait()
    mid-group, an empty shard, uneven shards -> every rank's rows equal the
    unsharded oracle's rows, and the ring's ordering protocol holds."""
    _ring_case(tmp_path, 3, gather=False)


def test_step_ring_two_ranks_gather(tmp_path):
    """Same, with the reassembly: every rank ends with the full [Q, N] tensor."""
    _ring_case(tmp_path, 2, gather=True)


def test_step_ring_four_ranks_gather(tmp_path):
    """Four ranks (the driver's N = 4 scaling point): batches of 1, 2 and 7
    rows leave three, two and one shards empty or ragged; every rank still
    ends with the unsharded oracle's full tensor and all four issue the same
    collectives."""
    _ring_case(tmp_path, 3, gather=True, world=4)


# ---------------------------------------------------------------------------
# sharded_infer's collective decisions, world size 2, the oracle as the device
# ---------------------------------------------------------------------------
class _LogDist:
    """torch.distributed as sharded_infer sees it, with every collective logged."""

    def __init__(self, log):
        self._log = log

    def __getattr__(self, name):
        f = getattr(dist, name)
        if name in ("all_reduce", "all_gather", "broadcast_object_list", "broadcast"):
            def logged(*a, **k):
                t = a[0]
                self._log.append([name, list(t.shape) if hasattr(t, "shape") else len(t)])
                return f(*a, **k)
            return logged
        return f


class _OracleEngine:
    """CPU stand-in for InferenceEngine behind sharded_infer: the real host
    logic decides whether the call redraws sample domains (engine.needs_redraw
    on a CPU mirror of the network) and consumes the call's draws through the
    real draw source (base.node.uniforms, i.e. through shared_draws); the
    oracle computes the rows, its ``random`` replaced by those draws.
    ``raw_ok``: whether this rank's plan takes a raw launch."""

    def __init__(self, bn, ora, raw_ok):
        self.bn, self.ora, self.raw_ok = bn, ora, raw_ok
        self.vals, self.raw = [], None

    def _order(self, target):
        return self.bn.get_ancestors(self.bn.initial_dag, target) + [target]

    def redraws(self, target, keys, N):
        from continuousbayesiannetwork_amd.inference.engine import needs_redraw, relevant_observed

        order = self._order(target)
        return needs_redraw(self.bn, order, relevant_observed(self.bn, order, keys), N)

    def call_plan(self, target, ev, N):
        from types import SimpleNamespace

        from continuousbayesiannetwork_amd.base.node import uniforms
        from continuousbayesiannetwork_amd.inference.engine import relevant_observed, sample_calls

        order = self._order(target)
        obs = relevant_observed(self.bn, order, ev.keys())
        total = sum(max(0, N - self.bn.nodes_obj[n].info[v][3].shape[0]) for _, n, v, _ in
                    sample_calls(self.bn, order, obs))
        self.vals = uniforms(total)  # this call's draws, in the reference's order
        self.target = target
        plan = SimpleNamespace(n_samples=N, deterministic=total == 0, reusable=True, target_observed=True,
                               target_domain=torch.zeros(N))
        fp = SimpleNamespace(words=torch.zeros(1, dtype=torch.int32) if self.raw_ok else None,
                             device=torch.device("cpu"), plan=plan)
        return plan, fp

    def _rows(self, ev, N):
        it = iter(self.vals)
        saved = random.random
        random.random = lambda: next(it)
        try:
            raw, dom = self.ora.infer_raw(self.target, {k: v.numpy() for k, v in ev.items()}, N)
        finally:
            random.random = saved
        return torch.tensor(raw), torch.tensor(dom)

    @staticmethod
    def check_columns(plan, ev):
        """InferenceEngine.check_columns raises the reference's shape errors
        for an empty shard (no launch checks it); the stand-in's shards are
        well-formed [Q, 1] columns."""
        for v in ev.values():
            assert v.dim() == 2 and v.shape[1] == 1

    @staticmethod
    def _bits(rows):
        m = float(rows.max()) if rows.numel() else 0.0
        return torch.tensor([np.float32(m).view(np.int32)], dtype=torch.int32)

    @staticmethod
    def _div(rows, bits):
        return rows.div_(torch.tensor(np.int32(bits.max().item()).view(np.float32)))

    def infer_raw(self, target, ev, N, out=None, fp=None):
        if not self.raw_ok:
            return None
        rows, dom = self._rows(ev, N)
        return rows, dom, self._bits(rows), self._div

    def prepare_plan(self, plan, ev):
        n = next(iter(ev.values())).shape[0]
        return list(ev.values()), n, torch.zeros((1, plan.n_samples)), torch.device("cpu")

    def query_max(self, plan, cols, nq, device):
        ev = dict(zip(self._keys, cols))
        self.raw = self._rows(ev, plan.n_samples)[0] if nq else torch.zeros((0, plan.n_samples))
        return self._bits(self.raw)

    def query_write(self, plan, cols, nq, bits, out, device):
        out[:] = self._div(self.raw.clone(), bits)
        return out


import random  # noqa: E402  (used by the stand-in engine)

CASES = {
    # name: (raw_ok per rank, shard sizes per step [rank 0, rank 1] as a split of Q, network kind)
    "raw_vs_two_pass": ((True, False), "chain"),
    "empty_shard_raw": ((True, True), "chain"),
    "empty_shard_two_pass": ((False, True), "chain"),
    "redrawn_binary": ((True, True), "binary"),
    "redrawn_two_pass": ((True, False), "binary"),
    # the parametrisation of tests/test_gpu_multi.py (configs[3] LR / NN [16]
    # plans with the reference-fitted parameters, a configs[4]-shaped grid)
    "config3_lr": ((True, True), "lr3"),
    "config3_nn": ((True, False), "nn3"),
    "config4_grid": ((True, True), "grid"),
}


def _case_net(kind):
    """(data, cols, edges, target, evidence keys, N, estimator, oracle)"""
    from helpers import chain_data, grid_data, random_dag_data
    from oracle.ref_infer import OracleBN

    if kind in ("lr3", "nn3"):
        from golden_io import load_param_golden, oracle_estimators

        g = load_param_golden("lr_mixed50_config3" if kind == "lr3" else "nn_mixed50_config3")
        m = g["meta"]
        cols = m["columns"]
        ora = OracleBN(m["edges"], cols, g["data"], nodes=m.get("nodes"), estimators=oracle_estimators(g))
        return (g["data"], cols, m["edges"], m["target"], [c for c in cols if c != m["target"]], m["N_max"],
                m["estimator"], ora)
    if kind == "chain":
        data, cols, edges = chain_data(6, 4, 3000, 7, stay=0.6)
        return data, cols, edges, "X5", ["X4", "X2"], 4, None, OracleBN(edges, cols, data)
    if kind == "grid":
        data, cols, edges = grid_data(20000, 3, side=5, d=8, keep=0.95, noise=0)
        return data, cols, edges, cols[-1], cols[:-1], 8, None, OracleBN(edges, cols, data)
    data, cols, edges = random_dag_data(7, 2, 3, 600, 5)
    return data, cols, edges, cols[-1], cols[:3], 16, None, OracleBN(edges, cols, data)


STEPS = [(301, 150), (9, 9), (64, 0), (1, 1), (40, 13)]  # (Q, rank-0 rows): uneven, equal, rank 1 empty, ...


def _sharded_worker(rank, world, port, case, out_dir):
    import json
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root, os.path.join(root, "tests")]
    from helpers import make_bn, sample_evidence
    from oracle.ref_infer import OracleBN

    import continuousbayesiannetwork_amd.distributed as D
    from continuousbayesiannetwork_amd import BayesianNetwork

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    raw_ok, kind = CASES[case]
    data, cols, edges, target, evk, N, est, ora = _case_net(kind)
    if est:  # the host logic only (parametric mirrors, one short fit on CPU)
        from helpers import param_config

        bn = make_bn(BayesianNetwork, edges, cols, data, device="cpu", estimator=est,
                     config=param_config(est, n_epochs=1))
    else:
        bn = make_bn(BayesianNetwork, edges, cols, data, device="cpu")
    eng = _OracleEngine(bn, ora, raw_ok[rank])
    log = []
    D.dist = _LogDist(log)
    fake = type("BN", (), {})()
    fake.engine = eng
    try:
        for k, (Q, q0) in enumerate(STEPS):
            ev = {c: torch.tensor(v) for c, v in sample_evidence(data, cols, evk, Q, 50 + k).items()}
            eng._keys = list(ev.keys())
            lo, hi = (0, q0) if rank == 0 else (q0, Q)
            mine = {c: v[lo:hi] for c, v in ev.items()}
            random.seed(1000 + k if rank == 0 else 777)  # only rank 0's draws may matter
            rows, _ = D.sharded_infer(fake, target, mine, N, gather=True)
            np.save(os.path.join(out_dir, f"{case}_r{rank}_s{k}.npy"), rows.numpy())
    finally:
        D.dist = dist
    with open(os.path.join(out_dir, f"{case}_log{rank}.json"), "w") as fh:
        json.dump(log, fh)
    dist.destroy_process_group()


import pytest  # noqa: E402


@pytest.mark.parametrize("case", list(CASES))
def test_sharded_infer_collectives_two_ranks(tmp_path, case):
    """sharded_infer on two gloo ranks with the oracle as the device: every
    rank issues the same collectives in the same order whatever its own plan
    can do (raw launch on one rank only -> both go two-pass; an empty shard
    contributes zero max words), redrawn sample domains (binary variables at
    N_max = 16, node.py:302-333) use rank 0's draws on both ranks, and every
    rank's gathered rows equal the single-process oracle under rank 0's seed
    (bayesian_network.py:296: one global max)."""
    import json
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root]
    from helpers import sample_evidence
    from oracle.ref_infer import OracleBN

    mp.spawn(_sharded_worker, args=(2, _free_port(), case, str(tmp_path)), nprocs=2, join=True)
    data, cols, edges, target, evk, N, _, ora = _case_net(CASES[case][1])
    for k, (Q, _) in enumerate(STEPS):
        random.seed(1000 + k)
        ref, _ = ora.infer(target, sample_evidence(data, cols, evk, Q, 50 + k), N)
        for r in range(2):
            got = np.load(tmp_path / f"{case}_r{r}_s{k}.npy")
            if CASES[case][1] in ("lr3", "nn3"):
                # the oracle's own rows: numpy's float32 matmul blocks by batch
                # shape, so a shard's mu can differ from the whole batch's in
                # the last ulp (the HIP kernels' rows do not: test_gpu_multi.py)
                np.testing.assert_allclose(got, ref, rtol=1e-6, atol=0)
            else:
                np.testing.assert_array_equal(got, ref)
    logs = [json.load(open(tmp_path / f"{case}_log{r}.json")) for r in range(2)]
    assert [e[0] for e in logs[0]] == [e[0] for e in logs[1]]
    if CASES[case][1] == "binary":
        assert sum(e[0] == "broadcast_object_list" for e in logs[0]) == len(STEPS)  # one draw exchange per call


# ---------------------------------------------------------------------------
# folded-scale ring (csrc/host_fast.cpp FoldRing, the rank-local stepper)
# ---------------------------------------------------------------------------
class _FoldOps:
    """CPU stand-in for FoldHipOps: the raw launch is the oracle's unnormalised
    product, the exchange a gloo all-reduce(MAX), a fold / scale a division.
    Stream order is modelled: a set's words become readable on the compute
    side only after a wait_set following its exchange; a launch may not
    overwrite words that are still to be consumed; every step is divided
    exactly once."""

    def __init__(self, G, W, ora, target, N):
        self.G, self.W, self.ora, self.target, self.N = G, W, ora, target, N
        self.words = torch.zeros((3 * G, W), dtype=torch.int32)
        self.valid = [set(), set(), set()]  # exchanged words not yet consumed
        self.comm_pending = [False, False, False]  # a comm op on the set not yet waited by compute
        self.rec = [None, None, None]  # a group's record on A: recorded -> passed / handed -> exchanged
        self.queries = 0
        self.log = []

    def _div(self, item, s, i):
        m = np.int32(int(self.words[s * self.G + i].max())).view(np.float32)
        assert i in self.valid[s], ("words consumed twice or never exchanged", s, i)
        self.valid[s].discard(i)
        item["rows"] /= torch.tensor(m)
        item["scaled"] += 1

    def launch(self, s, i, item, fold, fs, fi):
        assert not self.valid[s] or i not in self.valid[s], ("overwrites unconsumed words", s, i)
        if i == 0:
            assert not self.valid[s], ("group starts in a set with unconsumed words", s)
        w = self.words[s * self.G + i]
        w.zero_()
        ev = item["ev"]
        n = next(iter(ev.values())).shape[0]
        consumed = False
        if n:
            raw, _ = self.ora.infer_raw(self.target, ev, self.N)
            item["rows"][:] = torch.tensor(raw)
            w[0] = int(np.float32(raw.max()).view(np.int32))
            if fold is not None:
                assert not self.comm_pending[fs], ("fold before the compute side waited the exchange", fs)
                self._div(fold, fs, fi)
                consumed = True
        self.log.append(("launch", s, i, item["step"], None if fold is None or not consumed else fold["step"]))
        return consumed

    def exchange(self, s, nb):
        assert self.rec[s] in ("passed", "handed"), ("exchange before A passed the group", s)
        self.rec[s] = None
        grp = self.words[s * self.G: s * self.G + nb]
        dist.all_reduce(grp, op=dist.ReduceOp.MAX)
        self.valid[s] = set(range(nb))
        self.log.append(("exchange", s, nb))
        return 0

    def scale(self, run, on_comm):
        for item, s, i in run:
            if not on_comm:
                assert not self.comm_pending[s]
            self._div(item, s, i)
        self.log.append(("scale", on_comm, [it["step"] for it, _, _ in run]))
        return 0

    def mark_set(self, s, on_comm):
        if on_comm:
            self.comm_pending[s] = True

    def wait_set(self, s):
        self.comm_pending[s] = False

    def record(self, s):
        assert self.rec[s] is None, ("record over a group not yet exchanged", s)
        self.rec[s] = "recorded"

    def passed(self, s, block):
        # A passed the record: always when the host blocks, otherwise every other query
        assert self.rec[s] == "recorded", ("query of a set with no record", s)
        self.queries += 1
        if block or self.queries % 2:
            self.rec[s] = "passed"
            return True
        return False

    def handoff(self, s):
        assert self.rec[s] == "recorded", ("hand-off without a record", s)
        self.rec[s] = "handed"
        self.log.append(("handoff", s))

    def join(self):
        self.comm_pending = [False, False, False]
        self.log.append(("join",))


FOLD_SIZES = [301, 1, 64, 7, 128, 33, 2, 90, 50, 3, 0, 77, 12, 40, 9, 5, 64]  # an empty batch, empty shards


def _fold_worker(rank, world, port, G, waits, out_dir):
    import json
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root, os.path.join(root, "tests")]
    from helpers import chain_data, sample_evidence
    from oracle.ref_infer import OracleBN

    from continuousbayesiannetwork_amd import _native

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    data, cols, edges = chain_data(6, 4, 3000, 7, stay=0.6)
    ora = OracleBN(edges, cols, data)
    ops = _FoldOps(G, 4, ora, "X5", 4)
    ring = _native.load_host().CpuFoldRing(ops, G)
    items = []
    for k, Q in enumerate(FOLD_SIZES):
        ev = sample_evidence(data, cols, ["X4", "X2"], max(Q, 1), 40 + k)
        lo, hi = shard_bounds(Q, world, rank)
        mine = {c: v[lo:hi] for c, v in ev.items()}
        it = dict(step=k, ev=mine, rows=torch.zeros((hi - lo, 4)), scaled=0)
        assert ring.step(it) == 0
        items.append(it)
        if k in waits:
            assert ring.wait() == 0
            assert ring.unfinished() == 0
    assert ring.wait() == 0
    assert ring.unfinished() == 0
    for it in items:
        np.save(os.path.join(out_dir, f"f{rank}_s{it['step']}.npy"), it["rows"].numpy())
        assert it["scaled"] == 1, (it["step"], it["scaled"])
    with open(os.path.join(out_dir, f"flog{rank}.json"), "w") as fh:
        json.dump(ops.log, fh)
    dist.destroy_process_group()


@pytest.mark.parametrize("G,waits", [(2, ()), (3, (5,)), (1, (2, 9)), (4, (12,))])
def test_fold_ring_two_ranks(tmp_path, G, waits):
    """csrc/host_fast.cpp FoldRing (the rank-local ShardedStepper with the
    scale folded into later raw launches) over gloo with the oracle as the
    device: groups of G, wait() mid-stream, an empty batch and empty shards,
    uneven shards -> every rank's rows equal the unsharded oracle's rows,
    every step is divided exactly once, launches fold only exchanged and
    waited words, never overwrite words still to be consumed, and both ranks
    issue the same all-reduces."""
    import json
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root]
    from helpers import chain_data, sample_evidence
    from oracle.ref_infer import OracleBN

    mp.spawn(_fold_worker, args=(2, _free_port(), G, waits, str(tmp_path)), nprocs=2, join=True)
    data, cols, edges = chain_data(6, 4, 3000, 7, stay=0.6)
    ora = OracleBN(edges, cols, data)
    for k, Q in enumerate(FOLD_SIZES):
        if Q == 0:
            continue
        ref, _ = ora.infer("X5", sample_evidence(data, cols, ["X4", "X2"], Q, 40 + k), 4)
        for r in range(2):
            lo, hi = shard_bounds(Q, 2, r)
            np.testing.assert_array_equal(np.load(tmp_path / f"f{r}_s{k}.npy"), ref[lo:hi])
    logs = [json.load(open(tmp_path / f"flog{r}.json")) for r in range(2)]
    assert [e for e in logs[0] if e[0] == "exchange"] == [e for e in logs[1] if e[0] == "exchange"]
    folds = [e for e in logs[0] if e[0] == "launch" and e[4] is not None]
    assert folds, "no step was folded into a later launch"
    for e in folds:
        assert e[3] - e[4] >= 2 * G - (G - 1)  # a fold reaches at least one whole group back
