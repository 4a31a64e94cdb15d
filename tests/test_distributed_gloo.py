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


def _ring_case(tmp_path, G, gather):
    import json
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root]
    from helpers import chain_data, sample_evidence
    from oracle.ref_infer import OracleBN

    mp.spawn(_ring_worker, args=(2, _free_port(), G, gather, str(tmp_path)), nprocs=2, join=True)
    data, cols, edges = chain_data(6, 4, 3000, 7, stay=0.6)
    ora = OracleBN(edges, cols, data)
    for k, Q in enumerate(SIZES):
        ref, _ = ora.infer("X5", sample_evidence(data, cols, ["X4", "X2"], Q, 40 + k), 4)
        for r in range(2):
            got = np.load(tmp_path / f"r{r}_s{k}.npy")
            lo, hi = shard_bounds(Q, 2, r)
            np.testing.assert_array_equal(got, ref if gather else ref[lo:hi])
    logs = [json.load(open(tmp_path / f"log{r}.json")) for r in range(2)]
    # both ranks issue the same collectives in the same order
    coll = [[e for e in lg if e[0] in ("exchange", "gather")] for lg in logs]
    assert coll[0] == coll[1]
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
