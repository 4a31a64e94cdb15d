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
