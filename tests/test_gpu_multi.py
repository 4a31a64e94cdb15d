"""Two real GPUs, two ranks over RCCL (skipped on a one-GPU box).

ADVICE r03: the folded stepper (FoldStepper: each step's division folded into
a later raw launch, the group all-reduce handed to the comm stream after host
event queries) had only run over a one-rank communicator on hardware.  It is
off by default with real peers (ShardedStepper(fold=None) at world > 1); this
test pins it -- and the default step ring, with and without the all-gather --
bit for bit against ``sharded_infer`` and against the single-process ``infer``
of the concatenated batch, on two GPUs.  Reference anchor: the one global max
of bayesian_network.py:296 that every rank must exchange each step.
"""
import os
import socket

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, out_dir):
    import sys

    import torch.distributed as dist

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root, os.path.join(root, "tests")]
    from continuousbayesiannetwork_amd import BayesianNetwork
    from continuousbayesiannetwork_amd.distributed import ShardedStepper, shard_evidence, sharded_infer
    from helpers import chain_data, make_bn, sample_evidence

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    torch.cuda.set_device(rank)
    dev = torch.device("cuda", rank)
    dist.init_process_group("nccl", device_id=dev)
    data, cols, edges = chain_data(20, 32, 50_000, 3, stay=0.8)
    names = cols[:-1]
    Q = 8192
    bn = make_bn(BayesianNetwork, edges, cols, data, device=dev)
    batches = [{k: torch.tensor(v, device=dev) for k, v in sample_evidence(data, cols, names, Q, 40 + b).items()}
               for b in range(12)]
    ref = [sharded_infer(bn, "X19", shard_evidence(ev, world, rank), N_max=32)[0].clone() for ev in batches]
    full = [bn.infer("X19", ev, N_max=32)[0] for ev in batches]  # every rank: the whole batch
    res = {}
    for name, kw in (("fold", dict(fold=True)), ("ring", dict(fold=None)), ("gather", dict(gather=True))):
        st = ShardedStepper(bn, "X19", 32, exchange_every=4, **kw)
        outs = [st.step(shard_evidence(ev, world, rank), total_rows=Q if kw.get("gather") else None)[0]
                for ev in batches]
        st.wait()
        torch.cuda.synchronize()
        res[name] = [o.clone() for o in outs]
        if name == "fold":
            res["fold_used"] = bool(st._folded)
        st.close()
    lo, hi = rank * Q // world, (rank + 1) * Q // world
    ok = {
        "fold_used": res["fold_used"],
        "fold": all(torch.equal(a, b) for a, b in zip(res["fold"], ref)),
        "ring": all(torch.equal(a, b) for a, b in zip(res["ring"], ref)),
        "gather": all(torch.equal(a, b) for a, b in zip(res["gather"], full)),
        "vs_single": all(torch.equal(a, b[lo:hi]) for a, b in zip(ref, full)),
    }
    np.save(os.path.join(out_dir, f"r{rank}.npy"), np.array([ok[k] for k in sorted(ok)]))
    dist.destroy_process_group()


@pytest.mark.skipif(torch.cuda.device_count() < 2, reason="needs two GPUs (one rank per GPU over RCCL)")
def test_folded_and_ring_steppers_two_gpus_bit_equal(tmp_path):
    import torch.multiprocessing as mp

    mp.spawn(_worker, args=(2, _free_port(), str(tmp_path)), nprocs=2, join=True)
    for r in range(2):
        flags = np.load(tmp_path / f"r{r}.npy")
        assert flags.all(), (r, flags)  # fold (used), fold, gather, ring, vs_single: sorted keys
