"""Every GPU present, one rank per GPU over RCCL (skipped on a one-GPU box;
the driver's 8-GPU node runs it at world size 8).

ADVICE r03: the folded stepper (FoldStepper: each step's division folded into
a later raw launch, the group all-reduce handed to the comm stream after host
event queries) had only run over a one-rank communicator on hardware.  It is
off by default with real peers (ShardedStepper(fold=None) at world > 1); this
test pins it -- and the default step ring, with and without the all-gather --
bit for bit against ``sharded_infer`` and against the single-process ``infer``
of the concatenated batch.  VERDICT r05: the same for the plans the other
sharded configs run -- configs[3]'s parametric raw path (50-node mixed DAG,
LinearRegression and NeuralNetwork [16], the reference-fitted parameters of
tests/golden/*_mixed50_config3.npz) and configs[4]'s k_query_slots raw path
(10 x 10 grid, d = N = 64).  Ragged shards (Q not a multiple of the world
size).  Reference anchor: the one global max of bayesian_network.py:296 that
every rank must exchange each step.
"""
import os
import socket

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
WORLD = min(torch.cuda.device_count(), 8)
CASES = ("chain", "lr3", "nn3", "grid")


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def build_case(case, dev, tmp_dir):
    """(bn, target, N, batches(Q, seed) -> evidence dict on dev) for a case
    (also used by the gloo stand-in's parametrisation on CPU)."""
    from continuousbayesiannetwork_amd import BayesianNetwork
    from helpers import chain_data, grid_data, make_bn, sample_evidence

    if case == "chain":
        data, cols, edges = chain_data(20, 32, 50_000, 3, stay=0.8)
        bn = make_bn(BayesianNetwork, edges, cols, data, device=dev)
        target, names, N = "X19", cols[:-1], 32
    elif case == "grid":
        data, cols, edges = grid_data(60_000, 3, side=10, d=64, keep=0.995, noise=0)
        bn = make_bn(BayesianNetwork, edges, cols, data, device=dev)
        target, names, N = cols[-1], cols[:-1], 64
    else:
        from golden_io import load_param_golden
        from test_gpu_param import _fixture_bn

        g = load_param_golden("lr_mixed50_config3" if case == "lr3" else "nn_mixed50_config3")
        m = g["meta"]
        data, cols = g["data"], m["columns"]
        bn = _fixture_bn(g, dev, tmp_dir)
        target, names, N = m["target"], [c for c in cols if c != m["target"]], m["N_max"]

    def batches(Q, seed):
        return {k: torch.tensor(v, device=dev) for k, v in sample_evidence(data, cols, names, Q, seed).items()}

    return bn, target, N, batches


def _worker(rank, world, port, case, out_dir):
    import sys

    import torch.distributed as dist

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root, os.path.join(root, "tests")]
    from continuousbayesiannetwork_amd.distributed import ShardedStepper, shard_bounds, shard_evidence, sharded_infer

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    torch.cuda.set_device(rank)
    dev = torch.device("cuda", rank)
    dist.init_process_group("nccl", device_id=dev)
    tmp = os.path.join(out_dir, f"params_r{rank}")
    os.makedirs(tmp, exist_ok=True)
    bn, target, N, make = build_case(case, dev, tmp)
    Q = 8192 + 37  # ragged shards
    batches = [make(Q, 40 + b) for b in range(6 if case != "chain" else 12)]
    ref = [sharded_infer(bn, target, shard_evidence(ev, world, rank), N_max=N)[0].clone() for ev in batches]
    full = [bn.infer(target, ev, N_max=N)[0].clone() for ev in batches]  # every rank: the whole batch
    res = {}
    modes = [("ring", dict(fold=None)), ("gather", dict(gather=True))]
    if case == "chain":  # the folded scales run on staged plans only
        modes.insert(0, ("fold", dict(fold=True)))
    for name, kw in modes:
        st = ShardedStepper(bn, target, N, exchange_every=4, **kw)
        outs = [st.step(shard_evidence(ev, world, rank), total_rows=Q if kw.get("gather") else None)[0]
                for ev in batches]
        st.wait()
        torch.cuda.synchronize()
        res[name] = [o.clone() for o in outs]
        if name == "fold":
            res["fold_used"] = bool(st._folded)
        st.close()
    lo, hi = shard_bounds(Q, world, rank)
    ok = {
        "ring": all(torch.equal(a, b) for a, b in zip(res["ring"], ref)),
        "gather": all(torch.equal(a, b) for a, b in zip(res["gather"], full)),
        "vs_single": all(torch.equal(a, b[lo:hi]) for a, b in zip(ref, full)),
        "finite": all(bool(torch.isfinite(b).all()) and float(b.max()) == 1.0 for b in full),
    }
    if case == "chain":
        ok["fold_used"] = res["fold_used"]
        ok["fold"] = all(torch.equal(a, b) for a, b in zip(res["fold"], ref))
    np.save(os.path.join(out_dir, f"{case}_r{rank}.npy"), np.array([ok[k] for k in sorted(ok)]))
    with open(os.path.join(out_dir, f"{case}_r{rank}.txt"), "w") as fh:
        fh.write(repr(sorted(ok.items())))
    dist.destroy_process_group()


@pytest.mark.skipif(WORLD < 2, reason="needs two or more GPUs (one rank per GPU over RCCL)")
@pytest.mark.parametrize("case", CASES)
def test_sharded_paths_every_gpu_bit_equal(case, tmp_path):
    """sharded_infer, the step ring (rank-local rows) and the gathering ring
    on WORLD ranks == the single-process infer of the whole batch, bit for
    bit, for the configs[1] chain (also the folded stepper), the configs[3]
    LR / NN [16] parametric plans and the configs[4] slots plan."""
    import torch.multiprocessing as mp

    mp.spawn(_worker, args=(WORLD, _free_port(), case, str(tmp_path)), nprocs=WORLD, join=True)
    for r in range(WORLD):
        flags = np.load(tmp_path / f"{case}_r{r}.npy")
        assert flags.all(), (r, (tmp_path / f"{case}_r{r}.txt").read_text())
