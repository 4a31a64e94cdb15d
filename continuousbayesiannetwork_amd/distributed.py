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

from typing import Callable, Dict, Optional, Tuple

import torch
import torch.distributed as dist


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


def sharded_infer(bn, target_node: str, evidence_shard: Dict[str, torch.Tensor], N_max: int = 16,
                  group=None, gather: bool = False, out: Optional[torch.Tensor] = None):
    """``BayesianNetwork.infer`` over a query batch sharded across ranks.

    Each rank passes its own rows of the evidence; the result equals the rows
    of the single-process ``infer`` on the concatenated batch.

    Fast-path plans: ONE launch per rank stores the unnormalised rows and the
    rank's max word, RCCL all-reduces the word (MAX), and an in-place scale
    launch divides by the global max.  Other plans: max pass, all-reduce,
    write pass.
    """
    eng = bn.engine
    raw = eng.infer_raw(target_node, evidence_shard, N_max, out)
    if raw is not None:
        rows, tdom, bits, scale = raw
        multi = dist.is_initialized() and dist.get_world_size(group) > 1
        if multi:
            dist.all_reduce(bits, op=dist.ReduceOp.MAX, group=group)
        scale(rows, bits)
        if gather and multi:
            rows = gather_rows(rows, group)
        return rows, tdom
    plan, cols, nq, tdom, device = eng.prepare(target_node, evidence_shard, N_max)
    if out is None:
        out = torch.empty((nq, plan.n_samples), dtype=torch.float32, device=device)

    def local_max():
        return eng.query_max(plan, cols, nq, device)

    def local_write(bits):
        return eng.query_write(plan, cols, nq, bits, out, device)

    res = normalise_across_ranks(local_max, local_write, group=group, gather=gather)
    return res, tdom
