"""When do a query's accumulators become all-zero?  

The table kernels multiply one gathered CPD row per factor into each query's
accumulators in the reference's factor order (bayesian_network.py:269-295).
Table entries are finite and >= 0 (BruteForce conditionals), so once every
accumulator a lane holds is +0, the remaining factors cannot change that
lane's outputs: its remaining row gathers can be skipped bit-exactly.  This
tool computes, on the CPU in fp32 with the reference's factor order, the
factor index after which each (query, lane) -- and each wave -- is all-zero,
for BASELINE configs[4] (peaked 10 x 10 grid, d = N = 64, k_query_fast: 8
lanes per query, 8 columns per lane, 8 queries per wave, rows gathered in
batches of 6 factors) and configs[2] (alarm-like X35 / X36, d = N = 8,
k_query_cols: one lane per query, batches of 2 factors).

The factor rows are the BruteForce conditionals joint / (parent marginal +
1e-10) of the training counts (brute_force.py:17-53, 172-244; every parent
observed, so no free-parent means).  Writes profiles/r05_zero_histogram.json.

    python tools/zero_histogram.py [--queries 65536]
"""
import argparse
import json
import os
import sys

import networkx as nx
import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
from helpers import alarm_like_data, grid_data, sample_evidence  # noqa: E402


def factor_order(edges, cols, target):
    """get_ancestors (bayesian_network.py:86-102) + the target."""
    g = nx.DiGraph()
    g.add_nodes_from(cols)
    g.add_edges_from(edges)
    anc = nx.ancestors(g, target)
    order = list(nx.topological_sort(g.subgraph(anc | {target})))
    order.remove(target)
    return order + [target], {n: sorted(g.predecessors(n)) for n in cols}


def conditional_rows(data, cols, node, parents, ev, d):
    """[Q, d] rows P(node = j | parents = evidence) and, for a root, the
    scalar mean over its d sample points (node.py:115-204)."""
    S = data.shape[0]
    x = data[:, cols.index(node)].astype(np.int64)
    if not parents:
        p = (np.bincount(x, minlength=d).astype(np.float32) / np.float32(S))
        return np.float32(p.mean(dtype=np.float64))
    key = np.zeros(S, np.int64)
    for p in parents:
        key = key * d + data[:, cols.index(p)].astype(np.int64)
    joint = (np.bincount(key * d + x, minlength=d ** (len(parents) + 1)).astype(np.float32) / np.float32(S))
    joint = joint.reshape(-1, d)
    marg = joint.sum(1, dtype=np.float32)
    cond = (joint / (marg[:, None] + np.float32(1e-10))).astype(np.float32)
    qk = np.zeros(ev[parents[0]].shape[0], np.int64)
    for p in parents:
        qk = qk * d + ev[p][:, 0].astype(np.int64)
    return cond[qk]


def histogram(name, data, cols, edges, target, d, Q, lanes_per_query, batch, queries_per_wave):
    order, par = factor_order(edges, cols, target)
    names = [c for c in cols if c != target]
    ev = sample_evidence(data, cols, names, Q, 0)
    acc = np.ones((Q, d), np.float32)
    nf = len(order)
    cpl = d // lanes_per_query  # columns per lane
    dead_at = np.full((Q, lanes_per_query), nf, np.int64)  # factors multiplied when the lane became all-zero
    for f, n in enumerate(order):
        acc *= conditional_rows(data, cols, n, par[n], ev, d)
        lane_zero = (acc.reshape(Q, lanes_per_query, cpl) == 0).all(2)
        dead_at = np.where(lane_zero & (dead_at == nf), f + 1, dead_at)
    # a batched kernel sees the death at the end of the batch that caused it
    checked = np.minimum(((dead_at + batch - 1) // batch) * batch, nf)
    lane_skip = (nf - checked).sum() / (Q * lanes_per_query * nf)
    wave = checked.reshape(-1, queries_per_wave * lanes_per_query).max(1)
    wave_skip = (nf - wave).sum() / (wave.size * nf)
    qdead = dead_at.max(1)
    quart = {f"dead_by_factor_{k}": round(float((dead_at <= k).mean()), 4) for k in (nf // 4, nf // 2, 3 * nf // 4)}
    res = dict(case=name, target=target, factors=nf, queries=Q, lanes_per_query=lanes_per_query,
               columns_per_lane=cpl, check_every_factors=batch, queries_per_wave=queries_per_wave,
               lanes_never_zero=round(float((dead_at == nf).mean()), 4),
               queries_with_a_nonzero_marginal=round(float((acc.max(1) > 0).mean()), 4),
               nonzero_marginal_frac=round(float((acc > 0).mean()), 5),
               lane_dead_quantiles={f"p{p}": int(np.percentile(dead_at, p)) for p in (10, 25, 50, 75, 90)},
               query_dead_median=int(np.median(qdead)),
               **quart,
               gathers_skippable_per_lane_mask=round(float(lane_skip), 4),
               gathers_skippable_wave_uniform=round(float(wave_skip), 4),
               lane_dead_hist=np.bincount(dead_at.ravel(), minlength=nf + 1).tolist())
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--queries", type=int, default=65536)
    a = ap.parse_args()
    out = []
    data, cols, edges = grid_data(400_000, 3, side=10, d=64, keep=0.995, noise=0)
    out.append(histogram("configs[4] peaked grid (tools/bench_grid.py headline)", data, cols, edges, cols[-1], 64,
                         a.queries, 8, 6, 8))
    data, cols, edges = alarm_like_data(200_000, 5)
    for t in ("X35", "X36"):
        out.append(histogram("configs[2] alarm-like (tools/bench_alarm.py)", data, cols, edges, t, 8, a.queries,
                             1, 2, 64))
    for r in out:
        print(json.dumps({k: v for k, v in r.items() if k != "lane_dead_hist"}))
    path = os.path.join(ROOT, "profiles", "r05_zero_histogram.json")
    with open(path, "w") as fh:
        json.dump(dict(generator="tools/zero_histogram.py", note=__doc__.split("\n\n")[1], cases=out), fh, indent=1)


if __name__ == "__main__":
    main()
