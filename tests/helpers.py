"""Builders shared by the CPU and GPU tests (synthetic data; no reference import)."""
import networkx as nx
import numpy as np
import pandas as pd


def make_bn(cls, edges, columns, data, device, estimator="brute_force", config=None):
    dag = nx.DiGraph()
    dag.add_nodes_from(columns)
    dag.add_edges_from(edges)
    df = pd.DataFrame(data, columns=columns)
    cfg = {"estimator_name": estimator}
    cfg.update(config or {})
    return cls(dag, df, cfg, {"inference_obj": "exact"}, device=device)


def param_config(estimator, n_epochs=30, lr=0.05, model=None):
    """Estimator config in the reference's yaml shape (cbn/conf/parameter_learning)."""
    cfg = {"estimator_name": estimator, "optimizer": {"name": "Adam", "params": {"lr": lr}},
           "train": {"n_epochs": n_epochs}}
    if model is not None:
        cfg["model"] = model
    return cfg


def mixed_dag_data(S, seed, n=50, max_parents=3, discrete_every=2, card=20, unit=False):
    """BASELINE configs[3]-shaped network: n nodes, every ``discrete_every``-th
    node discrete (integer levels 0..card-1; card 20 is the reference's
    discrete/continuous boundary, cbn/base/__init__.py BASE_MAX_CARDINALITY),
    the rest continuous linear-Gaussian; in-degree <= max_parents, edges from
    lower to higher index, X{i-1} -> X{i} always (the last node's ancestors
    are all the others: an n-factor product per query).  ``unit``:
    scale every column into [0, 1] (targets the BCE-trained logistic models
    can fit)."""
    rng = np.random.default_rng(seed)
    X = np.zeros((S, n), np.float64)
    edges = []
    for i in range(n):
        k = 0 if i == 0 else int(rng.integers(1, min(i, max_parents) + 1))
        # backbone parent X{i-1} (every node is an ancestor of the last one) + random extras
        ps = sorted({i - 1} | set(rng.choice(i, size=k - 1, replace=False).tolist())) if k else []
        k = len(ps)
        edges += [(f"X{p}", f"X{i}") for p in ps]
        z = rng.normal(0, 1, S)
        for p in ps:
            col = X[:, p]
            z = z + rng.uniform(-0.8, 0.8) * (col - col.mean()) / (col.std() + 1e-9)
        z = z / np.sqrt(1 + 0.3 * k)
        if i % discrete_every == 1:
            X[:, i] = np.clip(np.round((z + 2.5) / 5.0 * (card - 1)), 0, card - 1)
        else:
            X[:, i] = np.round(z, 3)
    if unit:
        lo, hi = X.min(0), X.max(0)
        X = np.round((X - lo) / (hi - lo), 4)
    cols = [f"X{i}" for i in range(n)]
    return X.astype(np.float32), cols, edges


def chain_data(n, d, S, seed, values=None, noise=(0.6, 0.3, 0.1), stay=None):
    """Discrete chain X0 -> ... -> X{n-1}.  Default: X_i = X_{i-1} + noise (mod d),
    a sparse CPT.  ``stay=p``: X_i = X_{i-1} with probability p, else uniform --
    a dense CPT whose products along the chain stay well inside fp32 range."""
    rng = np.random.default_rng(seed)
    X = np.zeros((S, n), np.int64)
    X[:, 0] = rng.integers(0, d, S)
    for i in range(1, n):
        if stay is not None:
            keep = rng.random(S) < stay
            X[:, i] = np.where(keep, X[:, i - 1], rng.integers(0, d, S))
        else:
            X[:, i] = (X[:, i - 1] + rng.choice(len(noise), S, p=list(noise))) % d
    vals = np.arange(d, dtype=np.float32) if values is None else np.asarray(values, np.float32)
    cols = [f"X{i}" for i in range(n)]
    edges = [(f"X{i}", f"X{i+1}") for i in range(n - 1)]
    return vals[X], cols, edges


def random_dag_data(n, d, max_parents, S, seed):
    """Random DAG over X0..X{n-1} (edges only from lower to higher index)."""
    rng = np.random.default_rng(seed)
    edges = []
    X = np.zeros((S, n), np.int64)
    for i in range(n):
        k = int(rng.integers(0, min(i, max_parents) + 1))
        if i == n - 1:
            k = max(k, 1)
        ps = sorted(rng.choice(i, size=k, replace=False).tolist()) if k else []
        edges += [(f"X{p}", f"X{i}") for p in ps]
        base = rng.integers(0, d, S)
        for p in ps:
            base = base + X[:, p] * int(rng.integers(1, 3))
        X[:, i] = (base + rng.integers(0, 2, S)) % d
    cols = [f"X{i}" for i in range(n)]
    return X.astype(np.float32), cols, edges


def sample_evidence(data, cols, names, Q, seed, missing_frac=0.0, missing_value=7.5):
    rng = np.random.default_rng(seed)
    rows = rng.integers(0, data.shape[0], Q)
    ev = {}
    for nm in names:
        v = data[rows, cols.index(nm)].astype(np.float32).reshape(Q, 1)
        if missing_frac > 0:
            m = rng.random(Q) < missing_frac
            v[m, 0] = missing_value
        ev[nm] = v
    return ev


def alarm_like_data(S, seed, n=37, d=8, max_parents=4, n_edges=46):
    """ALARM-shaped synthetic network (BASELINE configs[2]): n nodes, n_edges
    edges, in-degree <= max_parents, card d.  Edges go from lower to higher
    index; X_i = (sum_p c_p X_p + c_0) mod d with probability 0.7, else
    uniform -- every CPT depends on every parent."""
    rng = np.random.default_rng(seed)
    parents = {i: [] for i in range(n)}
    cand = [(a, b) for b in range(1, n) for a in range(b)]
    rng.shuffle(cand)
    # a spanning backbone first (every node after X0 gets >= 1 parent), then extra edges
    for b in range(1, n):
        parents[b].append(int(rng.integers(max(0, b - 4), b)))
    extra = n_edges - (n - 1)
    for b in (n // 3, (2 * n) // 3, n - 2):  # a few 4-parent nodes, as in ALARM
        while len(parents[b]) < max_parents and extra > 0:
            a = int(rng.integers(0, b))
            if a not in parents[b]:
                parents[b].append(a)
                extra -= 1
    for a, b in cand:
        if extra <= 0:
            break
        if a not in parents[b] and len(parents[b]) < max_parents:
            parents[b].append(a)
            extra -= 1
    X = np.zeros((S, n), np.int64)
    for i in range(n):
        ps = sorted(parents[i])
        if not ps:
            X[:, i] = rng.integers(0, d, S)
            continue
        base = np.full(S, int(rng.integers(0, d)))
        for p in ps:
            base = base + X[:, p] * int(rng.integers(1, d))
        keep = rng.random(S) < 0.7
        X[:, i] = np.where(keep, base % d, rng.integers(0, d, S))
    cols = [f"X{i}" for i in range(n)]
    edges = [(f"X{p}", f"X{i}") for i in range(n) for p in sorted(parents[i])]
    return X.astype(np.float32), cols, edges


def grid_data(S, seed, side=10, d=64, keep=0.8, noise=2):
    """BASELINE configs[4]-shaped network: side x side grid DAG (node (r, c)
    has parents (r, c-1) and (r-1, c)), d levels per node: X = mean of the
    parents + small noise (mod d, |noise| <= ``noise``) with probability
    ``keep``, else uniform."""
    rng = np.random.default_rng(seed)
    n = side * side
    X = np.zeros((S, n), np.int64)
    edges = []
    for r in range(side):
        for c in range(side):
            i = r * side + c
            ps = ([i - 1] if c > 0 else []) + ([i - side] if r > 0 else [])
            edges += [(f"X{p}", f"X{i}") for p in ps]
            if not ps:
                X[:, i] = rng.integers(0, d, S)
                continue
            base = sum(X[:, p] for p in ps) // len(ps)
            k = rng.random(S) < keep
            X[:, i] = np.where(k, (base + rng.integers(-noise, noise + 1, S)) % d, rng.integers(0, d, S))
    return X.astype(np.float32), [f"X{i}" for i in range(n)], edges


def grid_rows_data(S, seed, side=10, d=64, keep_even=0.9, keep_odd=1.0):
    """configs[4]'s grid DAG (same edges as ``grid_data``) with data shaped for
    evidence on the EVEN grid rows (every interior factor then has one
    observed and one free parent): an even-row node copies its LEFT parent
    (its observed one) with probability ``keep_even``, else uniform, and
    column 0 of an even row is uniform (rows independent of each other); an
    odd-row node copies its UP parent (its observed one) with probability
    ``keep_odd``, else uniform.  So each factor is
    concentrated on the value its observed parent implies, and its free
    parent is independent enough of the observed one that most of the free
    parent's sample points meet training rows (the mean over them stays
    away from 0 for a 100-factor product)."""
    rng = np.random.default_rng(seed)
    n = side * side
    X = np.zeros((S, n), np.int64)
    edges = []
    for r in range(side):
        for c in range(side):
            i = r * side + c
            ps = ([i - 1] if c > 0 else []) + ([i - side] if r > 0 else [])
            edges += [(f"X{p}", f"X{i}") for p in ps]
            u = rng.integers(0, d, S)
            if r % 2 == 0:
                if c == 0:
                    X[:, i] = u
                else:
                    X[:, i] = np.where(rng.random(S) < keep_even, X[:, i - 1], u)
            else:
                X[:, i] = np.where(rng.random(S) < keep_odd, X[:, i - side], u)
    return X.astype(np.float32), [f"X{i}" for i in range(n)], edges


def wide_data(S, seed, k=10, d=2, dy=3):
    """One node Y with k parents P0..P{k-1} (uniform over d levels):
    Y = (sum of the parents + noise) mod dy.  k > 8 is beyond the table
    path's parent limit (direct plans)."""
    rng = np.random.default_rng(seed)
    P = rng.integers(0, d, (S, k))
    Y = (P.sum(1) + rng.choice(3, S, p=[0.7, 0.2, 0.1])) % dy
    X = np.concatenate([P, Y[:, None]], 1).astype(np.float32)
    cols = [f"P{i}" for i in range(k)] + ["Y"]
    return X, cols, [(f"P{i}", "Y") for i in range(k)]


def hicard_data(S, seed, d=40, k=4):
    """k uniform roots over d levels and a child E = (sum + noise) mod d:
    the child's dense CPD has d^(k+1) cells (40^5 ~ 1e8: hashed)."""
    rng = np.random.default_rng(seed)
    R = rng.integers(0, d, (S, k))
    E = (R.sum(1) + rng.choice(3, S, p=[0.6, 0.3, 0.1])) % d
    X = np.concatenate([R, E[:, None]], 1).astype(np.float32)
    cols = [f"R{i}" for i in range(k)] + ["E"]
    return X, cols, [(f"R{i}", "E") for i in range(k)]


def continuous_data(S, seed, decimals=1):
    """Continuous roots X0..X2 ~ N(0, 2^2) rounded to ``decimals`` and
    X3 = round(X0 + X1 + X2 + N(0, 1)): ~100 distinct values per root, the
    dense CPD of X3 ~ 1e6 x 25 cells (hashed)."""
    rng = np.random.default_rng(seed)
    R = np.round(rng.normal(0, 2, (S, 3)), decimals)
    X3 = np.round(R.sum(1) + rng.normal(0, 1, S), 0)
    X = np.concatenate([R, X3[:, None]], 1).astype(np.float32)
    cols = ["X0", "X1", "X2", "X3"]
    return X, cols, [("X0", "X3"), ("X1", "X3"), ("X2", "X3")]


def continuous_free_data(S, seed):
    """Two continuous roots X0, X1 ~ N(0, 2^2) rounded to 2 decimals (~1 500
    distinct values each), a 5-level root X2 and X3 = (round(X0 + X1) + X2)
    mod 8: X3's dense CPD would be ~1e8 cells (hashed); with X0, X1 observed
    and X2 free (N >= 8) every evidence row drawn from the data has support."""
    rng = np.random.default_rng(seed)
    R = np.round(rng.normal(0, 2, (S, 2)), 2)
    X2 = rng.integers(0, 5, S)
    X3 = (np.round(R.sum(1)).astype(np.int64) + X2) % 8
    X = np.concatenate([R, X2[:, None], X3[:, None]], 1).astype(np.float32)
    cols = ["X0", "X1", "X2", "X3"]
    return X, cols, [("X0", "X3"), ("X1", "X3"), ("X2", "X3")]


def grid_rows_evidence(names, Q, seed, d=64, perturb=2):
    """Evidence for ``grid_rows_data`` networks: every named (even-row) node of
    query q observes the same level v_q (the value every factor's mass sits on
    there), and every other query also changes ``perturb`` randomly chosen
    names to random levels (rows whose products drop by a few factors or
    vanish)."""
    rng = np.random.default_rng(seed)
    v = rng.integers(0, d, Q)
    ev = {nm: v[:, None].astype(np.float32).copy() for nm in names}
    for q in range(1, Q, 2):
        for nm in rng.choice(len(names), size=perturb, replace=False):
            ev[names[nm]][q, 0] = float(rng.integers(0, d))
    return ev
