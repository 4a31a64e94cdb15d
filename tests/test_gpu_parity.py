"""HIP path vs the reference (golden vectors) and vs the CPU oracle.

Tolerance (stated per the north star): rtol 1e-5, atol 1e-7 on fp32 pdfs --
the HIP tables average the parent axes in a different order than torch.mean.
Domains, shapes, zero patterns and error types must match exactly.
"""
import random

import numpy as np
import pytest
import torch

from continuousbayesiannetwork_amd import BayesianNetwork, Node
from continuousbayesiannetwork_amd.inference.engine import domain_index
from golden_io import golden_error, golden_names, load_golden, width_n_only
from helpers import alarm_like_data, chain_data, make_bn, random_dag_data, sample_evidence
from oracle.ref_infer import OracleBN, OracleBruteForce, OracleNode

pytestmark = pytest.mark.gpu
RTOL, ATOL = 1e-5, 1e-7


def _t(ev, dev):
    return {k: torch.tensor(v, device=dev) for k, v in ev.items()}


@pytest.mark.parametrize("name", golden_names())
def test_infer_matches_reference_golden(name, gpu):
    g = load_golden(name)
    m = g["meta"]
    bn = make_bn(BayesianNetwork, m["edges"], m["columns"], g["data"], device=gpu)
    ev = None if m["evidence_none"] else _t({k: g["evidence"][k] for k in m["evidence"]}, gpu)
    random.seed(m["seed"])
    if m["error"]:
        exc, msg = golden_error(m)
        for _ in range(2):  # the first call plans; the second finds the cached fast path
            with pytest.raises(exc) as info:
                bn.infer(m["target"], ev, N_max=m["N_max"])
            if exc is RuntimeError:  # evidence widths: the reference's message too
                assert str(info.value) == msg
        return
    pdf, dom = bn.infer(m["target"], ev, N_max=m["N_max"])
    assert pdf.device.type == "cuda"
    np.testing.assert_array_equal(dom.cpu().numpy(), g["domain"])
    np.testing.assert_allclose(pdf.cpu().numpy(), g["pdf"], rtol=RTOL, atol=ATOL)
    # a second call reuses the cached plan (or redraws, for oversampled domains)
    random.seed(m["seed"])
    pdf2, _ = bn.infer(m["target"], ev, N_max=m["N_max"])
    np.testing.assert_array_equal(pdf2.cpu().numpy(), pdf.cpu().numpy())


CASES = [
    # n, d, max_parents, S, seed, target, evidence names, Q, N
    (8, 3, 3, 3000, 1, "X7", ["X6", "X5", "X4", "X3"], 300, 3),
    (8, 4, 2, 4000, 2, "X7", ["X1", "X2", "X5"], 257, 4),
    (10, 3, 4, 5000, 3, "X9", ["X8", "X7", "X6", "X5", "X4", "X3"], 511, 2),
    (6, 5, 3, 5000, 4, "X5", ["X0", "X1", "X2", "X3", "X4"], 64, 5),
    (7, 4, 3, 2000, 5, "X6", ["X5", "X4", "X2"], 1000, 3),
]


@pytest.mark.parametrize("case", CASES, ids=[f"dag{c[4]}" for c in CASES])
def test_random_dags_match_oracle(case, gpu):
    n, d, mp, S, seed, target, evn, Q, N = case
    data, cols, edges = random_dag_data(n, d, mp, S, seed)
    ora = OracleBN(edges, cols, data)
    bn = make_bn(BayesianNetwork, edges, cols, data, device=gpu)
    ev = sample_evidence(data, cols, evn, Q, seed + 7, missing_frac=0.05)
    # keep only evidence on the target's parents plus others (target parents must be observed for Q>1)
    tpar = sorted(p for p, c in edges if c == target)
    if not any(p in ev for p in tpar):
        ev[tpar[0]] = sample_evidence(data, cols, [tpar[0]], Q, seed + 9)[tpar[0]]
    random.seed(seed)
    ref, rdom = ora.infer(target, ev, N)
    random.seed(seed)
    pdf, dom = bn.infer(target, _t(ev, gpu), N_max=N)
    np.testing.assert_array_equal(dom.cpu().numpy(), rdom)
    np.testing.assert_allclose(pdf.cpu().numpy(), ref, rtol=RTOL, atol=ATOL)


def test_vec1_path_and_oversampled_domains(gpu):
    """N not a multiple of 4 (scalar stores) and N > |domain| (random padding)."""
    data, cols, edges = chain_data(6, 5, 4000, 11)
    ora = OracleBN(edges, cols, data)
    bn = make_bn(BayesianNetwork, edges, cols, data, device=gpu)
    ev = sample_evidence(data, cols, ["X4", "X1"], 333, 5)
    for N, seed in [(5, 0), (7, 3), (3, 0)]:
        random.seed(seed)
        ref, rdom = ora.infer("X5", ev, N)
        random.seed(seed)
        pdf, dom = bn.infer("X5", _t(ev, gpu), N_max=N)
        np.testing.assert_array_equal(dom.cpu().numpy(), rdom)
        np.testing.assert_allclose(pdf.cpu().numpy(), ref, rtol=RTOL, atol=ATOL)


def test_node_get_prob_matches_oracle(gpu):
    """Node.get_prob (node.py:115-204) pdf tensor, all three evidence regimes."""
    g = load_golden("multi_partial")
    m = g["meta"]
    data, cols = g["data"], m["columns"]
    parents = ["C", "D"]
    on = OracleNode("E", parents)
    on.fit(data[:, cols.index("E")], np.stack([data[:, cols.index(p)] for p in parents]))
    nd = Node("E", "brute_force", {"estimator_name": "brute_force"}, parents, device=gpu)
    nd.fit(torch.tensor(data[:, cols.index("E")], device=gpu),
           torch.tensor(np.stack([data[:, cols.index(p)] for p in parents]), device=gpu))
    ev = sample_evidence(data, cols, ["C", "D"], 17, 3, missing_frac=0.2)
    for q in [{}, {"C": ev["C"]}, {"C": ev["C"], "D": ev["D"]}]:
        for N in (2, 3):
            ref, rdom = on.get_prob(dict(q), N)
            pdf, dom, _ = nd.get_prob({k: torch.tensor(v, device=gpu) for k, v in q.items()}, N)
            assert tuple(pdf.shape) == ref.shape
            np.testing.assert_allclose(pdf.cpu().numpy(), ref, rtol=RTOL, atol=ATOL)
            np.testing.assert_array_equal(dom.cpu().numpy(), rdom)


def test_bruteforce_get_prob_matches_oracle(gpu):
    """BruteForce._get_prob (brute_force.py:172-244) at on- and off-domain points."""
    from continuousbayesiannetwork_amd import BruteForce

    rng = np.random.default_rng(0)
    pd_ = rng.integers(0, 4, (2, 5000)).astype(np.float32)
    nd_ = ((pd_[0] + 2 * pd_[1] + rng.integers(0, 3, 5000)) % 5).astype(np.float32)
    ob = OracleBruteForce()
    ob.fit(nd_, pd_)
    bf = BruteForce({"estimator_name": "brute_force"}, device=gpu)
    bf.fit(torch.tensor(nd_, device=gpu), torch.tensor(pd_, device=gpu))
    pts = rng.integers(-1, 6, (300, 7)).astype(np.float32)
    q = rng.integers(-1, 5, (300, 2, 1)).astype(np.float32)
    ref = ob.get_prob(pts, q)
    got = bf.get_prob(torch.tensor(pts, device=gpu), torch.tensor(q, device=gpu)).cpu().numpy()
    np.testing.assert_allclose(got, ref, rtol=RTOL, atol=ATOL)
    assert (got[ref == 0] == 0).all()
    # root / marginal form (query=None)
    ob0 = OracleBruteForce()
    ob0.fit(nd_, None)
    bf0 = BruteForce({"estimator_name": "brute_force"}, device=gpu)
    bf0.fit(torch.tensor(nd_, device=gpu), None)
    p0 = rng.integers(-1, 6, (1, 9)).astype(np.float32)
    np.testing.assert_allclose(bf0.get_prob(torch.tensor(p0, device=gpu)).cpu().numpy(), ob0.get_prob(p0),
                               rtol=RTOL, atol=ATOL)


def test_empty_and_single_query_edges(gpu):
    data, cols, edges = chain_data(4, 3, 500, 2)
    bn = make_bn(BayesianNetwork, edges, cols, data, device=gpu)
    with pytest.raises(RuntimeError):
        bn.infer("X3", {"X2": torch.zeros((0, 1), device=gpu)}, N_max=3)
    ora = OracleBN(edges, cols, data)
    ev = {"X2": np.array([[1.0]], np.float32)}
    ref, _ = ora.infer("X3", ev, 3)
    pdf, _ = bn.infer("X3", _t(ev, gpu), N_max=3)
    np.testing.assert_allclose(pdf.cpu().numpy(), ref, rtol=RTOL, atol=ATOL)


def _full_golden(name):
    import json
    import os

    z = np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", name + ".npz"), allow_pickle=False)
    return z["rows"], z["pdf"], z["domain"], json.loads(str(z["meta"]))


def _digest(arrs):
    import hashlib

    h = hashlib.sha256()
    for a in arrs:
        h.update(np.ascontiguousarray(a).tobytes())
    return h.hexdigest()


def test_full_batch_config1_matches_reference(gpu):
    """BASELINE configs[1] at full size: bench.py's own rank-0 batch (20-node
    chain, d = 32, 200 000 training rows, 65 536 queries, evidence X0..X18) --
    EVERY row against the reference's BayesianNetwork.infer over the same batch
    (tests/golden/make_golden_full.py), normalised by the max of the whole batch
    (bayesian_network.py:296), at the north-star tolerance."""
    rows, ref, rdom, m = _full_golden("chain20_d32_bench65536")
    data, cols, edges = chain_data(20, 32, 200_000, 3, stay=0.8)
    names = [c for c in cols if c != "X19"]
    ev = sample_evidence(data, cols, names, 65536, 1000)
    assert _digest([data]) == m["data_sha256"] and _digest([ev[k] for k in sorted(ev)]) == m["evidence_sha256"]
    bn = make_bn(BayesianNetwork, edges, cols, data, device=gpu)
    pdf, dom = bn.infer("X19", _t(ev, gpu), N_max=32)
    p = pdf.cpu().numpy()
    assert rows.size == 65536 and p.shape == ref.shape
    np.testing.assert_array_equal(dom.cpu().numpy(), np.broadcast_to(rdom[:1], tuple(dom.shape)))
    assert float(p[m["argmax_row"]].max()) == 1.0 and float(p.max()) == 1.0
    np.testing.assert_allclose(p, ref, rtol=RTOL, atol=ATOL)
    # the raw launch + in-place scale (the sharded step's pieces) gives the same rows
    from continuousbayesiannetwork_amd.distributed import sharded_infer

    one, _ = sharded_infer(bn, "X19", _t(ev, gpu), N_max=32)
    np.testing.assert_array_equal(one.cpu().numpy(), p)


def test_full_batch_config2_slice_matches_reference(gpu):
    """BASELINE configs[2] at full size (tools/bench_alarm.py's batch:
    alarm-like 37-node DAG, target X35, 262 144 queries): a 4 097-row slice
    (every 64th row + the batch argmax row) of the reference's output over the
    WHOLE batch -- normalised by the max of all 262 144 rows -- at rtol 1e-5."""
    rows, ref, rdom, m = _full_golden("alarm37_d8_bench262144")
    data, cols, edges = alarm_like_data(200_000, 5)
    names = [c for c in cols if c != "X35"]
    ev = sample_evidence(data, cols, names, 262144, 0)
    assert _digest([data]) == m["data_sha256"] and _digest([ev[k] for k in sorted(ev)]) == m["evidence_sha256"]
    bn = make_bn(BayesianNetwork, edges, cols, data, device=gpu)
    pdf, dom = bn.infer("X35", _t(ev, gpu), N_max=8)
    p = pdf.cpu().numpy()
    np.testing.assert_array_equal(dom.cpu().numpy(), np.broadcast_to(rdom[:1], tuple(dom.shape)))
    assert float(p[m["argmax_row"]].max()) == 1.0 and float(p.max()) == 1.0
    np.testing.assert_allclose(p[rows], ref, rtol=RTOL, atol=ATOL)


def test_full_size_config1_properties(gpu):
    """BASELINE configs[1] at full size (20-node chain, d=32, 65 536 queries):
    global max is exactly 1, identical evidence rows give identical outputs,
    off-domain evidence rows are all-zero, a sample of rows matches the oracle
    run on the same sample plus the batch's argmax row (so both normalise by
    the same max)."""
    n, d, Q = 20, 32, 65536
    data, cols, edges = chain_data(n, d, 100000, 3, stay=0.8)
    bn = make_bn(BayesianNetwork, edges, cols, data, device=gpu)
    names = [c for c in cols if c != "X19"]
    ev = sample_evidence(data, cols, names, Q, 1)
    ev["X18"][:64] = 99.0  # off-domain
    ev["X18"][64:128] = ev["X18"][128:192]
    for k in names:
        ev[k][64:128] = ev[k][128:192]
    pdf, dom = bn.infer("X19", _t(ev, gpu), N_max=d)
    p = pdf.cpu().numpy()
    assert p.shape == (Q, d) and float(p.max()) == 1.0 and (p >= 0).all()
    assert (p[:64] == 0).all()
    np.testing.assert_array_equal(p[64:128], p[128:192])
    rstar = int(np.argmax(p.max(1)))
    sub = np.append(np.arange(200, 200 + 257), rstar)
    ora = OracleBN(edges, cols, data)
    ref, _ = ora.infer("X19", {k: v[sub] for k, v in ev.items()}, d)
    assert ref[-1].max() == 1.0
    np.testing.assert_allclose(p[sub], ref, rtol=RTOL, atol=ATOL)


def test_split_passes_equal_fused_and_sharded(gpu):
    """Two shards on one GPU with a host-side max exchange == the fused call."""
    from continuousbayesiannetwork_amd.distributed import shard_evidence

    data, cols, edges = chain_data(8, 6, 5000, 4)
    bn = make_bn(BayesianNetwork, edges, cols, data, device=gpu)
    ev = _t(sample_evidence(data, cols, ["X6", "X3", "X1"], 1001, 2), gpu)
    full, _ = bn.infer("X7", ev, N_max=6)
    parts, bits = [], []
    for r in range(2):
        sh = shard_evidence(ev, 2, r)
        plan, cols_, nq, _, dev = bn.engine.prepare("X7", sh, 6)
        bits.append(bn.engine.query_max(plan, cols_, nq, dev).clone())
        parts.append((plan, cols_, nq, dev))
    m = torch.maximum(bits[0], bits[1])
    outs = []
    for plan, cols_, nq, dev in parts:
        o = torch.empty((nq, 6), device=dev)
        outs.append(bn.engine.query_write(plan, cols_, nq, m, o, dev).clone())
    np.testing.assert_array_equal(torch.cat(outs).cpu().numpy(), full.cpu().numpy())


def test_domain_index(gpu):
    dom = torch.tensor([-1.5, 0.25, 2.0, 7.0], device=gpu)
    v = torch.tensor([0.25, 7.0, 3.0, -1.5, 8.0, -9.0], device=gpu)
    assert domain_index(v, dom).cpu().tolist() == [1, 3, -1, 0, -1, -1]


def _star_data(k, d, S, seed):
    """k root parents -> one child (C depends on all parents)."""
    rng = np.random.default_rng(seed)
    P = rng.integers(0, d, (S, k))
    C = (P.sum(1) + rng.integers(0, 3, S)) % d
    X = np.concatenate([P, C[:, None]], 1).astype(np.float32)
    cols = [f"P{i}" for i in range(k)] + ["C"]
    return X, cols, [(f"P{i}", "C") for i in range(k)]


@pytest.mark.parametrize("k,d,N", [(3, 16, 16), (4, 6, 6), (3, 5, 4)])
def test_many_observed_parents_generic_and_global_paths(k, d, N, gpu):
    """> 2 observed parents (generic kernel); k=3, d=16 makes a 256 KiB table
    image, beyond one CU's LDS (global-memory variant)."""
    data, cols, edges = _star_data(k, d, 40000, k * 10 + d)
    ora = OracleBN(edges, cols, data)
    bn = make_bn(BayesianNetwork, edges, cols, data, device=gpu)
    ev = sample_evidence(data, cols, [f"P{i}" for i in range(k)], 700, 3, missing_frac=0.05)
    random.seed(1)
    ref, rdom = ora.infer("C", ev, N)
    random.seed(1)
    pdf, dom = bn.infer("C", _t(ev, gpu), N_max=N)
    np.testing.assert_array_equal(dom.cpu().numpy(), rdom)
    np.testing.assert_allclose(pdf.cpu().numpy(), ref, rtol=RTOL, atol=ATOL)


def test_more_factors_than_fast_path(gpu):
    """40 ancestors (> 32 fast-path factors) and partial evidence (SHARED + QUERY mix)."""
    data, cols, edges = chain_data(40, 3, 4000, 21, stay=0.7)
    ora = OracleBN(edges, cols, data)
    bn = make_bn(BayesianNetwork, edges, cols, data, device=gpu)
    ev = sample_evidence(data, cols, ["X38", "X20", "X3"], 900, 4)
    ref, rdom = ora.infer("X39", ev, 3)
    pdf, dom = bn.infer("X39", _t(ev, gpu), N_max=3)
    np.testing.assert_allclose(pdf.cpu().numpy(), ref, rtol=RTOL, atol=ATOL)


def test_table_cache_mode_matches(gpu):
    data, cols, edges = chain_data(12, 8, 20000, 5, stay=0.8)
    bn = make_bn(BayesianNetwork, edges, cols, data, device=gpu)
    ev = _t(sample_evidence(data, cols, [c for c in cols if c != "X11"], 4097, 6), gpu)
    bn.engine.cache_tables = False
    a, _ = bn.infer("X11", ev, N_max=8)
    a = a.clone()
    bn.engine.cache_tables = True
    b, _ = bn.infer("X11", ev, N_max=8)
    c, _ = bn.infer("X11", ev, N_max=8)
    np.testing.assert_array_equal(a.cpu().numpy(), b.cpu().numpy())
    np.testing.assert_array_equal(a.cpu().numpy(), c.cpu().numpy())


@pytest.mark.parametrize("Q", [1, 100, 4096, 65536, 65537])
def test_single_launch_matches_two_launch(Q, gpu):
    """The fused single-launch path (grid barrier on the max) is bit-identical
    to the two-launch path; batches above its capacity fall back to two launches."""
    data, cols, edges = chain_data(20, 32, 60000, 8, stay=0.8)
    bn = make_bn(BayesianNetwork, edges, cols, data, device=gpu)
    names = [c for c in cols if c != "X19"]
    ev = _t(sample_evidence(data, cols, names, Q, 9), gpu)
    bn.engine.fused = False
    a, _ = bn.infer("X19", ev, N_max=32)
    a = a.clone()
    bn.engine.fused = True
    b, _ = bn.infer("X19", ev, N_max=32)
    torch.cuda.synchronize()
    bn.engine.check_status()
    cap = bn.engine.fused_capacity("X19", names, 32)
    assert cap >= 65536
    np.testing.assert_array_equal(a.cpu().numpy(), b.cpu().numpy())
    if Q <= 64:
        ref, _ = OracleBN(edges, cols, data).infer("X19", {k: v.cpu().numpy() for k, v in ev.items()}, 32)
        np.testing.assert_allclose(b.cpu().numpy(), ref, rtol=RTOL, atol=ATOL)


@pytest.mark.parametrize("Q,shards", [(1001, 2), (65536, 8), (7, 3)])
def test_raw_launch_sharded_equals_single_launch(Q, shards, gpu):
    """Sharded step (one raw launch per shard, MAX of the shards' max words,
    in-place scale) == the single-process infer, bit for bit."""
    from continuousbayesiannetwork_amd.distributed import shard_evidence, sharded_infer

    data, cols, edges = chain_data(20, 32, 60000, 8, stay=0.8)
    bn = make_bn(BayesianNetwork, edges, cols, data, device=gpu)
    names = [c for c in cols if c != "X19"]
    ev = _t(sample_evidence(data, cols, names, Q, 11), gpu)
    full, _ = bn.infer("X19", ev, N_max=32)
    full = full.clone()
    rows, bits, scales = [], [], []
    for r in range(shards):
        res = bn.engine.infer_raw("X19", shard_evidence(ev, shards, r), 32)
        assert res is not None  # fast-path plan takes the raw launch
        o, _, b, sc = res
        rows.append(o)
        bits.append(b.clone())
        scales.append(sc)
    m = torch.stack(bits).max(0).values
    for o, sc in zip(rows, scales):
        sc(o, m)
    np.testing.assert_array_equal(torch.cat(rows).cpu().numpy(), full.cpu().numpy())
    # no process group: sharded_infer over the whole batch == infer
    one, _ = sharded_infer(bn, "X19", ev, N_max=32)
    np.testing.assert_array_equal(one.cpu().numpy(), full.cpu().numpy())


@pytest.mark.parametrize("every,exchange,fold", [(1, False, True), (2, True, True), (3, False, True), (4, True, True),
                                                 (8, True, True), (2, True, False), (8, True, False)])
def test_sharded_stepper_pipelined_equals_infer(every, exchange, fold, gpu):
    """ShardedStepper (raw launch on the compute stream; exchange + batched
    scale of every ``every`` steps on its comm stream; ring of max-word slots)
    over a stream of distinct batches (7 per pass: partial groups flushed by
    wait()) == infer on each batch, bit for bit -- including rows released
    early (the allocator must not recycle them before the comm stream's scale)."""
    from continuousbayesiannetwork_amd.distributed import ShardedStepper

    data, cols, edges = chain_data(20, 32, 60000, 8, stay=0.8)
    bn = make_bn(BayesianNetwork, edges, cols, data, device=gpu)
    names = [c for c in cols if c != "X19"]
    batches = [_t(sample_evidence(data, cols, names, 4096 + 1000 * i, 30 + i), gpu) for i in range(7)]
    ref = [bn.infer("X19", b, N_max=32)[0].clone() for b in batches]
    # exchange: a one-rank RCCL communicator of the stepper's own (no process group)
    st = ShardedStepper(bn, "X19", 32, exchange_every=every, force_exchange=exchange, fold=fold)
    keep = []
    for rep in range(3):
        for i, b in enumerate(batches):
            rows, dom = st.step(b)
            if i % 2 == 0:
                keep.append((i, rows))  # odd steps' rows are dropped right away
    st.wait()
    torch.cuda.synchronize()
    assert st._folded == fold  # staged plan: the folded ring unless disabled
    st.close()
    for i, rows in keep:
        np.testing.assert_array_equal(rows.cpu().numpy(), ref[i].cpu().numpy())


def test_raw_launch_unsupported_plan_falls_back(gpu):
    """Plans off the fast path (a factor with > 4 observed parents) run the
    two-pass exchange."""
    from continuousbayesiannetwork_amd.distributed import sharded_infer

    data, cols, edges = _star_data(5, 4, 20000, 3)
    bn = make_bn(BayesianNetwork, edges, cols, data, device=gpu)
    ev = _t(sample_evidence(data, cols, [f"P{i}" for i in range(5)], 900, 4), gpu)
    assert bn.engine.infer_raw("C", ev, 4) is None
    a, _ = bn.infer("C", ev, N_max=4)
    b, _ = sharded_infer(bn, "C", ev, N_max=4)
    np.testing.assert_array_equal(a.cpu().numpy(), b.cpu().numpy())


@pytest.mark.parametrize("target,Q", [("X35", 262144), ("X35", 1000), ("X36", 262145)])
def test_alarm_like_single_launch_global_tables(target, Q, gpu):
    """configs[2]: table image beyond LDS (8^4-row factors) -> the fused kernel
    reads tables from L2/HBM; it equals the two-launch path bit for bit, and
    the sharded raw step equals both."""
    from continuousbayesiannetwork_amd.distributed import shard_evidence

    data, cols, edges = alarm_like_data(50000, 5)
    names = [c for c in cols if c != target]
    ev = _t(sample_evidence(data, cols, names, Q, 12), gpu)
    bn = make_bn(BayesianNetwork, edges, cols, data, device=gpu)
    bn.engine.fused = False
    a, _ = bn.infer(target, ev, N_max=8)
    a = a.clone()
    bn.engine.fused = True
    b, _ = bn.infer(target, ev, N_max=8)
    b = b.clone()
    torch.cuda.synchronize()
    bn.engine.check_status()
    np.testing.assert_array_equal(a.cpu().numpy(), b.cpu().numpy())
    rows, words, scales = [], [], []
    for r in range(3):
        o, _, w, sc = bn.engine.infer_raw(target, shard_evidence(ev, 3, r), 8)
        rows.append(o)
        words.append(w.clone())
        scales.append(sc)
    m = torch.stack(words).max(0).values
    for o, sc in zip(rows, scales):
        sc(o, m)
    np.testing.assert_array_equal(torch.cat(rows).cpu().numpy(), a.cpu().numpy())


@pytest.mark.parametrize("target,N,missing", [("X35", 8, 0.0), ("X35", 4, 0.05), ("X36", 8, 0.02)])
def test_alarm_like_config2_matches_oracle(target, N, missing, gpu):
    """BASELINE configs[2] shape: ALARM-like 37-node DAG, in-degree <= 4, d=8,
    evidence on every other node (factor tables up to 8^4 rows: beyond LDS,
    the global-memory variant), vs the oracle."""
    data, cols, edges = alarm_like_data(50000, 5)
    names = [c for c in cols if c != target]
    ev = sample_evidence(data, cols, names, 384, 7, missing_frac=missing)
    ora = OracleBN(edges, cols, data)
    bn = make_bn(BayesianNetwork, edges, cols, data, device=gpu)
    random.seed(2)
    ref, rdom = ora.infer(target, ev, N)
    random.seed(2)
    pdf, dom = bn.infer(target, _t(ev, gpu), N_max=N)
    np.testing.assert_array_equal(dom.cpu().numpy(), rdom)
    np.testing.assert_allclose(pdf.cpu().numpy(), ref, rtol=RTOL, atol=ATOL)


def test_config2_cols_off_domain_rows_through_lds_and_global_tables(gpu):
    """configs[2]'s kernel (k_query_cols, CBN_PLAN_COLS) with off-domain
    evidence on a parent of a 4 096-row table (gathered from the image in
    global memory) and on a parent of an 8-row table (in LDS): those rows are
    all zero (BruteForce gives 0 outside the fitted domain, brute_force.py:
    172-244), every other row matches the oracle at rtol 1e-5."""
    from continuousbayesiannetwork_amd import _native

    data, cols, edges = alarm_like_data(50000, 5)
    par = {c: [] for c in cols}
    for a, b in edges:
        par[b].append(a)
    anc, todo = set(), ["X35"]
    while todo:
        for p in par[todo.pop()]:
            if p not in anc:
                anc.add(p)
                todo.append(p)
    fam = sorted(anc) + ["X35"]
    p4 = par[next(n for n in fam if len(par[n]) == 4)][0]
    p1 = next(par[n][0] for n in fam if len(par[n]) == 1 and par[n][0] != p4)
    names = [c for c in cols if c != "X35"]
    ev = sample_evidence(data, cols, names, 512, 21)
    ev[p4][:64] = 99.0
    ev[p1][64:128] = -3.0
    ev[p1][128:130] = 2.5  # between two domain values
    bn = make_bn(BayesianNetwork, edges, cols, data, device=gpu)
    pdf, _ = bn.infer("X35", _t(ev, gpu), N_max=8)
    fp = bn.engine._fast[("X35", tuple(ev.keys()), 8)]
    assert _native.load().cbn_plan_flags(fp.plan.handle) & _native.CBN_PLAN_COLS
    p = pdf.cpu().numpy()
    assert (p[:130] == 0).all() and p.max() == 1.0
    ref, _ = OracleBN(edges, cols, data).infer("X35", ev, 8)
    np.testing.assert_allclose(p, ref, rtol=RTOL, atol=ATOL)


def test_alarm_like_config2_full_batch_properties(gpu):
    """262 144 queries (configs[2] size): max exactly 1; rows of duplicated
    evidence identical; a sample of rows plus the batch argmax row matches the
    oracle on that sample (same normaliser) at rtol 1e-5."""
    data, cols, edges = alarm_like_data(50000, 5)
    names = [c for c in cols if c != "X35"]
    Q = 262144
    ev = sample_evidence(data, cols, names, Q, 8)
    ev["X0"][1] = ev["X0"][0]
    for k in ev:
        ev[k][1] = ev[k][0]
    bn = make_bn(BayesianNetwork, edges, cols, data, device=gpu)
    pdf, _ = bn.infer("X35", _t(ev, gpu), N_max=8)
    p = pdf.cpu().numpy()
    assert p.max() == 1.0
    np.testing.assert_array_equal(p[0], p[1])
    rstar = int(np.argmax(p.max(1)))
    sub = np.append(np.arange(0, Q, Q // 97)[:96], rstar)
    ref, _ = OracleBN(edges, cols, data).infer("X35", {k: v[sub] for k, v in ev.items()}, 8)
    assert ref[-1].max() == 1.0  # the GPU's argmax row is the oracle's too
    np.testing.assert_allclose(p[sub], ref, rtol=RTOL, atol=ATOL)


def test_grid_beyond_64_factors_and_evidence_columns(gpu):
    """configs[4] shape at a size the oracle handles: 9 x 9 grid DAG (81
    factors, 80 evidence columns -- beyond 64 of both), d = 4, vs the oracle
    (N = 4: one lane per query, the per-wave offset table of 81 factors does
    not fit LDS, so this runs the generic kernel); sharded == single call."""
    from continuousbayesiannetwork_amd.distributed import shard_evidence, sharded_infer

    from helpers import grid_data

    data, cols, edges = grid_data(30000, 2, side=9, d=4, keep=0.9)
    target, names = cols[-1], cols[:-1]
    ev = sample_evidence(data, cols, names, 300, 5, missing_frac=0.01)
    ora = OracleBN(edges, cols, data)
    bn = make_bn(BayesianNetwork, edges, cols, data, device=gpu)
    ref, rdom = ora.infer(target, ev, 4)
    pdf, dom = bn.infer(target, _t(ev, gpu), N_max=4)
    np.testing.assert_array_equal(dom.cpu().numpy(), rdom)
    np.testing.assert_allclose(pdf.cpu().numpy(), ref, rtol=RTOL, atol=ATOL)
    evt = _t(ev, gpu)
    one, _ = sharded_infer(bn, target, evt, N_max=4)
    np.testing.assert_array_equal(one.cpu().numpy(), pdf.cpu().numpy())
    for r in range(2):
        part, _ = sharded_infer(bn, target, shard_evidence(evt, 2, r), N_max=4)
        assert part.shape[0] == 150


def test_grid_full_config4_shape_matches_reference_and_oracle(gpu):
    """The full configs[4] plan (10 x 10 grid, d = N = 64, 100 factors, 99
    evidence columns, 85 MB global-table image) with peaked CPDs whose fp32
    products stay finite, vs the REFERENCE's own infer on the same 64 queries
    (tests/golden/make_golden_full.py grid10_d64_peaked_ref64) and the oracle's
    marginals (tests/golden/make_grid_oracle.py; data + evidence regenerated
    from the same seeds); the raw launch + scale path (sharded_infer, no
    process group) == the single call bit for bit."""
    import os

    from continuousbayesiannetwork_amd.distributed import sharded_infer

    from helpers import grid_data

    z = np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "grid10_d64_peaked_oracle.npz"))
    data, cols, edges = grid_data(60000, 3, side=10, d=64, keep=0.995, noise=0)
    target, names = cols[-1], cols[:-1]
    ev = _t(sample_evidence(data, cols, names, 64, 5), gpu)
    bn = make_bn(BayesianNetwork, edges, cols, data, device=gpu)
    pdf, dom = bn.infer(target, ev, N_max=64)
    np.testing.assert_array_equal(dom.cpu().numpy(), z["domain"])
    out = pdf.cpu().numpy()
    assert np.isfinite(out).all()
    np.testing.assert_allclose(out, z["pdf"], rtol=RTOL, atol=ATOL)
    zr = np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "grid10_d64_peaked_ref64.npz"))
    assert list(zr["rows"]) == list(range(64))
    np.testing.assert_array_equal(dom.cpu().numpy()[:1], zr["domain"][:1])
    np.testing.assert_allclose(out, zr["pdf"], rtol=RTOL, atol=ATOL)
    one, _ = sharded_infer(bn, target, ev, N_max=64)
    np.testing.assert_array_equal(one.cpu().numpy(), out)


def test_grid_bench_batch_full_size(gpu):
    """configs[4] at the size it is benchmarked at (tools/bench_grid.py's
    headline batch: 10 x 10 grid, d = N = 64, 100 factors, 65 536 queries --
    k_query_slots' fused launch over two block rounds, round 0's products
    held across the grid barrier, phase B a 3-chunk survivor chain): fused ==
    raw launch + scale (two launches) bit for bit; the UNnormalised rows of
    40 sampled rows, the first and last 128-query block and the batch argmax
    row vs the oracle (tests/golden/make_grid_bench_oracle.py) at rtol 1e-5,
    and the normalised rows vs those over the GPU's max."""
    import os

    from continuousbayesiannetwork_amd import _native
    from continuousbayesiannetwork_amd.distributed import sharded_infer

    from helpers import grid_data

    z = np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "grid10_d64_bench65536_oracle.npz"))
    data, cols, edges = grid_data(400_000, 3, side=10, d=64, keep=0.995, noise=0)
    target, names = cols[-1], cols[:-1]
    ev = _t(sample_evidence(data, cols, names, 65536, 0), gpu)
    bn = make_bn(BayesianNetwork, edges, cols, data, device=gpu)
    pdf, dom = bn.infer(target, ev, N_max=64)
    fp = bn.engine._fast[(target, tuple(ev.keys()), 64)]
    assert _native.load().cbn_plan_flags(fp.plan.handle) & _native.CBN_PLAN_SLOTS
    cap = bn.engine.fused_capacity(target, names, 64)
    assert cap >= 65536 > cap // 2  # the fused two-round launch
    out = pdf.cpu().numpy()
    np.testing.assert_array_equal(dom.cpu().numpy()[:1], z["domain"])
    two, _ = sharded_infer(bn, target, ev, N_max=64)  # raw launch + scale
    np.testing.assert_array_equal(two.cpu().numpy(), out)
    rows, _, words, _ = bn.engine.infer_raw(target, ev, 64)
    raw = rows.cpu().numpy()
    gmax = raw.max()
    assert int(np.argmax(raw.max(1))) == int(z["argmax_row"])
    r = z["rows"]
    np.testing.assert_allclose(raw[r], z["raw"], rtol=RTOL, atol=0)
    assert z["raw"].max() == z["raw"][list(r).index(int(z["argmax_row"]))].max()
    np.testing.assert_allclose(out[r], z["raw"] / z["raw"].max(), rtol=RTOL, atol=ATOL)
    assert out.max() == 1.0 and np.isfinite(out).all()
    assert gmax > 0 and (raw[r] > 0).any(1).mean() > 0.05


def test_grid_fast_path_beyond_64_factors(gpu):
    """9 x 9 grid, d = N = 32 (4 lanes per query): the fast table kernel with
    81 factors and 80 evidence columns -- single launch == two launches ==
    sharded raw launches + scale, bit for bit."""
    from continuousbayesiannetwork_amd.distributed import shard_evidence

    from helpers import grid_data

    data, cols, edges = grid_data(200000, 4, side=9, d=32, keep=0.97)
    target, names = cols[-1], cols[:-1]
    ev = _t(sample_evidence(data, cols, names, 20000, 6), gpu)
    bn = make_bn(BayesianNetwork, edges, cols, data, device=gpu)
    bn.engine.fused = False
    a, _ = bn.infer(target, ev, N_max=32)
    a = a.clone()
    bn.engine.fused = True
    b, _ = bn.infer(target, ev, N_max=32)
    torch.cuda.synchronize()
    bn.engine.check_status()
    np.testing.assert_array_equal(a.cpu().numpy(), b.cpu().numpy())
    rows, words, scales = [], [], []
    for r in range(3):
        res = bn.engine.infer_raw(target, shard_evidence(ev, 3, r), 32)
        assert res is not None  # fast-path plan
        o, _, w, sc = res
        rows.append(o)
        words.append(w.clone())
        scales.append(sc)
    m = torch.stack(words).max(0).values
    for o, sc in zip(rows, scales):
        sc(o, m)
    np.testing.assert_array_equal(torch.cat(rows).cpu().numpy(), a.cpu().numpy())


@pytest.mark.parametrize("which,Q", [("chain16", 200001), ("alarm", 300001)])
def test_cols_plan_fused_two_rounds(which, Q, gpu):
    """k_query_cols' fused single launch over two block rounds (round 5: the
    first round's products held in registers across the grid barrier) == the
    two-launch path bit for bit, with more queries than one round of the
    co-resident grid holds (N = 16 chain: 2 lanes per query; the configs[2]
    alarm plan: 1 lane per query); a sample plus the argmax row matches the
    oracle on that sample (same normaliser)."""
    from continuousbayesiannetwork_amd import _native

    if which == "chain16":
        data, cols, edges = chain_data(20, 16, 60000, 8, stay=0.8)
        target, N = "X19", 16
    else:
        data, cols, edges = alarm_like_data(50000, 5)
        target, N = "X35", 8
    names = [c for c in cols if c != target]
    ev = sample_evidence(data, cols, names, Q, 12)
    bn = make_bn(BayesianNetwork, edges, cols, data, device=gpu)
    evt = _t(ev, gpu)
    pdf, _ = bn.infer(target, evt, N_max=N)
    fp = bn.engine._fast[(target, tuple(ev.keys()), N)]
    assert _native.load().cbn_plan_flags(fp.plan.handle) & _native.CBN_PLAN_COLS
    cap = bn.engine.fused_capacity(target, names, N)
    assert cap >= Q > cap // 2  # two rounds of the fused grid
    p = pdf.cpu().numpy()
    assert p.max() == 1.0
    bn.engine.fused = False
    p2, _ = bn.infer(target, evt, N_max=N)
    np.testing.assert_array_equal(p2.cpu().numpy(), p)
    rstar = int(np.argmax(p.max(1)))
    sub = np.append(np.append(np.arange(0, Q, Q // 40)[:40], [Q - 1]), rstar)
    ref, _ = OracleBN(edges, cols, data).infer(target, {k: v[sub] for k, v in ev.items()}, N)
    assert ref[-1].max() == 1.0
    np.testing.assert_allclose(p[sub], ref, rtol=RTOL, atol=ATOL)


@pytest.mark.parametrize("d,side,Q", [(32, 5, 70001), (64, 4, 40001), (128, 4, 20001)])
def test_slots_plan_lane_counts_rounds_and_survivors(d, side, Q, gpu):
    """k_query_slots (CBN_PLAN_SLOTS: global-table plans of >= 4 lanes per
    query) at L = 4, 8 and 16 lanes per query (N = 32, 64, 128), with more
    queries than one block round holds (ragged last round), a peaked grid whose
    products leave survivors for the phase-B chain, and off-domain evidence
    (the zero row) on a few queries: fused == two launches bit for bit; a
    sample of rows plus the batch argmax row matches the oracle on that
    sample (same normaliser) at rtol 1e-5."""
    from continuousbayesiannetwork_amd import _native

    from helpers import grid_data

    data, cols, edges = grid_data(100000, 7, side=side, d=d, keep=0.995, noise=0)
    target, names = cols[-1], cols[:-1]
    ev = sample_evidence(data, cols, names, Q, 3)
    ev[names[3]][5:9] = float(d + 7)  # off-domain: those queries' rows are all zero
    bn = make_bn(BayesianNetwork, edges, cols, data, device=gpu)
    evt = _t(ev, gpu)
    random.seed(4)
    pdf, _ = bn.infer(target, evt, N_max=d)
    fp = bn.engine._fast[(target, tuple(ev.keys()), d)]
    assert _native.load().cbn_plan_flags(fp.plan.handle) & _native.CBN_PLAN_SLOTS
    p = pdf.cpu().numpy()
    assert p.max() == 1.0 and (p[5:9] == 0).all()
    assert 0.05 < (p > 0).any(1).mean() < 1.0  # survivors and dead queries both present
    bn.engine.fused = not bn.engine.fused
    random.seed(4)
    p2, _ = bn.infer(target, evt, N_max=d)
    np.testing.assert_array_equal(p2.cpu().numpy(), p)
    rstar = int(np.argmax(p.max(1)))
    sub = np.append(np.append(np.arange(0, Q, Q // 40)[:40], [5, Q - 1]), rstar)
    random.seed(4)
    ref, _ = OracleBN(edges, cols, data).infer(target, {k: v[sub] for k, v in ev.items()}, d)
    assert ref[-1].max() == 1.0
    np.testing.assert_allclose(p[sub], ref, rtol=RTOL, atol=ATOL)


def test_redrawn_domains_reuse_one_plan(gpu):
    """N_max above a domain's size: the reference pads it with new random
    values on every call (node.py:302-333).  The engine keeps ONE plan per
    (target, observed set, N) and rewrites its sample-index arrays in place
    per call; every call still matches the oracle drawn with the same seed
    (table plan and direct plan)."""
    data, cols, edges = chain_data(6, 4, 4000, 21)
    ora = OracleBN(edges, cols, data)
    for force_direct in (False, True):
        bn = make_bn(BayesianNetwork, edges, cols, data, device=gpu)
        bn.engine.force_direct = force_direct
        ev = sample_evidence(data, cols, ["X4", "X2"], 200, 6)
        for seed in (1, 2, 3, 2):
            random.seed(seed)
            ref, rdom = ora.infer("X5", ev, 7)
            random.seed(seed)
            pdf, dom = bn.infer("X5", _t(ev, gpu), N_max=7)
            np.testing.assert_array_equal(dom.cpu().numpy(), rdom)
            np.testing.assert_allclose(pdf.cpu().numpy(), ref, rtol=RTOL, atol=ATOL)
        kept = [k for k in bn.engine._plans if k[0] == "redrawn"]
        assert len(kept) == 1 and len(bn.engine._plans) == 1


def test_redrawn_domains_on_the_sharded_path(gpu):
    """Binary variables at N_max = 16 (the reference's default, so every
    sampled domain is padded with random draws per call, node.py:302-333): the
    one-rank sharded_infer, the engine's prepare() (the two-pass route) and the
    ShardedStepper serve the redrawn plan, and each call equals infer drawn
    with the same seed bit for bit (table and direct plans)."""
    from continuousbayesiannetwork_amd.distributed import ShardedStepper, sharded_infer

    data, cols, edges = random_dag_data(9, 2, 3, 4000, 13)
    target = cols[-1]
    ora = OracleBN(edges, cols, data)
    ev = sample_evidence(data, cols, cols[:4], 3000, 8)
    for force_direct in (False, True):
        bn = make_bn(BayesianNetwork, edges, cols, data, device=gpu)
        bn.engine.force_direct = force_direct
        assert bn.engine.redraws(target, ev.keys(), 16)
        for seed in (5, 6):
            random.seed(seed)
            a, adom = bn.infer(target, _t(ev, gpu), N_max=16)
            a = a.clone()
            random.seed(seed)
            ref, _ = ora.infer(target, ev, 16)
            np.testing.assert_allclose(a.cpu().numpy(), ref, rtol=RTOL, atol=ATOL)
            random.seed(seed)
            b, bdom = sharded_infer(bn, target, _t(ev, gpu), N_max=16)
            np.testing.assert_array_equal(b.cpu().numpy(), a.cpu().numpy())
            np.testing.assert_array_equal(bdom.cpu().numpy(), adom.cpu().numpy())
            random.seed(seed)
            plan, cols_, nq, _, dev = bn.engine.prepare(target, _t(ev, gpu), 16)
            assert nq == 3000 and not plan.deterministic
            st = ShardedStepper(bn, target, 16, exchange_every=2)
            random.seed(seed)
            c, _ = st.step(_t(ev, gpu))
            st.wait()
            torch.cuda.synchronize()
            st.close()
            np.testing.assert_array_equal(c.cpu().numpy(), a.cpu().numpy())


@pytest.mark.parametrize("Q0,Q1", [(65536, 65536), (4096, 65536), (65536, 1000), (7, 3)])
def test_raw_launch_with_folded_scale(Q0, Q1, gpu):
    """cbn_plan_run_fold: a raw launch of batch 1 that also divides batch 0's
    raw rows by batch 0's max words (bayesian_network.py:296 for that batch):
    batch 1's raw rows and words equal a plain raw launch's, and batch 0's
    rows equal the single-process infer bit for bit (both batch-size orders:
    the fold slice per block differs from the launch's own)."""
    import ctypes

    from continuousbayesiannetwork_amd import _native

    data, cols, edges = chain_data(20, 32, 60000, 8, stay=0.8)
    bn = make_bn(BayesianNetwork, edges, cols, data, device=gpu)
    names = [c for c in cols if c != "X19"]
    e0 = _t(sample_evidence(data, cols, names, Q0, 71), gpu)
    e1 = _t(sample_evidence(data, cols, names, Q1, 72), gpu)
    ref0 = bn.infer("X19", e0, N_max=32)[0].clone()
    rows1, _, w1, sc1 = bn.engine.infer_raw("X19", e1, 32)
    rows1, w1 = rows1.clone(), w1.clone()
    rows0, _, w0, _ = bn.engine.infer_raw("X19", e0, 32)
    rows0, w0 = rows0.clone(), w0.clone()
    plan = next(iter(bn.engine._plans.values()))
    assert _native.load().cbn_plan_flags(plan.handle) & _native.CBN_PLAN_STAGED
    fp = bn.engine.raw_fast_path("X19", e1, 32)
    ptrs = (ctypes.c_void_p * len(fp.slot_keys))(*[e1[k].data_ptr() for k in fp.slot_keys])
    out1 = torch.empty_like(rows1)
    words = torch.zeros_like(w1)
    rc = _native.load().cbn_plan_run_fold(plan.handle, Q1, ptrs, len(fp.slot_keys), words.data_ptr(),
                                          out1.data_ptr(), rows0.data_ptr(), rows0.numel(), w0.data_ptr(),
                                          w0.numel(), 0, _native.stream_ptr(gpu))
    _native.check(rc, "cbn_plan_run_fold")
    torch.cuda.synchronize()
    np.testing.assert_array_equal(out1.cpu().numpy(), rows1.cpu().numpy())
    np.testing.assert_array_equal(words.cpu().numpy(), w1.cpu().numpy())
    np.testing.assert_array_equal(rows0.cpu().numpy(), ref0.cpu().numpy())


FREE_PARENT_GRIDS = ["grid10_d64_dense_ref", "grid10_d64_rows_ref", "grid10_d64_rows_x99_ref"]


@pytest.mark.parametrize("name", FREE_PARENT_GRIDS)
@pytest.mark.parametrize("direct", [False, True], ids=["tables", "direct"])
def test_grid_free_parent_means_match_reference(name, direct, gpu):
    """Free-parent means at configs[4]'s size, pinned by the REFERENCE's own
    infer (tests/golden/make_golden_full.py): d = N = 64 grids with evidence
    on the even grid rows only, so every factor with a parent in an odd row
    averages over that parent's 64 sample points (4 096 meshgrid combos in
    the reference, node.py:206-284 -> bayesian_network.py:271-293) --
    k_build_tables' table rows, and (``direct``) k_query_direct's per-(query,
    column) means.  Cases: the full 100-factor X99 plan (86 factors with a
    free parent, 4 queries), 32 queries on X33 (10 free-parent factors), and
    a dense case (X21, ~24 % of the marginals nonzero)."""
    import json
    import os
    import sys

    here = os.path.dirname(os.path.abspath(__file__))
    sys.path.insert(0, os.path.join(here, "golden"))
    from make_golden_full import CASES, digest, make_case

    z = np.load(os.path.join(here, "golden", name + ".npz"))
    meta = json.loads(str(z["meta"]))
    data, cols, edges, ev_np = make_case(CASES[name])
    assert digest([data]) == meta["data_sha256"]
    assert digest([ev_np[k] for k in sorted(ev_np)]) == meta["evidence_sha256"]
    bn = make_bn(BayesianNetwork, edges, cols, data, device=gpu)
    bn.engine.force_direct = direct
    random.seed(0)
    pdf, dom = bn.infer(meta["target"], _t(ev_np, gpu), N_max=meta["N_max"])
    out = pdf.cpu().numpy()
    ref = z["pdf"]
    assert list(z["rows"]) == list(range(meta["Q"]))
    np.testing.assert_array_equal(dom.cpu().numpy()[:1], z["domain"][:1])
    np.testing.assert_array_equal(out > 0, ref > 0)  # same support
    np.testing.assert_allclose(out, ref, rtol=RTOL, atol=ATOL)
    nz = ref > 0
    assert np.isfinite(ref).all() and nz.any()
    # relative agreement on the nonzero marginals themselves (atol aside)
    assert float(np.max(np.abs(out[nz] - ref[nz]) / ref[nz])) <= RTOL
