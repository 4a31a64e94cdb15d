"""Direct inference plans (csrc/cbn_direct.hip) and hashed BruteForce CPDs.

The reference's BruteForce (cbn/parameter_learning/brute_force.py:172-244)
answers any fitted data by scanning its unique rows, so networks with > 8
parents per node, continuous columns and high-cardinality domains all infer.
Here those plans evaluate every factor per (query, sample column) straight
from the CPD -- dense, or a hash table of the unique rows when the dense one
would exceed ``dense_limit`` cells.  Checked against the reference's own
outputs (tests/golden/make_golden.py: wide*, hicard*, cont4*), and every
other golden re-run with the direct plans forced and with every CPD forced
into the hash table.  Tolerance: rtol 1e-5, atol 1e-7 (north star); NaN rows
(all-zero products, 0/0 in the reference) must be NaN here too.
"""
import random

import numpy as np
import pytest
import torch

from continuousbayesiannetwork_amd import BayesianNetwork, BruteForce, _native
from golden_io import golden_names, load_golden, width_n_only
from helpers import continuous_free_data, hicard_data, make_bn, sample_evidence, wide_data
from oracle.ref_infer import OracleBN, OracleBruteForce

pytestmark = pytest.mark.gpu
RTOL, ATOL = 1e-5, 1e-7
DIRECT_GOLDENS = ["wide10_free2", "wide12_all", "hicard40_all", "hicard40_free1", "cont4_all", "cont4_free1",
                  "cont4_free_support"]
OK_GOLDENS = [n for n in golden_names() if not load_golden(n)["meta"]["error"]]
WIDE_GOLDENS = [n for n in OK_GOLDENS if width_n_only(load_golden(n)["meta"])]


def _t(ev, dev):
    return {k: torch.tensor(v, device=dev) for k, v in ev.items()}


def _run_golden(name, gpu, force_direct=False, dense_limit=None):
    g = load_golden(name)
    m = g["meta"]
    bn = make_bn(BayesianNetwork, m["edges"], m["columns"], g["data"], device=gpu)
    bn.engine.force_direct = force_direct
    if dense_limit is not None:
        for nd in bn.nodes_obj.values():
            nd.estimator.dense_limit = dense_limit
    ev = None if m["evidence_none"] else _t({k: g["evidence"][k] for k in m["evidence"]}, gpu)
    random.seed(m["seed"])
    pdf, dom = bn.infer(m["target"], ev, N_max=m["N_max"])
    np.testing.assert_array_equal(dom.cpu().numpy(), g["domain"])
    np.testing.assert_allclose(pdf.cpu().numpy(), g["pdf"], rtol=RTOL, atol=ATOL)
    return bn, pdf


def _plan_flags(bn):
    lib = _native.load()
    return [lib.cbn_plan_flags(p.handle) for p in bn.engine._plans.values()]


@pytest.mark.parametrize("name", DIRECT_GOLDENS)
def test_direct_goldens_route_to_direct_plans(name, gpu):
    """> 8 parents and CPDs above the dense limit take direct plans by themselves."""
    bn, _ = _run_golden(name, gpu)
    flags = _plan_flags(bn)
    if flags:  # deterministic plans are cached; oversampled ones are rebuilt per call
        assert all(f & _native.CBN_PLAN_DIRECT for f in flags)
    if name.startswith(("hicard", "cont")):
        tgt = load_golden(name)["meta"]["target"]
        assert bn.nodes_obj[tgt].estimator.sparse


@pytest.mark.parametrize("name", OK_GOLDENS)
def test_forced_direct_matches_reference(name, gpu):
    _run_golden(name, gpu, force_direct=True)


@pytest.mark.parametrize("name", OK_GOLDENS)
def test_forced_hashed_cpds_match_reference(name, gpu):
    """Every CPD in the hash table (dense_limit = 1): the sparse representation
    on the whole golden set, free parents and off-domain evidence included."""
    bn, _ = _run_golden(name, gpu, dense_limit=1)
    assert all(nd.estimator.sparse for nd in bn.nodes_obj.values() if nd.estimator._compiled and
               len(nd.estimator.domains) > 0 and nd.estimator.n_cells() > 1)


@pytest.mark.parametrize("dense_limit", [None, 1])
def test_bruteforce_get_prob_wide_and_hashed(dense_limit, gpu):
    """BruteForce._get_prob (brute_force.py:172-244) with 11 columns (beyond
    the dense evaluator) and with a hashed CPD, on- and off-domain points."""
    rng = np.random.default_rng(3)
    k = 10
    pd_ = rng.integers(0, 2, (k, 6000)).astype(np.float32)
    nd_ = ((pd_.sum(0) + rng.integers(0, 2, 6000)) % 3).astype(np.float32)
    ob = OracleBruteForce()
    ob.fit(nd_, pd_)
    kw = {} if dense_limit is None else {"dense_limit": dense_limit}
    bf = BruteForce({"estimator_name": "brute_force"}, device=gpu, **kw)
    bf.fit(torch.tensor(nd_, device=gpu), torch.tensor(pd_, device=gpu))
    pts = rng.integers(-1, 4, (200, 5)).astype(np.float32)
    q = rng.integers(0, 2, (200, k, 1)).astype(np.float32)
    q[::9, 3, 0] = -1  # off-domain parent value
    ref = ob.get_prob(pts, q)
    got = bf.get_prob(torch.tensor(pts, device=gpu), torch.tensor(q, device=gpu)).cpu().numpy()
    np.testing.assert_allclose(got, ref, rtol=RTOL, atol=ATOL)
    assert (got[ref == 0] == 0).all() and (ref > 0).mean() > 0.05
    assert bf.sparse == (dense_limit == 1)


def test_continuous_get_prob_hashed(gpu):
    """Continuous columns (~1 500 distinct values each): the CPD is hashed by
    size; conditionals at data rows and at perturbed (absent) values."""
    data, cols, _ = continuous_free_data(20000, 5)
    ob = OracleBruteForce()
    ob.fit(data[:, 3], data[:, :3].T)
    bf = BruteForce({"estimator_name": "brute_force"}, device=gpu)
    bf.fit(torch.tensor(data[:, 3], device=gpu), torch.tensor(data[:, :3].T.copy(), device=gpu))
    rng = np.random.default_rng(1)
    rows = rng.integers(0, 20000, 300)
    q = data[rows, :3][:, :, None].copy()
    q[::7, 0, 0] += 0.005  # off-domain
    pts = np.tile(np.arange(8, dtype=np.float32), (300, 1))
    ref = ob.get_prob(pts, q)
    got = bf.get_prob(torch.tensor(pts, device=gpu), torch.tensor(q, device=gpu)).cpu().numpy()
    assert bf.sparse
    np.testing.assert_allclose(got, ref, rtol=RTOL, atol=ATOL)
    assert (ref > 0).any(1).mean() > 0.8


def test_direct_raw_scale_and_stepper_equal_infer(gpu):
    """The raw launch (+ scale) and the sharded stepper on a direct plan give
    the infer result bit for bit."""
    from continuousbayesiannetwork_amd.distributed import ShardedStepper

    data, cols, edges = hicard_data(20000, 33)
    bn = make_bn(BayesianNetwork, edges, cols, data, device=gpu)
    ev = _t(sample_evidence(data, cols, ["R0", "R1", "R2", "R3"], 5000, 4), gpu)
    a, _ = bn.infer("E", ev, N_max=40)
    assert all(f & _native.CBN_PLAN_DIRECT for f in _plan_flags(bn))
    rows, _, words, scale = bn.engine.infer_raw("E", ev, 40)
    scale(rows, words)
    np.testing.assert_array_equal(rows.cpu().numpy(), a.cpu().numpy())
    for gather in (False, True):
        st = ShardedStepper(bn, "E", 40, exchange_every=2, force_exchange=True, gather=gather)
        outs = [st.step(ev)[0] for _ in range(3)]
        st.wait()
        torch.cuda.synchronize()
        for o in outs:
            np.testing.assert_array_equal(o.cpu().numpy(), a.cpu().numpy())
        st.close()


def test_direct_full_batch_matches_oracle(gpu):
    """65 536 queries on the continuous network (hashed CPD, one free parent,
    N_max above its cardinality: the random padding is redrawn per call):
    sampled rows and the GPU's argmax row against the oracle, normalised by
    the oracle's value of that argmax row (the reference divides by the max
    of the whole batch)."""
    data, cols, edges = continuous_free_data(20000, 37)
    bn = make_bn(BayesianNetwork, edges, cols, data, device=gpu)
    evn = sample_evidence(data, cols, ["X0", "X1"], 65536, 11, missing_frac=0.05)
    random.seed(21)
    pdf, _ = bn.infer("X3", _t(evn, gpu), N_max=8)
    pdf = pdf.cpu().numpy()
    assert bn.nodes_obj["X3"].estimator.sparse
    assert pdf.max() == 1.0
    r_star = int(np.argmax(pdf.max(1)))
    pick = sorted(set(range(0, 65536, 8191)) | {r_star})
    random.seed(21)
    raw = OracleBN(edges, cols, data).infer_raw("X3", {k: v[pick] for k, v in evn.items()}, 8)[0]
    ref = raw / raw[pick.index(r_star)].max()
    np.testing.assert_allclose(pdf[pick], ref, rtol=RTOL, atol=ATOL)


def test_wide_node_many_parents_oracle(gpu):
    """A 16-parent node (wide_data), every parent observed, off-domain values."""
    data, cols, edges = wide_data(6000, 8, k=16)
    ora = OracleBN(edges, cols, data)
    bn = make_bn(BayesianNetwork, edges, cols, data, device=gpu)
    ev = sample_evidence(data, cols, [f"P{i}" for i in range(16)], 300, 2, missing_frac=0.02)
    ref, rdom = ora.infer("Y", ev, 3)
    pdf, dom = bn.infer("Y", _t(ev, gpu), N_max=3)
    np.testing.assert_array_equal(dom.cpu().numpy(), rdom)
    np.testing.assert_allclose(pdf.cpu().numpy(), ref, rtol=RTOL, atol=ATOL)
    assert all(f & _native.CBN_PLAN_DIRECT for f in _plan_flags(bn))


def test_direct_free_combos_beyond_2_20_and_the_call_bound(gpu):
    """Direct-plan work bounds: a factor with 6 free 16-level
    parents at N = 16 has 16^6 = 16.7 M free-parent combos (refused before
    round 4 by a fixed 2^20 cap) -- it now runs, and its free-parent mean
    matches an fp64 numpy evaluation of the fitted CPD; a call whose work
    (queries x columns x combos) exceeds 2^40 CPD lookups is refused with
    NativeError (CBN_E_LIMIT) before anything launches, and so is a plan whose
    (query, column) threads would each loop over more than 2^26 combos."""
    S, k, d = 200_000, 7, 16
    rng = np.random.default_rng(11)
    P = rng.integers(0, d, (S, k))
    Y = (P[:, 0] + P[:, 1] + rng.choice(3, S, p=[0.7, 0.2, 0.1])) % 3
    X = np.concatenate([P, Y[:, None]], 1).astype(np.float32)
    cols = [f"P{i}" for i in range(k)] + ["Y"]
    edges = [(f"P{i}", "Y") for i in range(k)]
    bn = make_bn(BayesianNetwork, edges, cols, X, device=gpu)
    ev_np = {"P0": np.array([[3.0], [11.0]], np.float32)}
    random.seed(5)
    pdf, dom = bn.infer("Y", _t(ev_np, gpu), N_max=d)
    out, pts = pdf.cpu().numpy(), dom.cpu().numpy()[0]
    # fp64 reference of the Y factor: (1/16^6) sum over the present parent
    # combos p (p0 = e) of P(y | p) = joint / (parent marginal + 1e-10)
    rows, counts = np.unique(X, axis=0, return_counts=True)
    probs = counts.astype(np.float32) / np.float32(counts.sum())
    par = {}
    for r, pr in zip(rows, probs):
        key = tuple(r[:k])
        par[key] = np.float32(par.get(key, np.float32(0)) + pr)
    x = np.zeros((2, d))
    for qi, e in enumerate(ev_np["P0"][:, 0]):
        for r, pr in zip(rows, probs):
            if r[0] != e:
                continue
            for j, y in enumerate(pts):
                if r[k] == y:
                    x[qi, j] += float(np.float32(pr / (par[tuple(r[:k])] + np.float32(1e-10))))
    x /= float(d) ** 6
    np.testing.assert_allclose(out, x / x.max(), rtol=2e-5, atol=1e-7)
    assert (out > 0).sum() >= 4
    # the call bound: 8192 queries x 16 columns x 16^6 combos = 2.2e12 lookups > 2^40
    big = {"P0": torch.full((8192, 1), 3.0, device=gpu)}
    with pytest.raises(_native.NativeError, match="split the batch"):
        bn.infer("Y", big, N_max=d)
    # the per-thread bound: without evidence Y's factor averages
    # 16^7 = 2^28 combos per column in ONE thread's serial loop -- refused at
    # plan creation whatever the batch (a one-query call is no shorter)
    bn.engine.force_direct = True
    with pytest.raises(_native.NativeError, match=r"2\^26"):
        bn.infer("Y", {}, N_max=d)


# ---------------------------------------------------------------------------
# [Q, N] evidence columns read through .expand (round 6).  A node whose
# evidence keys are not all its parents expands each observed column to
# [Q, N] (node.py:246-248); a width-N column is then N per-query sample values
# of that parent, entering the meshgrid like a free parent's samples
# (node.py:335-375), and the factor is the mean over all the combos
# (bayesian_network.py:292).  The engine runs such calls on a direct plan
# whose wide parents read their values per (query, combo)
# (cbn_direct_factor.parent_ev_width, ABI 5).
def _wide_net(S=6000, seed=3, d=4):
    rng = np.random.default_rng(seed)
    A = rng.integers(0, d, S)
    B = rng.integers(0, d, S)
    C = (A + B + rng.integers(0, 2, S)) % d
    D = (A + rng.integers(0, 2, S)) % d
    E = (C + D + rng.integers(0, 2, S)) % d
    data = np.stack([A, B, C, D, E], 1).astype(np.float32)
    cols = ["A", "B", "C", "D", "E"]
    edges = [("A", "C"), ("B", "C"), ("C", "E"), ("D", "E"), ("A", "D")]
    return data, cols, edges


@pytest.mark.parametrize("name", WIDE_GOLDENS)
def test_wide_golden_raw_and_sharded_paths(name, gpu):
    """The reference's own [Q, N] fixture (multi_widthN_partial) through the
    raw launch + scale (sharded_infer, no process group) as well as infer."""
    from continuousbayesiannetwork_amd.distributed import sharded_infer

    bn, pdf = _run_golden(name, gpu)
    m = load_golden(name)["meta"]
    g = load_golden(name)
    ev = _t({k: g["evidence"][k] for k in m["evidence"]}, gpu)
    random.seed(m["seed"])
    two, _ = sharded_infer(bn, m["target"], ev, N_max=m["N_max"])
    np.testing.assert_array_equal(two.cpu().numpy(), pdf.cpu().numpy())


@pytest.mark.parametrize("N,Q", [(4, 3000), (3, 257), (6, 999)])
def test_wide_columns_match_oracle(N, Q, gpu):
    """E's parents C, D with evidence on C only (the expand path): C given as
    [Q, N] per-query values (some off the domain), plus D free -- N x N combos
    per query; A -> C and A -> D give the other factors.  N = 6 > |domain| = 4:
    the redrawn sample domains (node.py:302-333) of the same call, drawn in the
    reference's order.  infer, the repeat call (cached wide plan) and the raw
    path match the oracle; the [Q, 1] call on the same engine still takes its
    own plan.  ShardedStepper declines [Q, N] columns (NotImplementedError)."""
    from continuousbayesiannetwork_amd.distributed import ShardedStepper, sharded_infer

    data, cols, edges = _wide_net()
    rng = np.random.default_rng(N * 7 + Q)
    cw = rng.integers(0, 4, (Q, N)).astype(np.float32)
    cw[::17, 0] = 9.0  # off the fitted domain: that combo's pdf is 0
    ev = {"C": cw}
    ora = OracleBN(edges, cols, data)
    bn = make_bn(BayesianNetwork, edges, cols, data, device=gpu)
    for _ in range(2):
        random.seed(11)
        ref, rdom = ora.infer("E", ev, N)
        random.seed(11)
        pdf, dom = bn.infer("E", _t(ev, gpu), N_max=N)
        np.testing.assert_array_equal(dom.cpu().numpy(), rdom)
        np.testing.assert_allclose(pdf.cpu().numpy(), ref, rtol=RTOL, atol=ATOL)
    random.seed(11)
    two, _ = sharded_infer(bn, "E", _t(ev, gpu), N_max=N)
    np.testing.assert_allclose(two.cpu().numpy(), ref, rtol=RTOL, atol=ATOL)
    ev1 = {"C": cw[:, :1].copy()}
    random.seed(12)
    ref1, _ = ora.infer("E", ev1, N)
    random.seed(12)
    pdf1, _ = bn.infer("E", _t(ev1, gpu), N_max=N)
    np.testing.assert_allclose(pdf1.cpu().numpy(), ref1, rtol=RTOL, atol=ATOL)
    if N <= 4:  # deterministic plans: the pipelined stepper
        st = ShardedStepper(bn, "E", N)
        if bn.engine.raw_word_count("E", ev.keys(), N) > 0:  # its native ring takes [Q, 1] columns only
            with pytest.raises(NotImplementedError):
                st.step(_t(ev, gpu))
        else:  # no raw launch on the table plan: the stepper serves the call through sharded_infer
            random.seed(11)
            rows = st.step(_t(ev, gpu))[0]
            st.wait()
            np.testing.assert_allclose(rows.cpu().numpy(), ref, rtol=RTOL, atol=ATOL)
        st.close()


def test_redrawn_plan_rebuilds_tables_when_host_path_declines(gpu):
    """A redrawn plan (N = 6 > |domain| = 4: new sample points every call)
    whose next call's evidence the native host path declines (float64, a
    [Q, N] column) must still rebuild its tables for that call's draws: the
    flags computed for a declined host call do not count as a launch."""
    data, cols, edges = _wide_net()
    ora = OracleBN(edges, cols, data)
    bn = make_bn(BayesianNetwork, edges, cols, data, device=gpu)
    rng = np.random.default_rng(3)
    c1 = rng.integers(0, 4, (500, 1)).astype(np.float32)
    cw = rng.integers(0, 4, (500, 6)).astype(np.float32)
    for seed, ev, dt in ((21, {"C": c1}, torch.float32), (22, {"C": c1}, torch.float64), (23, {"C": cw}, torch.float32),
                         (24, {"C": c1}, torch.float32), (25, {"C": c1}, torch.float64)):
        random.seed(seed)
        ref, _ = ora.infer("E", ev, 6)
        random.seed(seed)
        pdf, _ = bn.infer("E", {k: torch.tensor(v, device=gpu, dtype=dt) for k, v in ev.items()}, N_max=6)
        np.testing.assert_allclose(pdf.cpu().numpy(), ref, rtol=RTOL, atol=ATOL)
