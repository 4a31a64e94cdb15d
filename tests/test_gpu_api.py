"""API-level behaviour of the HIP engine that the parity tests do not reach:
the default ``device="cuda"`` (no index), stale plans after a refit, the
timeout reporting of the single-launch path, caller-supplied ``out``
validation, and the pipelined sharded stepper with the all-gather reassembly
(one rank over RCCL).  Tolerance where values are compared: rtol 1e-5, atol
1e-7 (north star)."""
import ctypes
import random

import numpy as np
import pytest
import torch

from continuousbayesiannetwork_amd import BayesianNetwork, _native
from helpers import chain_data, make_bn, sample_evidence
from oracle.ref_infer import OracleBN

pytestmark = pytest.mark.gpu
RTOL, ATOL = 1e-5, 1e-7


def _t(ev, dev):
    return {k: torch.tensor(v, device=dev) for k, v in ev.items()}


def test_default_cuda_device_without_index(gpu):
    """BayesianNetwork(device="cuda") (the reference's default form): infer
    twice (the cached native fast path), infer_raw and the stepper all work."""
    from continuousbayesiannetwork_amd.distributed import ShardedStepper

    data, cols, edges = chain_data(8, 8, 5000, 4, stay=0.7)
    bn = make_bn(BayesianNetwork, edges, cols, data, device="cuda")
    names = [c for c in cols if c != "X7"]
    ev = _t(sample_evidence(data, cols, names, 777, 2), "cuda")
    a, _ = bn.infer("X7", ev, N_max=8)
    b, _ = bn.infer("X7", ev, N_max=8)
    ref, _ = OracleBN(edges, cols, data).infer("X7", {k: v.cpu().numpy() for k, v in ev.items()}, 8)
    np.testing.assert_allclose(a.cpu().numpy(), ref, rtol=RTOL, atol=ATOL)
    np.testing.assert_array_equal(a.cpu().numpy(), b.cpu().numpy())
    rows, _, words, scale = bn.engine.infer_raw("X7", ev, 8)
    scale(rows, words)
    np.testing.assert_array_equal(rows.cpu().numpy(), a.cpu().numpy())
    st = ShardedStepper(bn, "X7", 8, exchange_every=2)
    r, _ = st.step(ev)
    st.wait()
    torch.cuda.synchronize()
    np.testing.assert_array_equal(r.cpu().numpy(), a.cpu().numpy())
    st.close()


def test_refit_drops_cached_plans(gpu):
    """A node refitted on other data after a cached infer: the next infer
    follows the new CPD (plans hold raw pointers into the old one)."""
    from oracle.ref_infer import OracleNode

    data, cols, edges = chain_data(6, 4, 4000, 5, stay=0.8)
    data2, _, _ = chain_data(6, 4, 4000, 6, stay=0.3)
    bn = make_bn(BayesianNetwork, edges, cols, data, device=gpu)
    ev = sample_evidence(data, cols, ["X4", "X2"], 300, 3)
    bn.infer("X5", _t(ev, gpu), N_max=4)
    bn.infer("X5", _t(ev, gpu), N_max=4)
    # refit X5 | X4 on the second data set through the Node API
    y, x = data2[:, cols.index("X5")], data2[:, cols.index("X4")][None, :]
    bn.nodes_obj["X5"].fit(torch.tensor(y, device=gpu), torch.tensor(x, device=gpu))
    got, _ = bn.infer("X5", _t(ev, gpu), N_max=4)
    ora = OracleBN(edges, cols, data)
    node = OracleNode("X5", ["X4"])
    node.fit(y, x)
    ora.nodes["X5"] = node
    ref, _ = ora.infer("X5", ev, 4)
    np.testing.assert_allclose(got.cpu().numpy(), ref, rtol=RTOL, atol=ATOL)


def test_timeout_is_reported_on_next_call(gpu):
    """A fused launch that timed out in its grid barrier (simulated through the
    test hook) is reported by the plan's next call as CBN_E_TIMEOUT (NativeError),
    and cleared."""
    data, cols, edges = chain_data(20, 32, 60000, 8, stay=0.8)
    bn = make_bn(BayesianNetwork, edges, cols, data, device=gpu)
    names = [c for c in cols if c != "X19"]
    ev = _t(sample_evidence(data, cols, names, 4096, 9), gpu)
    a, _ = bn.infer("X19", ev, N_max=32)
    plan = next(iter(bn.engine._plans.values()))
    lib = _native.load()
    _native.check(lib.cbn_debug_flag_timeout(plan.handle), "flag")
    with pytest.raises(_native.NativeError, match="timed out"):
        bn.infer("X19", ev, N_max=32)
    b, _ = bn.infer("X19", ev, N_max=32)  # cleared
    np.testing.assert_array_equal(a.cpu().numpy(), b.cpu().numpy())


def test_timeout_is_reported_at_synchronize(gpu):
    """engine.synchronize() reports a timed-out fused call (simulated through
    the test hook) at the caller's sync point, not on the plan's next call."""
    data, cols, edges = chain_data(20, 32, 60000, 8, stay=0.8)
    bn = make_bn(BayesianNetwork, edges, cols, data, device=gpu)
    names = [c for c in cols if c != "X19"]
    ev = _t(sample_evidence(data, cols, names, 4096, 9), gpu)
    a, _ = bn.infer("X19", ev, N_max=32)
    bn.engine.synchronize()  # nothing to report
    plan = next(iter(bn.engine._plans.values()))
    _native.check(_native.load().cbn_debug_flag_timeout(plan.handle), "flag")
    with pytest.raises(_native.NativeError, match="timed out"):
        bn.engine.synchronize()
    b, _ = bn.infer("X19", ev, N_max=32)  # reported once, then cleared
    np.testing.assert_array_equal(a.cpu().numpy(), b.cpu().numpy())


def test_out_argument_is_validated(gpu):
    data, cols, edges = chain_data(6, 4, 3000, 5, stay=0.8)
    bn = make_bn(BayesianNetwork, edges, cols, data, device=gpu)
    ev = _t(sample_evidence(data, cols, ["X4"], 100, 3), gpu)
    bn.infer("X5", ev, N_max=4)
    good = torch.empty((100, 4), device=gpu)
    r, _ = bn.engine.infer("X5", ev, 4, out=good)
    assert r.data_ptr() == good.data_ptr()
    for bad in (torch.empty((99, 4), device=gpu), torch.empty((100, 4), device=gpu, dtype=torch.float64),
                torch.empty((4, 100), device=gpu).t()):
        with pytest.raises((ValueError, RuntimeError)):
            bn.engine.infer("X5", ev, 4, out=bad)


@pytest.mark.parametrize("every", [1, 3])
def test_stepper_gather_one_rank(every, gpu):
    """The reassembly path of the stepper over a one-rank RCCL communicator:
    the returned full tensor equals infer on the batch, for partial groups and
    an empty batch in the stream."""
    from continuousbayesiannetwork_amd.distributed import ShardedStepper

    data, cols, edges = chain_data(20, 32, 60000, 8, stay=0.8)
    bn = make_bn(BayesianNetwork, edges, cols, data, device=gpu)
    names = [c for c in cols if c != "X19"]
    sizes = [5000, 0, 777, 65536, 1]
    batches = [_t(sample_evidence(data, cols, names, q, 60 + i), gpu) for i, q in enumerate(sizes)]
    refs = [bn.infer("X19", b, N_max=32)[0].clone() if q else None for b, q in zip(batches, sizes)]
    st = ShardedStepper(bn, "X19", 32, exchange_every=every, force_exchange=True, gather=True)
    outs = [st.step(b)[0] for b in batches]
    st.wait()
    torch.cuda.synchronize()
    for o, r, q in zip(outs, refs, sizes):
        assert o.shape == (q, 32)
        if q:
            np.testing.assert_array_equal(o.cpu().numpy(), r.cpu().numpy())
    st.close()


def test_stepper_rebinds_after_refit_and_other_networks_keep_plans(gpu):
    """A refit of one of the network's nodes destroys its plans; the
    ShardedStepper, which holds the raw plan handle natively, finishes what it
    enqueued and rebinds to the rebuilt plan (no launch on a freed plan).  A
    refit in ANOTHER network leaves this network's plans alone."""
    from continuousbayesiannetwork_amd.distributed import ShardedStepper

    data, cols, edges = chain_data(8, 4, 4000, 5, stay=0.8)
    data2, _, _ = chain_data(8, 4, 4000, 6, stay=0.3)
    bn = make_bn(BayesianNetwork, edges, cols, data, device=gpu)
    other = make_bn(BayesianNetwork, edges, cols, data, device=gpu)
    ev = _t(sample_evidence(data, cols, ["X6", "X3"], 2000, 3), gpu)
    st = ShardedStepper(bn, "X7", 4, exchange_every=4)
    r0, _ = st.step(ev)
    h0 = next(iter(bn.engine._plans.values())).handle.value
    ep = bn.engine.epoch
    other.nodes_obj["X7"].fit(torch.tensor(data2[:, 7], device=gpu), torch.tensor(data2[:, 6][None, :], device=gpu))
    r1, _ = st.step(ev)  # another network changed: same plan
    assert bn.engine.epoch == ep and next(iter(bn.engine._plans.values())).handle.value == h0
    bn.nodes_obj["X7"].fit(torch.tensor(data2[:, 7], device=gpu), torch.tensor(data2[:, 6][None, :], device=gpu))
    r2, _ = st.step(ev)  # this network changed: plans rebuilt, the stepper rebinds
    assert bn.engine.epoch == ep + 1
    st.wait()
    torch.cuda.synchronize()
    st.close()
    a = bn.infer("X7", ev, N_max=4)[0]
    np.testing.assert_array_equal(r2.cpu().numpy(), a.cpu().numpy())
    np.testing.assert_array_equal(r0.cpu().numpy(), r1.cpu().numpy())
    assert not np.array_equal(r1.cpu().numpy(), r2.cpu().numpy())


def test_variable_elimination_query_matches_reference_golden(gpu):
    """cbn.inference.VariableElimination.query (the north star's entry point;
    the reference's ExactInference is a stub, so query is BayesianNetwork.infer,
    bayesian_network.py:208-305) against a reference-generated golden, through
    the plugin object the network constructs and through a standalone one."""
    from continuousbayesiannetwork_amd.inference import INFERENCE_OBJS, VariableElimination
    from golden_io import load_golden

    g = load_golden("chain5_d4_q1024_parent")
    m = g["meta"]
    bn = make_bn(BayesianNetwork, m["edges"], m["columns"], g["data"], device=gpu)
    ev = _t({k: g["evidence"][k] for k in m["evidence"]}, gpu)
    assert isinstance(bn.inference_obj, INFERENCE_OBJS["exact"])
    for ve in (VariableElimination({"inference_obj": "exact"}, bn=bn, device=gpu), bn.inference_obj):
        random.seed(m["seed"])
        pdf, dom = (ve.query(m["target"], ev, N_max=m["N_max"]) if hasattr(ve, "query")
                    else ve.infer(m["target"], ev, None, N_max=m["N_max"]))
        np.testing.assert_array_equal(dom.cpu().numpy(), g["domain"])
        np.testing.assert_allclose(pdf.cpu().numpy(), g["pdf"], rtol=RTOL, atol=ATOL)


def test_native_runner_path_matches_and_falls_back(gpu):
    """The native Runner (csrc/host_fast.cpp) serves repeat calls of the last
    (target, evidence keys, N): same outputs as the general path bit for bit;
    other key orders, extra keys, a float64 column, a CPU column, a missing
    key, evidence=None, out=, a timed call and a refit all take the general
    path with the reference's behaviour, and the runner comes back after."""
    data, cols, edges = chain_data(8, 8, 5000, 4, stay=0.7)
    bn = make_bn(BayesianNetwork, edges, cols, data, device=gpu)
    names = [c for c in cols if c != "X7"]
    ev = _t(sample_evidence(data, cols, names, 777, 2), gpu)
    eng = bn.engine
    a, da = bn.infer("X7", ev, N_max=8)  # plans + caches the fast path
    assert eng._runner is None
    a2, _ = bn.infer("X7", ev, N_max=8)  # cached fast path; sets the runner
    assert eng._runner is not None and eng._runner[:2] == ("X7", 8)
    np.testing.assert_array_equal(a.cpu().numpy(), a2.cpu().numpy())
    b, db = bn.infer("X7", dict(ev), N_max=8)  # runner path (a new dict, same keys)
    np.testing.assert_array_equal(a.cpu().numpy(), b.cpu().numpy())
    assert torch.equal(da, db) and db.shape == (777, 8)
    ref, _ = OracleBN(edges, cols, data).infer("X7", {k: v.cpu().numpy() for k, v in ev.items()}, 8)
    np.testing.assert_allclose(b.cpu().numpy(), ref, rtol=RTOL, atol=ATOL)
    # another key order: the general path (its own fast path), same values
    rev = {k: ev[k] for k in reversed(list(ev))}
    c, _ = bn.infer("X7", rev, N_max=8)
    np.testing.assert_array_equal(c.cpu().numpy(), a.cpu().numpy())
    # a float64 column / a CPU column: converted by the general path
    ev64 = dict(ev)
    ev64["X6"] = ev["X6"].double()
    np.testing.assert_array_equal(bn.infer("X7", ev64, N_max=8)[0].cpu().numpy(), a.cpu().numpy())
    evc = dict(ev)
    evc["X3"] = ev["X3"].cpu()
    np.testing.assert_allclose(bn.infer("X7", evc, N_max=8)[0].cpu().numpy(), ref, rtol=RTOL, atol=ATOL)
    # the reference's errors still raise
    with pytest.raises(AttributeError):
        bn.infer("X7", None, N_max=8)
    bad = dict(ev)
    bad["X6"] = ev["X6"][:5]
    with pytest.raises(AssertionError):
        bn.infer("X7", bad, N_max=8)
    # out= through the runner
    bn.infer("X7", ev, N_max=8)
    out = torch.empty((777, 8), device=gpu)
    r, _ = eng.infer("X7", dict(ev), 8, out=out)
    assert r.data_ptr() == out.data_ptr()
    np.testing.assert_array_equal(out.cpu().numpy(), a.cpu().numpy())
    # changing a per-call flag drops the runner
    eng.timed = True
    assert eng._runner is None
    np.testing.assert_array_equal(bn.infer("X7", ev, N_max=8)[0].cpu().numpy(), a.cpu().numpy())
    eng.timed = False
    eng.timing()
    bn.infer("X7", ev, N_max=8)  # cached fast path again: the runner is back
    assert eng._runner is not None
    # a refit drops it with the plans: the next call follows the new CPD
    from oracle.ref_infer import OracleNode

    data2, _, _ = chain_data(8, 8, 5000, 9, stay=0.3)
    y, x = data2[:, cols.index("X7")], data2[:, cols.index("X6")][None, :]
    bn.nodes_obj["X7"].fit(torch.tensor(y, device=gpu), torch.tensor(x, device=gpu))
    got, _ = bn.infer("X7", ev, N_max=8)
    ora = OracleBN(edges, cols, data)
    node = OracleNode("X7", ["X6"])
    node.fit(y, x)
    ora.nodes["X7"] = node
    ref2, _ = ora.infer("X7", {k: v.cpu().numpy() for k, v in ev.items()}, 8)
    np.testing.assert_allclose(got.cpu().numpy(), ref2, rtol=RTOL, atol=ATOL)
    got2, _ = bn.infer("X7", dict(ev), N_max=8)  # the rebuilt plan's runner
    np.testing.assert_array_equal(got2.cpu().numpy(), got.cpu().numpy())


def test_evidence_width_raises_like_the_reference(gpu):
    """An evidence column that is not [Q, 1] raises the reference's RuntimeError
    (node.py:233-234 copies a fully observed node's columns into [Q, 1] slots;
    :246-248 expands a partially observed node's to [Q, N]) on every path --
    the first (planning) call, a repeat call after valid ones (the native
    Runner declines it), infer_raw, sharded_infer and ShardedStepper.step,
    empty shards included -- instead of the kernels reading element q of a
    wider tensor as query q's value.  A strided [Q, 1] view (x[:, 1:2] of a
    [Q, 3] tensor) is still a valid column and matches the oracle."""
    import re

    from continuousbayesiannetwork_amd.distributed import ShardedStepper, sharded_infer

    data, cols, edges = chain_data(8, 8, 5000, 4, stay=0.7)
    bn = make_bn(BayesianNetwork, edges, cols, data, device=gpu)
    eng = bn.engine
    names = [c for c in cols if c != "X7"]
    ev = _t(sample_evidence(data, cols, names, 777, 2), gpu)
    msg = re.escape("The expanded size of the tensor (1) must match the existing size (2) at non-singleton "
                    "dimension 1.  Target sizes: [777, 1].  Tensor sizes: [777, 2]")
    wide = dict(ev)
    wide["X6"] = torch.cat([ev["X6"], ev["X5"]], 1).contiguous()
    with pytest.raises(RuntimeError, match=msg):  # first call: plans, then the general path
        bn.infer("X7", wide, N_max=8)
    a, _ = bn.infer("X7", ev, N_max=8)
    a2, _ = bn.infer("X7", ev, N_max=8)
    assert eng._runner is not None
    for _ in range(2):  # the runner path declines, the general path raises
        with pytest.raises(RuntimeError, match=msg):
            bn.infer("X7", dict(wide), N_max=8)
    first = dict(ev)
    first["X0"] = torch.cat([ev["X0"]] * 3, 1)
    with pytest.raises(RuntimeError, match=re.escape("existing size (3)")):
        bn.infer("X7", first, N_max=8)
    zero = dict(ev)
    zero["X3"] = ev["X3"][:, :0]
    with pytest.raises(RuntimeError, match=re.escape("existing size (0)")):
        bn.infer("X7", zero, N_max=8)
    # strided [Q, 1] views of [Q, 3] tensors are valid columns
    strided = {k: torch.cat([v + 100, v, v - 100], 1)[:, 1:2] for k, v in ev.items()}
    assert not strided["X6"].is_contiguous() and strided["X6"].shape == (777, 1)
    s1, _ = bn.infer("X7", strided, N_max=8)
    np.testing.assert_array_equal(s1.cpu().numpy(), a.cpu().numpy())
    ref, _ = OracleBN(edges, cols, data).infer("X7", {k: v.cpu().numpy() for k, v in ev.items()}, 8)
    np.testing.assert_allclose(s1.cpu().numpy(), ref, rtol=RTOL, atol=ATOL)
    # the raw launch and the sharded paths
    with pytest.raises(RuntimeError, match=msg):
        eng.infer_raw("X7", wide, 8)
    with pytest.raises(RuntimeError, match=msg):
        sharded_infer(bn, "X7", wide, 8)
    empty_wide = {k: v[:0] for k, v in wide.items()}
    with pytest.raises(RuntimeError, match=re.escape("existing size (2)")):
        sharded_infer(bn, "X7", empty_wide, 8)
    for fold in (False, True):
        st = ShardedStepper(bn, "X7", 8, exchange_every=2, fold=fold)
        r, _ = st.step(ev)
        with pytest.raises(RuntimeError, match=msg):
            st.step(wide)
        with pytest.raises(RuntimeError, match=re.escape("existing size (2)")):
            st.step(empty_wide)
        r2, _ = st.step(strided)
        st.wait()
        torch.cuda.synchronize()
        np.testing.assert_array_equal(r.cpu().numpy(), a.cpu().numpy())
        np.testing.assert_array_equal(r2.cpu().numpy(), a.cpu().numpy())
        st.close()
    np.testing.assert_array_equal(a2.cpu().numpy(), a.cpu().numpy())
    # the Node.get_prob mirror raises the same way (node.py:233-234)
    with pytest.raises(RuntimeError):
        bn.nodes_obj["X7"].get_prob({"X6": wide["X6"]}, 8)


def test_global_table_plan_with_many_factors_and_few_slots_takes_a_fast_kernel(gpu):
    """an N = 32 global-table plan (4 lanes per query) with ~100
    factors and few evidence slots -- the LDS budget for its small tables is
    sized against the larger of k_query_slots' and k_query_fast's side
    buffers, so the plan is not dropped to the generic k_query kernel.  A
    100-node chain d = 32 whose nodes X12, X22, X32 also have X10, X20, X30
    as parents (three 1 024-row tables: a 400 KB image, beyond LDS), evidence
    on 7 nodes; the marginals match the oracle."""
    rng = np.random.default_rng(17)
    S, d, n = 20000, 32, 100
    X = np.zeros((S, n), np.int64)
    X[:, 0] = rng.integers(0, d, S)
    for i in range(1, n):
        X[:, i] = (X[:, i - 1] + (rng.random(S) < 0.3) * rng.integers(0, d, S)) % d
        if i in (12, 22, 32):
            X[:, i] = (X[:, i - 1] + X[:, i - 2]) % d
    data = X.astype(np.float32)
    cols = [f"X{i}" for i in range(n)]
    edges = [(cols[i - 1], cols[i]) for i in range(1, n)] + [(cols[i - 2], cols[i]) for i in (12, 22, 32)]
    names = ["X10", "X11", "X20", "X21", "X30", "X31", "X98"]  # (X98: the target needs an observed parent)
    ev = sample_evidence(data, cols, names, 3000, 4)
    bn = make_bn(BayesianNetwork, edges, cols, data, device=gpu)
    pdf, _ = bn.infer("X99", {k: torch.tensor(v, device=gpu) for k, v in ev.items()}, N_max=32)
    fp = bn.engine._fast[("X99", tuple(ev.keys()), 32)]
    flags = _native.load().cbn_plan_flags(fp.plan.handle)
    assert flags & (_native.CBN_PLAN_FAST | _native.CBN_PLAN_SLOTS), flags
    assert not flags & _native.CBN_PLAN_LDS  # a global-table plan
    sub = np.arange(0, 3000, 97)
    random.seed(0)
    ref, _ = OracleBN(edges, cols, data).infer_raw("X99", {k: v[sub] for k, v in ev.items()}, 32)
    p = pdf.cpu().numpy()[sub]
    np.testing.assert_allclose(p / p.max(), ref / ref.max(), rtol=1e-5, atol=1e-7)
