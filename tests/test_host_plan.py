"""Host logic of the engine, without a GPU: factor kinds, observed slots and the
reference's random-draw order for sample domains (node.py:286-333)."""
import random

import numpy as np
import pytest
import torch

from continuousbayesiannetwork_amd import BayesianNetwork
from continuousbayesiannetwork_amd._native import CBN_FACTOR_QUERY, CBN_FACTOR_SCALAR, CBN_FACTOR_SHARED
from continuousbayesiannetwork_amd.inference.engine import InferenceEngine, Plan, build_factor_specs, relevant_observed
from golden_io import golden_error, golden_names, load_golden
from helpers import make_bn
from oracle.ref_infer import OracleBN


def _ok_cases():
    return [n for n in golden_names() if not load_golden(n)["meta"]["error"]]


@pytest.mark.parametrize("name", _ok_cases())
def test_plan_consumes_random_like_reference(name):
    g = load_golden(name)
    m = g["meta"]
    ev = {k: g["evidence"][k] for k in m["evidence"]}
    ora = OracleBN(m["edges"], m["columns"], g["data"])
    random.seed(m["seed"])
    ora.infer(m["target"], ev, m["N_max"])
    after_oracle = random.random()

    bn = make_bn(BayesianNetwork, m["edges"], m["columns"], g["data"], device="cpu")
    order = bn.get_ancestors(bn.initial_dag, m["target"]) + [m["target"]]
    obs = relevant_observed(bn, order, ev.keys())
    random.seed(m["seed"])
    order2, specs, tdom, det = build_factor_specs(bn, m["target"], obs, m["N_max"])
    after_engine = random.random()
    assert order2 == order
    assert after_engine == after_oracle
    np.testing.assert_array_equal(tdom.numpy(), g["domain"][0])


def test_factor_kinds_chain_all_evidence():
    g = load_golden("chain5_d4_all_evidence")
    m = g["meta"]
    bn = make_bn(BayesianNetwork, m["edges"], m["columns"], g["data"], device="cpu")
    obs = frozenset(m["evidence"])
    _, specs, _, det = build_factor_specs(bn, "X4", obs, 4)
    assert det
    assert [s.kind for s in specs] == [CBN_FACTOR_SCALAR] + [CBN_FACTOR_QUERY] * 4
    assert [s.observed for s in specs[1:]] == [["X0"], ["X1"], ["X2"], ["X3"]]


def test_factor_kinds_no_evidence_and_partial():
    g = load_golden("multi_partial")
    m = g["meta"]
    bn = make_bn(BayesianNetwork, m["edges"], m["columns"], g["data"], device="cpu")
    _, specs, _, _ = build_factor_specs(bn, "E", frozenset(), 3)
    kinds = {s.node: s.kind for s in specs}
    assert kinds["A"] == CBN_FACTOR_SCALAR and kinds["E"] == CBN_FACTOR_SHARED
    _, specs, _, _ = build_factor_specs(bn, "E", frozenset({"C", "A"}), 3)
    e = [s for s in specs if s.node == "E"][0]
    assert e.kind == CBN_FACTOR_QUERY and e.observed == ["C"] and list(e.free_samples) == ["D"]


def test_cpu_device_fails_loudly():
    g = load_golden("chain5_d4_q1024_parent")
    m = g["meta"]
    bn = make_bn(BayesianNetwork, m["edges"], m["columns"], g["data"], device="cpu")
    with pytest.raises(RuntimeError, match="HIP device"):
        bn.infer("X4", {"X3": torch.tensor(g["evidence"]["X3"])}, N_max=4)


def test_host_sample_points_match_sample_domain():
    """Node._sample_points (host points of a redrawn domain, engine-internal)
    consumes ``random`` exactly like sample_domain and gives the same points;
    domain_index_host == domain_index."""
    from continuousbayesiannetwork_amd.inference.engine import domain_index, domain_index_host
    from helpers import chain_data

    data, cols, edges = chain_data(4, 3, 500, 5)
    bn = make_bn(BayesianNetwork, edges, cols, data, device="cpu")
    nd = bn.nodes_obj["X2"]
    for N in (2, 3, 7, 16):
        random.seed(11)
        a = nd.sample_domain("X2", N)
        ra = random.random()
        random.seed(11)
        b, on_host = nd._sample_points("X2", N)
        rb = random.random()
        assert on_host == (N > 3)
        assert ra == rb
        assert torch.equal(a.cpu(), b.cpu())
        dom = nd.info["X2"][3]
        assert torch.equal(domain_index(b, dom).cpu(), domain_index_host(b.cpu(), dom.cpu()))


def _redraw_case(edges, cols, data, target, observed, N, seeds):
    """host_fast.redraw (RedrawProgram jobs, one native call) == the index
    arrays of build_factor_specs' points under the same seed, same random
    consumption, same target domain."""
    from continuousbayesiannetwork_amd import _native
    from continuousbayesiannetwork_amd.base.node import uniforms
    from continuousbayesiannetwork_amd.inference.engine import InferenceEngine, Plan, RedrawProgram

    bn = make_bn(BayesianNetwork, edges, cols, data, device="cpu")
    eng = bn.engine
    obs = frozenset(observed)

    def walk_plan():
        order, specs, tdom, det = build_factor_specs(bn, target, obs, N)
        p = Plan(target, N, order, specs, [], tdom, False, det)
        InferenceEngine._alloc_index_arrays(p, torch.device("cpu"))
        for f in range(len(specs)):
            eng._index_arrays(p, f, bn.nodes_obj[specs[f].node].estimator.domains, 0)
        return p

    random.seed(1)
    p = walk_plan()
    assert not p.deterministic
    prog = RedrawProgram(bn, p, obs)
    idx = p.idx_flat.clone()
    for s in seeds:
        random.seed(s)
        want = walk_plan()
        r_after_walk = random.random()
        random.seed(s)
        _native.load_host().redraw(uniforms(prog.total), prog.meta, prog.lospan, prog.doms, idx, prog.pts, N)
        assert random.random() == r_after_walk
        assert torch.equal(idx, want.idx_flat)
        if prog.target_pts:
            assert torch.equal(prog.pts, want.target_domain.cpu())


def test_redraw_program_binary_network():
    """Binary variables at N_max = 16: every domain padded by 14 draws
    (node.py:302-333), free and observed parents, the target's own points."""
    from helpers import random_dag_data

    data, cols, edges = random_dag_data(7, 2, 3, 400, 5)
    target = cols[-1]
    _redraw_case(edges, cols, data, target, cols[:2], 16, seeds=(3, 4, 99))
    _redraw_case(edges, cols, data, target, [], 16, seeds=(7,))


def test_redraw_program_mixed_cards():
    """Mixed domain sizes: some sample_domain calls deterministic (N <=
    |domain|: no draws, fixed indices), some redrawn."""
    from helpers import chain_data

    data, cols, edges = chain_data(6, 5, 800, 3, values=[0.0, 0.25, 0.5, 0.75, 1.0])
    data[:, 2] = np.round(data[:, 2] * 4) % 2  # a binary column among 5-level ones
    for N in (3, 5, 8):
        _redraw_case(edges, cols, data, "X5", ["X1", "X3"], N, seeds=(1, 2))


@pytest.mark.parametrize("name", [n for n in golden_names() if load_golden(n)["meta"].get("width")])
def test_evidence_width_checks_match_reference(name):
    """Evidence columns that are not [Q, 1] (reference fixtures
    err_width*, multi_widthN_partial): InferenceEngine.check_columns raises the
    reference's RuntimeError with its message (node.py:233-234, 246-248) --
    or returns the [Q, N] columns the reference reads as N per-sample values
    (the wide direct plan's columns).  Host logic only: the plan's factor
    specs, no launch."""
    g = load_golden(name)
    m = g["meta"]
    bn = make_bn(BayesianNetwork, m["edges"], m["columns"], g["data"], device="cpu")
    ev = {k: torch.tensor(g["evidence"][k]) for k in m["evidence"]}
    order = bn.get_ancestors(bn.initial_dag, m["target"]) + [m["target"]]
    obs = relevant_observed(bn, order, ev.keys())
    random.seed(m["seed"])
    order, specs, tdom, det = build_factor_specs(bn, m["target"], obs, m["N_max"])
    plan = Plan(m["target"], m["N_max"], order, specs, sorted(obs), tdom, True, det)
    if m["error"]:
        exc, msg = golden_error(m)
        with pytest.raises(exc) as info:
            InferenceEngine.check_columns(plan, ev)
        assert str(info.value) == msg
    else:
        assert InferenceEngine.check_columns(plan, ev) == {k for k, v in m["width"].items() if v != 1}
    # the same columns at width 1 pass
    assert InferenceEngine.check_columns(plan, {k: v[:, :1] if v.shape[1] else torch.zeros((v.shape[0], 1))
                                                for k, v in ev.items()}) == set()
