"""Host logic of the engine, without a GPU: factor kinds, observed slots and the
reference's random-draw order for sample domains (node.py:286-333)."""
import random

import numpy as np
import pytest
import torch

from continuousbayesiannetwork_amd import BayesianNetwork
from continuousbayesiannetwork_amd._native import CBN_FACTOR_QUERY, CBN_FACTOR_SCALAR, CBN_FACTOR_SHARED
from continuousbayesiannetwork_amd.inference.engine import build_factor_specs, relevant_observed
from golden_io import golden_names, load_golden
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
