"""The CPU oracle (oracle/ref_infer.py) against vectors produced by running the
reference itself (tests/golden/make_golden.py).  Tolerance: the oracle and the
reference sum the parent-axis means in different orders, so rtol 1e-5 (the
north-star fp32 bar) with atol 1e-7."""
import random

import numpy as np
import pytest

from golden_io import golden_error, golden_names, load_golden, load_param_golden, oracle_estimators, param_golden_names
from oracle.ref_infer import OracleBN

RTOL, ATOL = 1e-5, 1e-7


@pytest.mark.parametrize("name", golden_names())
def test_oracle_matches_reference_golden(name):
    g = load_golden(name)
    m = g["meta"]
    bn = OracleBN(m["edges"], m["columns"], g["data"])
    random.seed(m["seed"])
    ev = None if m["evidence_none"] else {k: g["evidence"][k] for k in m["evidence"]}
    if m["error"]:
        exc, msg = golden_error(m)
        with pytest.raises(exc) as info:
            if ev is None:
                ev.items()
            bn.infer(m["target"], ev, m["N_max"])
        if exc is RuntimeError:  # the evidence-width errors: the reference's message too
            assert str(info.value) == msg
        return
    pdf, dom = bn.infer(m["target"], ev, m["N_max"])
    assert pdf.shape == g["pdf"].shape
    np.testing.assert_array_equal(dom, g["domain"])
    np.testing.assert_allclose(pdf, g["pdf"], rtol=RTOL, atol=ATOL)


def test_golden_manifest_covers_config0():
    """BASELINE configs[0]: 5-node chain, d=4, 1024 queries on the reference CPU path."""
    g = load_golden("chain5_d4_q1024_parent")
    assert g["pdf"].shape == (1024, 4)
    assert len(g["meta"]["columns"]) == 5


@pytest.mark.parametrize("name", param_golden_names())
def test_oracle_parametric_matches_reference_golden(name):
    """LinearRegression / LogisticRegression / NeuralNetwork networks: the
    oracle, given the reference's fitted parameters, reproduces the reference's
    infer output (NaN where the reference's logistic density overflows)."""
    g = load_param_golden(name)
    m = g["meta"]
    bn = OracleBN(m["edges"], m["columns"], g["data"], estimators=oracle_estimators(g))
    random.seed(m["seed"])
    ev = {k: g["evidence"][k] for k in m["evidence"]}
    pdf, dom = bn.infer(m["target"], ev, m["N_max"])
    assert pdf.shape == g["pdf"].shape
    np.testing.assert_array_equal(dom, g["domain"])
    np.testing.assert_allclose(pdf, g["pdf"], rtol=RTOL, atol=ATOL)


def _full(name):
    import json
    import os

    z = np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", name + ".npz"), allow_pickle=False)
    return z["rows"], z["pdf"], z["domain"], json.loads(str(z["meta"]))


@pytest.mark.parametrize("name,gen", [("chain20_d32_bench65536", "chain"), ("alarm37_d8_bench262144", "alarm")])
def test_oracle_matches_full_batch_golden(name, gen):
    """The full-batch reference goldens (tests/golden/make_golden_full.py): the
    oracle on a few rows plus the batch argmax row (so it normalises by the same
    max as the reference's whole-batch call) reproduces those rows."""
    from helpers import alarm_like_data, chain_data, sample_evidence

    rows, ref, rdom, m = _full(name)
    if gen == "chain":
        data, cols, edges = chain_data(20, 32, 200_000, 3, stay=0.8)
    else:
        data, cols, edges = alarm_like_data(200_000, 5)
    ev = sample_evidence(data, cols, [c for c in cols if c != m["target"]], m["Q"], m["ev_seed"])
    pick = np.array([0, 1, 2, 3, 5, 8, 13, 21, int(np.searchsorted(rows, m["argmax_row"]))])
    sub = rows[pick]
    bn = OracleBN(edges, cols, data)
    pdf, dom = bn.infer(m["target"], {k: v[sub] for k, v in ev.items()}, m["N_max"])
    assert (rdom == rdom[:1]).all()  # one sample domain per query row
    np.testing.assert_array_equal(dom, np.broadcast_to(rdom[:1], dom.shape))
    assert pdf[-1].max() == 1.0
    np.testing.assert_allclose(pdf, ref[pick], rtol=RTOL, atol=ATOL)


def test_grid_oracle_fixture_matches_reference_run():
    """BASELINE configs[4]'s plan (10 x 10 grid, d = N = 64, 100 factors): the
    oracle fixture (tests/golden/make_grid_oracle.py, 64 queries) against the
    reference's own infer on the same 64 queries (make_golden_full.py
    grid10_d64_peaked_ref64), at the north-star tolerance; same domain."""
    import os

    rows, ref, rdom, m = _full("grid10_d64_peaked_ref64")
    assert m["Q"] == 64 and list(rows) == list(range(64)) and m["N_max"] == 64
    z = np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "grid10_d64_peaked_oracle.npz"))
    assert (rdom == rdom[:1]).all() and (z["domain"] == rdom[:1]).all()
    assert np.isfinite(ref).all() and ref.max() == 1.0
    np.testing.assert_allclose(z["pdf"], ref, rtol=RTOL, atol=ATOL)


def test_free_parent_grid_fixtures_regenerate_their_inputs():
    """The free-parent grid fixtures' data and evidence come back bit for bit
    from the committed generators (tests/helpers.py grid_rows_data /
    grid_rows_evidence / grid_data), so the GPU tests rebuild exactly the
    reference's inputs; their outputs are finite and non-degenerate."""
    import json
    import os
    import sys

    here = os.path.dirname(os.path.abspath(__file__))
    sys.path.insert(0, os.path.join(here, "golden"))
    from make_golden_full import CASES, digest, make_case

    for name in ("grid10_d64_dense_ref", "grid10_d64_rows_ref", "grid10_d64_rows_x99_ref"):
        z = np.load(os.path.join(here, "golden", name + ".npz"))
        meta = json.loads(str(z["meta"]))
        data, cols, edges, ev = make_case(CASES[name])
        assert digest([data]) == meta["data_sha256"], name
        assert digest([ev[k] for k in sorted(ev)]) == meta["evidence_sha256"], name
        assert sorted(ev) == meta["evidence_columns"]
        assert all((int(k[1:]) // 10) % 2 == 0 for k in ev)  # even grid rows only
        pdf = z["pdf"]
        assert np.isfinite(pdf).all() and pdf.max() == 1.0
        if name == "grid10_d64_dense_ref":
            assert (pdf > 0).mean() >= 0.2
