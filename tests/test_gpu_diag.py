"""Diagnostic kernel-selection switches stay out of the serving path
(VERDICT r04 weak 7): they count only when libcbn_amd.so is loaded with
CBN_DIAG=1.  Each case runs tests/diag_child.py in a child process started
with the environment under test (one child at a time)."""
import json
import os
import subprocess
import sys

import pytest

from continuousbayesiannetwork_amd import _native

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


def _child(mode: str, **env):
    e = {k: v for k, v in os.environ.items() if not k.startswith("CBN_")}
    e.update(env)
    p = subprocess.run([sys.executable, os.path.join(HERE, "diag_child.py"), mode], env=e, capture_output=True,
                       text=True, timeout=240)
    assert p.returncode == 0, p.stderr[-2000:]
    return json.loads(p.stdout.strip().splitlines()[-1]), p.stderr


def test_no_staged_ignored_without_cbn_diag(gpu):
    """CBN_NO_STAGED=1 alone leaves the configs[1] plan on k_query_staged;
    with CBN_DIAG=1 it takes effect and the override is listed on stderr."""
    base, _ = _child("flags")
    stray, err = _child("flags", CBN_NO_STAGED="1")
    assert stray["diag"] == 0 and "diagnostic override" not in err
    assert stray["flags"] == base["flags"] and all(f & _native.CBN_PLAN_STAGED for f in base["flags"])
    diag, err = _child("flags", CBN_DIAG="1", CBN_NO_STAGED="1")
    assert diag["diag"] == 1 and "diagnostic override CBN_NO_STAGED=1" in err
    assert not any(f & _native.CBN_PLAN_STAGED for f in diag["flags"])


def test_generic_kernel_equals_fast_kernel(gpu):
    """The generic parametric kernel (CBN_PARAM_GENERIC, under CBN_DIAG=1)
    runs the fast kernels' operations in the same order: bit-identical rows
    on an NN [16] network with free parents (moved here from
    test_gpu_param.py: the switch is read at plan creation, the gate at load)."""
    res, _ = _child("generic", CBN_DIAG="1")
    assert res["diag"] == 1 and res["equal"] and res["finite"] > 0


def test_grid_bench_batch_slots_equals_fast_kernel(gpu):
    """configs[4] at its benchmarked size (tools/bench_grid.py's headline
    batch: 100 factors, L = 8, 65 536 queries -- k_query_slots' fused
    two-round launch with a 3-chunk phase-B survivor chain) == k_query_fast
    (CBN_NO_SLOTS=1 under CBN_DIAG=1) bit for bit."""
    res, _ = _child("gridfull", CBN_DIAG="1")
    assert res["diag"] == 1 and res["equal"] and res["nonzero_rows"] > 1000
    assert res["flags"][0] & _native.CBN_PLAN_SLOTS and not res["flags"][1] & _native.CBN_PLAN_SLOTS


def test_grid_coalesced_index_phase_equals_per_lane(gpu, tmp_path):
    """k_query_slots' coalesced index phase (round 6: 16-B evidence loads per
    (slot, 4 queries), taken by launches of >= 3 block rounds) == the per-lane
    index phase (CBN_SLOTS_NO_COAL=1 under CBN_DIAG=1) bit for bit on a
    200 003-query grid batch (the raw launch + scale path, ragged last
    round), and == the same batch through 4-B-offset column views (the
    coalesced phase declines unaligned columns); 42 rows vs the oracle."""
    import random

    import numpy as np

    from helpers import grid_data, sample_evidence
    from oracle.ref_infer import OracleBN

    outp = str(tmp_path / "rows.npy")
    res, _ = _child("gridcoal", CBN_DIAG="1", CBN_CHILD_OUT=outp)
    assert res["diag"] == 1 and res["equal"] and res["equal_unaligned"] and res["nonzero_rows"] > 1000
    assert all(f & _native.CBN_PLAN_SLOTS for f in res["flags"])
    data, cols, edges = grid_data(100000, 7, side=5, d=64, keep=0.995, noise=0)
    target, names = cols[-1], cols[:-1]
    ev = sample_evidence(data, cols, names, 200003, 3)
    rows = np.asarray(res["rows"])
    random.seed(0)
    ref, _ = OracleBN(edges, cols, data).infer(target, {k: v[rows] for k, v in ev.items()}, 64)
    got = np.load(outp)
    np.testing.assert_allclose(got / got.max(), ref, rtol=1e-5, atol=1e-7)
