"""The C ABI library loads and exports every entry point include/cbn_amd.h declares
(no compute: runs without a GPU)."""
import ctypes
import os
import re

from continuousbayesiannetwork_amd import _native

HEADER = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "include", "cbn_amd.h")


def declared_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(cbn_[a-z0-9_]+)\s*\(", src)))


def test_library_exports_every_declared_symbol():
    lib = _native.load()
    names = declared_functions()
    assert len(names) >= 10
    for n in names:
        assert hasattr(lib, n), n
    assert set(names) == set(_native.EXPORTED_SYMBOLS)


def test_abi_version_and_struct_layout():
    lib = _native.load()
    assert lib.cbn_abi_version() == 5 == _native.ABI_VERSION
    # cbn_factor_desc: 3 int32 + 2*8 int32 + 3 pointers + 8 pointers (with alignment padding)
    assert ctypes.sizeof(_native.FactorDesc) == 4 * 19 + 4 + 8 * 11
    # cbn_param_model: 8 int32 (family, n_layers, width[5], act) + pointer + 2 float + widths pointer
    assert ctypes.sizeof(_native.ParamModel) == 4 * 8 + 8 + 8 + 8
    # cbn_param_factor: kind + 8 slots (+4 pad) + 2 pointers + model + input_slots pointer
    assert ctypes.sizeof(_native.ParamFactor) == 4 * 9 + 4 + 16 + ctypes.sizeof(_native.ParamModel) + 8
    # cbn_cpd_ref: n_cols (+4 pad) + 5 pointers + int64
    assert ctypes.sizeof(_native.CpdRef) == 8 + 5 * 8 + 8
    # cbn_direct_factor: 2 int32 + 3 pointers + cpd
    assert ctypes.sizeof(_native.DirectFactor) == 8 + 3 * 8 + ctypes.sizeof(_native.CpdRef) + 8


def test_argument_errors_are_reported_without_gpu():
    lib = _native.load()
    h = ctypes.c_void_p()
    rc = lib.cbn_plan_create(None, 0, 4, ctypes.byref(h))
    assert rc == -1
    assert b"bad arguments" in lib.cbn_last_error()


def test_host_fast_path_module_rejects_non_device_evidence():
    """The native host fast path loads and hands anything it cannot pass to the
    C ABI as-is (here: CPU tensors) back to the Python slow path (None), without
    touching the function pointer it was given."""
    import torch

    run = _native.load_host().run
    ev = {"a": torch.zeros(8, 1), "b": torch.zeros(8, 1)}
    assert run(0, 0, ev, ("a", "b"), "a", 0, 4, True, 0, 0, None) is None
    assert run(0, 0, ev, ("a", "missing"), "a", 0, 4, True, 0, 0, None) is None
    assert run(0, 0, {"a": torch.zeros(0, 1)}, ("a",), "a", 0, 4, True, 0, 0, None) is None


def test_param_argument_errors_are_reported_without_gpu():
    """cbn_plan_create_param / cbn_param_eval validate their descriptors before
    touching the device."""
    lib = _native.load()
    h = ctypes.c_void_p()
    assert lib.cbn_plan_create_param(None, 0, 4, ctypes.byref(h)) == -1
    f = (_native.ParamFactor * 1)()
    f[0].kind = 2
    f[0].model.family = 7  # no such family
    assert lib.cbn_plan_create_param(f, 1, 4, ctypes.byref(h)) == -1
    assert b"bad family" in lib.cbn_last_error()
    m = _native.ParamModel()
    m.family, m.n_layers = 1, 3
    m.width[0], m.width[1], m.width[2], m.width[3] = 2, 300, 8, 1  # hidden width above CBN_MAX_MODEL_WIDTH
    m.act, m.weights, m.scale = 1, 16, 1.0
    assert lib.cbn_param_eval(ctypes.byref(m), None, 0, 0, None, 0, None, None) == -3
    m.n_layers = 6  # deeper than width[] without the widths array
    assert lib.cbn_param_eval(ctypes.byref(m), None, 0, 0, None, 0, None, None) == -1
    widths = (ctypes.c_int32 * 7)(2, 64, 64, 64, 64, 64, 1)
    m.widths = ctypes.cast(widths, ctypes.POINTER(ctypes.c_int32))
    assert lib.cbn_param_eval(ctypes.byref(m), None, 0, 0, None, 0, None, None) == 0  # generic: empty, no launch
    m.widths = None
    m.n_layers = 3
    m.width[1] = 8
    m.scale = -1.0
    assert lib.cbn_param_eval(ctypes.byref(m), None, 0, 0, None, 0, None, None) == -1
    m.scale = 1.0
    assert lib.cbn_param_eval(ctypes.byref(m), None, 0, 0, None, 0, None, None) == 0  # empty: no launch


def test_direct_argument_errors_are_reported_without_gpu():
    """cbn_plan_create_direct / cbn_hash_build / cbn_cpd_ref_eval validate
    their arguments before touching the device."""
    lib = _native.load()
    h = ctypes.c_void_p()
    assert lib.cbn_plan_create_direct(None, 0, 4, ctypes.byref(h)) == -1
    f = (_native.DirectFactor * 1)()
    f[0].kind = 9
    assert lib.cbn_plan_create_direct(f, 1, 4, ctypes.byref(h)) == -1
    assert b"bad kind" in lib.cbn_last_error()
    f[0].kind, f[0].n_parents = 2, 33  # above CBN_MAX_DIRECT_PARENTS
    assert lib.cbn_plan_create_direct(f, 1, 4, ctypes.byref(h)) == -3
    f[0].n_parents = 1
    f[0].node_sample_idx = 16
    f[0].cpd.n_cols = 3  # parents + node = 2
    assert lib.cbn_plan_create_direct(f, 1, 4, ctypes.byref(h)) == -1
    assert b"columns" in lib.cbn_last_error()
    # capacity not a power of two / below 2n
    assert lib.cbn_hash_build(None, None, 0, 16, 16, 12, None) == -1
    assert lib.cbn_hash_build(16, 16, 5, 16, 16, 8, None) == -1
    doms = (ctypes.c_void_p * 2)(16, 16)
    cards = (ctypes.c_int32 * 2)(3, 0)
    r = _native.CpdRef()
    r.n_cols, r.dense = 2, 16
    r.domains = ctypes.cast(doms, ctypes.POINTER(ctypes.c_void_p))
    r.cards = ctypes.cast(cards, ctypes.POINTER(ctypes.c_int32))
    assert lib.cbn_cpd_ref_eval(ctypes.byref(r), None, 0, None, None) == -1  # card 0
    cards[1] = 4
    assert lib.cbn_cpd_ref_eval(ctypes.byref(r), None, 0, None, None) == 0  # empty: no launch
    r.dense, r.keys, r.vals, r.capacity = None, 16, 16, 6  # hashed, capacity not a power of two
    assert lib.cbn_cpd_ref_eval(ctypes.byref(r), None, 0, None, None) == -1


def test_sparse_conditionals_match_oracle_rows():
    """The hashed CPD's values (host logic, CPU tensors) equal the oracle's
    BruteForce conditional at every unique training row."""
    import numpy as np
    import torch

    from continuousbayesiannetwork_amd.parameter_learning.brute_force import hash_capacity, sparse_conditionals
    from oracle.ref_infer import OracleBruteForce

    rng = np.random.default_rng(0)
    pd_ = np.round(rng.normal(0, 1, (2, 3000)), 1).astype(np.float32)
    nd_ = (np.round(pd_.sum(0)) % 4).astype(np.float32)
    ob = OracleBruteForce()
    ob.fit(nd_, pd_)
    rows, probs = ob.mle[:, :-1], ob.mle[:, -1]
    doms = [np.unique(rows[:, c]) for c in range(3)]
    cell = np.zeros(rows.shape[0], np.int64)
    stride = 1
    for c in (2, 1, 0):
        cell += np.searchsorted(doms[c], rows[:, c]) * stride
        stride *= len(doms[c])
    vals = sparse_conditionals(torch.tensor(cell), torch.tensor(probs), len(doms[2]), True).numpy()
    ref = ob.get_prob(rows[:, 2:3], rows[:, :2, None])[:, 0]
    np.testing.assert_allclose(vals, ref, rtol=1e-6, atol=0)
    assert len(np.unique(cell)) == len(cell)
    assert hash_capacity(len(cell)) >= 2 * len(cell) and hash_capacity(1) == 2 and hash_capacity(5) == 16


def test_diagnostic_switches_need_cbn_diag():
    """Kernel-selection switches (CBN_NO_STAGED, CBN_PARAM_GENERIC, ...) count
    only when the library is loaded with CBN_DIAG=1 (cbn_diag_enabled), which
    then lists every CBN_* override on stderr; a stray CBN_NO_STAGED=1 alone is
    ignored (the GPU side, tests/test_gpu_diag.py, checks the plan flags)."""
    import json
    import subprocess
    import sys

    child = os.path.join(os.path.dirname(os.path.abspath(__file__)), "diag_child.py")
    base = {k: v for k, v in os.environ.items() if not k.startswith("CBN_")}

    def run(**env):
        p = subprocess.run([sys.executable, child, "enabled"], env={**base, **env}, capture_output=True, text=True,
                           timeout=120)
        assert p.returncode == 0, p.stderr[-2000:]
        return json.loads(p.stdout.strip().splitlines()[-1])["diag"], p.stderr

    d, err = run(CBN_NO_STAGED="1")
    assert d == 0 and "diagnostic override" not in err
    d, err = run(CBN_DIAG="1", CBN_NO_STAGED="1", CBN_FAST_VPL="1")
    assert d == 1
    assert "diagnostic override CBN_NO_STAGED=1" in err and "diagnostic override CBN_FAST_VPL=1" in err
    d, _ = run(CBN_DIAG="0", CBN_NO_STAGED="1")
    assert d == 0


def test_runner_key_whose_eq_raises_falls_back():
    """A dict key whose __eq__ raises: the Runner's key walk
    clears the error and declines the call (None) instead of leaving a Python
    exception set behind its return value."""
    import torch

    class Key(str):
        def __eq__(self, other):
            raise ValueError("no comparison")

        __hash__ = str.__hash__

    host = _native.load_host()
    tdom = torch.zeros(4)
    r = host.Runner(0, 0, ("a",), ("a",), 0, 4, True, 0, 0, tdom)
    assert r({Key("b"): torch.zeros(8, 1)}, None) is None
    assert r({"a": torch.zeros(8, 1)}, None) is None  # a CPU column: declined too


def test_lib_path_override_needs_cbn_diag(monkeypatch):
    """CBN_LIB_PATH names a diagnostic (unstamped) library build; like the
    kernel switches it counts only under CBN_DIAG=1 -- a stray variable in a
    serving process still loads the in-tree, stamp-checked libcbn_amd.so."""
    default = os.path.join(os.path.dirname(os.path.abspath(_native.__file__)), "libcbn_amd.so")
    monkeypatch.delenv("CBN_DIAG", raising=False)
    monkeypatch.setenv("CBN_LIB_PATH", "/tmp/libcbn_amd_stamps.so")
    assert _native.lib_path() == default
    monkeypatch.setenv("CBN_DIAG", "0")
    assert _native.lib_path() == default
    monkeypatch.setenv("CBN_DIAG", "1")
    assert _native.lib_path() == "/tmp/libcbn_amd_stamps.so"
    monkeypatch.delenv("CBN_LIB_PATH")
    assert _native.lib_path() == default
    assert _native.LIB_PATH == default  # this process: no override
