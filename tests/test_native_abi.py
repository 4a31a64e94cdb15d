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
    assert lib.cbn_abi_version() == 2 == _native.ABI_VERSION
    # cbn_factor_desc: 3 int32 + 2*8 int32 + 3 pointers + 8 pointers (with alignment padding)
    assert ctypes.sizeof(_native.FactorDesc) == 4 * 19 + 4 + 8 * 11
    # cbn_param_model: 8 int32 (family, n_layers, width[5], act) + pointer + 2 float
    assert ctypes.sizeof(_native.ParamModel) == 4 * 8 + 8 + 8
    # cbn_param_factor: kind + 8 slots (+4 pad) + 2 pointers + model
    assert ctypes.sizeof(_native.ParamFactor) == 4 * 9 + 4 + 16 + ctypes.sizeof(_native.ParamModel)


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
    m.width[0], m.width[1], m.width[2], m.width[3] = 2, 64, 8, 1  # hidden width above CBN_MAX_WIDTH
    m.act, m.weights, m.scale = 1, 16, 1.0
    assert lib.cbn_param_eval(ctypes.byref(m), None, 0, 0, None, 0, None, None) == -3
    m.width[1] = 8
    m.scale = -1.0
    assert lib.cbn_param_eval(ctypes.byref(m), None, 0, 0, None, 0, None, None) == -1
    m.scale = 1.0
    assert lib.cbn_param_eval(ctypes.byref(m), None, 0, 0, None, 0, None, None) == 0  # empty: no launch
