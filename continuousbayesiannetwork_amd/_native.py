"""ctypes binding of libcbn_amd.so (the C ABI declared in include/cbn_amd.h).

The library is loaded AFTER ``import torch`` so that its ``libamdhip64.so.7``
dependency resolves to the HIP runtime torch already mapped (same SONAME):
device pointers from torch's allocator and torch's streams are then valid
inside the library.  There is no CPU fallback: if the library or a GPU is
missing every product entry point raises.
"""
from __future__ import annotations

import ctypes
import os

import torch  # noqa: F401  (must be imported before the HIP library)

from . import _buildstamp

_HERE = os.path.dirname(os.path.abspath(__file__))
_DEFAULT_LIB = os.path.join(_HERE, "libcbn_amd.so")


def lib_path() -> str:
    """The library to load: the in-tree, stamped build -- or, only under
    ``CBN_DIAG=1`` (the same gate as the kernel switches, include/cbn_amd.h
    cbn_diag_enabled), a diagnostic variant named by ``CBN_LIB_PATH``.  A
    stray ``CBN_LIB_PATH`` alone never loads an unstamped library into a
    serving process."""
    alt = os.environ.get("CBN_LIB_PATH")
    if alt and os.environ.get("CBN_DIAG") == "1":
        return alt
    return _DEFAULT_LIB


LIB_PATH = lib_path()

ABI_VERSION = 5
CBN_MAX_PARENTS = 8
CBN_MAX_DIRECT_PARENTS = 32
CBN_MAX_EVIDENCE = 256
CBN_FACTOR_SCALAR = 0
CBN_FACTOR_SHARED = 1
CBN_FACTOR_QUERY = 2

CBN_MAX_LAYERS = 4
CBN_MAX_WIDTH = 32
CBN_MAX_MODEL_LAYERS = 64
CBN_MAX_MODEL_WIDTH = 256
CBN_FAMILY_GAUSS = 1
CBN_FAMILY_LOGISTIC = 2
CBN_ACT = {"tanh": 1, "relu": 2, "sigmoid": 3, "leakyrelu": 4, "gelu": 5, "elu": 6}
CBN_INPUT_FREE = -1
CBN_INPUT_ONE = -2

_c_float_p = ctypes.POINTER(ctypes.c_float)
_c_int_p = ctypes.POINTER(ctypes.c_int32)


class FactorDesc(ctypes.Structure):
    """Mirror of ``cbn_factor_desc`` (include/cbn_amd.h)."""

    _fields_ = [
        ("kind", ctypes.c_int32),
        ("n_parents", ctypes.c_int32),
        ("node_card", ctypes.c_int32),
        ("parent_card", ctypes.c_int32 * CBN_MAX_PARENTS),
        ("parent_ev_slot", ctypes.c_int32 * CBN_MAX_PARENTS),
        ("cpd", ctypes.c_void_p),
        ("node_sample_idx", ctypes.c_void_p),
        ("parent_sample_idx", ctypes.c_void_p),
        ("parent_domain", ctypes.c_void_p * CBN_MAX_PARENTS),
    ]


class ParamModel(ctypes.Structure):
    """Mirror of ``cbn_param_model`` (include/cbn_amd.h)."""

    _fields_ = [
        ("family", ctypes.c_int32),
        ("n_layers", ctypes.c_int32),
        ("width", ctypes.c_int32 * (CBN_MAX_LAYERS + 1)),
        ("act", ctypes.c_int32),
        ("weights", ctypes.c_void_p),
        ("scale", ctypes.c_float),
        ("norm", ctypes.c_float),
        ("widths", _c_int_p),
    ]


class ParamFactor(ctypes.Structure):
    """Mirror of ``cbn_param_factor`` (include/cbn_amd.h)."""

    _fields_ = [
        ("kind", ctypes.c_int32),
        ("input_slot", ctypes.c_int32 * CBN_MAX_PARENTS),
        ("input_samples", ctypes.c_void_p),
        ("node_samples", ctypes.c_void_p),
        ("model", ParamModel),
        ("input_slots", _c_int_p),
    ]


class CpdRef(ctypes.Structure):
    """Mirror of ``cbn_cpd_ref`` (include/cbn_amd.h)."""

    _fields_ = [
        ("n_cols", ctypes.c_int32),
        ("domains", ctypes.POINTER(ctypes.c_void_p)),
        ("cards", _c_int_p),
        ("dense", ctypes.c_void_p),
        ("keys", ctypes.c_void_p),
        ("vals", ctypes.c_void_p),
        ("capacity", ctypes.c_int64),
    ]


class DirectFactor(ctypes.Structure):
    """Mirror of ``cbn_direct_factor`` (include/cbn_amd.h)."""

    _fields_ = [
        ("kind", ctypes.c_int32),
        ("n_parents", ctypes.c_int32),
        ("parent_ev_slot", _c_int_p),
        ("node_sample_idx", ctypes.c_void_p),
        ("parent_sample_idx", ctypes.c_void_p),
        ("cpd", CpdRef),
        ("parent_ev_width", _c_int_p),  # ABI 5: 1 or N per observed parent (NULL: all 1)
    ]


# name -> (restype, argtypes)
_SIGNATURES = {
    "cbn_abi_version": (ctypes.c_int, []),
    "cbn_last_error": (ctypes.c_char_p, []),
    "cbn_bf_cpd_build": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64,
                                        ctypes.c_int32, ctypes.c_int32, ctypes.c_void_p, ctypes.c_void_p]),
    "cbn_bf_cpd_eval": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int32, ctypes.c_void_p, ctypes.c_void_p,
                                       ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p]),
    "cbn_plan_create": (ctypes.c_int, [ctypes.POINTER(FactorDesc), ctypes.c_int32, ctypes.c_int32,
                                       ctypes.POINTER(ctypes.c_void_p)]),
    "cbn_plan_destroy": (ctypes.c_int, [ctypes.c_void_p]),
    "cbn_plan_table_bytes": (ctypes.c_int64, [ctypes.c_void_p]),
    "cbn_plan_uses_lds": (ctypes.c_int, [ctypes.c_void_p]),
    "cbn_plan_build_tables": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p]),
    "cbn_plan_query_max": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p, ctypes.c_int32,
                                          ctypes.c_void_p, ctypes.c_void_p]),
    "cbn_plan_query_write": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p, ctypes.c_int32,
                                            ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]),
    "cbn_plan_infer": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p, ctypes.c_int32,
                                      ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]),
    "cbn_plan_run": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p, ctypes.c_int32,
                                    ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int32, ctypes.c_void_p]),
    "cbn_plan_timing": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(ctypes.c_int32),
                                       ctypes.POINTER(ctypes.c_float), ctypes.POINTER(ctypes.c_float)]),
    "cbn_plan_fused_capacity": (ctypes.c_int64, [ctypes.c_void_p]),
    "cbn_plan_status": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(ctypes.c_int32)]),
    "cbn_debug_flag_timeout": (ctypes.c_int, [ctypes.c_void_p]),
    "cbn_diag_enabled": (ctypes.c_int32, []),
    "cbn_plan_check": (ctypes.c_int, [ctypes.c_void_p]),
    "cbn_plan_flags": (ctypes.c_int32, [ctypes.c_void_p]),
    "cbn_scale": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p, ctypes.c_int32, ctypes.c_void_p]),
    "cbn_scale_batch": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int32, ctypes.c_void_p,
                                       ctypes.c_int32, ctypes.c_void_p]),
    "cbn_plan_max_words": (ctypes.c_int32, [ctypes.c_void_p]),
    "cbn_plan_run_fold": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p, ctypes.c_int32,
                                         ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64,
                                         ctypes.c_void_p, ctypes.c_int32, ctypes.c_int32, ctypes.c_void_p]),
    "cbn_plan_create_param": (ctypes.c_int, [ctypes.POINTER(ParamFactor), ctypes.c_int32, ctypes.c_int32,
                                             ctypes.POINTER(ctypes.c_void_p)]),
    "cbn_param_eval": (ctypes.c_int, [ctypes.POINTER(ParamModel), ctypes.c_void_p, ctypes.c_int64, ctypes.c_int32,
                                      ctypes.c_void_p, ctypes.c_int32, ctypes.c_void_p, ctypes.c_void_p]),
    "cbn_hash_build": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p,
                                      ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p]),
    "cbn_cpd_ref_eval": (ctypes.c_int, [ctypes.POINTER(CpdRef), ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p,
                                        ctypes.c_void_p]),
    "cbn_plan_create_direct": (ctypes.c_int, [ctypes.POINTER(DirectFactor), ctypes.c_int32, ctypes.c_int32,
                                              ctypes.POINTER(ctypes.c_void_p)]),
}
CBN_RUN_BUILD_TABLES = 1
CBN_RUN_TIMED = 2
CBN_RUN_TWO_PASS = 4
CBN_RUN_RAW = 8
CBN_E_LIMIT = -3
CBN_E_UNSUPPORTED = -4
CBN_E_TIMEOUT = -5
CBN_PLAN_FAST, CBN_PLAN_LDS, CBN_PLAN_PAIRED, CBN_PLAN_STAGED = 1, 2, 4, 8
CBN_PLAN_FUSED, CBN_PLAN_PARAMETRIC, CBN_PLAN_VPL2, CBN_PLAN_DIRECT = 16, 32, 64, 128
CBN_PLAN_COLS = 256
CBN_PLAN_SLOTS = 512

EXPORTED_SYMBOLS = tuple(_SIGNATURES)

_lib = None


class NativeError(RuntimeError):
    pass


def _check_stamp(path: str, digest: str) -> None:
    """Refuse a library not built from this tree's sources (its content stamp,
    written by __graft_entry__.build(), differs or is missing)."""
    got = _buildstamp.read_stamp(path)
    if got != digest:
        raise NativeError(
            f"{path} was not built from this tree's sources (stamp {got or 'missing'} != {digest[:16]}...): "
            "rebuild it with `python -c 'import __graft_entry__ as g; g.build()'`")


def load() -> ctypes.CDLL:
    """Load (once) and return the HIP library; raise if it is not built."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise NativeError(
                f"{LIB_PATH} is missing: build it with `python -c 'import __graft_entry__ as g; g.build()'` "
                "(no CPU fallback exists for the HIP inference path)")
        if LIB_PATH == _DEFAULT_LIB:  # (diagnostic variant builds under tools/ carry no stamp)
            _check_stamp(LIB_PATH, _buildstamp.lib_digest())
        lib = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in _SIGNATURES.items():
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        if lib.cbn_abi_version() != ABI_VERSION:
            raise NativeError("libcbn_amd.so ABI version mismatch")
        _lib = lib
    return _lib


_host = None
HOST_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "_cbn_host.so")


def load_host():
    """Load (once) the native host fast path (csrc/host_fast.cpp); raise if not built."""
    global _host
    if _host is None:
        if not os.path.exists(HOST_PATH):
            raise NativeError(f"{HOST_PATH} is missing: build it with `python -c 'import __graft_entry__ as g; "
                              "g.build()'`")
        import importlib.machinery
        import importlib.util

        _check_stamp(HOST_PATH, _buildstamp.host_digest())
        loader = importlib.machinery.ExtensionFileLoader("_cbn_host", HOST_PATH)
        spec = importlib.util.spec_from_file_location("_cbn_host", HOST_PATH, loader=loader)
        mod = importlib.util.module_from_spec(spec)
        loader.exec_module(mod)
        _host = mod
    return _host


def check(rc: int, what: str):
    if rc != 0:
        msg = load().cbn_last_error().decode(errors="replace")
        raise NativeError(f"{what} failed (rc={rc}): {msg}")


def require_gpu(device) -> torch.device:
    """The HIP device of ``device`` with an explicit index ("cuda" -> the
    current device): the native entry points take the index as an int."""
    device = torch.device(device)
    if device.type != "cuda" or not torch.cuda.is_available():
        raise NativeError(
            f"the MI355X inference path needs a HIP device, got device={device!s} "
            f"(torch.cuda.is_available()={torch.cuda.is_available()})")
    if device.index is None:
        device = torch.device("cuda", torch.cuda.current_device())
    load()
    return device


def stream_ptr(device) -> ctypes.c_void_p:
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)


def ptr(t: torch.Tensor) -> ctypes.c_void_p:
    return ctypes.c_void_p(t.data_ptr())
