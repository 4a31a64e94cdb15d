"""Content stamps of the native builds (build infrastructure, not on the
inference path).

``__graft_entry__.build()`` writes ``<library>.sha256`` next to each library
it links: a sha256 over the bytes of every source and header the library is
built from, plus the compiler flags (and, for the torch host extension, the
torch version it links).  ``build()`` skips a library only when its stamp
matches the tree, and ``_native.load()`` / ``load_host()`` refuse a library
whose stamp does not -- a checkout or copy that reorders mtimes can no longer
run stale kernels against new sources.
"""
from __future__ import annotations

import hashlib
import os

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)
CSRC = os.path.join(PKG, "csrc")

HIP_FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared", "-mcode-object-version=5",
             "-mllvm", "-amdgpu-kernarg-preload-count=16",
             "-Wall", "-Wno-unused-result"]
HOST_FLAGS = ["-O2", "-std=c++17", "-fPIC", "-shared", "-DTORCH_EXTENSION_NAME=_cbn_host",
              "-DTORCH_API_INCLUDE_EXTENSION_H", "-D__HIP_PLATFORM_AMD__=1", "-DUSE_ROCM=1"]

LIB_SOURCES = [os.path.join(CSRC, f) for f in ("cbn_infer.hip", "cbn_param.hip", "cbn_direct.hip")]
LIB_HEADERS = [os.path.join(CSRC, "cbn_internal.h"), os.path.join(ROOT, "include", "cbn_amd.h")]
HOST_SOURCES = [os.path.join(CSRC, "host_fast.cpp")]


def _digest(paths, extra) -> str:
    h = hashlib.sha256()
    for p in paths:
        h.update(os.path.relpath(p, ROOT).encode() + b"\0")
        with open(p, "rb") as fh:
            h.update(fh.read())
        h.update(b"\0")
    for e in extra:
        h.update(str(e).encode() + b"\0")
    return h.hexdigest()


def object_digest(src: str) -> str:
    """One HIP translation unit: its source, the shared headers, the flags."""
    return _digest([src, *LIB_HEADERS], HIP_FLAGS)


def lib_digest() -> str:
    """libcbn_amd.so: every HIP source and header, the flags."""
    return _digest([*LIB_SOURCES, *LIB_HEADERS], HIP_FLAGS)


def host_digest() -> str:
    """_cbn_host.so: host_fast.cpp, its flags, the torch it links."""
    import torch

    return _digest(HOST_SOURCES, [*HOST_FLAGS, "torch " + torch.__version__])


def stamp_path(artifact: str) -> str:
    return artifact + ".sha256"


def read_stamp(artifact: str):
    try:
        with open(stamp_path(artifact)) as fh:
            return fh.read().strip()
    except OSError:
        return None


def write_stamp(artifact: str, digest: str) -> None:
    with open(stamp_path(artifact), "w") as fh:
        fh.write(digest + "\n")


def is_current(artifact: str, digest: str) -> bool:
    """The artifact exists and was built from exactly this content."""
    return os.path.exists(artifact) and read_stamp(artifact) == digest
