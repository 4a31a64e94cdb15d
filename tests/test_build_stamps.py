"""build() is keyed on content, not mtimes: a source
edit whose file carries an OLDER mtime than the library still rebuilds it, an
unchanged tree skips every compiler call, and the loader refuses a library
whose stamp does not match the tree."""
import os
import shutil
import sys
import time

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import __graft_entry__ as ge  # noqa: E402
from continuousbayesiannetwork_amd import _buildstamp, _native  # noqa: E402


class _Proc:
    def __init__(self, cmd, **kw):
        self.out = cmd[cmd.index("-o") + 1]

    def wait(self):
        open(self.out, "wb").close()
        return 0


def _fake_tree(tmp_path, monkeypatch):
    """A copy of the sources / headers under tmp_path, with build() and the
    stamp module pointed at it and every compiler call recorded, not run."""
    pkg = tmp_path / "pkg"
    (pkg / "csrc").mkdir(parents=True)
    (tmp_path / "include").mkdir()
    st = ge._stamps()
    for p in [*st.LIB_SOURCES, *st.LIB_HEADERS, *st.HOST_SOURCES]:
        rel = os.path.relpath(p, st.ROOT)
        dst = tmp_path / rel.replace("continuousbayesiannetwork_amd", "pkg")
        dst.parent.mkdir(parents=True, exist_ok=True)
        shutil.copy(p, dst)
    st.ROOT, st.PKG, st.CSRC = str(tmp_path), str(pkg), str(pkg / "csrc")
    st.LIB_SOURCES = [str(pkg / "csrc" / os.path.basename(p)) for p in st.LIB_SOURCES]
    st.LIB_HEADERS = [str(pkg / "csrc" / "cbn_internal.h"), str(tmp_path / "include" / "cbn_amd.h")]
    st.HOST_SOURCES = [str(pkg / "csrc" / "host_fast.cpp")]
    calls = []

    def run(cmd):
        calls.append(cmd)
        open(cmd[cmd.index("-o") + 1], "wb").close()

    def popen(cmd, **kw):
        calls.append(cmd)
        return _Proc(cmd)

    monkeypatch.setattr(ge, "PKG", str(pkg))
    monkeypatch.setattr(ge, "_stamps", lambda: st)
    monkeypatch.setattr(ge, "_run", run)
    monkeypatch.setattr(ge.subprocess, "Popen", popen)
    return st, pkg, calls


def test_unchanged_tree_skips_and_old_mtime_edit_rebuilds(tmp_path, monkeypatch):
    st, pkg, calls = _fake_tree(tmp_path, monkeypatch)
    ge.build()  # first build: 3 objects + link + host extension
    assert len(calls) == 5
    lib = str(pkg / "libcbn_amd.so")
    assert st.is_current(lib, st.lib_digest())
    calls.clear()
    ge.build()  # nothing changed: no compiler call at all
    assert calls == []
    # edit one source, then make it look OLDER than the library
    src = pkg / "csrc" / "cbn_direct.hip"
    src.write_text(src.read_text() + "\n// edit\n")
    old = time.time() - 10 * 86400
    os.utime(src, (old, old))
    assert os.path.getmtime(src) < os.path.getmtime(lib)
    assert not st.is_current(lib, st.lib_digest())
    ge.build()
    compiled = [c[c.index("-o") + 1] for c in calls if "-c" in c]
    assert compiled == [str(pkg / "csrc" / "cbn_direct.o")]  # only the edited unit recompiles
    assert any(c[c.index("-o") + 1] == lib for c in calls if "-c" not in c)  # and the library relinks
    assert st.is_current(lib, st.lib_digest())
    calls.clear()
    # a header edit recompiles every unit
    hdr = pkg / "csrc" / "cbn_internal.h"
    hdr.write_text(hdr.read_text() + "\n")
    os.utime(hdr, (old, old))
    ge.build()
    assert len([c for c in calls if "-c" in c]) == 3


def test_loader_refuses_a_stale_library(tmp_path):
    lib = tmp_path / "libx.so"
    lib.write_bytes(b"\0")
    with pytest.raises(_native.NativeError, match="stamp missing"):
        _native._check_stamp(str(lib), "ab" * 32)
    _buildstamp.write_stamp(str(lib), "cd" * 32)
    with pytest.raises(_native.NativeError, match="not built from this tree"):
        _native._check_stamp(str(lib), "ab" * 32)
    _buildstamp.write_stamp(str(lib), "ab" * 32)
    _native._check_stamp(str(lib), "ab" * 32)


def test_shipped_libraries_match_the_tree():
    """The in-tree libraries the GPU box receives were built from these sources."""
    lib = os.path.join(ROOT, "continuousbayesiannetwork_amd", "libcbn_amd.so")
    host = os.path.join(ROOT, "continuousbayesiannetwork_amd", "_cbn_host.so")
    assert _buildstamp.is_current(lib, _buildstamp.lib_digest())
    assert _buildstamp.is_current(host, _buildstamp.host_digest())
