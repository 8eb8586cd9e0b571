"""The C-ABI library loads and exports every entry point include/shpl.h
declares (CPU only: no compute calls, no GPU needed)."""
import ctypes
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared():
    src = open(os.path.join(ROOT, "include", "shpl.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(shpl_[a-z0-9_]+)\s*\(", src)))


def test_header_declares_the_abi():
    names = _declared()
    for must in ["shpl_build_index", "shpl_gen_index", "shpl_produce_index", "shpl_pack_map",
                 "shpl_build_csr", "shpl_pull", "shpl_version"]:
        assert must in names


def test_library_exports_every_declared_symbol():
    from sparse_pooling_amd import _lib as L
    if not os.path.exists(L.LIB_PATH):
        from sparse_pooling_amd import build
        build.build()
    lib = L.lib()
    for name in _declared():
        assert hasattr(lib, name), name
    assert set(L.EXPORTED) == set(_declared())
    assert lib.shpl_version().decode().startswith("shpl")
    assert lib.shpl_status_string(2).decode() == "index out of bounds"


def test_workspace_queries_are_host_only():
    from sparse_pooling_amd import _lib as L
    assert L.csr_ws_bytes(563200 * 64, 20000 * 64) >= 4 * 20000 * 64
    assert L.index_ws_bytes(64, 20000) > 0


def test_missing_library_fails_loudly(monkeypatch, tmp_path):
    from sparse_pooling_amd import _lib as L
    monkeypatch.setattr(L, "_lib", None)
    monkeypatch.setattr(L, "LIB_PATH", str(tmp_path / "nope.so"))
    with pytest.raises(L.ShplLibraryError):
        L.lib()
