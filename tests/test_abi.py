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


def test_argument_validation_is_host_side():
    """Bad arguments are rejected with a status code before anything reaches the GPU
    (so this runs without one); fake non-null device pointers are never dereferenced."""
    import math
    from sparse_pooling_amd import _lib as L
    lib = L.lib()
    P = ctypes.c_void_p(256)  # a fake, aligned, non-null device pointer
    N = None
    # index builder: no frames / null offsets / voxel stride / workspace size
    assert lib.shpl_build_index(0, P, N, 10, P, L.F64, P, L.I64, 2, P, 1200., 360., 704., 800., 1., 1., N, P, P, P,
                                N, N, P, P, N, P, 1 << 20, N) == L.ERR_ARG
    assert lib.shpl_build_index(1, N, N, 10, P, L.F64, P, L.I64, 2, P, 1200., 360., 704., 800., 1., 1., N, P, P, P,
                                N, N, P, P, N, P, 1 << 20, N) == L.ERR_ARG
    assert lib.shpl_build_index(1, P, N, 10, P, L.F64, P, L.I64, 1, P, 1200., 360., 704., 800., 1., 1., N, P, P, P,
                                N, N, P, P, N, P, 1 << 20, N) == L.ERR_BAD_SHAPE
    assert lib.shpl_build_index(1, P, N, 10, P, L.F64, P, L.I64, 2, P, 1200., 360., 704., 800., 0., 1., N, P, P, P,
                                N, N, P, P, N, P, 1 << 20, N) == L.ERR_BAD_SHAPE
    assert lib.shpl_build_index(64, P, N, 100000, P, L.F64, P, L.I64, 2, P, 1200., 360., 704., 800., 1., 1., N, P,
                                P, P, N, N, P, P, N, P, 16, N) == L.ERR_WORKSPACE
    # CSR: bad order / direction / keys
    csr = L.ShplCsr(256, 256, 256, None, 100, 10)
    assert lib.shpl_build_csr(L.BY_CELL, 7, 1, P, N, 100, P, N, P, P, ctypes.byref(csr), P, 1 << 20, N) == L.ERR_ARG
    assert lib.shpl_build_csr(5, L.ORDER_ENTRY, 1, P, N, 100, P, N, P, P, ctypes.byref(csr), P, 1 << 20,
                              N) == L.ERR_ARG
    assert lib.shpl_build_csr(L.BY_PIXEL, L.ORDER_COL_ROW, 1, P, N, 100, P, N, P, P, ctypes.byref(csr), P, 1 << 20,
                              N) == L.ERR_ARG  # pixel-keyed lists need ent_col
    assert lib.shpl_build_csr(L.BY_CELL, L.ORDER_ENTRY, 2, P, N, 100, P, N, P, P, ctypes.byref(csr), P, 1 << 20,
                              N) == L.ERR_BAD_SHAPE  # n_keys < n_frames * keys_per_frame
    # pulls: bad enums, ADD with different widths, output narrower than the concat
    for fn in (lib.shpl_pull, lib.shpl_pull_dense, lib.shpl_pull_sparse):
        assert fn(9, L.F32, ctypes.byref(csr), P, 32, 0, 32, P, 32, 0, 32, L.OUT_CONCAT, P, 64, N) == L.ERR_ARG
        assert fn(L.BY_CELL, 7, ctypes.byref(csr), P, 32, 0, 32, P, 32, 0, 32, L.OUT_CONCAT, P, 64, N) == L.ERR_ARG
        assert fn(L.BY_CELL, L.F32, ctypes.byref(csr), P, 32, 0, 32, P, 16, 0, 16, L.OUT_ADD, P, 32,
                  N) == L.ERR_BAD_SHAPE
        assert fn(L.BY_CELL, L.F32, ctypes.byref(csr), P, 32, 0, 32, P, 32, 0, 32, L.OUT_CONCAT, P, 48,
                  N) == L.ERR_BAD_SHAPE
        assert fn(L.BY_CELL, L.F32, ctypes.byref(csr), P, 32, 0, 32, N, 32, 0, 32, L.OUT_CONCAT, P, 64,
                  N) == L.ERR_ARG
    # a pixel-keyed CSR without ent_col only when marked as one column per entry (SHPL_CSR_IDENTITY_COLS):
    # otherwise the pulls would sum without TF's per-column partials
    pix = L.ShplCsr(256, 256, 256, None, 100, 10)
    for fn in (lib.shpl_pull, lib.shpl_pull_dense, lib.shpl_pull_sparse, lib.shpl_pull_once):
        assert fn(L.BY_PIXEL, L.F32, ctypes.byref(pix), P, 32, 0, 32, P, 32, 0, 32, L.OUT_CONCAT, P, 64,
                  N) == L.ERR_ARG
    # shpl_pull_once: SHPL_OUT_POOL over a CSR with key_range only
    assert lib.shpl_pull_once(L.BY_CELL, L.F32, ctypes.byref(csr), P, 32, 0, 32, N, 0, 0, 0, L.OUT_POOL, P, 32,
                              N) == L.ERR_ARG  # no key_range
    kr = L.ShplCsr(256, 256, 256, None, 100, 10, 256)
    assert lib.shpl_pull_once(L.BY_CELL, L.F32, ctypes.byref(kr), P, 32, 0, 32, P, 32, 0, 32, L.OUT_CONCAT, P, 64,
                              N) == L.ERR_ARG  # not SHPL_OUT_POOL
    # the forward conv's row-streaming predicate (shpl_conv3x3_rows_form): f32 never, bf16 at 32 + 32 channels
    # without statistics yes, with training statistics over 32 + 16 pooled channels no (the tiled kernel)
    rf = ctypes.c_int(-1)
    ccell1 = L.ShplCsr(256, 256, 256, None, 176 * 200, 1000)
    for dt, cb, stats, want in ((L.F32, 32, 0, 0), (L.BF16, 32, 0, 1), (L.BF16, 16, 1, 0), (L.BF16, 32, 1, 1)):
        assert lib.shpl_conv3x3_rows_form(dt, 1, 176, 200, P, 32, 0, 32, P, cb, 0, cb, ctypes.byref(ccell1), P, P,
                                          32, L.ACT_NONE, P, 32, stats, ctypes.byref(rf)) == L.OK
        assert rf.value == want, (dt, cb, stats)
    assert lib.shpl_conv3x3_rows_form(L.BF16, 1, 176, 200, P, 32, 0, 32, P, 32, 0, 32, ctypes.byref(ccell1), P, P,
                                      16, L.ACT_NONE, P, 16, 0, ctypes.byref(rf)) == L.OK and rf.value == 0
    # the occupancy-limited input gradient: no pool / forward workspace / second map, keys that are not the map's,
    # a split outside (0, c_dx), a forward workspace smaller than that forward's plan -- all before any launch
    dg = (L.BF16, 1, 176, 200, P, 32, 32, P, 64, P, 32)
    fws = 1 << 24
    assert lib.shpl_conv3x3_dgrad_reuse(*dg, 32, P, 32, P, 1 << 20, None, P, fws, 0, N) == L.ERR_ARG
    assert lib.shpl_conv3x3_dgrad_reuse(*dg, 32, P, 32, P, 1 << 20, ctypes.byref(ccell1), N, fws, 0, N) == L.ERR_ARG
    assert lib.shpl_conv3x3_dgrad_reuse(*dg, 32, N, 32, P, 1 << 20, ctypes.byref(ccell1), P, fws, 0, N) == L.ERR_ARG
    assert lib.shpl_conv3x3_dgrad_reuse(*dg[:2], 175, *dg[3:], 32, P, 32, P, 1 << 20, ctypes.byref(ccell1), P, fws, 0,
                                        N) == L.ERR_BAD_SHAPE
    for split in (0, 64):
        assert lib.shpl_conv3x3_dgrad_reuse(*dg, split, P, 32, P, 1 << 20, ctypes.byref(ccell1), P, fws, 0,
                                            N) == L.ERR_BAD_SHAPE
    assert lib.shpl_conv3x3_dgrad_reuse(*dg, 32, P, 32, P, 1 << 20, ctypes.byref(ccell1), P, 16, 1, N) == L.ERR_ARG
    # buckets: shapes over the limits (65536 destinations per frame, 2^24 points per frame), workspace size,
    # missing bucket workspace; CSRs from buckets: null map, too few keys, small
    # workspace; pull pair: null CSR, the bad-shape checks of shpl_pull, no key_range
    nb = ctypes.c_size_t()
    assert lib.shpl_bucket_workspace_bytes(4, 20000, 80000, 8800, 6750, ctypes.byref(nb)) == L.OK and nb.value > 0
    assert lib.shpl_bucket_workspace_bytes(4, 20000, 80000, 70000, 6750, ctypes.byref(nb)) == L.ERR_BAD_SHAPE
    assert lib.shpl_bucket_workspace_bytes(4, (1 << 24) + 1, 80000, 8800, 6750, ctypes.byref(nb)) == L.ERR_BAD_SHAPE
    args = (4, P, N, 20000, P, L.F64, P, L.I64, 2, P, 1200., 360., 704., 800., 8., 8., N, P, P, P, P, P, P, P,
            1 << 20, 80000)
    assert lib.shpl_build_index_buckets(*args, N, 1 << 24, N, N, N) == L.ERR_ARG
    assert lib.shpl_build_index_buckets(*args, P, 64, N, N, N) == L.ERR_WORKSPACE
    assert lib.shpl_build_index_buckets(*args[:14], 1., 1., *args[16:], P, 1 << 24, N, N, N) == L.ERR_BAD_SHAPE
    odd = L.ShplPassCopy(L.BF16, 256, 12, 256, 24, 12)  # 24-byte rows: not 16-byte pieces
    assert lib.shpl_build_index_buckets(*args, P, 1 << 24, ctypes.byref(odd), N, N) == L.ERR_BAD_SHAPE
    bad = L.ShplPassCopy(7, 256, 32, 256, 64, 32)
    assert lib.shpl_build_index_buckets(*args, P, 1 << 24, N, ctypes.byref(bad), N) == L.ERR_ARG
    bk = L.ShplBuckets(4, 20000, 80000, 8800, 6750, 256, 256, 256, 256, 256, 256, nb.value)
    ccell = L.ShplCsr(256, 256, 256, None, 4 * 8800, 80000, 256)
    assert lib.shpl_build_csr_buckets(None, ctypes.byref(ccell), None, N) == L.ERR_ARG
    few = L.ShplCsr(256, 256, 256, None, 100, 80000, 256)  # fewer keys than frames x cells
    assert lib.shpl_build_csr_buckets(ctypes.byref(bk), ctypes.byref(few), None, N) == L.ERR_BAD_SHAPE
    small = L.ShplBuckets(4, 20000, 80000, 8800, 6750, 256, 256, 256, 256, 256, 256, 64)
    assert lib.shpl_build_csr_buckets(ctypes.byref(small), ctypes.byref(ccell), None, N) == L.ERR_WORKSPACE
    d32 = L.ShplPullDesc(L.F32, 256, 32, 0, 32, 256, 32, 0, 32, L.OUT_CONCAT, 256, 64)
    narrow = L.ShplPullDesc(L.F32, 256, 32, 0, 32, 256, 32, 0, 32, L.OUT_CONCAT, 256, 48)
    assert lib.shpl_pull_pair(None, ctypes.byref(d32), None, None, N) == L.ERR_ARG
    assert lib.shpl_pull_pair(ctypes.byref(ccell), ctypes.byref(narrow), None, None, N) == L.ERR_BAD_SHAPE
    norange = L.ShplCsr(256, 256, 256, None, 4 * 8800, 80000)  # row-keyed pulls need key_range
    assert lib.shpl_pull_pair(ctypes.byref(norange), ctypes.byref(d32), None, None, N) == L.ERR_ARG
    pnocol = L.ShplCsr(256, 256, 256, None, 4 * 6750, 80000, 256)  # pixel side: neither ent_col nor the flag
    assert lib.shpl_pull_pair(None, None, ctypes.byref(pnocol), ctypes.byref(d32), N) == L.ERR_ARG
    assert lib.shpl_build_csr_buckets(ctypes.byref(bk), None, ctypes.byref(pnocol), N) == L.ERR_ARG
    # run heads (shpl_csr.heads): head_k in [1, SHPL_CSR_MAX_HEAD] with key_range, built by the bucket CSR only
    for k, with_range in ((0, True), (L.CSR_MAX_HEAD + 1, True), (8, False)):
        hc = L.ShplCsr(256, 256, 256, None, 4 * 8800, 80000, 256 if with_range else None)
        hc.heads, hc.head_k = 256, k
        assert lib.shpl_build_csr_buckets(ctypes.byref(bk), ctypes.byref(hc), None, N) == L.ERR_ARG
        assert lib.shpl_pull_pair(ctypes.byref(hc), ctypes.byref(d32), None, None, N) == L.ERR_ARG
    hc = L.ShplCsr(256, 256, 256, None, 4 * 8800, 80000, 256)
    hc.heads, hc.head_k = 256, 8
    assert lib.shpl_build_csr(L.BY_CELL, L.ORDER_ENTRY, 4, P, N, 8800, P, N, P, P, ctypes.byref(hc), P, 1 << 24,
                              N) == L.ERR_ARG  # the other builders do not fill run heads
    # velodyne loader: P2 without image size, misaligned scan
    assert lib.shpl_velo_to_cam(1, P, 10, P, P, P, N, math.nan, N, P, P, N, P, 1 << 20, N) == L.ERR_ARG
    assert lib.shpl_velo_to_cam(1, P, 10, ctypes.c_void_p(260), P, N, N, math.nan, N, P, P, N, P, 1 << 20,
                                N) == L.ERR_BAD_SHAPE
    assert lib.shpl_velo_to_cam(1, P, -1, P, P, N, N, math.nan, N, P, P, N, P, 1 << 20, N) == L.ERR_BAD_SHAPE
    # BEV slices: slice count outside [1, 8]; MV3D: neither img_index2 nor P
    ext = (ctypes.c_double * 6)(-40, 40, -5, 3, 0, 70)
    lo = (ctypes.c_double * 9)()
    tab = (ctypes.c_double * 16)()
    for ns in (0, 9):
        assert lib.shpl_bev_slices(1, P, N, 10, P, L.F64, P, ext, 0.1, ns, lo, lo, 0., 1., 0.5, tab, P, P, P, N, N,
                                   N, P, 1 << 20, N) in (L.ERR_BAD_SHAPE, L.ERR_ARG)
    rng = (ctypes.c_double * 6)(0, 48, -20, 20, -1, 3)
    assert lib.shpl_mv3d_voxels(1, P, 10, P, 4, N, N, N, rng, 0.2, 0.4, 45, P, 10, P, P, P, N, N, P, 1 << 20,
                                N) == L.ERR_ARG
