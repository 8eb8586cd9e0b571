"""HIP path vs the CPU oracle (and the reference-generated goldens) on MI355X.

Integer / index outputs must be bit-exact. Floating-point outputs carry the
north_star contract ``max |gpu - ref| <= 1e-5`` (TOL below) and, since the
kernels keep TF-CPU's operation order with no FMA contraction, are also
asserted bit-identical where the oracle computes in the same precision.
"""
import glob
import os

import numpy as np
import pytest
import torch

from oracle import shpl_oracle as orc
from sparse_pooling_amd import synth

pytestmark = pytest.mark.gpu

TOL = 1e-5  # north_star: "within 1e-5 fp32" of the TF CPU reference
DEV = "cuda"
GOLD = os.path.join(os.path.dirname(__file__), "golden")


def _np(t):
    return t.detach().cpu().numpy() if isinstance(t, torch.Tensor) else np.asarray(t)


def _close_and_exact(a, b):
    a, b = _np(a).astype(np.float32), _np(b).astype(np.float32)
    assert a.shape == b.shape, (a.shape, b.shape)
    if a.size:
        assert np.nanmax(np.abs(a - b)) <= TOL
    np.testing.assert_array_equal(a, b)


@pytest.fixture(scope="module", autouse=True)
def _lib():
    from sparse_pooling_amd import _lib as L
    L.lib()
    assert torch.cuda.is_available()


# ---------------------------------------------------------------- index builder

INDEX = sorted(glob.glob(os.path.join(GOLD, "index_*.npz")))


@pytest.mark.parametrize("path", INDEX, ids=[os.path.basename(p) for p in INDEX])
def test_index_builder_vs_reference_goldens(path):
    from sparse_pooling_amd import sparse_pool_utils as spu
    g = np.load(path)
    calib = synth.StereoCalib(g["P"])
    gen = spu.gen_sparse_pooling_input_avod(g["points"], g["voxel_indices"], calib, list(g["im_size"]),
                                            tuple(g["bv_size"]))
    np.testing.assert_array_equal(_np(gen["bv_index"]), g["gen_bv_index"].reshape(-1, 2))
    np.testing.assert_array_equal(_np(gen["img_index"]), g["gen_img_index"].reshape(3, -1))
    mval = g["M_val_in"] if "M_val_in" in g.files else None
    out = spu.produce_sparse_pooling_input(gen, M_val=mval, stride=list(g["stride"]))
    np.testing.assert_array_equal(_np(out["Mij_pool"]), g["Mij_pool"].reshape(-1, 2))
    np.testing.assert_array_equal(_np(out["img_index_flip_pool"]), g["img_index_flip_pool"].reshape(-1, 3))
    np.testing.assert_array_equal(out["M_size"], g["M_size"])
    np.testing.assert_array_equal(_np(out["M_val"]), g["M_val"])
    np.testing.assert_array_equal(_np(gen["img_index"]), g["mutated_img_index"].reshape(3, -1))
    # the fused single-pass builder gives the same M
    fused = spu.build_sparse_pooling_input(g["points"], g["voxel_indices"], calib, list(g["im_size"]),
                                           tuple(g["bv_size"]), stride=tuple(g["stride"]))
    np.testing.assert_array_equal(_np(fused["Mij_pool"]), g["Mij_pool"].reshape(-1, 2))
    np.testing.assert_array_equal(_np(fused["img_index_flip_pool"]), g["img_index_flip_pool"].reshape(-1, 3))
    np.testing.assert_array_equal(fused["M_size"], g["M_size"])


def test_produce_mutates_numpy_input_like_reference():
    from sparse_pooling_amd import sparse_pool_utils as spu
    g = np.load(os.path.join(GOLD, "index_config1.npz"))
    d = {"bv_index": g["gen_bv_index"], "img_index": g["gen_img_index"].copy(),
         "bv_size": g["gen_bv_size"], "img_size": g["gen_img_size"]}
    spu.produce_sparse_pooling_input(d, stride=list(g["stride"]))
    np.testing.assert_array_equal(d["img_index"], g["mutated_img_index"])


def _oracle_frame(fr, stride):
    gen = orc.gen_sparse_pooling_input_avod(fr.points, fr.voxel_indices, fr.P, list(fr.spec.im_size),
                                            tuple(fr.spec.bv_size))
    return orc.produce_sparse_pooling_input(gen, stride=stride)


@pytest.mark.parametrize("cfg", [1, 2, 3])
def test_batched_index_builder_matches_oracle_per_frame(cfg):
    from sparse_pooling_amd import pipeline, shpl_map as sm
    spec = synth.CONFIGS[cfg]
    frames = [synth.make_frame(spec, seed=100 + f, n_outside=37 * f) for f in range(4)]
    pts, vox, off, P, maxp, N = pipeline.stack_frames(frames, DEV)
    ib = sm.build_index_batch(pts, vox, off, P, spec.im_size, spec.bv_size, spec.stride, maxp,
                              ref_outputs=True)
    fo, fn = _np(ib.frame_off), _np(ib.frame_nnz)
    for f, fr in enumerate(frames):
        ref = _oracle_frame(fr, spec.stride)
        a, b = fo[f], fo[f] + fn[f]
        assert (_np(ib.map.cell[b:fo[f + 1]]) == -1).all()  # capacity tail of the frame
        np.testing.assert_array_equal(_np(ib.mij[a:b]), ref["Mij_pool"])
        np.testing.assert_array_equal(_np(ib.flip[a:b]), ref["img_index_flip_pool"])
        R = int(ref["M_size"][0])
        np.testing.assert_array_equal(_np(ib.map.cell[a:b]), ref["Mij_pool"][:, 0] + f * R)
    assert ib.map.error_bits() == 0


def test_batched_index_builder_ragged_frames_across_chunks():
    """Frames straddling the builder's 4096-point workgroup chunks, an empty
    frame and a one-point frame, in one batch (SHPL_EBIT_CAPACITY when the
    declared max_points_per_frame is too small)."""
    from sparse_pooling_amd import pipeline, shpl_map as sm, _lib as L
    base = synth.CONFIGS[2]
    frames = []
    for f, n in enumerate([4097, 0, 1, 4095, 4096, 9000, 12289]):
        if n == 0:
            frames.append(synth.Frame(np.zeros((0, 3)), np.zeros((0, 2), dtype=np.int64), synth.KITTI_P2,
                                      synth.FrameSpec(0, base.im_size, base.bv_size, base.stride)))
            continue
        spec = synth.FrameSpec(n, base.im_size, base.bv_size, base.stride)
        frames.append(synth.make_frame(spec, seed=300 + f, n_outside=min(n, 41 * f)))
    pts, vox, off, P, maxp, N = pipeline.stack_frames(frames, DEV)
    ib = sm.build_index_batch(pts, vox, off, P, base.im_size, base.bv_size, base.stride, maxp, ref_outputs=True)
    fo, fn = _np(ib.frame_off), _np(ib.frame_nnz)
    for f, fr in enumerate(frames):
        a, b = fo[f], fo[f] + fn[f]
        assert (_np(ib.map.cell[b:fo[f + 1]]) == -1).all()
        ref = _oracle_frame(fr, base.stride)  # the oracle's FMA chain also for the 1-point frame
        np.testing.assert_array_equal(_np(ib.mij[a:b]), ref["Mij_pool"])
        np.testing.assert_array_equal(_np(ib.flip[a:b]), ref["img_index_flip_pool"])
    assert ib.map.error_bits() == 0
    small = sm.build_index_batch(pts, vox, off, P, base.im_size, base.bv_size, base.stride, 4096)
    torch.cuda.synchronize()
    assert small.map.error_bits() & L.EBIT_CAPACITY


# ---------------------------------------------------------------- pooling ops

def _frame_case(cfg, seed=0, dtype=np.float32):
    spec = synth.CONFIGS[cfg]
    fr = synth.make_frame(spec, seed=seed, n_outside=50)
    ref = _oracle_frame(fr, spec.stride)
    Hb, Wb = spec.bev_feat_hw
    Hi, Wi = spec.img_feat_hw
    bev = synth.make_features((1, Hb, Wb, spec.c_bev), seed + 1)
    img = synth.make_features((1, Hi, Wi, spec.c_img), seed + 2)
    return spec, ref, bev, img


def _M(ref):
    from sparse_pooling_amd.sparse_pool_utils import SparseTensor
    return SparseTensor(ref["Mij_pool"], ref["M_val"], ref["M_size"])


@pytest.mark.parametrize("cfg", [1, 2])
def test_sparse_pool_layer_forward(cfg):
    from sparse_pooling_amd import sparse_pool_utils as spu
    spec, ref, bev, img = _frame_case(cfg)
    tb, ti = torch.from_numpy(bev).to(DEV), torch.from_numpy(img).to(DEV)
    bv_f, img_f = spu.sparse_pool_layer([tb, ti], [spec.c_img, spec.c_bev], _M(ref),
                                        img_index_flip=ref["img_index_flip_pool"].astype(np.int32))
    eb, ei = orc.sparse_pool_layer(bev, img, ref["Mij_pool"], ref["M_val"], ref["M_size"],
                                   ref["img_index_flip_pool"])
    _close_and_exact(bv_f, eb)
    assert img_f is ti


@pytest.mark.parametrize("cfg", [1, 2])
def test_dual_layer_forward_backward(cfg):
    from sparse_pooling_amd import sparse_pool_utils as spu
    spec, ref, bev, img = _frame_case(cfg, seed=3)
    tb = torch.from_numpy(bev).to(DEV).requires_grad_(True)
    ti = torch.from_numpy(img).to(DEV).requires_grad_(True)
    bv_f, img_f = spu.sparse_pool_layer([tb, ti], [spec.c_img, spec.c_bev], _M(ref),
                                        img_index_flip=ref["img_index_flip_pool"], bv_index=np.zeros((1, 3)))
    eb, ei = orc.sparse_pool_layer(bev, img, ref["Mij_pool"], ref["M_val"], ref["M_size"],
                                   ref["img_index_flip_pool"], dual=True)
    _close_and_exact(bv_f, eb)
    _close_and_exact(img_f, ei)
    gb = synth.make_features(tuple(bv_f.shape), 11)
    gi = synth.make_features(tuple(img_f.shape), 12)
    torch.autograd.backward([bv_f, img_f], [torch.from_numpy(gb).to(DEV), torch.from_numpy(gi).to(DEV)])
    Cb, Ci = spec.c_bev, spec.c_img
    mij, mval, msize, idx = ref["Mij_pool"], ref["M_val"], ref["M_size"], ref["img_index_flip_pool"]
    # TF gradient: d_img = g_img[..., :Ci] + scatter_nd(idx, M^T g_bv[..., Cb:])
    d_img = orc.sparse_pool_grad_img(mij, mval, msize, gb[0, ..., Cb:].reshape(-1, Ci), idx, img.shape)
    d_img = (gi[..., :Ci] + d_img).astype(np.float32)
    # d_bev = g_bv[..., :Cb] + (M^T)^T gather_nd(g_img[..., Ci:], idx)
    d_bev = orc.sparse_pool_trans_grad_bev(mij, mval, msize, np.ascontiguousarray(gi[..., Ci:]), idx)
    d_bev = (gb[..., :Cb] + d_bev.reshape(bev.shape)).astype(np.float32)
    _close_and_exact(ti.grad, d_img)
    _close_and_exact(tb.grad, d_bev)


def test_single_direction_ops_and_grads():
    from sparse_pooling_amd import sparse_pool_utils as spu
    spec, ref, bev, img = _frame_case(1, seed=5)
    M = _M(ref)
    idx = ref["img_index_flip_pool"]
    ti = torch.from_numpy(img).to(DEV).requires_grad_(True)
    Hb, Wb = spec.bev_feat_hw
    y = spu._sparse_pool_op(M, ti, idx, [1, Hb, Wb, spec.c_img])
    ey = orc.sparse_pool_op(ref["Mij_pool"], ref["M_val"], ref["M_size"], img, idx)
    _close_and_exact(y, ey.reshape(1, Hb, Wb, -1))
    g = synth.make_features(tuple(y.shape), 9)
    y.backward(torch.from_numpy(g).to(DEV))
    _close_and_exact(ti.grad, orc.sparse_pool_grad_img(ref["Mij_pool"], ref["M_val"], ref["M_size"],
                                                       g.reshape(-1, spec.c_img), idx, img.shape))
    tb = torch.from_numpy(bev).to(DEV).requires_grad_(True)
    z = spu._sparse_pool_trans_op(M, tb, idx, [1, img.shape[1], img.shape[2], spec.c_bev])
    ez = orc.sparse_pool_trans_op(ref["Mij_pool"], ref["M_val"], ref["M_size"], bev.reshape(-1, spec.c_bev),
                                  idx, img.shape)
    _close_and_exact(z, ez)
    gz = synth.make_features(tuple(z.shape), 10)
    z.backward(torch.from_numpy(gz).to(DEV))
    _close_and_exact(tb.grad, orc.sparse_pool_trans_grad_bev(ref["Mij_pool"], ref["M_val"], ref["M_size"], gz,
                                                             idx).reshape(bev.shape))


def test_noncanonical_M_weights_and_collisions():
    """Shuffled nnz order, several entries per column, non-unit weights,
    heavy pixel / cell collisions, odd channel count (scalar path)."""
    from sparse_pooling_amd import sparse_pool_utils as spu
    rng = np.random.default_rng(21)
    n, R, hb, wb, h, w, c = 500, 600, 20, 30, 15, 17, 3
    idx = np.stack([np.zeros(n, np.int64), rng.integers(0, h, n), rng.integers(0, w, n)], 1)
    idx[: n // 4, 1:] = idx[0, 1:]
    rows = rng.integers(0, R, n)
    rows[100:180] = rows[100]
    extra = np.stack([rng.integers(0, R, 300), rng.integers(0, n, 300)], 1)
    mij = np.concatenate([np.stack([rows, np.arange(n)], 1), extra]).astype(np.int64)
    mij = mij[rng.permutation(len(mij))]
    mval = rng.uniform(-2, 2, len(mij)).astype(np.float32)
    img = rng.standard_normal((1, h, w, c)).astype(np.float32)
    bev = rng.standard_normal((1, hb, wb, c)).astype(np.float32)
    M = spu.SparseTensor(mij, mval, np.array([R, n]))
    y = spu._sparse_pool_op(M, torch.from_numpy(img).to(DEV), idx, [1, hb, wb, c])
    _close_and_exact(y, orc.sparse_pool_op(mij, mval, [R, n], img, idx).reshape(1, hb, wb, c))
    z = spu._sparse_pool_trans_op(M, torch.from_numpy(bev).to(DEV), idx, [1, h, w, c])
    _close_and_exact(z, orc.sparse_pool_trans_op(mij, mval, [R, n], bev.reshape(-1, c), idx, img.shape))
    tb = torch.from_numpy(bev).to(DEV).requires_grad_(True)
    ti = torch.from_numpy(img).to(DEV).requires_grad_(True)
    bv_f, img_f = spu.sparse_pool_layer([tb, ti], [c, c], M, img_index_flip=idx, bv_index=1)
    gb = rng.standard_normal(tuple(bv_f.shape)).astype(np.float32)
    gi = rng.standard_normal(tuple(img_f.shape)).astype(np.float32)
    torch.autograd.backward([bv_f, img_f], [torch.from_numpy(gb).to(DEV), torch.from_numpy(gi).to(DEV)])
    d_img = gi[..., :c] + orc.sparse_pool_grad_img(mij, mval, [R, n], gb[0, ..., c:].reshape(-1, c), idx,
                                                   img.shape)
    d_bev = gb[..., :c] + orc.sparse_pool_trans_grad_bev(mij, mval, [R, n], np.ascontiguousarray(gi[..., c:]),
                                                         idx).reshape(bev.shape)
    _close_and_exact(ti.grad, d_img)
    _close_and_exact(tb.grad, d_bev)


@pytest.mark.parametrize("c", [3, 8, 64])
def test_row_keyed_pulls_noncanonical_M(c):
    """k_rows (shpl_pull over a CSR with key_range) == k_dense + k_sparse == the oracle,
    bitwise, on a non-canonical M: shuffled nnz, repeated columns (TF's per-column
    partials), negative weights, a 160-entry run, 3 / 8 / 64 channels (scalar path,
    one chunk per lane, groups of 16 lanes), every direction / order / output mode."""
    from sparse_pooling_amd import _lib as L
    from sparse_pooling_amd import shpl_map as sm
    rng = np.random.default_rng(22)
    n, R, hb, wb, h, w = 500, 600, 20, 30, 15, 17
    idx = np.stack([np.zeros(n, np.int64), rng.integers(0, h, n), rng.integers(0, w, n)], 1)
    idx[: n // 4, 1:] = idx[0, 1:]
    rows = rng.integers(0, R, n)
    rows[100:260] = rows[100]
    extra = np.stack([rng.integers(0, R, 300), rng.integers(0, n, 300)], 1)
    mij = np.concatenate([np.stack([rows, np.arange(n)], 1), extra]).astype(np.int64)
    mij = mij[rng.permutation(len(mij))]
    mval = rng.uniform(-2, 2, len(mij)).astype(np.float32)
    img = rng.standard_normal((1, h, w, c)).astype(np.float32)
    bev = rng.standard_normal((1, hb, wb, c)).astype(np.float32)
    ti, tb = torch.from_numpy(img).to(DEV), torch.from_numpy(bev).to(DEV)
    outs = {}
    for rows_mode in (True, False):
        sm.ShplMap.ROW_PULLS = rows_mode
        try:
            smap = sm.pack_map(torch.from_numpy(mij).to(DEV), torch.from_numpy(mval).to(DEV),
                               np.array([R, n]), torch.from_numpy(idx).to(DEV), img.shape)
            res = []
            for direction, order, src, pas, nrow in ((L.BY_CELL, L.ORDER_ENTRY, ti, tb, R),
                                                     (L.BY_PIXEL, L.ORDER_COL_ROW, tb, ti, h * w),
                                                     (L.BY_PIXEL, L.ORDER_COL_ENTRY, tb, ti, h * w),
                                                     (L.BY_CELL, L.ORDER_COL_ENTRY, ti, tb, R)):
                pool = torch.full((nrow, c), float("nan"), device=DEV)
                sm.pull(smap, direction, order, src, c, 0, c, pool, c)
                p2 = pas.reshape(nrow, c)
                cat = torch.full((nrow, 2 * c), float("nan"), device=DEV)
                sm.pull(smap, direction, order, src, c, 0, c, cat, 2 * c, pass_=p2, pass_stride=c, c_pass=c,
                        mode=L.OUT_CONCAT)
                add = torch.full((nrow, c), float("nan"), device=DEV)
                sm.pull(smap, direction, order, src, c, 0, c, add, c, pass_=p2, pass_stride=c, c_pass=c,
                        mode=L.OUT_ADD)
                res += [cat, add, pool]
            torch.cuda.synchronize()
            outs[rows_mode] = [_np(t) for t in res]
        finally:
            sm.ShplMap.ROW_PULLS = None
    for a, b in zip(outs[True], outs[False]):
        np.testing.assert_array_equal(a.view(np.uint32), b.view(np.uint32))
    # against the oracle: img -> BEV (TF entry order) and BEV -> img (transpose + ScatterNd)
    _close_and_exact(outs[True][2], orc.sparse_pool_op(mij, mval, [R, n], img, idx).reshape(R, c))
    _close_and_exact(outs[True][5], orc.sparse_pool_trans_op(mij, mval, [R, n], bev.reshape(-1, c), idx,
                                                             img.shape).reshape(h * w, c))
    _close_and_exact(outs[True][0][:, :c], bev.reshape(R, c))


def test_invalid_indices_raise():
    from sparse_pooling_amd import sparse_pool_utils as spu
    from sparse_pooling_amd.errors import InvalidArgumentError
    spec, ref, bev, img = _frame_case(1, seed=7)
    ti = torch.from_numpy(img).to(DEV)
    tb = torch.from_numpy(bev).to(DEV)
    idx = ref["img_index_flip_pool"].copy()
    idx[5, 2] = img.shape[2]
    with pytest.raises(InvalidArgumentError):
        spu.sparse_pool_layer([tb, ti], [spec.c_img, spec.c_bev], _M(ref), img_index_flip=idx)
    mij = ref["Mij_pool"].copy()
    mij[3, 0] = ref["M_size"][0]
    from sparse_pooling_amd.sparse_pool_utils import SparseTensor
    with pytest.raises(InvalidArgumentError):
        spu.sparse_pool_layer([tb, ti], [spec.c_img, spec.c_bev], SparseTensor(mij, ref["M_val"], ref["M_size"]),
                              img_index_flip=ref["img_index_flip_pool"])
    with pytest.raises(InvalidArgumentError):  # len(M_val) != nnz
        spu.sparse_pool_layer([tb, ti], [spec.c_img, spec.c_bev],
                              SparseTensor(ref["Mij_pool"], ref["M_val"][:-1], ref["M_size"]),
                              img_index_flip=ref["img_index_flip_pool"])
    with pytest.raises(TypeError):  # concat_bn_op is broken in the reference
        spu.sparse_pool_layer([tb, ti], [spec.c_img, spec.c_bev], _M(ref),
                              img_index_flip=ref["img_index_flip_pool"], use_bn=True)


def test_empty_M():
    from sparse_pooling_amd import sparse_pool_utils as spu
    img = synth.make_features((1, 9, 11, 4), 1)
    bev = synth.make_features((1, 6, 7, 4), 2)
    M = spu.SparseTensor(np.zeros((0, 2), np.int64), np.zeros(0), np.array([42, 0]))
    bv_f, _ = spu.sparse_pool_layer([torch.from_numpy(bev).to(DEV), torch.from_numpy(img).to(DEV)], [4, 4], M,
                                    img_index_flip=np.zeros((0, 3), np.int32))
    out = _np(bv_f)
    np.testing.assert_array_equal(out[..., :4], bev)
    assert not out[..., 4:].any()


@pytest.mark.parametrize("rows_mode", [True, False])
def test_empty_map_pulls_every_form(rows_mode):
    """pack_map with nnz = 0, pulled through the row-keyed (key_range CSR) and the
    dense + sparse forms, every output mode: the pooled part is zeros, CONCAT copies
    the pass-through half, ADD is pass + 0 (-0 -> +0), no uninitialised key_range
    is walked (the outputs start as NaN)."""
    from sparse_pooling_amd import _lib as L
    from sparse_pooling_amd import shpl_map as sm
    c, R, h, w = 8, 42, 9, 11
    img = synth.make_features((1, h, w, c), 1)
    bev = synth.make_features((1, 6, 7, c), 2)
    bev.flat[0] = -0.0
    ti, tb = torch.from_numpy(img).to(DEV), torch.from_numpy(bev).to(DEV)
    sm.ShplMap.ROW_PULLS = rows_mode
    try:
        smap = sm.pack_map(torch.zeros((0, 2), dtype=torch.int64, device=DEV), torch.zeros(0, device=DEV),
                           np.array([R, 0]), torch.zeros((0, 3), dtype=torch.int64, device=DEV), img.shape)
        for direction, order, src, pas, nrow in ((L.BY_CELL, L.ORDER_ENTRY, ti, tb, R),
                                                 (L.BY_PIXEL, L.ORDER_COL_ROW, tb, ti, h * w)):
            p2 = pas.reshape(nrow, c)
            pool = torch.full((nrow, c), float("nan"), device=DEV)
            sm.pull(smap, direction, order, src, c, 0, c, pool, c)
            cat = torch.full((nrow, 2 * c), float("nan"), device=DEV)
            sm.pull(smap, direction, order, src, c, 0, c, cat, 2 * c, pass_=p2, pass_stride=c, c_pass=c,
                    mode=L.OUT_CONCAT)
            add = torch.full((nrow, c), float("nan"), device=DEV)
            sm.pull(smap, direction, order, src, c, 0, c, add, c, pass_=p2, pass_stride=c, c_pass=c,
                    mode=L.OUT_ADD)
            torch.cuda.synchronize()
            zero = np.zeros((nrow, c), np.float32)
            np.testing.assert_array_equal(_np(pool).view(np.uint32), zero.view(np.uint32))
            np.testing.assert_array_equal(_np(cat)[:, :c].view(np.uint32), _np(p2).view(np.uint32))
            np.testing.assert_array_equal(_np(cat)[:, c:].view(np.uint32), zero.view(np.uint32))
            np.testing.assert_array_equal(_np(add).view(np.uint32), (_np(p2) + np.float32(0)).view(np.uint32))
    finally:
        sm.ShplMap.ROW_PULLS = None


@pytest.mark.parametrize("n", [3000, 20000])
def test_range_csr_one_long_run(n):
    """Every entry of a frame on ONE destination (all points on one cell and one
    pixel): the range CSR's degenerate case (one run longer than its LDS list at
    n = 20000), row-keyed pulls in both directions against the oracle, bitwise;
    the per-frame builder (tile sort, no key ranges) gives the same cell-keyed entry list."""
    from sparse_pooling_amd import _lib as L
    from sparse_pooling_amd import shpl_map as sm
    rng = np.random.default_rng(5)
    c, R, h, w = 8, 64, 6, 7
    idx = np.tile(np.array([[0, 2, 3]], np.int64), (n, 1))
    mij = np.stack([np.full(n, 17), np.arange(n)], 1).astype(np.int64)
    mval = rng.uniform(-1, 1, n).astype(np.float32)
    img = rng.standard_normal((1, h, w, c)).astype(np.float32)
    bev = rng.standard_normal((1, 8, 8, c)).astype(np.float32)
    ti, tb = torch.from_numpy(img).to(DEV), torch.from_numpy(bev).to(DEV)
    sm.ShplMap.ROW_PULLS = True
    try:
        smap = sm.pack_map(torch.from_numpy(mij).to(DEV), torch.from_numpy(mval).to(DEV), np.array([R, n]),
                           torch.from_numpy(idx).to(DEV), img.shape)
        pool = torch.full((R, c), float("nan"), device=DEV)
        sm.pull(smap, L.BY_CELL, L.ORDER_ENTRY, ti, c, 0, c, pool, c)
        trans = torch.full((h * w, c), float("nan"), device=DEV)
        sm.pull(smap, L.BY_PIXEL, L.ORDER_COL_ROW, tb, c, 0, c, trans, c)
        torch.cuda.synchronize()
    finally:
        sm.ShplMap.ROW_PULLS = None
    _close_and_exact(_np(pool), orc.sparse_pool_op(mij, mval, [R, n], img, idx).reshape(R, c))
    _close_and_exact(_np(trans), orc.sparse_pool_trans_op(mij, mval, [R, n], bev.reshape(-1, c), idx,
                                                          img.shape).reshape(h * w, c))
    lists = []
    for path in (L.CSR_RANGE, L.CSR_FRAME):
        cs = L.Csr(smap.n_cells, smap.nnz_cap, DEV, with_col=False, key_range=path == L.CSR_RANGE)
        L.check(L.lib().shpl_build_csr_path(path, L.BY_CELL, L.ORDER_ENTRY, 1, L.ptr(smap.frame_off),
                                            L.ptr(smap.frame_nnz), smap.n_cells, L.ptr(smap.cell), L.ptr(smap.col),
                                            L.ptr(smap.val), L.ptr(smap.pix), cs.ref(), L.ptr(cs.ws), cs.ws.numel(),
                                            L.stream_of(torch.device(DEV))), "shpl_build_csr_path")
        torch.cuda.synchronize()
        lists.append([_np(t).copy() for t in (cs.ent_dst, cs.ent_src, cs.ent_val)])
    for a, b in zip(*lists):
        np.testing.assert_array_equal(a.view(np.uint32), b.view(np.uint32))


@pytest.mark.parametrize("dtype,c", [("f32", 8), ("f32", 256), ("f32", 320), ("bf16", 256), ("bf16", 24)])
def test_pull_once_runs_across_windows(dtype, c):
    """shpl_pull_once's cell-keyed run walk (a wave per 64 sorted entries from 32 chunks of 16 bytes up; the
    (entry, chunk) walk below): runs of 1-3 entries, runs that end on and cross the 64-entry window edges, runs
    of 64, 70 and 150 entries (continued past their window, a window with no head at all), pooled widths of 2
    to 80 chunks (a partial second chunk group at 320 f32 channels) -- every row written once, against the
    oracle's sparse_pool_op (bitwise, or bf16 output rounding)."""
    from sparse_pooling_amd import _lib as L
    from sparse_pooling_amd import shpl_map as sm
    rng = np.random.default_rng(11)
    R, h, w = 700, 9, 11
    lens = [1] * 63 + [2] + [150] + list(rng.integers(1, 4, 200)) + [64] + [1] * 5 + [70] + [3] * 30
    cells = np.sort(rng.choice(R, len(lens), replace=False))
    cell = np.repeat(cells, lens)
    n = cell.size
    mij = np.stack([cell, np.arange(n)], 1).astype(np.int64)
    mval = rng.uniform(-1, 1, n).astype(np.float32)
    idx = np.stack([np.zeros(n), rng.integers(0, h, n), rng.integers(0, w, n)], 1).astype(np.int64)
    img = rng.standard_normal((1, h, w, c)).astype(np.float32)
    dt = torch.bfloat16 if dtype == "bf16" else torch.float32
    if dtype == "bf16":
        img = orc.from_bf16_bits(orc.to_bf16_bits(img))
    ti = torch.from_numpy(img).to(DEV).to(dt)
    sm.ShplMap.ROW_PULLS = True
    try:
        smap = sm.pack_map(torch.from_numpy(mij).to(DEV), torch.from_numpy(mval).to(DEV), np.array([R, n]),
                           torch.from_numpy(idx).to(DEV), img.shape)
        pool = torch.full((R, c), float("nan"), device=DEV, dtype=dt)
        sm.pull(smap, L.BY_CELL, L.ORDER_ENTRY, ti, c, 0, c, pool, c, part="once")
        torch.cuda.synchronize()
    finally:
        sm.ShplMap.ROW_PULLS = None
    ref = orc.sparse_pool_op(mij, mval, [R, n], img, idx).reshape(R, c)
    if dtype == "bf16":
        ref = orc.from_bf16_bits(orc.to_bf16_bits(ref))
    _close_and_exact(pool.float().cpu().numpy(), ref)


def test_bf16_storage_fp32_accumulate():
    """Config 3 storage: bf16 in/out, f32 accumulation, rounded once (RNE)."""
    from sparse_pooling_amd import sparse_pool_utils as spu
    spec, ref, bev, img = _frame_case(3, seed=8)
    bev16, img16 = orc.to_bf16_bits(bev), orc.to_bf16_bits(img)
    tb = torch.from_numpy(bev16.view(np.int16)).to(DEV).view(torch.bfloat16)
    ti = torch.from_numpy(img16.view(np.int16)).to(DEV).view(torch.bfloat16)
    bv_f, img_f = spu.sparse_pool_layer([tb, ti], [spec.c_img, spec.c_bev], _M(ref),
                                        img_index_flip=ref["img_index_flip_pool"], bv_index=1)
    eb, ei = orc.sparse_pool_layer(orc.from_bf16_bits(bev16), orc.from_bf16_bits(img16), ref["Mij_pool"],
                                   ref["M_val"], ref["M_size"], ref["img_index_flip_pool"], dual=True)
    np.testing.assert_array_equal(_np(bv_f.view(torch.int16)).view(np.uint16), orc.to_bf16_bits(eb))
    np.testing.assert_array_equal(_np(img_f.view(torch.int16)).view(np.uint16), orc.to_bf16_bits(ei))


# ------------------------------------------------------------ batched pipeline

@pytest.mark.parametrize("cfg,dual", [(2, False), (5, True)])
def test_pipeline_batch_matches_oracle(cfg, dual):
    """The bench's exact hot path (index -> CSR -> fused layer) on 3 frames."""
    from sparse_pooling_amd import pipeline
    spec = synth.CONFIGS[cfg]
    frames = [synth.make_frame(spec, seed=40 + f, n_outside=25) for f in range(3)]
    pts, vox, off, P, maxp, N = pipeline.stack_frames(frames, DEV)
    pl = pipeline.FusedPipeline(3, maxp, N, spec.im_size, spec.bv_size, spec.stride, spec.c_bev, spec.c_img,
                                dual=dual)
    Hb, Wb = spec.bev_feat_hw
    Hi, Wi = spec.img_feat_hw
    bev = synth.make_features((3, Hb, Wb, spec.c_bev), 1)
    img = synth.make_features((3, Hi, Wi, spec.c_img), 2)
    pl.step(pts, vox, off, P, torch.from_numpy(bev).to(DEV), torch.from_numpy(img).to(DEV))
    torch.cuda.synchronize()
    assert int(pl.err.item()) == 0
    out = _np(pl.bv_fused)
    iout = _np(pl.img_fused) if dual else None
    for f, fr in enumerate(frames):
        ref = _oracle_frame(fr, spec.stride)
        eb, ei = orc.sparse_pool_layer(bev[f:f + 1], img[f:f + 1], ref["Mij_pool"], ref["M_val"], ref["M_size"],
                                       ref["img_index_flip_pool"], dual=dual)
        _close_and_exact(out[f:f + 1], eb)
        if dual:
            _close_and_exact(iout[f:f + 1], ei)


@pytest.mark.parametrize("cfg,dtype,graph,once,own", [(6, "f32", False, True, True), (6, "f32", True, True, True),
                                                      (6, "bf16", False, True, True), (2, "f32", False, True, True),
                                                      (6, "f32", False, False, True), (2, "bf16", True, False, True),
                                                      (6, "f32", False, True, False), (6, "bf16", True, True, False)])
def test_split_pipeline_matches_oracle(cfg, dtype, graph, once, own, monkeypatch):
    """FusedPipeline(split=True): the pass-through copy beside the index chain, the frame CSR with key ranges
    (k_csr_frame + k_key_range) and the pooled half written once (shpl_pull_once, or the row-keyed k_rows) -- eager and captured
    in a HIP graph (two replays) -- bitwise the oracle's bv_fused on 3 frames (one with no point). own: the chain
    on a stream of its own; else on the (high-priority) stream the step is called on (chain=None)."""
    from sparse_pooling_amd import pipeline
    monkeypatch.setattr(pipeline.FusedPipeline, "SPLIT_ONCE", once)
    monkeypatch.setattr(pipeline.FusedPipeline, "SPLIT_SERIAL", False)
    _split_run(cfg, dtype, graph, own)


@pytest.mark.parametrize("cfg,dtype,graph,own", [(6, "f32", True, True), (6, "f32", False, False),
                                                 (6, "bf16", True, False), (6, "bf16", False, True),
                                                 (2, "f32", True, False)])
def test_split_serial_matches_oracle(cfg, dtype, graph, own):
    """The split layer's default form (SPLIT_SERIAL: the pooled half -- shpl_pull_once, its wave per 64
    entries at 256 channels -- after the side stream's copy instead of beside it), eager and graph-replayed,
    bitwise the oracle's bv_fused on 3 frames (one with no point)."""
    from sparse_pooling_amd import pipeline
    assert pipeline.FusedPipeline.SPLIT_SERIAL
    _split_run(cfg, dtype, graph, own)


def _split_run(cfg, dtype, graph, own):
    from sparse_pooling_amd import pipeline
    spec = synth.CONFIGS[cfg]
    frames = [synth.make_frame(spec, seed=60 + f, n_outside=25) for f in range(2)]
    frames.insert(1, synth.make_frame(synth.FrameSpec(0, spec.im_size, spec.bv_size, spec.stride, spec.c_bev,
                                                      spec.c_img), seed=1))
    pts, vox, off, P, maxp, N = pipeline.stack_frames(frames, DEV)
    dt = torch.bfloat16 if dtype == "bf16" else torch.float32
    pl = pipeline.FusedPipeline(3, maxp, N, spec.im_size, spec.bv_size, spec.stride, spec.c_bev, spec.c_img,
                                dtype=dt, split=True)
    assert pl.split and pl.csr.key_range is not None
    Hb, Wb = spec.bev_feat_hw
    Hi, Wi = spec.img_feat_hw
    bev = synth.make_features((3, Hb, Wb, spec.c_bev), 3)
    img = synth.make_features((3, Hi, Wi, spec.c_img), 4)
    if dt == torch.bfloat16:
        bev, img = (orc.from_bf16_bits(orc.to_bf16_bits(a)) for a in (bev, img))
    tb, ti = torch.from_numpy(bev).to(DEV).to(dt), torch.from_numpy(img).to(DEV).to(dt)
    side = torch.cuda.Stream(device=DEV)
    chain = torch.cuda.Stream(device=DEV, priority=-1)
    pl.bv_fused.fill_(float("nan"))  # every element must be written
    torch.cuda.synchronize()
    if graph:
        g = torch.cuda.CUDAGraph()
        gs = torch.cuda.Stream(device=DEV)
        gs.wait_stream(torch.cuda.current_stream())
        with torch.cuda.graph(g, stream=gs):
            pl.step_split(pts, vox, off, P, tb, ti, side, chain if own else None)
        pl.bv_fused.fill_(float("nan"))
        g.replay()
        g.replay()
    elif own:
        pl.step_split(pts, vox, off, P, tb, ti, side, chain)
    else:
        with torch.cuda.stream(chain):
            pl.step_split(pts, vox, off, P, tb, ti, side, None)
    torch.cuda.synchronize()
    assert int(pl.err.item()) == 0
    out = pl.bv_fused.float().cpu().numpy()
    for f, fr in enumerate(frames):
        ref = _oracle_frame(fr, spec.stride)
        eb, _ = orc.sparse_pool_layer(bev[f:f + 1], img[f:f + 1], ref["Mij_pool"], ref["M_val"], ref["M_size"],
                                      ref["img_index_flip_pool"])
        if dt == torch.bfloat16:
            eb = orc.from_bf16_bits(orc.to_bf16_bits(eb))
        _close_and_exact(out[f:f + 1], eb)


def test_full_size_properties_config5():
    """Config 5 (40k points, 64 channels, both directions) at full size:
    adjointness <pool(x), y> == <x, trans(y)> and the pass-through halves."""
    from sparse_pooling_amd import pipeline
    spec = synth.CONFIGS[5]
    frames = [synth.make_frame(spec, seed=77)]
    pts, vox, off, P, maxp, N = pipeline.stack_frames(frames, DEV)
    pl = pipeline.FusedPipeline(1, maxp, N, spec.im_size, spec.bv_size, spec.stride, spec.c_bev, spec.c_img,
                                dual=True)
    Hb, Wb = spec.bev_feat_hw
    Hi, Wi = spec.img_feat_hw
    x = torch.randn((1, Hi, Wi, spec.c_img), device=DEV)
    y = torch.randn((1, Hb, Wb, spec.c_bev), device=DEV)
    pl.step(pts, vox, off, P, y, x)
    torch.cuda.synchronize()
    pooled = pl.bv_fused[..., spec.c_bev:]
    trans = pl.img_fused[..., spec.c_img:]
    assert torch.equal(pl.bv_fused[..., :spec.c_bev], y)
    assert torch.equal(pl.img_fused[..., :spec.c_img], x)
    lhs = (pooled.double() * y.double()).sum().item()
    rhs = (x.double() * trans.double()).sum().item()
    assert abs(lhs - rhs) <= 1e-4 * max(1.0, abs(lhs))
    assert int(pl.frame_nnz.item()) == frames[0].points.shape[0] - int(
        (frames[0].voxel_indices[:, 1] >= spec.bv_size[0]).sum())


@pytest.mark.parametrize("cfg,dtype,mode,rows", [
    (1, "f32", "eager", False), (1, "bf16", "eager", False), (1, "bf16", "streams", False), (1, "f32", "graph", False),
    (3, "bf16", "eager", False), (3, "bf16", "graph", False),
    (1, "f32", "eager", True), (1, "bf16", "streams", True), (1, "f32", "graph", True),
    (3, "bf16", "eager", True), (3, "bf16", "graph", True), (3, "f32", "streams", True),
    (1, "f32", "graph", "csr"), (3, "bf16", "eager", "csr"), (3, "bf16", "graph", "csr")])
def test_pipeline_backward_matches_oracle(cfg, dtype, mode, rows):
    """FusedPipeline forward + backward (the config-3 bench step) vs the oracle's TF
    forward and gradients; mode streams/graph: the bench's step (side streams for the
    streaming half and the pixel-keyed chain), launched eagerly or replayed from a
    captured HIP graph. cfg 3 is the bench's own shape: bf16, 256 channels (32 chunks
    per pooled row, the power-of-two path), stride 8, pixel runs far longer than
    k_sparse's 8 entries (k_sparse_long with per-column partials in OUT_ADD mode).
    rows True: the index build cuts M into destination buckets and each pull pair is one
    launch over them (shpl_pull_buckets, one stream); "csr": the CSRs carry key_range and
    every pull is one row-keyed launch (k_rows)."""
    from sparse_pooling_amd import pipeline
    spec = synth.CONFIGS[cfg]
    B = 2 if cfg == 1 else 4
    frames = [synth.make_frame(spec, seed=60 + f, n_outside=10) for f in range(B)]
    refs = [_oracle_frame(fr, spec.stride) for fr in frames]
    if cfg == 3:  # the long-run path is really exercised
        runs = max(np.unique(r["img_index_flip_pool"][:, 1:], axis=0, return_counts=True)[1].max() for r in refs)
        assert runs > 16, runs
    pts, vox, off, P, maxp, N = pipeline.stack_frames(frames, DEV)
    tdt = torch.float32 if dtype == "f32" else torch.bfloat16
    pl = pipeline.FusedPipeline(B, maxp, N, spec.im_size, spec.bv_size, spec.stride, spec.c_bev, spec.c_img,
                                dtype=tdt, dual=True, rows=bool(rows), buckets=rows is True)
    assert pl.buckets == (rows is True)
    Hb, Wb = spec.bev_feat_hw
    Hi, Wi = spec.img_feat_hw
    Cb, Ci = spec.c_bev, spec.c_img

    def mk(shape, seed):
        x = synth.make_features(shape, seed)
        if dtype == "bf16":
            x = orc.from_bf16_bits(orc.to_bf16_bits(x)).reshape(shape)
        return x, torch.from_numpy(x).to(DEV).to(tdt)
    bev, tb = mk((B, Hb, Wb, Cb), 1)
    img, ti = mk((B, Hi, Wi, Ci), 2)
    gb, tgb = mk((B, Hb, Wb, Cb + Ci), 3)
    gi, tgi = mk((B, Hi, Wi, Ci + Cb), 4)
    d_bev, d_img = torch.empty_like(tb), torch.empty_like(ti)
    if mode == "eager":
        pl.step(pts, vox, off, P, tb, ti)
        pl.backward(tgb, tgi, d_bev, d_img)
    else:
        side, side2 = torch.cuda.Stream(), torch.cuda.Stream()

        def step():
            pl.step_overlapped(pts, vox, off, P, tb, ti, side, side2=side2)
            pl.backward(tgb, tgi, d_bev, d_img, side2=side2)
        step()
        if mode == "graph":
            torch.cuda.synchronize()
            for t in (pl.bv_fused, pl.img_fused, d_bev, d_img):
                t.fill_(float("nan"))
            g = torch.cuda.CUDAGraph()
            gs = torch.cuda.Stream()
            gs.wait_stream(torch.cuda.current_stream())
            with torch.cuda.graph(g, stream=gs):
                step()
            g.replay()
            g.replay()
    torch.cuda.synchronize()
    if pl.buckets:  # the one-launch index build's frame barrier words: zero again after every call, no timeout
        assert int(pl.err.item()) == 0
        assert not pl.bkt_ws[:8 * B].view(torch.int32).any()

    def same(got, want):
        if dtype == "f32":
            _close_and_exact(got, want)
        else:
            np.testing.assert_array_equal(_np(got.view(torch.int16)).view(np.uint16),
                                          orc.to_bf16_bits(want.astype(np.float32)))
    for f, ref in enumerate(refs):
        mij, mval, msize, idx = ref["Mij_pool"], ref["M_val"], ref["M_size"], ref["img_index_flip_pool"]
        eb, ei = orc.sparse_pool_layer(bev[f:f + 1], img[f:f + 1], mij, mval, msize, idx, dual=True)
        same(pl.bv_fused[f:f + 1], eb)
        same(pl.img_fused[f:f + 1], ei)
        e_img = gi[f:f + 1, ..., :Ci] + orc.sparse_pool_grad_img(
            mij, mval, msize, gb[f, ..., Cb:].reshape(-1, Ci), idx, (1, Hi, Wi, Ci))
        e_bev = gb[f:f + 1, ..., :Cb] + orc.sparse_pool_trans_grad_bev(
            mij, mval, msize, np.ascontiguousarray(gi[f:f + 1, ..., Ci:]), idx).reshape(1, Hb, Wb, Cb)
        same(d_img[f:f + 1], e_img)
        same(d_bev[f:f + 1], e_bev)


def test_index1_barrier_give_up_and_dirty_words():
    """k_index1's frame barrier (the one-launch bucketed index build at config 3's shape) fails loudly,
    never silently: (1) a bucket workspace whose barrier words were never zeroed (0xFF) -> FusedPipeline.check()
    raises RuntimeError and resets them, and the next step is bitwise the oracle's; (2) the fault-injection
    build (libshpl_fault.so: SHPL_IDX1_FAULT, chunk 0 of frame 0 never arrives) -> every chunk of frame 0 gives
    up after 20 ms, check() raises RuntimeError, and the call still leaves the words zero."""
    import ctypes

    from sparse_pooling_amd import _lib as L
    from sparse_pooling_amd import build as B_
    from sparse_pooling_amd import pipeline
    assert os.path.exists(B_.FAULT_OUT), "build the test library: python -m sparse_pooling_amd.build"
    spec = synth.CONFIGS[3]
    B = 4
    frames = [synth.make_frame(spec, seed=90 + f, n_outside=10) for f in range(B)]
    pts, vox, off, P, maxp, N = pipeline.stack_frames(frames, DEV)
    pl = pipeline.FusedPipeline(B, maxp, N, spec.im_size, spec.bv_size, spec.stride, spec.c_bev, spec.c_img,
                                dtype=torch.bfloat16, dual=True)
    assert pl.buckets
    Hb, Wb = spec.bev_feat_hw
    Hi, Wi = spec.img_feat_hw
    tb = torch.randn((B, Hb, Wb, spec.c_bev), device=DEV).to(torch.bfloat16)
    ti = torch.randn((B, Hi, Wi, spec.c_img), device=DEV).to(torch.bfloat16)

    def clean_step_matches_oracle():
        pl.step(pts, vox, off, P, tb, ti)
        pl.check()  # no bit set
        assert not pl.bkt_ws[:8 * B].view(torch.int32).any()
        bev, img = tb[:1].float().cpu().numpy(), ti[:1].float().cpu().numpy()
        ref = _oracle_frame(frames[0], spec.stride)
        eb, ei = orc.sparse_pool_layer(bev, img, ref["Mij_pool"], ref["M_val"], ref["M_size"],
                                       ref["img_index_flip_pool"], dual=True)
        for got, want in ((pl.bv_fused[:1], eb), (pl.img_fused[:1], ei)):
            np.testing.assert_array_equal(_np(got.view(torch.int16)).view(np.uint16),
                                          orc.to_bf16_bits(want.astype(np.float32)))

    # (1) dirty barrier words
    pl.bkt_ws.fill_(0xFF)
    pl.step(pts, vox, off, P, tb, ti)
    with pytest.raises(RuntimeError, match="frame barrier"):
        pl.check()
    assert int(pl.err.item()) == 0 and not pl.bkt_ws[:8 * B].view(torch.int32).any()  # check() reset both
    clean_step_matches_oracle()
    # (2) the give-up, forced
    fault = ctypes.CDLL(B_.FAULT_OUT)
    L._declare(fault)
    pl._lib = fault
    try:
        pl.step(pts, vox, off, P, tb, ti)
        torch.cuda.synchronize()
        assert not pl.bkt_ws[:8 * B].view(torch.int32).any()  # the timed-out call left them zero too
        with pytest.raises(RuntimeError, match="frame barrier"):
            pl.check()
    finally:
        pl._lib = L.lib()
    clean_step_matches_oracle()


@pytest.mark.parametrize("dtype,cb,ci,sizes", [("bf16", 256, 256, [1500, 1500, 700]), ("f32", 128, 128, [1500, 900]),
                                               ("bf16", 256, 256, [0, 3000, 1, 5]), ("bf16", 256, 128, [2500, 2500])])
def test_window_pulls_short_stretches(dtype, cb, ci, sizes):
    """The bucketed step's pull pairs at config 3's row width (32 chunks of 16 bytes: bf16 256 / f32 128
    channels, the entry-window form k_win2 when the library has it) on batches so small that every workgroup
    owns one or two 32-entry windows: pixel runs of up to ~50 entries cross several workgroups' stretches (the
    run's owner fetches past its stretch; the others skip it), frames without entries, and (256 / 128) one side
    of another row width (k_rows2 then) -- bitwise against the oracle, forward and gradients."""
    _ragged_pipeline_run(3, sizes, dtype, ["buckets"], channels=(cb, ci))


# ---------------------------------------------------------------- BEV voxelizer

def _ragged_frames(base, sizes, seed):
    """Frames of the given inside-point counts: 0 = no points at all, negative =
    -n points that all fall outside the image (no survivor)."""
    frames = []
    for f, n in enumerate(sizes):
        if n == 0:
            frames.append(synth.Frame(np.zeros((0, 3)), np.zeros((0, 2), dtype=np.int64), synth.KITTI_P2,
                                      synth.FrameSpec(0, base.im_size, base.bv_size, base.stride, base.c_bev,
                                                      base.c_img)))
            continue
        spec = synth.FrameSpec(max(n, 0), base.im_size, base.bv_size, base.stride, base.c_bev, base.c_img)
        frames.append(synth.make_frame(spec, seed=seed + f, n_outside=-n if n < 0 else 13 * f))
    return frames


def _ragged_pipeline_run(cfg, sizes, dtype, paths, channels=None, frames=None):
    """FusedPipeline forward + backward over a ragged batch, once per CSR path
    (shpl_build_csr_path: frame / segment / range; None = the default; "buckets": the
    index build's destination buckets, both CSRs in one launch (shpl_build_csr_buckets) and
    the one-launch pull pairs (shpl_pull_pair); "csr_rows": range CSRs + k_rows), each
    compared with the oracle frame by frame
    (f32: bitwise; bf16: bitwise on the bf16 bits). channels: (Cb, Ci) instead of the config's."""
    from sparse_pooling_amd import _lib as L
    from sparse_pooling_amd import pipeline
    base = synth.CONFIGS[cfg]
    if channels is not None:
        base = synth.FrameSpec(base.n_points, base.im_size, base.bv_size, base.stride, *channels)
    frames = _ragged_frames(base, sizes, 500) if frames is None else frames
    refs = [_oracle_frame(fr, base.stride) for fr in frames]
    B = len(frames)
    pts, vox, off, P, maxp, N = pipeline.stack_frames(frames, DEV)
    tdt = torch.float32 if dtype == "f32" else torch.bfloat16
    Hb, Wb = base.bev_feat_hw
    Hi, Wi = base.img_feat_hw
    Cb, Ci = base.c_bev, base.c_img

    def mk(shape, seed):
        x = synth.make_features(shape, seed)
        if dtype == "bf16":
            x = orc.from_bf16_bits(orc.to_bf16_bits(x)).reshape(shape)
        return x, torch.from_numpy(x).to(DEV).to(tdt)
    bev, tb = mk((B, Hb, Wb, Cb), 1)
    img, ti = mk((B, Hi, Wi, Ci), 2)
    gb, tgb = mk((B, Hb, Wb, Cb + Ci), 3)
    gi, tgi = mk((B, Hi, Wi, Ci + Cb), 4)
    want = []
    for f, ref in enumerate(refs):
        mij, mval, msize, idx = ref["Mij_pool"], ref["M_val"], ref["M_size"], ref["img_index_flip_pool"]
        eb, ei = orc.sparse_pool_layer(bev[f:f + 1], img[f:f + 1], mij, mval, msize, idx, dual=True)
        e_img = gi[f:f + 1, ..., :Ci] + orc.sparse_pool_grad_img(
            mij, mval, msize, gb[f, ..., Cb:].reshape(-1, Ci), idx, (1, Hi, Wi, Ci))
        e_bev = gb[f:f + 1, ..., :Cb] + orc.sparse_pool_trans_grad_bev(
            mij, mval, msize, np.ascontiguousarray(gi[f:f + 1, ..., Ci:]), idx).reshape(1, Hb, Wb, Cb)
        want.append((eb, ei, e_bev, e_img))

    def same(got, exp):
        if dtype == "f32":
            _close_and_exact(got, exp)
        else:
            np.testing.assert_array_equal(_np(got.view(torch.int16)).view(np.uint16),
                                          orc.to_bf16_bits(exp.astype(np.float32)))
    codes = {None: L.CSR_AUTO, "frame": L.CSR_FRAME, "segment": L.CSR_SEGMENT, "range": L.CSR_RANGE}
    for path in paths:
        # a named CSR builder: the CSR pulls (no buckets); None: the pipeline's default
        # "buckets_hK": the bucketed step with K run heads per destination in its CSRs (shpl_csr.heads)
        kw = {"buckets": dict(rows=True, buckets=True),
              "csr_rows": dict(rows=True, buckets=False), None: {}}.get(
                  path, dict(rows=True, buckets=True) if path and path.startswith("buckets_h") else dict(buckets=False))
        head_k = pipeline.FusedPipeline.HEAD_K
        if path and path.startswith("buckets_h"):
            pipeline.FusedPipeline.HEAD_K = int(path[len("buckets_h"):])
        try:
            pl = pipeline.FusedPipeline(B, maxp, N, base.im_size, base.bv_size, base.stride, Cb, Ci, dtype=tdt,
                                        dual=True, **kw)
        finally:
            pipeline.FusedPipeline.HEAD_K = head_k
        if path is not None:
            assert pl.buckets == path.startswith("buckets")
        pl.csr_path = codes.get(path, L.CSR_AUTO)
        d_bev, d_img = torch.empty_like(tb), torch.empty_like(ti)
        pl.step(pts, vox, off, P, tb, ti)
        pl.backward(tgb, tgi, d_bev, d_img)
        torch.cuda.synchronize()
        assert int(pl.err.item()) == 0
        nnz = _np(pl.frame_nnz)
        for f, (eb, ei, e_bev, e_img) in enumerate(want):
            assert nnz[f] == refs[f]["M_size"][1], (path, f)
            same(pl.bv_fused[f:f + 1], eb)
            same(pl.img_fused[f:f + 1], ei)
            same(d_bev[f:f + 1], e_bev)
            same(d_img[f:f + 1], e_img)
        del pl


@pytest.mark.parametrize("dtype,cb,ci", [("bf16", 256, 256), ("f32", 256, 256), ("f32", 16, 32), ("bf16", 64, 64),
                                         ("f32", 3, 5), ("bf16", 8, 24), ("f32", 64, 128), ("f32", 4, 6)])
def test_bucket_pulls_ragged_batch(dtype, cb, ci):
    """The bucketed step (shpl_build_index_buckets -> shpl_build_csr_buckets -> shpl_pull_pair:
    both CSRs in one launch, both pulls in one launch (k_rows2), forward then gradients) at config 3's
    geometry over a ragged batch -- no points,
    one point, no survivor, one survivor among 14 points (the dgemv projection order: no
    bucket, the entry read from the index arrays), chunk-straddling and full frames --
    bitwise against the oracle and against the range CSR + k_rows path, for every lane
    group width (G = 8 .. 64) and the unvectorised form (3 / 5 and 4 / 6 f32 channels); with the default
    run heads (shpl_csr.heads), none and one per destination."""
    _ragged_pipeline_run(3, [0, 1, -40, 1025, 20000, 2], dtype, ["buckets", "csr_rows", "buckets_h0", "buckets_h1"],
                         channels=(cb, ci))


def test_bucket_pulls_long_runs():
    """One frame whose 3000 points are one point repeated (one cell, one pixel: one bucket, one
    run of 3000 entries, sorted in 12 rounds) beside a frame with half its points on one cell:
    bitwise against the oracle, f32 and bf16, with the default run heads, 32 (more than some lane groups
    hold) and none."""
    base = synth.CONFIGS[3]
    rng = np.random.default_rng(9)
    one = synth.make_frame(synth.FrameSpec(1, base.im_size, base.bv_size, base.stride, 32, 32), seed=3)
    pts = np.repeat(one.points, 3000, axis=0)
    vox = np.repeat(one.voxel_indices, 3000, axis=0)
    heavy = synth.Frame(pts, vox, synth.KITTI_P2, base)
    mixed = synth.make_frame(synth.FrameSpec(4000, base.im_size, base.bv_size, base.stride, 32, 32), seed=4)
    half = mixed.points.shape[0] // 2  # half of a frame's points on one cell too (a long run among others)
    mixed.voxel_indices[:half] = mixed.voxel_indices[0]
    frames = [heavy, synth.make_frame(synth.FrameSpec(3000, base.im_size, base.bv_size, base.stride, 32, 32),
                                      seed=5, n_outside=int(rng.integers(1, 50))), mixed]
    for dtype in ("f32", "bf16"):
        _ragged_pipeline_run(3, None, dtype, ["buckets", "buckets_h32", "buckets_h0"], channels=(32, 32),
                             frames=frames)


def test_pipeline_ragged_batch_every_csr_path():
    """Empty and ragged inputs through the whole batched path (index -> both CSRs
    -> dual layer -> both gradients) at config-2 shape: a frame without points,
    a one-point frame, a frame whose points all fall outside the image, frames
    straddling the index builder's chunks -- under each CSR builder (per-frame
    workgroup, segments, destination ranges), bitwise against the oracle."""
    _ragged_pipeline_run(2, [0, 1, -40, 1025, 20000, 2], "f32", ["frame", "segment", "range"])


def test_pipeline_ragged_batch_row_keyed_bf16():
    """The same ragged batch at config-3 shape (bf16, 256 channels): the default
    (bucketed pulls) and the row-keyed pulls over key_range CSRs, bitwise on the bf16 bits."""
    _ragged_pipeline_run(3, [0, 1, -40, 1025, 20000, 2], "bf16", [None, "range"])


def test_bev_slices_vs_reference_golden():
    from sparse_pooling_amd import bev
    g = np.load(os.path.join(GOLD, "bev_slices.npz"))
    import types
    cfg = types.SimpleNamespace(height_lo=float(g["height_lo"]), height_hi=float(g["height_hi"]),
                                num_slices=int(g["num_slices"]))
    maps, vox, upts = bev.BevSlices(cfg).generate_bev("lidar", g["point_cloud"], g["ground_plane"],
                                                      g["area_extents"], float(g["voxel_size"]),
                                                      output_indices=True)
    np.testing.assert_array_equal(_np(vox), g["voxel_indices"])
    np.testing.assert_array_equal(_np(upts), g["pts_in_voxel"])
    np.testing.assert_array_equal(np.stack([_np(m) for m in maps["height_maps"]]), g["height_maps"])
    np.testing.assert_array_equal(_np(maps["density_map"]), g["density_map"])


def test_bev_slices_batch_vs_oracle():
    from sparse_pooling_amd import bev
    clouds = [synth.make_cloud(15000 + 3000 * f, seed=200 + f) for f in range(3)]
    planes = [synth.GROUND_PLANE + np.array([0.01 * f, 0, -0.005 * f, 0.02 * f]) for f in range(3)]
    pts = torch.from_numpy(np.concatenate([c.T for c in clouds])).to(DEV)
    off = torch.tensor(np.concatenate([[0], np.cumsum([c.shape[1] for c in clouds])]), device=DEV)
    pl = torch.from_numpy(np.stack(planes)).to(DEV)
    b = bev.bev_slices_batch(pts, off, pl, synth.AREA_EXTENTS, synth.VOXEL_SIZE, synth.HEIGHT_LO,
                             synth.HEIGHT_HI, synth.NUM_SLICES)
    torch.cuda.synchronize()
    o, n = _np(off), _np(b.frame_nvox)
    for f, c in enumerate(clouds):
        hm, dm, vox, upts = orc.bev_slices(c, planes[f], synth.AREA_EXTENTS, synth.VOXEL_SIZE, synth.HEIGHT_LO,
                                           synth.HEIGHT_HI, synth.NUM_SLICES)
        a = o[f]
        np.testing.assert_array_equal(_np(b.voxel_indices[a:a + n[f]]), vox)
        np.testing.assert_array_equal(_np(b.pts_in_voxel[a:a + n[f]]), upts)
        np.testing.assert_array_equal(_np(b.height_maps[f]), hm)
        np.testing.assert_array_equal(_np(b.density_map[f]), dm)
    assert int(b.err.item()) == 0
    # the network's BEV input (shpl_bev_input): kitti_dataset.py:368's dstack of the maps, as its tf.float32
    # placeholder holds it (one rounding), bitwise
    S = synth.NUM_SLICES
    bin_ = b.write_bev_input(torch.full((3,) + tuple(b.density_map.shape[1:]) + (S + 1,), float("nan"),
                                        dtype=torch.float32, device=DEV))
    torch.cuda.synchronize()
    for f in range(3):
        want = np.dstack((*_np(b.height_maps[f]), _np(b.density_map[f]))).astype(np.float32)
        np.testing.assert_array_equal(_np(bin_[f]).view(np.uint32), want.view(np.uint32))
    # output tensors of the wrong shape / dtype / layout are refused before any device write
    nz, nx = b.density_map.shape[1:]
    f64 = dict(dtype=torch.float64, device=DEV)
    for hm, dm in [(torch.empty((3, S, nz, nx - 1), **f64), torch.empty((3, nz, nx), **f64)),
                   (torch.empty((3, S, nz, nx), **f64), torch.empty((3, nz, nx), dtype=torch.float32, device=DEV)),
                   (torch.empty((3, S, nx, nz), **f64).transpose(2, 3), torch.empty((3, nz, nx), **f64))]:
        with pytest.raises(ValueError):
            b.write_maps(hm, dm)
    with pytest.raises(ValueError):
        b.write_bev_input(torch.empty((3, nz, nx, S), dtype=torch.float32, device=DEV))


def test_bev_slices_more_frames_than_map_table():
    """shpl_bev_slices over more frames than shpl_bev_maps can read back (4096): the voxelizer and its own
    maps work (the round-3 API regression fixed), only the deferred maps call refuses the batch."""
    from sparse_pooling_amd import bev
    F = 4100
    cloud = synth.make_cloud(64, seed=7)
    pts = torch.from_numpy(np.ascontiguousarray(np.tile(cloud.T, (F, 1)))).to(DEV)
    off = torch.arange(F + 1, dtype=torch.int64, device=DEV) * cloud.shape[1]
    pl = torch.from_numpy(np.tile(synth.GROUND_PLANE, (F, 1))).to(DEV)
    b = bev.bev_slices_batch(pts, off, pl, synth.AREA_EXTENTS, synth.VOXEL_SIZE, synth.HEIGHT_LO,
                             synth.HEIGHT_HI, synth.NUM_SLICES, maps=False)  # 4100 frames of maps: 92 GB
    torch.cuda.synchronize()
    hm, dm, vox, upts = orc.bev_slices(cloud, synth.GROUND_PLANE, synth.AREA_EXTENTS, synth.VOXEL_SIZE,
                                       synth.HEIGHT_LO, synth.HEIGHT_HI, synth.NUM_SLICES)
    n = _np(b.frame_nvox)
    assert (n == vox.shape[0]).all() and int(b.err.item()) == 0
    for f in (0, F // 2, F - 1):
        a = f * cloud.shape[1]
        np.testing.assert_array_equal(_np(b.voxel_indices[a:a + n[f]]), vox)
        np.testing.assert_array_equal(_np(b.pts_in_voxel[a:a + n[f]]), upts)
    from sparse_pooling_amd import _lib as L
    with pytest.raises(L.ShplLibraryError, match="shpl_bev_maps"):
        b.write_maps(None, None)  # the deferred maps call: SHPL_ERR_BAD_SHAPE


def test_points_to_fused_layer_pipeline():
    """Raw clouds -> device BEV voxelizer -> index builder -> sorted M -> fused
    layer, against the oracle chain (bev_slices -> gen -> produce -> pool)."""
    from sparse_pooling_amd import pipeline
    F = 2
    clouds = [synth.make_cloud(30000, seed=300 + f) for f in range(F)]
    planes = np.stack([synth.GROUND_PLANE] * F)
    Ps = [synth.KITTI_P2, synth.KITTI_P2 + np.array([[0.5, 0, 1.0, 0], [0, 0.5, -1.0, 0], [0, 0, 0, 0]])]
    im_size, stride, C = (1242, 375), (4, 4), 8
    pts = torch.from_numpy(np.concatenate([c.T for c in clouds])).to(DEV)
    off = torch.tensor(np.concatenate([[0], np.cumsum([c.shape[1] for c in clouds])]), device=DEV)
    pl = pipeline.FramePipeline(F, int(pts.shape[0]), im_size, synth.AREA_EXTENTS, synth.VOXEL_SIZE,
                                synth.HEIGHT_LO, synth.HEIGHT_HI, synth.NUM_SLICES, stride, C, C, dual=True)
    bev = synth.make_features((F, pl.Hb, pl.Wb, C), 1)
    img = synth.make_features((F, pl.Hi, pl.Wi, C), 2)
    pl.frame_step(pts, off, torch.from_numpy(planes).to(DEV), torch.from_numpy(np.stack([p.reshape(12) for p in Ps])).to(DEV),
                  torch.from_numpy(bev).to(DEV), torch.from_numpy(img).to(DEV))
    torch.cuda.synchronize()
    assert int(pl.err.item()) == 0
    out, iout = _np(pl.bv_fused), _np(pl.img_fused)
    for f, c in enumerate(clouds):
        hm, dm, vox, upts = orc.bev_slices(c, planes[f], synth.AREA_EXTENTS, synth.VOXEL_SIZE, synth.HEIGHT_LO,
                                           synth.HEIGHT_HI, synth.NUM_SLICES)
        g = orc.gen_sparse_pooling_input_avod(upts, vox, Ps[f], list(im_size), (hm.shape[1], hm.shape[2]))
        ref = orc.produce_sparse_pooling_input(g, stride=stride)
        assert int(_np(pl.frame_nnz)[f]) == ref["Mij_pool"].shape[0]
        eb, ei = orc.sparse_pool_layer(bev[f:f + 1], img[f:f + 1], ref["Mij_pool"], ref["M_val"], ref["M_size"],
                                       ref["img_index_flip_pool"], dual=True)
        _close_and_exact(out[f:f + 1], eb)
        _close_and_exact(iout[f:f + 1], ei)


# ---------------------------------------------------------------- MV3D producer

@pytest.mark.parametrize("name", ["mv3d_voxel.npz", "mv3d_voxel_dense.npz"])
def test_mv3d_producer_vs_reference_golden(name):
    from sparse_pooling_amd import mv3d
    g = np.load(os.path.join(GOLD, name))
    img, bv, mv = mv3d.mv3d_sparse_pooling_input(g["points"], img_index2=g["img_index2"])
    np.testing.assert_array_equal(_np(img), g["img_index"])
    np.testing.assert_array_equal(_np(bv), g["bv_index"])
    np.testing.assert_array_equal(_np(mv), g["M_val"])
    # projecting on the device gives the same img_index2
    img_p, _, _ = mv3d.mv3d_sparse_pooling_input(g["points"], P=synth.KITTI_P2)
    np.testing.assert_array_equal(_np(img_p), g["img_index"])


def test_mv3d_chain_to_pooling():
    """MV3D: device producer -> produce_sparse_pooling_input(stride [8,2]) with
    M_val = 1/count -> sparse_pool (network.py:243-246) vs the oracle chain,
    on image-visible points (MV3D's minibatches are FOV-filtered) with
    clustered voxels over the 45-point cap."""
    from sparse_pooling_amd import mv3d
    from sparse_pooling_amd.sparse_pool_utils import SparseTensor
    fr = synth.make_frame(synth.FrameSpec(8000, (1280, 384), (200, 240)), seed=9)
    rng = np.random.default_rng(9)
    pts = np.concatenate([fr.points, rng.uniform(0, 1, (len(fr.points), 1))], axis=1)
    pts[:3000, :3] = pts[rng.integers(0, 40, 3000), :3] + rng.normal(0, 0.05, (3000, 3))
    uvw = synth.KITTI_P2 @ np.vstack((pts[:, :3].T, np.ones(len(pts))))
    img2 = np.round(uvw[:2] / uvw[2]).astype(np.int64)
    img2 = np.clip(img2, 0, [[1279], [383]])
    img, bv, mv = mv3d.mv3d_sparse_pooling_input(pts, img_index2=img2)
    e_img, e_bv, e_mv, _ = orc.mv3d_voxels(pts, img2, **orc.MV3D_PED)
    np.testing.assert_array_equal(_np(img), e_img)
    np.testing.assert_array_equal(_np(mv), e_mv)
    assert (e_mv < 1).any()
    Mij, M_val, M_size, flip = mv3d.produce_sparse_pooling_input(img.clone(), np.array([1280, 384]), bv, [200, 240],
                                                                 M_val=mv, stride=[8, 2])
    ref = orc.produce_sparse_pooling_input({"img_index": e_img.copy(), "bv_index": e_bv,
                                            "img_size": np.array([1280, 384]), "bv_size": np.array([200, 240])},
                                           M_val=e_mv, stride=(8, 2))
    np.testing.assert_array_equal(_np(Mij), ref["Mij_pool"])
    np.testing.assert_array_equal(_np(flip), ref["img_index_flip_pool"])
    feat = synth.make_features((1, 48, 160, 8), 5)
    out = mv3d.sparse_pool([SparseTensor(Mij, M_val, M_size), torch.from_numpy(feat).to(DEV), flip],
                           [1, 100, 120, 8])
    e = orc.sparse_pool_op(ref["Mij_pool"], ref["M_val"], ref["M_size"], feat, ref["img_index_flip_pool"])
    _close_and_exact(out, e.reshape(1, 100, 120, 8))


def test_mv3d_augment_fv_index_transform():
    """augment_fv's img_index transform (minibatch_mv3d_img.py:205-206) fused into the producer."""
    from sparse_pooling_amd import mv3d
    g = np.load(os.path.join(GOLD, "mv3d_voxel.npz"))
    for ratio, sx, sy in ((1.0312, 3.7, 8.25), (0.9514, 0.0, 9.99)):
        img, _, _ = mv3d.mv3d_sparse_pooling_input(g["points"], img_index2=g["img_index2"], fv_aug=(ratio, sx, sy))
        np.testing.assert_array_equal(_np(img), orc.augment_fv_index(g["img_index"], ratio, sx, sy))


# ---------------------------------------------------------------- KITTI loader (§8f item 3)

def test_kitti_loader_vs_reference_golden(kitti_dir):
    """get_lidar_point_cloud from the KITTI files, transform + FOV filter on the device."""
    from sparse_pooling_amd import kitti
    d, g = kitti_dir
    for idx in (7, 8):
        h, w = g[f"{idx}_image_shape"]
        pc = kitti.get_lidar_point_cloud(idx, os.path.join(d, "calib"), os.path.join(d, "velodyne"), im_size=[w, h])
        np.testing.assert_array_equal(_np(pc), g[f"{idx}_point_cloud"])
        pa = kitti.get_lidar_point_cloud(idx, os.path.join(d, "calib"), os.path.join(d, "velodyne"))
        np.testing.assert_array_equal(_np(pa), g[f"{idx}_point_cloud_all"])
    fr = kitti.KittiFrames.from_dirs(os.path.join(d, "calib"), os.path.join(d, "velodyne"), os.path.join(d, "planes"),
                           [7, 8, 7], [tuple(g["7_image_shape"]), tuple(g["8_image_shape"]),
                                       tuple(g["7_image_shape"])], flips=[False, True, True])
    b = fr.point_clouds()
    torch.cuda.synchronize()
    off, n = _np(fr.point_offsets), _np(b.counts)
    want = [g["7_point_cloud"], g["8_flip_point_cloud"], g["7_flip_point_cloud"]]
    for f in range(3):
        np.testing.assert_array_equal(_np(b.points[off[f]:off[f] + n[f]]).T, want[f])
        assert np.isnan(_np(b.points[off[f] + n[f]:off[f + 1]])).all()
    np.testing.assert_array_equal(_np(fr.planes[1]), g["8_flip_ground_plane"])
    np.testing.assert_array_equal(_np(fr.P2[1]), g["8_flip_p2"])


def test_kitti_loader_batch_vs_oracle():
    """Scans of ragged sizes across the 4096-point chunks, the intensity filter, flips."""
    from sparse_pooling_amd import kitti
    mg = synth
    rng = np.random.default_rng(5)
    sizes = [4097, 1, 0, 12000, 4096, 30000]
    scans = [mg.synthetic_scan(rng, n) if n else np.zeros((0, 4), np.float32) for n in sizes]
    fc = kitti.FrameCalibrationData()
    fc.r0_rect = np.array(mg.KITTI_CALIB["R0_rect"]).reshape(3, 3)
    fc.tr_velodyne_to_cam = np.array(mg.KITTI_CALIB["Tr_velo_to_cam"]).reshape(3, 4)
    rect = kitti.rect_matrix(fc)
    P = np.array(mg.KITTI_CALIB["P2"]).reshape(3, 4)
    flips = [0, 1, 0, 1, 0, 0]
    off = np.concatenate([[0], np.cumsum(sizes)]).astype(np.int64)
    xyzi = torch.from_numpy(np.concatenate(scans)).to(DEV)
    for mi in (None, 0.35):
        b = kitti.velo_to_cam_batch(xyzi, torch.from_numpy(off).to(DEV), np.stack([rect] * 6), np.stack([P] * 6),
                                    [[1242, 375]] * 6, min_intensity=mi, flip=flips)
        torch.cuda.synchronize()
        n = _np(b.counts)
        for f in range(6):
            e = orc.velo_to_cam(scans[f], rect, P, [1242, 375], min_intensity=mi, flip=flips[f])
            np.testing.assert_array_equal(_np(b.points[off[f]:off[f] + n[f]]).T, e)
        assert int(b.err.item()) == 0


def test_kitti_loader_single_column_vs_reference_golden(golden_dir):
    """One-point scan / one point in front of the camera: numpy's products have one
    column there (OpenBLAS dgemv's order), reproduced on the device, in a batch with
    an ordinary scan."""
    from sparse_pooling_amd import kitti
    g = np.load(os.path.join(golden_dir, "kitti_single.npz"))
    h, w = g["image_shape"]
    fc = kitti.FrameCalibrationData()
    fc.r0_rect, fc.tr_velodyne_to_cam = g["0_r0_rect"], g["0_tr"]
    rect = kitti.rect_matrix(fc)
    big = synth.synthetic_scan(np.random.default_rng(3), 5000)
    scans = [g["0_velo"], big, g["1_velo"]]
    off = np.concatenate([[0], np.cumsum([len(x) for x in scans])]).astype(np.int64)
    xyzi = torch.from_numpy(np.concatenate(scans)).to(DEV)
    for filt in (True, False):
        b = kitti.velo_to_cam_batch(xyzi, torch.from_numpy(off).to(DEV), np.stack([rect] * 3),
                                    np.stack([g["0_p2"]] * 3) if filt else None, [[w, h]] * 3 if filt else None)
        torch.cuda.synchronize()
        n = _np(b.counts)
        key = "point_cloud" if filt else "point_cloud_all"
        for f, want in ((0, g[f"0_{key}"]), (2, g[f"1_{key}"])):
            np.testing.assert_array_equal(_np(b.points[off[f]:off[f] + n[f]]).T, want)
        e = orc.velo_to_cam(big, rect, g["0_p2"] if filt else None, [w, h] if filt else None)
        np.testing.assert_array_equal(_np(b.points[off[1]:off[1] + n[1]]).T, e)


def test_mv3d_one_point_frame_projects_like_numpy():
    """MV3D with img_index2 projected on the device: a one-point frame is np.dot with
    one column (dgemv's order), as minibatch_mv3d_img.py:88-90 computes it."""
    from sparse_pooling_amd import mv3d
    t = np.load(os.path.join(GOLD, "index_single_tie.npz"))
    pts = np.array([[*t["points"][0], 0.5]])
    mat = np.vstack((pts[:, :3].T, np.ones((1, 1))))
    uvw = np.dot(synth.KITTI_P2, mat)          # the reference's projectToImage, one column
    want = np.round(uvw[:2] / uvw[2]).astype(np.int64)
    img_p, bv, _ = mv3d.mv3d_sparse_pooling_input(pts, P=synth.KITTI_P2)
    img_r, _, _ = mv3d.mv3d_sparse_pooling_input(pts, img_index2=want)
    assert _np(bv).shape[0] == 1
    np.testing.assert_array_equal(_np(img_p), _np(img_r))


def test_velodyne_to_fused_layer_pipeline(kitti_dir):
    """KITTI files -> device velodyne loader -> BEV slices -> index -> sorted M -> fused
    layer (kitti_dataset.py:285-379), against the oracle chain."""
    from sparse_pooling_amd import kitti, pipeline
    d, g = kitti_dir
    shapes = [tuple(g["7_image_shape"]), tuple(g["8_image_shape"])]
    fr = kitti.KittiFrames.from_dirs(os.path.join(d, "calib"), os.path.join(d, "velodyne"), os.path.join(d, "planes"),
                           [7, 8], shapes, flips=[False, True])
    im_size, stride, C = (1242, 375), (4, 4), 8
    pl = pipeline.FramePipeline(2, fr.total_points, im_size, synth.AREA_EXTENTS, synth.VOXEL_SIZE,
                                synth.HEIGHT_LO, synth.HEIGHT_HI, synth.NUM_SLICES, stride, C, C, dual=True,
                                max_points_per_frame=fr.max_points)
    bev = synth.make_features((2, pl.Hb, pl.Wb, C), 3)
    img = synth.make_features((2, pl.Hi, pl.Wi, C), 4)
    pl.velo_step(fr, torch.from_numpy(bev).to(DEV), torch.from_numpy(img).to(DEV))
    torch.cuda.synchronize()
    assert int(pl.err.item()) == 0 and int(pl.bev.err.item()) == 0
    out, iout = _np(pl.bv_fused), _np(pl.img_fused)
    clouds = [g["7_point_cloud"], g["8_flip_point_cloud"]]
    planes = [g["7_ground_plane"], g["8_flip_ground_plane"]]
    Ps = [g["7_p2"], g["8_flip_p2"]]
    for f in range(2):
        hm, dm, vox, upts = orc.bev_slices(clouds[f], planes[f], synth.AREA_EXTENTS, synth.VOXEL_SIZE,
                                           synth.HEIGHT_LO, synth.HEIGHT_HI, synth.NUM_SLICES)
        np.testing.assert_array_equal(_np(pl.bev.height_maps[f]), hm)
        gi = orc.gen_sparse_pooling_input_avod(upts, vox, Ps[f], list(im_size), (hm.shape[1], hm.shape[2]))
        ref = orc.produce_sparse_pooling_input(gi, stride=stride)
        assert int(_np(pl.frame_nnz)[f]) == ref["Mij_pool"].shape[0] > 0
        eb, ei = orc.sparse_pool_layer(bev[f:f + 1], img[f:f + 1], ref["Mij_pool"], ref["M_val"], ref["M_size"],
                                       ref["img_index_flip_pool"], dual=True)
        _close_and_exact(out[f:f + 1], eb)
        _close_and_exact(iout[f:f + 1], ei)


@pytest.mark.parametrize("form", ["f64", "bev_input"])
def test_velodyne_pipeline_overlapped_maps_equal_sequential(kitti_dir, form):
    """velo_step with a side stream (the streaming pass beside the index chain, the BEV maps written
    after it by shpl_bev_maps / shpl_bev_input from the voxelizer's sorted words) == the sequential step
    (maps written by shpl_bev_slices itself, or its bev_input), bitwise: layer outputs and the maps in
    either form (f64 height + density maps; the f32 network input)."""
    from sparse_pooling_amd import kitti, pipeline
    d, g = kitti_dir
    shapes = [tuple(g["7_image_shape"]), tuple(g["8_image_shape"])]
    fr = kitti.KittiFrames.from_dirs(os.path.join(d, "calib"), os.path.join(d, "velodyne"), os.path.join(d, "planes"),
                                     [7, 8], shapes, flips=[False, True])
    im_size, stride, C = (1242, 375), (4, 4), 8
    outs = []
    for side in (None, torch.cuda.Stream()):
        pl = pipeline.FramePipeline(2, fr.total_points, im_size, synth.AREA_EXTENTS, synth.VOXEL_SIZE,
                                    synth.HEIGHT_LO, synth.HEIGHT_HI, synth.NUM_SLICES, stride, C, C, dual=True,
                                    max_points_per_frame=fr.max_points)
        pl.maps_form = form
        bev = torch.from_numpy(synth.make_features((2, pl.Hb, pl.Wb, C), 3)).to(DEV)
        img = torch.from_numpy(synth.make_features((2, pl.Hi, pl.Wi, C), 4)).to(DEV)
        for _ in range(2):  # the second step reuses every workspace
            pl.velo_step(fr, bev, img, side=side)
        torch.cuda.synchronize()
        assert int(pl.err.item()) == 0 and int(pl.bev.err.item()) == 0
        maps = (pl.bev.height_maps, pl.bev.density_map) if form == "f64" else (pl.bev.bev_input,)
        outs.append([_np(t).copy() for t in (pl.bv_fused, pl.img_fused, *maps)])
    for a, b in zip(*outs):
        np.testing.assert_array_equal(a.view(np.uint8), b.view(np.uint8))


@pytest.mark.parametrize("cfg,dtype,counts", [
    (1, "f32", (1.0, 0.0, 0.5)), (3, "bf16", (0.3, 1.0, 0.0, 0.7)), (1, "f32", (0.0, 0.0)), (1, "bf16", (0.2,))])
def test_sparse_live_entries_equal_capacity_walk(cfg, dtype, counts):
    """The sparse passes with the CSR's frame layout (Csr.live_frames: k_sparse walks the live entries
    of each frame with a bounded grid, k_sparse_long skips empty stretches) against the capacity walk,
    forward (both directions) and backward, bitwise: frames whose live points are a fraction of their
    slots (point_counts), empty frames, a frame alone; cfg 3 has pixel runs longer than k_sparse's 8
    entries (k_sparse_long). The capacity walk is the oracle-pinned path of the other tests."""
    from sparse_pooling_amd import pipeline
    spec = synth.CONFIGS[cfg]
    B = len(counts)
    frames = [synth.make_frame(spec, seed=700 + f, n_outside=10) for f in range(B)]
    pts, vox, off, P, maxp, N = pipeline.stack_frames(frames, DEV)
    n = np.diff(_np(off))
    cnt = torch.tensor([int(round(c * k)) for c, k in zip(counts, n)], dtype=torch.int64, device=DEV)
    tdt = torch.float32 if dtype == "f32" else torch.bfloat16
    Hb, Wb = spec.bev_feat_hw
    Hi, Wi = spec.img_feat_hw
    Cb, Ci = spec.c_bev, spec.c_img
    g = torch.Generator(device=DEV).manual_seed(5)
    bev = torch.randn((B, Hb, Wb, Cb), device=DEV, generator=g).to(tdt)
    img = torch.randn((B, Hi, Wi, Ci), device=DEV, generator=g).to(tdt)
    gb = torch.randn((B, Hb, Wb, Cb + Ci), device=DEV, generator=g).to(tdt)
    gi = torch.randn((B, Hi, Wi, Ci + Cb), device=DEV, generator=g).to(tdt)
    outs = []
    for live in (False, True):
        pl = pipeline.FusedPipeline(B, maxp, N, spec.im_size, spec.bv_size, spec.stride, Cb, Ci, dtype=tdt,
                                    dual=True, rows=False, live=live)
        assert (pl.csr.struct.n_frames > 0) == live
        pl.build_index(pts, vox, off, P, point_counts=cnt)
        pl.build_csr()
        pl.layer(bev, img)
        d_bev, d_img = torch.empty_like(bev), torch.empty_like(img)
        pl.backward(gb, gi, d_bev, d_img)
        torch.cuda.synchronize()
        assert int(pl.err.item()) == 0
        if cfg == 3 and live:  # a long run is really there
            e = pl.pcsr.ent_dst[pl.pcsr.ent_dst >= 0]
            assert int(torch.unique_consecutive(e, return_counts=True)[1].max().item()) > 8
        outs.append([t.clone() for t in (pl.bv_fused, pl.img_fused, d_bev, d_img)])
    for a, b in zip(*outs):
        assert torch.equal(a.view(torch.int16) if a.dtype == torch.bfloat16 else a.view(torch.int32),
                           b.view(torch.int16) if b.dtype == torch.bfloat16 else b.view(torch.int32))


def test_sparse_live_frame_limit():
    """shpl_csr.n_frames above SHPL_LIVE_MAX_FRAMES (or negative) is an argument error of the sparse
    pass, raised before any launch; Csr.live_frames keeps the capacity walk for such batches."""
    from sparse_pooling_amd import _lib as L
    F = L.LIVE_MAX_FRAMES + 1
    c = L.Csr(8, 64, DEV, with_col=False)
    off = torch.zeros(F + 1, dtype=torch.int64, device=DEV)
    nnz = torch.zeros(F, dtype=torch.int64, device=DEV)
    assert c.live_frames(off, nnz).struct.n_frames == 0  # too many frames: capacity walk
    src = torch.zeros((8, 4), device=DEV)
    out = torch.zeros((8, 4), device=DEV)
    for bad in (F, -1):
        c.struct.frame_off, c.struct.frame_nnz, c.struct.n_frames = off.data_ptr(), nnz.data_ptr(), bad
        rc = L.lib().shpl_pull_sparse(L.BY_CELL, L.F32, c.ref(), L.ptr(src), 4, 0, 4, None, 0, 0, 0, L.OUT_POOL,
                                      L.ptr(out), 4, L.stream_of(torch.device(DEV)))
        assert rc == L.ERR_ARG, rc
