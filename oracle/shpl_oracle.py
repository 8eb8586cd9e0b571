"""ctypes front-end of the C oracle (oracle/shpl_oracle.c).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg -- as the checker, never as the product path.
See the header of shpl_oracle.c for what is restated from where and for the
parity status (index builder pinned by the reference-generated goldens;
pooling ops restated from TensorFlow 1.8's kernel order, "parity unpinned"
beyond that; BEV slices, MV3D producer and the KITTI velodyne loader pinned
by reference-generated goldens).
"""
import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
# SHPL_ORACLE_LIB: an alternative build of the same source, e.g. the
# ASan/UBSan one (`make -C oracle san`, tests/test_oracle_sanitized.py)
_LIB_PATH = os.environ.get("SHPL_ORACLE_LIB") or os.path.join(_HERE, "build", "libshpl_oracle.so")
_lib = None


class OracleError(ValueError):
    """Mirror of TF's InvalidArgumentError for the oracle."""


def build():
    subprocess.run(["make", "-s", "-C", _HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        _lib = ctypes.CDLL(_LIB_PATH)
        i64, p = ctypes.c_int64, ctypes.c_void_p
        d = ctypes.c_double
        _lib.shplo_gen_index.restype = i64
        _lib.shplo_gen_index.argtypes = [i64, p, p, p, d, d, p, p, i64]
        _lib.shplo_produce.restype = i64
        _lib.shplo_produce.argtypes = [i64, p, p, i64, d, d, d, d, d, d, p, p, p]
        _lib.shplo_pool.restype = ctypes.c_int
        _lib.shplo_pool.argtypes = [p, i64, i64, i64, i64, p, i64, p, p, i64, i64, i64, p]
        _lib.shplo_pool_trans.restype = ctypes.c_int
        _lib.shplo_pool_trans.argtypes = [p, i64, i64, p, p, i64, i64, p, i64, i64, i64, i64, p]
        _lib.shplo_pool_grad_img.restype = ctypes.c_int
        _lib.shplo_pool_grad_img.argtypes = [p, i64, i64, p, p, i64, i64, p, i64, i64, i64, i64, p]
        _lib.shplo_pool_trans_grad_bev.restype = ctypes.c_int
        _lib.shplo_pool_trans_grad_bev.argtypes = [p, i64, i64, i64, i64, p, i64, p, p, i64, i64,
                                                    i64, p]
        _lib.shplo_mv3d_voxels.restype = i64
        _lib.shplo_mv3d_voxels.argtypes = [i64, p, i64, p, p, d, d, ctypes.c_int, p, i64, p, p, p, p]
        _lib.shplo_velo_to_cam.restype = i64
        _lib.shplo_velo_to_cam.argtypes = [i64, p, p, p, ctypes.c_int, d, d, d, ctypes.c_int, p]
        _lib.shplo_bev_slices.restype = i64
        _lib.shplo_bev_slices.argtypes = [i64, p, p, p, d, ctypes.c_int, p, p, d, d, d, p, i64, p, p,
                                          p, p]
        _lib.shplo_conv3x3.restype = None
        _lib.shplo_conv3x3.argtypes = [p, i64, i64, i64, i64, p, i64, p, p, p, ctypes.c_int, p, p]
        _lib.shplo_conv3x3_wgrad.restype = None
        _lib.shplo_conv3x3_wgrad.argtypes = [p, i64, i64, i64, i64, p, i64, p]
        _lib.shplo_bn_bwd.restype = None
        _lib.shplo_bn_bwd.argtypes = [p, p, i64, i64, ctypes.c_int, p, p, d, p, p, ctypes.c_int, p, p, p]
        _lib.shplo_bn_train.restype = None
        _lib.shplo_bn_train.argtypes = [p, i64, i64, d, p, p, ctypes.c_int, p, p, p, d, p, p]
    return _lib


def _p(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def _c(a, dtype):
    return np.ascontiguousarray(a, dtype=dtype)


# ---- index builder -------------------------------------------------------

def gen_sparse_pooling_input_avod(points, voxel_indices, p2, im_size, bv_size):
    """Restates avod/avod/utils/sparse_pool_utils.py:6-20. ``p2`` is the 3x4 P."""
    pts = _c(points, np.float64).reshape(-1, 3)
    vox = _c(np.asarray(voxel_indices)[:, :2], np.int64)
    n = pts.shape[0]
    bv = np.zeros((max(n, 1), 2), np.int64)
    img = np.zeros((3, max(n, 1)), np.float64)
    nv = lib().shplo_gen_index(n, _p(pts), _p(vox), _p(_c(p2, np.float64)),
                               float(im_size[0]), float(im_size[1]), _p(bv), _p(img), img.shape[1])
    return {"bv_index": bv[:nv].copy(), "img_index": np.ascontiguousarray(img[:, :nv]),
            "bv_size": np.array([bv_size[0], bv_size[1]]), "img_size": np.array(im_size)}


def produce_sparse_pooling_input(input_dict, M_val=None, stride=(1, 1)):
    """Restates avod/avod/utils/sparse_pool_utils.py:22-58, including the
    in-place update of ``input_dict['img_index']``."""
    img = input_dict["img_index"]
    assert img.shape[0] == 3, "wrong img_index shape, should be 3xN instead " + str(img.shape)
    work = _c(img, np.float64)
    bv = _c(input_dict["bv_index"], np.int64).reshape(-1, 2)
    nv = work.shape[1]
    mij = np.zeros((max(nv, 1), 2), np.int64)
    flip = np.zeros((max(nv, 1), 3), np.int64)
    msize = np.zeros(2, np.int64)
    im = input_dict["img_size"]
    bs = input_dict["bv_size"]
    nk = lib().shplo_produce(nv, _p(bv), _p(work), work.shape[1], float(im[0]), float(im[1]),
                             float(bs[0]), float(bs[1]), float(stride[0]), float(stride[1]),
                             _p(mij), _p(flip), _p(msize))
    img[...] = work  # the reference mutates the caller's array
    if M_val is None:
        M_val = np.ones(nk)
    return {"Mij_pool": mij[:nk].copy(), "M_val": M_val, "M_size": msize,
            "img_index_flip_pool": flip[:nk].copy(), "bev_index_flip_pool": np.zeros((0, 3))}


# ---- BEV slices (a5/a6) ------------------------------------------------------

def slice_bounds(height_lo, height_hi, num_slices):
    """BevSlices' per-slice plane offsets, computed exactly as bev_slices.py:30-31, :66-67."""
    hpd = (height_hi - height_lo) / num_slices
    lo = [height_lo + s * hpd for s in range(num_slices)]
    return hpd, np.array(lo), np.array([v + hpd for v in lo])


def density_table(norm_value=np.log(16)):
    """min(1, log(n + 1) / norm) for n = 0..15 (bev_generator.py:33-34)."""
    return np.minimum(1.0, np.log(np.arange(16) + 1) / norm_value)


def bev_slices(point_cloud, ground_plane, area_extents, voxel_size, height_lo, height_hi, num_slices):
    """Restates BevSlices.generate_bev(output_indices=True): returns
    (height_maps [S,nz,nx], density_map [nz,nx], voxel_indices [M,2], pts_in_voxel [M,3])."""
    pts = _c(np.asarray(point_cloud).T, np.float64)
    ext = _c(area_extents, np.float64).reshape(3, 2)
    n = pts.shape[0]
    hpd, lo, hi = slice_bounds(height_lo, height_hi, num_slices)
    min_x, min_z = np.floor(ext[0, 0] / voxel_size), np.floor(ext[2, 0] / voxel_size)
    nx = int(np.ceil(ext[0, 1] / voxel_size - 1) - min_x + 1)
    nz = int(np.ceil(ext[2, 1] / voxel_size - 1) - min_z + 1)
    cap = max(n * num_slices, 1)
    vox = np.zeros((cap, 2), np.int64)
    upts = np.zeros((cap, 3), np.float64)
    hm = np.zeros((num_slices, nz, nx), np.float64)
    dm = np.zeros((nz, nx), np.float64)
    m = lib().shplo_bev_slices(n, _p(pts), _p(_c(ground_plane, np.float64)), _p(ext), float(voxel_size),
                               num_slices, _p(_c(lo, np.float64)), _p(_c(hi, np.float64)), float(height_lo),
                               float(height_hi), float(hpd), _p(_c(density_table(), np.float64)), cap,
                               _p(vox), _p(upts), _p(hm), _p(dm))
    return hm, dm, vox[:m].copy(), upts[:m].copy()


# ---- MV3D producer (a7) ------------------------------------------------------

# MV3D cfg (MV3D_TF_release/lib/utils/config_voxels.py:49-59, DETECT_OBJ != 'Car') and the
# ranges construct_voxel.py:11-13 derives from it.
MV3D_PED = dict(ranges=(0.0, 48 - 0.01, -20.0, 20 - 0.01, -1.0, 3 - 0.01), res=0.2, zres=0.4, cap=45)


def mv3d_voxels(points, img_index2, ranges, res, zres, cap):
    """Restates point_cloud_2_top_sparse's SHPL outputs: (img_index [3,n'] f64,
    bv_index [n',2] (fwd, side), M_val [n'], number_buffer [V])."""
    pts = _c(points, np.float64)
    n, stride = pts.shape
    img2 = _c(img_index2, np.int64).reshape(2, n)
    img = np.zeros((3, max(n, 1)), np.float64)
    bv = np.zeros((max(n, 1), 2), np.int64)
    mv = np.zeros(max(n, 1), np.float64)
    nb = np.zeros(max(n, 1), np.int32)
    nvox = ctypes.c_int64()
    k = lib().shplo_mv3d_voxels(n, _p(pts), stride, _p(img2), _p(_c(ranges, np.float64)), float(res),
                                float(zres), int(cap), _p(img), img.shape[1], _p(bv), _p(mv), _p(nb),
                                ctypes.byref(nvox))
    return np.ascontiguousarray(img[:, :k]), bv[:k].copy(), mv[:k].copy(), nb[:nvox.value].copy()


def augment_fv_index(img_index, expansion_ratio, sx, sy):
    """augment_fv's index transform (MV3D_TF_release/lib/roi_data_layer/minibatch_mv3d_img.py:205-206)
    on an int img_index [3, n]: row = (row * ratio + shift).astype(int)."""
    out = np.array(img_index, dtype=np.int64, copy=True)
    r = np.array([expansion_ratio], dtype=np.float64)  # np.random.uniform(0.95, 1.05, 1)
    out[0, :] = (out[0, :] * r + sx).astype(int)
    out[1, :] = (out[1, :] * r + sy).astype(int)
    return out


# ---- KITTI velodyne -> camera frame (§8f item 3) ------------------------------

def rect_matrix(r0_rect, tr_velodyne_to_cam):
    """Rows 0-2 of np.dot(R0_rect padded 4x4, Tr_velo_to_cam padded 4x4), computed
    exactly as calib_utils.lidar_to_cam_frame does (calib_utils.py:388-404)."""
    r0 = np.pad(np.asarray(r0_rect, np.float64).reshape(3, 3), ((0, 1), (0, 1)), "constant", constant_values=0)
    r0[3, 3] = 1
    tf = np.pad(np.asarray(tr_velodyne_to_cam, np.float64).reshape(3, 4), ((0, 1), (0, 0)), "constant",
                constant_values=0)
    tf[3, 3] = 1
    return np.ascontiguousarray(np.dot(r0, tf)[0:3])


def velo_to_cam(xyzi, rect, p2=None, im_size=None, min_intensity=None, flip=False):
    """get_lidar_point_cloud (obj_utils.py:220-268) on an [n,4] f32 velodyne scan:
    returns the (3, n') camera-frame cloud (im_size=None: no filter)."""
    x = _c(xyzi, np.float32).reshape(-1, 4)
    n = x.shape[0]
    out = np.zeros((max(n, 1), 3), np.float64)
    has = im_size is not None
    P = _c(p2 if p2 is not None else np.zeros((3, 4)), np.float64)
    w, h = (float(im_size[0]), float(im_size[1])) if has else (0.0, 0.0)
    k = lib().shplo_velo_to_cam(n, _p(x), _p(_c(rect, np.float64)), _p(P), int(has), w, h,
                                float("nan") if min_intensity is None else float(min_intensity), int(bool(flip)),
                                _p(out))
    return np.ascontiguousarray(out[:k].T)


# ---- TF op restatements ----------------------------------------------------

def _check(rc):
    if rc == 1:
        raise OracleError("shape mismatch")
    if rc == 2:
        raise OracleError("index out of bounds")


def sparse_pool_op(mij, mval, m_size, img, idx):
    """_sparse_pool_op (sparse_pool_utils.py:96-103) before the reshape: R x C."""
    img = _c(img, np.float32)
    B, H, W, C = img.shape
    mij = _c(mij, np.int64).reshape(-1, 2)
    mval = _c(mval, np.float32).reshape(-1)
    idx = _c(idx, np.int64).reshape(-1, 3)
    if mval.shape[0] != mij.shape[0]:
        raise OracleError("values/indices length mismatch")
    R, ncols = int(m_size[0]), int(m_size[1])
    out = np.empty((R, C), np.float32)
    _check(lib().shplo_pool(_p(img), B, H, W, C, _p(idx), idx.shape[0], _p(mij), _p(mval),
                            mij.shape[0], R, ncols, _p(out)))
    return out


def sparse_pool_trans_op(mij, mval, m_size, bev_flat, idx, img_shape):
    """_sparse_pool_trans_op (sparse_pool_utils.py:105-117): returns [B,H,W,C]."""
    bev = _c(bev_flat, np.float32)
    R, C = bev.shape
    mij = _c(mij, np.int64).reshape(-1, 2)
    mval = _c(mval, np.float32).reshape(-1)
    idx = _c(idx, np.int64).reshape(-1, 3)
    if mval.shape[0] != mij.shape[0]:
        raise OracleError("values/indices length mismatch")
    if int(m_size[0]) != R:
        raise OracleError("matmul inner dimension mismatch")
    B, H, W = img_shape[:3]
    out = np.empty((B, H, W, C), np.float32)
    _check(lib().shplo_pool_trans(_p(bev), R, C, _p(mij), _p(mval), mij.shape[0], int(m_size[1]),
                                  _p(idx), idx.shape[0], B, H, W, _p(out)))
    return out


def sparse_pool_grad_img(mij, mval, m_size, dY, idx, img_shape):
    dY = _c(dY, np.float32)
    R, C = dY.shape
    mij = _c(mij, np.int64).reshape(-1, 2)
    mval = _c(mval, np.float32).reshape(-1)
    idx = _c(idx, np.int64).reshape(-1, 3)
    B, H, W = img_shape[:3]
    out = np.empty((B, H, W, C), np.float32)
    _check(lib().shplo_pool_grad_img(_p(dY), R, C, _p(mij), _p(mval), mij.shape[0],
                                     int(m_size[1]), _p(idx), idx.shape[0], B, H, W, _p(out)))
    return out


def sparse_pool_trans_grad_bev(mij, mval, m_size, dZ, idx):
    dZ = _c(dZ, np.float32)
    B, H, W, C = dZ.shape
    mij = _c(mij, np.int64).reshape(-1, 2)
    mval = _c(mval, np.float32).reshape(-1)
    idx = _c(idx, np.int64).reshape(-1, 3)
    R = int(m_size[0])
    out = np.empty((R, C), np.float32)
    _check(lib().shplo_pool_trans_grad_bev(_p(dZ), B, H, W, C, _p(idx), idx.shape[0], _p(mij),
                                           _p(mval), mij.shape[0], R, int(m_size[1]), _p(out)))
    return out


def sparse_pool_layer(bev, img, mij, mval, m_size, idx, dual=False):
    """sparse_pool_layer (sparse_pool_utils.py:61-92), use_bn=False:
    returns (bv_fused, img_fused) as [1,H,W,C] arrays."""
    bev = _c(bev, np.float32)
    img = _c(img, np.float32)
    _, Hb, Wb, Cb = bev.shape
    pooled = sparse_pool_op(mij, mval, m_size, img, idx).reshape(1, Hb, Wb, img.shape[3])
    bv_fused = np.concatenate([bev, pooled], axis=3)
    if dual:
        tp = sparse_pool_trans_op(mij, mval, m_size, bev.reshape(-1, Cb), idx, img.shape)
        img_fused = np.concatenate([img, tp], axis=3)
    else:
        img_fused = img
    return bv_fused, img_fused


def to_bf16_bits(x):
    """f32 -> bf16 round-to-nearest-even (as uint16 bits)."""
    u = np.ascontiguousarray(x, np.float32).view(np.uint32).astype(np.uint64)
    r = ((u + 0x7FFF + ((u >> 16) & 1)) >> 16).astype(np.uint16)
    nan = np.isnan(np.asarray(x, np.float32))
    r[nan] = 0x7FC0
    return r


def from_bf16_bits(b):
    return (np.asarray(b, np.uint16).astype(np.uint32) << 16).view(np.float32)


# ---- f4: post-fusion conv + BatchNorm (rpn_model.py:338-355, retinanet_model.py:343-348)

def _opt(a):
    return None if a is None else _p(_c(a, np.float32))


def conv3x3(x, w, center=None, scale=None, shift=None, relu=False, raw=False):
    """SAME 3x3 conv of NHWC ``x`` [B,H,W,Cin] with HWIO ``w`` [3,3,Cin,Cout],
    summed in double, then act((acc - center) * scale + shift) rounded to f32.
    raw=True also returns the double pre-epilogue sums."""
    x = _c(x, np.float32)
    w = _c(w, np.float32)
    B, H, W, Cin = x.shape
    Cout = w.shape[3]
    assert w.shape == (3, 3, Cin, Cout)
    out = np.empty((B, H, W, Cout), np.float32)
    r = np.empty((B, H, W, Cout), np.float64) if raw else None
    keep = [_c(a, np.float32) if a is not None else None for a in (center, scale, shift)]
    lib().shplo_conv3x3(_p(x), B, H, W, Cin, _p(w), Cout, *[None if a is None else _p(a) for a in keep],
                        int(bool(relu)), _p(out), None if r is None else _p(r))
    return (out, r) if raw else out


def batch_norm_train(raw, eps=1e-3, gamma=None, beta=None, relu=True, moving_mean=None, moving_var=None,
                     decay=0.999):
    """FusedBatchNorm (is_training) over the channels of ``raw`` (double, [..., C]).
    Returns (y f32, batch_mean, batch_var (Bessel-corrected), moving_mean, moving_var)."""
    raw = _c(raw, np.float64)
    C = raw.shape[-1]
    rows = raw.size // C
    out = np.empty(raw.shape, np.float32)
    mm = None if moving_mean is None else _c(moving_mean, np.float32).copy()
    mv = None if moving_var is None else _c(moving_var, np.float32).copy()
    bm, bv = np.empty(C, np.float64), np.empty(C, np.float64)
    g = None if gamma is None else _c(gamma, np.float32)
    b = None if beta is None else _c(beta, np.float32)
    lib().shplo_bn_train(_p(raw), rows, C, float(eps), None if g is None else _p(g), None if b is None else _p(b),
                         int(bool(relu)), _p(out), None if mm is None else _p(mm), None if mv is None else _p(mv),
                         float(decay), _p(bm), _p(bv))
    return out, bm, bv, mm, mv


def conv3x3_dgrad(g, w):
    """Input gradient of the SAME 3x3 conv: the conv of ``g`` [B,H,W,Cout] with
    the flipped, transposed weights W'[ky][kx][co][ci] = W[2-ky][2-kx][ci][co]
    (double sums, rounded once)."""
    wt = np.ascontiguousarray(np.asarray(w, np.float32)[::-1, ::-1].transpose(0, 1, 3, 2))
    return conv3x3(g, wt)


def conv3x3_wgrad(x, g):
    """Weight gradient [3,3,Cin,Cout] (double) of the SAME 3x3 conv."""
    x = _c(x, np.float32)
    g = _c(g, np.float32)
    B, H, W, Cin = x.shape
    Cout = g.shape[3]
    dw = np.empty((3, 3, Cin, Cout), np.float64)
    lib().shplo_conv3x3_wgrad(_p(x), B, H, W, Cin, _p(g), Cout, _p(dw))
    return dw


def batch_norm_backward(raw, g, training=True, mean=None, var=None, eps=1e-3, gamma=None, beta=None, relu=True):
    """(d_raw, dbeta, dgamma) in double of BatchNorm (+ ReLU) over [..., C]."""
    raw = _c(raw, np.float64)
    g = _c(g, np.float32)
    C = raw.shape[-1]
    rows = raw.size // C
    d_raw = np.empty(raw.shape, np.float64)
    db, dg = np.empty(C, np.float64), np.empty(C, np.float64)
    m = None if mean is None else _c(mean, np.float64)
    v = None if var is None else _c(var, np.float64)
    gm = None if gamma is None else _c(gamma, np.float32)
    bt = None if beta is None else _c(beta, np.float32)
    lib().shplo_bn_bwd(_p(raw), _p(g), rows, C, int(bool(training)), None if m is None else _p(m),
                       None if v is None else _p(v), float(eps), None if gm is None else _p(gm),
                       None if bt is None else _p(bt), int(bool(relu)), _p(d_raw), _p(db), _p(dg))
    return d_raw, db, dg
