"""Drop-in mirror of ``avod.utils.sparse_pool_utils`` (and MV3D's copy) on
MI355X.

Same function names, argument order, dict keys and failure behaviour as
avod/avod/utils/sparse_pool_utils.py; torch tensors on the GPU take the
place of numpy arrays / tf.Tensors. Every numeric step runs in libshpl's
HIP kernels -- there is no CPU path; if the library is missing the calls
raise ``ShplLibraryError``.

Differences a caller can observe (documented in DESIGN.md):

* index-builder outputs are device tensors (``M_size``, ``bv_size`` and
  ``img_size`` stay host numpy arrays: they are shapes);
* ``sparse_pool_layer`` returns torch tensors with autograd (the gradient is
  TF 1.8's, computed by the same pull kernels);
* ``concat_bn_op`` raises ``TypeError`` exactly where the reference's does
  (it passes ``training=`` to ``slim.batch_norm``, which has no such argument).
"""
from __future__ import annotations

from typing import NamedTuple

import numpy as np
import torch

from . import _lib as L
from . import shpl_map as sm
from .errors import InvalidArgumentError

__all__ = ["SparseTensor", "gen_sparse_pooling_input_avod", "produce_sparse_pooling_input",
           "sparse_pool_layer", "_sparse_pool_op", "_sparse_pool_trans_op", "concat_bn_op",
           "build_sparse_pooling_input"]


class SparseTensor(NamedTuple):
    """Stand-in for tf.SparseTensor(indices, values, dense_shape) as built from
    the placeholders at rpn_model.py:330-331 / retinanet_model.py:330-332."""
    indices: object
    values: object
    dense_shape: object


def _device():
    if not torch.cuda.is_available():
        raise L.ShplLibraryError("SHPL runs on the GPU (HIP); no device is visible")
    return torch.device("cuda", torch.cuda.current_device())


def _to_dev(a, dtype, dev):
    if isinstance(a, torch.Tensor):
        return a.to(device=dev, dtype=dtype).contiguous()
    return torch.as_tensor(np.ascontiguousarray(a), dtype=dtype).to(dev)


def _host_ints(a):
    if isinstance(a, torch.Tensor):
        a = a.detach().cpu().numpy()
    return np.asarray(a)


# ------------------------------------------------------------ index builder

def gen_sparse_pooling_input_avod(points, voxel_indices, stereo_calib, im_size, bv_size):
    """avod/avod/utils/sparse_pool_utils.py:6-20 on the device.

    points [N,3] camera frame (numpy or tensor, f64/f32), voxel_indices [N,>=2],
    stereo_calib with ``.p2`` (3x4), im_size [W,H], bv_size (H,W).
    Returns {'bv_index' [Nv,2] i64, 'img_index' [3,Nv] f64 (rows u, v, 0),
    'bv_size', 'img_size'} -- the index arrays as device tensors."""
    dev = _device()
    pts = _to_dev(points, torch.float64 if not (isinstance(points, torch.Tensor) and
                                                 points.dtype == torch.float32) else torch.float32, dev)
    pts = pts.reshape(-1, 3)
    vox = voxel_indices if isinstance(voxel_indices, torch.Tensor) else np.asarray(voxel_indices)
    vox = _to_dev(vox, torch.int64 if vox.dtype in (np.int64, torch.int64) else torch.int32, dev)
    vox = vox.reshape(pts.shape[0], -1) if pts.shape[0] else vox.reshape(0, 2)
    P = _to_dev(np.asarray(stereo_calib.p2, dtype=np.float64).reshape(12), torch.float64, dev)
    n = pts.shape[0]
    bv_index = torch.empty((max(n, 1), 2), dtype=torch.int64, device=dev)
    img_index = torch.empty((3, max(n, 1)), dtype=torch.float64, device=dev)
    nv = torch.zeros(1, dtype=torch.int64, device=dev)
    ws = L.workspace(L.index_ws_bytes(1, n), dev)
    L.check(L.lib().shpl_gen_index(n, L.ptr(pts), L.F64 if pts.dtype == torch.float64 else L.F32,
                                   L.ptr(vox), L.I64 if vox.dtype == torch.int64 else L.I32,
                                   int(vox.shape[1]) if vox.dim() == 2 else 2, L.ptr(P),
                                   float(im_size[0]), float(im_size[1]), L.ptr(bv_index),
                                   L.ptr(img_index), img_index.shape[1], L.ptr(nv), L.ptr(ws),
                                   ws.numel(), L.stream_of(dev)), "shpl_gen_index")
    k = int(nv.item())
    return {"bv_index": bv_index[:k], "img_index": img_index[:, :k].contiguous(),
            "bv_size": np.array([bv_size[0], bv_size[1]]), "img_size": np.array(im_size)}


def produce_sparse_pooling_input(input_dict, M_val=None, stride=[1, 1]):  # noqa: B006 (reference signature)
    """avod/avod/utils/sparse_pool_utils.py:22-58 on the device.

    stride[0] applies to the image and stride[1] to BEV (the reference's
    comment at :23 says the opposite; its code does this). Like the
    reference, ``input_dict['img_index']`` is updated in place (tensor: on
    the device; numpy array: written back). Returns {'Mij_pool' [N,2] i64,
    'M_val', 'M_size' (host), 'img_index_flip_pool' [N,3] i64,
    'bev_index_flip_pool' zeros((0,3))}."""
    img = input_dict["img_index"]
    assert img.shape[0] == 3, "wrong img_index shape, should be 3xN instead " + str(tuple(img.shape))
    dev = _device()
    bv = input_dict["bv_index"]
    bv = bv if isinstance(bv, torch.Tensor) else np.asarray(bv)
    bv_t = _to_dev(bv, torch.int64 if bv.dtype in (np.int64, torch.int64) else torch.int32, dev)
    nv = int(img.shape[1])
    bv_t = bv_t.reshape(nv, -1) if nv else bv_t.reshape(0, 2)
    if isinstance(img, torch.Tensor) and img.is_cuda and img.dtype == torch.float64 and img.is_contiguous():
        img_t = img
    else:
        img_t = _to_dev(img, torch.float64, dev)
    im_size = np.asarray(input_dict["img_size"], dtype=np.float64)
    bv_size = np.asarray(input_dict["bv_size"], dtype=np.float64)
    mij = torch.empty((max(nv, 1), 2), dtype=torch.int64, device=dev)
    flip = torch.empty((max(nv, 1), 3), dtype=torch.int64, device=dev)
    nk = torch.zeros(1, dtype=torch.int64, device=dev)
    err = torch.zeros(1, dtype=torch.int32, device=dev)
    ws = L.workspace(L.index_ws_bytes(1, nv), dev)
    L.check(L.lib().shpl_produce_index(nv, L.ptr(bv_t), L.I64 if bv_t.dtype == torch.int64 else L.I32,
                                       int(bv_t.shape[1]) if bv_t.dim() == 2 else 2, L.ptr(img_t),
                                       img_t.shape[1], float(im_size[0]), float(im_size[1]),
                                       float(bv_size[0]), float(bv_size[1]), float(stride[0]),
                                       float(stride[1]), L.ptr(mij), L.ptr(flip), None, None,
                                       L.ptr(nk), L.ptr(err), L.ptr(ws), ws.numel(),
                                       L.stream_of(dev)), "shpl_produce_index")
    k = int(nk.item())
    if img_t is not img:  # write the in-place update back to the caller's array
        if isinstance(img, torch.Tensor):
            img.copy_(img_t)
        else:
            img[...] = img_t.cpu().numpy()
    s_bv = float(stride[1])
    n_cells = np.floor(bv_size / s_bv)
    M_size = np.array([n_cells[0] * n_cells[1], k]).astype(int)
    if M_val is None:
        M_val = torch.ones(k, dtype=torch.float64, device=dev)
    return {"Mij_pool": mij[:k], "M_val": M_val, "M_size": M_size,
            "img_index_flip_pool": flip[:k], "bev_index_flip_pool": np.zeros((0, 3))}


def build_sparse_pooling_input(points, voxel_indices, stereo_calib, im_size, bv_size,
                               stride=(1, 1), M_val=None):
    """gen_sparse_pooling_input_avod + produce_sparse_pooling_input fused into
    one device pass -- the call KittiDataset.load_samples makes per frame
    (avod/avod/datasets/kitti/kitti_dataset.py:374-379). Returns the same dict
    as produce_sparse_pooling_input."""
    dev = _device()
    pts = _to_dev(points, torch.float64, dev).reshape(-1, 3)
    vox = _to_dev(np.asarray(voxel_indices) if not isinstance(voxel_indices, torch.Tensor)
                  else voxel_indices, torch.int64, dev)
    n = pts.shape[0]
    vox = vox.reshape(n, -1) if n else vox.reshape(0, 2)
    P = _to_dev(np.asarray(stereo_calib.p2, dtype=np.float64).reshape(1, 12), torch.float64, dev)
    off = torch.tensor([0, n], dtype=torch.int64, device=dev)
    ib = sm.build_index_batch(pts, vox, off, P, im_size, bv_size, stride, n, ref_outputs=True)
    k = int(ib.frame_nnz.item())
    bq = np.floor(np.asarray(bv_size, dtype=np.float64) / float(stride[1]))
    M_size = np.array([bq[0] * bq[1], k]).astype(int)
    if M_val is None:
        M_val = torch.ones(k, dtype=torch.float64, device=dev)
    return {"Mij_pool": ib.mij[:k], "M_val": M_val, "M_size": M_size,
            "img_index_flip_pool": ib.flip[:k], "bev_index_flip_pool": np.zeros((0, 3))}


# ---------------------------------------------------------------- op layer

def _pack(M, source_index, img_shape, n_rows_expected=None):
    dev = _device()
    shape = _host_ints(M.dense_shape).astype(np.int64)
    if n_rows_expected is not None and int(shape[0]) != int(n_rows_expected):
        raise InvalidArgumentError(
            f"Input to reshape has {int(shape[0])} rows, but the pooled map has {n_rows_expected} cells")
    mij = _to_dev(M.indices, torch.int64, dev)
    vals = _to_dev(M.values, torch.float32, dev)
    idx = source_index if isinstance(source_index, torch.Tensor) else np.asarray(source_index)
    idx = _to_dev(idx, torch.int32 if idx.dtype in (np.int32, torch.int32) else torch.int64, dev)
    return sm.pack_map(mij, vals, shape, idx, img_shape)


def _sparse_pool_op(M, input, source_index, pooled_size):  # noqa: A002 (reference signature)
    """sparse_pool_utils.py:96-103: reshape(matmul(M, gather_nd(input, idx)), pooled_size)."""
    pooled_size = [int(s) for s in pooled_size]
    if pooled_size[0] != 1:
        raise InvalidArgumentError("only batch size 1 is supported (as in the reference)")
    if pooled_size[3] != input.shape[-1]:
        raise InvalidArgumentError("pooled depth must equal the depth of the source feature map")
    smap = _pack(M, source_index, tuple(input.shape), pooled_size[1] * pooled_size[2])
    return sm.pool_op(input, smap, pooled_size[:3])


def _sparse_pool_trans_op(M, input, source_index, pooled_size):  # noqa: A002
    """sparse_pool_utils.py:105-117: scatter_nd(idx, matmul(sparse_transpose(M),
    reshape(input, [-1, C])), pooled_size)."""
    pooled_size = [int(s) for s in pooled_size]
    if pooled_size[3] != input.shape[-1]:
        raise InvalidArgumentError("scatter_nd updates depth must equal pooled depth")
    n_rows = int(np.prod(input.shape[:-1]))
    smap = _pack(M, source_index, tuple(pooled_size), n_rows)
    return sm.trans_op(input, smap, pooled_size[:3])


def concat_bn_op(inputs, axis, training):
    """sparse_pool_utils.py:120-124 calls slim.batch_norm(..., training=...),
    which TF-slim rejects; this mirror fails the same way."""
    raise TypeError("batch_norm() got an unexpected keyword argument 'training' "
                    "(concat_bn_op is broken in the reference, sparse_pool_utils.py:122)")


def sparse_pool_layer(inputs, feature_depths, M, img_index_flip=None, bv_index=None, use_bn=False,
                      training=True):
    """sparse_pool_utils.py:61-92.

    inputs = [bev [1,Hb,Wb,Cb], img [1,Hi,Wi,Ci]]; feature_depths =
    [depth pooled into BEV (= Ci), depth pooled into the image (= Cb)].
    img->BEV runs when img_index_flip is given; BEV->img additionally when
    bv_index is not None (its value is a sentinel only: img_index_flip is the
    scatter index, :83). Returns (bv_fused, img_fused)."""
    input_bv, input_img = inputs[0], inputs[1]
    if img_index_flip is None:
        if bv_index is not None:
            # the reference hands None to scatter_nd here and fails
            raise ValueError("dual sparse pooling needs img_index_flip (reference :83)")
        return input_bv, input_img
    if use_bn:
        return concat_bn_op([input_bv, None], axis=3, training=training)
    if int(feature_depths[0]) != input_img.shape[-1]:
        raise InvalidArgumentError("feature_depths[0] must equal the image feature depth")
    Hb, Wb = int(input_bv.shape[1]), int(input_bv.shape[2])
    dual = bv_index is not None
    if dual:
        print('using dual sparse pooling')
        if int(feature_depths[1]) != input_bv.shape[-1]:
            raise InvalidArgumentError("feature_depths[1] must equal the BEV feature depth")
    if input_bv.shape[0] != 1:
        raise InvalidArgumentError("only batch size 1 is supported (as in the reference)")
    smap = _pack(M, img_index_flip, tuple(input_img.shape), Hb * Wb)
    return sm.layer(input_bv, input_img, smap, dual=dual)
