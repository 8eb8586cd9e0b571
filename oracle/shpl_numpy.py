"""numpy restatement of the reference's CPU path for the bench's cpu_baseline leg.

TEST INFRASTRUCTURE ONLY: imported by tests/ and bench.py's cpu_baseline leg,
as a baseline / checker, never by the product path.

The reference builds the index in numpy inside the data loader and pools with
stock TensorFlow 1.8 CPU kernels. This module does the same work the same way,
with numpy, so that the bench can time "the reference CPU path" on the GPU
box, where the reference itself (and TensorFlow) is absent:

* index build -- avod/avod/utils/sparse_pool_utils.py:6-20 and :22-58, with
  the projection of avod/avod/utils/transform.py:3-26 (np.dot of P by the
  homogeneous 4xN points, then the two divisions) and the clip of :28-40;
  np.round / np.floor / boolean masks as the reference uses them.
* pooling -- the four TF ops of sparse_pool_utils.py:96-117: GatherNd (row
  copy), SparseTensorDenseMatMul (zero-initialised, one entry after the other,
  out[row] += val * rhs[col] with the product rounded before the add -- TF
  1.8's CPU kernel, sparse_tensor_dense_matmul_op.cc, takes its scalar loop
  below 32 right-hand columns and its Eigen `chip += chip * scalar` loop from
  32 on; both evaluate the same separate multiply and add in nnz order, since
  the pip builds carry no FMA), SparseTranspose (stable sort by (col, row)),
  ScatterNd (duplicates summed in update order); np.add.at is numpy's
  unbuffered sequential scatter-add, the same order.
* concat -- sparse_pool_utils.py:72, :87.

Outputs equal oracle/shpl_oracle.c bit for bit (tests/test_oracle_numpy.py),
which the index goldens pin to the reference's own numpy run here.
"""
import numpy as np


def project_to_image(pts_3d, P):
    """transform.py:3-26: 3xN camera-frame points -> 2xN pixel coordinates."""
    hom = np.concatenate([pts_3d, np.ones((1, pts_3d.shape[1]))], axis=0)
    uvw = np.dot(P, hom)
    return np.stack([uvw[0] / uvw[2], uvw[1] / uvw[2]])


def clip_within_image(pts_3d, P, image_size):
    """transform.py:28-40: points whose projection lies strictly inside [0, W-1) x [0, H-1)."""
    uv = project_to_image(pts_3d, P)
    return (uv[0] < image_size[0] - 1) & (uv[0] >= 0) & (uv[1] >= 0) & (uv[1] < image_size[1] - 1)


def gen_sparse_pooling_input_avod(points, voxel_indices, P, im_size, bv_size):
    """sparse_pool_utils.py:6-20 (P = stereo_calib.p2 passed directly)."""
    keep = clip_within_image(points.T, P, im_size)
    bv_index = np.stack([voxel_indices[:, 0], voxel_indices[:, 1]], axis=1)[keep]
    uv = np.round(project_to_image(points[keep].T, P)).astype(int)
    img_index = np.concatenate([uv, np.zeros((1, uv.shape[1]))], axis=0)
    return {"bv_index": bv_index, "img_index": img_index, "bv_size": np.array([bv_size[0], bv_size[1]]),
            "img_size": np.array(im_size)}


def produce_sparse_pooling_input(d, M_val=None, stride=(1, 1)):
    """sparse_pool_utils.py:22-58: strides, clamp, flip to (b, v, u), flatten, drop rows
    past the BEV map; img_index is updated in place as in the reference."""
    img_index, bv_index = d["img_index"], d["bv_index"]
    img_index[0:2, :] = np.floor(img_index[0:2, :] / stride[0])
    im = np.floor(d["img_size"] / stride[0])
    img_index[0, img_index[0, :] >= im[0]] = im[0] - 1
    img_index[1, img_index[1, :] >= im[1]] = im[1] - 1
    flip = np.floor(img_index.T[:, ::-1]).astype(int)
    bv = np.floor(np.array(d["bv_size"]) / stride[1])
    down = np.floor(bv_index / stride[1])
    cell = (down[:, 1] * bv[1] + down[:, 0]).astype(int)
    inside = cell < int(bv[0] * bv[1])
    flip, cell = flip[inside], cell[inside]
    n = cell.shape[0]
    return {"Mij_pool": np.stack([cell, np.arange(n)], axis=1), "M_val": np.ones(n) if M_val is None else M_val,
            "M_size": np.array([bv[0] * bv[1], n]).astype(int), "img_index_flip_pool": flip}


def sparse_pool_op(mij, mval, m_size, img, idx):
    """_sparse_pool_op (sparse_pool_utils.py:96-103): GatherNd + SparseTensorDenseMatMul."""
    gathered = img[idx[:, 0], idx[:, 1], idx[:, 2]]
    out = np.zeros((int(m_size[0]), img.shape[3]), np.float32)
    np.add.at(out, mij[:, 0], (mval[:, None].astype(np.float32) * gathered[mij[:, 1]]).astype(np.float32))
    return out


def sparse_pool_trans_op(mij, mval, m_size, bev_flat, idx, img_shape):
    """_sparse_pool_trans_op (sparse_pool_utils.py:105-117): SparseTranspose (stable by
    (col, row)) + SparseTensorDenseMatMul into per-column partials + ScatterNd."""
    order = np.lexsort((np.arange(len(mij)), mij[:, 0], mij[:, 1]))
    q = np.zeros((int(m_size[1]), bev_flat.shape[1]), np.float32)
    np.add.at(q, mij[order, 1], (mval[order, None].astype(np.float32) * bev_flat[mij[order, 0]]).astype(np.float32))
    out = np.zeros(tuple(img_shape[:3]) + (bev_flat.shape[1],), np.float32)
    np.add.at(out, (idx[:, 0], idx[:, 1], idx[:, 2]), q)
    return out


def sparse_pool_grad_img(mij, mval, m_size, dY, idx, img_shape):
    """TF 1.8's gradient of _sparse_pool_op w.r.t. the image: the SparseTensorDenseMatMul
    gradient matmul(M, dY, adjoint_a=True) in nnz order, then GatherNd's gradient, ScatterNd."""
    q = np.zeros((int(m_size[1]), dY.shape[1]), np.float32)
    np.add.at(q, mij[:, 1], (mval[:, None].astype(np.float32) * dY[mij[:, 0]]).astype(np.float32))
    out = np.zeros(tuple(img_shape[:3]) + (dY.shape[1],), np.float32)
    np.add.at(out, (idx[:, 0], idx[:, 1], idx[:, 2]), q)
    return out


def sparse_pool_trans_grad_bev(mij, mval, m_size, dZ, idx):
    """TF 1.8's gradient of _sparse_pool_trans_op w.r.t. the BEV map: ScatterNd's gradient
    (GatherNd of dZ), then matmul(M^T, dQ, adjoint_a=True) over M^T's (col, row) order."""
    dq = dZ[idx[:, 0], idx[:, 1], idx[:, 2]]
    order = np.lexsort((np.arange(len(mij)), mij[:, 0], mij[:, 1]))
    out = np.zeros((int(m_size[0]), dZ.shape[3]), np.float32)
    np.add.at(out, mij[order, 0], (mval[order, None].astype(np.float32) * dq[mij[order, 1]]).astype(np.float32))
    return out


def sparse_pool_layer(bev, img, mij, mval, m_size, idx, dual=False):
    """sparse_pool_layer (sparse_pool_utils.py:61-92) without batch norm: the concats of :72 / :87."""
    pooled = sparse_pool_op(mij, mval, m_size, img, idx).reshape(bev.shape[:3] + (img.shape[3],))
    bv_fused = np.concatenate([bev, pooled], axis=3)
    if not dual:
        return bv_fused, img
    trans = sparse_pool_trans_op(mij, mval, m_size, bev.reshape(-1, bev.shape[3]), idx, img.shape)
    return bv_fused, np.concatenate([img, trans], axis=3)
