"""MV3D_TF's SHPL entry points on MI355X.

* ``produce_sparse_pooling_input`` mirrors
  ``fusion_voxel_train.produce_sparse_pooling_input``
  (MV3D_TF_release/lib/networks/MV3D_voxel_train.py:89-91): same argument
  order, default stride ``[8, 2]`` (``_feat_stride_pool``: image stride 8,
  BEV stride 2, :14), returns ``(Mij, M_val, M_size, img_index_flip)``.
* ``sparse_pool`` mirrors the ``@layer sparse_pool`` of
  MV3D_TF_release/lib/networks/network.py:243-246:
  ``input = [M, img_features, img_index_flip]``.
* ``calib_to_P`` / ``calib_to_L2C`` mirror MV3D_TF_release/lib/utils/
  transform.py:13-30: the camera matrix the minibatch projects with
  (minibatch_mv3d_img.py:89) from the imdb's 4x12 calib rows.

M_val here is the MV3D voxel weight 1/count (construct_voxel.py:160); it is
carried unchanged to the pull kernels, which then compute per-voxel means
summed over the z-voxels of a BEV cell.
"""
from . import sparse_pool_utils as spu

_feat_stride_pool = [8, 2]  # 0 is img, 1 is bv (MV3D_voxel_train.py:14)


def produce_sparse_pooling_input(img_index, im_size, bv_index, bv_size, M_val=None,
                                 stride=_feat_stride_pool):
    out = spu.produce_sparse_pooling_input({'img_index': img_index, 'img_size': im_size,
                                            'bv_index': bv_index, 'bv_size': bv_size},
                                           M_val=M_val, stride=stride)
    return out['Mij_pool'], out['M_val'], out['M_size'], out['img_index_flip_pool']


def sparse_pool(input, pooled_size):  # noqa: A002 (reference signature)
    """0 is the sparse matrix M, 1 the source feature map, 2 the pooling index."""
    return spu._sparse_pool_op(input[0], input[1], input[2], pooled_size)


def calib_to_P(calib, from_camera=False):
    """Lidar (or camera, from_camera=True) coordinates -> image: the 3x4 P with
    uvw = P [X; Y; Z; 1]. calib rows (imdb layout): 0 = P2 (3x4), 2 = R0 read
    as 4x3 and closed by the column [0, 0, 0, 1], 3 = Tr_velo_to_cam (3x4)
    closed by the row [0, 0, 0, 1]; P = (P2 . R0) . C2V, evaluated in that
    association (numpy matmul) like transform.py:22-23."""
    import numpy as np
    calib = np.asarray(calib, dtype=np.float64)
    p2 = calib[0].reshape(3, 4)
    if from_camera:
        return p2
    return np.matmul(np.matmul(p2, _r0_4x4(calib)), _c2v_4x4(calib))


def calib_to_L2C(calib):
    """Lidar -> camera frame: R0 . C2V (transform.py:26-30), both closed to 4x4."""
    import numpy as np
    calib = np.asarray(calib, dtype=np.float64)
    return np.matmul(_r0_4x4(calib), _c2v_4x4(calib))


def _r0_4x4(calib):
    import numpy as np
    return np.concatenate([calib[2].reshape(4, 3), np.array([[0.0], [0.0], [0.0], [1.0]])], axis=1)


def _c2v_4x4(calib):
    import numpy as np
    return np.concatenate([calib[3].reshape(3, 4), np.array([[0.0, 0.0, 0.0, 1.0]])], axis=0)


# MV3D voxel config (MV3D_TF_release/lib/utils/config_voxels.py:49-59, DETECT_OBJ != 'Car')
# and the ranges construct_voxel.py:11-13 derives from it.
PED_RANGES = (0.0, 48 - 0.01, -20.0, 20 - 0.01, -1.0, 3 - 0.01)   # fwd, side, height
CAR_RANGES = (0.0, 70.4 - 0.01, -40.0, 40 - 0.01, -1.0, 3 - 0.01)


def mv3d_voxels_batch(points, point_offsets, img_index2=None, P=None, ranges=PED_RANGES, res=0.2, zres=0.4,
                      voxel_point_count=45, number_buffer=False, fv_aug=None):
    """The SHPL outputs of point_cloud_2_top_sparse (construct_voxel.py:37-162)
    for a batch of frames on the device. points [N, >=3] f64 camera frame;
    img_index2 [2, N] i64 (or P [F,3,4] f64 to project on the device);
    fv_aug [F,3] f64 (expansion_ratio, sx, sy): augment_fv's index transform
    (minibatch_mv3d_img.py:191-209) applied to img_index.
    Returns dict(img_index [3,N] f64, bv_index [N,2] i64, M_val [N] f64,
    frame_n [F]; number_buffer [N] i32 + frame_nvox [F]), capacity layout."""
    import ctypes

    import numpy as np
    import torch

    from . import _lib as L
    dev = points.device
    points = points.to(torch.float64).contiguous()
    point_offsets = point_offsets.to(torch.int64).contiguous()
    if img_index2 is not None:
        img_index2 = img_index2.to(torch.int64).contiguous()
    if P is not None:
        P = P.to(torch.float64).contiguous()
    if fv_aug is not None:
        fv_aug = torch.as_tensor(fv_aug, dtype=torch.float64).to(dev).reshape(-1, 3).contiguous()
    F = int(point_offsets.numel()) - 1
    N = int(points.shape[0])
    cap = max(N, 1)
    img = torch.empty((3, cap), dtype=torch.float64, device=dev)
    bv = torch.empty((cap, 2), dtype=torch.int64, device=dev)
    mv = torch.empty(cap, dtype=torch.float64, device=dev)
    fn = torch.empty(F, dtype=torch.int64, device=dev)
    nb = torch.empty(cap, dtype=torch.int32, device=dev) if number_buffer else None
    nvox = torch.empty(F, dtype=torch.int64, device=dev) if number_buffer else None
    nbytes = ctypes.c_size_t()
    L.check(L.lib().shpl_mv3d_workspace_bytes(N, ctypes.byref(nbytes)), "shpl_mv3d_workspace_bytes")
    ws = L.workspace(nbytes.value, dev)
    rng = np.ascontiguousarray(ranges, dtype=np.float64)
    L.check(L.lib().shpl_mv3d_voxels(F, L.ptr(point_offsets), N, L.ptr(points), int(points.stride(0)),
                                     L.ptr(img_index2), L.ptr(P), L.ptr(fv_aug), rng.ctypes.data_as(ctypes.c_void_p),
                                     float(res),
                                     float(zres), int(voxel_point_count), L.ptr(img), cap, L.ptr(bv), L.ptr(mv),
                                     L.ptr(fn), L.ptr(nb), L.ptr(nvox), L.ptr(ws), ws.numel(),
                                     L.stream_of(dev)), "shpl_mv3d_voxels")
    return {"img_index": img, "bv_index": bv, "M_val": mv, "frame_n": fn, "number_buffer": nb,
            "frame_nvox": nvox}


def mv3d_sparse_pooling_input(points, img_index2=None, P=None, ranges=PED_RANGES, res=0.2, zres=0.4,
                              voxel_point_count=45, fv_aug=None):
    """One frame: (img_index [3,n'], bv_index [n',2], M_val [n']) as
    point_cloud_2_top_sparse returns them (construct_voxel.py:156-162)."""
    import numpy as np
    import torch
    dev = torch.device("cuda", torch.cuda.current_device())
    pts = torch.as_tensor(np.ascontiguousarray(points, dtype=np.float64)).to(dev)
    off = torch.tensor([0, pts.shape[0]], dtype=torch.int64, device=dev)
    i2 = None if img_index2 is None else torch.as_tensor(np.ascontiguousarray(img_index2, dtype=np.int64)).to(dev)
    Pd = None if P is None else torch.as_tensor(np.asarray(P, dtype=np.float64).reshape(1, 12)).to(dev)
    out = mv3d_voxels_batch(pts, off, i2, Pd, ranges, res, zres, voxel_point_count,
                            fv_aug=None if fv_aug is None else np.asarray(fv_aug, dtype=np.float64).reshape(1, 3))
    k = int(out["frame_n"][0].item())
    return out["img_index"][:, :k], out["bv_index"][:k], out["M_val"][:k]
