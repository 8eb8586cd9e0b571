"""MV3D_TF's SHPL entry points on MI355X.

* ``produce_sparse_pooling_input`` mirrors
  ``fusion_voxel_train.produce_sparse_pooling_input``
  (MV3D_TF_release/lib/networks/MV3D_voxel_train.py:89-91): same argument
  order, default stride ``[8, 2]`` (``_feat_stride_pool``: image stride 8,
  BEV stride 2, :14), returns ``(Mij, M_val, M_size, img_index_flip)``.
* ``sparse_pool`` mirrors the ``@layer sparse_pool`` of
  MV3D_TF_release/lib/networks/network.py:243-246:
  ``input = [M, img_features, img_index_flip]``.

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
