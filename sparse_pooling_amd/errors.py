"""Exceptions mirroring the reference's failure modes."""


class InvalidArgumentError(ValueError):
    """What TF-CPU raises (tf.errors.InvalidArgumentError) for an out-of-range
    GatherNd / SparseTensorDenseMatMul / ScatterNd index, a values/indices
    length mismatch or an inconsistent reshape, at the reference's call sites
    (avod/avod/utils/sparse_pool_utils.py:101-103, :111-116)."""
