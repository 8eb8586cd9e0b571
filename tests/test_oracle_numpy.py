"""The numpy restatement of the reference CPU path (oracle/shpl_numpy.py, the
bench's numpy cpu_baseline leg) against the reference-generated index goldens
and the C oracle (CPU only)."""
import glob
import os

import numpy as np
import pytest

from oracle import shpl_numpy as onp
from oracle import shpl_oracle as orc
from sparse_pooling_amd import synth

INDEX_CASES = sorted(glob.glob(os.path.join(os.path.dirname(__file__), "golden", "index_*.npz")))


@pytest.mark.parametrize("path", INDEX_CASES, ids=[os.path.basename(p) for p in INDEX_CASES])
def test_numpy_index_builder_matches_reference(path):
    g = np.load(path)
    gen = onp.gen_sparse_pooling_input_avod(g["points"], g["voxel_indices"], g["P"], list(g["im_size"]),
                                            tuple(g["bv_size"]))
    np.testing.assert_array_equal(gen["bv_index"], g["gen_bv_index"].reshape(-1, 2))
    np.testing.assert_array_equal(gen["img_index"], g["gen_img_index"].reshape(3, -1))
    mval = g["M_val_in"] if "M_val_in" in g.files else None
    out = onp.produce_sparse_pooling_input(gen, M_val=mval, stride=tuple(g["stride"]))
    np.testing.assert_array_equal(out["Mij_pool"], g["Mij_pool"].reshape(-1, 2))
    np.testing.assert_array_equal(out["img_index_flip_pool"], g["img_index_flip_pool"].reshape(-1, 3))
    np.testing.assert_array_equal(out["M_size"], g["M_size"])
    np.testing.assert_array_equal(gen["img_index"], g["mutated_img_index"].reshape(3, -1))


@pytest.mark.parametrize("dual", [False, True])
def test_numpy_layer_equals_c_oracle(dual):
    spec = synth.CONFIG1
    fr = synth.make_frame(spec, seed=3, n_outside=20)
    ref = orc.produce_sparse_pooling_input(
        orc.gen_sparse_pooling_input_avod(fr.points, fr.voxel_indices, fr.P, list(spec.im_size),
                                          tuple(spec.bv_size)), stride=spec.stride)
    got = onp.produce_sparse_pooling_input(
        onp.gen_sparse_pooling_input_avod(fr.points, fr.voxel_indices, fr.P, list(spec.im_size),
                                          tuple(spec.bv_size)), stride=spec.stride)
    for k in ("Mij_pool", "M_size", "img_index_flip_pool"):
        np.testing.assert_array_equal(got[k], ref[k])
    Hb, Wb = spec.bev_feat_hw
    Hi, Wi = spec.img_feat_hw
    bev = synth.make_features((1, Hb, Wb, spec.c_bev), 1)
    img = synth.make_features((1, Hi, Wi, spec.c_img), 2)
    a = orc.sparse_pool_layer(bev, img, ref["Mij_pool"], ref["M_val"], ref["M_size"], ref["img_index_flip_pool"],
                              dual=dual)
    b = onp.sparse_pool_layer(bev, img, got["Mij_pool"], got["M_val"], got["M_size"], got["img_index_flip_pool"],
                              dual=dual)
    for x, y in zip(a, b):
        np.testing.assert_array_equal(np.asarray(x).view(np.uint32), np.asarray(y).view(np.uint32))


def test_numpy_gradients_equal_c_oracle():
    rng = np.random.default_rng(4)
    n, R, h, w, c = 400, 300, 9, 13, 8
    idx = np.stack([np.zeros(n, np.int64), rng.integers(0, h, n), rng.integers(0, w, n)], 1)
    idx[: n // 3, 1:] = idx[0, 1:]
    mij = np.stack([rng.integers(0, R, n), np.arange(n)], 1).astype(np.int64)
    extra = np.stack([rng.integers(0, R, 100), rng.integers(0, n, 100)], 1)
    mij = np.concatenate([mij, extra])[rng.permutation(n + 100)]
    mval = rng.uniform(-1, 1, len(mij)).astype(np.float32)
    dY = rng.standard_normal((R, c)).astype(np.float32)
    dZ = rng.standard_normal((1, h, w, c)).astype(np.float32)
    a = orc.sparse_pool_grad_img(mij, mval, [R, n], dY, idx, (1, h, w, c))
    b = onp.sparse_pool_grad_img(mij, mval, [R, n], dY, idx, (1, h, w, c))
    np.testing.assert_array_equal(a.view(np.uint32), b.view(np.uint32))
    a = orc.sparse_pool_trans_grad_bev(mij, mval, [R, n], dZ, idx)
    b = onp.sparse_pool_trans_grad_bev(mij, mval, [R, n], dZ, idx)
    np.testing.assert_array_equal(a.view(np.uint32), b.view(np.uint32))
