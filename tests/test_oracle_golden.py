"""The CPU oracle against the reference-generated golden fixtures (CPU only).

tests/golden/index_*.npz were produced by running the reference's own numpy
builders (tests/golden/make_golden.py); the oracle must reproduce them
bit-for-bit. The pooling restatement is cross-checked against an
independent numpy formulation of the same TF 1.8 semantics (np.add.at is
unbuffered and applies updates in index order, like TF's CPU loops).
"""
import glob
import os

import numpy as np
import pytest

from oracle import shpl_oracle as orc

INDEX_CASES = sorted(glob.glob(os.path.join(os.path.dirname(__file__), "golden", "index_*.npz")))


@pytest.mark.parametrize("path", INDEX_CASES, ids=[os.path.basename(p) for p in INDEX_CASES])
def test_index_builder_matches_reference(path):
    g = np.load(path)
    gen = orc.gen_sparse_pooling_input_avod(g["points"], g["voxel_indices"], g["P"],
                                            list(g["im_size"]), tuple(g["bv_size"]))
    np.testing.assert_array_equal(gen["bv_index"], g["gen_bv_index"].reshape(-1, 2))
    np.testing.assert_array_equal(gen["img_index"], g["gen_img_index"].reshape(3, -1))
    np.testing.assert_array_equal(gen["bv_size"], g["gen_bv_size"])
    np.testing.assert_array_equal(gen["img_size"], g["gen_img_size"])
    mval = g["M_val_in"] if "M_val_in" in g.files else None
    out = orc.produce_sparse_pooling_input(gen, M_val=mval, stride=tuple(g["stride"]))
    np.testing.assert_array_equal(out["Mij_pool"], g["Mij_pool"].reshape(-1, 2))
    np.testing.assert_array_equal(out["img_index_flip_pool"], g["img_index_flip_pool"].reshape(-1, 3))
    np.testing.assert_array_equal(out["M_size"], g["M_size"])
    np.testing.assert_array_equal(out["M_val"], g["M_val"])
    # quirk 6: the caller's img_index is mutated in place
    np.testing.assert_array_equal(gen["img_index"], g["mutated_img_index"].reshape(3, -1))


def _np_pool(mij, mval, R, img, idx):
    P = img[idx[:, 0], idx[:, 1], idx[:, 2]]
    out = np.zeros((R, img.shape[3]), np.float32)
    prod = (mval[:, None].astype(np.float32) * P[mij[:, 1]]).astype(np.float32)
    np.add.at(out, mij[:, 0], prod)
    return out


def _np_trans(mij, mval, bev_flat, idx, shape):
    order = np.lexsort((np.arange(len(mij)), mij[:, 0], mij[:, 1]))
    q = np.zeros((len(idx), bev_flat.shape[1]), np.float32)
    prod = (mval[order, None].astype(np.float32) * bev_flat[mij[order, 0]]).astype(np.float32)
    np.add.at(q, mij[order, 1], prod)
    out = np.zeros(tuple(shape[:3]) + (bev_flat.shape[1],), np.float32)
    np.add.at(out, (idx[:, 0], idx[:, 1], idx[:, 2]), q)
    return out


def _case(seed, n=600, R=900, hb=30, wb=30, h=20, w=25, c=8, dup=True):
    rng = np.random.default_rng(seed)
    idx = np.stack([np.zeros(n, np.int64), rng.integers(0, h, n), rng.integers(0, w, n)], 1)
    if dup:  # force heavy pixel and cell collisions
        idx[: n // 3, 1:] = idx[0, 1:]
    rows = rng.integers(0, hb * wb, n)
    rows[n // 2: n // 2 + 50] = rows[n // 2]
    mij = np.stack([rows, np.arange(n)], 1).astype(np.int64)
    mval = rng.uniform(0.1, 1.0, n).astype(np.float32)
    img = rng.standard_normal((1, h, w, c)).astype(np.float32)
    bev = rng.standard_normal((1, hb, wb, c)).astype(np.float32)
    return mij, mval, np.array([hb * wb, n]), img, bev, idx


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_pool_ops_two_restatements_agree(seed):
    mij, mval, msize, img, bev, idx = _case(seed)
    a = orc.sparse_pool_op(mij, mval, msize, img, idx)
    b = _np_pool(mij, mval, int(msize[0]), img, idx)
    np.testing.assert_array_equal(a, b)
    t = orc.sparse_pool_trans_op(mij, mval, msize, bev.reshape(-1, bev.shape[3]), idx, img.shape)
    u = _np_trans(mij, mval, bev.reshape(-1, bev.shape[3]), idx, img.shape)
    np.testing.assert_array_equal(t, u)


def test_pool_ops_noncanonical_M():
    """Shuffled nnz order and columns with several entries: trans sorts by (col,row)."""
    rng = np.random.default_rng(5)
    mij, mval, msize, img, bev, idx = _case(9, n=300)
    extra = np.stack([rng.integers(0, int(msize[0]), 200), rng.integers(0, 300, 200)], 1)
    mij = np.concatenate([mij, extra])[rng.permutation(500)]
    mval = rng.uniform(-1, 1, 500).astype(np.float32)
    a = orc.sparse_pool_op(mij, mval, msize, img, idx)
    np.testing.assert_array_equal(a, _np_pool(mij, mval, int(msize[0]), img, idx))
    bf = bev.reshape(-1, bev.shape[3])
    t = orc.sparse_pool_trans_op(mij, mval, msize, bf, idx, img.shape)
    np.testing.assert_array_equal(t, _np_trans(mij, mval, bf, idx, img.shape))


def test_pool_grads_are_adjoints():
    """<pool(x), y> == <x, pool^T(y)> (float64 check of the linear maps)."""
    mij, mval, msize, img, bev, idx = _case(3, dup=True)
    R, C = int(msize[0]), img.shape[3]
    y = np.random.default_rng(1).standard_normal((R, C)).astype(np.float32)
    fx = orc.sparse_pool_op(mij, mval, msize, img, idx)
    gy = orc.sparse_pool_grad_img(mij, mval, msize, y, idx, img.shape)
    np.testing.assert_allclose(np.sum(fx.astype(np.float64) * y), np.sum(img.astype(np.float64) * gy),
                               rtol=1e-5)
    z = np.random.default_rng(2).standard_normal(img.shape).astype(np.float32)
    tb = orc.sparse_pool_trans_op(mij, mval, msize, bev.reshape(R, C), idx, img.shape)
    gb = orc.sparse_pool_trans_grad_bev(mij, mval, msize, z, idx)
    np.testing.assert_allclose(np.sum(tb.astype(np.float64) * z),
                               np.sum(bev.reshape(R, C).astype(np.float64) * gb), rtol=1e-5)


def test_oob_raises_like_tf():
    mij, mval, msize, img, bev, idx = _case(4)
    bad = idx.copy()
    bad[7, 2] = img.shape[2]
    with pytest.raises(orc.OracleError):
        orc.sparse_pool_op(mij, mval, msize, img, bad)
    badm = mij.copy()
    badm[3, 0] = msize[0]
    with pytest.raises(orc.OracleError):
        orc.sparse_pool_op(badm, mval, msize, img, idx)
    with pytest.raises(orc.OracleError):
        orc.sparse_pool_trans_op(mij, mval, msize, bev.reshape(-1, img.shape[3]), bad, img.shape)


def test_projection_fma_chain_matches_numpy():
    """The oracle's dgemm emulation equals np.dot bit-for-bit (N >= 2)."""
    from sparse_pooling_amd import synth
    rng = np.random.default_rng(0)
    pts = np.stack([rng.uniform(-20, 20, 200000), rng.uniform(-2, 2, 200000),
                    rng.uniform(5, 70, 200000)], 1)
    P = synth.KITTI_P2
    uvw = P @ np.vstack((pts.T, np.ones(len(pts))))
    u = uvw[0] / uvw[2]
    v = uvw[1] / uvw[2]
    W, H = 1e9, 1e9  # keep everything: compare rounded indices of all points
    pts_in = pts[(u >= 0) & (v >= 0)]
    g = orc.gen_sparse_pooling_input_avod(pts_in, np.zeros((len(pts_in), 2), np.int64), P, [W, H],
                                          (10, 10))
    ok = (u >= 0) & (v >= 0)
    np.testing.assert_array_equal(g["img_index"][0], np.round(u[ok]))
    np.testing.assert_array_equal(g["img_index"][1], np.round(v[ok]))


def test_bev_slices_oracle_matches_reference(golden_dir):
    g = np.load(os.path.join(golden_dir, "bev_slices.npz"))
    hm, dm, vox, upts = orc.bev_slices(g["point_cloud"], g["ground_plane"], g["area_extents"],
                                       float(g["voxel_size"]), float(g["height_lo"]), float(g["height_hi"]),
                                       int(g["num_slices"]))
    np.testing.assert_array_equal(vox, g["voxel_indices"])
    np.testing.assert_array_equal(upts, g["pts_in_voxel"])
    np.testing.assert_array_equal(hm, g["height_maps"])
    np.testing.assert_array_equal(dm, g["density_map"])


@pytest.mark.parametrize("name", ["mv3d_voxel.npz", "mv3d_voxel_dense.npz"])
def test_mv3d_oracle_matches_reference(golden_dir, name):
    path = os.path.join(golden_dir, name)
    if not os.path.exists(path):
        pytest.skip("golden not generated")
    g = np.load(path)
    img, bv, mv, nb = orc.mv3d_voxels(g["points"], g["img_index2"], **orc.MV3D_PED)
    np.testing.assert_array_equal(img, g["img_index"])
    np.testing.assert_array_equal(bv, g["bv_index"])
    np.testing.assert_array_equal(mv, g["M_val"])
    np.testing.assert_array_equal(nb, g["number_buffer"])


# ---------------------------------------------------------------- KITTI loader (§8f item 3)

def test_kitti_host_readers_vs_reference_golden(kitti_dir):
    from sparse_pooling_amd import kitti
    d, g = kitti_dir
    for idx in (7, 8):
        fc = kitti.read_calibration(os.path.join(d, "calib"), idx)
        np.testing.assert_array_equal(fc.p2, g[f"{idx}_p2"])
        np.testing.assert_array_equal(fc.r0_rect, g[f"{idx}_r0_rect"])
        np.testing.assert_array_equal(fc.tr_velodyne_to_cam, g[f"{idx}_tr"])
        gp = kitti.get_road_plane(idx, os.path.join(d, "planes"))
        np.testing.assert_array_equal(gp, g[f"{idx}_ground_plane"])
        np.testing.assert_array_equal(kitti.flip_ground_plane(gp), g[f"{idx}_flip_ground_plane"])
        np.testing.assert_array_equal(kitti.flip_stereo_calib_p2(fc.p2, tuple(g[f"{idx}_image_shape"])),
                                      g[f"{idx}_flip_p2"])
        x, y, z, i = kitti.read_lidar(os.path.join(d, "velodyne"), idx)
        np.testing.assert_array_equal(np.stack([x, y, z, i], 1), g[f"{idx}_velo"])
        np.testing.assert_array_equal(kitti.rect_matrix(fc), orc.rect_matrix(fc.r0_rect, fc.tr_velodyne_to_cam))
    assert kitti.read_lidar(os.path.join(d, "velodyne"), 99) == []


def test_kitti_oracle_vs_reference_golden(kitti_dir):
    """get_lidar_point_cloud with and without the image filter, and flip_point_cloud,
    restated in C, against the reference run on the same files."""
    _, g = kitti_dir
    for idx in (7, 8):
        rect = orc.rect_matrix(g[f"{idx}_r0_rect"], g[f"{idx}_tr"])
        h, w = g[f"{idx}_image_shape"]
        pc = orc.velo_to_cam(g[f"{idx}_velo"], rect, g[f"{idx}_p2"], [w, h])
        np.testing.assert_array_equal(pc, g[f"{idx}_point_cloud"])
        np.testing.assert_array_equal(orc.velo_to_cam(g[f"{idx}_velo"], rect), g[f"{idx}_point_cloud_all"])
        np.testing.assert_array_equal(orc.velo_to_cam(g[f"{idx}_velo"], rect, g[f"{idx}_p2"], [w, h], flip=True),
                                      g[f"{idx}_flip_point_cloud"])


def test_kitti_single_column_oracle_vs_reference_golden(golden_dir):
    """One-point scan and a scan with one point in front of the camera: numpy's
    products have one column (dgemv order) -- pinned by the reference's output."""
    g = np.load(os.path.join(golden_dir, "kitti_single.npz"))
    h, w = g["image_shape"]
    for idx in (0, 1):
        rect = orc.rect_matrix(g[f"{idx}_r0_rect"], g[f"{idx}_tr"])
        np.testing.assert_array_equal(orc.velo_to_cam(g[f"{idx}_velo"], rect, g[f"{idx}_p2"], [w, h]),
                                      g[f"{idx}_point_cloud"])
        np.testing.assert_array_equal(orc.velo_to_cam(g[f"{idx}_velo"], rect), g[f"{idx}_point_cloud_all"])


def test_single_column_goldens_discriminate_the_order(golden_dir):
    """The single-column goldens are not satisfied by dgemm's FMA chain: evaluated
    that way the one-point frames round / clip differently, and the one-point scan's
    camera coordinates differ -- so passing them pins dgemv's order."""
    from fractions import Fraction

    def chain(p, a):
        s = p[0] * a[0]
        for k in range(1, 4):
            s = float(Fraction(p[k]) * Fraction(a[k]) + Fraction(s))
        return s
    for name in ("index_single_tie.npz", "index_single_clip.npz"):
        g = np.load(os.path.join(golden_dir, name))
        a = [*g["points"][0], 1.0]
        u = chain(g["P"][0], a) / chain(g["P"][2], a)
        v = chain(g["P"][1], a) / chain(g["P"][2], a)
        W, H = g["im_size"]
        inside = 0 <= u < W - 1 and 0 <= v < H - 1
        if not inside:
            assert g["gen_bv_index"].reshape(-1, 2).shape[0] == 1   # the reference kept it
        else:
            assert np.round(u) != g["gen_img_index"].reshape(3, -1)[0, 0]
    k = np.load(os.path.join(golden_dir, "kitti_single.npz"))
    rect = orc.rect_matrix(k["0_r0_rect"], k["0_tr"])
    a = [float(x) for x in k["0_velo"][0, :3]] + [1.0]
    cam = [chain(rect[r], a) for r in range(3)]
    assert cam != list(k["0_point_cloud_all"][:, 0])
