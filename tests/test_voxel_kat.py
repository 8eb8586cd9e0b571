"""The reference's VoxelGrid2D known-answer tests
(avod/wavedata/wavedata/tools/core/voxel_grid_2d_test.py:13-79), restated
through the path's voxelizer (BevSlices.generate_bev, bev_slices.py:58-154,
which calls voxelize_2d with the area extents). The inputs are that test's 12
corner points and its 70000-point extents case; the expectations are its own
(voxel size 0.1, 800 x 700 cells for the points' span, 1000 x 700 for the
[-50, 50] extents, filled cells at floor(p * 10) + [400, 0, 0]), carried into
generate_bev's output conventions: indices (x, nz - z) (bev_slices.py:106-108),
maps transposed and flipped (bev_slices.py:117, bev_generator.py:39), the
voxel's height that of its lowest-y point (voxel_grid_2d.py:73,108-112),
density min(1, ln(n + 1) / ln 16) (bev_generator.py:35, bev_slices.py:11).
generate_bev's slice filter keeps points strictly inside the extents
(obj_utils.py:465-470), so the KAT's z = 0 corners, on the extents' boundary,
drop out: that edge is part of what is checked.

The CPU case checks the oracle; the GPU case runs the device voxelizer
(shpl_bev_slices through bev.BevSlices) on the same inputs.
"""
import types

import numpy as np
import pytest

from oracle import shpl_oracle as orc

KAT_POINTS = np.array([[-39.99, 4.99, 0], [39.99, 4.99, 0], [-39.99, -4.99, 0], [39.99, -4.99, 0],
                       [-39.99, 4.99, 69.99], [39.99, 4.99, 69.99], [-39.99, -4.99, 69.99],
                       [39.99, -4.99, 69.99], [-39.99, 4.99, 69.99], [39.99, 4.99, 69.99],
                       [-39.99, -4.99, 69.99], [39.99, -4.99, 69.99]])
PLANE = np.array([0.0, -1.0, 0.0, 0.0])  # height above ground = -y
EXT40 = np.array([[-40.0, 40.0], [-5.0, 5.0], [0.0, 70.0]])
EXT50 = np.array([[-50.0, 50.0], [-5.0, 5.0], [0.0, 70.0]])
VS = 0.1


def _kat_expected():
    # voxels in lexsort order (x, then z): the cells (x, z) = floor(p * 10) + [400, 0] of the z = 69.99
    # corners (the z = 0 ones lie on the extents' boundary), each represented by its y = -4.99 point, 4 points each
    cells = [(0, 699, 4), (799, 699, 4)]
    vox = np.array([[x, 700 - z] for x, z, _ in cells])
    upts = np.array([[-39.99, -4.99, 69.99], [39.99, -4.99, 69.99]])
    hm = np.zeros((1, 700, 800))
    dm = np.zeros((700, 800))
    for x, z, n in cells:
        hm[0, 699 - z, x] = (4.99 + 5.0) / 10.0
        dm[699 - z, x] = min(1.0, np.log(n + 1) / np.log(16))
    return hm, dm, vox, upts


def _random_case():
    rng = np.random.default_rng(70000)
    pts = rng.random((70000, 3)) * [80, 8, 60] - [40, 4, 0]
    d = np.floor(pts / VS).astype(np.int64)
    cells = np.unique(np.stack([d[:, 0] + 500, 700 - d[:, 2]], 1), axis=0)
    return pts, cells


def _check_kat(hm, dm, vox, upts):
    ehm, edm, evox, eupts = _kat_expected()
    assert hm.shape == ehm.shape and dm.shape == edm.shape
    np.testing.assert_array_equal(np.asarray(vox), evox)
    np.testing.assert_allclose(np.asarray(upts), eupts, rtol=0, atol=1e-12)
    np.testing.assert_allclose(np.asarray(hm), ehm, rtol=0, atol=1e-12)
    np.testing.assert_allclose(np.asarray(dm), edm, rtol=0, atol=1e-12)


def _check_random(hm, vox, cells):
    assert np.asarray(hm).shape == (1, 700, 1000)  # num_divisions [1000, 1, 700]
    got = np.unique(np.asarray(vox), axis=0)
    np.testing.assert_array_equal(got, cells)


def test_voxel_grid_kat_oracle():
    _check_kat(*orc.bev_slices(KAT_POINTS.T, PLANE, EXT40, VS, -5.0, 5.0, 1))


def test_voxel_grid_extents_oracle():
    pts, cells = _random_case()
    hm, _, vox, _ = orc.bev_slices(pts.T, PLANE, EXT50, VS, -5.0, 5.0, 1)
    _check_random(hm, vox, cells)


def _device(pts, ext):
    import torch
    from sparse_pooling_amd import bev
    cfg = types.SimpleNamespace(height_lo=-5.0, height_hi=5.0, num_slices=1)
    maps, vox, upts = bev.BevSlices(cfg).generate_bev("lidar", pts.T, PLANE, ext, VS, output_indices=True)
    torch.cuda.synchronize()
    f = lambda t: t.cpu().numpy() if hasattr(t, "cpu") else np.asarray(t)
    return np.stack([f(m) for m in maps["height_maps"]]), f(maps["density_map"]), f(vox), f(upts)


@pytest.mark.gpu
def test_voxel_grid_kat_device():
    _check_kat(*_device(KAT_POINTS, EXT40))


@pytest.mark.gpu
def test_voxel_grid_extents_device():
    pts, cells = _random_case()
    hm, dm, vox, upts = _device(pts, EXT50)
    _check_random(hm, vox, cells)
    ohm, odm, ovox, oupts = orc.bev_slices(pts.T, PLANE, EXT50, VS, -5.0, 5.0, 1)
    np.testing.assert_array_equal(vox, ovox)
    np.testing.assert_array_equal(upts, oupts)
    np.testing.assert_array_equal(hm, ohm)
    np.testing.assert_array_equal(dm, odm)
