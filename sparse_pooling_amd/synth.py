"""Seeded synthetic KITTI-shaped SHPL frames.

There is no network and no KITTI data on the GPU box, so every test and the
bench draw frames from this generator:

* ``P`` is a KITTI-like left colour camera matrix ``P2`` (3x4, f64);
* points are camera-frame ``x~U(-20,20), y~U(-2,2), z~U(5,70)`` and are
  re-drawn until exactly ``n_points`` of them survive the image clip of
  ``clip3DwithinImage`` (avod/avod/utils/transform.py:28-40), so ``nnz`` is
  controlled;
* voxel indices are ``[:,0]~U{0..Wb-1}``, ``[:,1]~U{1..Hb}`` -- the value
  ``Hb`` is out of range after flattening and exercises the reference's
  ``ind_inside`` drop (avod/avod/utils/sparse_pool_utils.py:44);
* features are ``N(0,1)`` NHWC.

Only numpy is used here; the device path receives these arrays as inputs.
"""
from __future__ import annotations

from dataclasses import dataclass, field

import numpy as np

# KITTI-like P2.
KITTI_P2 = np.array(
    [[721.5377, 0.0, 609.5593, 44.85728],
     [0.0, 721.5377, 172.854, 0.2163791],
     [0.0, 0.0, 1.0, 0.002745884]], dtype=np.float64)


@dataclass
class FrameSpec:
    """Shape of one SHPL frame (names follow BASELINE.json configs)."""
    n_points: int
    im_size: tuple          # (W, H) of the image the projection is clipped to
    bv_size: tuple          # (H, W) of the full-resolution BEV grid
    stride: tuple = (1, 1)  # (s_img, s_bv) as passed to produce_sparse_pooling_input
    c_bev: int = 32
    c_img: int = 32

    @property
    def img_feat_hw(self):
        s = self.stride[0]
        return (int(np.floor(self.im_size[1] / s)), int(np.floor(self.im_size[0] / s)))

    @property
    def bev_feat_hw(self):
        s = self.stride[1]
        return (int(np.floor(self.bv_size[0] / s)), int(np.floor(self.bv_size[1] / s)))


# BASELINE.json configs expressed as frame specs.
CONFIG1 = FrameSpec(2000, (1200, 360), (704, 800), (4, 4), 16, 16)
CONFIG2 = FrameSpec(20000, (1200, 360), (704, 800), (1, 1), 32, 32)
CONFIG3 = FrameSpec(20000, (1200, 360), (704, 800), (8, 8), 256, 256)
CONFIG5 = FrameSpec(40000, (1200, 360), (704, 800), (1, 1), 64, 64)
# Not a BASELINE config: the RetinaNet P2 fusion (avod/avod/core/models/retinanet_model.py:320-348 with
# configs/retinanet_car_SHPL.config: SHPL at pyramid level P2, stride 4, FPN 256 channels both sides,
# bv_index None -- the img->BEV direction only), BEV 176x200, image 90x300, f32.
CONFIG6 = FrameSpec(20000, (1200, 360), (704, 800), (4, 4), 256, 256)
CONFIGS = {1: CONFIG1, 2: CONFIG2, 3: CONFIG3, 5: CONFIG5, 6: CONFIG6}


def _clip_mask(pts, P, im_size):
    mat = np.vstack((pts.T, np.ones(pts.shape[0])))
    uvw = P @ mat
    u = uvw[0] / uvw[2]
    v = uvw[1] / uvw[2]
    return (u < im_size[0] - 1) & (u >= 0) & (v >= 0) & (v < im_size[1] - 1)


@dataclass
class Frame:
    points: np.ndarray          # [N,3] f64 camera frame
    voxel_indices: np.ndarray   # [N,2] int64 (x, z_rot) BEV voxel indices
    P: np.ndarray               # [3,4] f64
    spec: FrameSpec
    extra: dict = field(default_factory=dict)


def make_frame(spec: FrameSpec, seed: int, P: np.ndarray = KITTI_P2,
               n_outside: int = 0) -> Frame:
    """One seeded frame with exactly ``spec.n_points`` points inside the clip
    window, plus ``n_outside`` points that the clip must drop (interleaved)."""
    rng = np.random.default_rng(seed)
    keep = []
    have = 0
    while have < spec.n_points:
        m = max(1024, 2 * (spec.n_points - have))
        pts = np.stack([rng.uniform(-20, 20, m), rng.uniform(-2, 2, m),
                        rng.uniform(5, 70, m)], axis=1)
        ok = _clip_mask(pts, P, spec.im_size)
        pts = pts[ok][: spec.n_points - have]
        keep.append(pts)
        have += pts.shape[0]
    pts = np.concatenate(keep, axis=0) if keep else np.zeros((0, 3))
    if n_outside:
        # behind the camera or far off to the side: projection falls outside
        out = np.stack([rng.uniform(60, 90, n_outside), rng.uniform(-2, 2, n_outside),
                        rng.uniform(5, 10, n_outside)], axis=1)
        pos = np.sort(rng.choice(pts.shape[0] + n_outside, n_outside, replace=False))
        pts = np.insert(pts, pos - np.arange(n_outside), out, axis=0)
    n = pts.shape[0]
    hb, wb = spec.bv_size
    vox = np.stack([rng.integers(0, wb, n), rng.integers(1, hb + 1, n)], axis=1).astype(np.int64)
    return Frame(np.ascontiguousarray(pts, dtype=np.float64), vox, np.array(P, dtype=np.float64), spec)


def make_features(shape, seed: int, dtype=np.float32) -> np.ndarray:
    rng = np.random.default_rng(seed)
    return rng.standard_normal(shape, dtype=np.float32).astype(dtype)


class StereoCalib:
    """Minimal stand-in for wavedata's StereoCalib: only ``.p2`` is read by
    gen_sparse_pooling_input_avod (avod/avod/utils/sparse_pool_utils.py:12)."""

    def __init__(self, p2):
        self.p2 = np.asarray(p2, dtype=np.float64)


# Area / slicing of the reference's SHPL configs (e.g. configs/retinanet_car_SHPL.config:115-124)
AREA_EXTENTS = np.array([[-40.0, 40.0], [-5.0, 3.0], [0.0, 70.0]])
GROUND_PLANE = np.array([0.0, -1.0, 0.0, 1.65])
VOXEL_SIZE, HEIGHT_LO, HEIGHT_HI, NUM_SLICES = 0.1, -0.2, 2.3, 5


def make_cloud(n, seed, plane=GROUND_PLANE):
    """A raw camera-frame LiDAR-like cloud (3, n): x across, y down, z forward,
    heights spread over the BEV slices above the ground plane, some points
    outside the area extents and the height range."""
    rng = np.random.default_rng(seed)
    x = rng.uniform(-42, 42, n)
    z = rng.uniform(-1, 72, n)
    h = rng.uniform(-0.6, 2.8, n)                  # height above the ground plane
    a, b, c, d = plane
    y = (h * np.sqrt(a * a + b * b + c * c) - a * x - c * z - d) / b
    return np.stack([x, y, z])


# KITTI object-detection calib layout (values of a typical left-camera setup), in file order.
KITTI_CALIB = {
    "P0": [7.215377e+02, 0, 6.095593e+02, 0, 0, 7.215377e+02, 1.728540e+02, 0, 0, 0, 1, 0],
    "P1": [7.215377e+02, 0, 6.095593e+02, -3.875744e+02, 0, 7.215377e+02, 1.728540e+02, 0, 0, 0, 1, 0],
    "P2": [7.215377e+02, 0, 6.095593e+02, 4.485728e+01, 0, 7.215377e+02, 1.728540e+02, 2.163791e-01,
           0, 0, 1, 2.745884e-03],
    "P3": [7.215377e+02, 0, 6.095593e+02, -3.395242e+02, 0, 7.215377e+02, 1.728540e+02, 2.199936e+00,
           0, 0, 1, 2.729905e-03],
    "R0_rect": [9.999239e-01, 9.837760e-03, -7.445048e-03, -9.869795e-03, 9.999421e-01, -4.278459e-03,
                7.402527e-03, 4.351614e-03, 9.999631e-01],
    "Tr_velo_to_cam": [7.533745e-03, -9.999714e-01, -6.166020e-04, -4.069766e-03, 1.480249e-02,
                       7.280733e-04, -9.998902e-01, -7.631618e-02, 9.998621e-01, 7.523790e-03,
                       1.480755e-02, -2.717806e-01],
    "Tr_imu_to_velo": [9.999976e-01, 7.553071e-04, -2.035826e-03, -8.086759e-01, -7.854027e-04,
                       9.998898e-01, -1.482298e-02, 3.195559e-01, 2.024406e-03, 1.482454e-02,
                       9.998881e-01, -7.997231e-01],
}
KITTI_IMAGE_SHAPE = (375, 1242)  # (h, w)
KITTI_PLANE = np.array([-1.851372e-02, -9.998285e-01, -5.362401e-04, 1.678541e+00])


def synthetic_scan(rng, n):
    """A 64-beam-like velodyne sweep in the lidar frame (x fwd, y left, z up), [n,4] f32 (x, y, z, i)."""
    az = rng.uniform(-np.pi, np.pi, n)
    el = np.deg2rad(rng.uniform(-24.8, 2.0, n))
    rng_m = rng.uniform(2.0, 80.0, n)
    xyz = np.stack([rng_m * np.cos(el) * np.cos(az), rng_m * np.cos(el) * np.sin(az), rng_m * np.sin(el)], 1)
    xyz[:, 2] = np.maximum(xyz[:, 2], -1.73 + rng.normal(0, 0.02, n))  # ground
    return np.concatenate([xyz, rng.uniform(0, 1, (n, 1))], 1).astype(np.float32)
