"""KITTI on-disk formats and the velodyne -> camera-frame loader.

Host side (file parsing, as the reference does it):
  read_calibration   avod/wavedata/wavedata/tools/core/calib_utils.py:55-112
  read_lidar         calib_utils.py:328-368   (velodyne .bin, f32 x 4)
  get_road_plane     avod/wavedata/wavedata/tools/obj_detection/obj_utils.py:271-303
  flip_stereo_calib_p2 / flip_ground_plane   avod/avod/datasets/kitti/kitti_aug.py:85-121
Device side (``shpl_velo_to_cam``, csrc/shpl_kitti.hip):
  lidar_to_cam_frame        calib_utils.py:371-410
  get_lidar_point_cloud     obj_utils.py:220-268 (z > 0, P2 projection, strict image bounds)
  flip_point_cloud          kitti_aug.py:24-29

``velo_to_cam_batch`` converts many scans in one pass into the capacity
layout that ``bev.bev_slices_batch(point_counts=...)`` consumes directly, so a
batch goes from raw scans to the fused SHPL layer without leaving the GPU
(``pipeline.FramePipeline.velo_step``).
"""
from __future__ import annotations

import ctypes
import os

import numpy as np
import torch

from . import _lib as L


class FrameCalibrationData:
    """calib_utils.FrameCalibrationData (calib_utils.py:7-50): p0-p3 (3x4), r0_rect (3x3),
    tr_velodyne_to_cam (3x4)."""

    def __init__(self):
        self.p0 = self.p1 = self.p2 = self.p3 = None
        self.r0_rect = None
        self.tr_velodyne_to_cam = None


def _row(line):
    # csv.reader(delimiter=' ') then float() of every field after the label (calib_utils.py:79-110)
    return [float(v) for v in line.rstrip("\n").split(" ")[1:]]


def read_calibration(calib_dir, img_idx):
    """calib_utils.read_calibration (calib_utils.py:55-112)."""
    with open(os.path.join(calib_dir, "%06d.txt" % img_idx)) as fh:
        rows = fh.readlines()
    fc = FrameCalibrationData()
    p_all = [np.reshape(_row(rows[i]), (3, 4)) for i in range(4)]
    fc.p0, fc.p1, fc.p2, fc.p3 = p_all
    fc.r0_rect = np.reshape(_row(rows[4]), (3, 3))
    fc.tr_velodyne_to_cam = np.reshape(_row(rows[5]), (3, 4))
    return fc


def read_lidar_xyzi(velo_dir, img_idx):
    """The velodyne scan as one [N,4] f32 array (calib_utils.read_lidar's file read); None if absent."""
    path = os.path.join(velo_dir, "%06d.bin" % img_idx)
    if not os.path.exists(path):
        return None
    return np.fromfile(path, np.single).reshape(-1, 4)


def read_lidar(velo_dir, img_idx):
    """calib_utils.read_lidar (calib_utils.py:328-368): x, y, z, i, or [] if the file is missing."""
    xyzi = read_lidar_xyzi(velo_dir, img_idx)
    if xyzi is None:
        return []
    return xyzi[:, 0], xyzi[:, 1], xyzi[:, 2], xyzi[:, 3]


def get_road_plane(img_idx, planes_dir):
    """obj_utils.get_road_plane (obj_utils.py:271-303): 4th line, normal up (+y down), unit normal."""
    with open(os.path.join(planes_dir, "%06d.txt" % img_idx)) as fh:
        lines = fh.readlines()
    plane = np.asarray([float(v) for v in lines[3].split()])
    if plane[1] > 0:
        plane = -plane
    return plane / np.linalg.norm(plane[0:3])


def flip_stereo_calib_p2(calib_p2, image_shape):
    """kitti_aug.flip_stereo_calib_p2 (kitti_aug.py:100-121); image_shape (h, w)."""
    flipped = np.copy(calib_p2)
    flipped[0, 2] = image_shape[1] - calib_p2[0, 2]
    flipped[0, 3] = -calib_p2[0, 3]
    return flipped


def flip_ground_plane(ground_plane):
    """kitti_aug.flip_ground_plane (kitti_aug.py:85-97)."""
    flipped = np.copy(ground_plane)
    flipped[0] = -ground_plane[0]
    return flipped


def rect_matrix(frame_calib):
    """Rows 0-2 of R0_rect4 . Tr_velo_to_cam4, formed exactly as lidar_to_cam_frame does
    (calib_utils.py:388-404); the per-point product runs on the device."""
    r0 = np.pad(frame_calib.r0_rect, ((0, 1), (0, 1)), "constant", constant_values=0)
    r0[3, 3] = 1
    tf = np.pad(frame_calib.tr_velodyne_to_cam, ((0, 1), (0, 0)), "constant", constant_values=0)
    tf[3, 3] = 1
    return np.ascontiguousarray(np.dot(r0, tf)[0:3])


class VeloBatch:
    def __init__(self, points, counts, point_offsets, err):
        self.points, self.counts, self.point_offsets, self.err = points, counts, point_offsets, err


def velo_to_cam_batch(xyzi, point_offsets, rect, P=None, im_size=None, min_intensity=None, flip=None,
                      max_points_per_frame=None, ws=None, out=None):
    """Device get_lidar_point_cloud over a batch of scans.

    xyzi [N,4] f32, point_offsets [F+1] i64, rect [F,3,4] f64 (``rect_matrix``),
    P [F,3,4] f64 and im_size [F,2] (w, h) -- both None: no FOV filter --, flip [F]
    (nonzero: kitti_aug.flip_point_cloud). All device tensors (or array-likes).
    Returns a VeloBatch: points [N,3] f64 with frame f's kept points at
    [off[f], off[f] + counts[f]) in scan order (NaN rows after)."""
    dev = xyzi.device
    xyzi = xyzi.to(torch.float32).contiguous()
    point_offsets = point_offsets.to(torch.int64).contiguous()
    F = int(point_offsets.numel()) - 1
    N = int(xyzi.shape[0])
    t = lambda a: None if a is None else torch.as_tensor(np.asarray(a) if not isinstance(a, torch.Tensor) else a)  # noqa: E731
    rect = t(rect).to(dev, torch.float64).reshape(F, 12).contiguous()
    if (P is None) != (im_size is None):
        raise ValueError("P and im_size go together (the FOV filter needs both)")
    if P is not None:
        P = t(P).to(dev, torch.float64).reshape(F, 12).contiguous()
        im_size = t(im_size).to(dev, torch.float64).reshape(F, 2).contiguous()
    if flip is not None:
        flip = t(flip).to(dev, torch.int32).reshape(F).contiguous()
    if max_points_per_frame is None:
        max_points_per_frame = int((point_offsets[1:] - point_offsets[:-1]).max().item()) if F else 0
    if ws is None:
        nb = ctypes.c_size_t()
        L.check(L.lib().shpl_velo_workspace_bytes(F, int(max_points_per_frame), ctypes.byref(nb)),
                "shpl_velo_workspace_bytes")
        ws = L.workspace(nb.value, dev)
    pts = out if out is not None else torch.empty((max(N, 1), 3), dtype=torch.float64, device=dev)
    counts = torch.empty(F, dtype=torch.int64, device=dev)
    err = torch.zeros(1, dtype=torch.int32, device=dev)
    L.check(L.lib().shpl_velo_to_cam(F, L.ptr(point_offsets), int(max_points_per_frame), L.ptr(xyzi), L.ptr(rect),
                                     L.ptr(P), L.ptr(im_size),
                                     float("nan") if min_intensity is None else float(min_intensity),
                                     L.ptr(flip), L.ptr(pts), L.ptr(counts), L.ptr(err), L.ptr(ws), ws.numel(),
                                     L.stream_of(dev)), "shpl_velo_to_cam")
    return VeloBatch(pts, counts, point_offsets, err)


def lidar_to_cam_frame(xyz_lidar, frame_calib):
    """calib_utils.lidar_to_cam_frame (calib_utils.py:371-410) on the device: [N,3] -> [N,3] f64."""
    dev = torch.device("cuda", torch.cuda.current_device())
    xyz = np.asarray(xyz_lidar)
    xyzi = np.zeros((xyz.shape[0], 4), np.float32)
    xyzi[:, :3] = xyz
    off = torch.tensor([0, xyz.shape[0]], dtype=torch.int64, device=dev)
    b = velo_to_cam_batch(torch.as_tensor(xyzi).to(dev), off, rect_matrix(frame_calib)[None])
    return b.points[:xyz.shape[0]]


def get_lidar_point_cloud(img_idx, calib_dir, velo_dir, im_size=None, min_intensity=None):
    """obj_utils.get_lidar_point_cloud (obj_utils.py:220-268) with the transform and the
    filter on the device: returns the (3, N') camera-frame cloud as a device f64 tensor.
    im_size [w, h]. min_intensity compares each kept point's own intensity (the
    reference's mask-length bug is not replicated)."""
    fc = read_calibration(calib_dir, img_idx)
    xyzi = read_lidar_xyzi(velo_dir, img_idx)
    dev = torch.device("cuda", torch.cuda.current_device())
    off = torch.tensor([0, xyzi.shape[0]], dtype=torch.int64, device=dev)
    filt = im_size is not None and len(im_size) > 0
    b = velo_to_cam_batch(torch.as_tensor(xyzi).to(dev), off, rect_matrix(fc)[None],
                          fc.p2[None] if filt else None, [list(im_size)] if filt else None, min_intensity)
    k = int(b.counts[0].item())
    return b.points[:k].t()


class KittiFrames:
    """A batch of KITTI samples laid out for the device: what KittiDataset.load_samples
    (kitti_dataset.py:285-311) gathers per sample before the BEV maps and the SHPL
    inputs are built -- the scans as one [N,4] f32 array with frame offsets, the
    per-frame lidar->camera matrices, P2, image sizes, ground planes and flips.

    image_shapes: (h, w) per sample (the reference reads them from the PNGs).
    flips: per-sample AUG_FLIPPING. The flipped P2 is the one the index builder
    gets here (the reference hands it the unflipped calib, kitti_dataset.py:376:
    SURVEY §8a quirk 3, a bug not replicated)."""

    def __init__(self, scans, calibs, planes, image_shapes, flips=None, device="cuda"):
        dev = torch.device(device)
        flips = list(flips) if flips is not None else [False] * len(scans)
        rects, p2s, p2_index, sizes, gps = [], [], [], [], []
        for fc, gp, shape, fl in zip(calibs, planes, image_shapes, flips):
            rects.append(rect_matrix(fc))
            p2s.append(fc.p2)  # the FOV filter projects with the file's P2 (before the flip)
            p2_index.append(flip_stereo_calib_p2(fc.p2, shape) if fl else fc.p2)
            gps.append(flip_ground_plane(gp) if fl else gp)
            sizes.append([shape[1], shape[0]])
        off = np.zeros(len(scans) + 1, np.int64)
        off[1:] = np.cumsum([s.shape[0] for s in scans])
        self.n_frames = len(scans)
        self.total_points = int(off[-1])
        self.max_points = int(max(s.shape[0] for s in scans)) if scans else 0
        self.xyzi = torch.as_tensor(np.concatenate(scans) if scans else np.zeros((0, 4), np.float32)).to(dev)
        self.point_offsets = torch.as_tensor(off).to(dev)
        self.rect = torch.as_tensor(np.stack(rects)).to(dev)
        self.P2_filter = torch.as_tensor(np.stack(p2s)).to(dev)
        self.P2 = torch.as_tensor(np.stack(p2_index)).to(dev)
        self.im_size = torch.as_tensor(np.asarray(sizes, np.float64)).to(dev)
        self.planes = torch.as_tensor(np.stack(gps)).to(dev)
        self.flip = torch.as_tensor(np.asarray(flips, np.int32)).to(dev)
        self.image_shapes = [tuple(s) for s in image_shapes]

    @classmethod
    def from_dirs(cls, calib_dir, velo_dir, planes_dir, indices, image_shapes, flips=None, device="cuda"):
        """Read the samples' calib / velodyne / planes files (KITTI layout)."""
        scans = [read_lidar_xyzi(velo_dir, idx) for idx in indices]
        calibs = [read_calibration(calib_dir, idx) for idx in indices]
        planes = [get_road_plane(idx, planes_dir) for idx in indices]
        return cls(scans, calibs, planes, image_shapes, flips, device)

    def point_clouds(self, ws=None, out=None):
        """All samples' camera-frame clouds (get_point_cloud + flip_point_cloud), capacity layout."""
        return velo_to_cam_batch(self.xyzi, self.point_offsets, self.rect, self.P2_filter, self.im_size,
                                 flip=self.flip, max_points_per_frame=self.max_points, ws=ws, out=out)


def synthetic_frames(n_frames, points_per_scan, seed=0, device="cuda", flips=None, frame_ids=None):
    """Seeded synthetic KITTI samples (synth.synthetic_scan, synth.KITTI_CALIB) for the bench.
    frame_ids: scan i is drawn from a generator seeded with (seed, frame_ids[i]), so a
    frame is the same whichever batch holds it; None: one generator for all scans."""
    from . import synth
    rng = np.random.default_rng(seed)
    fc = FrameCalibrationData()
    c = synth.KITTI_CALIB
    fc.p0, fc.p1, fc.p2, fc.p3 = (np.array(c[k]).reshape(3, 4) for k in ("P0", "P1", "P2", "P3"))
    fc.r0_rect = np.array(c["R0_rect"]).reshape(3, 3)
    fc.tr_velodyne_to_cam = np.array(c["Tr_velo_to_cam"]).reshape(3, 4)
    if frame_ids is None:
        scans = [synth.synthetic_scan(rng, points_per_scan) for _ in range(n_frames)]
    else:
        assert len(frame_ids) == n_frames
        scans = [synth.synthetic_scan(np.random.default_rng([seed, int(f)]), points_per_scan) for f in frame_ids]
    plane = synth.KITTI_PLANE / np.linalg.norm(synth.KITTI_PLANE[:3])
    return KittiFrames(scans, [fc] * n_frames, [plane] * n_frames, [synth.KITTI_IMAGE_SHAPE] * n_frames,
                       flips, device)
