"""Device BEV slice maps + SHPL voxel indices.

``BevSlices`` mirrors avod.core.bev_generators.bev_slices.BevSlices
(avod/avod/core/bev_generators/bev_slices.py:8-156): same constructor config
fields (``height_lo``, ``height_hi``, ``num_slices``) and the same
``generate_bev(source, point_cloud, ground_plane, area_extents, voxel_size,
output_indices)`` contract, computed by ``shpl_bev_slices`` on the GPU.
``bev_slices_batch`` runs many frames in one launch and feeds the batched
index builder directly (capacity layout, no host round trip).

Reference bug not replicated: a slice with <= 1 point reuses the previous
slice's voxel grid in the reference (bev_slices.py:79-93); here every slice
is voxelized from its own points.
"""
from __future__ import annotations

import numpy as np
import torch

from . import _lib as L


def slice_bounds(height_lo, height_hi, num_slices):
    """Per-slice plane offsets exactly as bev_slices.py:30-31 and :66-67 compute them."""
    hpd = (height_hi - height_lo) / num_slices
    lo = [height_lo + s * hpd for s in range(num_slices)]
    return hpd, lo, [v + hpd for v in lo]


def density_table(norm_value):
    """min(1, log(n + 1) / norm_value) for n = 0..15 (bev_generator.py:33-34);
    counts of 15 and more saturate at 1.0 for norm_value = log(16)."""
    t = np.minimum(1.0, np.log(np.arange(16) + 1) / norm_value)
    if not t[15] >= 1.0:
        raise ValueError("density table needs norm_value <= log(16)")
    return np.ascontiguousarray(t, dtype=np.float64)


def grid_divisions(area_extents, voxel_size):
    ext = np.asarray(area_extents, dtype=np.float64).reshape(3, 2)
    min_x, min_z = np.floor(ext[0, 0] / voxel_size), np.floor(ext[2, 0] / voxel_size)
    nx = int(np.ceil(ext[0, 1] / voxel_size - 1) - min_x + 1)
    nz = int(np.ceil(ext[2, 1] / voxel_size - 1) - min_z + 1)
    return nx, nz


class BevBatch:
    def __init__(self, voxel_indices, pts_in_voxel, frame_nvox, height_maps, density_map, err, call=None):
        self.voxel_indices, self.pts_in_voxel, self.frame_nvox = voxel_indices, pts_in_voxel, frame_nvox
        self.height_maps, self.density_map, self.err = height_maps, density_map, err
        self._call = call  # the voxelizer call's arguments, for write_maps

    def write_maps(self, height_maps, density_map, zero=True):
        """The height / density maps of this batch (shpl_bev_maps) into the given [F,S,nz,nx] /
        [F,nz,nx] f64 tensors, on the current stream, from the sorted words the voxelizer left in its
        workspace (the workspace must not be reused in between): bitwise the maps bev_slices_batch
        writes with maps=True."""
        c = self._call
        nx, nz = grid_divisions(c["ext"].reshape(3, 2), c["vs"])
        for t, shape in ((height_maps, (c["F"], c["S"], nz, nx)), (density_map, (c["F"], nz, nx))):
            if t is not None and (t.dtype != torch.float64 or not t.is_contiguous() or tuple(t.shape) != shape
                                  or t.device != c["pts"].device):
                raise ValueError(f"map tensors must be contiguous f64 {shape} on {c['pts'].device}, "
                                 f"got {tuple(t.shape)} {t.dtype}")
        L.check(L.lib().shpl_bev_maps(c["F"], L.ptr(c["off"]), c["N"], L.ptr(c["pts"]), L.F64, L.ptr(c["planes"]),
                                      c["p"](c["ext"]), c["vs"], c["S"], c["p"](c["lo"]), c["p"](c["hi"]), c["hlo"],
                                      c["hhi"], c["hpd"], c["p"](c["table"]), L.ptr(height_maps),
                                      L.ptr(density_map), int(bool(zero)), L.ptr(c["ws"]), c["ws"].numel(),
                                      L.stream_of(c["pts"].device)), "shpl_bev_maps")
        self.height_maps, self.density_map = height_maps, density_map
        return height_maps, density_map

    def write_bev_input(self, bev_input):
        """The network's BEV input of this batch (shpl_bev_input) into the given [F,nz,nx,S+1] f32 tensor:
        np.dstack((*height_maps, density_map)) (kitti_dataset.py:368) as the tf.float32 placeholder holds it
        (each map value rounded to f32 once), from the voxelizer's sorted words like write_maps."""
        c = self._call
        nx, nz = grid_divisions(c["ext"].reshape(3, 2), c["vs"])
        shape = (c["F"], nz, nx, c["S"] + 1)
        if (bev_input.dtype != torch.float32 or not bev_input.is_contiguous() or tuple(bev_input.shape) != shape
                or bev_input.device != c["pts"].device):
            raise ValueError(f"bev_input must be a contiguous f32 {shape} tensor on {c['pts'].device}, "
                             f"got {tuple(bev_input.shape)} {bev_input.dtype}")
        L.check(L.lib().shpl_bev_input(c["F"], L.ptr(c["off"]), c["N"], L.ptr(c["pts"]), L.F64, L.ptr(c["planes"]),
                                       c["p"](c["ext"]), c["vs"], c["S"], c["p"](c["lo"]), c["p"](c["hi"]), c["hlo"],
                                       c["hhi"], c["hpd"], c["p"](c["table"]), L.ptr(bev_input), L.ptr(c["ws"]),
                                       c["ws"].numel(), L.stream_of(c["pts"].device)), "shpl_bev_input")
        self.bev_input = bev_input
        return bev_input


def bev_slices_batch(points, point_offsets, planes, area_extents, voxel_size, height_lo, height_hi,
                     num_slices, norm_value=np.log(16), maps=True, ws=None, point_counts=None):
    """points [N,3] f64 (camera frame), point_offsets [F+1] i64, planes [F,4] f64 -- all on the device;
    point_counts [F] i64: only the first count[f] points of each frame are live (shpl_velo_to_cam output).
    Returns a BevBatch; frame f's voxels are rows [off[f], off[f] + frame_nvox[f])."""
    dev = points.device
    F = int(point_offsets.numel()) - 1
    N = int(points.shape[0])
    if points.dtype != torch.float64:
        raise TypeError("BEV slicing runs on f64 camera-frame points, as the reference does")
    points = points.contiguous()
    point_offsets = point_offsets.to(torch.int64).contiguous()
    planes = planes.to(torch.float64).contiguous()
    if point_counts is not None:
        point_counts = point_counts.to(torch.int64).contiguous()
    nx, nz = grid_divisions(area_extents, voxel_size)
    hpd, lo, hi = slice_bounds(float(height_lo), float(height_hi), int(num_slices))
    ext = np.ascontiguousarray(np.asarray(area_extents, dtype=np.float64).reshape(6))
    lo_a, hi_a = np.ascontiguousarray(lo, dtype=np.float64), np.ascontiguousarray(hi, dtype=np.float64)
    table = density_table(norm_value)
    vox = torch.empty((max(N, 1), 2), dtype=torch.int32, device=dev)
    upts = torch.empty((max(N, 1), 3), dtype=torch.float64, device=dev)
    nvox = torch.empty(F, dtype=torch.int64, device=dev)
    hm = torch.empty((F, num_slices, nz, nx), dtype=torch.float64, device=dev) if maps else None
    dm = torch.empty((F, nz, nx), dtype=torch.float64, device=dev) if maps else None
    err = torch.zeros(1, dtype=torch.int32, device=dev)
    if ws is None:
        import ctypes
        nb = ctypes.c_size_t()
        L.check(L.lib().shpl_bev_workspace_bytes(N, int(num_slices), ctypes.byref(nb)), "shpl_bev_workspace_bytes")
        ws = L.workspace(nb.value, dev)
    p = lambda a: a.ctypes.data_as(L.ctypes.c_void_p)  # noqa: E731
    L.check(L.lib().shpl_bev_slices(F, L.ptr(point_offsets), L.ptr(point_counts), N, L.ptr(points), L.F64, L.ptr(planes), p(ext),
                                    float(voxel_size), int(num_slices), p(lo_a), p(hi_a), float(height_lo),
                                    float(height_hi), float(hpd), p(table), L.ptr(vox), L.ptr(upts), L.ptr(nvox),
                                    L.ptr(hm), L.ptr(dm), L.ptr(err), L.ptr(ws), ws.numel(),
                                    L.stream_of(dev)), "shpl_bev_slices")
    call = dict(F=F, off=point_offsets, N=N, pts=points, planes=planes, p=p, ext=ext, vs=float(voxel_size),
                S=int(num_slices), lo=lo_a, hi=hi_a, hlo=float(height_lo), hhi=float(height_hi), hpd=float(hpd),
                table=table, ws=ws)
    return BevBatch(vox, upts, nvox, hm, dm, err, call)


class BevSlices:
    """avod/avod/core/bev_generators/bev_slices.py:8-156 on the GPU."""

    NORM_VALUES = {'lidar': np.log(16)}

    def __init__(self, config, kitti_utils=None):
        self.height_lo = config.height_lo
        self.height_hi = config.height_hi
        self.num_slices = config.num_slices
        self.kitti_utils = kitti_utils
        self.height_per_division = (self.height_hi - self.height_lo) / self.num_slices

    def generate_bev(self, source, point_cloud, ground_plane, area_extents, voxel_size, output_indices=False):
        """point_cloud (3, N) camera frame. Returns {'height_maps': [S x (nz, nx)], 'density_map': (nz, nx)}
        (device f64 tensors, rotated like the reference) and, with output_indices,
        also voxel_indices [M,2] and pts_in_voxel [M,3]."""
        dev = torch.device("cuda", torch.cuda.current_device())
        pc = point_cloud if isinstance(point_cloud, torch.Tensor) else torch.as_tensor(np.asarray(point_cloud))
        pts = pc.to(device=dev, dtype=torch.float64).t().contiguous()
        off = torch.tensor([0, pts.shape[0]], dtype=torch.int64, device=dev)
        plane = torch.as_tensor(np.asarray(ground_plane, dtype=np.float64).reshape(1, 4)).to(dev)
        b = bev_slices_batch(pts, off, plane, area_extents, voxel_size, self.height_lo, self.height_hi,
                             self.num_slices, self.NORM_VALUES[source])
        bev_maps = {'height_maps': [b.height_maps[0, s] for s in range(self.num_slices)],
                    'density_map': b.density_map[0]}
        if not output_indices:
            return bev_maps
        m = int(b.frame_nvox[0].item())
        return bev_maps, b.voxel_indices[:m].to(torch.int64), b.pts_in_voxel[:m]
