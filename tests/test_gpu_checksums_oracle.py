"""The bench's stored per-frame checksum tables, pinned to the oracle.

bench.py reports ``frame_checksums.match_n1`` by comparing its per-frame output
checksums with ``profiles/frame_checksums.json``; a table there was written by
a GPU run (``bench.py --write-checksums``). This test recomputes every frame of
those tables with the CPU oracle (oracle/shpl_oracle.c: the reference's index
builder, avod/avod/utils/sparse_pool_utils.py:6-58, and TF 1.8's CPU pooling
order, :61-117) from the same inputs the bench draws -- ``synth.make_frame(spec,
seed=frame id, n_outside=200)`` and ``dist.fill_features`` on the device, copied
to the host -- and forms the same checksum (``dist.frame_checksums``: the int64
sum of the output elements' bit patterns, summed over the step's outputs). So
``match_n1`` means "equals the TF-order restatement", not "equals an earlier
GPU run". A table that disagrees with the oracle in any frame fails here.

Tables: config 2 (64 frames, bv_fused), config 3 (4 frames, bf16: both fused
forward outputs and both gradients), config 5 (64 frames, both fused forward
outputs), config 6 (the RetinaNet P2 shape, 64 frames, the first 16 recomputed), the raw-scan workload (64 scans of 120k points: velodyne -> camera
frame + FOV filter -> BEV slices -> index -> bv_fused)."""
import json
import os

import numpy as np
import pytest
import torch

from oracle import shpl_oracle as orc
from sparse_pooling_amd import dist as sd, synth

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DEV = torch.device("cuda", 0)


def _table(key):
    with open(os.path.join(ROOT, "profiles", "frame_checksums.json")) as fh:
        return json.load(fh)[key]


def _feats(shape, fid, seed, dtype=torch.float32):
    """One frame's features exactly as bench.py draws them (on the device), as host f32."""
    t = sd.fill_features(torch.empty((1,) + tuple(shape), dtype=dtype, device=DEV), [fid], seed)
    return t.float().cpu().numpy()


def _cs32(a):
    """dist.frame_checksums of one f32 frame, on the host."""
    return int(np.ascontiguousarray(a, dtype=np.float32).view(np.int32).astype(np.int64).sum())


def _cs16(a):
    """dist.frame_checksums of one bf16 frame (the oracle's f32 result rounded once, RNE)."""
    return int(orc.to_bf16_bits(np.ascontiguousarray(a, dtype=np.float32)).view(np.int16).astype(np.int64).sum())


def _index(fr, spec):
    g = orc.gen_sparse_pooling_input_avod(fr.points, fr.voxel_indices, fr.P, list(spec.im_size), tuple(spec.bv_size))
    return orc.produce_sparse_pooling_input(g, stride=spec.stride)


def _layer_checksums(cfg, fids):
    spec = synth.CONFIGS[cfg]
    Hb, Wb = spec.bev_feat_hw
    Hi, Wi = spec.img_feat_hw
    Cb, Ci = spec.c_bev, spec.c_img
    bf16 = cfg == 3
    dt = torch.bfloat16 if bf16 else torch.float32
    cs = _cs16 if bf16 else _cs32
    out = []
    for fid in fids:
        fr = synth.make_frame(spec, seed=fid, n_outside=200)
        ref = _index(fr, spec)
        m = (ref["Mij_pool"], ref["M_val"], ref["M_size"])
        idx = ref["img_index_flip_pool"]
        bev = _feats((Hb, Wb, Cb), fid, 1, dt)
        img = _feats((Hi, Wi, Ci), fid, 2, dt)
        eb, ei = orc.sparse_pool_layer(bev, img, *m, idx, dual=cfg in (3, 5))
        total = cs(eb) + (cs(ei) if cfg in (3, 5) else 0)
        if cfg == 3:  # the gradients of both fused outputs (TF autodiff; the concat split and add_n fused)
            gb = _feats((Hb, Wb, Cb + Ci), fid, 3, dt)
            gi = _feats((Hi, Wi, Ci + Cb), fid, 4, dt)
            d_img = gi[..., :Ci] + orc.sparse_pool_grad_img(*m, gb[0, ..., Cb:].reshape(-1, Ci), idx, (1, Hi, Wi, Ci))
            d_bev = gb[..., :Cb] + orc.sparse_pool_trans_grad_bev(
                *m, np.ascontiguousarray(gi[..., Ci:]), idx).reshape(1, Hb, Wb, Cb)
            total += cs(d_bev) + cs(d_img)
        out.append(total)
    return out


@pytest.mark.parametrize("cfg,key,n,m", [(2, "layer_config2_frames64", 64, 64), (3, "layer_config3_frames4", 4, 4),
                                         (5, "layer_config5_frames64", 64, 64), (6, "layer_config6_frames64", 64, 16)])
def test_stored_layer_table_equals_oracle(cfg, key, n, m):
    """m: the frames recomputed (config 6, 256 channels: the first 16 of the table's 64)."""
    table = _table(key)
    assert len(table) == n
    got = _layer_checksums(cfg, range(m))
    bad = [f for f in range(m) if got[f] != table[f]]
    assert not bad, f"{key}: frames {bad[:8]} differ from the oracle ({len(bad)} of {m})"
    assert len(set(table)) == n  # every frame its own inputs


def test_stored_raw_scan_table_equals_oracle():
    """bench.py --workload frames: 64 synthetic 120k-point scans (kitti.synthetic_frames, seed 1000, scan f
    seeded by its frame id) through the oracle chain of cpu_baseline_frames."""
    from sparse_pooling_amd import kitti
    table = _table("frames_120000_frames64")
    F, C = len(table), 32
    assert F == 64
    h, w = synth.KITTI_IMAGE_SHAPE
    im_size = (w, h)
    fr = kitti.synthetic_frames(F, 120000, seed=1000, device=DEV, frame_ids=list(range(F)))
    calib = kitti.FrameCalibrationData()
    c = synth.KITTI_CALIB
    calib.p2 = np.array(c["P2"]).reshape(3, 4)
    rect = orc.rect_matrix(np.array(c["R0_rect"]).reshape(3, 3), np.array(c["Tr_velo_to_cam"]).reshape(3, 4))
    off = fr.point_offsets.cpu().numpy()
    xyzi = fr.xyzi.cpu().numpy()
    planes = fr.planes.cpu().numpy()
    from sparse_pooling_amd import bev as sbev
    nx, nz = sbev.grid_divisions(synth.AREA_EXTENTS, synth.VOXEL_SIZE)
    bad = []
    for f in range(F):
        pc = orc.velo_to_cam(xyzi[off[f]:off[f + 1]], rect, calib.p2, im_size)
        _, _, vox, upts = orc.bev_slices(pc, planes[f], synth.AREA_EXTENTS, synth.VOXEL_SIZE, synth.HEIGHT_LO,
                                         synth.HEIGHT_HI, synth.NUM_SLICES)
        g = orc.gen_sparse_pooling_input_avod(upts, vox, calib.p2, list(im_size), (nz, nx))
        ref = orc.produce_sparse_pooling_input(g, stride=(1, 1))
        bev = _feats((nz, nx, C), f, 5)
        img = _feats((h, w, C), f, 6)
        eb, _ = orc.sparse_pool_layer(bev, img, ref["Mij_pool"], ref["M_val"], ref["M_size"],
                                      ref["img_index_flip_pool"])
        if _cs32(eb) != table[f]:
            bad.append(f)
    assert not bad, f"raw-scan table: frames {bad[:8]} differ from the oracle ({len(bad)} of {F})"
