"""The oracle side of bench.py's per-frame checksum tables (profiles/frame_checksums.json).

Test infrastructure (imports the CPU oracle): used by tests/test_checksum_tables.py (CPU, a sample of every
table's frames) and tests/golden/make_checksum_tables.py (all frames: the generator of the file).

bench.py reports ``frame_checksums.match_n1`` by comparing each frame's output checksum with these tables.
Each entry is computed here, on the host, from the inputs the bench draws for that global frame id --
``synth.make_frame(spec, seed=frame id, n_outside=200)`` and ``dist.fill_features`` (integer-hash features
whose host mirror is ``dist.feature_values_np``) -- run through the C oracle (oracle/shpl_oracle.c: the
reference's index builder, avod/avod/utils/sparse_pool_utils.py:6-58, and TF 1.8's CPU pooling order,
:61-117), and reduced with ``dist.frame_checksum_np`` (position-weighted: sum_i bits[i] * (2i + 1) mod 2^64)
and, for several outputs, ``dist.combine_checksums_int``. So ``match_n1`` means "equals the TF-order
restatement at every element position", not "equals an earlier GPU run".

Tables: config 2 (64 frames, bv_fused), config 3 (4 frames, bf16: both fused forward outputs and both
gradients), config 5 (64 frames, both fused forward outputs), config 6 (the RetinaNet P2 shape, 64 frames),
the raw-scan workload (64 scans of 120k points: velodyne -> camera frame + FOV filter -> BEV slices ->
index -> bv_fused)."""
import numpy as np

from oracle import shpl_oracle as orc
from sparse_pooling_amd import dist as sd, synth

LAYER_TABLES = {2: ("layer_config2_frames64", 64), 3: ("layer_config3_frames4", 4),
                5: ("layer_config5_frames64", 64), 6: ("layer_config6_frames64", 64)}
RAW_TABLE = ("frames_120000_frames64", 64)
RAW_POINTS = 120000


def _feats(shape, fid, seed, bf16=False):
    """One frame's features as the bench draws them (dist.fill_features), on the host as f32; bf16: rounded
    once to bf16 (RNE), as the bench's bf16 tensors hold them."""
    a = sd.feature_values_np(shape, fid, seed)[None]
    if bf16:
        a = (orc.to_bf16_bits(a).astype(np.uint32) << np.uint32(16)).view(np.float32)
    return a


def _cs(a, bf16):
    """The checksum of one output; bf16: the oracle's f32 result rounded once (RNE), as the device stores it."""
    if bf16:
        a = (orc.to_bf16_bits(np.ascontiguousarray(a, dtype=np.float32)).astype(np.uint32)
             << np.uint32(16)).view(np.float32)
    return sd.frame_checksum_np(a, bf16=bf16)


def layer_checksum(cfg, fid):
    """Checksum of global frame ``fid`` of bench.py's layer workload at ``cfg``: the step's outputs in the
    bench's order (bv_fused, img_fused, d_bev, d_img), combined."""
    spec = synth.CONFIGS[cfg]
    Hb, Wb = spec.bev_feat_hw
    Hi, Wi = spec.img_feat_hw
    Cb, Ci = spec.c_bev, spec.c_img
    bf16 = cfg == 3
    dual = cfg in (3, 5)
    fr = synth.make_frame(spec, seed=fid, n_outside=200)
    g = orc.gen_sparse_pooling_input_avod(fr.points, fr.voxel_indices, fr.P, list(spec.im_size), tuple(spec.bv_size))
    ref = orc.produce_sparse_pooling_input(g, stride=spec.stride)
    m = (ref["Mij_pool"], ref["M_val"], ref["M_size"])
    idx = ref["img_index_flip_pool"]
    bev = _feats((Hb, Wb, Cb), fid, 1, bf16)
    img = _feats((Hi, Wi, Ci), fid, 2, bf16)
    eb, ei = orc.sparse_pool_layer(bev, img, *m, idx, dual=dual)
    outs = [_cs(eb, bf16)] + ([_cs(ei, bf16)] if dual else [])
    if cfg == 3:  # the gradients of both fused outputs (TF autodiff; the concat split and add_n fused)
        gb = _feats((Hb, Wb, Cb + Ci), fid, 3, bf16)
        gi = _feats((Hi, Wi, Ci + Cb), fid, 4, bf16)
        d_bev = gb[..., :Cb] + orc.sparse_pool_trans_grad_bev(
            *m, np.ascontiguousarray(gi[..., Ci:]), idx).reshape(1, Hb, Wb, Cb)
        d_img = gi[..., :Ci] + orc.sparse_pool_grad_img(*m, np.ascontiguousarray(gb[0, ..., Cb:]).reshape(-1, Ci),
                                                        idx, (1, Hi, Wi, Ci))
        outs += [_cs(d_bev, bf16), _cs(d_img, bf16)]
    return sd.combine_checksums_int(outs)


def raw_scan_checksum(fid):
    """bench.py --workload frames, global frame ``fid``: the synthetic 120k-point scan (kitti.synthetic_frames,
    seed 1000, scan seeded by its frame id) through the oracle chain of cpu_baseline_frames."""
    from sparse_pooling_amd import bev as sbev, kitti
    h, w = synth.KITTI_IMAGE_SHAPE
    im_size = (w, h)
    C = 32
    fr = kitti.synthetic_frames(1, RAW_POINTS, seed=1000, device="cpu", frame_ids=[fid])
    c = synth.KITTI_CALIB
    p2 = np.array(c["P2"]).reshape(3, 4)
    rect = orc.rect_matrix(np.array(c["R0_rect"]).reshape(3, 3), np.array(c["Tr_velo_to_cam"]).reshape(3, 4))
    nx, nz = sbev.grid_divisions(synth.AREA_EXTENTS, synth.VOXEL_SIZE)
    pc = orc.velo_to_cam(fr.xyzi.numpy(), rect, p2, im_size)
    _, _, vox, upts = orc.bev_slices(pc, fr.planes[0].numpy(), synth.AREA_EXTENTS, synth.VOXEL_SIZE,
                                     synth.HEIGHT_LO, synth.HEIGHT_HI, synth.NUM_SLICES)
    g = orc.gen_sparse_pooling_input_avod(upts, vox, p2, list(im_size), (nz, nx))
    ref = orc.produce_sparse_pooling_input(g, stride=(1, 1))
    bev = _feats((nz, nx, C), fid, 5)
    img = _feats((h, w, C), fid, 6)
    eb, _ = orc.sparse_pool_layer(bev, img, ref["Mij_pool"], ref["M_val"], ref["M_size"], ref["img_index_flip_pool"])
    return sd.combine_checksums_int([_cs(eb, False)])


def table_entry(key, fid):
    """The checksum of frame ``fid`` of table ``key``."""
    if key == RAW_TABLE[0]:
        return raw_scan_checksum(fid)
    cfg = next(c for c, (k, _) in LAYER_TABLES.items() if k == key)
    return layer_checksum(cfg, fid)


ORACLE_TABLES = dict([v for v in LAYER_TABLES.values()] + [RAW_TABLE])
