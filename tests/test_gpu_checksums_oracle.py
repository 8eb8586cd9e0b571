"""bench.py's device outputs against the oracle-generated checksum tables.

profiles/frame_checksums.json's layer and raw-scan tables are written by tests/golden/make_checksum_tables.py
from the CPU oracle (tests/checksum_tables.py), never by a GPU run; tests/test_checksum_tables.py re-checks a
sample of them on the CPU. Here bench.py runs each of those workloads on the GPU -- the whole step: device
index build, CSRs, overlapped streams, the captured HIP graph -- and its per-frame position-weighted checksums
(dist.frame_checksums) must equal the tables frame for frame (``match_n1``), so a pooled row written to the
wrong cell, two channels exchanged or two outputs swapped fail."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
pytestmark = pytest.mark.gpu


def _bench(args, timeout=300):
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "1", "--steps", "4", "--warmup", "1",
                        "--no-cpu-baseline", *args], cwd=ROOT, env=env, capture_output=True, text=True,
                       timeout=timeout)
    assert p.returncode == 0, p.stdout[-2000:] + p.stderr[-4000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout[-2000:]
    return json.loads(lines[0])


@pytest.mark.parametrize("args,key,frames", [
    (["--config", "2", "--frames", "64"], "layer_config2_frames64", 64),
    (["--config", "3"], "layer_config3_frames4", 4),
    (["--config", "5", "--frames", "16"], "layer_config5_frames64", 16),
    (["--config", "6", "--frames", "64"], "layer_config6_frames64", 64),
    (["--workload", "frames", "--frames", "8"], "frames_120000_frames64", 8),
])
def test_bench_outputs_equal_oracle_tables(args, key, frames):
    out = _bench(args)
    c = out["frame_checksums"]
    assert c["compared_with"] == key and c["frames"] == frames and c["pinned_to"] == "oracle", c
    assert c["match_n1"] is True, c
    assert out.get("index_errors", 0) == 0


@pytest.mark.parametrize("cfg,dtype", [(2, "bf16"), (2, "f32"), (6, "bf16"), (6, "f32")])
def test_conv_table_is_a_tolerance_checked_output(cfg, dtype):
    """The conv workload's tables (conv[_c6]_<dtype>_frames64) come from a GPU run: TF's Conv2D fixes no
    summation order, so no oracle checksum exists (bench.py labels them self-referential). What pins them: the
    bench's conv of global frames 0 and 1 -- built here as run_conv builds it, 2 frames instead of 64 -- has the
    stored checksums (the output does not depend on the batch), and a band of each frame is within the conv
    tests' tolerance of the oracle's double-precision conv of the oracle's bv_fused (tests/test_gpu_conv.py
    bounds). cfg 6: RetinaNet's 512 -> 256 conv with a bias and ReLU (bf16: k_conv_wide)."""
    import numpy as np
    import torch

    from oracle import shpl_oracle as orc
    from sparse_pooling_amd import dist as sd, fusion_conv as fc, pipeline, synth
    retina = cfg == 6
    with open(os.path.join(ROOT, "profiles", "frame_checksums.json")) as fh:
        table = json.load(fh)[f"conv{'_c6' if retina else ''}_{dtype}_frames64"]
    dev = torch.device("cuda", 0)
    dt = torch.bfloat16 if dtype == "bf16" else torch.float32
    spec = synth.CONFIGS[cfg]
    fids = [0, 1]
    frames = [synth.make_frame(spec, seed=s, n_outside=200) for s in fids]
    pts, vox, off, P, maxp, N = pipeline.stack_frames(frames, dev)
    pl = pipeline.FusedPipeline(len(fids), maxp, N, spec.im_size, spec.bv_size, spec.stride, spec.c_bev,
                                spec.c_img, dtype=dt, device=dev)
    Hb, Wb = spec.bev_feat_hw
    Hi, Wi = spec.img_feat_hw
    cb, ci = spec.c_bev, spec.c_img
    bev = sd.fill_features(torch.empty((2, Hb, Wb, cb), dtype=dt, device=dev), fids, 1)
    img = sd.fill_features(torch.empty((2, Hi, Wi, ci), dtype=dt, device=dev), fids, 2)
    c_out = 256 if retina else ci
    if retina:  # as bench.py run_conv builds it
        conv = fc.FusionConv(cb + ci, c_out, batch_norm=False, bias=True, relu=True, dtype=dt, device=dev, seed=0)
        conv.bias.copy_(torch.linspace(-0.5, 0.5, c_out, device=dev))
    else:
        conv = fc.FusionConv(cb + ci, ci, dtype=dt, device=dev, seed=0)
    out = torch.empty((2, Hb, Wb, c_out), dtype=dt, device=dev)
    pl.build_index(pts, vox, off, P)
    pl.build_csr(("cell",))
    conv.fused_csr(bev, img, pl.csr, pl.frame_off, is_training=False, out=out)
    torch.cuda.synchronize()
    cs = sd.frame_checksums(out).tolist()
    assert cs == table[:2], (cs, table[:2])
    w = conv.weights.float().cpu().numpy()
    center, scale, shift = (None if v is None else v.float().cpu().numpy() for v in conv._inference_epilogue())
    y0, y1 = (80, 88) if retina else (296, 344)  # a band of rows (the 512-channel oracle conv is slow)
    for k, fid in enumerate(fids):
        fr = frames[k]
        g = orc.gen_sparse_pooling_input_avod(fr.points, fr.voxel_indices, fr.P, list(spec.im_size),
                                              tuple(spec.bv_size))
        ref = orc.produce_sparse_pooling_input(g, stride=spec.stride)
        hb = bev[k:k + 1].float().cpu().numpy()
        hi = img[k:k + 1].float().cpu().numpy()
        eb, _ = orc.sparse_pool_layer(hb, hi, ref["Mij_pool"], ref["M_val"], ref["M_size"], ref["img_index_flip_pool"])
        if dtype == "bf16":  # bv_fused as the bf16 path holds it (the pooled sums rounded once)
            eb = orc.from_bf16_bits(orc.to_bf16_bits(eb))
        x = np.ascontiguousarray(eb[:, y0 - 1:y1 + 1])
        want = orc.conv3x3(x, w, center, scale, shift, True)
        _, ab = orc.conv3x3(np.abs(x), np.abs(w), raw=True)
        bound = 1e-5 + 2.0 ** -19 * ab * (np.abs(scale) if scale is not None else 1.0)
        if dtype == "bf16":
            bound = bound + np.abs(want) * 2.0 ** -8
        got = out[k:k + 1, y0 - 1:y1 + 1].float().cpu().numpy()
        err = np.abs(got[:, 1:-1].astype(np.float64) - want[:, 1:-1])
        assert (err <= bound[:, 1:-1]).all(), (err.max(), (err / bound[:, 1:-1]).max())
