"""Per-wave phase cycles of k_conv_rows (probe build SHPL_ROWS_PROBE=3 through SHPL_LIB) at the bench's conv
shapes (config 2, 64 frames, bf16): the fused inference conv (Q 4: bev + pooled), the training forward with
statistics, and the input gradient (32 -> 64 channels). Prints mean cycles per row step of each phase."""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from sparse_pooling_amd import _lib as L, dist as sd, fusion_conv as fc, pipeline, synth  # noqa: E402

dev = torch.device("cuda", 0)
spec = synth.CONFIG2
F = int(os.environ.get("FRAMES", "64"))
frames = [synth.make_frame(spec, seed=s, n_outside=200) for s in range(F)]
pts, vox, off, P, maxp, N = pipeline.stack_frames(frames, dev)
dt = torch.bfloat16
pl = pipeline.FusedPipeline(F, maxp, N, spec.im_size, spec.bv_size, spec.stride, spec.c_bev, spec.c_img, dtype=dt,
                            device=dev)
Hb, Wb = spec.bev_feat_hw
Hi, Wi = spec.img_feat_hw
bev = sd.fill_features(torch.empty((F, Hb, Wb, spec.c_bev), dtype=dt, device=dev), range(F), 1)
img = sd.fill_features(torch.empty((F, Hi, Wi, spec.c_img), dtype=dt, device=dev), range(F), 2)
conv = fc.FusionConv(spec.c_bev + spec.c_img, spec.c_img, dtype=dt, device=dev, seed=0)
out = torch.empty((F, Hb, Wb, spec.c_img), dtype=dt, device=dev)
lib = L.lib()
n_items = F * ((Hb + 58) // 59) * ((Wb + 31) // 32) * 2
buf = np.zeros(10 * n_items, dtype=np.uint64)
names = ["ring wait", "reads+MFMA issue", "epilogue", "staging"]


def report(tag, nw):
    L.check(lib.shpl_probe_conv_phases(buf.ctypes.data_as(ctypes.c_void_p), ctypes.c_size_t(nw)), "probe")
    t = buf[:10 * nw].reshape(nw, 10).astype(np.float64)
    t = t[t[:, 5] > 0]
    rt = t[:, 6:9] - t[:, 6].min()  # 100 MHz ticks
    pro, loop = (rt[:, 1] - rt[:, 0]) / 100, (rt[:, 2] - rt[:, 1]) / 100
    print(f"  kernel span {rt[:, 2].max() / 100:.1f} us; per wave prologue mean {pro.mean():.2f} p90 "
          f"{np.percentile(pro, 90):.2f} us, loop mean {loop.mean():.2f} us; wave starts p50 "
          f"{np.percentile(rt[:, 0], 50) / 100:.1f} max {rt[:, 0].max() / 100:.1f} us; live waves at 10/50/90% of the "
          f"span: " + ", ".join(str(int(((rt[:, 0] <= x) & (rt[:, 2] > x)).sum())) for x in
                                 (0.1 * rt[:, 2].max(), 0.5 * rt[:, 2].max(), 0.9 * rt[:, 2].max())))
    print(f"  loop cycles / loop us = {t[:, 4].sum() / (loop.sum()):.0f} MHz")
    rows = t[:, 5].sum()
    per = t[:, :5].sum(0) / rows
    print(f"{tag}: {len(t)} waves, {rows:.0f} row steps; cycles per row step: " +
          ", ".join(f"{n} {v:.0f}" for n, v in zip(names + ["loop"], per)) +
          f"; unaccounted {per[4] - per[:4].sum():.0f}; wave loop mean {t[:, 4].mean():.0f} cycles")


for _ in range(int(os.environ.get("WARM", "30"))):
    pl.build_index(pts, vox, off, P)
    pl.build_csr(("cell",))
    conv.fused_csr(bev, img, pl.csr, pl.frame_off, is_training=False, out=out)
torch.cuda.synchronize()
report("fused inference conv (Q4, CMP)", F * 12 * 25)
stats = torch.empty((2, 32), dtype=torch.float64, device=dev)
raw = fc.conv3x3(bev, conv.weights, b=img, pool=pl.csr, frame_off=pl.frame_off, relu=False, stats=stats)
torch.cuda.synchronize()
report("training forward (Q4, CMP, ST)", F * 12 * 25)
g = sd.fill_features(torch.empty((F, Hb, Wb, 32), dtype=dt, device=dev), range(F), 7)
dx = fc.conv3x3_dgrad(g, conv.weights, 64, split=32)
torch.cuda.synchronize()
report("input gradient (Q2, 2 output blocks)", F * 12 * 25 * 2)
