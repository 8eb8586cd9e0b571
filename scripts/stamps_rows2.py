"""Per-wave timeline of k_rows2 at config 3 (probe build SHPL_RPROBE=3, loaded through SHPL_LIB): each
wave's s_memrealtime start / end (100 MHz) for the forward pair and the gradient pair, with the wave's
rows and their run lengths, saved to gpurun_out/r04_stamps.npz; a summary is printed."""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from sparse_pooling_amd import _lib as L, dist as sd, pipeline, synth  # noqa: E402

dev = torch.device("cuda", 0)
spec = synth.CONFIGS[3]
F = 4
frames = [synth.make_frame(spec, seed=s, n_outside=200) for s in range(F)]
pts, vox, off, P, maxp, N = pipeline.stack_frames(frames, dev)
pl = pipeline.FusedPipeline(F, maxp, N, spec.im_size, spec.bv_size, spec.stride, spec.c_bev, spec.c_img,
                            dtype=torch.bfloat16, dual=True, device=dev)
Hb, Wb = spec.bev_feat_hw
Hi, Wi = spec.img_feat_hw
feats = lambda shape, seed: sd.fill_features(torch.empty(shape, dtype=torch.bfloat16, device=dev), range(F), seed)  # noqa
bev, img = feats((F, Hb, Wb, spec.c_bev), 1), feats((F, Hi, Wi, spec.c_img), 2)
g_bv, g_img = feats(tuple(pl.bv_fused.shape), 3), feats(tuple(pl.img_fused.shape), 4)
d_bev, d_img = torch.empty_like(bev), torch.empty_like(img)
side = torch.cuda.Stream()
lib = L.lib()
nw = ((27000 + 7) // 8 + (35200 + 7) // 8) * 4
buf = np.zeros(2 * nw, dtype=np.uint64)
out = {}
for it in range(6):
    pl.step_overlapped(pts, vox, off, P, bev, img, side)
    torch.cuda.synchronize()
    if it == 5:
        L.check(lib.shpl_probe_stamps(buf.ctypes.data_as(ctypes.c_void_p), ctypes.c_size_t(nw)), "stamps")
        out["fwd"] = buf.copy().reshape(-1, 2)
    pl.backward(g_bv, g_img, d_bev, d_img)
    torch.cuda.synchronize()
    if it == 5:
        L.check(lib.shpl_probe_stamps(buf.ctypes.data_as(ctypes.c_void_p), ctypes.c_size_t(nw)), "stamps")
        out["bwd"] = buf.copy().reshape(-1, 2)
kr_pix = pl.pcsr.key_range.cpu().numpy()
kr_cell = pl.csr.key_range.cpu().numpy()
np.savez("gpurun_out/r04_stamps.npz", fwd=out["fwd"], bwd=out["bwd"], kr_pix=kr_pix, kr_cell=kr_cell)
lp = kr_pix[:, 1] - kr_pix[:, 0]
lc = kr_cell[:, 1] - kr_cell[:, 0]
wl = np.concatenate([np.maximum(lp[0::2], lp[1::2]), np.maximum(lc[0::2], lc[1::2])])
for k in ("fwd", "bwd"):
    t = out[k].astype(np.int64)
    t0 = t[:, 0].min()
    s, e = t[:, 0] - t0, t[:, 1] - t0
    d = e - s
    npw = 27000 // 2
    print(k, "span %.2f us" % (e.max() / 100), "waves", len(t))
    for name, sl in (("pix", slice(0, npw)), ("cell", slice(npw, len(t)))):
        print("  %s start p50 %.2f p90 %.2f max %.2f | end p50 %.2f p90 %.2f p99 %.2f max %.2f | dur mean %.2f p50 %.2f p90 %.2f max %.2f" % (
            name, *(np.percentile(s[sl], [50, 90, 100]) / 100), *(np.percentile(e[sl], [50, 90, 99, 100]) / 100),
            d[sl].mean() / 100, *(np.percentile(d[sl], [50, 90, 100]) / 100)))
    for lo, hi in ((0, 1), (1, 3), (3, 6), (6, 9), (9, 17), (17, 33), (33, 99)):
        m = (wl >= lo) & (wl < hi)
        if m.any():
            print("  wlen [%d,%d): %5d waves, dur mean %.2f us, end p90 %.2f" % (lo, hi, m.sum(), d[m].mean() / 100,
                                                                            np.percentile(e[m], 90) / 100))
    # concurrency over time
    tt = np.arange(0, e.max(), 100)
    conc = [(s <= x).sum() - (e <= x).sum() for x in tt]
    print("  live waves per us:", conc)
