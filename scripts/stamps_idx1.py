"""Per-chunk timeline of k_index1 at config 3 (probe build SHPL_IDX1_PROBE=1, loaded through SHPL_LIB): each
chunk workgroup's s_memrealtime stamps (start, arrival, past the frame barrier, aggregates read, points placed,
buckets placed, holes written, end), 100 MHz,
relative to the launch's first stamp; printed as percentiles per phase."""
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
riders = "--no-riders" not in sys.argv
pl = pipeline.FusedPipeline(F, maxp, N, spec.im_size, spec.bv_size, spec.stride, spec.c_bev, spec.c_img,
                            dtype=torch.bfloat16, dual=True, device=dev)
pl.riders = riders
Hb, Wb = spec.bev_feat_hw
Hi, Wi = spec.img_feat_hw
feats = lambda shape, seed: sd.fill_features(torch.empty(shape, dtype=torch.bfloat16, device=dev), range(F), seed)  # noqa
bev, img = feats((F, Hb, Wb, spec.c_bev), 1), feats((F, Hi, Wi, spec.c_img), 2)
side = torch.cuda.Stream()
lib = L.lib()
lib.shpl_probe_idx1.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
n_ch = (maxp + 1023) // 1024
nb = F * n_ch
buf = np.zeros(8 * nb, dtype=np.uint64)
rows = []
for it in range(12):
    pl.step_overlapped(pts, vox, off, P, bev, img, side)
    torch.cuda.synchronize()
    if it >= 2:
        L.check(lib.shpl_probe_idx1(buf.ctypes.data_as(ctypes.c_void_p), nb), "stamps")
        t = buf.reshape(-1, 8).astype(np.int64)
        rows.append(t - t[:, 0].min())
t = np.stack(rows).astype(np.float64) / 100.0  # us
print("riders" if riders else "no riders", "chunks", nb, "per frame", n_ch, "err", int(pl.err.item()))
names = ["start", "arrive", "past barrier", "aggregates", "placed", "multisplit", "prefix", "end"]
for k in range(8):
    v = t[:, :, k]
    print("%-13s p0 %.2f p50 %.2f p90 %.2f max %.2f" % (names[k], v.min(), np.median(v), np.percentile(v, 90), v.max()))
for k in range(1, 8):
    d = t[:, :, k] - t[:, :, k - 1]
    print("%-13s <- %-13s mean %.2f p50 %.2f p90 %.2f max %.2f" % (names[k], names[k - 1], d.mean(), np.median(d),
                                                                  np.percentile(d, 90), d.max()))
last = t[:, :, 1].reshape(t.shape[0], F, n_ch).max(2, keepdims=True)
lag = t[:, :, 2].reshape(t.shape[0], F, n_ch) - last
print("barrier exit after the frame's last arrival: mean %.2f p90 %.2f max %.2f" % (lag.mean(), np.percentile(lag, 90), lag.max()))
