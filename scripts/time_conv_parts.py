"""Times the bf16 training convs one at a time at the bench's shape (64 frames
of 704x800, 32 + 32 -> 32 channels): the forward with statistics, the input
gradient (two maps) and the weight gradient (two sources), HIP events on the
current stream. SHPL_LIB selects a variant build (A/B of compile-time switches).

    python scripts/time_conv_parts.py [--frames 64] [--reps 10]
"""
import argparse
import hashlib
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from sparse_pooling_amd import fusion_conv as fc  # noqa: E402


def timed(fn, reps):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=64)
    ap.add_argument("--reps", type=int, default=10)
    args = ap.parse_args()
    B, H, W, C = args.frames, 704, 800, 32
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(0)
    mk = lambda c: torch.randn((B, H, W, c), device=dev, generator=g).to(torch.bfloat16)  # noqa: E731
    a, b, gy = mk(C), mk(C), mk(C)
    w = (0.05 * torch.randn((3, 3, 2 * C, C), device=dev, generator=g)).to(torch.bfloat16)
    stats = torch.empty((2, C), dtype=torch.float64, device=dev)
    out = {}
    out["fwd_stats_ms"] = timed(lambda: fc.conv3x3(a, w, b=b, relu=False, stats=stats), args.reps)
    out["dgrad_two_maps_ms"] = timed(lambda: fc.conv3x3_dgrad(gy, w, 2 * C, split=C), args.reps)
    out["wgrad_two_sources_ms"] = timed(lambda: fc.conv3x3_wgrad(a, gy, b=b), args.reps)
    flops = 2.0 * 9 * (2 * C) * C * B * H * W
    out.update({k.replace("_ms", "_tflops"): round(flops / (v * 1e-3) / 1e12, 1) for k, v in list(out.items())})
    dw = fc.conv3x3_wgrad(a, gy, b=b)
    torch.cuda.synchronize()
    out["wgrad_sha"] = hashlib.sha256(dw.float().cpu().numpy().tobytes()).hexdigest()[:16]  # bitwise A/B check
    out["lib"] = os.environ.get("SHPL_LIB", "default")
    print(json.dumps(out))


if __name__ == "__main__":
    main()
