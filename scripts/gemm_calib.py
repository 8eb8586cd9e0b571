"""Calibration for the wide conv's MFMA roofline: hipBLASLt (torch.matmul) on the GEMM of the same FLOPs as
the RetinaNet post-fusion conv at 64 frames (M = 64 x 176 x 200 pixels, K = 9 x 512, N = 256, bf16 in, f32
accumulate) -- an implicit-GEMM conv cannot beat the library GEMM of its im2col matrix by much."""
import sys
import time

import torch

M, K, N = 64 * 176 * 200, 9 * 512, 256
dev = torch.device("cuda", 0)
for m in (M // 8, M):
    a = torch.randn((m, K), dtype=torch.bfloat16, device=dev)
    b = torch.randn((K, N), dtype=torch.bfloat16, device=dev)
    for _ in range(3):
        c = a @ b
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    reps = 10
    e0.record()
    for _ in range(reps):
        c = a @ b
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / reps
    tf = 2.0 * m * K * N / (ms * 1e-3) / 1e12
    print(f"gemm M={m} K={K} N={N}: {ms:.3f} ms, {tf:.1f} TFLOP/s ({tf / 2500:.3f} of 2.5 PF)", flush=True)
    del a, b, c
    torch.cuda.empty_cache()
sys.exit(0)
