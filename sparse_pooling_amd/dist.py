"""Frame-parallel orchestration across GPUs.

SHPL frames are independent -- no parameters, no cross-frame state, no
halo -- so a node scales by giving every rank its own frames. The only
collectives are control-plane: barriers around the timed region, one MAX
all-reduce of the elapsed time and one all-gather of per-rank output
checksums (a few bytes over RCCL/xGMI). Backend "nccl" (RCCL) on the GPUs,
"gloo" in the CPU tests.
"""
import os
import time

import torch
import torch.distributed as dist


def world():
    return int(os.environ.get("WORLD_SIZE", "1")), int(os.environ.get("RANK", "0"))


def frame_seeds(rank, frames_per_rank, base=100000):
    """Disjoint seeds per rank: rank r owns frames [r*base, r*base + F)."""
    return [base * rank + f for f in range(frames_per_rank)]


def _coll_device(device):
    """Where the control-plane tensors live: on the GPU for RCCL, on the host
    for gloo (the CPU tests and the one-GPU rehearsal of the N>1 bench)."""
    if device is None or device.type != "cuda":
        return "cpu"
    if dist.is_available() and dist.is_initialized() and dist.get_backend() == "gloo":
        return "cpu"
    return device


def _sync(device):
    if device is not None and device.type == "cuda":
        torch.cuda.synchronize(device)


def timed(fn, steps, device=None):
    """Run ``fn`` ``steps`` times between barriers + device syncs; returns the
    elapsed seconds maximised over ranks."""
    on = dist.is_available() and dist.is_initialized()
    if on:
        dist.barrier()
    _sync(device)
    t0 = time.perf_counter()
    for k in range(steps):
        fn(k)
    _sync(device)
    if on:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if on:
        t = torch.tensor([elapsed], dtype=torch.float64, device=_coll_device(device))
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    return elapsed


def gather_checksums(value, device=None):
    """All ranks' scalar checksums, rank order."""
    on = dist.is_available() and dist.is_initialized()
    t = torch.tensor([float(value)], dtype=torch.float64, device=_coll_device(device))
    if not on:
        return [float(value)]
    out = [torch.zeros_like(t) for _ in range(dist.get_world_size())]
    dist.all_gather(out, t)
    return [float(x.item()) for x in out]
