"""Frame-parallel orchestration across GPUs.

SHPL frames are independent -- no parameters, no cross-frame state, no
halo -- so a node scales by splitting the frames of a batch over the ranks.
Every frame is named by its global frame id, and everything drawn for it
(points, voxel indices, feature maps) is seeded by that id, so a frame's
output does not depend on which rank computes it or on how many frames share
its launch.

Partitioning (config 4, BASELINE.json configs[3]):
* ``strong`` (default): a fixed global batch of G frames; rank r of w owns
  the contiguous block [r*G/w, (r+1)*G/w) (G must divide by w).
* ``weak``: every rank owns F frames of a global batch of F*w: rank r the
  block [r*F, (r+1)*F).

The only collectives are control-plane (RCCL over xGMI on the GPUs, gloo in
the CPU tests): barriers around the timed region, one MAX all-reduce of the
elapsed time and one all-gather of the per-frame output checksums (8 B per
frame), which must equal the N=1 run's.
"""
import os
import time

import numpy as np
import torch
import torch.distributed as dist


def world():
    return int(os.environ.get("WORLD_SIZE", "1")), int(os.environ.get("RANK", "0"))


def partition(frames, world_size, rank, mode="strong"):
    """Global frame ids owned by `rank`.

    strong: `frames` is the global batch, split into contiguous blocks of
    frames / world_size; weak: `frames` is the per-rank count."""
    if mode == "strong":
        if frames % world_size:
            raise ValueError(f"strong partitioning: the global batch of {frames} frames does not split "
                             f"over {world_size} ranks (use a multiple, or --partition weak)")
        per = frames // world_size
        return list(range(rank * per, (rank + 1) * per))
    if mode == "weak":
        return list(range(rank * frames, (rank + 1) * frames))
    raise ValueError(f"unknown partition mode {mode!r}")


def frame_seeds(rank, frames_per_rank):
    """Weak partitioning's global frame ids of `rank` (seed = global frame id)."""
    return partition(frames_per_rank, rank + 1, rank, "weak")


MASK32 = 0xFFFFFFFF


def _frame_key(seed_base, fid):
    """The 32-bit stream key of one frame's features: (seed_base, global frame id)."""
    return ((int(seed_base) * 1_000_003 + int(fid)) * 0x9E3779B9 + 0x632BE5AB) & MASK32


def _mix32(x, mask):
    """A 32-bit integer mix (xorshift-multiply rounds, multipliers below 2^31 so every product of a 32-bit
    value fits a signed 64-bit lane): identical on torch int64 (any device) and numpy uint64."""
    x = x ^ (x >> 16)
    x = (x * 0x7FEB352D) & mask
    x = x ^ (x >> 15)
    x = (x * 0x2C1B3C6D) & mask
    x = x ^ (x >> 13)
    x = (x * 0x297A2D39) & mask
    return x ^ (x >> 16)


def feature_values_np(shape, fid, seed_base):
    """One frame's features on the host, bit for bit fill_features' (the oracle side of the checksum tables):
    element i (flat, row-major) = (mix32(i + key) >> 8) * 2^-23 - 1, uniform on [-1, 1) in steps of 2^-23 --
    integer arithmetic and exact float steps, so every device and numpy agree."""
    n = int(np.prod(shape))
    x = (np.arange(n, dtype=np.uint64) + np.uint64(_frame_key(seed_base, fid))) & np.uint64(MASK32)
    x = _mix32(x, np.uint64(MASK32))
    return ((x >> np.uint64(8)).astype(np.float32) * np.float32(2.0 ** -23) - np.float32(1.0)).reshape(shape)


def fill_features(out, frame_ids, seed_base):
    """out[i] = the features of global frame frame_ids[i] for stream seed_base (feature_values_np's values,
    computed on out's device and rounded once to out's dtype): a frame's features are the same whichever rank
    draws them, however many frames share the tensor, and on the host."""
    assert out.shape[0] == len(frame_ids)
    n = out[0].numel() if out.shape[0] else 0
    if n == 0:
        return out
    idx = torch.arange(n, dtype=torch.int64, device=out.device)
    for i, fid in enumerate(frame_ids):
        x = (idx + _frame_key(seed_base, fid)) & MASK32
        x = _mix32(x, MASK32)
        v = (x >> 8).to(torch.float32) * (2.0 ** -23) - 1.0
        out[i].copy_(v.view(out.shape[1:]))
    return out


def _weights(n, device):
    """2i + 1 for the n elements of a frame (int64), cached per (n, device)."""
    key = (int(n), str(device))
    w = _WEIGHTS.get(key)
    if w is None:
        w = torch.arange(n, dtype=torch.int64, device=device) * 2 + 1
        _WEIGHTS.clear()  # one shape at a time: the maps are large
        _WEIGHTS[key] = w
    return w


_WEIGHTS = {}


def frame_checksums(t):
    """Per-frame checksum of a [F, ...] f32/bf16 map: sum_i bits[i] * (2i + 1) mod 2^64 over the frame's
    elements in row-major order (bits: the element's pattern as a signed integer), as a signed int64.
    Integer arithmetic mod 2^64 is exact in any order, so the value does not depend on the reduction's launch
    shape or on the batch; the odd position weights make it see where each value sits -- a row written to the
    wrong cell or two channels swapped change it (the plain bit sum could not)."""
    bits = {4: torch.int32, 2: torch.int16}[t.element_size()]
    out = torch.empty(t.shape[0], dtype=torch.int64, device=t.device)
    if t.shape[0] == 0:
        return out
    w = _weights(t[0].numel(), t.device)
    for i in range(t.shape[0]):
        out[i] = (t[i].contiguous().view(bits).reshape(-1).to(torch.int64) * w).sum()
    return out


def combine_checksums(per_output):
    """One checksum per frame over several outputs of a step: sum_k cs_k * (2k + 1) mod 2^64 (int64 tensors,
    wrapping), so that exchanging two outputs of one shape changes it too."""
    total = None
    for k, cs in enumerate(per_output):
        term = cs.to(torch.int64) * (2 * k + 1)
        total = term if total is None else total + term
    return total


def frame_checksum_np(a, bf16=False):
    """frame_checksums of ONE frame on the host (the oracle side): a is the frame's values as f32 (bf16: the
    values already rounded to bf16, their upper 16 bits taken)."""
    a = np.ascontiguousarray(a, dtype=np.float32).reshape(-1)
    if bf16:
        bits = (a.view(np.uint32) >> np.uint32(16)).astype(np.uint16).view(np.int16)
    else:
        bits = a.view(np.int32)
    s, step = 0, 1 << 22
    with np.errstate(over="ignore"):
        for lo in range(0, a.size, step):  # in pieces: the maps run to 10^8 elements
            b = bits[lo:lo + step].astype(np.int64).astype(np.uint64)
            w = np.arange(lo, lo + b.size, dtype=np.uint64) * np.uint64(2) + np.uint64(1)
            s = (s + int((b * w).sum(dtype=np.uint64))) % (1 << 64)
    return s - (1 << 64) if s >= 1 << 63 else s


def combine_checksums_int(per_output):
    """combine_checksums over Python ints (host side), as a signed int64."""
    s = sum(int(c) * (2 * k + 1) for k, c in enumerate(per_output)) % (1 << 64)
    return s - (1 << 64) if s >= 1 << 63 else s


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


TIMING_METHOD = ("per-rank span from after the opening barrier + device sync to the rank's closing device "
                 "sync (the closing barrier is not timed); MAX over ranks")


def timed(fn, steps, device=None, info=None):
    """Run ``fn`` ``steps`` times between barriers + device syncs; returns the
    elapsed seconds maximised over ranks.

    Each rank's clock runs from after the opening barrier and device sync to
    its closing device sync; the closing barrier comes after the clock stops,
    so a collective's own latency (a visible share of an 8-rank run's ~6 ms
    window) is never timed. The MAX over ranks is then the slowest rank's
    compute span, all ranks having started together.
    info (a dict, optional) receives the method and, for comparison with
    rounds 1-2 (whose clock stopped after the closing barrier), the
    barrier-inclusive elapsed time, MAX over ranks."""
    on = dist.is_available() and dist.is_initialized()
    if on:
        dist.barrier()
    _sync(device)
    t0 = time.perf_counter()
    for k in range(steps):
        fn(k)
    _sync(device)
    elapsed = time.perf_counter() - t0
    if on:
        dist.barrier()
    with_barrier = time.perf_counter() - t0
    if on:
        t = torch.tensor([elapsed, with_barrier], dtype=torch.float64, device=_coll_device(device))
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed, with_barrier = float(t[0].item()), float(t[1].item())
    if info is not None:
        info.update(method=TIMING_METHOD, elapsed_s=elapsed, barrier_inclusive_s=with_barrier)
    return elapsed


def gather_floats(values, device=None):
    """All ranks' lists of floats (every rank the same length), rank order."""
    t = torch.tensor([float(v) for v in values], dtype=torch.float64, device=_coll_device(device))
    on = dist.is_available() and dist.is_initialized()
    if not on:
        return [[float(x) for x in t.cpu().tolist()]]
    out = [torch.zeros_like(t) for _ in range(dist.get_world_size())]
    dist.all_gather(out, t)
    return [[float(x) for x in o.cpu().tolist()] for o in out]


def gather_frame_checksums(local, device=None):
    """All-gather the ranks' per-frame checksums (int64 [F_rank], every rank
    the same F_rank) into one list in rank order -- global frame order for
    both partitionings."""
    local = local.to(torch.int64)
    on = dist.is_available() and dist.is_initialized()
    if not on:
        return [int(x) for x in local.cpu().tolist()]
    t = local.to(_coll_device(device))
    out = [torch.zeros_like(t) for _ in range(dist.get_world_size())]
    dist.all_gather(out, t)
    return [int(x) for o in out for x in o.cpu().tolist()]


def device_identity(device):
    """This rank's device: ordinal, PCI location and name (for the bench line's
    evidence that the ranks ran on distinct GPUs)."""
    if device is None or device.type != "cuda":
        return {"device": "cpu"}
    p = torch.cuda.get_device_properties(device)
    pci = None
    if hasattr(p, "pci_bus_id"):
        pci = f"{getattr(p, 'pci_domain_id', 0):04x}:{p.pci_bus_id:02x}:{getattr(p, 'pci_device_id', 0):02x}"
    return {"ordinal": device.index, "pci": pci, "uuid": str(getattr(p, "uuid", "")) or None,
            "name": p.name, "visible": os.environ.get("HIP_VISIBLE_DEVICES") or os.environ.get("CUDA_VISIBLE_DEVICES")}


def comm_report(device):
    """Control-plane evidence: backend, world size, RCCL version and every
    rank's device identity (all-gathered, rank order)."""
    on = dist.is_available() and dist.is_initialized()
    me = dict(device_identity(device), rank=dist.get_rank() if on else 0, host_pid=os.getpid())
    ranks = [me]
    if on:
        ranks = [None] * dist.get_world_size()
        dist.all_gather_object(ranks, me)
    rccl = None
    try:
        v = torch.cuda.nccl.version()
        rccl = ".".join(str(x) for x in v) if isinstance(v, tuple) else str(v)
    except Exception:  # noqa: BLE001 -- no RCCL in this build
        pass
    pcis = [r.get("pci") or r.get("uuid") for r in ranks]
    return {"backend": dist.get_backend() if on else None,
            "world_size": dist.get_world_size() if on else 1,
            "rccl_version": rccl,
            "distinct_devices": len(set(pcis)) if all(pcis) else None,
            "ranks": ranks}
