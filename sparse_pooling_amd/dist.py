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


def fill_features(out, frame_ids, seed_base):
    """out[i] = N(0,1) drawn on out's device by a generator seeded with
    (seed_base, frame_ids[i]): a frame's features are the same whichever rank
    draws them and however many frames share the tensor."""
    assert out.shape[0] == len(frame_ids)
    g = torch.Generator(device=out.device)
    tmp = torch.empty(out.shape[1:], dtype=torch.float32, device=out.device)
    for i, fid in enumerate(frame_ids):
        g.manual_seed(int(seed_base) * 1_000_003 + int(fid))
        torch.randn(tmp.shape, generator=g, out=tmp, device=out.device)
        out[i].copy_(tmp)
    return out


def frame_checksums(t):
    """Per-frame checksum of a [F, ...] f32/bf16 map: the int64 sum of its
    elements' bit patterns. Integer sums are exact in any order, so the value
    is independent of the reduction's launch shape (and of the batch)."""
    bits = {4: torch.int32, 2: torch.int16}[t.element_size()]
    out = torch.empty(t.shape[0], dtype=torch.int64, device=t.device)
    for i in range(t.shape[0]):
        out[i] = t[i].contiguous().view(bits).to(torch.int64).sum()
    return out


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


def gather_checksums(value, device=None):
    """All ranks' scalar checksums, rank order."""
    on = dist.is_available() and dist.is_initialized()
    t = torch.tensor([float(value)], dtype=torch.float64, device=_coll_device(device))
    if not on:
        return [float(value)]
    out = [torch.zeros_like(t) for _ in range(dist.get_world_size())]
    dist.all_gather(out, t)
    return [float(x.item()) for x in out]


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
