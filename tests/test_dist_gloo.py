"""Frame-parallel orchestration with world_size 2 over gloo (CPU only):
disjoint frame ownership, MAX-over-ranks timing and the checksum all-gather
that bench.py runs over RCCL on the GPUs."""
import os

import numpy as np
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), HSA_ENABLE_IPC_MODE_LEGACY="0")
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from sparse_pooling_amd import dist as sd, synth
    seeds = sd.frame_seeds(rank, 3)
    frames = [synth.make_frame(synth.FrameSpec(500, (1200, 360), (704, 800)), s) for s in seeds]
    # per-rank work is only the rank's own frames; rank 1 is slower on purpose
    import time
    el = sd.timed(lambda k: time.sleep(0.05 * (rank + 1)), 2)
    cs = sd.gather_checksums(sum(float(f.points.sum()) for f in frames))
    q.put((rank, seeds, el, cs))
    dist.destroy_process_group()


def test_two_rank_frame_sharding():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29500 + (os.getpid() % 1000)
    ps = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = sorted(q.get(timeout=120) for _ in ps)
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    (r0, s0, e0, c0), (r1, s1, e1, c1) = res
    assert not set(s0) & set(s1)                 # disjoint frames
    assert abs(e0 - e1) < 1e-9 and e0 >= 0.2      # both see the max (rank 1: 2 x 0.1 s)
    assert c0 == c1 and len(c0) == 2 and c0[0] != c0[1]
