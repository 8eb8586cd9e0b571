"""Config-4 orchestration with world_size 2 over gloo (CPU only): the strong
partition of a global batch by global frame id, MAX-over-ranks timing and
the per-frame checksum all-gather that bench.py runs over RCCL on the GPUs.

Each rank computes the SHPL layer of the frames it owns (the CPU oracle
stands in for the HIP path, which needs a GPU: the GPU-side identity is
tests/test_gpu_dist.py) and the gathered per-frame checksums must equal the
single-process run over the whole batch."""
import os

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from sparse_pooling_amd import dist as sd, synth

GLOBAL = 4


def _frame_outputs(fids):
    """bv_fused of each owned frame (config-1 shape), features seeded by the global frame id."""
    from oracle import shpl_oracle as orc
    spec = synth.CONFIG1
    Hb, Wb = spec.bev_feat_hw
    Hi, Wi = spec.img_feat_hw
    outs = []
    for fid in fids:
        fr = synth.make_frame(spec, seed=fid, n_outside=20)
        g = orc.gen_sparse_pooling_input_avod(fr.points, fr.voxel_indices, fr.P, list(spec.im_size),
                                              tuple(spec.bv_size))
        ref = orc.produce_sparse_pooling_input(g, stride=spec.stride)
        bev = torch.empty((1, Hb, Wb, spec.c_bev))
        img = torch.empty((1, Hi, Wi, spec.c_img))
        sd.fill_features(bev, [fid], 1)
        sd.fill_features(img, [fid], 2)
        eb, _ = orc.sparse_pool_layer(bev.numpy(), img.numpy(), ref["Mij_pool"], ref["M_val"], ref["M_size"],
                                      ref["img_index_flip_pool"])
        outs.append(torch.from_numpy(np.ascontiguousarray(eb[0])))
    return torch.stack(outs)


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), HSA_ENABLE_IPC_MODE_LEGACY="0")
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import time
    fids = sd.partition(GLOBAL, world, rank, "strong")
    out = _frame_outputs(fids)
    info = {}
    el = sd.timed(lambda k: time.sleep(0.05 * (rank + 1)), 2, info=info)   # rank 1 is slower on purpose
    assert info["elapsed_s"] == el and info["barrier_inclusive_s"] >= el and "MAX over ranks" in info["method"]
    # the bench's per-rank kernel times: every rank's list, rank order
    assert sd.gather_floats([rank, 0.5 * rank]) == [[float(r), 0.5 * r] for r in range(world)]
    cs = sd.gather_frame_checksums(sd.frame_checksums(out))
    comm = sd.comm_report(None)
    assert comm["backend"] == "gloo" and comm["world_size"] == world
    assert [r["rank"] for r in comm["ranks"]] == list(range(world))
    q.put((rank, fids, el, cs))
    dist.destroy_process_group()


def test_partition():
    assert sd.partition(64, 8, 3, "strong") == list(range(24, 32))
    assert sd.partition(64, 1, 0, "strong") == list(range(64))
    assert sd.partition(8, 4, 2, "weak") == list(range(16, 24))
    assert sd.frame_seeds(0, 4) == [0, 1, 2, 3]
    with pytest.raises(ValueError):
        sd.partition(4, 8, 0, "strong")
    for w in (1, 2, 4, 8):   # strong blocks tile the batch exactly, in rank order
        assert sum((sd.partition(64, w, r) for r in range(w)), []) == list(range(64))


def test_frame_checksums_exact_and_batch_independent():
    x = torch.randn(3, 5, 7, 8)
    cs = sd.frame_checksums(x)
    assert cs.dtype == torch.int64 and cs.shape == (3,)
    assert torch.equal(sd.frame_checksums(x[1:2]), cs[1:2])
    y = x.clone()
    y[2, 4, 6, 7] = torch.nextafter(y[2, 4, 6, 7], torch.tensor(1e9))  # one ulp in one element
    assert torch.equal(sd.frame_checksums(y)[:2], cs[:2]) and sd.frame_checksums(y)[2] != cs[2]
    b = x.to(torch.bfloat16)
    assert torch.equal(sd.frame_checksums(b[1:]), sd.frame_checksums(b)[1:])


def test_two_rank_strong_partition_matches_one_process():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29500 + (os.getpid() % 1000)
    ps = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = sorted(q.get(timeout=180) for _ in ps)
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    (r0, f0, e0, c0), (r1, f1, e1, c1) = res
    assert f0 == [0, 1] and f1 == [2, 3]          # contiguous blocks of the global batch
    assert abs(e0 - e1) < 1e-9 and e0 >= 0.2      # both see the max (rank 1: 2 x 0.1 s)
    one = sd.frame_checksums(_frame_outputs(range(GLOBAL))).tolist()
    assert c0 == c1 == one                        # == the single-process run, frame by frame
    assert len(set(one)) == GLOBAL


def test_bench_gpus_must_match_world_size():
    """Under a launcher, --gpus N must equal WORLD_SIZE (checked before any device call)."""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, WORLD_SIZE="2", RANK="0")
    p = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "8"], env=env,
                       capture_output=True, text=True, timeout=120)
    assert p.returncode != 0 and "WORLD_SIZE=2" in p.stderr
