"""SHPL bench: fused frames/s + achieved HBM GB/s of the SHPL gather/scatter.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--frames F] [--config 2|3|5]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N \
        --master-addr 127.0.0.1 --master-port P bench.py --gpus N ...

Default workload (BASELINE.json configs[1], "config 2"): synthetic
KITTI-shaped frames of 20k camera-frame points, BEV 704x800x32, image
360x1200x32, fp32, img->BEV fused SHPL forward. One step processes F frames
per GPU (default 64, the config-4 batch) through the whole hot path with the
inputs resident in HBM: device index build (projection, clip, strides,
flatten, compaction) -> destination-sorted M -> fused pooled gather + concat
write of bv_fused. The streaming half of the layer needs no index and runs
on a side stream beside the index build (--no-overlap: strictly sequential).
Other configs: 3 = bf16 dual SHPL forward + backward at the fusion_vgg
conv4 level (88x100x256 / 45x150x256, 4 frames); 5 = fp32 dual forward,
40k points, 64 channels.

Multi-GPU (config 4): `--gpus N` without a launcher starts N
ranks itself (torch.distributed.run, before this process touches HIP); under
a launcher --gpus must equal WORLD_SIZE. Frames are independent and named by
global frame id (points, voxel indices and features seeded by it), so ranks
need no data-path collective. --partition strong (default): a fixed global
batch of --frames frames (default 64), rank r owning the contiguous block
[r*G/w, (r+1)*G/w), value = G / max elapsed, "scaling": "strong"; weak: every
rank --frames frames of a global batch of frames*w. The only collectives are
the barriers around the timed loop, a MAX all-reduce of the elapsed time and
an all-gather of per-frame output checksums, compared with the N=1 run's
(profiles/frame_checksums.json, --write-checksums).

roofline: the SHPL layer kernels (k_dense + k_sparse of every pull in the
step); algorithmic bytes per step (SURVEY §8d per frame x F) over their
summed mean durations, timed with events on their launch streams.
cpu_baseline: the C restatement of the reference path (oracle/: index build +
TF-order pooling + concat), one core, on a bounded sample of the same
frames (rank 0, N=1 only).
"""
import argparse
import hashlib
import json
import os
import subprocess
import sys
import time

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E peak (MI355X_MICROARCH.md, chip-level parameters)
# dense MFMA peaks (MI355X_MICROARCH.md, Matrix cores): f32-input 157.3 TF, bf16 ~2.5 PF
MFMA_PEAK_TFS = {"f32": 157.3, "bf16": 2500.0}
DEFAULT_FRAMES = {2: 64, 3: 4, 5: 64, 6: 64}
CHECKSUM_FILE = os.path.join(HERE, "profiles", "frame_checksums.json")


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--frames", type=int, default=None,
                    help="frames per step: the global batch (--partition strong) or per GPU (weak)")
    ap.add_argument("--partition", default="strong", choices=["strong", "weak"],
                    help="strong: the global batch split into contiguous blocks over the ranks (config 4); "
                         "weak: every rank its own --frames frames")
    ap.add_argument("--write-checksums", action="store_true",
                    help="store this run's per-frame output checksums in profiles/frame_checksums.json "
                         "(the N=1 reference the N>1 runs are compared with)")
    ap.add_argument("--config", type=int, default=2, choices=[2, 3, 5, 6],
                    help="BASELINE configs 2 / 3 / 5; 6: the RetinaNet P2 SHPL shape (stride 4, 256 ch, f32)")
    ap.add_argument("--cpu-seconds", type=float, default=10.0, help="budget of the CPU-baseline sample")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-cpu-parallel", action="store_true",
                    help="skip the frame-parallel (one process per core, up to 16) CPU-baseline sample")
    ap.add_argument("--no-overlap", action="store_true",
                    help="run the layer's streaming pass after the index build instead of beside it")
    ap.add_argument("--no-interleave", action="store_true",
                    help="dual configs: start both sparse passes after both dense passes (A/B of the overlap)")
    ap.add_argument("--csr-path", default="auto", choices=["auto", "frame", "segment", "range"],
                    help="force the CSR builder (shpl_build_csr_path; A/B measurements: the conv / training workloads' segmented CSR 115 / 687 us vs 84 / 112 us per frame sort, profiles/r04_csr_ab.log)")
    ap.add_argument("--no-buckets", action="store_true",
                    help="row-keyed layers (config 3): range CSRs + one k_rows launch per pull on two streams "
                         "instead of the index build's buckets, one CSR launch and one shpl_pull_pair launch per pull pair")
    ap.add_argument("--rows", action="store_true",
                    help="layer workload: the row-keyed pipeline (bucketed index, one launch per pull pair) at any batch "
                         "(A/B: config 6 1.95-1.99 vs 1.57 ms, profiles/r04_rows_ab.log)")
    ap.add_argument("--split", default="auto", choices=["auto", "on", "off"],
                    help="img->BEV layer: the pass-through copy beside the index chain and the pooled half written once "
                         "by a row-keyed pull after it, on a high-priority stream (FusedPipeline split); auto: on "
                         "for 1 KB halves (config 6)")
    ap.add_argument("--split-chain", default="current", choices=["current", "stream"],
                    help="split layer: the index chain on the (high-priority) stream the step runs on, only the copy "
                         "forked (current), or on a stream of its own forked beside the copy (stream; A/B)")
    ap.add_argument("--split-pull", default="once", choices=["once", "rows"],
                    help="split layer: the pooled half by shpl_pull_once (sparse walk + the empty rows' zeros) or by "
                         "the row-keyed k_rows (A/B)")
    ap.add_argument("--split-form", default="serial", choices=["serial", "overlap"],
                    help="split layer: the pooled half after the pass-through copy, the step captured in a graph "
                         "(serial), or beside the copy, eager with the chain at high priority (overlap; A/B)")
    ap.add_argument("--head-k", type=int, default=None,
                    help="bucketed pipelines: run heads per destination in the CSRs (FusedPipeline.HEAD_K; 0 = none; "
                         "A/B)")
    ap.add_argument("--pixel-cols", action="store_true",
                    help="bucketed config 3: the pixel-keyed CSR keeps ent_col (per-column partials in its pulls) "
                         "instead of the identity-column form")
    ap.add_argument("--no-riders", action="store_true",
                    help="bucketed config 3: copy the forward's pass-through halves with their own launches before the "
                         "index build instead of as extra workgroups of the index launches")
    ap.add_argument("--graph-steps", type=int, default=None,
                    help="layer workloads: consecutive steps captured in one HIP graph (the timed loop replays it "
                         "steps / graph-steps times; --steps must divide). Default at config 3: 8 when --steps divides, "
                         "else 4 when it divides (0.107 -> 0.103 ms per step with 4: the replay boundary's ~8 us "
                         "once per 4 steps; 8: -1 %, profiles/r05_c3gs_ab.log), else 1; elsewhere 1 (config 2: "
                         "no change, profiles/r03_graph_steps_ab.log; configs 2 and 6 with 4: within 0.2 %, r05_c6gs_ab.log)")
    ap.add_argument("--no-pool-report", action="store_true",
                    help="config 2: skip the separate pool_fwd measurement (PMC passes count the step's launches only)")
    ap.add_argument("--graph", action="store_true",
                    help="capture the step in a HIP graph even where the default is eager (the split step)")
    ap.add_argument("--no-graph", action="store_true",
                    help="launch every step eagerly instead of replaying one captured HIP graph of it")
    ap.add_argument("--workload", default="layer", choices=["layer", "frames", "conv"],
                    help="layer: BASELINE configs 2/3/5 from prepared points + voxel indices (default); "
                         "frames: raw velodyne scans -> loader -> BEV slices -> index -> fused layer; "
                         "conv: config 2 + the post-fusion 3x3 conv/BN/ReLU (rpn_model.py:338-346) with the "
                         "pooling fused into the conv (SURVEY §8f row 4)")
    ap.add_argument("--dtype", default="f32", choices=["f32", "bf16"], help="conv workload storage dtype")
    ap.add_argument("--train-bn", action="store_true", help="conv workload: BatchNorm in training mode")
    ap.add_argument("--train", action="store_true",
                    help="conv workload: training step (batch-statistics BatchNorm forward + the whole backward: "
                         "BN/ReLU, input and weight gradients of the conv, the pooled channels' gradient to the image)")
    ap.add_argument("--no-wgrad-reuse", action="store_true",
                    help="conv training (bf16): the weight gradient prepares its own pooled operand instead of "
                         "reading the forward's (shpl_conv3x3_wgrad_reuse; A/B)")
    ap.add_argument("--no-dgrad-occ", action="store_true",
                    help="conv training (bf16): the input gradient writes its pooled channels' map whole instead of "
                         "at the occupied cells only (shpl_conv3x3_dgrad_reuse; A/B)")
    ap.add_argument("--wgrad-side", choices=["on", "off"], default=None,
                    help="conv training: the weight gradient on a side stream beside the input gradient "
                         "(FusionConv.WGRAD_SIDE; default: the class's)")
    ap.add_argument("--img-beside", choices=["dgrad", "wgrad"], default=None,
                    help="conv training: the image gradient's side-stream work beside the input gradient (its zero "
                         "rows) or beside the weight gradient (zero rows and pull; FusionConv.IMG_BESIDE_WGRAD)")
    ap.add_argument("--img-zero-side", choices=["on", "off"], default=None,
                    help="conv training: the image gradient's zero rows on a side stream beside the input gradient "
                         "(FusionConv.IMG_ZERO_SIDE; default: the class's)")
    ap.add_argument("--scan-points", type=int, default=120000, help="points per velodyne scan (frames)")
    ap.add_argument("--maps-form", default="f64", choices=["f64", "bev_input"],
                    help="frames: the BEV maps as the reference's f64 height / density maps, or as the network's "
                         "f32 BEV input (np.dstack of the maps as its tf.float32 placeholder holds them: half the "
                         "bytes; shpl_bev_input)")
    ap.add_argument("--stream-priority", default="chain", choices=["chain", "dense", "both", "none"],
                    help="frames workload: which of the index chain / the streaming pass runs on a high-priority stream")
    ap.add_argument("--dense-after", default="start", choices=["start", "velo", "bev", "csr"],
                    help="frames workload: where the streaming pass starts beside the index chain")
    ap.add_argument("--maps-after", default="chain", choices=["stream", "chain"],
                    help="frames: write the BEV maps after the streaming pass (side stream) or after the CSR "
                         "(index chain)")
    return ap.parse_args()


def pull_bytes(rows, c_pass, c_pool, u_src, nnz, esz, write_width):
    """read the pass-through rows, write the output rows, gather
    the unique source rows, 12 B per entry (int32 dst, int32 src, f32 val)."""
    return rows * c_pass * esz + rows * write_width * esz + u_src * c_pool * esz + 12 * nnz


def layer_bytes(spec, nnz, u_pix, frames, esz=4):
    """img->BEV layer_fwd of config 2 (kept for scripts/pull_sweep.py)."""
    Hb, Wb = spec.bev_feat_hw
    return pull_bytes(frames * Hb * Wb, spec.c_bev, spec.c_img, u_pix, nnz, esz, spec.c_bev + spec.c_img)


def pool_fwd_report(pl, img, spec, F, u_pix, nnz, esz, dev, reps=10):
    """SURVEY §8d's pool_fwd beside the official layer_fwd: the img->BEV pooling
    alone (shpl_pull, SHPL_OUT_POOL: k_dense writing the zeros, then k_sparse)
    into a [F, Hb, Wb, Ci] map, over the CSR the step just built; HIP events
    around `reps` launches, after the timed loop. Checked bitwise against the
    pooled half of bv_fused."""
    from sparse_pooling_amd import _lib as L
    Hb, Wb = spec.bev_feat_hw
    ci = spec.c_img
    out = torch.empty((F, Hb, Wb, ci), dtype=pl.bv_fused.dtype, device=dev)
    lib = L.lib()

    def run():
        L.check(lib.shpl_pull(L.BY_CELL, L.dtype_code(out), pl.csr.ref(), L.ptr(img), ci, 0, ci, None, 0, 0, 0,
                              L.OUT_POOL, L.ptr(out), ci, L.stream_of(dev)), "shpl_pull")
    run()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        run()
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / reps
    nb = pull_bytes(F * Hb * Wb, 0, ci, u_pix, nnz, esz, ci)
    return {"algorithmic_bytes_per_launch": nb, "ms": round(ms, 4), "achieved_GBps": round(nb / (ms * 1e-3) / 1e9, 1),
            "frac": round(nb / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
            "equals_layer_pooled_half": bool(torch.equal(out, pl.bv_fused[..., spec.c_bev:]))}


def step_bytes(cfg, spec, nnz, u_pix, u_cell, F, esz):
    Hb, Wb = spec.bev_feat_hw
    Hi, Wi = spec.img_feat_hw
    cb, ci = spec.c_bev, spec.c_img
    nb, ni = F * Hb * Wb, F * Hi * Wi
    b = pull_bytes(nb, cb, ci, u_pix, nnz, esz, cb + ci)                  # bv_fused = [bev || pool(img)]
    if cfg in (3, 5):
        b += pull_bytes(ni, ci, cb, u_cell, nnz, esz, ci + cb)            # img_fused = [img || trans(bev)]
    if cfg == 3:
        b += pull_bytes(nb, cb, cb, u_pix, nnz, esz, cb)                  # d_bev = g[:, :Cb] + M^T g_img
        b += pull_bytes(ni, ci, ci, u_cell, nnz, esz, ci)                 # d_img = g[:, :Ci] + M g_bv
    return b


def cpu_baseline(spec, frames_np, budget_s, dual, backward=False, impl="c"):
    """The reference CPU path on one core, bounded sample (frames cycled until the budget):
    impl "numpy": the numpy restatement of the reference's own numpy index builder and of
    TF 1.8's sequential CPU pooling kernels (oracle/shpl_numpy.py: np.dot / np.round / masks,
    np.add.at); impl "c": the C port of the same path (oracle/shpl_oracle.c)."""
    if impl == "numpy":
        from oracle import shpl_numpy as orc
        what = "oracle/shpl_numpy.py (numpy: the reference's index builder, TF-CPU-order np.add.at pooling)"
    else:
        from oracle import shpl_oracle as orc
        what = "oracle/shpl_oracle.c (C port)"
    Hb, Wb = spec.bev_feat_hw
    Hi, Wi = spec.img_feat_hw
    rng = np.random.default_rng(0)
    bev = rng.standard_normal((1, Hb, Wb, spec.c_bev), dtype=np.float32)
    img = rng.standard_normal((1, Hi, Wi, spec.c_img), dtype=np.float32)
    if backward:
        g_bev_pool = rng.standard_normal((1, Hb, Wb, spec.c_img), dtype=np.float32)
        g_img_pool = rng.standard_normal((1, Hi, Wi, spec.c_bev), dtype=np.float32)
    t_index = t_pool = 0.0
    done = 0
    t0 = time.perf_counter()
    while done < 3 or (time.perf_counter() - t0 < budget_s and done < len(frames_np)):
        fr = frames_np[done % len(frames_np)]
        a = time.perf_counter()
        g = orc.gen_sparse_pooling_input_avod(fr.points, fr.voxel_indices, fr.P, list(spec.im_size),
                                              tuple(spec.bv_size))
        ref = orc.produce_sparse_pooling_input(g, stride=spec.stride)
        b = time.perf_counter()
        orc.sparse_pool_layer(bev, img, ref["Mij_pool"], ref["M_val"], ref["M_size"],
                              ref["img_index_flip_pool"], dual=dual)
        if backward:  # TF's gradients of both directions (the concat split is a view)
            Cb, Ci = spec.c_bev, spec.c_img
            orc.sparse_pool_grad_img(ref["Mij_pool"], ref["M_val"], ref["M_size"], g_bev_pool.reshape(-1, Ci),
                                     ref["img_index_flip_pool"], (1, Hi, Wi, Ci))
            orc.sparse_pool_trans_grad_bev(ref["Mij_pool"], ref["M_val"], ref["M_size"], g_img_pool,
                                           ref["img_index_flip_pool"])
        c = time.perf_counter()
        t_index += b - a
        t_pool += c - b
        done += 1
    total = t_index + t_pool
    return {"value": round(done / total, 3), "unit": "frames/s", "cores": 1, "kind": impl if impl == "numpy" else "port",
            "index_ms_per_frame": round(1e3 * t_index / done, 3), "pool_ms_per_frame": round(1e3 * t_pool / done, 3),
            "sample": (f"{done} frames of this workload ({spec.n_points} pts) through {what}: "
                       f"index build {1e3 * t_index / done:.2f} ms/frame + TF-order pooling and concat "
                       f"{1e3 * t_pool / done:.2f} ms/frame"
                       + ((" (both directions, forward + gradients, f32)" if backward else
                           " (both directions, forward only)") if dual else "")
                       + f", single thread, {os.cpu_count()} host cpus visible")}


def cpu_baselines(spec, frames_np, budget_s, dual, backward, parallel):
    """SURVEY §8d's CPU baseline: the C port of the reference path is the headline `value`
    ("kind": "port", since round 4; rounds 1-3 quoted the numpy leg), the numpy restatement
    beside it ("numpy": "kind": "numpy", the reference's own numpy index builder and TF-order
    np.add.at pooling), and the C port frame-parallel over the usable cores. Compare rounds by
    `kind`: the port leg is the faster one on every workload measured."""
    npy = cpu_baseline(spec, frames_np, budget_s, dual, backward, impl="numpy")
    port = cpu_baseline(spec, frames_np, budget_s, dual, backward, impl="c")
    out = dict(port, numpy=npy, port=dict(port))
    if parallel:
        out["parallel"] = cpu_baseline_parallel(spec, frames_np, budget_s, dual, backward)
    return out


def _cpu_worker(q, barrier, spec, frames_np, budget_s, dual, backward):
    barrier.wait()
    q.put(cpu_baseline(spec, frames_np, budget_s, dual, backward))


def usable_cores():
    """Host cores this process may run on: its affinity set, capped by the
    cgroup CPU quota when one is set (cpu.max; a GPU box's share of a large
    host shows every CPU in the affinity set but allows only its quota)."""
    aff = len(os.sched_getaffinity(0))
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as fh:
            q, period = fh.read().split()[:2]
        if q != "max":
            quota = max(1, int(-(-int(q) // int(period))))
    except (OSError, ValueError):
        pass
    return (min(aff, quota) if quota else aff), aff, quota


def cpu_baseline_parallel(spec, frames_np, budget_s, dual, backward=False):
    """Frame-parallel form of cpu_baseline (single thread and
    N-process frame-parallel): one spawned process per usable host core (every
    core of the affinity set, capped by the cgroup quota), each starting at
    its own frame, started together; the aggregate is the sum of the
    processes' rates."""
    import multiprocessing as mp
    n, aff, quota = usable_cores()
    ctx = mp.get_context("spawn")
    q, bar = ctx.Queue(), ctx.Barrier(n)
    procs = [ctx.Process(target=_cpu_worker,
                         args=(q, bar, spec, frames_np[i:] + frames_np[:i], budget_s, dual, backward))
             for i in range(n)]
    for p in procs:
        p.start()
    try:
        res = [q.get(timeout=10 * budget_s + 300) for _ in procs]
    finally:
        for p in procs:
            p.join(timeout=60)
    return {"value": round(sum(r["value"] for r in res), 3), "unit": "frames/s", "cores": n, "processes": n,
            "sample": f"{n} processes started together (all usable cores: affinity set of {aff} cpus, cgroup "
                      f"quota {quota if quota else 'none'}), each the single-thread sample ({budget_s:.0f} s) "
                      f"from its own first frame"}


def self_launch(args):
    """`--gpus N` (N > 1) without a launcher: start N ranks, one per GPU, as
    torch.distributed.run children, and wait for them. Nothing in this
    process has touched HIP (no device call before this point), so it is a
    plain parent, not an exec of a GPU process."""
    import socket
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", f"--master-port={port}", os.path.abspath(__file__), *sys.argv[1:]]
    return subprocess.call(cmd)


def checksum_report(base, local, fids, dev, rank, args):
    """All-gather the per-frame checksums and their global frame ids (rank order),
    compare each frame with the N=1 run's checksum of the same global frame id
    (profiles/frame_checksums.json: tables `<base>_frames<n>`, frame i at index i;
    a frame's output does not depend on its rank or on what shares its launch, so
    any partition or sub-batch is checked), store them with --write-checksums."""
    from sparse_pooling_amd import dist as sd
    allcs = sd.gather_frame_checksums(local, device=dev)
    allfids = sd.gather_frame_checksums(torch.as_tensor(fids, dtype=torch.int64, device=dev), device=dev)
    tab = {}
    if os.path.exists(CHECKSUM_FILE):
        with open(CHECKSUM_FILE) as fh:
            tab = json.load(fh)
    tables = [(k, v) for k, v in tab.items() if k.startswith(base + "_frames")]
    ref_key, ref = max(tables, key=lambda kv: len(kv[1])) if tables else (None, None)
    match = None
    if ref is not None and allfids and max(allfids) < len(ref):
        match = all(ref[f] == c for f, c in zip(allfids, allcs))
    if args.write_checksums and rank == 0:
        if allfids != list(range(len(allfids))):
            raise SystemExit("--write-checksums needs the frames 0..n-1 of a whole batch")
        tab[f"{base}_frames{len(allcs)}"] = allcs
        with open(CHECKSUM_FILE, "w") as fh:
            json.dump(tab, fh, indent=0)
    return {"key": base, "frames": len(allcs), "frame_ids": [min(allfids), max(allfids)] if allfids else None,
            "compared_with": ref_key, "pinned_to": pinned_to(ref_key), "checksum": CHECKSUM_DEF,
            "digest": hashlib.sha256(json.dumps(allcs).encode()).hexdigest()[:16],
            "match_n1": match, "first": allcs[:4]}


CHECKSUM_DEF = "sum_i bits[i]*(2i+1) mod 2^64 per output (row-major), outputs combined as sum_k cs_k*(2k+1)"


def pinned_to(key):
    """What a stored table was computed by: the layer and raw-scan tables by the CPU oracle
    (tests/golden/make_checksum_tables.py; TF-order arithmetic, so bitwise); the conv tables by a GPU run
    (TF's Conv2D fixes no summation order, so no oracle checksum exists: the conv is tolerance-tested against
    the oracle's double-precision conv in tests/test_gpu_conv.py) -- self-referential."""
    if key is None:
        return None
    if key.startswith("layer_config") or key.startswith("frames_"):
        return "oracle"
    return ("gpu-run (self-referential; frames 0-1 rebuilt and checked against the oracle's double conv within "
            "tolerance: tests/test_gpu_checksums_oracle.py::test_conv_table_is_a_tolerance_checked_output)")


def lib_sha256():
    """Content hash of the HIP library this run loaded (traffic provenance)."""
    from sparse_pooling_amd import _lib as L
    with open(L.LIB_PATH, "rb") as fh:
        return hashlib.sha256(fh.read()).hexdigest()[:16]


def traffic_lookup(key, field="hbm_bytes_per_launch"):
    """PMC HBM bytes of `key` in profiles/traffic.json, only when they were
    measured on the library this run loaded: (value, note, entry)."""
    tpath = os.path.join(HERE, "profiles", "traffic.json")
    if not os.path.exists(tpath):
        return None, "no profiles/traffic.json", None
    with open(tpath) as fh:
        tj = json.load(fh).get(key)
    if not tj:
        return None, f"no PMC entry {key}", None
    here = lib_sha256()
    if tj.get("lib_sha256") != here:
        return None, (f"stale: {key} was measured on libshpl.so {tj.get('lib_sha256')} "
                      f"(commit {tj.get('commit')}), this run loaded {here}"), None
    return tj[field], f"PMC of {key}, libshpl.so {here}, commit {tj.get('commit')}", tj


def main():
    args = parse()
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(self_launch(args))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if args.gpus != world:
        sys.exit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world} (launch one rank per GPU, or drop the "
                 "launcher and let --gpus start the ranks)")
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # SHPL_DIST_BACKEND=gloo: rehearsal of the N>1 path with several ranks on
    # one GPU (ranks share device LOCAL_RANK mod the device count); the
    # driver's runs use RCCL ("nccl"), one rank per GPU.
    backend = os.environ.get("SHPL_DIST_BACKEND", "nccl")
    if backend != "nccl":
        local %= max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        import torch.distributed as dist
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)

    from sparse_pooling_amd import dist as sd, pipeline, synth

    if args.workload in ("frames", "conv"):
        (run_frames if args.workload == "frames" else run_conv)(args, world, rank, dev)
        if world > 1:
            dist.destroy_process_group()
        return

    cfg = args.config
    if args.graph_steps is None:
        # config 3 (~70 us steps): several steps per replay, so the graph launch is amortised (8: 0.0694-0.0701 vs
        # 4: 0.0704-0.0707 ms per step, profiles/r05_c3gs_ab.log)
        args.graph_steps = (8 if args.steps % 8 == 0 else 4 if args.steps % 4 == 0 else 1) if cfg == 3 else 1
    spec = synth.CONFIGS[cfg]
    dual = cfg in (3, 5)
    backward = cfg == 3
    dtype = torch.bfloat16 if cfg == 3 else torch.float32
    esz = 2 if dtype == torch.bfloat16 else 4
    fids = sd.partition(args.frames or DEFAULT_FRAMES[cfg], world, rank, args.partition)
    F = len(fids)
    frames = [synth.make_frame(spec, seed=s, n_outside=200) for s in fids]
    pts, vox, off, P, maxp, N = pipeline.stack_frames(frames, dev)
    pipeline.FusedPipeline.PIXEL_COLS = args.pixel_cols
    pipeline.FusedPipeline.SPLIT_ONCE = args.split_pull == "once"
    pipeline.FusedPipeline.SPLIT_SERIAL = args.split_form == "serial"
    if args.head_k is not None:
        pipeline.FusedPipeline.HEAD_K = args.head_k
    esz0 = 2 if dtype == torch.bfloat16 else 4
    split = (not dual and not args.rows and not args.no_overlap and
             (args.split == "on" or (args.split == "auto" and min(spec.c_bev, spec.c_img) * esz0 >= 1024)))
    pl = pipeline.FusedPipeline(F, maxp, N, spec.im_size, spec.bv_size, spec.stride, spec.c_bev,
                                spec.c_img, dtype=dtype, dual=dual, device=dev, rows=True if args.rows else None,
                                buckets=False if args.no_buckets else None, split=split)
    chain = torch.cuda.Stream(device=dev, priority=-1) if split else None
    if split and args.split_chain == "current":
        # every launch of this run on the high-priority stream: a caller whose layer runs on such a stream
        torch.cuda.set_stream(chain)
    Hb, Wb = spec.bev_feat_hw
    Hi, Wi = spec.img_feat_hw
    feats = lambda shape, seed: sd.fill_features(torch.empty(shape, dtype=dtype, device=dev), fids, seed)  # noqa
    bev = feats((F, Hb, Wb, spec.c_bev), 1)
    img = feats((F, Hi, Wi, spec.c_img), 2)
    if backward:
        g_bv = feats(tuple(pl.bv_fused.shape), 3)
        g_img = feats(tuple(pl.img_fused.shape), 4)
        d_bev, d_img = torch.empty_like(bev), torch.empty_like(img)
    side = torch.cuda.Stream(device=dev)
    side2 = torch.cuda.Stream(device=dev) if dual else None  # pixel-keyed CSR / pulls beside the cell-keyed
    pl.interleave = not args.no_interleave
    pl.riders = not args.no_riders
    from sparse_pooling_amd import _lib as L
    pl.csr_path = {"auto": L.CSR_AUTO, "frame": L.CSR_FRAME, "segment": L.CSR_SEGMENT,
                   "range": L.CSR_RANGE}[args.csr_path]

    def step(ev=None):
        # ev: [dense start, dense end, sparse start, sparse end, bwd start, bwd end]
        if args.no_overlap:
            pl.build_index(pts, vox, off, P)
            pl.build_csr()
            if ev is not None:
                ev[0].record()
            pl.layer_dense(bev, img)
            if ev is not None:
                ev[1].record()
                ev[2].record()
            pl.layer_sparse(bev, img)
            if ev is not None:
                ev[3].record()
        elif split and args.split_chain == "current":
            # the layer called on the high-priority stream the whole run is on (below): the chain runs there,
            # only the copy forks to `side`
            pl.step_split(pts, vox, off, P, bev, img, side, None, events=ev[:4] if ev else None)
        elif split:
            pl.step_split(pts, vox, off, P, bev, img, side, chain, events=ev[:4] if ev else None)
        else:
            pl.step_overlapped(pts, vox, off, P, bev, img, side, events=ev[:4] if ev else None, side2=side2)
        if backward:
            if ev is not None:
                ev[4].record()
            pl.backward(g_bv, g_img, d_bev, d_img, side2=None if args.no_overlap else side2)
            if ev is not None:
                ev[5].record()

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    nnz = int(pl.frame_nnz.sum().item())
    u_pix = int(torch.unique(pl.pix[pl.pix >= 0]).numel())
    u_cell = int(torch.unique(pl.cell[pl.cell >= 0]).numel())
    err = int(pl.err.item())

    # One step captured as a HIP graph (torch.cuda.graph over hipStreamBeginCapture):
    # the timed loop replays it, so host launch gaps leave the step. Kernel
    # durations for the roofline come from the same step run eagerly with events.
    graph, graph_note = None, None
    if split and not args.graph and args.split_form == "overlap":
        # a captured graph of the split step ran its two branches nearly in series (the chain's nodes start
        # after the copy has filled the chip: no stream priority inside a graph): 1.77 vs 1.40 ms eager at
        # config 6 (profiles/r05_c6b_ab.log); --graph forces the capture
        graph_note = "split step: eager launches (the chain's high-priority stream; a captured graph serialised it)"
    elif not args.no_graph:
        try:
            gstream = torch.cuda.Stream(device=dev)
            gstream.wait_stream(torch.cuda.current_stream(dev))
            graph = torch.cuda.CUDAGraph()
            if args.steps % args.graph_steps:
                sys.exit(f"bench.py: --steps {args.steps} is not a multiple of --graph-steps {args.graph_steps}")
            with torch.cuda.graph(graph, stream=gstream):
                for _ in range(args.graph_steps):
                    step()
            graph.replay()
            torch.cuda.synchronize()
        except Exception as e:  # noqa: BLE001 -- report and run eagerly
            graph, graph_note = None, f"graph capture failed, eager launches: {type(e).__name__}: {e}"[:200]
    n_ev = min(args.steps, 10) if graph is not None else args.steps
    evs = [[torch.cuda.Event(enable_timing=True) for _ in range(6)] for _ in range(n_ev)]
    issue_ms = replay_step_ms = None
    if graph is not None:
        replays = args.steps // args.graph_steps
        tinfo = {}
        elapsed = sd.timed(lambda k: graph.replay(), replays, device=dev, info=tinfo)
        # host cost of one replay: issue the replays without waiting (after the timed loop); well
        # under the step at every config (0.03 ms at config 3), so the timed loop is not launch-bound
        torch.cuda.synchronize()
        r0, r1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        r0.record()
        t0 = time.perf_counter()
        for _ in range(replays):
            graph.replay()
        issue_ms = 1e3 * (time.perf_counter() - t0) / replays
        r1.record()
        torch.cuda.synchronize()
        # the replayed step's device time by HIP events on the replay stream (every kernel back to back)
        replay_step_ms = r0.elapsed_time(r1) / (replays * args.graph_steps)
        for k in range(n_ev):
            step(evs[k])
        torch.cuda.synchronize()
    else:
        tinfo = {}
        elapsed = sd.timed(lambda k: step(evs[k]), args.steps, device=dev, info=tinfo)
    args_steps_ev = n_ev
    # every error bit the steps set, the timed ones included (FusedPipeline.check: one read, outside the timed
    # region): SHPL_EBIT_BARRIER or an input error ends the run here instead of reporting invalid results
    pl.check()
    outs = [pl.bv_fused] + ([pl.img_fused] if dual else []) + ([d_bev, d_img] if backward else [])
    checks = checksum_report(f"layer_config{cfg}", sd.combine_checksums([sd.frame_checksums(t) for t in outs]), fids,
                             dev, rank, args)
    comm = sd.comm_report(dev)
    nbytes = step_bytes(cfg, spec, nnz, u_pix, u_cell, F, esz)
    interleaved = dual and not args.no_overlap and not pl.rows and pl.interleave
    dense_ms = sum(e[0].elapsed_time(e[1]) for e in evs) / args_steps_ev
    sparse_ms = sum(e[2].elapsed_time(e[3]) for e in evs) / args_steps_ev
    bwd_ms = sum(e[4].elapsed_time(e[5]) for e in evs) / args_steps_ev if backward else 0.0
    layer_ms = dense_ms + sparse_ms + bwd_ms
    if interleaved:
        # the cell-keyed sparse pass runs beside img_fused's dense pass: the layer's window
        # (first k_dense start -> last k_sparse end) instead of the summed durations
        layer_ms = sum(e[0].elapsed_time(e[3]) for e in evs) / args_steps_ev + bwd_ms
    eager_ms = None
    if split:
        # the two halves' passes overlap each other and the chain: the layer's window from the first start to
        # the last end (eager), or the replayed step (every kernel of it)
        layer_ms = sum(max(e[2].elapsed_time(e[1]), e[2].elapsed_time(e[3])) for e in evs) / args_steps_ev
        if replay_step_ms is not None:
            eager_ms, layer_ms = layer_ms, replay_step_ms
    if getattr(pl, "buckets", False) and replay_step_ms is not None:
        # the bucketed one-queue step: its brackets span every kernel of the step, and run eagerly they
        # also hold the host's launch gaps between ~10 us kernels; the replayed step is the same kernels
        # back to back (rocprof's per-kernel averages sum to it)
        eager_ms, layer_ms = layer_ms, replay_step_ms
    # N > 1: every rank's kernel times and bytes; the roofline describes the slowest rank (its own bytes
    # over its own layer time), the per-rank list beside it
    per_rank = sd.gather_floats([layer_ms, dense_ms, sparse_ms, bwd_ms, nbytes], device=dev)
    slow = max(range(len(per_rank)), key=lambda r: per_rank[r][0])
    layer_ms, dense_ms, sparse_ms, bwd_ms, nbytes = per_rank[slow][:4] + [int(per_rank[slow][4])]
    achieved = nbytes / (layer_ms * 1e-3) / 1e9
    pool = (pool_fwd_report(pl, img, spec, F, u_pix, nnz, esz, dev)
            if cfg == 2 and not args.no_pool_report else None)

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baselines(spec, frames[: min(F, 64)], args.cpu_seconds, dual, backward, not args.no_cpu_parallel)

    if rank == 0:
        total_frames = F * world * args.steps
        traffic, traffic_note, _ = traffic_lookup(f"config{cfg}_F{F}")
        what = {2: "img->BEV SHPL fwd", 3: "dual SHPL fwd + bwd (bf16 storage, f32 accumulate)",
                5: "dual SHPL fwd (img->BEV and BEV->img)",
                6: "img->BEV SHPL fwd at RetinaNet's P2 (stride 4, FPN 256 ch; not a BASELINE config)"}[cfg]
        out = {
            "metric": "SHPL fused frames/sec + achieved HBM GB/s (% of MI355X peak), 1/2/4/8 GPU",
            "value": round(total_frames / elapsed, 2),
            "unit": "frames/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(1e3 * elapsed / args.steps, 4),
            "higher_is_better": True,
            "scaling": args.partition,
            "vs_baseline": None,
            "dtype": "bf16" if esz == 2 else "f32",
            "data": "synthetic (seeded KITTI-shaped frames; no dataset on the box)",
            "config": {
                "workload": (f"config{cfg}: {spec.n_points} pts/frame, BEV {Hb}x{Wb}x{spec.c_bev}, "
                             f"img {Hi}x{Wi}x{spec.c_img}, {what}; step = device index build + sorted M "
                             "+ fused layer" + (" + gradient" if backward else "")),
                "global_batch": F * world,
                "frames_per_gpu_per_step": F,
                "partition": (f"{args.partition}: rank r owns global frames [r*{F}, (r+1)*{F}) of {F * world}"),
                "nnz_per_step_rank0": nnz,
                "unique_src_pixels_rank0": u_pix,
                "unique_cells_rank0": u_cell,
                "overlap_index_build": not args.no_overlap,
                **({"split": True} if split else {}),
                "hip_graph": graph is not None,
                **({"steps_per_graph": args.graph_steps} if graph is not None and args.graph_steps > 1 else {}),
                **({"graph_issue_ms_per_replay": round(issue_ms, 4)} if issue_ms is not None else {}),
                **({"graph_note": graph_note} if graph_note else {}),
                "parallelism": f"frame-sharded x{world}",
            },
            "roofline": {
                "bound": "hbm",
                "kernel": ("SHPL layer pulls: k_dense (concat stream) + k_sparse (pooled gather); achieved over "
                           + (("the layer's window (first k_dense start to last k_sparse end: the cell-keyed "
                               "gathers run beside img_fused's stream)") if interleaved else
                              "their summed durations")
                           + (("; split step (the pass-through copy k_dense beside the index chain, then the "
                               "pooled half written once by shpl_pull_once's k_once): every kernel of the step, "
                               + ("timed as the replayed step (HIP events around the graph replays)"
                                  if graph is not None else "the eager step's window from the chain's start"))
                              if split else "")
                           + ("; bucketed one-stream step: the forward bracket spans the whole forward "
                              "(index + buckets with the pass-through copies riding its launches, both CSRs, the "
                              "pooled pull pair), the backward bracket the gradient pull pair -- every kernel of "
                              "the step, so achieved = the step's algorithmic bytes over all of its kernel time, timed as the replayed "
                              "step (HIP events around the graph replays)"
                              if pl.buckets else
                              "; step pulls are row-keyed k_rows (one launch per pull), timed as the sparse and "
                              "backward brackets" if pl.rows else "")),
                "achieved": round(achieved, 1),
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4),
                "traffic": traffic,
                "traffic_note": traffic_note,
                "algorithmic_bytes_per_launch": nbytes,
                "kernel_ms": round(layer_ms, 4),
                **({"kernel_ms_source": "HIP events around the graph replays (per step)",
                    "eager_brackets_ms": round(eager_ms, 4)} if eager_ms is not None else {}),
                "k_dense_ms": round(dense_ms, 4),
                "k_sparse_ms": round(sparse_ms, 4),
                "backward_ms": round(bwd_ms, 4),
                "rank": slow,
                **({"per_rank": [{"rank": r, "kernel_ms": round(v[0], 4), "k_dense_ms": round(v[1], 4),
                                  "k_sparse_ms": round(v[2], 4), "backward_ms": round(v[3], 4),
                                  "algorithmic_bytes": int(v[4]),
                                  "frac": round(v[4] / (v[0] * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)}
                                 for r, v in enumerate(per_rank)]} if world > 1 else {}),
                **({"pool_fwd": pool} if pool else {}),
            },
            "cpu_baseline": cpu,
            "index_errors": err,
            "timing": tinfo,
            "frame_checksums": checks,
            "comm": comm,
            "lib_sha256": lib_sha256(),
        }
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


def cpu_baseline_frames(frames_np, calib, plane, im_size, c, budget_s):
    """Oracle chain of the frames workload on one core: velodyne -> camera frame + FOV
    filter -> BEV slices (maps + voxel indices) -> gen + produce -> pool + concat."""
    from oracle import shpl_oracle as orc
    from sparse_pooling_amd import synth
    rect = orc.rect_matrix(calib.r0_rect, calib.tr_velodyne_to_cam)
    nx, nz = 800, 700
    rng = np.random.default_rng(0)
    bev = rng.standard_normal((1, nz, nx, c), dtype=np.float32)
    img = rng.standard_normal((1, im_size[1], im_size[0], c), dtype=np.float32)
    t = {"load": 0.0, "bev": 0.0, "index": 0.0, "pool": 0.0}
    done = 0
    t0 = time.perf_counter()
    while done < 2 or (time.perf_counter() - t0 < budget_s and done < len(frames_np)):
        a = time.perf_counter()
        pc = orc.velo_to_cam(frames_np[done % len(frames_np)], rect, calib.p2, im_size)
        b = time.perf_counter()
        hm, dm, vox, upts = orc.bev_slices(pc, plane, synth.AREA_EXTENTS, synth.VOXEL_SIZE, synth.HEIGHT_LO,
                                           synth.HEIGHT_HI, synth.NUM_SLICES)
        cc = time.perf_counter()
        g = orc.gen_sparse_pooling_input_avod(upts, vox, calib.p2, list(im_size), (nz, nx))
        ref = orc.produce_sparse_pooling_input(g, stride=(1, 1))
        d = time.perf_counter()
        orc.sparse_pool_layer(bev, img, ref["Mij_pool"], ref["M_val"], ref["M_size"], ref["img_index_flip_pool"])
        e = time.perf_counter()
        t["load"] += b - a
        t["bev"] += cc - b
        t["index"] += d - cc
        t["pool"] += e - d
        done += 1
    total = sum(t.values())
    return {"value": round(done / total, 3), "unit": "frames/s", "cores": 1, "kind": "port",
            "sample": (f"{done} scans through oracle/shpl_oracle.c, single thread: velodyne->camera + FOV "
                       f"{1e3 * t['load'] / done:.2f} ms, BEV slices {1e3 * t['bev'] / done:.2f} ms, index "
                       f"{1e3 * t['index'] / done:.2f} ms, pooling + concat {1e3 * t['pool'] / done:.2f} ms per "
                       f"frame; {os.cpu_count()} host cpus visible")}



def run_frames(args, world, rank, dev):
    """Raw-scan workload: the whole per-frame SHPL path of kitti_dataset.py:285-379 +
    rpn_model.py's fused layer, from velodyne scans resident in HBM."""
    from sparse_pooling_amd import dist as sd, kitti, pipeline, synth
    fids = sd.partition(args.frames or 64, world, rank, args.partition)
    F = len(fids)
    C = 32
    h, w = synth.KITTI_IMAGE_SHAPE
    im_size = (w, h)
    fr = kitti.synthetic_frames(F, args.scan_points, seed=1000, device=dev, frame_ids=fids)
    pl = pipeline.FramePipeline(F, fr.total_points, im_size, synth.AREA_EXTENTS, synth.VOXEL_SIZE,
                                synth.HEIGHT_LO, synth.HEIGHT_HI, synth.NUM_SLICES, (1, 1), C, C, device=dev,
                                max_points_per_frame=fr.max_points)
    pl.maps_after = args.maps_after
    pl.dense_after = args.dense_after
    pl.maps_form = args.maps_form
    bev = sd.fill_features(torch.empty((F, pl.Hb, pl.Wb, C), device=dev), fids, 5)
    img = sd.fill_features(torch.empty((F, pl.Hi, pl.Wi, C), device=dev), fids, 6)
    # the index chain on a high-priority stream: its 1024-thread workgroups otherwise wait for
    # whole CUs to drain of k_dense's workgroups (BEV slices 1.07 -> 0.68 ms, step 2.86 -> 2.84 ms,
    # profiles/r02_priority.log; the step is then bound by k_dense + the sparse pass).
    # --stream-priority dense|both: A/B of the streaming pass at high priority (profiles/r04_prio_ab.log)
    side = torch.cuda.Stream(device=dev, priority=-1 if args.stream_priority in ("dense", "both") else 0)
    chain = torch.cuda.Stream(device=dev, priority=-1 if args.stream_priority in ("chain", "both") else 0)

    def velo_step(ev=None):
        with torch.cuda.stream(chain):
            pl.velo_step(fr, bev, img, side=side, events=ev)

    for _ in range(args.warmup):
        velo_step()
    torch.cuda.synchronize()
    nnz = int(pl.frame_nnz.sum().item())
    u_pix = int(torch.unique(pl.pix[pl.pix >= 0]).numel())
    n_cam = int(pl.velo.counts.sum().item())
    n_vox = int(pl.bev.frame_nvox.sum().item())
    errs = int(pl.err.item()) | int(pl.bev.err.item()) | int(pl.velo.err.item())
    evs = [[torch.cuda.Event(enable_timing=True) for _ in range(9)] for _ in range(args.steps)]
    tinfo = {}
    elapsed = sd.timed(lambda k: velo_step(evs[k]), args.steps, device=dev, info=tinfo)
    mean = lambda i, j: sum(e[i].elapsed_time(e[j]) for e in evs) / args.steps  # noqa: E731
    dense_ms, sparse_ms = mean(0, 1), mean(7, 8)
    stages = {"velo_to_cam_ms": mean(2, 3), "bev_slices_ms": mean(3, 4), "index_ms": mean(4, 5),
              "csr_ms": mean(5, 6), "k_dense_ms": dense_ms, "k_sparse_ms": sparse_ms}
    nbytes = pull_bytes(F * pl.Hb * pl.Wb, C, C, u_pix, nnz, 4, 2 * C)
    achieved = nbytes / ((dense_ms + sparse_ms) * 1e-3) / 1e9
    # the whole step's algorithmic bytes: scans in (16 B/point), camera-frame points out and back in (24 B),
    # the BEV maps out (5 height slices + density, f64), voxel indices + unique points (40 B/voxel), the index
    # (~16 B/entry out, 40 B/point in), the CSR (~40 B/entry) and the layer
    n_maps = synth.NUM_SLICES + 1
    map_esz = 8 if args.maps_form == "f64" else 4
    step_bytes = (nbytes + 16 * int(fr.total_points) + 2 * 24 * n_cam + F * pl.Hb * pl.Wb * n_maps * map_esz
                  + 40 * n_vox + 40 * n_vox + 56 * nnz)
    step_gbs = step_bytes / (elapsed / args.steps) / 1e9
    # PMC (scripts/r02_pmc.sh TAG=frames, traffic.py step frames_F64 ...), when measured on this library
    traffic, traffic_note, tj = traffic_lookup(f"frames_F{F}" if args.maps_form == "f64" else f"frames_bev_input_F{F}")
    step_traffic = tj.get("step_bytes_all_kernels") if tj else None
    checks = checksum_report(f"frames_{args.scan_points}", sd.frame_checksums(pl.bv_fused), fids, dev, rank, args)
    comm = sd.comm_report(dev)
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        scans = [fr.xyzi[int(fr.point_offsets[f]):int(fr.point_offsets[f + 1])].cpu().numpy() for f in range(min(F, 8))]
        calib = kitti.FrameCalibrationData()
        c = synth.KITTI_CALIB
        calib.p2 = np.array(c["P2"]).reshape(3, 4)
        calib.r0_rect = np.array(c["R0_rect"]).reshape(3, 3)
        calib.tr_velodyne_to_cam = np.array(c["Tr_velo_to_cam"]).reshape(3, 4)
        cpu = cpu_baseline_frames(scans, calib, fr.planes[0].cpu().numpy(), im_size, C, args.cpu_seconds)
    if rank == 0:
        out = {
            "metric": "SHPL frames/sec from raw velodyne scans (loader + BEV slices + index + fused layer)",
            "value": round(F * world * args.steps / elapsed, 2), "unit": "frames/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(1e3 * elapsed / args.steps, 4),
            "higher_is_better": True, "scaling": args.partition, "vs_baseline": None, "dtype": "f32",
            "data": "synthetic (seeded 64-beam-like velodyne scans, KITTI calib; no dataset on the box)",
            "config": {"workload": (f"frames: {args.scan_points} pts/scan -> {n_cam / F:.0f} FOV pts -> "
                                    f"{n_vox / F:.0f} BEV voxel pts -> {nnz / F:.0f} M entries; BEV "
                                    f"{pl.Hb}x{pl.Wb}x{C} (5 slices + density maps"
                                    + (", f64" if args.maps_form == "f64" else
                                       " as the network's f32 BEV input [F,nz,nx,6]") + f"), img "
                                    f"{pl.Hi}x{pl.Wi}x{C}, img->BEV fused layer"),
                       "maps_form": args.maps_form,
                       **({"dense_after": args.dense_after} if args.dense_after != "start" else {}),
                       "global_batch": F * world, "frames_per_gpu_per_step": F,
                       "parallelism": f"frame-sharded x{world}"},
            "stages_ms": {k: round(v, 4) for k, v in stages.items()},
            "frame_checksums": checks,
            "roofline": {"bound": "hbm", "kernel": "k_dense + k_sparse (fused layer)", "achieved": round(achieved, 1),
                         "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                         "traffic": traffic, "traffic_note": traffic_note, "algorithmic_bytes_per_launch": nbytes,
                         "step_traffic": step_traffic, "step_algorithmic_bytes": step_bytes, "step_GBps": round(step_gbs, 1),
                         "step_frac": round(step_gbs / HBM_PEAK_GBS, 4)},
            "cpu_baseline": cpu,
            "index_errors": errs,
            "timing": tinfo,
            "comm": comm,
            "lib_sha256": lib_sha256(),
        }
        print(json.dumps(out), flush=True)


def cpu_baseline_conv(spec, frames_np, budget_s, c_out=None, bias=False):
    """Oracle on one core: index build + TF-order pooling + concat of one frame,
    and the conv/BN/ReLU (bias: bias + ReLU) over a band of rows of it, scaled to the frame."""
    from oracle import shpl_oracle as orc
    Hb, Wb = spec.bev_feat_hw
    Hi, Wi = spec.img_feat_hw
    cb, ci = spec.c_bev, spec.c_img
    rng = np.random.default_rng(0)
    bev = rng.standard_normal((1, Hb, Wb, cb), dtype=np.float32)
    img = rng.standard_normal((1, Hi, Wi, ci), dtype=np.float32)
    c_out = ci if c_out is None else c_out
    w = (rng.standard_normal((3, 3, cb + ci, c_out)) * 0.05).astype(np.float32)
    sc = None if bias else np.full(c_out, 1.0 / np.sqrt(1.0 + 1e-3), np.float32)
    shift = np.linspace(-0.5, 0.5, c_out).astype(np.float32) if bias else None
    fr = frames_np[0]
    a = time.perf_counter()
    g = orc.gen_sparse_pooling_input_avod(fr.points, fr.voxel_indices, fr.P, list(spec.im_size), tuple(spec.bv_size))
    ref = orc.produce_sparse_pooling_input(g, stride=spec.stride)
    b = time.perf_counter()
    eb, _ = orc.sparse_pool_layer(bev, img, ref["Mij_pool"], ref["M_val"], ref["M_size"], ref["img_index_flip_pool"])
    c = time.perf_counter()
    rows, t_conv = 0, 0.0
    band = 8
    while rows < band or (t_conv < budget_s and rows + band <= Hb):
        d = time.perf_counter()
        orc.conv3x3(eb[:, max(rows - 1, 0):min(rows + band + 1, Hb)], w, None, sc, shift, True)
        t_conv += time.perf_counter() - d
        rows += band
    conv_frame = t_conv * Hb / rows
    total = (b - a) + (c - b) + conv_frame
    return {"value": round(1.0 / total, 4), "unit": "frames/s", "cores": 1, "kind": "port",
            "sample": (f"1 frame ({spec.n_points} pts) through oracle/shpl_oracle.c, single thread: index "
                       f"{1e3 * (b - a):.1f} ms + TF-order pooling and concat {1e3 * (c - b):.1f} ms + 3x3 conv "
                       f"{cb + ci}->{c_out}/{'bias' if bias else 'BN'}/ReLU (double accumulation) timed on {rows} of "
                       f"{Hb} rows, scaled: {1e3 * conv_frame:.0f} ms; "
                       f"{os.cpu_count()} host cpus visible")}


def cpu_baseline_train(spec, frames_np, budget_s):
    """Oracle on one core, the training step of the conv workload per frame: index build + TF-order pooling
    and concat (whole frame), the pooled channels' gradient back to the image (whole frame), and over bands
    of rows, scaled to the frame: the conv forward (double sums), BatchNorm forward with batch statistics +
    ReLU, BatchNorm / ReLU backward, the input gradient (conv on the flipped, transposed weights) and the
    weight gradient (oracle/shpl_oracle.c)."""
    from oracle import shpl_oracle as orc
    Hb, Wb = spec.bev_feat_hw
    Hi, Wi = spec.img_feat_hw
    cb, ci = spec.c_bev, spec.c_img
    rng = np.random.default_rng(0)
    bev = rng.standard_normal((1, Hb, Wb, cb), dtype=np.float32)
    img = rng.standard_normal((1, Hi, Wi, ci), dtype=np.float32)
    w = (rng.standard_normal((3, 3, cb + ci, ci)) * 0.05).astype(np.float32)
    gy = rng.standard_normal((1, Hb, Wb, ci), dtype=np.float32)
    fr = frames_np[0]
    a = time.perf_counter()
    g = orc.gen_sparse_pooling_input_avod(fr.points, fr.voxel_indices, fr.P, list(spec.im_size), tuple(spec.bv_size))
    ref = orc.produce_sparse_pooling_input(g, stride=spec.stride)
    b = time.perf_counter()
    eb, _ = orc.sparse_pool_layer(bev, img, ref["Mij_pool"], ref["M_val"], ref["M_size"], ref["img_index_flip_pool"])
    c = time.perf_counter()
    d_pool = rng.standard_normal((Hb * Wb, ci), dtype=np.float32)
    orc.sparse_pool_grad_img(ref["Mij_pool"], ref["M_val"], ref["M_size"], d_pool, ref["img_index_flip_pool"],
                             (1, Hi, Wi, ci))
    d = time.perf_counter()
    rows, t_band = 0, 0.0
    band = 8
    while rows < band or (t_band < budget_s and rows + band <= Hb):
        x = eb[:, max(rows - 1, 0):min(rows + band + 1, Hb)]
        e = time.perf_counter()
        _, raw = orc.conv3x3(x, w, raw=True)
        y, mean, var, _, _ = orc.batch_norm_train(raw, relu=True)
        g_raw, _, _ = orc.batch_norm_backward(raw, gy[:, :raw.shape[1]], True, mean, var, 1e-3, None, None, True)
        g32 = g_raw.astype(np.float32)
        orc.conv3x3_dgrad(g32, w)
        orc.conv3x3_wgrad(x, g32)
        t_band += time.perf_counter() - e
        rows += band
    band_frame = t_band * Hb / rows
    total = (b - a) + (c - b) + (d - c) + band_frame
    return {"value": round(1.0 / total, 5), "unit": "frames/s", "cores": 1, "kind": "port",
            "sample": (f"1 frame ({spec.n_points} pts) through oracle/shpl_oracle.c, single thread: index "
                       f"{1e3 * (b - a):.1f} ms + TF-order pooling and concat {1e3 * (c - b):.1f} ms + the pooled "
                       f"gradient to the image {1e3 * (d - c):.1f} ms + conv forward / BatchNorm (batch statistics) "
                       f"+ ReLU / their backward / input gradient / weight gradient (double accumulation) timed on "
                       f"{rows} of {Hb} rows, scaled: {1e3 * band_frame:.0f} ms; {os.cpu_count()} host cpus visible")}


def run_conv_train(args, world, rank, dev, spec, fids, dtype, pl, pts, vox, off, P, bev, img, conv):
    """Training step of the fused SHPL + post-fusion conv: index build, then
    FusionConv.fused with batch-statistics BatchNorm, then its backward
    (autograd over the device kernels): gradients of bev, img, the weights and
    beta. Eager launches (autograd allocates per step). BatchNorm statistics
    are the rank's own frames' (no cross-rank sync; data-parallel weight
    gradients would need an all-reduce, out of scope per SURVEY §8e)."""
    from sparse_pooling_amd import dist as sd, synth
    F = len(fids)
    Hb, Wb = spec.bev_feat_hw
    cb, ci = spec.c_bev, spec.c_img
    esz = 2 if dtype == torch.bfloat16 else 4
    conv.WGRAD_REUSE = not args.no_wgrad_reuse
    conv.DGRAD_OCC = not args.no_dgrad_occ
    if args.img_beside is not None:
        conv.IMG_BESIDE_WGRAD = args.img_beside == "wgrad"
    if args.wgrad_side is not None:
        conv.WGRAD_SIDE = args.wgrad_side == "on"
    if args.img_zero_side is not None:
        conv.IMG_ZERO_SIDE = args.img_zero_side == "on"
    conv.weights.requires_grad_(True)
    conv.beta.requires_grad_(True)
    tb, ti = bev.clone().requires_grad_(True), img.clone().requires_grad_(True)
    gy = sd.fill_features(torch.empty((F, Hb, Wb, ci), dtype=dtype, device=dev), fids, 7)

    def step(ev=None):
        pl.build_index(pts, vox, off, P)
        smap = pl.map()
        for t in (tb, ti, conv.weights, conv.beta):
            t.grad = None
        if ev is not None:
            ev[0].record()
        y = conv.fused(tb, ti, smap, is_training=True)
        if ev is not None:
            ev[1].record()
        y.backward(gy)
        if ev is not None:
            ev[2].record()

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    tinfo = {}
    elapsed = sd.timed(lambda k: step(), args.steps, device=dev, info=tinfo)
    n_ev = min(args.steps, 5)
    evs = [[torch.cuda.Event(enable_timing=True) for _ in range(3)] for _ in range(n_ev)]
    for k in range(n_ev):
        step(evs[k])
    torch.cuda.synchronize()
    fwd_ms = sum(e[0].elapsed_time(e[1]) for e in evs) / n_ev
    bwd_ms = sum(e[1].elapsed_time(e[2]) for e in evs) / n_ev
    flops = 3 * 2.0 * F * Hb * Wb * 9 * (cb + ci) * ci  # forward, input gradient, weight gradient
    dname = "bf16" if esz == 2 else "f32"
    step_s = (fwd_ms + bwd_ms) * 1e-3
    tflops = flops / step_s / 1e12
    # algorithmic HBM bytes of the step's passes: pooled map written once (+ gathers), conv forward
    # reads [bev || pooled] and writes the pre-activation map, BN apply reads / writes it, BN backward reads gy and
    # raw twice and writes g_raw, the input gradient reads g_raw and writes both sources' gradients, the pooled
    # channels' gradient is gathered back to the image, the weight gradient reads [bev || pooled] and g_raw
    nnz = int(pl.frame_nnz.sum().item())
    ents = pl.cell[pl.cell >= 0]
    u_cell = int(torch.unique(ents).numel())
    u_pix = int(torch.unique(pl.pix[pl.pix >= 0]).numel())
    Hi, Wi = spec.img_feat_hw
    px = F * Hb * Wb * esz
    if esz == 2:  # bf16: both convs gather the pooled rows (compact per-run buffer), bv_fused is never stored
        # per pixel, in channels: forward cb read (the pooled half is gathered: u_pix rows below) + ci written,
        # BN apply 2 ci, BN backward 5 ci, input gradient ci read + (cb + ci) written (with DGRAD_OCC its pooled
        # channels' ci only at the u_cell occupied cells), weight gradient cb + ci read (its pooled half again
        # gathered); the image gradient's ci per image pixel written; the pooled rows' gathers (once per step
        # with the weight gradient reading the forward's operand, else twice) and the image gradient's gathers
        # of u_cell rows; the entries read by each of those passes
        n_pool = 1 if conv.WGRAD_REUSE else 2
        dgrad_occ = conv.WGRAD_REUSE and conv.DGRAD_OCC
        hbm_bytes = (px * ((cb + ci) + 2 * ci + 5 * ci + (ci + cb + (0 if dgrad_occ else ci)) + (cb + ci))
                     + F * Hi * Wi * ci * esz + (n_pool * u_pix + u_cell + (u_cell if dgrad_occ else 0)) * ci * esz
                     + (n_pool + 1) * 12 * nnz)
    else:  # f32: the pooled map written once in the forward, read by the forward and the weight gradient
        hbm_bytes = (px * (ci + (cb + ci + ci) + 2 * ci + 2 * ci + 3 * ci + (ci + cb + ci) + (cb + ci + ci))
                     + F * Hi * Wi * ci * esz + (u_pix + u_cell) * ci * esz + 2 * 12 * nnz)
    hbm_gbs = hbm_bytes / step_s / 1e9
    # the bound: the larger of the two floors (f32: MFMA; bf16: HBM)
    hbm_bound = hbm_bytes / (HBM_PEAK_GBS * 1e9) > flops / (MFMA_PEAK_TFS[dname] * 1e12)
    # PMC bytes of every SHPL kernel of a step (scripts/r02_pmc.sh TAG=train..., traffic.py step)
    traffic, traffic_note, _ = traffic_lookup(f"train_{dname}_F{F}")
    comm = sd.comm_report(dev)
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline_train(spec, [synth.make_frame(spec, seed=fids[0], n_outside=200)], args.cpu_seconds)
    if rank == 0:
        print(json.dumps({
            "metric": "SHPL + post-fusion conv training frames/sec (fwd + bwd), 1/2/4/8 GPU",
            "value": round(F * world * args.steps / elapsed, 2), "unit": "frames/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(1e3 * elapsed / args.steps, 4),
            "higher_is_better": True, "scaling": args.partition, "vs_baseline": None, "dtype": dname,
            "data": "synthetic (seeded KITTI-shaped frames, xavier-initialised conv weights)",
            "config": {"workload": (f"conv training: config2 -> index -> conv3x3 {cb + ci}->{ci} + BatchNorm (batch "
                                    "statistics) + ReLU of [bev || pool(img)] (bf16: pooling inside the forward conv and "
                                    "the weight gradient, bv_fused never stored; f32: the pooled map built once in the "
                                    "forward, reused by the weight gradient), backward to bev, img, weights, beta"),
                       "global_batch": F * world, "frames_per_gpu_per_step": F, "hip_graph": False,
                       "wgrad_reuse": conv.WGRAD_REUSE, "dgrad_occ": esz == 2 and conv.WGRAD_REUSE and conv.DGRAD_OCC,
                       "wgrad_side_stream": conv.WGRAD_SIDE,
                       "img_zero_side_stream": conv.IMG_ZERO_SIDE, "img_beside_wgrad": conv.IMG_BESIDE_WGRAD,
                       "bn_statistics": "per rank (no cross-rank sync)", "parallelism": f"frame-sharded x{world}"},
            "roofline": ({"bound": "hbm", "kernel": "the whole forward + backward step: algorithmic bytes of its passes "
                          "(pooled map, conv fwd, BN apply, BN backward x2, input and weight gradients, image "
                          "gradient) over the forward + backward time",
                          "achieved": round(hbm_gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                          "frac": round(hbm_gbs / HBM_PEAK_GBS, 4), "traffic": traffic, "traffic_note": traffic_note,
                          "algorithmic_bytes_per_step": hbm_bytes, "mfma_tflops": round(tflops, 2),
                          "mfma_frac": round(tflops / MFMA_PEAK_TFS[dname], 4)} if hbm_bound else
                         {"bound": "mfma", "kernel": "fwd + input-gradient + weight-gradient convs (3x the forward "
                          "flops) over the forward + backward time (BN, ReLU and the pooling gradient included)",
                          "achieved": round(tflops, 2), "peak": MFMA_PEAK_TFS[dname], "unit": "TFLOP/s",
                          "frac": round(tflops / MFMA_PEAK_TFS[dname], 4), "traffic": None,
                          "algorithmic_bytes_per_step": hbm_bytes, "hbm_GBps": round(hbm_gbs, 1),
                          "hbm_traffic_per_step": traffic, "traffic_note": traffic_note}),
            "fwd_ms": round(fwd_ms, 4), "bwd_ms": round(bwd_ms, 4),
            "cpu_baseline": cpu,
            "timing": tinfo,
            "comm": comm,
            "lib_sha256": lib_sha256(),
        }), flush=True)


def run_conv(args, world, rank, dev):
    """Config 2 + the post-fusion conv: index build -> cell CSR ->
    conv3x3(BN, ReLU) of [bev || pool(img)] with the pooling inside the conv's staging
    (bv_fused never written). The unfused form (fused layer -> bv_fused -> conv) is
    timed beside it."""
    from sparse_pooling_amd import dist as sd, fusion_conv as fc, pipeline, synth
    # config 2: rpn_model.py:338-346 (64 -> 32, BatchNorm + ReLU); config 6: retinanet_model.py:334-348, the
    # RetinaNet P2 SHPL's slim.conv2d(bev_fused, 256, [3, 3]) -- 512 -> 256 channels, bias + ReLU, no normalizer
    retina = args.config == 6
    if args.config not in (2, 6):
        sys.exit("bench.py --workload conv: --config 2 (rpn) or 6 (RetinaNet P2)")
    if retina and args.train:
        sys.exit("bench.py --workload conv --config 6: forward only (the reference trains it, but round 5 measures "
                 "the forward at its shape)")
    spec = synth.CONFIGS[args.config]
    fids = sd.partition(args.frames or 64, world, rank, args.partition)
    F = len(fids)
    dtype = torch.bfloat16 if args.dtype == "bf16" else torch.float32
    frames = [synth.make_frame(spec, seed=s, n_outside=200) for s in fids]
    pts, vox, off, P, maxp, N = pipeline.stack_frames(frames, dev)
    pipeline.FusedPipeline.PIXEL_COLS = args.pixel_cols
    pl = pipeline.FusedPipeline(F, maxp, N, spec.im_size, spec.bv_size, spec.stride, spec.c_bev, spec.c_img,
                                dtype=dtype, device=dev)
    from sparse_pooling_amd import _lib as L, shpl_map as sm
    pl.csr_path = sm.ShplMap.CSR_PATH = {"auto": L.CSR_AUTO, "frame": L.CSR_FRAME, "segment": L.CSR_SEGMENT,
                                         "range": L.CSR_RANGE}[args.csr_path]
    Hb, Wb = spec.bev_feat_hw
    Hi, Wi = spec.img_feat_hw
    cb, ci = spec.c_bev, spec.c_img
    bev = sd.fill_features(torch.empty((F, Hb, Wb, cb), dtype=dtype, device=dev), fids, 1)
    img = sd.fill_features(torch.empty((F, Hi, Wi, ci), dtype=dtype, device=dev), fids, 2)
    c_out = 256 if retina else ci
    # the same weights on every rank
    conv = (fc.FusionConv(cb + ci, c_out, batch_norm=False, bias=True, relu=True, dtype=dtype, device=dev, seed=0)
            if retina else fc.FusionConv(cb + ci, ci, dtype=dtype, device=dev, seed=0))
    if retina:  # a bias that is not all zeros (slim's zeros initializer would hide the epilogue)
        conv.bias.copy_(torch.linspace(-0.5, 0.5, c_out, device=dev))
    out = torch.empty((F, Hb, Wb, c_out), dtype=dtype, device=dev)
    out_unf = torch.empty_like(out)
    train = args.train_bn
    if args.train:
        run_conv_train(args, world, rank, dev, spec, fids, dtype, pl, pts, vox, off, P, bev, img, conv)
        return

    def step(ev=None):
        pl.build_index(pts, vox, off, P)
        pl.build_csr(("cell",))
        if ev is not None:
            ev[0].record()
        conv.fused_csr(bev, img, pl.csr, pl.frame_off, is_training=train, out=out)
        if ev is not None:
            ev[1].record()

    def unfused(ev):
        ev[0].record()
        pl.layer_dense(bev, img)
        pl.layer_sparse(bev, img)
        ev[1].record()
        conv(pl.bv_fused, is_training=train, out=out_unf)
        ev[2].record()

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    err = int(pl.err.item())
    graph = None
    if not args.no_graph and not train:
        gstream = torch.cuda.Stream(device=dev)
        gstream.wait_stream(torch.cuda.current_stream(dev))
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph, stream=gstream):
            step()
        graph.replay()
        torch.cuda.synchronize()
    n_ev = min(args.steps, 10)
    evs = [[torch.cuda.Event(enable_timing=True) for _ in range(2)] for _ in range(n_ev)]
    if graph is not None:
        tinfo = {}
        elapsed = sd.timed(lambda k: graph.replay(), args.steps, device=dev, info=tinfo)
    else:
        tinfo = {}
        elapsed = sd.timed(lambda k: step(), args.steps, device=dev, info=tinfo)
    for k in range(n_ev):
        step(evs[k])
    uev = [[torch.cuda.Event(enable_timing=True) for _ in range(3)] for _ in range(n_ev)]
    for k in range(n_ev):
        unfused(uev[k])
    torch.cuda.synchronize()
    same = bool(torch.equal(out, out_unf))
    conv_ms = sum(e[0].elapsed_time(e[1]) for e in evs) / n_ev
    pull_ms = sum(e[0].elapsed_time(e[1]) for e in uev) / n_ev
    uconv_ms = sum(e[1].elapsed_time(e[2]) for e in uev) / n_ev
    esz = 2 if dtype == torch.bfloat16 else 4
    flops = 2.0 * F * Hb * Wb * 9 * (cb + ci) * c_out
    nnz = int(pl.frame_nnz.sum().item())
    u_pix = int(torch.unique(pl.pix[pl.pix >= 0]).numel())
    hbm_bytes = F * Hb * Wb * (cb + c_out) * esz + u_pix * ci * esz + 12 * nnz  # read bev, write out, gather
    tflops = flops / (conv_ms * 1e-3) / 1e12
    checks = None if train else checksum_report(f"conv{'_c6' if retina else ''}_{args.dtype}", sd.frame_checksums(out),
                                                fids, dev, rank, args)
    comm = sd.comm_report(dev)
    traffic, traffic_note, tj = traffic_lookup(f"conv{'_c6' if retina else ''}_{args.dtype}_F{F}")
    mfma_busy = tj.get("mfma_busy_share") if tj else None
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline_conv(spec, frames[:1], args.cpu_seconds, c_out=c_out, bias=retina)
    if rank == 0:
        dname = "bf16" if esz == 2 else "f32"
        out_j = {
            "metric": "SHPL + post-fusion conv frames/sec (MFMA roofline), 1/2/4/8 GPU",
            "value": round(F * world * args.steps / elapsed, 2), "unit": "frames/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(1e3 * elapsed / args.steps, 4),
            "higher_is_better": True, "scaling": args.partition, "vs_baseline": None, "dtype": dname,
            "data": "synthetic (seeded KITTI-shaped frames, xavier-initialised conv weights; no dataset on the box)",
            "config": {"workload": (f"conv: config{args.config} ({spec.n_points} pts/frame, BEV {Hb}x{Wb}x{cb}, img "
                                    f"{Hi}x{Wi}x{ci}) -> index -> cell CSR -> conv3x3 {cb + ci}->{c_out} + "
                                    + ("bias + ReLU of [bev || pool(img)] (retinanet_model.py:334-348)" if retina else
                                       f"BatchNorm ({'training' if train else 'inference'}) + ReLU of [bev || "
                                       "pool(img)], pooling fused into the conv's staging (rpn_model.py:338-346)")),
                       "global_batch": F * world, "frames_per_gpu_per_step": F, "hip_graph": graph is not None,
                       "parallelism": f"frame-sharded x{world}"},
            "frame_checksums": checks,
            "roofline": {"bound": "mfma",
                         "kernel": ("shpl_conv3x3 call = k_pack_wide + k_occ_frame + k_pool_runs_wide + k_conv_wide "
                                    "(16x16-pixel tiles x 256 output channels per workgroup, halo and weights by "
                                    "LDS-DMA, pooled half gathered from the per-run buffer), MFMA "
                                    "v_mfma_f32_16x16x32_bf16" if esz == 2 and retina else
                                    "shpl_conv3x3 call = k_pack_w + k_occ_frame + k_pool_runs + k_conv_rows "
                                    "(row-streaming, pooled half gathered from the per-run buffer), MFMA "
                                    "v_mfma_f32_32x32x16_bf16" if esz == 2 else
                                    "shpl_conv3x3 call = k_pack_w + k_row_ptr + k_conv3x3 (tiled, pooling in the "
                                    "staging), MFMA v_mfma_f32_32x32x2_f32"),
                         "achieved": round(tflops, 2), "peak": MFMA_PEAK_TFS[dname], "unit": "TFLOP/s",
                         "frac": round(tflops / MFMA_PEAK_TFS[dname], 4), "traffic": traffic,
                         "traffic_note": traffic_note, "mfma_busy_share_pmc": mfma_busy,
                         "algorithmic_flops_per_launch": flops, "kernel_ms": round(conv_ms, 4),
                         "hbm_algorithmic_bytes_per_launch": hbm_bytes,
                         "hbm_GBps": round(hbm_bytes / (conv_ms * 1e-3) / 1e9, 1),
                         "hbm_frac": round(hbm_bytes / (conv_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                         # time at each peak: bf16 sits between the two (HBM's floor the higher), f32 is MFMA-bound
                         "floor_ms": {"mfma": round(flops / (MFMA_PEAK_TFS[dname] * 1e12) * 1e3, 4),
                                      "hbm": round(hbm_bytes / (HBM_PEAK_GBS * 1e9) * 1e3, 4)}},
            "unfused": {"pull_ms": round(pull_ms, 4), "conv_ms": round(uconv_ms, 4),
                        "total_ms": round(pull_ms + uconv_ms, 4), "fused_conv_ms": round(conv_ms, 4),
                        "bitwise_equal": same},
            "cpu_baseline": cpu,
            "index_errors": err,
            "timing": tinfo,
            "comm": comm,
            "lib_sha256": lib_sha256(),
        }
        print(json.dumps(out_j), flush=True)


if __name__ == "__main__":
    main()
