"""Config 4 on the GPU: bench.py's strong partition over 2 ranks
on one device (gloo control plane, SHPL_DIST_BACKEND=gloo; the driver's
scaling runs use RCCL, one rank per GPU) computes per-frame outputs identical
to the single-rank run of the same global batch. The 2-rank run goes
through bench.py's own `--gpus 2` self-launch."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
pytestmark = pytest.mark.gpu

COMMON = ["--frames", "4", "--steps", "2", "--warmup", "1", "--no-cpu-baseline"]


def _bench(args, env_extra=None, timeout=240):
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0", **(env_extra or {}))
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args], cwd=ROOT, env=env,
                       capture_output=True, text=True, timeout=timeout)
    assert p.returncode == 0, p.stdout[-2000:] + p.stderr[-4000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout[-2000:]
    return json.loads(lines[0])


@pytest.mark.parametrize("extra", [[], ["--config", "3"]])
def test_strong_partition_two_ranks_matches_one(extra):
    one = _bench(["--gpus", "1", *COMMON, *extra])
    two = _bench(["--gpus", "2", *COMMON, *extra], {"SHPL_DIST_BACKEND": "gloo"})
    assert one["n_gpus"] == 1 and two["n_gpus"] == 2
    assert two["scaling"] == "strong" and two["config"]["global_batch"] == 4
    assert two["config"]["frames_per_gpu_per_step"] == 2
    c1, c2 = one["frame_checksums"], two["frame_checksums"]
    assert c1["frames"] == c2["frames"] == 4
    assert c1["digest"] == c2["digest"], (c1, c2)
    assert one["index_errors"] == 0 and two["index_errors"] == 0
    assert two["comm"]["backend"] == "gloo" and two["comm"]["world_size"] == 2
    assert [r["rank"] for r in two["comm"]["ranks"]] == [0, 1]
    assert one["comm"]["world_size"] == 1 and one["lib_sha256"] == two["lib_sha256"]
    # the N > 1 roofline describes the slowest rank, every rank's kernel times beside it
    per = two["roofline"]["per_rank"]
    assert [r["rank"] for r in per] == [0, 1]
    assert two["roofline"]["kernel_ms"] == max(r["kernel_ms"] for r in per)
    assert two["roofline"]["rank"] == max(per, key=lambda r: r["kernel_ms"])["rank"]
    assert "per_rank" not in one["roofline"]
    assert two["timing"]["barrier_inclusive_s"] >= two["timing"]["elapsed_s"] > 0


def test_eight_frame_rank_shape_matches_stored_n1_table():
    """One rank of the driver's N=8 config-4 run owns 8 frames (the segmented CSR
    path): its per-frame checksums equal frames 0-7 of the stored 64-frame N=1
    table (profiles/frame_checksums.json), compared by global frame id."""
    one = _bench(["--gpus", "1", "--frames", "8", "--steps", "2", "--warmup", "1", "--no-cpu-baseline"])
    c = one["frame_checksums"]
    assert c["frames"] == 8 and c["frame_ids"] == [0, 7]
    assert c["compared_with"] == "layer_config2_frames64"
    assert c["match_n1"] is True, c
    assert one["config"]["frames_per_gpu_per_step"] == 8 and one["index_errors"] == 0


def test_sub_batch_over_two_ranks_matches_stored_n1_table():
    """A 32-frame global batch over 2 ranks on one device (16 frames per rank, the
    N=4 rank shape): every gathered frame matches the 64-frame N=1 table by its
    global frame id."""
    two = _bench(["--gpus", "2", "--frames", "32", "--steps", "2", "--warmup", "1", "--no-cpu-baseline",
                  "--partition", "strong"], {"SHPL_DIST_BACKEND": "gloo"})
    c = two["frame_checksums"]
    assert c["frames"] == 32 and c["frame_ids"] == [0, 31] and c["match_n1"] is True, c


def test_weak_partition_is_the_global_batch_of_frames_times_ranks():
    one = _bench(["--gpus", "1", *COMMON])
    two = _bench(["--gpus", "2", "--frames", "2", "--partition", "weak", "--steps", "2", "--warmup", "1",
                  "--no-cpu-baseline"], {"SHPL_DIST_BACKEND": "gloo"})
    assert two["scaling"] == "weak" and two["config"]["global_batch"] == 4
    assert one["frame_checksums"]["digest"] == two["frame_checksums"]["digest"]


def test_config4_eight_ranks_on_one_device_matches_stored_n1_table():
    """Config 4 at its real rank count: `bench.py --gpus 8` (self-launched, 8 ranks, gloo control plane on one
    device) strong-partitions the 64-frame batch, 8 frames per rank; every gathered frame equals the oracle-written
    64-frame N=1 table by its global frame id, the 8 ranks are distinct, and the roofline lists all 8 ranks."""
    eight = _bench(["--gpus", "8", "--steps", "2", "--warmup", "1", "--no-cpu-baseline", "--partition", "strong"],
                   {"SHPL_DIST_BACKEND": "gloo"}, timeout=420)
    assert eight["n_gpus"] == 8 and eight["config"]["global_batch"] == 64
    assert eight["config"]["frames_per_gpu_per_step"] == 8
    c = eight["frame_checksums"]
    assert c["frames"] == 64 and c["frame_ids"] == [0, 63] and c["compared_with"] == "layer_config2_frames64"
    assert c["match_n1"] is True, c
    assert eight["comm"]["world_size"] == 8
    assert sorted(r["rank"] for r in eight["comm"]["ranks"]) == list(range(8))
    per = eight["roofline"]["per_rank"]
    assert len(per) == 8 and [r["rank"] for r in per] == list(range(8))
    assert eight["roofline"]["kernel_ms"] == max(r["kernel_ms"] for r in per)
    assert eight["index_errors"] == 0
