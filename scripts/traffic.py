"""Per-launch HBM traffic of the SHPL kernels from the rocprofv3 PMC passes
(scripts/gpu_round.sh step `pmc`) -> profiles/traffic.json.

gfx950 corrections (MI355X_MICROARCH.md §HBM): FETCH_SIZE and WRITE_SIZE are
in KiB; FETCH_SIZE counts half the bytes of a wide (16 B/lane) coalesced
read, so it is doubled; WRITE_SIZE is exact for 16 B/lane stores."""
import csv
import glob
import json
import os
import re
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


SHORT = (("k_conv_wide", "k_conv_wide"), ("k_pool_runs_wide", "k_pool_runs_wide"), ("k_pack_wide", "k_pack_wide"),
         ("k_conv_rows<4, 2, true", "k_conv_rows_pooled_bf16"), ("k_conv_rows<4, 4, false", "k_conv_rows_dense_bf16"),
         ("k_pool_runs", "k_pool_runs"), ("k_occ_frame", "k_occ_frame"), ("k_pack_w", "k_pack_w"),
         ("k_conv3x3<float, true", "k_conv3x3_pooled_f32"), ("k_conv3x3<float, false", "k_conv3x3_dense_f32"),
         ("k_conv3x3<unsigned short, true", "k_conv3x3_pooled_bf16"),
         ("k_conv3x3<unsigned short, false", "k_conv3x3_dense_bf16"),
         ("k_dense", "k_dense"), ("k_sparse_long", "k_sparse_long"), ("k_sparse", "k_sparse"), ("k_csr_frame", "k_csr_frame"), ("k_compact", "k_compact"),
         ("k_count", "k_count"))


def stamp(*logs):
    """Provenance of a PMC entry: the lib_sha256 the profiled bench run printed (the library it loaded),
    the commit it was measured at (this tree's HEAD) and the pass logs it came from."""
    sha = None
    for name in logs:
        f = os.path.join(ROOT, "gpurun_out", name)
        if not os.path.exists(f):
            continue
        for line in open(f, errors="replace"):
            if line.startswith("{") and '"lib_sha256"' in line:
                sha = json.loads(line).get("lib_sha256") or sha
    if sha is None:
        sys.exit(f"traffic.py: no lib_sha256 in {logs}: the entry would not be bound to a library")
    try:
        import subprocess
        commit = subprocess.run(["git", "-C", ROOT, "rev-parse", "--short", "HEAD"], capture_output=True,
                                text=True).stdout.strip() or None
    except OSError:
        commit = None
    return {"lib_sha256": sha, "commit": commit, "pass_logs": list(logs)}


def per_kernel(counter, pattern=None):
    pattern = pattern or f"pmc_{counter}"
    files = glob.glob(os.path.join(ROOT, "gpurun_out", pattern, "**", "*counter_collection.csv"), recursive=True)
    acc = defaultdict(list)
    for f in files:
        for r in csv.DictReader(open(f)):
            if r.get("Counter_Name") != counter:
                continue
            name = r["Kernel_Name"]
            short = next((s for k, s in SHORT if k in name), name)
            acc[short].append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in acc.items()}


def conv(key, dt, tag=None):
    """scripts/gpu_conv_prof.sh passes: pmc_conv_<tag>_1 FETCH_SIZE, _2 WRITE_SIZE,
    _3 SQ_VALU_MFMA_BUSY_CYCLES + GRBM_GUI_ACTIVE (MFMA busy share, clock); tag = dt, or c6_<dt> (CFG=6)."""
    tag = tag or dt
    fetch = per_kernel("FETCH_SIZE", f"pmc_conv_{tag}_1")
    write = per_kernel("WRITE_SIZE", f"pmc_conv_{tag}_2")
    mfma = per_kernel("SQ_VALU_MFMA_BUSY_CYCLES", f"pmc_conv_{tag}_3")
    grbm = per_kernel("GRBM_GUI_ACTIVE", f"pmc_conv_{tag}_3")
    out = {}
    for k in sorted(set(fetch) | set(write)):
        f_b, w_b = 2 * fetch.get(k, 0.0) * 1024, write.get(k, 0.0) * 1024
        cyc = grbm.get(k, 0.0) / 8.0  # GRBM_GUI_ACTIVE sums the 8 XCDs
        out[k] = {"fetch_bytes": f_b, "write_bytes": w_b, "raw_FETCH_SIZE_KiB": fetch.get(k),
                  "raw_WRITE_SIZE_KiB": write.get(k), "SQ_VALU_MFMA_BUSY_CYCLES": mfma.get(k),
                  "GRBM_GUI_ACTIVE": grbm.get(k),
                  "mfma_busy_share": mfma.get(k, 0.0) / (1024 * cyc) if cyc else None}
    # bf16: the fused call is k_pack_w + k_occ_frame + k_pool_runs + k_conv_rows (row-streaming kernel);
    # f32: k_pack_w + k_row_ptr + k_conv3x3 (tiled)
    wide = tag.startswith("c6_") and dt == "bf16"
    main_k = "k_conv_wide" if wide else "k_conv_rows_pooled_bf16" if dt == "bf16" else f"k_conv3x3_pooled_{dt}"
    call = [main_k] + (["k_pool_runs_wide", "k_occ_frame", "k_pack_wide"] if wide else
                       ["k_pool_runs", "k_occ_frame", "k_pack_w"] if dt == "bf16" else [])
    path = os.path.join(ROOT, "profiles", "traffic.json")
    tj = json.load(open(path)) if os.path.exists(path) else {}
    tj[key] = {"hbm_bytes_per_launch": sum(out[k]["fetch_bytes"] + out[k]["write_bytes"] for k in call if k in out),
               **stamp(f"pmc_conv_{tag}_1.log", f"pmc_conv_{tag}_2.log"),
               "main_kernel": main_k, "mfma_busy_share": out[main_k]["mfma_busy_share"], "kernels": out,
               "note": (f"hbm_bytes_per_launch: the fused conv call ({' + '.join(call)}); FETCH_SIZE x2 (gfx950 "
                        "wide-read correction), KiB -> bytes; WRITE_SIZE exact (16 B/lane stores); mfma_busy_share "
                        "= MFMA busy cycles / (1024 SIMDs x GRBM_GUI_ACTIVE / 8 XCDs)")}
    json.dump(tj, open(path, "w"), indent=1)
    print(json.dumps(tj[key], indent=1))


def main(key):
    fetch = per_kernel("FETCH_SIZE")
    write = per_kernel("WRITE_SIZE")
    out = {}
    for k in sorted(set(fetch) | set(write)):
        f_b = 2 * fetch.get(k, 0.0) * 1024
        w_b = write.get(k, 0.0) * 1024
        out[k] = {"fetch_bytes": f_b, "write_bytes": w_b, "raw_FETCH_SIZE_KiB": fetch.get(k),
                  "raw_WRITE_SIZE_KiB": write.get(k)}
    layer = sum(out[k]["fetch_bytes"] + out[k]["write_bytes"] for k in ("k_dense", "k_sparse", "k_sparse_long")
                if k in out)
    path = os.path.join(ROOT, "profiles", "traffic.json")
    tj = json.load(open(path)) if os.path.exists(path) else {}
    tj[key] = {"hbm_bytes_per_launch": layer, "kernels": out,
               "note": "layer = k_dense + k_sparse (+ k_sparse_long); FETCH_SIZE x2 (gfx950 wide-read correction), KiB -> bytes"}
    json.dump(tj, open(path, "w"), indent=1)
    print(json.dumps(tj[key], indent=1))


LAYER = ("k_dense", "k_sparse", "k_sparse_long", "k_rows", "k_bpull", "k_once")


def step_traffic(key, tag, layer_kernels=LAYER, anchor="k_count"):
    """Per-step HBM bytes of the layer kernels of one bench workload from the
    scripts/r02_pmc.sh passes (gpurun_out/pmc_<tag>_FETCH_SIZE, _WRITE_SIZE):
    every launch's counters summed, divided by the steps profiled (the number of
    k_count launches: one index build per step)."""
    def launches(counter):
        files = glob.glob(os.path.join(ROOT, "gpurun_out", f"pmc_{tag}_{counter}", "**", "*counter_collection.csv"),
                          recursive=True)
        acc = defaultdict(lambda: [0.0, 0])
        for f in files:
            for r in csv.DictReader(open(f)):
                if r.get("Counter_Name") != counter:
                    continue
                name = r["Kernel_Name"]
                short = next((s for k, s in SHORT if k in name), None)
                if short is None:
                    m = re.search(r"(k_[A-Za-z0-9_]+)", name)
                    short = m.group(1) if m else name[:40]
                acc[short][0] += float(r["Counter_Value"])
                acc[short][1] += 1
        return acc
    fetch, write = launches("FETCH_SIZE"), launches("WRITE_SIZE")
    steps = fetch.get(anchor, [0, 0])[1] or 1
    out = {}
    for k in sorted(set(fetch) | set(write)):
        f_b = 2 * fetch.get(k, [0, 0])[0] * 1024 / steps
        w_b = write.get(k, [0, 0])[0] * 1024 / steps
        out[k] = {"fetch_bytes_per_step": f_b, "write_bytes_per_step": w_b,
                  "launches_per_step": fetch.get(k, [0, 0])[1] / steps}
    total = sum(v["fetch_bytes_per_step"] + v["write_bytes_per_step"] for v in out.values())
    layer = sum(v["fetch_bytes_per_step"] + v["write_bytes_per_step"] for k, v in out.items()
                if layer_kernels is None or k in layer_kernels)
    path = os.path.join(ROOT, "profiles", "traffic.json")
    tj = json.load(open(path)) if os.path.exists(path) else {}
    tj[key] = {"hbm_bytes_per_launch": layer, "step_bytes_all_kernels": total, "steps_profiled": steps,
               **stamp(f"pmc_{tag}_FETCH_SIZE.log", f"pmc_{tag}_WRITE_SIZE.log"), "kernels": out,
               "note": ("layer = " + (" + ".join(layer_kernels) if layer_kernels else "every profiled kernel")
                        + " per step (every launch of the step summed); FETCH_SIZE x2 (gfx950 wide-read "
                        "correction), KiB -> bytes; scripts/r03_pmc.sh")}
    json.dump(tj, open(path, "w"), indent=1)
    print(key, f"{layer / 1e9:.4f} GB per step", {k: round((v['fetch_bytes_per_step'] + v['write_bytes_per_step']) / 1e6, 2)
                                                   for k, v in out.items()})


if __name__ == "__main__":
    key = sys.argv[1] if len(sys.argv) > 1 else "config2_F64"
    if key == "step":  # traffic.py step KEY TAG [all] [ANCHOR]: per-step bytes of a bench workload's PMC passes
        every = len(sys.argv) > 4 and sys.argv[4] == "all"
        step_traffic(sys.argv[2], sys.argv[3], None if every else LAYER, sys.argv[5] if len(sys.argv) > 5 else "k_count")
        sys.exit(0)
    if key.startswith("conv_c6_"):  # conv_c6_<dt>_F64: the RetinaNet conv (gpu_conv_prof.sh CFG=6)
        conv(key, key.split("_")[2], "c6_" + key.split("_")[2])
    elif key.startswith("conv_"):
        conv(key, key.split("_")[1])
    else:
        main(key)
