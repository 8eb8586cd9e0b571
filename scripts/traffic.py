"""Per-launch HBM traffic of the SHPL kernels from the rocprofv3 PMC passes
(scripts/gpu_round.sh step `pmc`) -> profiles/traffic.json.

gfx950 corrections (MI355X_MICROARCH.md §HBM): FETCH_SIZE and WRITE_SIZE are
in KiB; FETCH_SIZE counts half the bytes of a wide (16 B/lane) coalesced
read, so it is doubled; WRITE_SIZE is exact for 16 B/lane stores."""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def per_kernel(counter):
    files = glob.glob(os.path.join(ROOT, "gpurun_out", f"pmc_{counter}", "**", "*counter_collection.csv"),
                      recursive=True)
    acc = defaultdict(list)
    for f in files:
        for r in csv.DictReader(open(f)):
            if r.get("Counter_Name") != counter:
                continue
            name = r["Kernel_Name"]
            short = next((k for k in ("k_dense", "k_sparse", "k_csr_frame", "k_compact", "k_count") if k in name), name)
            acc[short].append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in acc.items()}


def main(key):
    fetch = per_kernel("FETCH_SIZE")
    write = per_kernel("WRITE_SIZE")
    out = {}
    for k in sorted(set(fetch) | set(write)):
        f_b = 2 * fetch.get(k, 0.0) * 1024
        w_b = write.get(k, 0.0) * 1024
        out[k] = {"fetch_bytes": f_b, "write_bytes": w_b, "raw_FETCH_SIZE_KiB": fetch.get(k),
                  "raw_WRITE_SIZE_KiB": write.get(k)}
    layer = sum(out[k]["fetch_bytes"] + out[k]["write_bytes"] for k in ("k_dense", "k_sparse") if k in out)
    path = os.path.join(ROOT, "profiles", "traffic.json")
    tj = json.load(open(path)) if os.path.exists(path) else {}
    tj[key] = {"hbm_bytes_per_launch": layer, "kernels": out,
               "note": "layer = k_dense + k_sparse; FETCH_SIZE x2 (gfx950 wide-read correction), KiB -> bytes"}
    json.dump(tj, open(path, "w"), indent=1)
    print(json.dumps(tj[key], indent=1))


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "config2_F64")
