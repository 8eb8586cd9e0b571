"""Write profiles/frame_checksums.json's oracle-pinned tables from the CPU oracle.

    python tests/golden/make_checksum_tables.py [--jobs 8] [--only KEY ...]

Every frame of every table in tests/checksum_tables.ORACLE_TABLES is computed on the host
(tests/checksum_tables.py: the bench's inputs for that global frame id through oracle/shpl_oracle.c, then the
position-weighted checksum) -- no GPU run writes these tables. Tables the oracle does not pin (the conv
workloads: TF's Conv2D fixes no summation order) are kept as they are and labelled by bench.py."""
import argparse
import json
import multiprocessing as mp
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
OUT = os.path.join(ROOT, "profiles", "frame_checksums.json")


def _one(job):
    import checksum_tables as ct
    key, fid = job
    return key, fid, ct.table_entry(key, fid)


def main():
    import checksum_tables as ct
    ap = argparse.ArgumentParser()
    ap.add_argument("--jobs", type=int, default=min(8, os.cpu_count() or 1))
    ap.add_argument("--only", nargs="*", default=None)
    args = ap.parse_args()
    keys = args.only or list(ct.ORACLE_TABLES)
    jobs = [(k, f) for k in keys for f in range(ct.ORACLE_TABLES[k])]
    tab = {}
    if os.path.exists(OUT):
        with open(OUT) as fh:
            tab = json.load(fh)
    res = {k: [None] * ct.ORACLE_TABLES[k] for k in keys}
    t0 = time.time()
    with mp.get_context("spawn").Pool(args.jobs, maxtasksperchild=8) as pool:
        for n, (key, fid, cs) in enumerate(pool.imap_unordered(_one, jobs), 1):
            res[key][fid] = cs
            if n % 16 == 0 or n == len(jobs):
                print(f"{n}/{len(jobs)} frames, {time.time() - t0:.0f} s", flush=True)
    for k in keys:
        assert len(set(res[k])) == len(res[k]), f"{k}: two frames with one checksum"
        tab[k] = res[k]
    with open(OUT, "w") as fh:
        json.dump(tab, fh, indent=0)
    print("wrote", OUT, {k: len(v) for k, v in tab.items()})


if __name__ == "__main__":
    main()
