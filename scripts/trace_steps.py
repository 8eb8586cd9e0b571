"""Print replayed steps' kernel timelines from a rocprofv3 kernel-trace CSV.

    python scripts/trace_steps.py gpurun_out/prof_c3/run_kernel_trace.csv [anchor] [first] [count]
A step starts at a launch of the anchor kernel (default k_count); prints
`count` steps from step index `first` (the bench's graph replays come after
its warmup steps)."""
import csv
import re
import sys


def short(name):
    name = name.replace("shpl::(anonymous namespace)::", "")
    m = re.match(r"(?:void )?([A-Za-z_0-9:]+(?:<[^()]*>)?)", name)
    return (m.group(1) if m else name)[:64]


def main():
    path = sys.argv[1]
    anchor = sys.argv[2] if len(sys.argv) > 2 else "k_count"
    first = int(sys.argv[3]) if len(sys.argv) > 3 else 8
    count = int(sys.argv[4]) if len(sys.argv) > 4 else 1
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    idx = [i for i, r in enumerate(rows) if anchor in r["Kernel_Name"]]
    for k in range(first, min(first + count, len(idx) - 1)):
        s, e = idx[k], idx[k + 1]
        t0 = int(rows[s]["Start_Timestamp"])
        for r in rows[s:e]:
            st, en = int(r["Start_Timestamp"]) - t0, int(r["End_Timestamp"]) - t0
            print(f"{st / 1e3:8.1f} {en / 1e3:8.1f} {(en - st) / 1e3:7.1f} us  q{r.get('Queue_Id', '?'):>2}  "
                  f"{short(r['Kernel_Name'])}")
        print(f"--- next step at {(int(rows[e]['Start_Timestamp']) - t0) / 1e3:.1f} us")


if __name__ == "__main__":
    main()
