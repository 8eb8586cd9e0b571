"""Print one step's kernel timeline from a rocprofv3 kernel-trace CSV.

    python scripts/trace_step.py gpurun_out/prof_c3/run_kernel_trace.csv [anchor-substring] [n]
The step is taken to start at the second-to-last launch of the anchor kernel
(default k_compact)."""
import csv
import re
import sys


def short(name):
    name = name.replace("shpl::(anonymous namespace)::", "")
    m = re.match(r"(?:void )?([A-Za-z_0-9:]+(?:<[^()]*>)?)", name)
    return (m.group(1) if m else name)[:70]


def main():
    path = sys.argv[1]
    anchor = sys.argv[2] if len(sys.argv) > 2 else "k_compact"
    n = int(sys.argv[3]) if len(sys.argv) > 3 else 24
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    idx = [i for i, r in enumerate(rows) if anchor in r["Kernel_Name"]]
    s = idx[-2] if len(idx) > 1 else idx[-1]
    t0 = int(rows[s]["Start_Timestamp"])
    for r in rows[s:s + n]:
        st, en = int(r["Start_Timestamp"]) - t0, int(r["End_Timestamp"]) - t0
        print(f"{st / 1e3:9.1f} {en / 1e3:9.1f} {(en - st) / 1e3:8.1f} us  q{r.get('Queue_Id', '?')}  "
              f"{short(r['Kernel_Name'])}")


if __name__ == "__main__":
    main()
