"""GPU idle gaps of the last iteration(s) in a rocprofv3 --kernel-trace csv (dev tool): the union of
every queue's kernel intervals, each gap above a threshold with the kernels around it, and the total
idle time per kind of boundary.  Usage: python tools/probes/gaps.py kernel_trace.csv [min_gap_us=50] [last_ms=0]"""
import csv
import sys
from collections import defaultdict


def short(name):
    return name.replace("(anonymous namespace)::", "").replace("void ", "")[:70]


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    min_gap = float(sys.argv[2]) * 1e3 if len(sys.argv) > 2 else 50e3
    last = float(sys.argv[3]) * 1e6 if len(sys.argv) > 3 else 0
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    t_end = max(int(r["End_Timestamp"]) for r in rows)
    if last:
        rows = [r for r in rows if int(r["Start_Timestamp"]) >= t_end - last]
    t0 = int(rows[0]["Start_Timestamp"])
    cur_end, prev = None, None
    idle, gaps, kinds = 0, [], defaultdict(float)
    for r in rows:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        if cur_end is not None and s > cur_end:
            g = s - cur_end
            idle += g
            key = (short(prev["Kernel_Name"])[:40], short(r["Kernel_Name"])[:40])
            kinds[key] += g
            if g >= min_gap:
                gaps.append(((cur_end - t0) / 1e3, g / 1e3, short(prev["Kernel_Name"]), short(r["Kernel_Name"])))
        if cur_end is None or e > cur_end:
            cur_end, prev = e, r
    span = cur_end - t0
    print(f"span {span/1e6:.2f} ms, busy {(span-idle)/1e6:.2f} ms, idle {idle/1e6:.2f} ms, kernels {len(rows)}")
    for at, g, a, b in gaps:
        print(f"at {at/1e3:9.2f} ms gap {g:8.1f} us  after {a}  before {b}")
    print("idle by boundary (top 15):")
    for (a, b), g in sorted(kinds.items(), key=lambda kv: -kv[1])[:15]:
        print(f"  {g/1e3:9.1f} us  {a} -> {b}")


if __name__ == "__main__":
    main()
