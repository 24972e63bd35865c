"""Per-(kernel, grid size) launch statistics of a rocprofv3 kernel-trace CSV (dev tool): separates
a kernel's training-size launches from its collect-size ones, whose rocprof --stats average mixes
them.  Usage: python tools/trace_by_grid.py kernel_trace.csv out.csv"""
import csv
import sys
from collections import defaultdict


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    agg = defaultdict(list)
    for r in rows:
        grid = int(r.get("Grid_Size_X") or r.get("Grid_Size") or 0) * int(r.get("Grid_Size_Y") or 1) * \
            int(r.get("Grid_Size_Z") or 1)
        wg = int(r.get("Workgroup_Size_X") or r.get("Workgroup_Size") or 1) * int(r.get("Workgroup_Size_Y") or 1) * \
            int(r.get("Workgroup_Size_Z") or 1)
        agg[(r["Kernel_Name"], grid // max(wg, 1))].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    out = sorted(((sum(v), k, v) for k, v in agg.items()), reverse=True)
    with open(sys.argv[2], "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["Name", "Workgroups", "Calls", "TotalDurationNs", "AverageNs", "MinNs", "MaxNs"])
        for tot, (name, wgs), v in out:
            w.writerow([name, wgs, len(v), tot, round(tot / len(v), 1), min(v), max(v)])
    for tot, (name, wgs), v in out[:12]:
        print(f"{name[:90]:90s} wgs={wgs:7d} n={len(v):4d} avg={tot / len(v) / 1e3:8.1f} us")


if __name__ == "__main__":
    main()
