"""Per-kernel difference of two rocprofv3 kernel_stats.csv files (dev tool):
python tools/probes/stats_diff.py A.csv B.csv [N=12] — the N largest savings and losses of B against A, per call."""
import csv
import sys


def load(f):
    return {r["Name"]: (float(r["TotalDurationNs"]), int(r["Calls"])) for r in csv.DictReader(open(f))}


def main():
    a, b = load(sys.argv[1]), load(sys.argv[2])
    n = int(sys.argv[3]) if len(sys.argv) > 3 else 12
    print("total A %.1f ms  B %.1f ms" % (sum(v[0] for v in a.values()) / 1e6, sum(v[0] for v in b.values()) / 1e6))
    rows = []
    for k in set(a) | set(b):
        ta, tb = a.get(k, (0.0, 0)), b.get(k, (0.0, 0))
        rows.append((tb[0] - ta[0], k, ta[0] / max(ta[1], 1) / 1e3, tb[0] / max(tb[1], 1) / 1e3, ta[1], tb[1]))
    rows.sort()
    for d, k, x, y, ca, cb in rows[:n] + rows[-n:]:
        name = k.replace("(anonymous namespace)::", "").replace("void ", "")[:90]
        print(f"{d / 1e6:8.2f} ms  A {x:7.1f}us x{ca:5d}  B {y:7.1f}us x{cb:5d}  {name}")


if __name__ == "__main__":
    main()
