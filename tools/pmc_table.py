"""Per-kernel mean of every counter in rocprofv3 --pmc CSVs (one or more passes).
Usage: python tools/pmc_table.py a.csv [b.csv ...]"""
import csv
import sys
from collections import defaultdict

sys.path.insert(0, __file__.rsplit("/", 1)[0])
from pmc_summary import short  # noqa: E402


def main():
    vals = defaultdict(lambda: defaultdict(list))
    for path in sys.argv[1:]:
        for r in csv.DictReader(open(path)):
            k = short(r["Kernel_Name"])
            vals[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
            vals[k]["_dur_us"].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    for k, cs in vals.items():
        print(k)
        for c in sorted(cs):
            v = cs[c]
            print(f"   {c:28s} {sum(v) / len(v):16.1f}  (n={len(v)})")


if __name__ == "__main__":
    main()
