"""Derive per-launch HBM bytes from rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes.
gfx950 correction (MI355X_MICROARCH.md, HBM/rocprofv3): FETCH_SIZE counts 1/2 of the
streamed read bytes, so bytes = (2*FETCH_SIZE + WRITE_SIZE) * 1024 (counters are KB).
Usage: python tools/pmc_summary.py FETCH.csv WRITE.csv OUT.json"""
import csv
import json
import re
import sys
from collections import defaultdict


def short(name):
    n = name.replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0]
    return re.sub(r"Geo<([^>]*)>", r"\1", n).replace(" >", ">")


def load(path, counter):
    """per kernel: the counter values of its launches with the largest grid (the training
    minibatch's; the forward kernels also run at the collect batch in the same command)"""
    vals = defaultdict(lambda: defaultdict(list))
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] == counter:
            vals[short(r["Kernel_Name"])][int(r["Grid_Size"])].append(float(r["Counter_Value"]))
    return {k: v[max(v)] for k, v in vals.items()}


def main():
    fetch, write, out = sys.argv[1:4]
    f, w = load(fetch, "FETCH_SIZE"), load(write, "WRITE_SIZE")
    res = {}
    for k in sorted(set(f) & set(w)):
        fm, wm = sum(f[k]) / len(f[k]), sum(w[k]) / len(w[k])
        res[k] = {"FETCH_SIZE_KB_mean": fm, "WRITE_SIZE_KB_mean": wm, "launches": len(f[k]),
                  "hbm_bytes_per_launch_corrected": (2 * fm + wm) * 1024,
                  "correction": "MI355X_MICROARCH.md HBM: gfx950 FETCH_SIZE counts 1/2 of streamed read "
                                "bytes -> 2*FETCH + WRITE, x1024 (KB)"}
    json.dump(res, open(out, "w"), indent=1)
    for k, v in res.items():
        print(f"{k:60s} {v['launches']:5d} {v['hbm_bytes_per_launch_corrected'] / 1e6:10.1f} MB/launch")


if __name__ == "__main__":
    main()
