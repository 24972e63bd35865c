"""Per-kernel SQ/GRBM counter table from tools/kernel_pmc.sh passes (dev tool): the mean per dispatch of every
counter, grouped by kernel (and grid size), plus the derived fractions that say what bounds a kernel:
  mfma_busy = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 x 1024 SIMDs)   (the matrix cores' duty cycle:
              MFMA_BUSY counts cycles, 32 per 32x32x16 f16 MFMA; GRBM_GUI_ACTIVE is summed over the 8 XCDs)
  valu/mfma = SQ_INSTS_VALU / SQ_INSTS_MFMA, lds_conf = SQ_LDS_BANK_CONFLICT / SQ_ACTIVE_INST_LDS,
  wait_any  = SQ_WAIT_ANY / SQ_WAVE_CYCLES  (share of wave time waiting on anything)
Usage: python tools/pmc_table.py pass1.csv [pass2.csv ...]"""
import csv
import sys
from collections import defaultdict

SIMDS = 1024


def short(name):
    return name.replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0][:70]


def main():
    acc = defaultdict(lambda: defaultdict(list))
    for f in sys.argv[1:]:
        for r in csv.DictReader(open(f)):
            key = (short(r["Kernel_Name"]), int(r["Grid_Size"]))
            acc[key][r["Counter_Name"]].append(float(r["Counter_Value"]))
    # one line per kernel: the grid size with the most dispatches (the training launches)
    best = {}
    for (k, g), c in acc.items():
        n = max(len(v) for v in c.values())
        if k not in best or n > best[k][1]:
            best[k] = (g, n)
    cols = ["mfma_busy", "valu/mfma", "lds_conf", "wait_any", "wait_lds", "SQ_INSTS_MFMA", "SQ_INSTS_VALU",
            "SQ_INSTS_LDS"]
    print(f"{'kernel':70s} {'grid':>9s} " + " ".join(f"{c:>13s}" for c in cols))
    for k, (g, _) in sorted(best.items()):
        c = {n: sum(v) / len(v) for n, v in acc[(k, g)].items()}
        get = lambda n: c.get(n, float("nan"))
        row = {
            "mfma_busy": get("SQ_VALU_MFMA_BUSY_CYCLES") / (get("GRBM_GUI_ACTIVE") / 8 * SIMDS),
            "valu/mfma": get("SQ_INSTS_VALU") / get("SQ_INSTS_MFMA") if get("SQ_INSTS_MFMA") else float("nan"),
            "lds_conf": get("SQ_LDS_BANK_CONFLICT") / get("SQ_ACTIVE_INST_LDS") if get("SQ_ACTIVE_INST_LDS") else float("nan"),
            "wait_any": get("SQ_WAIT_ANY") / get("SQ_WAVE_CYCLES"),
            "wait_lds": get("SQ_WAIT_INST_LDS") / get("SQ_WAVE_CYCLES"),
            "SQ_INSTS_MFMA": get("SQ_INSTS_MFMA"), "SQ_INSTS_VALU": get("SQ_INSTS_VALU"),
            "SQ_INSTS_LDS": get("SQ_INSTS_LDS"),
        }
        print(f"{k:70s} {g:9d} " + " ".join(f"{row[c]:13.4g}" for c in cols))


if __name__ == "__main__":
    main()
