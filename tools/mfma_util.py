"""Per-family MFMA utilisation from a rocprofv3 --pmc counter_collection.csv holding
SQ_VALU_MFMA_BUSY_CYCLES, SQ_BUSY_CYCLES and GRBM_GUI_ACTIVE (tools/gpu_mfma_util.sh).

util = sum(SQ_VALU_MFMA_BUSY_CYCLES) / (GRBM_GUI_ACTIVE / 8 XCDs * 1024 SIMDs): the fraction of
the chip's MFMA pipe-cycles busy while the family's dispatches ran (GRBM_GUI_ACTIVE is summed
over the 8 XCDs, MI355X_MICROARCH.md)."""
import collections
import csv
import re
import sys


def family(name):
    n = re.sub(r"^void ", "", name)
    n = re.sub(r"\(.*", "", n)
    n = re.sub(r"<.*", "", n)
    return n[:60]


def main(path):
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    for r in csv.DictReader(open(path)):
        key = (r["Dispatch_Id"], r["Kernel_Name"])
        per[key][r["Counter_Name"]] += float(r["Counter_Value"])
    fam = collections.defaultdict(lambda: collections.defaultdict(float))
    for (_, k), d in per.items():
        f = family(k)
        for c, v in d.items():
            fam[f][c] += v
        fam[f]["n"] += 1
    rows = []
    for f, d in fam.items():
        gui = d.get("GRBM_GUI_ACTIVE", 0.0)
        if gui <= 0:
            continue
        util = d.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0) / (gui / 8 * 1024)
        rows.append((gui, f, int(d["n"]), util))
    rows.sort(reverse=True)
    tot = sum(r[0] for r in rows)
    print(f"{'family':60s} {'launches':>8s} {'time%':>6s} {'MFMA util':>9s}")
    for gui, f, n, u in rows[:25]:
        print(f"{f:60s} {n:8d} {100 * gui / tot:6.1f} {u:9.3f}")


if __name__ == "__main__":
    main(sys.argv[1])
