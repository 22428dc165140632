"""Group a rocprofv3 kernel trace by (kernel, grid size): count, average and total duration.

    python tools/kernels_by_grid.py trace.csv[.gz] [--match REGEX] [--top N]
"""
import argparse
import collections
import csv
import gzip
import re


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--match", default=None)
    ap.add_argument("--top", type=int, default=60)
    a = ap.parse_args()
    op = gzip.open if a.trace.endswith(".gz") else open
    agg = collections.defaultdict(lambda: [0, 0.0])
    with op(a.trace, "rt") as f:
        for r in csv.DictReader(f):
            name = r["Kernel_Name"]
            if a.match and not re.search(a.match, name):
                continue
            key = (name[:90], int(r["Grid_Size_X"]) * int(r["Grid_Size_Y"]) * int(r["Grid_Size_Z"]))
            agg[key][0] += 1
            agg[key][1] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    rows = sorted(agg.items(), key=lambda kv: -kv[1][1])[: a.top]
    for (name, grid), (n, tot) in rows:
        print(f"{tot / n:9.1f} us  n={n:4d}  grid={grid:9d}  {name}")


if __name__ == "__main__":
    main()
