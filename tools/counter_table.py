"""Per-kernel-family counter table of one deterministic eager bench command, from four rocprofv3 runs of it
(tools/gpu_counters.sh): a kernel trace (durations), FETCH_SIZE, WRITE_SIZE and the MFMA-busy pass.

    python tools/counter_table.py DIR [--out profiles/r04_counters.json]

Per family (kernel name without template arguments): launches of one run, average duration (trace run),
HBM bytes per launch = FETCH_SIZE(KB) * 1024 * 2 (gfx950 reports half of a wide coalesced read,
MI355X_MICROARCH.md) + WRITE_SIZE(KB) * 1024, achieved HBM GB/s = bytes / duration and its fraction of
8 TB/s, and MFMA utilisation = sum SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 XCDs * 1024 SIMDs).
"""
import argparse
import collections
import csv
import glob
import json
import os
import re

HBM = 8000.0


def family(name):
    n = re.sub(r"^void ", "", name)
    n = re.sub(r"\(.*", "", n)
    if n.startswith("_ZN3ogv"):
        m = re.match(r"_ZN3ogv(\d+)", n)
        if m:
            k = int(m.group(1))
            n = "ogv::" + n[len("_ZN3ogv") + len(m.group(1)):][:k]
    return re.sub(r"<.*", "", n)[:60]


def rows_of(d, pattern):
    files = glob.glob(os.path.join(d, "**", pattern), recursive=True)
    if not files:
        raise SystemExit(f"no {pattern} under {d}")
    with open(files[0]) as f:
        return list(csv.DictReader(f))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--out", default=None)
    ap.add_argument("--top", type=int, default=40)
    a = ap.parse_args()
    dur = collections.defaultdict(list)
    for r in rows_of(os.path.join(a.dir, "trace"), "*kernel_trace.csv"):
        dur[family(r["Kernel_Name"])].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-3)
    cnt = collections.defaultdict(lambda: collections.defaultdict(float))
    launches = collections.Counter()
    for sub in ("fetch", "write", "mfma", "stall"):
        if sub == "stall" and not os.path.isdir(os.path.join(a.dir, sub)):
            continue
        seen = set()
        for r in rows_of(os.path.join(a.dir, sub), "*counter_collection.csv"):
            f = family(r["Kernel_Name"])
            cnt[f][r["Counter_Name"]] += float(r["Counter_Value"])
            if sub == "fetch" and r["Counter_Name"] == "FETCH_SIZE":
                key = r["Dispatch_Id"]
                if key not in seen:
                    seen.add(key)
                    launches[f] += 1
    table = []
    for f, ds in dur.items():
        n = launches.get(f, 0)
        c = cnt.get(f, {})
        avg_us = sum(ds) / len(ds)
        row = {"family": f, "launches": len(ds), "avg_us": round(avg_us, 2), "total_ms": round(sum(ds) / 1e3, 3)}
        if n:
            b = (2 * 1024 * c.get("FETCH_SIZE", 0.0) + 1024 * c.get("WRITE_SIZE", 0.0)) / n
            row["hbm_bytes_per_launch"] = int(b)
            row["hbm_GBs"] = round(b / (avg_us * 1e3), 1)
            row["hbm_frac"] = round(b / (avg_us * 1e3) / HBM, 4)
        wc = c.get("SQ_WAVE_CYCLES", 0.0)
        if wc > 0:   # where the waves' cycles went (disjoint: parked on s_waitcnt / barrier, issue-stalled, issuing)
            row["wait_frac"] = round(c.get("SQ_WAIT_ANY", 0.0) / wc, 3)
            row["issue_stall_frac"] = round(c.get("SQ_WAIT_INST_ANY", 0.0) / wc, 3)
            row["active_frac"] = round(c.get("SQ_ACTIVE_INST_ANY", 0.0) / wc, 3)
        if c.get("SQ_LDS_IDX_ACTIVE", 0.0) > 0:
            row["lds_conflict_frac"] = round(c.get("SQ_LDS_BANK_CONFLICT", 0.0) / c["SQ_LDS_IDX_ACTIVE"], 3)
        gui = c.get("GRBM_GUI_ACTIVE", 0.0)
        if gui > 0:
            row["mfma_util"] = round(c.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0) / (gui / 8 * 1024), 4)
        table.append(row)
    table.sort(key=lambda r: -r["total_ms"])
    print(f"{'family':52s} {'n':>5s} {'avg us':>8s} {'total ms':>9s} {'MB/launch':>10s} {'GB/s':>7s} {'frac':>6s} {'MFMA':>6s}"
          f" {'wait':>5s} {'stall':>5s} {'issue':>5s} {'ldsCF':>5s}")
    for r in table[: a.top]:
        print(f"{r['family']:52s} {r['launches']:5d} {r['avg_us']:8.1f} {r['total_ms']:9.3f} "
              f"{r.get('hbm_bytes_per_launch', 0) / 1e6:10.2f} {r.get('hbm_GBs', 0):7.0f} {r.get('hbm_frac', 0):6.3f} "
              f"{r.get('mfma_util', 0):6.3f} {r.get('wait_frac', 0):5.2f} {r.get('issue_stall_frac', 0):5.2f} "
              f"{r.get('active_frac', 0):5.2f} {r.get('lds_conflict_frac', 0):5.2f}")
    if a.out:
        with open(a.out, "w") as fo:
            json.dump(table, fo, indent=1)


if __name__ == "__main__":
    main()
