"""HBM traffic per launch of the roofline kernel from two rocprofv3 PMC passes.

    rocprofv3 --pmc FETCH_SIZE -d DIR/fetch -o run -- python3 bench.py --eager --steps 2 --warmup 1 ...
    rocprofv3 --pmc WRITE_SIZE -d DIR/write -o run -- python3 bench.py --eager --steps 2 --warmup 1 ...
    python tools/pmc_traffic.py DIR/fetch DIR/write --out profiles/pmc_traffic.json

FETCH_SIZE / WRITE_SIZE are kilobytes of L2 memory-side traffic (TCC_EA0 requests).  On gfx950
FETCH_SIZE reports half the bytes of a wide coalesced streaming read (MI355X_MICROARCH.md, HBM
section), so it is doubled; WRITE_SIZE is exact for 16-B-per-lane stores.  Both passes run the
same deterministic command, so the k-th matching dispatch of each pass is the same launch.
"""
import argparse
import csv
import glob
import json
import os
import re

PROBES = {
    "gemm_tiled": r"(?<!s)(?<!p)gemm_bf16_kernel",
    "gemm_panel": r"pgemm_bf16_kernel",
    "outlook_bwd": r"outlook_bwd",
    "sgemm": r"sgemm_bf16_kernel",
    # bench.py's "gemm_fwd" probe: every Linear / 1x1-conv forward GEMM launch (the only users of the
    # plain bf16 GEMM instantiation: no BN statistics, no conv gather, no transposed weights)
    "gemm_fwd": r"gemm_bf16_kernel<(128|64), (128|64), (true|false), false, 0, false>",
    "outlook_fwd": r"outlook_fwd_kernel",
    "grid_fwd": r"grid_fwd_kernel",
    # bench.py's "wgrad" probe (the 14M / 22M dominant family): the weight-gradient kernels themselves
    "wgrad": r"wgrad2_bf16_kernel|(?<![s2])wgrad_bf16_kernel|swgrad_bf16_kernel",
}


def behind_sleep(rows):
    """Indices of launches queued right behind bench.py's probe spin (gpu_sleep_kernel): exactly the
    launches the live probe timed."""
    return {i for i in range(1, len(rows)) if "gpu_sleep_kernel" in rows[i - 1][1]}


def read_counter(d, name):
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not files:
        raise SystemExit(f"no counter_collection.csv under {d}")
    rows = []
    with open(files[0]) as f:
        for r in csv.DictReader(f):
            if r.get("Counter_Name") != name:
                continue
            rows.append((int(r["Dispatch_Id"]), r["Kernel_Name"], float(r["Counter_Value"])))
    rows.sort()
    return rows


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("fetch_dir")
    ap.add_argument("write_dir")
    ap.add_argument("--out", default="profiles/pmc_traffic.json")
    ap.add_argument("--probe", default=None, help="the bench.py --probe of this run: only its entry is (re)written, "
                    "from the launches queued behind the probe's spin; other entries of --out are kept")
    ap.add_argument("--key", default=None, help="entry name in --out (default: the probe name; bench.py reads "
                    "'<model>/bs<B>:<probe>' for workloads other than Model-A-7M bs=512)")
    ap.add_argument("--skip-steps", type=int, default=1, help="leading launches per probe treated as warmup: "
                    "steps to drop (the probe keeps the last step's launches)")
    ap.add_argument("--tag", default="", help="measurement tag stored in the entry (e.g. the round and box run)")
    a = ap.parse_args()
    fetch = read_counter(a.fetch_dir, "FETCH_SIZE")
    write = read_counter(a.write_dir, "WRITE_SIZE")
    out = {}
    if a.probe and os.path.exists(a.out):
        out = json.load(open(a.out))
    fsel, wsel = behind_sleep(fetch), behind_sleep(write)
    for probe, rx in PROBES.items():
        if a.probe and probe != a.probe:
            continue
        if (probe == "sgemm" or a.probe) and fsel:   # the probed launches only (same subset as the live probe)
            f = [v for i, (_, n, v) in enumerate(fetch) if i in fsel and re.search(rx, n)]
            w = [v for i, (_, n, v) in enumerate(write) if i in wsel and re.search(rx, n)]
        else:
            f = [v for _, n, v in fetch if re.search(rx, n)]
            w = [v for _, n, v in write if re.search(rx, n)]
        n = min(len(f), len(w))
        if n == 0:
            continue
        f, w = f[-n:], w[-n:]
        fb = [2 * 1024 * x for x in f]   # KB -> bytes, x2 gfx950 read correction
        wb = [1024 * x for x in w]
        key = a.key or probe
        out[key] = {"launches": n, "kernel_regex": rx,
                      "fetch_bytes_per_launch": sum(fb) / n, "write_bytes_per_launch": sum(wb) / n,
                      "hbm_bytes_per_launch": (sum(fb) + sum(wb)) / n,
                      "correction": "FETCH_SIZE(KB)*1024*2 (gfx950 half-count of wide reads) + WRITE_SIZE(KB)*1024"}
        if a.tag:
            out[key]["measured"] = a.tag
        print(key, json.dumps(out[key]))
    os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
    with open(a.out, "w") as fo:
        json.dump(out, fo, indent=1)


if __name__ == "__main__":
    main()
