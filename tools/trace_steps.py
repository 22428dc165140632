"""Per-step kernel breakdown from a rocprofv3 kernel_trace.csv of bench.py.

Steps are delimited by the optimizer's fused AdamW kernel (last kernel of a step).  Prints the
kernel-time table of the LAST step (steady state), grouped by kernel name, plus step wall span.
    python tools/trace_steps.py gpurun_out/prof/bench_kernel_trace.csv [--top 40] [--step -1]
"""
import argparse
import collections
import csv
import re


def short(name):
    name = re.sub(r"\(.*", "", name)
    name = name.replace("void ", "")
    return name[:100]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--top", type=int, default=40)
    ap.add_argument("--step", type=int, default=-1)
    ap.add_argument("--marker", default="adam")
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.trace)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    ends = [i for i, r in enumerate(rows) if a.marker.lower() in r["Kernel_Name"].lower()]
    # a fused AdamW step is several launches close together (one per param group / chunk):
    # keep the last launch of each cluster
    marks = [i for j, i in enumerate(ends) if j + 1 == len(ends) or ends[j + 1] > i + 32]
    if len(marks) < 2:
        print("fewer than 2 step markers found"); return
    k = a.step if a.step >= 0 else len(marks) + a.step
    lo, hi = marks[k - 1] + 1, marks[k] + 1
    # a negative --step counts replayed steps only: skip the eager probe / census steps bench.py runs after
    # the timed region (their launches are queued behind gpu_sleep_kernel spins)
    while a.step < 0 and k > 1 and any("gpu_sleep" in r["Kernel_Name"] for r in rows[lo:hi]):
        k -= 1
        lo, hi = marks[k - 1] + 1, marks[k] + 1
    step = rows[lo:hi]
    t0, t1 = int(step[0]["Start_Timestamp"]), int(step[-1]["End_Timestamp"])
    agg = collections.defaultdict(lambda: [0, 0])
    busy = 0
    for r in step:
        d = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        busy += d
        agg[short(r["Kernel_Name"])][0] += d
        agg[short(r["Kernel_Name"])][1] += 1
    print(f"step {k}: {len(step)} kernels, wall span {(t1 - t0) / 1e6:.2f} ms, kernel busy {busy / 1e6:.2f} ms "
          f"({len(marks)} steps found)")
    for name, (d, n) in sorted(agg.items(), key=lambda kv: -kv[1][0])[: a.top]:
        print(f"{d / 1e6:8.3f} ms {100 * d / busy:5.1f}%  n={n:4d} avg={d / n / 1e3:8.1f}us  {name}")


if __name__ == "__main__":
    main()
