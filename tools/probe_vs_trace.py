"""Cross-check bench.py's live roofline probe against the rocprofv3 kernel trace of the same run.

The probed launches are the ones queued right behind an ogv gpu_sleep_kernel (bench.py's eager
probe step); their rocprof durations are averaged and compared with the probe's `avg_launch_ms`
(HIP events).  Also prints the average over every launch of the probed kernel family in the
graph-replayed steps.

    python tools/probe_vs_trace.py bench_kernel_trace.csv bench_stdout.log [unprofiled_bench.log]

Under rocprofv3 the HIP-event intervals themselves are inflated by the tracer (its completion
handling sits between the events), so the like-for-like check is the probe of an UNPROFILED bench
run on the same box (third argument) against the rocprof durations of the probed launches.
"""
import csv
import json
import re
import sys


def main(trace, log, clean_log=None):
    rows = list(csv.DictReader(open(trace)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    line = [ln for ln in open(log) if ln.startswith("{")][-1]
    rec = json.loads(line)
    roof = rec.get("roofline") or {}
    fams = {"sgemm": "sgemm_bf16_kernel", "gemm_tiled": "::gemm_bf16_kernel", "gemm_panel": "pgemm_bf16_kernel", "outlook_bwd": "outlook_bwd",
            "outlook_fwd": "outlook_fwd", "grid_fwd": "grid_fwd",
            "wgrad": r"wgrad2_bf16_kernel|(?<![s2])wgrad_bf16_kernel|swgrad_bf16_kernel"}   # regexes
    fam = fams.get(roof.get("probe", "sgemm" if "sgemm" in roof.get("kernel", "") else ""))
    if fam is None:
        print("probe family has no single-kernel trace match; nothing to compare")
        return
    probed, allk = [], []
    for i, r in enumerate(rows):
        if not re.search(fam, r["Kernel_Name"]):
            continue
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6  # ms
        # same queue, the previous launch on it is the sleep kernel
        prev = next((rows[j] for j in range(i - 1, max(-1, i - 40), -1) if rows[j]["Queue_Id"] == r["Queue_Id"]), None)
        if prev is not None and "gpu_sleep_kernel" in prev["Kernel_Name"]:
            probed.append(d)
        else:
            allk.append(d)
    if not probed:
        print("no probed launches found in the trace")
        return
    avg_p = sum(probed) / len(probed)
    print(f"probe (HIP events): n={roof.get('launches')} avg={roof.get('avg_launch_ms'):.5f} ms "
          f"achieved={roof.get('achieved')} GB/s")
    print(f"rocprof, same launches (behind the sleep kernel): n={len(probed)} avg={avg_p:.5f} ms "
          f"-> ratio events/rocprof = {roof.get('avg_launch_ms') / avg_p:.3f}")
    if allk:
        print(f"rocprof, every other {fam} launch (graph replays + MBConv-internal): n={len(allk)} "
              f"avg={sum(allk) / len(allk):.5f} ms")
    if clean_log:
        rc = json.loads([ln for ln in open(clean_log) if ln.startswith("{")][-1]).get("roofline") or {}
        if rc.get("avg_launch_ms"):
            print(f"probe of the unprofiled bench (HIP events): n={rc.get('launches')} avg={rc['avg_launch_ms']:.5f} ms "
                  f"achieved={rc.get('achieved')} GB/s -> ratio events/rocprof = {rc['avg_launch_ms'] / avg_p:.3f}")
    bpl = roof.get("algorithmic_bytes_per_launch")
    if bpl:
        print(f"algorithmic bytes/launch {bpl} -> rocprof-timed achieved {bpl / (avg_p * 1e-3) / 1e9:.1f} GB/s")


if __name__ == "__main__":
    main(*sys.argv[1:4])
