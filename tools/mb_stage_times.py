"""Per-stage average durations of the MBConv kernels in a rocprofv3 trace of tools/bench_mbconv.py
(4 stages x reps launches per kernel, stage loop outermost; the first rep of each stage dropped).

    python tools/mb_stage_times.py DIR/mb_kernel_trace.csv
"""
import collections
import csv
import sys

KEYS = ("dw_fwd", "dw_dgrad", "dw_wgrad", "se_bwd_reduce", "se_pool", "se_mlp_fwd", "se_mlp_bwd", "wgrad_f32", "bn2_apply",
        "bn_bwd_apply", "sgemm", "gemm_bf16")


def main(path):
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    seq = collections.defaultdict(list)
    for r in rows:
        for k in KEYS:
            if k in r["Kernel_Name"]:
                seq[k].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000)
                break
    for k in KEYS:
        v = seq.get(k)
        if not v or len(v) % 4:
            continue
        per = len(v) // 4
        print(f"{k:14s}", [round(sum(v[i * per + 1:(i + 1) * per]) / max(1, per - 1), 1) for i in range(4)], f"x{per}")


if __name__ == "__main__":
    main(sys.argv[1])
