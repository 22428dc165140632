"""Outlooker: the fused projection + aggregation kernels vs the unfused pair, per Model-A stage
shape, cold L2 (512 MB flush before each rep), HIP events, median of --reps.
Forward: ogv_outlook_vproj_fwd (fused_eval: writes y; fused_train: also the cat [v | logits | 0]
the aggregation backward would read) vs the concatenated [Wv; Wattn; 0] GEMM -> cat, then the
aggregation reading cat (unfused).  Backward: ogv_outlook_vproj_bwd (fused_bwd: [v | logits]
recomputed from x in LDS, writes dcat) vs the LDS-tiled aggregation backward on cat (unfused_bwd).
Algorithmic bytes: fused_eval 2*M*2C, fused_train 2*M*(2C + ld), unfused 2*M*(C + ld) + 2*M*(2C + 9h),
fused_bwd 2*M*(2C + ld), unfused_bwd 2*M*(C + ld) (dy, cat) + 2*M*ld (dcat).
    python tools/bench_vproj.py [--reps 20]"""
import argparse
import pathlib
import sys

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "outlook-grid-vision-transformer_amd"))
import torch  # noqa: E402

import ogv  # noqa: E402
from ogv import functional as OF  # noqa: E402
from ogv._lib import ACT, OGV_BF16, OgvError, load  # noqa: E402

SHAPES = [("7m_s0", 512, 48, 2, 32), ("7m_s1", 512, 96, 3, 16), ("14m_s0", 256, 64, 2, 64),
          ("22m_s0", 128, 64, 2, 224),
          # wide stages: the weight-streaming fused forward (no recompute backward: fused_bwd skipped)
          ("7m_s2", 512, 192, 6, 8), ("7m_s3", 512, 256, 8, 4), ("14m_s1", 256, 128, 4, 32),
          ("14m_s2", 256, 256, 8, 16), ("14m_s3", 256, 384, 6, 8), ("22m_s1", 128, 128, 4, 112),
          ("22m_s2", 128, 256, 8, 56), ("22m_s3", 128, 384, 6, 28)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--opt", action="append", default=[], metavar="NAME=VALUE")
    ap.add_argument("--shapes", default="", help="comma list of shape names (default all)")
    ap.add_argument("--kinds", default="unfused,fused_train,fused_eval,unfused_bwd,fused_bwd")
    a = ap.parse_args()
    ogv.load()
    lib = load()
    for o in a.opt:
        k, v = o.split("=")
        assert lib.ogv_set_option(k.encode(), int(v)) == 0, o
    s = lambda: OF._stream()  # noqa: E731
    flush = torch.empty(512 << 20, dtype=torch.uint8, device="cuda")
    for name, B, C, h, S in SHAPES:
        if a.shapes and name not in a.shapes.split(","):
            continue
        M = B * S * S
        ld = (C + 9 * h + 7) // 8 * 8
        x = torch.randn(M, C, device="cuda").to(torch.bfloat16)
        w = torch.randn(ld, C, device="cuda") / C ** 0.5
        w[C + 9 * h:] = 0
        b = torch.zeros(ld, device="cuda")
        cat = torch.empty(M, ld, device="cuda", dtype=torch.bfloat16)
        y = torch.empty(M, C, device="cuda", dtype=torch.bfloat16)
        dy = torch.randn(M, C, device="cuda").to(torch.bfloat16)
        dcat = torch.empty(M, ld, device="cuda", dtype=torch.bfloat16)
        OF.check(lib.ogv_gemm_fwd(OF._ptr(x), C, OF._ptr(w), OF._ptr(b), None, None, 1, OF._ptr(cat), ld, M, ld, C,
                                  ACT[None], OGV_BF16, s()), "gemm")   # cat for the unfused backward
        p = OF._ptr
        runs = {
            "unfused": lambda: (OF.check(lib.ogv_gemm_fwd(p(x), C, p(w), p(b), None, None, 1, p(cat), ld, M, ld, C,
                                                          ACT[None], OGV_BF16, s()), "gemm"),
                                OF.check(lib.ogv_outlook_agg_fwd(p(cat), OF._vp(cat.data_ptr() + 2 * C), p(y), B, S,
                                                                 S, C, h, 3, ld, ld, OGV_BF16, s()), "agg")),
            "fused_train": lambda: OF.check(lib.ogv_outlook_vproj_fwd(p(x), C, p(w), p(b), p(cat), ld, p(y), B, S, S, C,
                                                                      h, 3, OGV_BF16, s()), "vproj"),
            "fused_eval": lambda: OF.check(lib.ogv_outlook_vproj_fwd(p(x), C, p(w), p(b), None, ld, p(y), B, S, S, C, h,
                                                                     3, OGV_BF16, s()), "vproj"),
            "unfused_bwd": lambda: OF._outlook_bwd(dy, cat.data_ptr(), ld, cat.data_ptr() + 2 * C, ld, dcat.data_ptr(), ld,
                                                   dcat.data_ptr() + 2 * C, ld, ld - C, B, S, S, C, h, 3),
            "fused_bwd": lambda: OF.check(lib.ogv_outlook_vproj_bwd(p(x), C, p(w), p(b), p(dy), p(dcat), ld, B, S, S, C, h,
                                                                    3, OGV_BF16, s()), "vproj_bwd"),
        }
        nbytes = {"unfused": 2 * M * (C + ld) + 2 * M * (2 * C + 9 * h), "fused_train": 2 * M * (2 * C + ld),
                  "fused_eval": 2 * M * 2 * C, "unfused_bwd": 2 * M * (C + 2 * ld), "fused_bwd": 2 * M * (2 * C + ld)}
        row = [f"{name:7s} M={M:8d}"]
        for kind, fn in runs.items():
            if kind not in a.kinds.split(","):
                continue
            try:
                fn()
            except OgvError:            # a forced plan (vp_tile) this kind cannot take
                row.append(f"{kind} n/a")
                continue
            ts = []
            for _ in range(a.reps):
                flush.zero_()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                fn()
                e1.record()
                ts.append((e0, e1))
            torch.cuda.synchronize()
            ms = sorted(u.elapsed_time(v) for u, v in ts)[len(ts) // 2]
            row.append(f"{kind} {ms * 1e3:8.1f}us {nbytes[kind] / ms / 1e6:6.0f}GB/s")
        print("  ".join(row) + (f"  {a.opt}" if a.opt else ""), flush=True)


if __name__ == "__main__":
    main()
