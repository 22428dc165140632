"""Per-kernel microbenchmark of the hot-path kernels at Model-A-7M bs=512 shapes (MI355X).

For every 1x1-projection GEMM of an OutGridBlock at each stage (fwd, dgrad, wgrad) and for the
outlook / grid / LN kernels: average time over N launches (HIP events on torch's stream),
algorithmic HBM bytes, achieved GB/s and fraction of the 8 TB/s peak.

    python tools/bench_kernels.py [--batch 512] [--reps 20] [--json out.json]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "outlook-grid-vision-transformer_amd"))

import torch  # noqa: E402

PEAK = 8000.0
STAGES = [(48, 32, 2, 8), (96, 16, 3, 8), (192, 8, 6, 4), (256, 4, 8, 2)]  # C, H, heads, g


def timeit(fn, reps):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3  # us


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=512)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--json", default=None)
    a = ap.parse_args()
    import ogv
    from ogv import functional as OF
    from ogv._lib import ACT, load
    ogv.load()
    lib = load()
    dev = "cuda"
    bf = torch.bfloat16
    rows = []

    def rec(kind, name, M, N, K, us, nbytes, flops):
        gbs = nbytes / (us * 1e-6) / 1e9
        rows.append(dict(kind=kind, name=name, M=M, N=N, K=K, us=round(us, 2), GBs=round(gbs, 1),
                         frac=round(gbs / PEAK, 3), TFLOPs=round(flops / (us * 1e-6) / 1e12, 2)))
        print(f"{kind:8s} {name:26s} M={M:7d} N={N:5d} K={K:5d} {us:8.1f} us {gbs:8.1f} GB/s ({gbs / PEAK:5.1%})"
              f" {flops / (us * 1e-6) / 1e12:6.1f} TF/s", flush=True)

    for (C, H, h, g) in STAGES:
        M = a.batch * H * H
        gemms = [("outlook.attn", C, 9 * h, None), ("outlook.v", C, C, None), ("outlook.proj", C, C, None),
                 ("mlp2d.fc1", C, 2 * C, None), ("mlp2d.fc2(gelu)", 2 * C, C, "gelu"),
                 ("mbconv.expand", C, 4 * C, None), ("mbconv.project", 4 * C, C, None),
                 ("grid.qkv", C, 3 * C, None), ("grid.proj", C, C, None),
                 ("mlp.fc1", C, 4 * C, None), ("mlp.fc2(gelu)", 4 * C, C, "gelu")]
        for name, K, N, act in gemms:
            x = torch.randn(M, K, device=dev, dtype=bf)
            w = torch.randn(N, K, device=dev) / K ** 0.5
            b = torch.zeros(N, device=dev)
            out = torch.empty(M, N, device=dev, dtype=bf)
            st = torch.cuda.current_stream().cuda_stream
            p = lambda t: t.data_ptr()
            us = timeit(lambda: lib.ogv_gemm_fwd(p(x), K, p(w), p(b), None, None, 1, p(out), N, M, N, K, ACT[act], 1,
                                                 st), a.reps)
            rec("fwd", f"s{C}.{name}", M, N, K, us, 2 * M * (K + N) + 4 * N * K, 2 * M * N * K)
            dout = torch.randn(M, N, device=dev, dtype=bf)
            dx = torch.empty(M, K, device=dev, dtype=bf)
            ws = torch.empty(max(lib.ogv_gemm_dgrad_ws_bytes(N, K), lib.ogv_gemm_wgrad_ws_bytes(M, N, K)),
                             dtype=torch.uint8, device=dev)
            us = timeit(lambda: lib.ogv_gemm_dgrad(p(dout), N, p(w), p(x) if act else None, K, None, 1, p(dx), K, M, N, K,
                                                   ACT[act], p(ws), 1, st), a.reps)
            rec("dgrad", f"s{C}.{name}", M, N, K, us, 2 * M * (K + N) + (2 * M * K if act else 0), 2 * M * N * K)
            dw = torch.empty(N, K, device=dev)
            db = torch.empty(N, device=dev)
            us = timeit(lambda: lib.ogv_gemm_wgrad(p(dout), N, p(x), K, None, 1, p(dw), p(db), M, N, K, ACT[act], p(ws),
                                                   1, st), a.reps)
            rec("wgrad", f"s{C}.{name}", M, N, K, us, 2 * M * (K + N), 2 * M * N * K)
            del x, out, dout, dx, ws
        # outlook aggregation
        v = torch.randn(M, C, device=dev, dtype=bf)
        lg = torch.randn(M, 9 * h, device=dev, dtype=bf)
        y = torch.empty_like(v)
        st = torch.cuda.current_stream().cuda_stream
        us = timeit(lambda: lib.ogv_outlook_agg_fwd(v.data_ptr(), lg.data_ptr(), y.data_ptr(), a.batch, H, H, C, h, 3,
                                                     9 * h, C, 1, st), a.reps)   # ld_logits, ld_v, dtype
        rec("outlook", f"s{C}.fwd", M, C, 9 * h, us, 2 * M * (2 * C + 9 * h), 18 * M * C)
        # grid attention
        qkv = torch.randn(M, 3 * C, device=dev, dtype=bf)
        o = torch.empty(M, C, device=dev, dtype=bf)
        lse = torch.empty(M, h, device=dev)
        us = timeit(lambda: lib.ogv_grid_attn_fwd(qkv.data_ptr(), o.data_ptr(), lse.data_ptr(), None, a.batch, H, H, C,
                                                   h, g, (C // h) ** -0.5, 1, st), a.reps)
        N_tok = (H // g) ** 2
        rec("grid", f"s{C}.fwd N={N_tok}", M, C, N_tok, us, 2 * M * 4 * C + 4 * M * h, 4 * M * N_tok * C)
        # layernorm
        xn = torch.empty_like(v)
        mu = torch.empty(M, device=dev)
        rs = torch.empty(M, device=dev)
        gam = torch.ones(C, device=dev)
        us = timeit(lambda: lib.ogv_layernorm_fwd(v.data_ptr(), gam.data_ptr(), gam.data_ptr(), xn.data_ptr(),
                                                   mu.data_ptr(), rs.data_ptr(), M, C, 1e-5, 1, st), a.reps)
        rec("ln", f"s{C}.fwd", M, C, 0, us, 2 * M * 2 * C + 8 * M, 8 * M * C)
        del v, lg, y, qkv, o
        torch.cuda.empty_cache()
    if a.json:
        with open(a.json, "w") as f:
            json.dump(rows, f, indent=1)


if __name__ == "__main__":
    main()
