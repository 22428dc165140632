"""Per-shape GEMM census of one train step: our kernels vs hipBLASLt (torch bf16 matmul).

Reads the OGV_LOG_GEMM=1 stderr log of an eager bench step, groups the bf16 launches by
(kind, M, N, K), and times each shape through the C ABI (plain variant: no prologue, no
epilogue extras) and as a torch bf16 matmul, caches flushed before every launch.

    OGV_LOG_GEMM=1 python bench.py --eager --steps 1 --warmup 0 ... 2> shapes.log
    python tools/gemm_shapes.py shapes.log [--reps 5] [--div STEPS]
"""
import argparse
import collections
import os
import re
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "outlook-grid-vision-transformer_amd"))

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("log")
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--div", type=float, default=1, help="steps in the log (counts are divided by it)")
    ap.add_argument("--opt", action="append", default=[], help="ogv_set_option name=value (repeatable)")
    ap.add_argument("--kinds", default="fwd,dgrad,wgrad")
    ap.add_argument("--max-m", type=int, default=1 << 30)
    a = ap.parse_args()
    cnt = collections.Counter()
    for ln in open(a.log):
        m = re.match(r"OGVGEMM (\w+) dt=(\d) M=(\d+) N=(\d+) K=(\d+)(.*)", ln)
        if not m or m.group(2) != "1":  # bf16 only
            continue
        cnt[(m.group(1), int(m.group(3)), int(m.group(4)), int(m.group(5)))] += 1
    import ogv
    from ogv._lib import load
    ogv.load()
    lib = load()
    for o in a.opt:
        k, v = o.split("=")
        assert lib.ogv_set_option(k.encode(), int(v)) == 0, o
    dev, bf = "cuda", torch.bfloat16
    flush = torch.ones(128 << 20, dtype=torch.float32, device=dev)
    st = torch.cuda.current_stream().cuda_stream
    ws = torch.empty(256 << 20, dtype=torch.uint8, device=dev)

    def timeit(fn):
        ts = []
        for _ in range(a.reps + 1):
            flush.sum()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            fn()
            e1.record()
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1))
        return statistics.median(ts[1:]) * 1e3

    rows = []
    for (kind, M, N, K), n in sorted(cnt.items(), key=lambda kv: -kv[0][1] * kv[0][2] * kv[0][3] * kv[1]):
        n = n / a.div
        if kind not in a.kinds.split(",") or M > a.max_m:
            continue
        if kind == "fwd":  # out[M,N] = A[M,K] W[N,K]^T
            A = torch.randn(M, K, device=dev).to(bf)
            W = torch.randn(N, K, device=dev) * 0.05
            out = torch.empty(M, N, device=dev, dtype=bf)
            Wb = W.to(bf)

            def ours():
                assert lib.ogv_gemm_fwd(A.data_ptr(), K, W.data_ptr(), None, None, None, 0, out.data_ptr(), N,
                                        M, N, K, 0, 1, st) == 0

            def ref():
                torch.matmul(A, Wb.t())
        elif kind == "dgrad":  # dA[M,K] = dout[M,N] W[N,K]
            D = torch.randn(M, N, device=dev).to(bf)
            W = torch.randn(N, K, device=dev) * 0.05
            dA = torch.empty(M, K, device=dev, dtype=bf)
            Wb = W.to(bf)

            def ours():
                assert lib.ogv_gemm_dgrad(D.data_ptr(), N, W.data_ptr(), None, 0, None, 0, dA.data_ptr(), K,
                                          M, N, K, 0, ws.data_ptr(), 1, st) == 0

            def ref():
                torch.matmul(D, Wb)
        else:  # dW[N,K] = G[M,N]^T X[M,K]
            G = torch.randn(M, N, device=dev).to(bf)
            X = torch.randn(M, K, device=dev).to(bf)
            dW = torch.empty(N, K, device=dev)
            db = torch.empty(N, device=dev)
            if lib.ogv_gemm_wgrad_ws_bytes(M, N, K) > ws.numel():
                continue

            def ours():
                assert lib.ogv_gemm_wgrad(G.data_ptr(), N, X.data_ptr(), K, None, 0, dW.data_ptr(), db.data_ptr(),
                                          M, N, K, 0, ws.data_ptr(), 1, st) == 0

            def ref():
                torch.matmul(G.t(), X)
        t_o, t_r = timeit(ours), timeit(ref)
        rows.append((kind, M, N, K, n, t_o, t_r))
        print(f"{kind:5s} M={M:7d} N={N:5d} K={K:5d} x{n:5.1f}  ours {t_o:8.1f} us  hipBLASLt {t_r:8.1f} us  "
              f"ratio {t_o / t_r:5.2f}  step-cost {t_o * n:8.1f} us  loss {max(0.0, t_o - t_r) * n:7.1f} us",
              flush=True)
    tot_o = sum(r[4] * r[5] for r in rows)
    tot_b = sum(r[4] * min(r[5], r[6]) for r in rows)
    print(f"total ours {tot_o:.0f} us / step; with the faster of the two per shape {tot_b:.0f} us")


if __name__ == "__main__":
    main()
