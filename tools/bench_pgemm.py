"""Time one bf16 projection GEMM shape through the C ABI (tuning aid for ogv_pgemm.hip).

    python tools/bench_pgemm.py fwd 32768 768 192 [--act gelu] [--opt pgemm=0] [--reps 50] [--cold]

Warm: back-to-back launches between two events (average per launch).  Cold: a 512 MB read before
each launch.  Prints us per launch and algorithmic GB/s (A + W(fp32) + out [+ residual]).
"""
import argparse
import ctypes
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "outlook-grid-vision-transformer_amd"))

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("kind", choices=["fwd", "dgrad"])
    ap.add_argument("M", type=int)
    ap.add_argument("N", type=int)
    ap.add_argument("K", type=int)
    ap.add_argument("--act", default=None, choices=[None, "gelu", "silu"])
    ap.add_argument("--opt", action="append", default=[])
    ap.add_argument("--reps", type=int, default=50)
    ap.add_argument("--cold", action="store_true")
    a = ap.parse_args()
    import ogv
    from ogv._lib import load
    ogv.load()
    lib = load()
    for o in a.opt:
        k, v = o.split("=")
        assert lib.ogv_set_option(k.encode(), int(v)) == 0, o
    dev, bf = "cuda", torch.bfloat16
    M, N, K = a.M, a.N, a.K
    act = {None: 0, "gelu": 1, "silu": 2}[a.act]
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    W = torch.randn(N, K, device=dev) * 0.05
    if a.kind == "fwd":
        A = torch.randn(M, K, device=dev).to(bf)
        out = torch.empty(M, N, device=dev, dtype=bf)
        nbytes = 2 * M * K + 4 * N * K + 2 * M * N

        def run():
            assert lib.ogv_gemm_fwd(A.data_ptr(), K, W.data_ptr(), None, None, None, 0, out.data_ptr(), N, M, N, K,
                                    act, 1, st) == 0
    else:
        D = torch.randn(M, N, device=dev).to(bf)
        Z = torch.randn(M, K, device=dev).to(bf)
        dA = torch.empty(M, K, device=dev, dtype=bf)
        ws = torch.empty(1 << 16, device=dev, dtype=torch.uint8)
        nbytes = 2 * M * N + 4 * N * K + 2 * M * K + (2 * M * K if act else 0)

        def run():
            assert lib.ogv_gemm_dgrad(D.data_ptr(), N, W.data_ptr(), Z.data_ptr() if act else None, K, None, 0,
                                      dA.data_ptr(), K, M, N, K, act, ws.data_ptr(), 1, st) == 0
    for _ in range(5):
        run()
    torch.cuda.synchronize()
    if a.cold:
        flush = torch.ones(128 << 20, dtype=torch.float32, device=dev)
        ts = []
        for _ in range(a.reps):
            flush.sum()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            run()
            e1.record()
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1) * 1e3)
        us = statistics.median(ts)
    else:
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.reps):
            run()
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / a.reps
    flops = 2.0 * M * N * K
    print(f"{a.kind} M={M} N={N} K={K} act={a.act} opts={a.opt} {'cold' if a.cold else 'warm'}: {us:.1f} us  "
          f"{nbytes / us / 1e3:.0f} GB/s  {flops / us / 1e6:.0f} TFLOP/s")


if __name__ == "__main__":
    main()
