"""A/B microbenchmark of the projection GEMMs: persistent streaming kernel (sgemm) vs tiled kernel.

For every 1x1 projection of an OutGridBlock at the Model-A-7M bs=512 shapes: fwd (plain, GELU
prologue, +residual) and dgrad, each timed with sgemm on and off.  Caches are flushed (a 512 MB
write) before every timed launch so A is read from HBM as in the train step; HIP events bracket
the launch only (the flush keeps the GPU ahead of the host, so no launch gap is timed).
Checks both variants against a torch fp32 reference of the same op.

    python tools/bench_sgemm.py [--batch 512] [--reps 10] [--stages 48,96]
"""
import argparse
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "outlook-grid-vision-transformer_amd"))

import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

PEAK = 8000.0
HW = {48: 32, 96: 16, 192: 8, 256: 4}
HEADS = {48: 2, 96: 3, 192: 6, 256: 8}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=512)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--stages", default="48,96,192,256")
    ap.add_argument("--wgrad", action="store_true")
    ap.add_argument("--min-m", type=int, default=0, help="sgemm_min_m option (0: library default)")
    ap.add_argument("--bk64-max-m", type=int, default=-1, help="bk64_max_m option (-1: library default)")
    a = ap.parse_args()
    import ogv
    from ogv._lib import ACT, load
    ogv.load()
    lib = load()
    dev = "cuda"
    bf = torch.bfloat16
    # cache flush = a READ of 512 MB (a write would leave dirty lines whose write-back lands inside
    # the timed launch)
    if a.bk64_max_m >= 0:
        assert lib.ogv_set_option(b"bk64_max_m", a.bk64_max_m) == 0
    if a.min_m:
        assert lib.ogv_set_option(b"sgemm_min_m", a.min_m) == 0
    flush = torch.ones(128 << 20, dtype=torch.float32, device=dev)
    torch.cuda.synchronize()
    st = torch.cuda.current_stream().cuda_stream
    p = lambda t: None if t is None else t.data_ptr()  # noqa: E731

    def timeit(fn):
        ts = []
        for _ in range(a.reps + 1):
            flush.sum()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            fn()
            e1.record()
            e1.synchronize()
            ts.append(e0.elapsed_time(e1) * 1e3)
        return statistics.median(ts[1:])

    def both(fn):
        r = {}
        for mode in (0, 1):
            assert lib.ogv_set_option(b"sgemm", mode) == 0
            r[mode] = timeit(fn)
        return r

    # calibration: torch copy / fill / read-reduce of 256 MB (cold)
    src = torch.randn(64 << 20, device=dev)
    dst = torch.empty_like(src)
    t = timeit(lambda: dst.copy_(src))
    print(f"calib copy 256MB->256MB   {t:7.1f} us {2 * src.numel() * 4 / t / 1e3:6.0f} GB/s", flush=True)
    t = timeit(lambda: dst.fill_(1.0))
    print(f"calib fill 256MB          {t:7.1f} us {src.numel() * 4 / t / 1e3:6.0f} GB/s", flush=True)
    t = timeit(lambda: src.sum())
    print(f"calib sum  256MB          {t:7.1f} us {src.numel() * 4 / t / 1e3:6.0f} GB/s", flush=True)
    del src, dst
    for C in [int(c) for c in a.stages.split(",")]:
        H = HW[C]
        M = a.batch * H * H
        gemms = [("outlook.attn", C, 9 * HEADS[C], None), ("outlook.v", C, C, None),
                 ("mlp2d.fc1", C, 2 * C, None), ("mlp2d.fc2(gelu)", 2 * C, C, "gelu"),
                 ("mbconv.expand", C, 4 * C, None), ("mbconv.project", 4 * C, C, None),
                 ("grid.qkv", C, 3 * C, None), ("mlp.fc1", C, 4 * C, None), ("mlp.fc2(gelu)+res", 4 * C, C, "gelu")]
        for name, K, N, act in gemms:
            g = torch.Generator(device=dev).manual_seed(1)
            x = torch.randn(M, K, device=dev, dtype=bf, generator=g)
            w = torch.randn(N, K, device=dev, generator=g) / K ** 0.5
            b = torch.randn(N, device=dev, generator=g)
            res = torch.randn(M, N, device=dev, dtype=bf, generator=g) if "res" in name else None
            out = torch.empty(M, N, device=dev, dtype=bf)
            outs = {}

            def fwd():
                lib.ogv_gemm_fwd(p(x), K, p(w), p(b), p(res), None, 1, p(out), N, M, N, K, ACT[act], 1, st)

            t = {}
            for mode in (0, 1):
                assert lib.ogv_set_option(b"sgemm", mode) == 0
                t[mode] = timeit(fwd)
                outs[mode] = out.float().clone()
            if act is None and res is None:  # hipBLASLt reference point (torch.nn.functional.linear, bf16)
                wb = w.to(bf)
                tl = timeit(lambda: F.linear(x, wb))
                print(f"      torch/hipBLASLt linear {tl:7.1f} us {2 * M * (K + N) / tl / 1e3:6.0f} GB/s", flush=True)
            xa = F.gelu(x.float()) if act else x.float()
            ref = xa @ w.t() + b
            if res is not None:
                ref = ref + res.float()
            tol = 2e-2 * ref.abs().max().item()
            e0 = (outs[0] - ref).abs().max().item()
            e1 = (outs[1] - ref).abs().max().item()
            nbytes = 2 * M * (K + N) + (2 * M * N if res is not None else 0) + 4 * N * K
            print(f"fwd   s{C:<3d} {name:20s} M={M:7d} N={N:5d} K={K:5d}  tiled {t[0]:7.1f} us "
                  f"{nbytes / t[0] / 1e3:6.0f} GB/s | sgemm {t[1]:7.1f} us {nbytes / t[1] / 1e3:6.0f} GB/s "
                  f"({t[0] / t[1]:4.2f}x)  err {e0:.1e}/{e1:.1e} {'OK' if max(e0, e1) < tol else 'BAD'}", flush=True)
            # dgrad
            dout = torch.randn(M, N, device=dev, dtype=bf, generator=g)
            dx = torch.empty(M, K, device=dev, dtype=bf)
            ws = torch.empty(lib.ogv_gemm_dgrad_ws_bytes(N, K) + 256, dtype=torch.uint8, device=dev)
            Z = x if act else None

            def dg():
                lib.ogv_gemm_dgrad(p(dout), N, p(w), p(Z), K, None, 1, p(dx), K, M, N, K, ACT[act], p(ws), 1, st)

            for mode in (0, 1):
                assert lib.ogv_set_option(b"sgemm", mode) == 0
                t[mode] = timeit(dg)
                outs[mode] = dx.float().clone()
            ref = dout.float() @ w
            if act:
                xx = x.float().requires_grad_(True)
                yy = F.gelu(xx)
                (gr,) = torch.autograd.grad(yy, xx, ref)
                ref = gr
            tol = 2e-2 * ref.abs().max().item()
            e0 = (outs[0] - ref).abs().max().item()
            e1 = (outs[1] - ref).abs().max().item()
            nbytes = 2 * M * (K + N) + (2 * M * K if act else 0) + 4 * N * K
            print(f"dgrad s{C:<3d} {name:20s} M={M:7d} N={N:5d} K={K:5d}  tiled {t[0]:7.1f} us "
                  f"{nbytes / t[0] / 1e3:6.0f} GB/s | sgemm {t[1]:7.1f} us {nbytes / t[1] / 1e3:6.0f} GB/s "
                  f"({t[0] / t[1]:4.2f}x)  err {e0:.1e}/{e1:.1e} {'OK' if max(e0, e1) < tol else 'BAD'}", flush=True)
            # wgrad: dW = dout^T . act(x), dbias (fp32, split-M partials + column reduction)
            if a.wgrad:
                dw = torch.empty(N, K, device=dev)
                db = torch.empty(N, device=dev)
                wsw = torch.empty(lib.ogv_gemm_wgrad_ws_bytes(M, N, K), dtype=torch.uint8, device=dev)
                xa = F.gelu(x.float()) if act else x.float()
                refw = dout.float().t() @ xa
                refb = dout.float().sum(0)
                tw, ew = {}, {}
                for mode in (0, 1):
                    assert lib.ogv_set_option(b"sgemm", mode) == 0
                    tw[mode] = timeit(lambda: lib.ogv_gemm_wgrad(p(dout), N, p(x), K, None, 1, p(dw), p(db), M, N, K,
                                                                 ACT[act], p(wsw), 1, st))
                    ew[mode] = max((dw - refw).abs().max().item() / max(1e-6, refw.abs().max().item()),
                                   (db - refb).abs().max().item() / max(1e-6, refb.abs().max().item()))
                nbytes = 2 * M * (K + N) + 4 * N * K
                print(f"wgrad s{C:<3d} {name:20s} M={M:7d} N={N:5d} K={K:5d}  tiled {tw[0]:7.1f} us "
                      f"{nbytes / tw[0] / 1e3:6.0f} GB/s | stream {tw[1]:7.1f} us {nbytes / tw[1] / 1e3:6.0f} GB/s "
                      f"({tw[0] / tw[1]:4.2f}x)  relerr {ew[0]:.1e}/{ew[1]:.1e} "
                      f"{'OK' if max(ew.values()) < 2e-2 else 'BAD'}", flush=True)
                del dw, db, wsw
            del x, out, dout, dx, res
        torch.cuda.empty_cache()
    lib.ogv_set_option(b"sgemm", 1)


if __name__ == "__main__":
    main()
