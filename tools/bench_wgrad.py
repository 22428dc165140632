"""Isolated timing of every bf16 weight-gradient shape of a model step through the C ABI
(tuning aid for ogv_gemm.hip / ogv_swgrad.hip).

    python tools/bench_wgrad.py [--shapes tools/gemm_shapes_7m.txt] [--cfg base:] [--cfg t64:wg_tile=64] [--reps 20]

Shapes come from an OGV_LOG_GEMM=1 log (lines "OGVGEMM wgrad dt=1 M= N= K= pro= conv= bias=").  A
prologue (pro=1) shape is timed with a GELU prologue (the MLP fc2 form; the MBConv BN+SiLU+gate form is
internal to the fused MBConv op).  Each --cfg NAME:k=v,k=v sets knobs before its pass and resets them
after (every knob listed in any cfg is reset to the value given by --defaults).  Prints us per launch
(warm, back-to-back between two events, incl. the colreduce), algorithmic GB/s and the per-step total
(us x occurrences).
"""
import argparse
import collections
import ctypes
import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "outlook-grid-vision-transformer_amd"))

import torch  # noqa: E402


def parse_shapes(path):
    pat = re.compile(r"OGVGEMM wgrad dt=1 M=(\d+) N=(\d+) K=(\d+) pro=(\d) conv=(\d) bias=(\d)")
    cnt = collections.Counter()
    with open(path) as f:
        for line in f:
            m = pat.search(line)
            if m and m.group(5) == "0":
                cnt[tuple(int(x) for x in (m.group(1), m.group(2), m.group(3), m.group(4), m.group(6)))] += 1
    return sorted(cnt.items(), key=lambda kv: -kv[0][0] * kv[0][1] * kv[0][2] * kv[1])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shapes", default=os.path.join(ROOT, "tools", "gemm_shapes_7m.txt"))
    ap.add_argument("--cfg", action="append", default=[])
    ap.add_argument("--defaults", default="")
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--only", default=None, help="M,N,K filter")
    a = ap.parse_args()
    import ogv
    from ogv._lib import load
    ogv.load()
    lib = load()
    cfgs = []
    for c in (a.cfg or ["base:"]):
        name, _, kv = c.partition(":")
        cfgs.append((name, [tuple(x.split("=")) for x in kv.split(",") if x]))
    defaults = dict(tuple(x.split("=")) for x in a.defaults.split(",") if x)
    dev, bf = "cuda", torch.bfloat16
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    shapes = parse_shapes(a.shapes)
    if a.only:
        want = tuple(int(x) for x in a.only.split(","))
        shapes = [s for s in shapes if s[0][:3] == want]
    tot = collections.Counter()
    for (M, N, K, pro, bias), n in shapes:
        G = torch.randn(M, N, device=dev).to(bf)
        X = torch.randn(M, K, device=dev).to(bf)
        dW = torch.empty(N, K, device=dev)
        db = torch.empty(N, device=dev)
        act = 1 if pro else 0
        wsb = [None]

        def run():
            assert lib.ogv_gemm_wgrad(G.data_ptr(), N, X.data_ptr(), K, None, 1, dW.data_ptr(),
                                      db.data_ptr() if bias else None, M, N, K, act, wsb[0].data_ptr(), 1, st) == 0
        nbytes = 2 * M * (N + K) + 4 * N * K
        line = f"M={M:7d} N={N:5d} K={K:5d} pro={pro} bias={bias} x{n:2d}:"
        ref = None
        for name, kvs in cfgs:
            for k, v in kvs:
                assert lib.ogv_set_option(k.encode(), int(v)) == 0, (k, v)
            # the workspace size depends on the plan, i.e. on the knobs in force: size it after setting them
            wsb[0] = torch.empty(lib.ogv_gemm_wgrad_ws_bytes(M, N, K), device=dev, dtype=torch.uint8)
            for _ in range(3):
                run()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.reps):
                run()
            e1.record()
            torch.cuda.synchronize()
            us = e0.elapsed_time(e1) * 1e3 / a.reps
            out = dW.clone()
            if ref is None:
                ref = out
            err = (out - ref).abs().max().item() / max(ref.abs().max().item(), 1e-30)
            for k, _ in kvs:
                assert lib.ogv_set_option(k.encode(), int(defaults.get(k, 0))) == 0, k
            wsb[0] = None
            tot[name] += us * n
            line += f"  {name} {us:7.1f} us {nbytes / us / 1e3:5.0f} GB/s" + (f" (rel {err:.1e})" if err > 1e-3 else "")
        print(line, flush=True)
        del G, X
        torch.cuda.empty_cache()
    print("per-step total: " + "  ".join(f"{k} {v:8.1f} us" for k, v in tot.items()), flush=True)


if __name__ == "__main__":
    main()
