"""Grid-attention kernel timing at the large-group shapes (224^2 stage 0: N = 784 tokens per group).

For each kernel generation selected by the ``grid_big`` knob (1: first generation, 2: exp2 /
lazy-rescale / paired 16x16x32 products), times ogv_grid_attn_fwd and ogv_grid_attn_bwd (HIP
events on torch's stream, average over --reps launches) and reports TFLOP/s against the 2.5 PF bf16
dense MFMA peak (4*M*N*C flops forward, 10*M*N*C backward: the recomputed S and the dP, dQ, dK,
dV products).  Also prints the max |difference| of out / lse / dqkv between the generations.

    python tools/bench_grid.py [--batch 128 --hw 224 --c 64 --heads 2 --g 8] [--reps 10]
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "outlook-grid-vision-transformer_amd"))

import torch  # noqa: E402

PEAK_TF = 2500.0


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
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--hw", type=int, default=224)
    ap.add_argument("--c", type=int, default=64)
    ap.add_argument("--heads", type=int, default=2)
    ap.add_argument("--g", type=int, default=8)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--gens", default="1,2")
    a = ap.parse_args()
    import ogv
    from ogv._lib import check, load
    ogv.load()
    lib = load()
    B, H, C, h, g = a.batch, a.hw, a.c, a.heads, a.g
    M, N = B * H * H, (H // g) ** 2
    scale = (C // h) ** -0.5
    gen = torch.Generator(device="cuda").manual_seed(0)
    qkv = torch.randn(M, 3 * C, device="cuda", generator=gen).to(torch.bfloat16)
    dy = torch.randn(M, C, device="cuda", generator=gen).to(torch.bfloat16)
    st = torch.cuda.current_stream().cuda_stream
    res = {}
    print(f"M={M} N={N} C={C} heads={h} hd={C // h}", flush=True)
    for gen_id in [int(x) for x in a.gens.split(",")]:
        check(lib.ogv_set_option(b"grid_big", gen_id), "grid_big")
        out = torch.empty(M, C, device="cuda", dtype=torch.bfloat16)
        lse = torch.empty(M, h, device="cuda")
        dqkv = torch.empty(M, 3 * C, device="cuda", dtype=torch.bfloat16)
        dws = torch.empty(M, h, device="cuda")
        fwd = lambda: check(lib.ogv_grid_attn_fwd(qkv.data_ptr(), out.data_ptr(), lse.data_ptr(), None, B, H, H, C, h, g,
                                                  scale, 1, st), "grid fwd")
        bwd = lambda: check(lib.ogv_grid_attn_bwd(dy.data_ptr(), qkv.data_ptr(), out.data_ptr(), lse.data_ptr(),
                                                  dqkv.data_ptr(), dws.data_ptr(), B, H, H, C, h, g, scale, 1, st),
                            "grid bwd")
        uf = timeit(fwd, a.reps)
        ub = timeit(bwd, a.reps)
        ff, fb = 4.0 * M * N * C, 10.0 * M * N * C
        print(f"grid_big={gen_id}: fwd {uf:9.1f} us {ff / uf / 1e6:7.1f} TF/s ({ff / uf / 1e6 / PEAK_TF:.3f}) | "
              f"bwd {ub:9.1f} us {fb / ub / 1e6:7.1f} TF/s ({fb / ub / 1e6 / PEAK_TF:.3f})", flush=True)
        res[gen_id] = (out.float(), lse.clone(), dqkv.float())
    if len(res) == 2:
        (o1, l1, d1), (o2, l2, d2) = res.values()
        print(f"max|d| out {(o1 - o2).abs().max().item():.3e} (|out| {o1.abs().max().item():.2f}) "
              f"lse {(l1 - l2).abs().max().item():.3e} dqkv {(d1 - d2).abs().max().item():.3e} "
              f"(|dqkv| {d1.abs().max().item():.2f})", flush=True)
    check(lib.ogv_set_option(b"grid_big", 2), "grid_big")


if __name__ == "__main__":
    main()
