"""Fused MBConv fwd+bwd at the Model-A-7M stage shapes (bs=512, bf16), for kernel profiling:

    rocprofv3 --kernel-trace -d DIR -o mb -- python3 tools/bench_mbconv.py [--reps 5]
    python tools/kernels_by_grid.py DIR/mb_kernel_trace.csv
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "outlook-grid-vision-transformer_amd"))

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--batch", type=int, default=512)
    ap.add_argument("--dw-blocks", type=int, default=0, help="dw_blocks option (0: library default)")
    ap.add_argument("--opt", action="append", default=[], metavar="NAME=VALUE")
    a = ap.parse_args()
    import ogv
    from ogv._lib import load
    ogv.load()
    assert load().ogv_set_option(b"dw_blocks", a.dw_blocks) == 0
    for o in a.opt:
        k, v = o.split("=")
        assert load().ogv_set_option(k.encode(), int(v)) == 0, o
    from src.model.mbc_conv import MBConv, MBConvConfig
    for C, H in ((48, 32), (96, 16), (192, 8), (256, 4)):
        m = MBConv(C, C, 1, MBConvConfig()).cuda().to(memory_format=torch.channels_last).train()
        x = torch.randn(a.batch, C, H, H, device="cuda").contiguous(memory_format=torch.channels_last)
        x = x.to(torch.bfloat16).requires_grad_(True)
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
        for r in range(a.reps + 1):
            if r == 1:
                ev[0].record()
            y = m(x)
            if r == 1:
                ev[1].record()
            y.backward(torch.ones_like(y))
            if r == 1:
                ev[2].record()
        torch.cuda.synchronize()
        print(f"mbconv C={C} H={H}: fwd {ev[0].elapsed_time(ev[1]):.3f} ms  bwd {ev[1].elapsed_time(ev[2]):.3f} ms",
              flush=True)


if __name__ == "__main__":
    main()
