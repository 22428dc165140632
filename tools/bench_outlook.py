"""Outlook aggregation kernels per stage shape: LDS-tiled vs thread-per-chunk (knob outlook_tile),
fwd and bwd, HIP events over back-to-back launches (warm L2 excluded by a 512 MB flush between
reps).  Algorithmic bytes: fwd 2*M*(2C + 9h), bwd 2*M*(4C + 18h) (read dy, v, logits; write dv,
dlogits).   python tools/bench_outlook.py [--reps 20]"""
import argparse
import pathlib
import sys

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "outlook-grid-vision-transformer_amd"))
import torch  # noqa: E402

import ogv  # noqa: E402
from ogv import functional as OF  # noqa: E402
from ogv._lib import load  # noqa: E402

SHAPES = [("7m_s0", 512, 48, 2, 32), ("7m_s1", 512, 96, 3, 16), ("7m_s2", 512, 192, 6, 8), ("7m_s3", 512, 256, 8, 4),
          ("14m_s0", 256, 64, 2, 64), ("22m_s0", 128, 64, 2, 224)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    ogv.load()
    lib = load()
    flush = torch.empty(512 << 20, dtype=torch.uint8, device="cuda")
    for name, B, C, h, S in SHAPES:
        M = B * S * S
        ld = (C + 9 * h + 7) // 8 * 8
        cat = torch.randn(M, ld, device="cuda").to(torch.bfloat16)
        dy = torch.randn(M, C, device="cuda").to(torch.bfloat16)
        fb = 2 * M * (2 * C + 9 * h)
        bb = 2 * M * (4 * C + 18 * h)
        row = [name]
        for mode in (3, 0):
            assert lib.ogv_set_option(b"outlook_tile", mode) == 0
            ts = {"fwd": [], "bwd": []}
            for _ in range(a.reps):
                for kind in ("fwd", "bwd"):
                    flush.zero_()
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    if kind == "fwd":
                        e0.record()
                        OF._OutlookAggCat.forward(_Ctx(), cat, C, B, S, S, h, 3)
                        e1.record()
                    else:
                        e0.record()
                        OF._outlook_bwd(dy, cat.data_ptr(), ld, cat.data_ptr() + 2 * C, ld, cat.data_ptr(), ld,
                                        cat.data_ptr() + 2 * C, ld, ld - C, B, S, S, C, h, 3)
                        e1.record()
                    ts[kind].append((e0, e1))
            torch.cuda.synchronize()
            for kind, nb in (("fwd", fb), ("bwd", bb)):
                ms = sorted(x.elapsed_time(y) for x, y in ts[kind])[len(ts[kind]) // 2]
                row.append(f"{'tile' if mode else 'thr'}-{kind} {ms * 1e3:7.1f}us {nb / ms / 1e6:6.0f}GB/s")
        assert lib.ogv_set_option(b"outlook_tile", 2) == 0
        print("  ".join(row), flush=True)


class _Ctx:
    def save_for_backward(self, *a):
        pass


if __name__ == "__main__":
    main()
