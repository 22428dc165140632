"""Owners of the ATen glue launches (fills, zeros, copies, cats, clones) of one eager Model-A-7M
training step: torch.profiler over one step after warm-up, each glue op with its input shapes and
the chain of enclosing profiler events (autograd nodes / Python functions) that issued it.
    python tools/diag_glue.py [--batch 512]"""
import argparse
import collections
import pathlib
import sys

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "outlook-grid-vision-transformer_amd"))
import torch  # noqa: E402
from torch.profiler import ProfilerActivity, profile  # noqa: E402

import ogv  # noqa: E402
from ogv.train import MODEL_CONFIGS, Trainer, build_model  # noqa: E402

GLUE = ("aten::fill_", "aten::zero_", "aten::zeros", "aten::new_zeros", "aten::zeros_like", "aten::copy_",
        "aten::cat", "aten::clone", "aten::add", "aten::add_", "aten::mul", "aten::mul_", "aten::sum", "aten::div",
        "aten::neg", "aten::masked_fill_", "aten::stack", "aten::ones_like")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=512)
    ap.add_argument("--graphs", type=int, default=0)
    a = ap.parse_args()
    ogv.load()
    cfg = MODEL_CONFIGS["model_a_7m"]
    torch.manual_seed(7)
    m = build_model({k: v for k, v in cfg.items() if k != "img"}).cuda().to(memory_format=torch.channels_last)
    t = Trainer(m, total_steps=100, graphs=False)
    x = torch.randn(a.batch, 3, 32, 32, device="cuda").contiguous(memory_format=torch.channels_last)
    y = torch.randint(0, 100, (a.batch,), device="cuda")
    for _ in range(2):
        t.step(x, y)
    torch.cuda.synchronize()
    with profile(activities=[ProfilerActivity.CPU], record_shapes=True) as prof:
        t.step(x, y)
        torch.cuda.synchronize()
    cnt = collections.Counter()
    for ev in prof.events():
        if ev.name not in GLUE:
            continue
        chain, p = [], ev.cpu_parent
        while p is not None and len(chain) < 4:
            if not p.name.startswith("aten::"):
                chain.append(p.name[:70])
            p = p.cpu_parent
        shapes = str(ev.input_shapes)[:60] if ev.input_shapes else ""
        # direct children that are aten ops launching work would double count: keep only leaves
        if any(c.name in GLUE for c in ev.cpu_children):
            continue
        cnt[(ev.name, " < ".join(chain) or "(top)", shapes)] += 1
    for (name, chain, shp), n in sorted(cnt.items(), key=lambda kv: -kv[1]):
        print(f"{n:4d}  {name:18s} {shp:60s} {chain}")


if __name__ == "__main__":
    main()
