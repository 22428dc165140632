"""Where the ATen (non-ogv) launches of one eager Model-A-7M training step come from: torch.profiler
over one step after warm-up, ATen ops that launched device work, grouped by op and the innermost
frame of this repository in their Python stack.    python tools/diag_aten_ops.py [--batch 512]"""
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=512)
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
    with profile(activities=[ProfilerActivity.CPU], with_stack=True) as prof:
        t.step(x, y)
        torch.cuda.synchronize()
    cnt = collections.Counter()
    for ev in prof.events():
        if not ev.name.startswith("aten::") or ev.name in ("aten::empty", "aten::empty_strided", "aten::view",
                                                           "aten::as_strided", "aten::reshape", "aten::permute",
                                                           "aten::detach", "aten::t", "aten::slice", "aten::select",
                                                           "aten::alias", "aten::split", "aten::narrow",
                                                           "aten::expand", "aten::_reshape_alias",
                                                           "aten::resolve_conj", "aten::resolve_neg", "aten::lift_fresh",
                                                           "aten::unsqueeze", "aten::squeeze", "aten::view_as",
                                                           "aten::chunk", "aten::unbind", "aten::transpose",
                                                           "aten::contiguous", "aten::result_type", "aten::item",
                                                           "aten::_local_scalar_dense", "aten::is_nonzero",
                                                           "aten::empty_like", "aten::new_empty", "aten::to",
                                                           "aten::_to_copy"):
            continue
        frames = [f for f in (ev.stack or []) if "outlook-grid" in f or "ogv" in f or "/src/" in f]
        where = frames[0].split("/")[-1] if frames else (ev.stack[0].split("/")[-1] if ev.stack else "?")
        cnt[(ev.name, where)] += 1
    for (name, where), n in cnt.most_common(60):
        print(f"{n:5d}  {name:40s} {where}")


if __name__ == "__main__":
    main()
