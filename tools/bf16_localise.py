"""Localise the bf16 forward error of Model-A on a golden case: per-module max|bf16 - fp32| of
our own path (fp32 path == reference to ~4e-6), relative to the fp32 activation scale.
    python tools/bf16_localise.py [model_a_7m_eval_b2]
"""
import json
import pathlib
import sys

ROOT = pathlib.Path(__file__).resolve().parents[1]
for p in (ROOT / "outlook-grid-vision-transformer_amd", ROOT / "tests", ROOT / "tests" / "golden", ROOT / "oracle"):
    sys.path.insert(0, str(p))
import numpy as np
import torch

import _fixtures as fx
import gen_params as gp
import ogv
from test_gpu_parity import _module

ogv.load()
name = sys.argv[1] if len(sys.argv) > 1 else "model_a_7m_eval_b2"
meta, arr = fx.load(name)
mod = _module(meta)
gp.fill_module(mod, meta["seed"])
mod = mod.cuda().eval()
x = torch.from_numpy(gp.input_from_spec(meta["x"])).cuda().contiguous(memory_format=torch.channels_last)

acts = {}


def hook(nm):
    def f(m, i, o):
        acts.setdefault(nm, []).append(o.detach().float().clone())
    return f


names = ["stem", "proj_in", "head_norm", "classifier"]
for s, blocks in enumerate(mod.stages):
    for b, blk in enumerate(blocks):
        for sub in ("outlook", "mbconv"):
            names.append(f"stages.{s}.{b}.{sub}")
        names.append(f"stages.{s}.{b}")
for s in range(len(mod.downs)):
    names.append(f"downs.{s}")
mods = dict(mod.named_modules())
for n in names:
    mods[n].register_forward_hook(hook(n))
with torch.no_grad():
    l32 = mod(x)
    with torch.autocast("cuda", dtype=torch.bfloat16):
        l16 = mod(x)
ref = torch.from_numpy(arr["logits"]).cuda()
print(f"{name}: logits |ref| {ref.abs().max().item():.3f}  fp32 err {(l32 - ref).abs().max().item():.2e}  "
      f"bf16 err {(l16.float() - ref).abs().max().item():.3e}")
order = sorted(acts, key=lambda n: names.index(n))
for n in order:
    a, b = acts[n]
    sc = a.abs().max().item()
    e = (b - a).abs().max().item()
    rms = ((b - a) ** 2).mean().sqrt().item() / max(a.pow(2).mean().sqrt().item(), 1e-30)
    print(f"  {n:24s} |fp32|max {sc:9.3f}  max|d| {e:.3e}  rel(max) {e / max(sc, 1e-30):.2e}  rel(rms) {rms:.2e}")
