"""Helpers to load the golden fixtures (tests/golden/*.npz) and rebuild their inputs/params."""
from __future__ import annotations

import json
import pathlib

import numpy as np
import torch
import torch.utils._python_dispatch
import torch.utils._pytree

import gen_params as gp
import ogv_oracle as orc

GOLDEN = pathlib.Path(__file__).resolve().parent / "golden"


def load(name: str):
    z = np.load(GOLDEN / f"{name}.npz", allow_pickle=False)
    meta = json.loads(bytes(z["meta"]).decode())
    return meta, {k: z[k] for k in z.files if k != "meta"}


def fixture_names(prefix: str):
    return sorted(p.stem for p in GOLDEN.glob(prefix + "*.npz"))


def inputs(meta):
    x = gp.input_from_spec(meta["x"])
    dy = gp.input_from_spec(meta["dy"]) if "dy" in meta else None
    return x, dy


def shapes_for(meta) -> dict:
    """state_dict shapes of the module a fixture was recorded on (module-relative keys)."""
    kind = meta["kind"]
    if kind == "outlook_attn":
        C, h, k = meta["dim"], meta["heads"], meta["k"]
        return {"attn.weight": (h * k * k, C, 1, 1), "attn.bias": (h * k * k,), "v.weight": (C, C, 1, 1),
                "v.bias": (C,), "proj.weight": (C, C, 1, 1), "proj.bias": (C,)}
    if kind in ("grid_attn", "grid_attn_capture"):
        C = meta["dim"]
        return {"mhsa.qkv.weight": (3 * C, C), "mhsa.qkv.bias": (3 * C,), "mhsa.proj.weight": (C, C),
                "mhsa.proj.bias": (C,)}
    if kind == "layernorm2d":
        return {"ln.weight": (meta["dim"],), "ln.bias": (meta["dim"],)}
    if kind == "outlooker_block":
        full = orc.block_shapes("", dict(dim=meta["dim"], num_heads=1, grid_size=1, outlook_heads=meta["heads"]))
        return {k[len("outlook."):]: v for k, v in full.items() if k.startswith("outlook.")}
    if kind == "mbconv":
        full = orc.block_shapes("", dict(dim=meta["dim"], num_heads=1, grid_size=1, outlook_heads=1))
        return {k[len("mbconv."):]: v for k, v in full.items() if k.startswith("mbconv.")}
    if kind == "outgrid_block":
        return orc.block_shapes("", meta["stage"])
    if kind == "gridonly_block":
        return orc.gridonly_block_shapes("", meta["stage"])
    if kind == "stage_out_then_grid":
        return orc.stage_out_then_grid_shapes("", meta["stage"], meta["depth"], meta["out_depth"])
    if kind == "model_b":
        return orc.model_b_shapes(meta["stages"], meta["num_classes"], 3, meta["stem_dim"],
                                  meta["outlooker_front_depth"])
    if kind == "model_a":
        return orc.model_a_shapes(meta["stages"], meta["num_classes"], 3, meta["stem_dim"])
    raise KeyError(kind)


def oracle_params(meta, requires_grad=True):
    seed = meta["seed"]
    return orc.make_params(shapes_for(meta), lambda k, s: gp.param_value(k, s, seed), requires_grad)


def compare_grads(named_grads, arrays, rtol, atol, label="", floor_tag=None, floor_scale=1.0):
    """Check full grads ('grad.<k>') or sketches ('gsketch.<k>' + 'gnorm.<k>') of a fixture.
    floor_tag (e.g. "bf16"): where the fixture also holds the REFERENCE'S OWN gradients of that
    precision ('<tag>grad.<k>' / '<tag>gsketch.<k>' / '<tag>gnorm.<k>'), the tolerance of that tensor
    is at least floor_scale x the reference's own deviation from its fp32 gradient."""
    checked = 0
    for k, g in named_grads.items():
        if g is None:
            continue
        g = g.detach().double().cpu()
        if "grad." + k in arrays:
            ref = torch.from_numpy(arrays["grad." + k]).double()
            err = (g - ref).abs().max().item()
            tol = atol + rtol * ref.abs().max().item()
            if floor_tag and floor_tag + "grad." + k in arrays:
                tol = max(tol, floor_scale * (torch.from_numpy(arrays[floor_tag + "grad." + k]).double() - ref).abs().max().item())
            assert err <= tol, f"{label} grad {k}: max|d|={err:.3e} > {tol:.3e}"
            checked += 1
        elif "gsketch." + k in arrays:
            g2 = g.reshape(g.shape[0], -1)
            sk = g2 @ torch.from_numpy(gp.sketch_matrix(k, g2.shape[1]))
            ref = torch.from_numpy(arrays["gsketch." + k]).double()
            scale = float(arrays["gnorm." + k][0])
            err = (sk - ref).abs().max().item()
            tol = atol * max(1.0, scale) + rtol * ref.abs().max().item()
            ntol = tol + rtol * scale
            if floor_tag and floor_tag + "gsketch." + k in arrays:
                tol = max(tol, floor_scale * (torch.from_numpy(arrays[floor_tag + "gsketch." + k]).double() - ref).abs().max().item())
                ntol = max(ntol, floor_scale * abs(float(arrays[floor_tag + "gnorm." + k][0]) - scale))
            assert err <= tol, f"{label} gsketch {k}: max|d|={err:.3e} > {tol:.3e}"
            n = g2.norm().item()
            assert abs(n - scale) <= ntol, f"{label} gnorm {k}: {n} vs {scale}"
            checked += 1
    return checked


def maxrel(a, b):
    a = torch.as_tensor(a).double().cpu()
    b = torch.as_tensor(b).double().cpu()
    return ((a - b).abs().max() / b.abs().max().clamp_min(1e-12)).item()


def maxabs(a, b):
    return (torch.as_tensor(a).double().cpu() - torch.as_tensor(b).double().cpu()).abs().max().item()


class Bf16Storage(torch.utils._python_dispatch.TorchDispatchMode):
    """fp32 emulation of bf16 activation storage (test infrastructure): every floating-point
    tensor an op produces is rounded to bf16 and carried on in fp32.  Parameters enter unrounded
    (the kernels multiply by hi + lo weight halves: split_w), arithmetic is fp32.  Run the CPU
    oracle's functions under it (on any device) to get the error that storing every intermediate
    activation in bf16 costs a forward -- a superset of the fused kernels' own rounding points."""

    def __torch_dispatch__(self, func, types, args=(), kwargs=None):
        out = func(*args, **(kwargs or {}))

        def rnd(t):
            if isinstance(t, torch.Tensor) and t.dtype == torch.float32 and t.ndim >= 1 and t.numel() > 1:
                return t.to(torch.bfloat16).to(torch.float32)
            return t
        return torch.utils._pytree.tree_map(rnd, out)


def bf16_storage_error(fn, x, ref):
    """max|fn(bf16(x)) - ref| with fn run under Bf16Storage (fn: oracle forward of x)."""
    with torch.no_grad(), Bf16Storage():
        y = fn(x.to(torch.bfloat16).to(torch.float32))
    return maxabs(y.float(), ref)
