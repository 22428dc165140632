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


# ------------------------------------------------------------------ training-step fixture (make_golden.py r4)
def train_batches(meta):
    """The fixture's batches: images gen_params.tensor('train_x_<t>'), labels gen_params.labels('train_t_<t>');
    step meta['nan_step'] holds one NaN pixel (the reference skips that step)."""
    out = []
    for t in range(meta["steps"]):
        x = gp.tensor(f"train_x_{t}", (meta["B"], 3, 32, 32))
        if t == meta["nan_step"]:
            x[0, 0, 0, 0] = np.nan
        out.append((torch.from_numpy(x), torch.from_numpy(gp.labels(f"train_t_{t}", meta["B"], meta["num_classes"]))))
    return out


def update_sketch(key, d):
    """tests/golden/make_golden.py::update_sketch on a torch / numpy update (float64)."""
    d = torch.as_tensor(d).double().cpu()
    d = d.reshape(d.shape[0], -1) if d.dim() > 0 else d.reshape(1, 1)
    L = torch.from_numpy(gp.sketch_matrix(key + ":rows", d.shape[0], 8))
    R = torch.from_numpy(gp.sketch_matrix(key, d.shape[1], 8))
    return L.T @ d @ R


def train_stable_masks(meta, arr, params):
    """name -> float64 0/1 mask of the elements the fixture's update sketches cover (make_golden.py main_r4:
    elements whose gradient was rounding noise at some step take a +-lr Adam step of random sign in any
    fp32 implementation and are left out)."""
    flat = torch.ones(sum(params[k].numel() for k in meta["param_names"]), dtype=torch.float64)
    flat[torch.from_numpy(arr["unstable"])] = 0.0
    out, off = {}, 0
    for k in meta["param_names"]:
        n = params[k].numel()
        out[k] = flat[off:off + n].view(params[k].shape)
        off += n
    return out


def train_step_errors(meta, arr, t, params, p0, masks=None, prefix=""):
    """Deviation of parameters ``params`` (name -> tensor, any device) after fixture step t from the
    reference's, with p0 (name -> tensor) the common start.  Returns a dict of maxima over parameters:
      upd    max|sketch(ours) - sketch(ref)| / max(|update_ref|_F, 1e-12) on the stable elements -- the
             relative error of the update
      dn     max| |update|_F ours - ref | / max(|update_ref|_F, 1e-12)
      norm   max| |p|_F ours - ref | / max(1, |p|_F ref)
      full   (steps recorded in full) max|p - p_ref| / max(1, max|p_ref|) over the stable elements of every
             small parameter
    'worst' = the parameter name behind the largest 'upd', and per parameter (numpy arrays in param_names
    order): 'upd_all', 'pn_abs' = | |p|_F ours - ref |, 'pns_abs' (with a 'pns{t}' array: the same on the
    stable elements).  ``prefix`` selects the fixture arrays' prefix ('amp_' for the bf16 fixture's)."""
    names = meta["param_names"]
    if masks is None:
        masks = train_stable_masks(meta, arr, params)
    dsk, dn, pn = arr[f"dsk{t}"], arr[f"dn{t}"], arr[f"pn{t}"]
    upd = dnerr = norm = 0.0
    worst = None
    upd_all, pn_abs, pns_abs = np.zeros(len(names)), np.zeros(len(names)), np.zeros(len(names))
    for i, k in enumerate(names):
        p = params[k].detach().double().cpu()
        d = (p - p0[k].detach().double().cpu()) * masks[k]
        scale = max(float(dn[i]), 1e-12)
        e = (update_sketch(k, d) - torch.from_numpy(dsk[i])).abs().max().item() / scale
        if float(dn[i]) > 0:
            upd_all[i] = e
        if float(dn[i]) > 0 and e > upd:
            upd, worst = e, k
        if float(dn[i]) > 0:
            dnerr = max(dnerr, abs(d.norm().item() - float(dn[i])) / scale)
        pn_abs[i] = abs(p.norm().item() - float(pn[i]))
        norm = max(norm, pn_abs[i] / max(1.0, float(pn[i])))
        if f"pns{t}" in arr:
            pns_abs[i] = abs((p * masks[k]).norm().item() - float(arr[f"pns{t}"][i]))
    out = dict(upd=upd, dn=dnerr, norm=norm, worst=worst, upd_all=upd_all, pn_abs=pn_abs, pns_abs=pns_abs)
    if f"p{t}" in arr:
        flat, off, full = arr[f"p{t}"], 0, 0.0
        for k in names:
            p = params[k].detach().double().cpu()
            if p.numel() > meta["full_max"]:
                continue
            ref = torch.from_numpy(flat[off:off + p.numel()]).double().view_as(p.contiguous())
            off += p.numel()
            full = max(full, ((p.contiguous() - ref) * masks[k]).abs().max().item() / max(1.0, ref.abs().max().item()))
        assert off == flat.size
        out["full"] = full
    return out


def amp_reference_errors(meta, arr, amp, t, params, masks):
    """The REFERENCE'S OWN bf16-autocast step's deviation from its fp32 step after step t (fixtures
    train_steps_7m_b16 = ``arr`` and train_steps_7m_b16_amp = ``amp``, make_golden.py r5: the same sketches,
    the same noise mask), in train_step_errors' terms: 'upd_all' / 'upd' (relative update-sketch error per
    parameter / max), 'dn', 'norm', 'full' (steps recorded in full, stable elements of every small
    parameter), 'loss' (|loss_bf16 - loss_fp32|).  ``params`` / ``masks`` give the parameter sizes and the
    stable-element masks (train_stable_masks)."""
    names = meta["param_names"]
    dn = arr[f"dn{t}"]
    scale = np.maximum(dn, 1e-12)
    upd_all = np.abs(amp[f"amp_dsk{t}"] - arr[f"dsk{t}"]).reshape(len(names), -1).max(1) / scale
    upd_all[dn == 0] = 0.0
    dn_err = np.abs(amp[f"amp_dn{t}"] - dn) / scale
    dn_err[dn == 0] = 0.0
    pn = arr[f"pn{t}"]
    out = dict(upd_all=upd_all, upd=float(upd_all.max()), dn=float(dn_err.max()),
               norm=float((np.abs(amp[f"amp_pn{t}"] - pn) / np.maximum(1.0, pn)).max()),
               loss=abs(float(amp["amp_loss"][t]) - float(arr["loss"][t])))
    if f"p{t}" in arr:
        a, b, off, full = arr[f"p{t}"].astype(np.float64), amp[f"amp_p{t}"].astype(np.float64), 0, 0.0
        for k in names:
            n = params[k].numel()
            if n > meta["full_max"]:
                continue
            m = masks[k].contiguous().reshape(-1).numpy() if masks[k].dim() else masks[k].reshape(-1).numpy()
            ref = a[off:off + n]
            full = max(full, float((np.abs(b[off:off + n] - ref) * m).max() / max(1.0, np.abs(ref).max())))
            off += n
        assert off == a.size
        out["full"] = full
    return out


def record(kind: str, **fields):
    """Append one JSON line of measured parity numbers to $OGV_PARITY_LOG (when set): the GPU runs
    write the achieved errors next to their bars, and the committed copy under profiles/ is the
    evidence each bar cites."""
    import json
    import os
    path = os.environ.get("OGV_PARITY_LOG")
    if not path:
        return

    def _py(v):
        if isinstance(v, (np.floating, np.integer)):
            return v.item()
        if isinstance(v, torch.Tensor):
            return v.item() if v.numel() == 1 else v.tolist()
        return v
    with open(path, "a") as f:
        f.write(json.dumps(dict(kind=kind, **{k: _py(v) for k, v in fields.items()})) + "\n")
