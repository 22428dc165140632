"""ORACLE — CPU fp32 restatement of the OutGridBlock hot path.  TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this module, and
only as the checker / the timed CPU baseline — never as a product path.  The product (the
drop-in modules in outlook-grid-vision-transformer_amd/src) has no CPU execution path at all.

It restates, op for op on stock ATen CPU kernels, the reference algorithm of
pablo-reyes8/outlook-grid-vision-transformer (snapshot 2026-01-28).  Functions take a flat
parameter dict keyed like the reference state_dict, so the same deterministic parameters
(tests/golden/gen_params.py) fill both.  Cited reference lines (file:line):

  ln2d                src/model/outlook_attention.py:26-31       (permute, LN eps 1e-6, permute)
  outlook_attention   src/model/outlook_attention.py:91-124      (1x1 logits, softmax over k*k,
                                                                  1x1 v, unfold, mul+sum, 1x1 proj)
  mlp2d               src/model/outlook_attention.py:43-49
  outlooker_block     src/model/Outlook_Block.py:61-64
  mbconv              src/model/mbc_conv.py:22-27, 90-98
  grid_partition      src/model/grid_partition.py:3-17 / 20-32
  mhsa                src/model/grid_attention.py:62-89
  grid_attention      src/model/grid_attention.py:112-131
  outgrid_block       src/model/Out_Grid_Block.py:88-107 (MLP :24-32)
  gridonly_block      src/model/Grid_Only_Block.py:47-59
  stage_out_then_grid src/model/Grid_Only_Block.py:103-108
  model_b             src/Model_B_OutGridNet.py:10-104
  mix_apply           src/training/cutmix_mixup_aug.py:6-7, 36-64 (given the drawn perm/lam/box)
  model_a             src/Model_A_OutGridNet.py:14-67, stem_head.py:17-32, downsampling.py:50-65
  train_steps         src/training/one_epoch_train.py:85-153, train_full_model.py:56-66, warmup.py:4-59

Parity: pinned against golden vectors produced by running the reference itself in the build
container (tests/golden/make_golden.py; tests/test_oracle_golden.py checks this file against
them).  DropPath is stochastic, so the oracle (like the fixtures) runs it only as identity; the
CPU-baseline timing uses the same drop-path-free step.
"""
from __future__ import annotations

import math
from typing import Dict, List

import torch
import torch.nn.functional as F

P = Dict[str, torch.Tensor]


# ---------------------------------------------------------------------------- parameter shapes
def _ln(pre, c):
    return {pre + "weight": (c,), pre + "bias": (c,)}


def _bn(pre, c):
    return {pre + "weight": (c,), pre + "bias": (c,), pre + "running_mean": (c,), pre + "running_var": (c,),
            pre + "num_batches_tracked": ()}


def outlooker_shapes(pre: str, cfg: dict) -> Dict[str, tuple]:
    """OutlookerBlock2d (Outlook_Block.py:26-64): norm1.ln, attn.{attn,v,proj}, norm2.ln, mlp.fc1/fc2."""
    C = cfg["dim"]
    ho, k = cfg.get("outlook_heads", 6), cfg.get("outlook_kernel", 3)
    s = {}
    s.update(_ln(pre + "norm1.ln.", C))
    s[pre + "attn.attn.weight"] = (ho * k * k, C, 1, 1)
    s[pre + "attn.attn.bias"] = (ho * k * k,)
    for n in ("v", "proj"):
        s[pre + f"attn.{n}.weight"] = (C, C, 1, 1)
        s[pre + f"attn.{n}.bias"] = (C,)
    s.update(_ln(pre + "norm2.ln.", C))
    hid = max(1, int(C * cfg.get("outlook_mlp_ratio", 2.0)))
    s[pre + "mlp.fc1.weight"], s[pre + "mlp.fc1.bias"] = (hid, C, 1, 1), (hid,)
    s[pre + "mlp.fc2.weight"], s[pre + "mlp.fc2.bias"] = (C, hid, 1, 1), (C,)
    return s


def mbconv_shapes(pre: str, cfg: dict) -> Dict[str, tuple]:
    """MBConv (mbc_conv.py:44-89): expand.0/1, depthwise.0/1, se.fc1/fc2, project.0/1."""
    C = cfg["dim"]
    s = {}
    mid = max(1, int(round(C * cfg.get("mbconv_expand_ratio", 4.0))))
    use_bn = cfg.get("use_bn", True)
    if mid != C:
        s[pre + "expand.0.weight"] = (mid, C, 1, 1)
        if use_bn:
            s.update(_bn(pre + "expand.1.", mid))
        else:
            s[pre + "expand.0.bias"] = (mid,)
    s[pre + "depthwise.0.weight"] = (mid, 1, 3, 3)
    if use_bn:
        s.update(_bn(pre + "depthwise.1.", mid))
    else:
        s[pre + "depthwise.0.bias"] = (mid,)
    se_ratio = cfg.get("mbconv_se_ratio", 0.25)
    if se_ratio > 0:
        sq = max(1, int(mid * se_ratio))
        s[pre + "se.fc1.weight"], s[pre + "se.fc1.bias"] = (sq, mid, 1, 1), (sq,)
        s[pre + "se.fc2.weight"], s[pre + "se.fc2.bias"] = (mid, sq, 1, 1), (mid,)
    s[pre + "project.0.weight"] = (C, mid, 1, 1)
    if use_bn:
        s.update(_bn(pre + "project.1.", C))
    else:
        s[pre + "project.0.bias"] = (C,)
    return s


def grid_tail_shapes(pre: str, cfg: dict) -> Dict[str, tuple]:
    """norm2, grid_attn.mhsa.{qkv,proj}, norm3, mlp.fc1/fc2 (Out_Grid_Block.py:74-86)."""
    C = cfg["dim"]
    s = {}
    s.update(_ln(pre + "norm2.", C))
    s[pre + "grid_attn.mhsa.qkv.weight"], s[pre + "grid_attn.mhsa.qkv.bias"] = (3 * C, C), (3 * C,)
    s[pre + "grid_attn.mhsa.proj.weight"], s[pre + "grid_attn.mhsa.proj.bias"] = (C, C), (C,)
    s.update(_ln(pre + "norm3.", C))
    hid = max(1, int(C * cfg.get("mlp_ratio", 4.0)))
    s[pre + "mlp.fc1.weight"], s[pre + "mlp.fc1.bias"] = (hid, C), (hid,)
    s[pre + "mlp.fc2.weight"], s[pre + "mlp.fc2.bias"] = (C, hid), (C,)
    return s


def block_shapes(pre: str, cfg: dict) -> Dict[str, tuple]:
    """Parameter/buffer shapes of one OutGridBlock, keys as in the reference state_dict."""
    s = outlooker_shapes(pre + "outlook.", cfg)
    s.update(mbconv_shapes(pre + "mbconv.", cfg))
    s.update(grid_tail_shapes(pre, cfg))
    return s


def gridonly_block_shapes(pre: str, cfg: dict) -> Dict[str, tuple]:
    """GridOnlyBlock (Grid_Only_Block.py:21-59): mbconv, norm2, grid_attn, norm3, mlp."""
    s = mbconv_shapes(pre + "mbconv.", cfg)
    s.update(grid_tail_shapes(pre, cfg))
    return s


def stage_out_then_grid_shapes(pre: str, cfg: dict, depth: int, out_depth: int = 1) -> Dict[str, tuple]:
    """StageOutThenGrid (Grid_Only_Block.py:75-108): outlookers.<i>, blocks.<j>."""
    s = {}
    for i in range(out_depth):
        s.update(outlooker_shapes(f"{pre}outlookers.{i}.", cfg))
    for j in range(depth):
        s.update(gridonly_block_shapes(f"{pre}blocks.{j}.", cfg))
    return s


def model_b_shapes(stages: List[dict], num_classes=100, in_ch=3, stem_dim=64, front_depth=2) -> Dict[str, tuple]:
    """OutlookerFrontGridNet (Model_B_OutGridNet.py:10-82): stem, proj_in, front, stages, downs, head."""
    s = {"stem.stem.0.weight": (stem_dim, in_ch, 3, 3)}
    s.update(_bn("stem.stem.1.", stem_dim))
    if stem_dim != stages[0]["dim"]:
        s["proj_in.weight"], s["proj_in.bias"] = (stages[0]["dim"], stem_dim, 1, 1), (stages[0]["dim"],)
    for i in range(front_depth):
        s.update(outlooker_shapes(f"front.{i}.", stages[0]))
    for si, st in enumerate(stages):
        for b in range(st["depth"]):
            s.update(gridonly_block_shapes(f"stages.{si}.{b}.", st))
    for si in range(len(stages) - 1):
        s[f"downs.{si}.op.0.weight"] = (stages[si + 1]["dim"], stages[si]["dim"], 3, 3)
        s.update(_bn(f"downs.{si}.op.1.", stages[si + 1]["dim"]))
    s.update(_bn("head_norm.", stages[-1]["dim"]))
    s["classifier.weight"], s["classifier.bias"] = (num_classes, stages[-1]["dim"]), (num_classes,)
    return s


def model_a_shapes(stages: List[dict], num_classes=100, in_ch=3, stem_dim=64) -> Dict[str, tuple]:
    s = {"stem.stem.0.weight": (stem_dim, in_ch, 3, 3)}
    s.update(_bn("stem.stem.1.", stem_dim))
    if stem_dim != stages[0]["dim"]:
        s["proj_in.weight"], s["proj_in.bias"] = (stages[0]["dim"], stem_dim, 1, 1), (stages[0]["dim"],)
    for si, st in enumerate(stages):          # ModuleList `stages` is registered before `downs`
        for b in range(st["depth"]):
            s.update(block_shapes(f"stages.{si}.{b}.", st))
    for si in range(len(stages) - 1):
        s[f"downs.{si}.op.0.weight"] = (stages[si + 1]["dim"], stages[si]["dim"], 3, 3)
        s.update(_bn(f"downs.{si}.op.1.", stages[si + 1]["dim"]))
    s.update(_bn("head_norm.", stages[-1]["dim"]))
    s["classifier.weight"], s["classifier.bias"] = (num_classes, stages[-1]["dim"]), (num_classes,)
    return s


def make_params(shapes: Dict[str, tuple], value_fn, requires_grad=True) -> P:
    """value_fn(key, shape) -> numpy array.  Float params become leaf tensors."""
    out = {}
    for k, shp in shapes.items():
        t = torch.from_numpy(value_fn(k, shp))
        if t.is_floating_point() and not k.endswith(("running_mean", "running_var")) and requires_grad:
            t.requires_grad_(True)
        out[k] = t
    return out


# ---------------------------------------------------------------------------- building blocks
def _act(name: str, x):
    return {"gelu": F.gelu, "silu": F.silu, "relu": F.relu}[name](x)


def _bn_apply(x, p, pre, train):
    return F.batch_norm(x, p[pre + "running_mean"], p[pre + "running_var"], p[pre + "weight"], p[pre + "bias"],
                        training=train, momentum=0.1, eps=1e-5)


def ln2d(x, w, b, eps=1e-6):
    C = x.shape[1]
    y = F.layer_norm(x.permute(0, 2, 3, 1).contiguous(), (C,), w, b, eps)
    return y.permute(0, 3, 1, 2).contiguous()


def outlook_attention(x, p: P, pre: str, heads: int, k: int = 3, stride: int = 1):
    """outlook_attention.py:91-124 (stride > 1: logits average-pooled by the stride, strided unfold,
    output at H/s x W/s)."""
    B, C, H, W = x.shape
    kk, hd = k * k, C // heads
    logits = F.conv2d(x, p[pre + "attn.weight"], p.get(pre + "attn.bias"))
    if stride > 1:
        logits = F.avg_pool2d(logits, kernel_size=stride, stride=stride)
    Hs, Ws = logits.shape[-2:]
    L = Hs * Ws
    prob = logits.reshape(B, heads, kk, L).permute(0, 3, 1, 2).contiguous().softmax(dim=-1)   # [B,L,h,kk]
    v = F.conv2d(x, p[pre + "v.weight"], p.get(pre + "v.bias"))
    cols = F.unfold(v, kernel_size=k, padding=k // 2, stride=stride)                        # [B,C*kk,L]
    cols = cols.view(B, heads, hd, kk, L).permute(0, 4, 1, 2, 3).contiguous()                # [B,L,h,hd,kk]
    y = (cols * prob.unsqueeze(3)).sum(dim=-1)                                               # [B,L,h,hd]
    y = y.permute(0, 2, 3, 1).contiguous().view(B, C, Hs, Ws)
    return F.conv2d(y, p[pre + "proj.weight"], p[pre + "proj.bias"])


def mlp2d(x, p, pre, act="gelu"):
    return F.conv2d(_act(act, F.conv2d(x, p[pre + "fc1.weight"], p[pre + "fc1.bias"])), p[pre + "fc2.weight"],
                    p[pre + "fc2.bias"])


def outlooker_block(x, p, pre, heads, k=3, act="gelu", eps=1e-6):
    x = x + outlook_attention(ln2d(x, p[pre + "norm1.ln.weight"], p[pre + "norm1.ln.bias"], eps), p,
                              pre + "attn.", heads, k)
    return x + mlp2d(ln2d(x, p[pre + "norm2.ln.weight"], p[pre + "norm2.ln.bias"], eps), p, pre + "mlp.", act)


def mbconv(x, p, pre, train, act="silu"):
    h = x
    if pre + "expand.0.weight" in p:
        h = F.conv2d(h, p[pre + "expand.0.weight"], p.get(pre + "expand.0.bias"))
        if pre + "expand.1.weight" in p:
            h = _bn_apply(h, p, pre + "expand.1.", train)
        h = _act(act, h)
    mid = h.shape[1]
    h = F.conv2d(h, p[pre + "depthwise.0.weight"], p.get(pre + "depthwise.0.bias"), padding=1, groups=mid)
    if pre + "depthwise.1.weight" in p:
        h = _bn_apply(h, p, pre + "depthwise.1.", train)
    h = _act(act, h)
    if pre + "se.fc1.weight" in p:
        s = h.mean(dim=(2, 3), keepdim=True)
        s = _act(act, F.conv2d(s, p[pre + "se.fc1.weight"], p[pre + "se.fc1.bias"]))
        s = torch.sigmoid(F.conv2d(s, p[pre + "se.fc2.weight"], p[pre + "se.fc2.bias"]))
        h = h * s
    h = F.conv2d(h, p[pre + "project.0.weight"], p.get(pre + "project.0.bias"))
    if pre + "project.1.weight" in p:
        h = _bn_apply(h, p, pre + "project.1.", train)
    return x + h if h.shape == x.shape else h


def grid_partition(x, g):
    B, H, W, C = x.shape
    return x.view(B, H // g, g, W // g, g, C).permute(0, 2, 4, 1, 3, 5).contiguous().view(B * g * g, H // g, W // g, C)


def grid_unpartition(t, B, H, W, g):
    C = t.shape[-1]
    return t.view(B, g, g, H // g, W // g, C).permute(0, 3, 1, 4, 2, 5).contiguous().view(B, H, W, C)


def mhsa(tokens, p, pre, heads, want_probs=False):
    Bg, N, C = tokens.shape
    hd = C // heads
    qkv = F.linear(tokens, p[pre + "qkv.weight"], p.get(pre + "qkv.bias"))
    q, k, v = qkv.reshape(Bg, N, 3, heads, hd).permute(2, 0, 3, 1, 4)
    att = ((q @ k.transpose(-2, -1)) * (hd ** -0.5)).softmax(dim=-1)
    o = (att @ v).transpose(1, 2).reshape(Bg, N, C)
    o = F.linear(o, p[pre + "proj.weight"], p[pre + "proj.bias"])
    return (o, att) if want_probs else o


def grid_attention(x, p, pre, heads, g, want_probs=False):
    B, H, W, C = x.shape
    t = grid_partition(x, g)
    out = mhsa(t.view(t.shape[0], -1, C), p, pre + "mhsa.", heads, want_probs)
    o, att = out if want_probs else (out, None)
    y = grid_unpartition(o.view(t.shape), B, H, W, g)
    return (y, att) if want_probs else y


def grid_tail(x, p, pre, cfg):
    """permute -> x + Grid(LN(x)) -> x + MLP(LN(x)) -> permute (Out_Grid_Block.py:96-107,
    Grid_Only_Block.py:47-59)."""
    xb = x.permute(0, 2, 3, 1).contiguous()
    C = xb.shape[-1]
    y = F.layer_norm(xb, (C,), p[pre + "norm2.weight"], p[pre + "norm2.bias"], 1e-5)
    xb = xb + grid_attention(y, p, pre + "grid_attn.", cfg["num_heads"], cfg["grid_size"])
    y = F.layer_norm(xb, (C,), p[pre + "norm3.weight"], p[pre + "norm3.bias"], 1e-5)
    y = F.linear(_act(cfg.get("mlp_act", "gelu"), F.linear(y, p[pre + "mlp.fc1.weight"], p[pre + "mlp.fc1.bias"])),
                 p[pre + "mlp.fc2.weight"], p[pre + "mlp.fc2.bias"])
    return (xb + y).permute(0, 3, 1, 2).contiguous()


def outgrid_block(x, p, pre, cfg, train=False):
    x = outlooker_block(x, p, pre + "outlook.", cfg.get("outlook_heads", 6), cfg.get("outlook_kernel", 3),
                        cfg.get("mlp_act", "gelu"))
    x = mbconv(x, p, pre + "mbconv.", train, cfg.get("mbconv_act", "silu"))
    return grid_tail(x, p, pre, cfg)


def gridonly_block(x, p, pre, cfg, train=False):
    """GridOnlyBlock.forward (Grid_Only_Block.py:47-59): MBConv -> grid tail."""
    return grid_tail(mbconv(x, p, pre + "mbconv.", train, cfg.get("mbconv_act", "silu")), p, pre, cfg)


def stage_out_then_grid(x, p, pre, cfg, depth, out_depth=1, train=False):
    """StageOutThenGrid.forward (Grid_Only_Block.py:103-108)."""
    for i in range(out_depth):
        x = outlooker_block(x, p, f"{pre}outlookers.{i}.", cfg.get("outlook_heads", 6),
                            cfg.get("outlook_kernel", 3), cfg.get("mlp_act", "gelu"))
    for j in range(depth):
        x = gridonly_block(x, p, f"{pre}blocks.{j}.", cfg, train)
    return x


def model_b(x, p, stages, front_depth=2, train=False):
    """OutlookerFrontGridNet.forward (Model_B_OutGridNet.py:84-104)."""
    h = F.conv2d(x, p["stem.stem.0.weight"], None, padding=1)
    h = F.silu(_bn_apply(h, p, "stem.stem.1.", train))
    if "proj_in.weight" in p:
        h = F.conv2d(h, p["proj_in.weight"], p["proj_in.bias"])
    s0 = stages[0]
    for i in range(front_depth):
        h = outlooker_block(h, p, f"front.{i}.", s0.get("outlook_heads", 6), s0.get("outlook_kernel", 3),
                            s0.get("mlp_act", "gelu"))
    for si, st in enumerate(stages):
        for b in range(st["depth"]):
            h = gridonly_block(h, p, f"stages.{si}.{b}.", st, train)
        if si + 1 < len(stages):
            h = F.conv2d(h, p[f"downs.{si}.op.0.weight"], None, stride=2, padding=1)
            h = F.silu(_bn_apply(h, p, f"downs.{si}.op.1.", train))
    h = _bn_apply(h, p, "head_norm.", train).mean(dim=(2, 3))
    return F.linear(h, p["classifier.weight"], p["classifier.bias"])


def model_a(x, p, stages, train=False):
    h = F.conv2d(x, p["stem.stem.0.weight"], None, padding=1)
    h = F.silu(_bn_apply(h, p, "stem.stem.1.", train))
    if "proj_in.weight" in p:
        h = F.conv2d(h, p["proj_in.weight"], p["proj_in.bias"])
    for si, st in enumerate(stages):
        for b in range(st["depth"]):
            h = outgrid_block(h, p, f"stages.{si}.{b}.", st, train)
        if si + 1 < len(stages):
            h = F.conv2d(h, p[f"downs.{si}.op.0.weight"], None, stride=2, padding=1)
            h = F.silu(_bn_apply(h, p, f"downs.{si}.op.1.", train))
    h = _bn_apply(h, p, "head_norm.", train).mean(dim=(2, 3))
    return F.linear(h, p["classifier.weight"], p["classifier.bias"])


# ---------------------------------------------------------------------------- CPU training step
def no_decay(name: str) -> bool:
    """build_param_groups_no_wd's rule (src/training/warmup.py:4-26)."""
    n = name.lower()
    return name.endswith(".bias") or any(t in n for t in ("norm", "bn", "ln", "pos", "cls_token"))


def make_optimizer(p: P, lr=5e-4, weight_decay=0.05):
    names = [k for k, t in p.items() if t.requires_grad]
    dec = [p[k] for k in names if not no_decay(k)]
    nod = [p[k] for k in names if no_decay(k)]
    return torch.optim.AdamW([{"params": dec, "weight_decay": weight_decay}, {"params": nod, "weight_decay": 0.0}],
                             lr=lr)


def train_step(x, y, p, stages, opt, clip=1.0, label_smoothing=0.1):
    """fwd + CE(label smoothing) + bwd + clip_grad_norm + AdamW: the measured loop of
    src/training/one_epoch_train.py:85-131 without the host-side metrics."""
    opt.zero_grad(set_to_none=True)
    logits = model_a(x, p, stages, train=True)
    loss = F.cross_entropy(logits.float(), y, label_smoothing=label_smoothing)
    loss.backward()
    params = [t for t in p.values() if t.requires_grad]
    torch.nn.utils.clip_grad_norm_(params, clip)
    opt.step()
    return loss.detach()


def lr_at(t: int, base: float, warmup_steps: int, total_steps: int, min_lr: float) -> float:
    """WarmupCosineLR.step's lr for step count t (src/training/warmup.py:38-52)."""
    if warmup_steps > 0 and t <= warmup_steps:
        return base * (t / warmup_steps)
    prog = (min(t, total_steps) - warmup_steps) / max(1, total_steps - warmup_steps)
    return min_lr + (base - min_lr) * 0.5 * (1.0 + math.cos(math.pi * prog))


def train_steps(batches, p, stages, lr=5e-4, weight_decay=0.05, clip=1.0, label_smoothing=0.1, total_steps=8,
                warmup_steps=2, min_lr=0.0, on_step=None, autocast=False):
    """The reference's training loop over ``batches`` (src/training/one_epoch_train.py:85-153 with the
    optimizer / schedule of train_full_model.py:56-66 and warmup.py:29-59): zero_grad, forward, CE with
    label smoothing; a non-finite loss skips the step (no update, no scheduler.step -- :98-108); else
    backward, clip_grad_norm_, AdamW.step, scheduler.step.  The first step runs at the base lr (the
    schedule only writes the lr after a step).  on_step(t, loss, lr_used, skipped, step_num) per batch.
    autocast=True runs the forward under CPU bf16 autocast as use_amp=True does (one_epoch_train.py:88-90,
    autocast.py:71-78); the loss stays fp32 on logits.float() (:92-96)."""
    opt = make_optimizer(p, lr, weight_decay)
    step_num = 0
    for t, (x, y) in enumerate(batches):
        lr_used = [float(g["lr"]) for g in opt.param_groups]
        opt.zero_grad(set_to_none=True)
        with torch.autocast("cpu", dtype=torch.bfloat16, enabled=autocast):
            logits = model_a(x, p, stages, train=True)
        loss = F.cross_entropy(logits.float(), y, label_smoothing=label_smoothing)
        skipped = not bool(torch.isfinite(loss))
        if not skipped:
            loss.backward()
            torch.nn.utils.clip_grad_norm_([q for q in p.values() if q.requires_grad], clip)
            opt.step()
            step_num += 1
            for g in opt.param_groups:
                g["lr"] = lr_at(step_num, lr, warmup_steps, total_steps, min_lr)
        if on_step is not None:
            on_step(t, loss.detach(), lr_used, skipped, step_num)
    return opt


# ---------------------------------------------------------------------------- kernel-level oracles
def outlook_aggregate(v, logits, heads: int, k: int):
    """softmax over k*k + unfold-gather only (outlook_attention.py:106-120), NCHW in/out."""
    B, C, H, W = v.shape
    kk, hd, L = k * k, C // heads, H * W
    prob = logits.reshape(B, heads, kk, L).permute(0, 3, 1, 2).softmax(dim=-1)
    cols = F.unfold(v, kernel_size=k, padding=k // 2).view(B, heads, hd, kk, L).permute(0, 4, 1, 2, 3)
    y = (cols * prob.unsqueeze(3)).sum(dim=-1)
    return y.permute(0, 2, 3, 1).reshape(B, C, H, W)


def grid_core(qkv, heads: int, g: int, want_probs=False):
    """q@k^T*scale, softmax, @v inside strided grid groups (grid_attention.py:70-86 with the
    partition of grid_partition.py:13-15); qkv BHWC [B,H,W,3C] -> out BHWC [B,H,W,C]."""
    B, H, W, C3 = qkv.shape
    C = C3 // 3
    hd = C // heads
    t = grid_partition(qkv, g)
    Bg, N = t.shape[0], t.shape[1] * t.shape[2]
    q, k, v = t.reshape(Bg, N, 3, heads, hd).permute(2, 0, 3, 1, 4)
    att = ((q @ k.transpose(-2, -1)) * (hd ** -0.5)).softmax(dim=-1)
    o = (att @ v).transpose(1, 2).reshape(Bg, H // g, W // g, C)
    y = grid_unpartition(o, B, H, W, g)
    return (y, att) if want_probs else y


# ---------------------------------------------------------------------------- batch mixing
def mix_apply(images, targets, num_classes, mix, cutmix=False, perm=None, lam=1.0, box=(0, 0, 0, 0)):
    """apply_mixup_cutmix's tensor work once its random draws are known (cutmix_mixup_aug.py:36-64;
    the no-mix returns :30-34).  box = (y1, y2, x1, x2)."""
    y1h = F.one_hot(targets, num_classes=num_classes).float()
    if not mix:
        return images, y1h
    y2h = F.one_hot(targets[perm], num_classes=num_classes).float()
    if cutmix:
        yb1, yb2, xb1, xb2 = box
        out = images.clone()
        out[:, :, yb1:yb2, xb1:xb2] = images[perm, :, yb1:yb2, xb1:xb2]
    else:
        out = images * lam + images[perm] * (1.0 - lam)
    return out, y1h * lam + y2h * (1.0 - lam)
