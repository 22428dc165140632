"""Parameter-compatible replacements for the dense layers of the hot path.

They subclass the stock modules (so state_dict keys/shapes, isinstance checks and forward hooks
are exactly those of the reference) and override ``forward`` to run the MFMA GEMM / LayerNorm
kernels on channels-last rows.  Extra keyword arguments carry the fusions the blocks ask for:
``residual`` (+ ``row_scale`` for DropPath) in the epilogue and ``act_in`` in the prologue.
"""
from __future__ import annotations

import torch
import torch.nn as nn

from . import functional as OF


def act_name(mod: nn.Module):
    """Map an activation module to the kernels' prologue/epilogue activation."""
    if isinstance(mod, nn.GELU):
        if getattr(mod, "approximate", "none") != "none":
            return None
        return "gelu"
    if isinstance(mod, nn.SiLU):
        return "silu"
    if isinstance(mod, nn.ReLU):
        return "relu"
    return None


class Conv1x1(nn.Conv2d):
    """nn.Conv2d(in, out, kernel_size=1) on NCHW tensors, computed as a GEMM over B*H*W rows.
    The output is a channels_last NCHW tensor (physically [B*H*W, out])."""

    def __init__(self, in_channels: int, out_channels: int, bias: bool = True):
        super().__init__(in_channels, out_channels, kernel_size=1, bias=bias)

    def forward(self, x, residual=None, row_scale=None, act_in=None, x_act=None, emit_act=None, then_norm=None):
        """emit_act: return (y, emit_act(y)) from one launch (bf16); x_act: act_in(x) as emitted by
        the previous layer (the product and the weight gradient read it, x feeds act'(x)).
        then_norm: the residual stream's next LayerNorm2d -- returns (then_norm(y), y as the residual), the
        normalisation in this GEMM's epilogue where it can run there (OF.linear_rows_ln)."""
        B, C, H, W = x.shape
        dt = OF.compute_dtype(x)
        x2d = OF.nchw_to_rows(x.to(dt))
        if emit_act is not None:
            y, a = OF.linear_rows_act(x2d, self.weight, self.bias, emit_act)
            return OF.rows_to_nchw(y, B, H, W), OF.rows_to_nchw(a, B, H, W)
        r2d = OF.nchw_to_rows(residual.to(dt)) if residual is not None else None
        if then_norm is not None:
            lnp = OF.ln_epilogue_params(then_norm, self) if act_in is None and x_act is None else None
            if lnp is not None:
                yn, y = OF.linear_rows_ln(x2d, self.weight, self.bias, r2d, row_scale, H * W, *lnp)
                return OF.rows_to_nchw(yn, B, H, W), OF.rows_to_nchw(y, B, H, W)
            return then_norm.forward_pair(self(x, residual, row_scale, act_in, x_act))
        xa2d = OF.nchw_to_rows(x_act) if x_act is not None else None
        y = OF.linear_rows(x2d, self.weight, self.bias, r2d, row_scale, H * W, act_in, xa2d)
        return OF.rows_to_nchw(y, B, H, W)


class DepthwiseConv3x3(nn.Conv2d):
    """nn.Conv2d(C, C, 3, stride, padding=1, groups=C) on the ogv depthwise kernels (NHWC)."""

    def __init__(self, channels: int, stride: int = 1, bias: bool = True):
        super().__init__(channels, channels, kernel_size=3, stride=stride, padding=1, groups=channels, bias=bias)

    def forward(self, x):
        return OF.dwconv3x3_nchw(x.to(OF.compute_dtype(x)), self.weight, self.bias, self.stride[0])


class Linear(nn.Linear):
    """nn.Linear over the last dim of a contiguous [..., in] tensor (BHWC or [B, N, C]).
    ``rps`` = rows per sample for the DropPath row scale."""

    def forward(self, x, residual=None, row_scale=None, rps=None, act_in=None, x_act=None, emit_act=None,
                then_norm=None):
        """emit_act / x_act / then_norm: as Conv1x1.forward (then_norm: the next ogv LayerNorm)."""
        lead = x.shape[:-1]
        dt = OF.compute_dtype(x)
        x2d = x.to(dt).reshape(-1, x.shape[-1])
        if emit_act is not None:
            y, a = OF.linear_rows_act(x2d, self.weight, self.bias, emit_act)
            return y.view(*lead, self.out_features), a.view(*lead, self.out_features)
        r2d = residual.to(dt).reshape(-1, self.out_features) if residual is not None else None
        if rps is None:
            rps = max(1, x2d.shape[0] // max(1, lead[0] if len(lead) else 1))
        if then_norm is not None:
            lnp = OF.ln_epilogue_params(then_norm, self) if act_in is None and x_act is None else None
            if lnp is not None:
                yn, y = OF.linear_rows_ln(x2d, self.weight, self.bias, r2d, row_scale, rps, *lnp)
                return yn.view(*lead, self.out_features), y.view(*lead, self.out_features)
            return then_norm.forward_pair(self(x, residual, row_scale, rps, act_in, x_act))
        xa2d = x_act.reshape(-1, x.shape[-1]) if x_act is not None else None
        y = OF.linear_rows(x2d, self.weight, self.bias, r2d, row_scale, rps, act_in, xa2d)
        return y.view(*lead, self.out_features)


class LayerNorm(nn.LayerNorm):
    """nn.LayerNorm over the last dim (normalized_shape must be 1-D)."""

    def forward(self, x):
        if len(self.normalized_shape) != 1:
            raise NotImplementedError("ogv LayerNorm supports a 1-D normalized_shape")
        dt = OF.compute_dtype(x)
        x2d = x.to(dt).reshape(-1, x.shape[-1])
        y = OF.layer_norm_rows(x2d, self.weight, self.bias, self.eps)
        return y.view(x.shape)

    def forward_pair(self, x):
        """(LN(x), x as the residual) with the residual's gradient summed in the LN backward.
        Falls back to (self(x), x) when hooks are registered on this module."""
        if (self._forward_hooks or self._forward_pre_hooks or not torch.is_grad_enabled()
                or len(self.normalized_shape) != 1):
            return self(x), x
        x2d = x.to(OF.compute_dtype(x)).reshape(-1, x.shape[-1])
        y, r = OF.layer_norm_rows_pair(x2d, self.weight, self.bias, self.eps)
        return y.view(x.shape), r.view(x.shape)


class BatchNorm2d(nn.BatchNorm2d):
    """nn.BatchNorm2d on the native BN kernels (NHWC rows; train batch statistics with the
    running-stat update, or eval running statistics).  Same parameters/buffers as the stock module."""

    def forward(self, x):
        return OF.batchnorm_act_nchw(x, self, None)


def drop_path_scale(dp: nn.Module, x: torch.Tensor):
    """Per-sample DropPath factor mask/keep as an fp32 [B] tensor, or None when the module is an
    identity (eval, p == 0, nn.Identity).  Same Bernoulli(keep) draw as the reference
    DropPath (src/model/Outlook_Block.py:15-22), applied inside the GEMM epilogue."""
    p = float(getattr(dp, "drop_prob", 0.0))
    if p <= 0.0 or not dp.training:
        return None
    pre = getattr(dp, "_ogv_scale", None)  # drawn for the whole forward by draw_drop_path_scales
    if pre is not None and pre.shape[0] == x.shape[0]:
        dp._ogv_scale = None
        return pre
    keep = 1.0 - p
    mask = torch.empty((x.shape[0],), device=x.device, dtype=torch.float32).bernoulli_(keep)
    return mask / keep


_KEEP_CACHE = {}


def draw_drop_path_scales(modules, batch: int, device) -> None:
    """One draw for every live DropPath of a forward pass: row i of (floor(U + keep_i) / keep_i),
    U ~ Uniform[0,1)^(n x B), is module i's per-sample factor — the same Bernoulli(keep) / keep law
    as each module drawing its own mask (src/model/Outlook_Block.py:15-22), in four launches per
    step instead of two per module.  Each row is consumed by that module's next drop_path_scale."""
    live = [m for m in modules if float(getattr(m, "drop_prob", 0.0)) > 0.0 and m.training]
    if len(live) < 2:
        return
    key = (str(device), tuple(float(m.drop_prob) for m in live))
    keep = _KEEP_CACHE.get(key)
    if keep is None:  # built on the first (eager) step, reused inside captured graphs
        keep = _KEEP_CACHE[key] = torch.tensor([[1.0 - p] for p in key[1]], dtype=torch.float32, device=device)
    u = torch.rand((len(live), batch), dtype=torch.float32, device=device)
    scales = u.add_(keep).floor_().div_(keep)
    for i, m in enumerate(live):
        m._ogv_scale = scales[i]
