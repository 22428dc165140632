"""Outlooker attention, channel LayerNorm and the 1x1-conv MLP — MI355X kernels.

Drop-in for src/model/outlook_attention.py of the reference:
  make_activation            :6-14     (same names / errors)
  LayerNorm2d                :17-31    (LN over C of NCHW; eps 1e-6) -> ogv_layernorm_* on rows
  MLP2d                      :33-49    (1x1 C->hidden, act, 1x1 hidden->C) -> two MFMA GEMMs,
                                        the activation applied in the second GEMM's prologue
  OutlookAttention2d         :52-124   logits/v/proj 1x1 convs -> MFMA GEMMs; softmax over k*k +
                                        unfold-gather (:100-120) -> ogv_outlook_agg_{fwd,bwd}.
                                        With no hooks on .attn / .v the two projections of the same
                                        input run as ONE GEMM over [Wv; Wattn; 0] (v and the logits
                                        are column ranges of its output, read in place by the
                                        LDS-tiled gather; the backward is one gradient buffer,
                                        one dgrad and one wgrad).  For inference (no gradient)
                                        the projections, softmax and gather run as ONE kernel
                                        (ogv_outlook_vproj_fwd: the v / logits tile lives in LDS;
                                        knob outlook_vproj=2 uses it in training too)
Parameters and their names/shapes are unchanged (attn.weight [heads*k*k, C, 1, 1], v.*, proj.*).
Tensors are NCHW logically and channels_last physically.
"""
import torch
import torch.nn as nn
import torch.nn.functional as F

from ogv import functional as OF
from ogv.layers import Conv1x1, act_name


def make_activation(act: str) -> nn.Module:
    name = act.lower()
    table = {"silu": lambda: nn.SiLU(inplace=True), "relu": lambda: nn.ReLU(inplace=True), "gelu": nn.GELU}
    if name not in table:
        raise ValueError(f"Unknown activation '{act}'. Use one of: silu|gelu|relu")
    return table[name]()


class LayerNorm2d(nn.Module):
    """LayerNorm across channels at every (h, w) of an NCHW tensor."""

    def __init__(self, num_channels: int, eps: float = 1e-6, affine: bool = True):
        super().__init__()
        self.ln = nn.LayerNorm(num_channels, eps=eps, elementwise_affine=affine)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        B, C, H, W = x.shape
        rows = OF.nchw_to_rows(x.to(OF.compute_dtype(x)))
        y = OF.layer_norm_rows(rows, self.ln.weight, self.ln.bias, self.ln.eps)
        return OF.rows_to_nchw(y, B, H, W)

    def forward_pair(self, x: torch.Tensor):
        """(LN2d(x), x as the residual) with the residual's gradient summed in the LN backward.
        Falls back to (self(x), x) when hooks are registered on this module."""
        if self._forward_hooks or self._forward_pre_hooks or not torch.is_grad_enabled():
            return self(x), x
        B, C, H, W = x.shape
        rows = OF.nchw_to_rows(x.to(OF.compute_dtype(x)))
        y, r = OF.layer_norm_rows_pair(rows, self.ln.weight, self.ln.bias, self.ln.eps)
        return OF.rows_to_nchw(y, B, H, W), OF.rows_to_nchw(r, B, H, W)


class MLP2d(nn.Module):
    """fc1 (1x1) -> act -> drop -> fc2 (1x1) -> drop.  fc1 stores the pre-activation; fc2 applies
    the activation while loading it and fuses the block's residual + DropPath into its epilogue."""

    def __init__(self, dim, mlp_ratio=4.0, drop=0.0, act="gelu"):
        super().__init__()
        hidden = max(1, int(dim * mlp_ratio))
        self.fc1 = Conv1x1(dim, hidden)
        self.act = make_activation(act)
        self.drop1 = nn.Dropout(drop)
        self.fc2 = Conv1x1(hidden, dim)
        self.drop2 = nn.Dropout(drop)

    def forward(self, x, residual=None, row_scale=None):
        a = act_name(self.act)
        dropping = self.training and (self.drop1.p > 0 or self.drop2.p > 0)
        if a is None or dropping:
            h = self.drop1(self.act(self.fc1(x)))
            y = self.drop2(self.fc2(h))
            if residual is None:
                return y
            if row_scale is not None:
                y = y * row_scale.view(-1, 1, 1, 1).to(y.dtype)
            return residual + y
        if OF.materialise_act(x, self.fc1, self.fc2):   # fc1 also writes act(fc1(x)): fc2 and its wgrad skip the prologue
            z, az = self.fc1(x, emit_act=a)
            return self.fc2(z, residual=residual, row_scale=row_scale, act_in=a, x_act=az)
        return self.fc2(self.fc1(x), residual=residual, row_scale=row_scale, act_in=a)


class OutlookAttention2d(nn.Module):
    """Dynamic local aggregation on NCHW: per pixel and head, a softmax over the k*k logits
    weights the zero-padded k*k neighbourhood of v (padded neighbours keep their mass)."""

    def __init__(self, dim: int, num_heads: int = 6, kernel_size: int = 3, stride: int = 1,
                 attn_drop: float = 0.0, proj_drop: float = 0.0, qkv_bias: bool = True):
        super().__init__()
        assert dim % num_heads == 0, "dim must be divisible by num_heads"
        if kernel_size <= 0 or kernel_size % 2 == 0:
            raise ValueError("kernel_size must be odd and >0 (e.g., 3,5,7)")
        if stride <= 0:
            raise ValueError("stride must be > 0")
        self.dim = dim
        self.num_heads = num_heads
        self.head_dim = dim // num_heads
        self.kernel_size = kernel_size
        self.stride = stride
        kk = kernel_size * kernel_size
        self.attn = Conv1x1(dim, num_heads * kk, bias=bool(qkv_bias))   # logits (hooks read this)
        self.v = Conv1x1(dim, dim, bias=bool(qkv_bias))
        self.attn_drop = nn.Dropout(attn_drop)
        self.proj = Conv1x1(dim, dim, bias=True)
        self.proj_drop = nn.Dropout(proj_drop)

    def _hooked(self) -> bool:
        return any(m._forward_hooks or m._forward_pre_hooks for m in (self.attn, self.v))

    def _cat_store(self, ld):
        """One fp32 [ld, C] weight buffer (+ [ld] bias buffer) whose row blocks ARE v.weight and
        attn.weight (v.bias, attn.bias): the parameters are re-pointed into it once (values copied,
        names / shapes / state_dict unchanged), so [Wv; Wattn; 0] needs no concatenation per
        forward.  Re-binds if the parameters were replaced since (e.g. .to(), assign-loading);
        None when the parameters are not fp32 device tensors (the copying path then runs)."""
        C, n = self.dim, self.attn.out_channels
        wv, wa, bv, ba = self.v.weight, self.attn.weight, self.v.bias, self.attn.bias
        if not wv.is_cuda or any(t is not None and t.dtype != torch.float32 for t in (wv, wa, bv, ba)):
            return None
        st = self.__dict__.get("_cat_buf")
        if st is not None:
            fw, fb = st
            base = fw.data_ptr()
            ok = (fw.device == wv.device and fw.shape[0] == ld and wv.data_ptr() == base and wv.is_contiguous()
                  and wa.data_ptr() == base + 4 * C * C and wa.is_contiguous()
                  and (fb is None) == (bv is None and ba is None))
            if ok and fb is not None:
                ok = ((bv is None or bv.data_ptr() == fb.data_ptr()) and (ba is None or ba.data_ptr() == fb.data_ptr() + 4 * C))
            if ok:
                return st
        with torch.no_grad():
            fw = torch.zeros(ld, C, device=wv.device)
            fw[:C].copy_(wv.reshape(C, C))
            fw[C:C + n].copy_(wa.reshape(n, C))
            wv.data = fw[:C].view(wv.shape)
            wa.data = fw[C:C + n].view(wa.shape)
            fb = None
            if bv is not None or ba is not None:
                fb = torch.zeros(ld, device=wv.device)
                if bv is not None:
                    fb[:C].copy_(bv)
                    bv.data = fb[:C]
                if ba is not None:
                    fb[C:C + n].copy_(ba)
                    ba.data = fb[C:C + n]
        self.__dict__["_cat_buf"] = (fw, fb)
        return fw, fb

    def _cat_params(self):
        """[Wv; Wattn; 0] ([ld, C], ld = C + heads*k*k rounded up to 8 so every row of the GEMM
        output is 16-B aligned) and the matching bias, differentiable w.r.t. both convs.  With the
        parameters living in one buffer (_cat_store) this is that buffer: no copy launch."""
        C, n = self.dim, self.attn.out_channels
        ld = (C + n + 7) // 8 * 8
        st = self._cat_store(ld)
        if st is not None:
            fw, fb = st
            w = OF.aliased_concat(fw, (0, C), self.v.weight, self.attn.weight)
            if fb is None:
                return w, None
            bs = [(o, t) for o, t in ((0, self.v.bias), (C, self.attn.bias)) if t is not None]
            return w, OF.aliased_concat(fb, [o for o, _ in bs], *[t for _, t in bs])
        wv, wa = self.v.weight.reshape(C, C), self.attn.weight.reshape(n, C)
        zw, zb = self._zero_pads(wv.device, ld - C - n)
        parts = [wv.float(), wa.float()] + ([zw] if ld > C + n else [])
        w = torch.cat(parts)
        if self.v.bias is None and self.attn.bias is None:
            return w, None
        bv = self.v.bias if self.v.bias is not None else wv.new_zeros(C)
        ba = self.attn.bias if self.attn.bias is not None else wa.new_zeros(n)
        bparts = [bv.float(), ba.float()] + ([zb] if ld > C + n else [])
        return w, torch.cat(bparts)

    def _forward_materialised(self, x):
        """stride > 1, or training with attn_drop > 0 (no reference config uses either): the softmax
        probabilities are materialised -- outlook_attention.py:100-120 in torch ops on the device
        (fp32) around the two 1x1 convs on the HIP GEMM: logits average-pooled by the stride, the
        unfold strided, Dropout on the probabilities.  Output [B, C, H/s, W/s]."""
        B, C, H, W = x.shape
        k, s, heads, hd = self.kernel_size, self.stride, self.num_heads, self.head_dim
        kk = k * k
        a = self.attn(x).float()
        if s > 1:
            a = F.avg_pool2d(a, kernel_size=s, stride=s)
        Hs, Ws = a.shape[-2:]
        a = a.reshape(B, heads, kk, Hs * Ws).permute(0, 3, 1, 2).softmax(dim=-1)
        a = self.attn_drop(a)                                                     # [B, L, heads, kk]
        v = self.v(x).float()
        v_unf = F.unfold(v, kernel_size=k, padding=k // 2, stride=s)
        v_unf = v_unf.view(B, heads, hd, kk, Hs * Ws).permute(0, 4, 1, 2, 3)
        y = (v_unf * a.unsqueeze(3)).sum(dim=-1)                                  # [B, L, heads, hd]
        y = y.permute(0, 2, 3, 1).reshape(B, C, Hs, Ws).to(OF.compute_dtype(x))
        return y.contiguous(memory_format=torch.channels_last)

    def _zero_pads(self, device, rows):
        """Zero rows of the concatenated weight / bias, allocated once per device (not parameters or
        buffers: the state_dict is unchanged) -- no fill launches per forward."""
        pads = self.__dict__.setdefault("_pads", {})
        z = pads.get(device)
        if z is None or z[0].shape[0] != rows:
            z = pads[device] = (torch.zeros(max(rows, 0), self.dim, device=device),
                                torch.zeros(max(rows, 0), device=device))
        return z

    def forward(self, x: torch.Tensor, residual=None, row_scale=None, then_norm=None):
        """then_norm: the residual stream's next LayerNorm2d -> (then_norm(out), out as the residual)."""
        B, C, H, W = x.shape
        if self.stride != 1 or (self.training and self.attn_drop.p > 0):
            y = self._forward_materialised(x)
        elif self._hooked():
            a = self.attn(x)                     # [B, heads*k*k, H, W]  (analysis hooks read this)
            v = self.v(x)                        # [B, C, H, W]
            y = OF.outlook_aggregate_rows(OF.nchw_to_rows(v), OF.nchw_to_rows(a), B, H, W,
                                          self.num_heads, self.kernel_size)
        else:
            dt = OF.compute_dtype(x)
            w, b = self._cat_params()
            xr = OF.nchw_to_rows(x.to(dt))
            train = torch.is_grad_enabled() and (x.requires_grad or w.requires_grad)
            if OF.outlook_vproj_supported(B, H, W, C, self.num_heads, self.kernel_size, w.shape[0], dt, train):
                # projections + softmax + gather in one kernel (the v / logits tile lives in LDS)
                y = OF.outlook_vproj(xr, w, b, C, B, H, W, self.num_heads, self.kernel_size)
            else:
                cat = OF.linear_rows(xr, w, b)     # [M, v | logits | 0]
                y = OF.outlook_aggregate_cat(cat, C, B, H, W, self.num_heads, self.kernel_size)
        if y.dim() == 2:
            y = OF.rows_to_nchw(y, B, H, W)
        if self.training and self.proj_drop.p > 0:
            y = self.proj_drop(self.proj(y))
            if residual is not None:
                if row_scale is not None:
                    y = y * row_scale.view(-1, 1, 1, 1).to(y.dtype)
                y = residual + y
            return then_norm.forward_pair(y) if then_norm is not None else y
        return self.proj(y, residual=residual, row_scale=row_scale, then_norm=then_norm)
