"""Grid multi-head self-attention — drop-in for src/model/grid_attention.py.

  AttentionConfig / GridAttention2DConfig   :12-30
  MultiHeadSelfAttention                    :33-89   qkv / proj Linear -> MFMA GEMMs;
        reshape/permute + (q@k^T)*scale + softmax + @v (:70-86) -> ogv_grid_attn_{fwd,bwd}
        capture_attn (:77-83) -> the kernel also writes the softmax matrix (last_attn)
  GridAttention2D                           :93-131  partition/unpartition folded into the
        kernel's addressing; _last_meta / _last_grid_hw / _last_g kept for the analysis hooks
"""
from dataclasses import dataclass
from typing import Literal

import torch
import torch.nn as nn
import torch.nn.functional as F

from src.model.grid_partition import *  # noqa: F401,F403
from ogv import functional as OF
from ogv.layers import Linear

AttnMode = Literal["grid"]


@dataclass(frozen=True)
class AttentionConfig:
    dim: int
    num_heads: int
    qkv_bias: bool = True
    attn_drop: float = 0.0
    proj_drop: float = 0.0


@dataclass(frozen=True)
class GridAttention2DConfig:
    mode: AttnMode
    dim: int
    num_heads: int
    grid_size: int
    window_size: int = 1
    qkv_bias: bool = True
    attn_drop: float = 0.0
    proj_drop: float = 0.0


class MultiHeadSelfAttention(nn.Module):
    """MHSA over token sets: [B, N, C] -> [B, N, C] (grid groups are token sets too)."""

    def __init__(self, cfg: AttentionConfig):
        super().__init__()
        if cfg.dim <= 0:
            raise ValueError("cfg.dim must be > 0")
        if cfg.num_heads <= 0:
            raise ValueError("cfg.num_heads must be > 0")
        if cfg.dim % cfg.num_heads != 0:
            raise ValueError(f"dim ({cfg.dim}) must be divisible by num_heads ({cfg.num_heads})")
        self.dim = cfg.dim
        self.num_heads = cfg.num_heads
        self.head_dim = cfg.dim // cfg.num_heads
        self.scale = self.head_dim ** -0.5
        self.qkv = Linear(cfg.dim, 3 * cfg.dim, bias=cfg.qkv_bias)
        self.attn_drop = nn.Dropout(cfg.attn_drop)
        self.proj = Linear(cfg.dim, cfg.dim, bias=True)
        self.proj_drop = nn.Dropout(cfg.proj_drop)

    def _attend_dropout(self, qkv, B, H, W, g, capture):
        """Training with attn_drop > 0 (no reference config uses it): the probability matrix is
        materialised so Dropout can act on it -- grid_attention.py:70-86 in torch ops on the device
        (fp32), with the grid partition of grid_partition.py:13-15 as a view."""
        h, hd, N = self.num_heads, self.head_dim, (H // g) * (W // g)
        t = qkv.view(B, H // g, g, W // g, g, 3, h, hd).permute(5, 0, 2, 4, 6, 1, 3, 7).reshape(3, B * g * g, h, N, hd)
        q, k, v = t[0].float(), t[1].float(), t[2].float()
        attn = ((q @ k.transpose(-2, -1)) * self.scale).softmax(dim=-1)
        if capture:
            self.last_attn = attn.detach()
        attn = self.attn_drop(attn)
        if capture:
            self.last_attn_postdrop = attn.detach()
        out = (attn @ v).to(qkv.dtype)                                   # [B g g, h, N, hd]
        return out.view(B, g, g, h, H // g, W // g, hd).permute(0, 4, 1, 5, 2, 3, 6).reshape(B * H * W, self.dim)

    def attend_rows(self, x2d, B, H, W, g, residual=None, row_scale=None, then_norm=None):
        """Rows of a [B, H, W, C] image (or [B, 1, N, C] token set) -> attended rows (+ residual); with
        then_norm (the residual stream's next LayerNorm): (then_norm(rows), rows as the residual)."""
        capture = bool(getattr(self, "capture_attn", False))
        qkv = self.qkv(x2d, rps=H * W)
        if self.training and self.attn_drop.p > 0:
            out = self._attend_dropout(qkv, B, H, W, g, capture)
        else:
            out, probs = OF.grid_attention_rows(qkv, B, H, W, self.num_heads, g, self.scale, want_probs=capture)
            if capture:
                self.last_attn = probs.detach()
                self.last_attn_postdrop = self.last_attn
        if self.training and self.proj_drop.p > 0:
            y = self.proj_drop(self.proj(out, rps=H * W))
            if residual is not None:
                if row_scale is not None:
                    y = y * row_scale.repeat_interleave(H * W).view(-1, 1).to(y.dtype)
                y = residual + y
            return then_norm.forward_pair(y) if then_norm is not None else y
        return self.proj(out, residual=residual, row_scale=row_scale, rps=H * W, then_norm=then_norm)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        if x.ndim != 3:
            raise ValueError(f"Expected x.ndim==3 with shape [B, N, C]. Got {tuple(x.shape)}")
        B, N, C = x.shape
        if C != self.dim:
            raise ValueError(f"Expected last dim C={self.dim}. Got C={C}")
        x2d = x.to(OF.compute_dtype(x)).reshape(B * N, C)
        return self.attend_rows(x2d, B, 1, N, 1).view(B, N, C)


class GridAttention2D(nn.Module):
    """BHWC [B, H, W, C] -> [B, H, W, C] attention inside each strided grid group."""

    def __init__(self, cfg: GridAttention2DConfig):
        super().__init__()
        if cfg.mode != "grid":
            raise ValueError("This minimal version only supports mode='grid'")
        self.cfg = cfg
        self.mhsa = MultiHeadSelfAttention(AttentionConfig(dim=cfg.dim, num_heads=cfg.num_heads,
                                                           qkv_bias=cfg.qkv_bias, attn_drop=cfg.attn_drop,
                                                           proj_drop=cfg.proj_drop))

    def forward(self, x: torch.Tensor, residual=None, row_scale=None, then_norm=None):
        """then_norm: the residual stream's next LayerNorm -> (then_norm(out), out as the residual), BHWC."""
        if x.ndim != 4:
            raise ValueError(f"Expected x.ndim==4 (BHWC). Got {tuple(x.shape)}")
        B, H, W, C = x.shape
        if C != self.cfg.dim:
            raise ValueError(f"Expected C=={self.cfg.dim}. Got C={C}")
        g = self.cfg.grid_size
        if g <= 0:
            raise ValueError("grid_size must be > 0")
        if H % g or W % g:
            raise ValueError(f"H and W must be divisible by grid_size. Got H={H}, W={W}, g={g}")
        self._last_meta = (B, H, W, C, g)
        self._last_grid_hw = (H // g, W // g)
        self._last_g = g
        dt = OF.compute_dtype(x)
        x2d = x.to(dt).reshape(B * H * W, C)
        r2d = residual.to(dt).reshape(B * H * W, C) if residual is not None else None
        out = self.mhsa.attend_rows(x2d, B, H, W, g, residual=r2d, row_scale=row_scale, then_norm=then_norm)
        if then_norm is not None:
            return out[0].view(B, H, W, C), out[1].view(B, H, W, C)
        return out.view(B, H, W, C)


LocalAttention2D = GridAttention2D  # older name used by the reference notebooks
