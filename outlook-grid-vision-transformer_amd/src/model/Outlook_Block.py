"""DropPath and the Outlooker block — drop-in for src/model/Outlook_Block.py.

  DropPath          :7-22   per-sample stochastic depth (module kept for direct use; inside the
                            blocks the per-sample factor is fused into the GEMM epilogue)
  OutlookerBlock2d  :26-64  x + DP(OA(LN2d(x))); x + DP(MLP2d(LN2d(x)))  -> the residual adds and
                            DropPath scales run in the proj / fc2 GEMM epilogues
"""
import torch
import torch.nn as nn
import torch.nn.functional as F

from src.model.outlook_attention import *  # noqa: F401,F403  (reference re-exports these)
from src.model.outlook_attention import LayerNorm2d, MLP2d, OutlookAttention2d
from ogv import functional as OF
from ogv.layers import drop_path_scale


class DropPath(nn.Module):
    """Stochastic depth for any tensor with the batch in dim 0."""

    def __init__(self, drop_prob: float = 0.0):
        super().__init__()
        self.drop_prob = float(drop_prob)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        if self.drop_prob == 0.0 or not self.training:
            return x
        keep = 1.0 - self.drop_prob
        mask = torch.empty((x.shape[0],) + (1,) * (x.ndim - 1), device=x.device, dtype=x.dtype)
        return x * mask.bernoulli_(keep) / keep


class OutlookerBlock2d(nn.Module):
    """NCHW: LN2d -> OutlookAttention2d -> DropPath + residual; LN2d -> MLP2d -> DropPath + residual."""

    def __init__(self, dim: int, num_heads: int, kernel_size: int = 3, stride: int = 1,
                 mlp_ratio: float = 2.0, attn_drop: float = 0.0, proj_drop: float = 0.0,
                 drop_path: float = 0.0, mlp_drop: float = 0.0, act: str = "gelu", norm_eps: float = 1e-6):
        super().__init__()
        self.norm1 = LayerNorm2d(dim, eps=norm_eps)
        # qkv_bias is not forwarded by the reference either (:47-53) -> default True
        self.attn = OutlookAttention2d(dim=dim, num_heads=num_heads, kernel_size=kernel_size, stride=stride,
                                       attn_drop=attn_drop, proj_drop=proj_drop)
        self.dp1 = DropPath(drop_path) if drop_path > 0 else nn.Identity()
        self.norm2 = LayerNorm2d(dim, eps=norm_eps)
        self.mlp = MLP2d(dim=dim, mlp_ratio=mlp_ratio, drop=mlp_drop, act=act)
        self.dp2 = DropPath(drop_path) if drop_path > 0 else nn.Identity()

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        x = x.to(OF.compute_dtype(x))
        xn, xr = self.norm1.forward_pair(x)
        if self.attn._forward_hooks or self.attn._forward_pre_hooks:   # hooks see the reference's single output
            x = self.attn(xn, residual=xr, row_scale=drop_path_scale(self.dp1, x))
            xn, xr = self.norm2.forward_pair(x)
        else:   # the proj GEMM's epilogue also applies norm2 to the rows it stores (ogv_gemm_fwd_ln)
            xn, xr = self.attn(xn, residual=xr, row_scale=drop_path_scale(self.dp1, x), then_norm=self.norm2)
        x = self.mlp(xn, residual=xr, row_scale=drop_path_scale(self.dp2, x))
        return x

