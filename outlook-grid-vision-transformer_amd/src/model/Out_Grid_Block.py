"""OutGridBlock and the BHWC MLP — drop-in for src/model/Out_Grid_Block.py.

  MLP           :10-32   Linear C->4C, act, Linear 4C->C on BHWC (ValueError on a wrong last dim)
  OutGridBlock  :35-107  Outlooker -> MBConv -> x + DP(Grid(LN(x))) -> x + DP(MLP(LN(x)))
The NCHW<->BHWC permutes (:96, :107) are free views: activations stay channels_last from block
to block; residual adds and DropPath run in the GEMM epilogues.
"""
import torch
import torch.nn as nn
import torch.nn.functional as F

from src.model.Outlook_Block import *  # noqa: F401,F403
from src.model.grid_attention import *  # noqa: F401,F403
from src.model.mbc_conv import *  # noqa: F401,F403
from src.model.Outlook_Block import DropPath, OutlookerBlock2d
from src.model.outlook_attention import make_activation
from src.model.grid_attention import GridAttention2D, GridAttention2DConfig
from src.model.mbc_conv import MBConv, MBConvConfig
from ogv import functional as OF
from ogv.layers import LayerNorm, Linear, act_name, drop_path_scale


class MLP(nn.Module):
    """Token MLP over the last dim of a BHWC tensor."""

    def __init__(self, dim: int, mlp_ratio: float = 4.0, drop: float = 0.0, act: str = "gelu"):
        super().__init__()
        hidden = max(1, int(dim * mlp_ratio))
        self.fc1 = Linear(dim, hidden)
        self.act = make_activation(act)
        self.drop1 = nn.Dropout(drop)
        self.fc2 = Linear(hidden, dim)
        self.drop2 = nn.Dropout(drop)

    def forward(self, x: torch.Tensor, residual=None, row_scale=None) -> torch.Tensor:
        if x.shape[-1] != self.fc1.in_features:
            raise ValueError(f"MLP expected last dim={self.fc1.in_features}, got {x.shape[-1]}")
        rps = x[0].numel() // x.shape[-1] if x.ndim > 2 else 1
        a = act_name(self.act)
        if a is None or (self.training and (self.drop1.p > 0 or self.drop2.p > 0)):
            y = self.drop2(self.fc2(self.drop1(self.act(self.fc1(x)))))
            if residual is None:
                return y
            if row_scale is not None:
                y = y * row_scale.view(-1, *([1] * (y.ndim - 1))).to(y.dtype)
            return residual + y
        if OF.materialise_act(x, self.fc1, self.fc2):   # fc1 also writes act(fc1(x)): fc2 and its wgrad skip the prologue
            z, az = self.fc1(x, rps=rps, emit_act=a)
            return self.fc2(z, residual=residual, row_scale=row_scale, rps=rps, act_in=a, x_act=az)
        return self.fc2(self.fc1(x, rps=rps), residual=residual, row_scale=row_scale, rps=rps, act_in=a)


class OutGridBlock(nn.Module):
    """Hybrid block on [B, C, H, W]: local dynamic (Outlooker) -> MBConv -> grid MHSA -> MLP."""

    def __init__(self, cfg):
        super().__init__()
        C = cfg.dim
        self.outlook = OutlookerBlock2d(dim=C, num_heads=cfg.outlook_heads, kernel_size=cfg.outlook_kernel,
                                        stride=1, mlp_ratio=cfg.outlook_mlp_ratio, attn_drop=cfg.attn_drop,
                                        proj_drop=cfg.proj_drop, mlp_drop=cfg.ffn_drop, drop_path=cfg.drop_path,
                                        act=cfg.mlp_act)
        self.mbconv = MBConv(in_ch=C, out_ch=C, stride=1,
                             cfg=MBConvConfig(expand_ratio=cfg.mbconv_expand_ratio, se_ratio=cfg.mbconv_se_ratio,
                                              act=cfg.mbconv_act, use_bn=cfg.use_bn, drop_path=0.0))
        self.norm2 = LayerNorm(C)
        self.grid_attn = GridAttention2D(GridAttention2DConfig(mode="grid", dim=C, num_heads=cfg.num_heads,
                                                               window_size=cfg.window_size, grid_size=cfg.grid_size,
                                                               qkv_bias=True, attn_drop=cfg.attn_drop,
                                                               proj_drop=cfg.proj_drop))
        self.dp2 = DropPath(cfg.drop_path) if cfg.drop_path > 0 else nn.Identity()
        self.norm3 = LayerNorm(C)
        self.mlp = MLP(dim=C, mlp_ratio=cfg.mlp_ratio, drop=cfg.ffn_drop, act=cfg.mlp_act)
        self.dp3 = DropPath(cfg.drop_path) if cfg.drop_path > 0 else nn.Identity()

    def forward(self, x):
        return grid_tail(self, self.mbconv(self.outlook(x)))


def grid_tail(blk, x):
    """permute -> x + DP(Grid(LN(x))) -> x + DP(MLP(LN(x))) -> permute back, shared by OutGridBlock
    (Out_Grid_Block.py:96-107) and GridOnlyBlock (Grid_Only_Block.py:50-59).  `blk` holds norm2,
    grid_attn, dp2, norm3, mlp, dp3; the residual adds / DropPath run in the proj and fc2 epilogues."""
    xb = x.to(OF.compute_dtype(x)).permute(0, 2, 3, 1)            # BHWC view of channels_last
    if not xb.is_contiguous():
        xb = xb.contiguous()
    xn, xr = blk.norm2.forward_pair(xb)
    if blk.grid_attn._forward_hooks or blk.grid_attn._forward_pre_hooks:   # hooks see the reference's output
        xb = blk.grid_attn(xn, residual=xr, row_scale=drop_path_scale(blk.dp2, xb))
        xn, xr = blk.norm3.forward_pair(xb)
    else:   # the grid proj GEMM's epilogue also applies norm3 to the rows it stores (ogv_gemm_fwd_ln)
        xn, xr = blk.grid_attn(xn, residual=xr, row_scale=drop_path_scale(blk.dp2, xb), then_norm=blk.norm3)
    xb = blk.mlp(xn, residual=xr, row_scale=drop_path_scale(blk.dp3, xb))
    return xb.permute(0, 3, 1, 2)                                  # NCHW (channels_last) view
