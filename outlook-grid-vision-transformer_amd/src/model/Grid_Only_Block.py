"""Grid-only blocks — drop-in for src/model/Grid_Only_Block.py.

  MaxOutStage       :11-19   depth x OutGridBlock
  GridOnlyBlock     :21-59   MBConv -> x + DP(Grid(LN(x))) -> x + DP(MLP(LN(x)))  (no Outlooker)
  StageOutThenGrid  :62-108  out_depth x OutlookerBlock2d, then depth x GridOnlyBlock
Same module names / state_dict keys as the reference; the math runs on the same HIP kernels as
OutGridBlock (fused MBConv, LN pair, grid attention, GEMM epilogues with residual + DropPath).
"""
import torch.nn as nn

from src.model.Outlook_Block import *  # noqa: F401,F403  (the reference star-imports these)
from src.model.grid_attention import *  # noqa: F401,F403
from src.model.mbc_conv import *  # noqa: F401,F403
from src.model.Out_Grid_Block import *  # noqa: F401,F403
from src.model.Outlook_Block import DropPath, OutlookerBlock2d
from src.model.grid_attention import GridAttention2D, GridAttention2DConfig
from src.model.mbc_conv import MBConv, MBConvConfig
from src.model.Out_Grid_Block import MLP, OutGridBlock, grid_tail
from ogv.layers import LayerNorm


class MaxOutStage(nn.Module):
    def __init__(self, block_cfg, depth: int):
        super().__init__()
        self.blocks = nn.ModuleList([OutGridBlock(block_cfg) for _ in range(depth)])

    def forward(self, x):
        for b in self.blocks:
            x = b(x)
        return x


class GridOnlyBlock(nn.Module):
    """MBConv -> grid MHSA -> MLP on [B, C, H, W] (no Outlooker)."""

    def __init__(self, cfg):
        super().__init__()
        C = cfg.dim
        self.mbconv = MBConv(in_ch=C, out_ch=C, stride=1,
                             cfg=MBConvConfig(expand_ratio=cfg.mbconv_expand_ratio, se_ratio=cfg.mbconv_se_ratio,
                                              act=cfg.mbconv_act, use_bn=cfg.use_bn, drop_path=0.0))
        self.norm2 = LayerNorm(C)
        # the reference reads window_size with a default of 1 here (:39)
        self.grid_attn = GridAttention2D(GridAttention2DConfig(mode="grid", dim=C, num_heads=cfg.num_heads,
                                                               window_size=getattr(cfg, "window_size", 1),
                                                               grid_size=cfg.grid_size, qkv_bias=True,
                                                               attn_drop=cfg.attn_drop, proj_drop=cfg.proj_drop))
        self.dp2 = DropPath(cfg.drop_path) if cfg.drop_path > 0 else nn.Identity()
        self.norm3 = LayerNorm(C)
        self.mlp = MLP(dim=C, mlp_ratio=cfg.mlp_ratio, drop=cfg.ffn_drop, act=cfg.mlp_act)
        self.dp3 = DropPath(cfg.drop_path) if cfg.drop_path > 0 else nn.Identity()

    def forward(self, x):
        return grid_tail(self, self.mbconv(x))


class StageOutThenGrid(nn.Module):
    """One (or out_depth) Outlooker block(s) at the start of the stage, then GridOnlyBlocks."""

    def __init__(self, cfg, depth: int, out_depth: int = 1):
        super().__init__()
        self.outlookers = nn.ModuleList([
            OutlookerBlock2d(dim=cfg.dim, num_heads=cfg.outlook_heads, kernel_size=cfg.outlook_kernel, stride=1,
                             mlp_ratio=cfg.outlook_mlp_ratio, attn_drop=cfg.attn_drop, proj_drop=cfg.proj_drop,
                             mlp_drop=cfg.ffn_drop, drop_path=cfg.drop_path, act=cfg.mlp_act)
            for _ in range(out_depth)])
        self.blocks = nn.ModuleList([GridOnlyBlock(cfg) for _ in range(depth)])

    def forward(self, x):
        for o in self.outlookers:
            x = o(x)
        for b in self.blocks:
            x = b(x)
        return x
