"""Model B (OutlookerFrontGridNet): stem -> Outlooker front (L blocks) -> [GridOnlyBlock x depth
(+ Downsample)] per stage -> BN/GAP/Linear.

Drop-in for src/Model_B_OutGridNet.py:10-104 — the same constructor, module names (stem, proj_in,
front.<i>, stages.<s>.<b>, downs.<s>, head_norm, classifier), state_dict and drop-path schedule
(front blocks first, then the stage blocks, :37-72).  Every block runs on the HIP kernels of
Model A (src/model/Grid_Only_Block.py, src/model/Outlook_Block.py).
"""
from dataclasses import dataclass  # noqa: F401  (the reference module exports these names)
from typing import List

import torch.nn as nn

from src.model.stem_head import *  # noqa: F401,F403
from src.model.Grid_Only_Block import *  # noqa: F401,F403
from src.model.downsampling import *  # noqa: F401,F403
from src.stage_config import *  # noqa: F401,F403
from src.model.Grid_Only_Block import GridOnlyBlock, OutlookerBlock2d
from src.model.downsampling import Downsample, DownsampleConfig
from src.model.stem_head import ConvStem, make_dpr
from src.stage_config import StageCfg
from src.Model_A_OutGridNet import classifier_head, train_prologue
from ogv.layers import BatchNorm2d, Conv1x1


class OutlookerFrontGridNet(nn.Module):
    def __init__(self, num_classes: int, stages: List[StageCfg], in_ch: int = 3, stem_dim: int = 64,
                 outlooker_front_depth: int = 2, dpr_max: float = 0.1,
                 down_cfg: DownsampleConfig = DownsampleConfig(kind="conv", act="silu", use_bn=True)):
        super().__init__()
        assert len(stages) >= 1
        self.stem = ConvStem(in_ch, stem_dim, act="silu", use_bn=True)
        self.proj_in = Conv1x1(stem_dim, stages[0].dim, bias=True) if stem_dim != stages[0].dim else nn.Identity()
        rates = iter(make_dpr(outlooker_front_depth + sum(s.depth for s in stages), dpr_max))
        c = stages[0]
        self.front = nn.ModuleList(
            OutlookerBlock2d(dim=c.dim, num_heads=c.outlook_heads, kernel_size=c.outlook_kernel, stride=1,
                             mlp_ratio=c.outlook_mlp_ratio, attn_drop=c.attn_drop, proj_drop=c.proj_drop,
                             mlp_drop=c.ffn_drop, drop_path=next(rates), act=c.mlp_act)
            for _ in range(outlooker_front_depth))
        self.stages = nn.ModuleList()
        self.downs = nn.ModuleList()
        for si, scfg in enumerate(stages):
            self.stages.append(nn.ModuleList(
                GridOnlyBlock(StageCfg(**{**scfg.__dict__, "drop_path": next(rates)})) for _ in range(scfg.depth)))
            if si < len(stages) - 1:
                self.downs.append(Downsample(scfg.dim, stages[si + 1].dim, cfg=down_cfg))
        self.head_norm = BatchNorm2d(stages[-1].dim)
        self.classifier = nn.Linear(stages[-1].dim, num_classes)

    def forward(self, x):
        train_prologue(self, x)
        x = self.proj_in(self.stem(x))
        for blk in self.front:
            x = blk(x)
        for si, blocks in enumerate(self.stages):
            for blk in blocks:
                x = blk(x)
            if si < len(self.downs):
                x = self.downs[si](x)
        return classifier_head(x, self.classifier, self.head_norm)
