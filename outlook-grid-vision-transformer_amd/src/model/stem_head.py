"""Stem conv and drop-path schedule — drop-in for src/model/stem_head.py (stock PyTorch-ROCm ops;
the 3x3 stem is outside the OutGridBlock hot path)."""
from dataclasses import dataclass
from typing import List
import torch.nn as nn


def _make_activation(act) -> nn.Module:
    from src.model.outlook_attention import make_activation
    return make_activation(act)


def make_dpr(total_blocks: int, dpr_max: float) -> List[float]:
    """Linear stochastic-depth ramp 0 .. dpr_max over the blocks (a single block gets dpr_max)."""
    if total_blocks <= 1:
        return [dpr_max]
    last = total_blocks - 1
    return [dpr_max * i / last for i in range(total_blocks)]


class ConvStem(nn.Module):
    def __init__(self, in_ch: int, out_ch: int, act: str = "silu", use_bn: bool = True):
        super().__init__()
        self.stem = nn.Sequential(
            nn.Conv2d(in_ch, out_ch, kernel_size=3, stride=1, padding=1, bias=not use_bn),
            nn.BatchNorm2d(out_ch) if use_bn else nn.Identity(),
            _make_activation(act),
        )

    def forward(self, x):
        return self.stem(x)
