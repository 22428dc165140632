"""Stem conv and drop-path schedule — drop-in for src/model/stem_head.py.

ConvStem keeps the reference's module tree (``stem.0`` Conv2d, ``stem.1`` BatchNorm2d, ``stem.2``
activation; same state_dict) and runs conv3x3 -> BN -> act as one native op
(ogv_convbn_fwd/bwd: implicit-GEMM conv on MFMA with the BN statistics in its epilogue)."""
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
        from ogv import functional as OF
        from ogv.layers import act_name
        conv, norm, act = self.stem[0], self.stem[1], self.stem[2]
        a = act_name(act)
        if a is None and not isinstance(act, nn.Identity):
            raise NotImplementedError(f"ogv ConvStem: unsupported activation {type(act).__name__}")
        return OF.conv3x3_bn_act(x, conv, norm if isinstance(norm, nn.BatchNorm2d) else None, a)
