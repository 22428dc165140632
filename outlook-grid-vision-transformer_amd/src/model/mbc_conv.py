"""MBConv with Squeeze-Excite — drop-in for src/model/mbc_conv.py.

  SqueezeExcite  :9-27   GAP -> 1x1 -> act -> 1x1 -> sigmoid gate (tiny [B, C, 1, 1] tensors)
  MBConvConfig   :32-38
  MBConv         :44-98  expand 1x1 (+BN+act) -> dw3x3 (+BN+act) -> SE -> project 1x1 (+BN) (+x)

Round-1 status: the two 1x1 convolutions (expand / project: the GEMM-shaped >90% of the FLOPs)
run on the ogv MFMA GEMM and the depthwise 3x3 on the ogv NHWC depthwise kernels; BatchNorm and
the SE gate still run on PyTorch-ROCm ops over channels_last tensors.  Fusing BN/SiLU/SE into the
kernels is SURVEY.md §8(f) rank 1 ("next").
"""
from typing import Literal
from dataclasses import dataclass
import torch
import torch.nn as nn
import torch.nn.functional as F

from src.model.Outlook_Block import *  # noqa: F401,F403
from src.model.Outlook_Block import DropPath
from src.model.outlook_attention import make_activation
from ogv import functional as OF
from ogv.layers import Conv1x1, DepthwiseConv3x3


class SqueezeExcite(nn.Module):
    def __init__(self, channels: int, se_ratio: float = 0.25, act: str = "silu"):
        super().__init__()
        if not (0.0 < se_ratio <= 1.0):
            raise ValueError("se_ratio must be in (0, 1].")
        squeezed = max(1, int(channels * se_ratio))
        self.pool = nn.AdaptiveAvgPool2d(1)
        self.fc1 = nn.Conv2d(channels, squeezed, kernel_size=1, bias=True)
        self.act = make_activation(act)
        self.fc2 = nn.Conv2d(squeezed, channels, kernel_size=1, bias=True)
        self.gate = nn.Sigmoid()

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        g = self.gate(self.fc2(self.act(self.fc1(self.pool(x)))))
        return x * g


ActType = Literal["silu", "gelu", "relu"]


@dataclass(frozen=True)
class MBConvConfig:
    expand_ratio: float = 4.0
    se_ratio: float = 0.25
    act: ActType = "silu"
    use_bn: bool = True
    drop_path: float = 0.0


class MBConv(nn.Module):
    """NCHW inverted bottleneck; residual when stride == 1 and in_ch == out_ch."""

    def __init__(self, in_ch: int, out_ch: int, stride: int = 1, cfg: MBConvConfig = MBConvConfig()):
        super().__init__()
        if in_ch <= 0 or out_ch <= 0:
            raise ValueError("in_ch and out_ch must be > 0")
        if stride not in (1, 2):
            raise ValueError("stride must be 1 or 2")
        self.in_ch, self.out_ch, self.stride = in_ch, out_ch, stride

        def norm(c):
            return nn.BatchNorm2d(c) if cfg.use_bn else nn.Identity()

        mid = max(1, int(round(in_ch * cfg.expand_ratio)))
        if mid != in_ch:
            self.expand = nn.Sequential(Conv1x1(in_ch, mid, bias=not cfg.use_bn), norm(mid),
                                        make_activation(cfg.act))
        else:
            self.expand = nn.Identity()
        self.depthwise = nn.Sequential(DepthwiseConv3x3(mid, stride=stride, bias=not cfg.use_bn),
                                       norm(mid), make_activation(cfg.act))
        self.se = SqueezeExcite(mid, se_ratio=cfg.se_ratio, act=cfg.act) if cfg.se_ratio > 0 else nn.Identity()
        self.project = nn.Sequential(Conv1x1(mid, out_ch, bias=not cfg.use_bn), norm(out_ch))
        self.use_res = stride == 1 and in_ch == out_ch
        self.drop_path = DropPath(cfg.drop_path) if (cfg.drop_path and cfg.drop_path > 0) else nn.Identity()

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        dt = OF.compute_dtype(x)
        x = x.to(dt)
        # the stock-op parts (BN, depthwise, SE) follow the activation dtype even outside autocast
        with torch.autocast("cuda", dtype=torch.bfloat16, enabled=(dt == torch.bfloat16 and x.is_cuda)):
            h = self.project(self.se(self.depthwise(self.expand(x))))
        return x + self.drop_path(h) if self.use_res else h
