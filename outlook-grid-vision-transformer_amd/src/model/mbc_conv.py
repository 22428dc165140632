"""MBConv with Squeeze-Excite — drop-in for src/model/mbc_conv.py.

  SqueezeExcite  :9-27   GAP -> 1x1 -> act -> 1x1 -> sigmoid gate (tiny [B, C, 1, 1] tensors)
  MBConvConfig   :32-38
  MBConv         :44-98  expand 1x1 (+BN+act) -> dw3x3 (+BN+act) -> SE -> project 1x1 (+BN) (+x)

The OutGridBlock configuration (BN, expand, SE, stride 1, residual) runs as ONE fused HIP
forward and ONE hand-scheduled HIP backward (ogv_mbconv_fwd/bwd): BatchNorm statistics in the
GEMM / depthwise epilogues, BN-apply + activation (+ SE gate) in the consumers' prologues, the
SE and BN2 backward reductions in a single pass.  Other configurations (no BN, stride 2, active
DropPath, ...) run the same modules unfused (1x1 GEMMs and depthwise conv on the ogv kernels,
BN/SE on PyTorch-ROCm ops).
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
from ogv.layers import Conv1x1, DepthwiseConv3x3, act_name


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

    def _fusable(self):
        """The fused HIP path covers the OutGridBlock configuration: BN everywhere, a real expand,
        SE, stride 1, residual, no active DropPath, one BN eps/momentum."""
        if getattr(self, "ogv_unfused", False):
            return False
        if not (isinstance(self.expand, nn.Sequential) and isinstance(self.se, SqueezeExcite)):
            return False
        if self.stride != 1 or not self.use_res:
            return False
        bns = [self.expand[1], self.depthwise[1], self.project[1]]
        if not all(isinstance(b, nn.BatchNorm2d) and b.affine and b.track_running_stats and b.momentum is not None
                   for b in bns):
            return False
        if len({(b.eps, b.momentum) for b in bns}) != 1 or len({b.training for b in bns}) != 1:
            return False
        acts = {act_name(self.expand[2]), act_name(self.depthwise[2]), act_name(self.se.act)}
        if len(acts) != 1 or None in acts:
            return False
        dp = self.drop_path
        return not (isinstance(dp, DropPath) and dp.training and dp.drop_prob > 0)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        dt = OF.compute_dtype(x)
        x = x.to(dt)
        if x.is_cuda and self._fusable():
            B, C, H, W = x.shape
            e, bn1, dw, bn2, pj, bn3 = self.expand[0], self.expand[1], self.depthwise[0], self.depthwise[1], \
                self.project[0], self.project[1]
            params = [e.weight, bn1.weight, bn1.bias, dw.weight, bn2.weight, bn2.bias, self.se.fc1.weight,
                      self.se.fc1.bias, self.se.fc2.weight, self.se.fc2.bias, pj.weight, bn3.weight, bn3.bias]
            buffers = {"bn1_rm": bn1.running_mean, "bn1_rv": bn1.running_var, "bn2_rm": bn2.running_mean,
                       "bn2_rv": bn2.running_var, "bn3_rm": bn3.running_mean, "bn3_rv": bn3.running_var}
            train = bn1.training
            if train and not getattr(bn1, "_ogv_nbt_pooled", False):  # one multi-tensor launch
                torch._foreach_add_([bn1.num_batches_tracked, bn2.num_batches_tracked,
                                     bn3.num_batches_tracked], 1)
            return OF.mbconv_fused(x, B, H, W, e.out_channels, self.se.fc1.out_channels, train, bn1.eps,
                                   bn1.momentum, act_name(self.expand[2]), params, buffers)
        # the stock-op parts (BN, depthwise, SE) follow the activation dtype even outside autocast
        with torch.autocast("cuda", dtype=torch.bfloat16, enabled=(dt == torch.bfloat16 and x.is_cuda)):
            h = self.project(self.se(self.depthwise(self.expand(x))))
        bns = (self.expand[1], self.depthwise[1], self.project[1])
        if bns[0].training and getattr(bns[0], "_ogv_nbt_pooled", False):
            # stock BatchNorm2d counted itself; the model-level pooled add counted it too
            torch._foreach_add_([b.num_batches_tracked for b in bns if isinstance(b, nn.BatchNorm2d)], -1)
        return x + self.drop_path(h) if self.use_res else h
