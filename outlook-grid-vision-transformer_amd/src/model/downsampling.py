"""Stage-transition downsampling — drop-in for src/model/downsampling.py.

kind="conv" (every reference config) keeps the module tree ``op.0`` Conv2d(3x3, stride 2),
``op.1`` BatchNorm2d / Identity, ``op.2`` activation and runs them as one native op
(ogv_convbn_fwd/bwd).  kind="pool" (AvgPool2d + 1x1 conv) stays on stock ops."""
import torch
import torch.nn as nn
import torch.nn.functional as F

from typing import Literal
from dataclasses import dataclass

DownsampleType = Literal["conv", "pool"]
ActType = Literal["silu", "gelu", "relu"]


def make_activation(act) -> nn.Module:
    from src.model.outlook_attention import make_activation as _mk
    return _mk(act)


@dataclass(frozen=True)
class DownsampleConfig:
    kind: DownsampleType = "conv"
    act: ActType = "silu"
    use_bn: bool = True


class Downsample(nn.Module):
    """[B, in, H, W] -> [B, out, H/2, W/2]: 3x3/s2 conv ("conv") or 2x2 avg-pool + 1x1 ("pool"),
    then BN and the activation."""

    def __init__(self, in_ch: int, out_ch: int, cfg: DownsampleConfig = DownsampleConfig()):
        super().__init__()
        if in_ch <= 0 or out_ch <= 0:
            raise ValueError("in_ch and out_ch must be > 0")
        self.in_ch, self.out_ch, self.kind = in_ch, out_ch, cfg.kind
        norm = nn.BatchNorm2d(out_ch) if cfg.use_bn else nn.Identity()
        if cfg.kind == "conv":
            layers = [nn.Conv2d(in_ch, out_ch, kernel_size=3, stride=2, padding=1, bias=not cfg.use_bn)]
        elif cfg.kind == "pool":
            layers = [nn.AvgPool2d(kernel_size=2, stride=2),
                      nn.Conv2d(in_ch, out_ch, kernel_size=1, stride=1, padding=0, bias=not cfg.use_bn)]
        else:
            raise ValueError("cfg.kind must be 'conv' or 'pool'")
        self.op = nn.Sequential(*layers, norm, make_activation(cfg.act))

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        if self.kind != "conv":
            return self.op(x)
        from ogv import functional as OF
        from ogv.layers import act_name
        conv, norm, act = self.op[0], self.op[1], self.op[2]
        a = act_name(act)
        if a is None and not isinstance(act, nn.Identity):
            raise NotImplementedError(f"ogv Downsample: unsupported activation {type(act).__name__}")
        return OF.conv3x3_bn_act(x, conv, norm if isinstance(norm, nn.BatchNorm2d) else None, a)
