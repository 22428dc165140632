"""Model A (MaxOutNet): stem -> [OutGridBlock x depth (+ Downsample)] per stage -> BN/GAP/Linear.

Drop-in for src/Model_A_OutGridNet.py:9-67 — the same constructor, module names
(stem, proj_in, stages.<s>.<b>, downs.<s>, head_norm, classifier) and state_dict.  The blocks
come from our src.model (HIP kernels); the stem / downsample conv3x3+BN+SiLU, the 1x1 proj_in and
the head BatchNorm run on the native conv/GEMM/BN kernels as well (ogv_convbn_*, ogv_gemm_*,
ogv_bn_act_*).
"""
from src.model.Out_Grid_Block import *  # noqa: F401,F403
from src.model.downsampling import *  # noqa: F401,F403
from src.model.stem_head import *  # noqa: F401,F403
from src.stage_config import *  # noqa: F401,F403
from src.model.Out_Grid_Block import OutGridBlock
from src.model.downsampling import Downsample, DownsampleConfig
from src.model.stem_head import ConvStem, List, make_dpr
from src.stage_config import StageCfg
import torch
import torch.nn as nn
from ogv.layers import BatchNorm2d, Conv1x1, draw_drop_path_scales


class MaxOutNet(nn.Module):
    def __init__(self, num_classes: int, stages: List[StageCfg], in_ch: int = 3, stem_dim: int = 64,
                 dpr_max: float = 0.1,
                 down_cfg: DownsampleConfig = DownsampleConfig(kind="conv", act="silu", use_bn=True)):
        super().__init__()
        assert len(stages) >= 1
        self.stem = ConvStem(in_ch, stem_dim, act="silu", use_bn=True)
        first = stages[0].dim
        self.proj_in = Conv1x1(stem_dim, first, bias=True) if stem_dim != first else nn.Identity()
        rates = iter(make_dpr(sum(s.depth for s in stages), dpr_max))
        self.stages = nn.ModuleList()
        self.downs = nn.ModuleList()
        for si, scfg in enumerate(stages):
            self.stages.append(nn.ModuleList(
                OutGridBlock(StageCfg(**{**scfg.__dict__, "drop_path": next(rates)})) for _ in range(scfg.depth)))
            if si + 1 < len(stages):
                self.downs.append(Downsample(scfg.dim, stages[si + 1].dim, cfg=down_cfg))
        self.head_norm = BatchNorm2d(stages[-1].dim)
        self.classifier = nn.Linear(stages[-1].dim, num_classes)

    def forward(self, x):
        train_prologue(self, x)
        x = self.proj_in(self.stem(x))
        for si, blocks in enumerate(self.stages):
            for blk in blocks:
                x = blk(x)
            if si < len(self.downs):
                x = self.downs[si](x)
        return classifier_head(x, self.classifier, self.head_norm)


def classifier_head(x, classifier: nn.Linear, norm=None):
    """head_norm -> GAP -> Linear (Model_A_OutGridNet.py:64-67) in fp32 even under bf16 autocast: the pooled
    features are averaged in fp32 and the classifier keeps its fp32 weights, so the logits carry no
    bf16 rounding of their own.  A plain ogv BatchNorm2d `norm` (no hooks) and the pool run as ONE op,
    BN of the per-image channel means (BN is per-channel affine, so the two commute: ogv_head_bn_pool_*,
    one pass over x forward and backward); otherwise norm(x) runs as its own module first.  The Linear
    runs on the native fp32 GEMM (ogv_gemm_fwd: the thread-group kernel for [B, K] outputs, its dgrad /
    weight gradient on the exact-f32 MFMA kernels) -- the module itself is called instead whenever the
    call must be observable or is not a plain Linear on the GPU: a subclass or wrapper (its own forward),
    module or global forward (pre-)hooks, or CPU features (the native kernels take device pointers only)."""
    if norm is not None and _fused_head_norm_ok(norm, x):
        from ogv import functional as OF
        pooled = OF.head_bn_pool(x, norm)
    else:
        if norm is not None:
            x = norm(x)
        pooled = x.mean(dim=(2, 3), dtype=torch.float32)
    if not _native_classifier_ok(classifier, pooled):
        with torch.autocast(pooled.device.type, enabled=False):
            return classifier(pooled)
    from ogv import functional as OF
    return OF.linear_rows(pooled, classifier.weight, classifier.bias)


def _fused_head_norm_ok(norm, x) -> bool:
    """The head BatchNorm may fold into the pool: exactly the ogv BatchNorm2d (its forward is the native
    kernel anyway), on the GPU, with no module or global forward hooks (its output would have to exist)."""
    from torch.nn.modules import module as _m
    from ogv.layers import BatchNorm2d
    return (type(norm) is BatchNorm2d and x.is_cuda and x.dim() == 4 and norm.track_running_stats
            and not (norm._forward_hooks or norm._forward_pre_hooks
                     or _m._global_forward_hooks or _m._global_forward_pre_hooks))


def _native_classifier_ok(classifier, pooled) -> bool:
    from torch.nn.modules import module as _m
    return (type(classifier) is nn.Linear and pooled.is_cuda
            and not (classifier._forward_hooks or classifier._forward_pre_hooks
                     or _m._global_forward_hooks or _m._global_forward_pre_hooks))


def train_prologue(model: nn.Module, x):
    """Per-forward work shared by Model A and Model B in training mode: every block's DropPath
    factors in one draw (ogv.layers.draw_drop_path_scales) and every BatchNorm counter of the model
    in one multi-tensor add (the modules skip theirs)."""
    if not model.training:
        return
    dps = getattr(model, "_ogv_droppaths", None)
    if dps is None:
        from src.model.Outlook_Block import DropPath
        dps = model._ogv_droppaths = [m for m in model.modules() if isinstance(m, DropPath)]
    draw_drop_path_scales(dps, x.shape[0], x.device)
    bns = getattr(model, "_ogv_bns", None)
    if bns is None:
        bns = model._ogv_bns = [m for m in model.modules() if isinstance(m, nn.modules.batchnorm._BatchNorm)
                                and m.track_running_stats and m.num_batches_tracked is not None]
        for m in bns:
            m._ogv_nbt_pooled = True
    if bns and bns[0].training:
        torch._foreach_add_([m.num_batches_tracked for m in bns], 1)
