"""Model-A training harness on MI355X: builder, optimizer/schedule, one-process-per-GPU data
parallelism, and the per-step function the benchmark times.

Restates the reference's training semantics (not its host-side logging):
  build_model            scripts/train.py:29-60 (StageCfg(**s) per stage -> MaxOutNet)
  param_groups_no_wd     src/training/warmup.py:4-26
  WarmupCosineLR         src/training/warmup.py:29-59 (step-based, state_dict = step_num)
  train step             src/training/one_epoch_train.py:85-153: autocast fwd, CE(label
                         smoothing) in fp32, backward, clip_grad_norm_(1.0), AdamW, scheduler
The reference loop syncs the host ~5x per step (isfinite, float(gnorm), .item()s); this step has
no host syncs: the grad-norm stays on device (clip_grad_norm_ foreach path) and the loss is
returned as a device tensor.

Data parallelism (the reference has none): one process per GPU, torch.distributed with the
"nccl" backend (= RCCL on ROCm) over xGMI; DistributedDataParallel buckets the fp32 gradients
(7.5 M params = 30 MB for Model-A-7M) and all-reduces them during backward.  Each rank keeps its
own BatchNorm batch statistics (DDP default).
"""
from __future__ import annotations

import math
import os
from typing import List, Optional

import torch
import torch.nn as nn
import torch.nn.functional as F

# Stage layouts of the reference configs (configs/cifar100_model_a_7m.yaml:7-27,
# configs/cifar100_model_a_14m.yaml:7-27, configs/tinyimagenet200_model_a.yaml:7-27).
MODEL_CONFIGS = {
    "model_a_7m": dict(num_classes=100, stem_dim=64, dpr_max=0.07, img=32, stages=[
        dict(dim=48, depth=1, num_heads=2, grid_size=8, outlook_heads=2),
        dict(dim=96, depth=2, num_heads=3, grid_size=8, outlook_heads=3),
        dict(dim=192, depth=3, num_heads=6, grid_size=4, outlook_heads=6),
        dict(dim=256, depth=1, num_heads=8, grid_size=2, outlook_heads=8)]),
    "model_a_14m_tin64": dict(num_classes=200, stem_dim=64, dpr_max=0.08, img=64, stages=[
        dict(dim=64, depth=2, num_heads=2, grid_size=8, outlook_heads=2),
        dict(dim=128, depth=2, num_heads=4, grid_size=8, outlook_heads=4),
        dict(dim=256, depth=3, num_heads=8, grid_size=4, outlook_heads=8),
        dict(dim=384, depth=1, num_heads=6, grid_size=2, outlook_heads=6)]),
    "model_a_22m_224": dict(num_classes=1000, stem_dim=64, dpr_max=0.11, img=224, stages=[
        dict(dim=64, depth=2, num_heads=2, grid_size=8, outlook_heads=2),
        dict(dim=128, depth=3, num_heads=4, grid_size=8, outlook_heads=4),
        dict(dim=256, depth=4, num_heads=8, grid_size=4, outlook_heads=8),
        dict(dim=384, depth=2, num_heads=6, grid_size=2, outlook_heads=6)]),
}


def build_model(model_cfg: dict) -> nn.Module:
    """YAML `model:` section -> MaxOutNet (only Model A is on the hot path)."""
    from src.Model_A_OutGridNet import MaxOutNet
    from src.model.downsampling import DownsampleConfig
    from src.stage_config import StageCfg

    kind = str(model_cfg.get("type", "model_a")).lower()
    if kind not in ("a", "model_a", "maxout", "outgrid"):
        raise ValueError(f"model.type '{kind}' is not built by this framework (Model A only)")
    stages = [StageCfg(**s) for s in model_cfg.get("stages", [])]
    if not stages:
        raise ValueError("model.stages must have at least one stage config")
    return MaxOutNet(num_classes=int(model_cfg.get("num_classes", 100)), stages=stages,
                     in_ch=int(model_cfg.get("in_ch", 3)), stem_dim=int(model_cfg.get("stem_dim", 64)),
                     dpr_max=float(model_cfg.get("dpr_max", 0.1)),
                     down_cfg=DownsampleConfig(**model_cfg.get("downsample", {})))


def param_groups_no_wd(model: nn.Module, weight_decay: float):
    decay, no_decay = [], []
    for name, p in model.named_parameters():
        if not p.requires_grad:
            continue
        low = name.lower()
        skip = name.endswith(".bias") or any(tag in low for tag in ("norm", "bn", "ln", "pos", "cls_token"))
        (no_decay if skip else decay).append(p)
    return [{"params": decay, "weight_decay": weight_decay}, {"params": no_decay, "weight_decay": 0.0}]


class WarmupCosineLR:
    """Linear warmup for warmup_steps, then cosine from the base lr down to min_lr."""

    def __init__(self, optimizer, total_steps: int, warmup_steps: int, min_lr: float = 0.0):
        self.optimizer = optimizer
        self.total_steps, self.warmup_steps, self.min_lr = int(total_steps), int(warmup_steps), float(min_lr)
        self.base_lrs = [g["lr"] for g in optimizer.param_groups]
        self.step_num = 0

    def lr_at(self, t: int, base: float) -> float:
        if self.warmup_steps > 0 and t <= self.warmup_steps:
            return base * t / self.warmup_steps
        prog = (min(t, self.total_steps) - self.warmup_steps) / max(1, self.total_steps - self.warmup_steps)
        return self.min_lr + (base - self.min_lr) * 0.5 * (1.0 + math.cos(math.pi * prog))

    def step(self):
        self.step_num += 1
        for g, base in zip(self.optimizer.param_groups, self.base_lrs):
            g["lr"] = self.lr_at(self.step_num, base)

    def state_dict(self):
        return {"step_num": self.step_num}

    def load_state_dict(self, d):
        self.step_num = int(d.get("step_num", 0))


# ------------------------------------------------------------------------------- distributed
def setup_distributed():
    """One process per GPU (torchrun env).  Returns (rank, world, local_rank, device)."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if torch.cuda.is_available():
        torch.cuda.set_device(local)
        device = torch.device("cuda", local)
    else:
        device = torch.device("cpu")
    if world > 1 and not torch.distributed.is_initialized():
        backend = "nccl" if device.type == "cuda" else "gloo"
        torch.distributed.init_process_group(backend=backend, device_id=device if device.type == "cuda" else None)
    return rank, world, local, device


def wrap_ddp(model: nn.Module, device, bucket_cap_mb: float = 8.0):
    if not (torch.distributed.is_available() and torch.distributed.is_initialized()):
        return model
    if torch.distributed.get_world_size() == 1:
        return model
    return nn.parallel.DistributedDataParallel(
        model, device_ids=[device.index] if device.type == "cuda" else None, bucket_cap_mb=bucket_cap_mb,
        gradient_as_bucket_view=True, broadcast_buffers=True)


# ------------------------------------------------------------------------------- step
class Trainer:
    """Holds model/optimizer/schedule; ``step(x, y)`` is one full training iteration."""

    def __init__(self, model: nn.Module, lr=5e-4, weight_decay=0.05, clip=1.0, label_smoothing=0.1,
                 total_steps=10_000, warmup_ratio=0.05, min_lr=1e-6, amp_dtype: Optional[torch.dtype] = torch.bfloat16):
        self.model = model
        core = model.module if hasattr(model, "module") else model
        fused = next(core.parameters()).is_cuda
        self.opt = torch.optim.AdamW(param_groups_no_wd(core, weight_decay), lr=lr, fused=fused)
        self.sched = WarmupCosineLR(self.opt, total_steps, int(warmup_ratio * total_steps), min_lr)
        self.params = [p for p in core.parameters() if p.requires_grad]
        self.clip, self.ls, self.amp_dtype = clip, label_smoothing, amp_dtype

    def step(self, x: torch.Tensor, y: torch.Tensor) -> torch.Tensor:
        self.opt.zero_grad(set_to_none=True)
        with torch.autocast("cuda", dtype=self.amp_dtype or torch.float32, enabled=self.amp_dtype is not None):
            logits = self.model(x)
        loss = F.cross_entropy(logits.float(), y, label_smoothing=self.ls)
        loss.backward()
        if self.clip is not None:
            torch.nn.utils.clip_grad_norm_(self.params, self.clip, foreach=True)
        self.opt.step()
        self.sched.step()
        return loss.detach()
