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

Execution: the whole step is captured once as a hipGraph (torch.cuda.CUDAGraph) and replayed,
so ~1200 kernel launches per step cost one graph launch instead of ~1200 Python/HIP launches.
The learning rate lives in a device tensor the schedule updates before each replay.

Data parallelism (the reference has none): one process per GPU, torch.distributed with the
"nccl" backend (= RCCL on ROCm) over xGMI.  The step is split at the one exchange the path has:
graph A = fwd + bwd + flatten of the fp32 gradients into ONE bucket (7.5 M params = 30 MB for
Model-A-7M, pre-divided by world size); one all_reduce of that bucket (a single large ring
collective: xGMI links are point-to-point, so one 30 MB message beats many small DDP buckets);
graph B = unflatten + clip_grad_norm + AdamW.  Parameters and buffers are broadcast from rank 0
once at start; each rank keeps its own BatchNorm batch statistics.
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
    # Model B (OutlookerFrontGridNet), configs/cifar100_model_b.yaml:1-29
    "model_b_cifar100": dict(type="model_b", num_classes=100, stem_dim=64, dpr_max=0.1, img=32,
                             outlooker_front_depth=3, stages=[
        dict(dim=64, depth=2, num_heads=2, grid_size=8, outlook_heads=2),
        dict(dim=128, depth=2, num_heads=4, grid_size=8, outlook_heads=4),
        dict(dim=256, depth=3, num_heads=8, grid_size=4, outlook_heads=8),
        dict(dim=384, depth=1, num_heads=6, grid_size=2, outlook_heads=6)]),
}


def build_model(model_cfg: dict) -> nn.Module:
    """YAML `model:` section -> MaxOutNet (Model A) or OutlookerFrontGridNet (Model B), the
    dispatch of scripts/train.py:33-60 (same type aliases, same errors)."""
    from src.Model_A_OutGridNet import MaxOutNet
    from src.Model_B_OutGridNet import OutlookerFrontGridNet
    from src.model.downsampling import DownsampleConfig
    from src.stage_config import StageCfg

    kind = str(model_cfg.get("type", "model_a")).lower()
    stages = [StageCfg(**s) for s in model_cfg.get("stages", [])]
    if not stages:
        raise ValueError("model.stages must have at least one stage config")
    common = dict(num_classes=int(model_cfg.get("num_classes", 100)), stages=stages,
                  in_ch=int(model_cfg.get("in_ch", 3)), stem_dim=int(model_cfg.get("stem_dim", 64)),
                  dpr_max=float(model_cfg.get("dpr_max", 0.1)),
                  down_cfg=DownsampleConfig(**model_cfg.get("downsample", {})))
    if kind in ("a", "model_a", "maxout", "outgrid"):
        return MaxOutNet(**common)
    if kind in ("b", "model_b", "outlooker_front", "front"):
        return OutlookerFrontGridNet(outlooker_front_depth=int(model_cfg.get("outlooker_front_depth", 2)), **common)
    raise ValueError(f"Unknown model.type '{kind}'. Use 'model_a' (MaxOutNet) or 'model_b' (OutlookerFrontGridNet)")


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
        self.base_lrs = [float(g["lr"]) for g in optimizer.param_groups]
        self.step_num = 0

    def lr_at(self, t: int, base: float) -> float:
        if self.warmup_steps > 0 and t <= self.warmup_steps:
            return base * t / self.warmup_steps
        prog = (min(t, self.total_steps) - self.warmup_steps) / max(1, self.total_steps - self.warmup_steps)
        return self.min_lr + (base - self.min_lr) * 0.5 * (1.0 + math.cos(math.pi * prog))

    def step(self):
        self.step_num += 1
        for g, base in zip(self.optimizer.param_groups, self.base_lrs):
            v = self.lr_at(self.step_num, base)
            if isinstance(g["lr"], torch.Tensor):
                g["lr"].fill_(v)      # device-resident lr read by the captured AdamW
            else:
                g["lr"] = v

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
def _dist_world():
    if torch.distributed.is_available() and torch.distributed.is_initialized():
        return torch.distributed.get_world_size()
    return 1


class Trainer:
    """Holds model/optimizer/schedule; ``step(x, y)`` is one full training iteration.

    ``graphs=True`` (HIP device only): the first ``capture_warmup`` calls run eagerly, the next one
    runs eagerly on a side stream and records the step into hipGraphs, every later call replays
    them (inputs are copied into the recorded x / y tensors when other tensors are passed).
    With world_size > 1 gradients are averaged by one all_reduce of a flat bucket (see module doc);
    pass the bare model (not DDP-wrapped)."""

    def __init__(self, model: nn.Module, lr=5e-4, weight_decay=0.05, clip=1.0, label_smoothing=0.1,
                 total_steps=10_000, warmup_ratio=0.05, min_lr=1e-6, amp_dtype: Optional[torch.dtype] = torch.bfloat16,
                 graphs: bool = False, capture_warmup: int = 3, capture_hook=None):
        self.model = model
        core = model.module if hasattr(model, "module") else model
        self.ddp = core is not model
        dev = next(core.parameters()).device
        fused = dev.type == "cuda"
        self.graphs = bool(graphs) and fused
        lr0 = torch.tensor(float(lr), device=dev) if self.graphs else lr
        self.opt = torch.optim.AdamW(param_groups_no_wd(core, weight_decay), lr=lr0, fused=fused,
                                     capturable=self.graphs)
        self.sched = WarmupCosineLR(self.opt, total_steps, int(warmup_ratio * total_steps), min_lr)
        self.params = [p for p in core.parameters() if p.requires_grad]
        self.clip, self.ls, self.amp_dtype = clip, label_smoothing, amp_dtype
        self.world = 1 if self.ddp else _dist_world()
        self.capture_warmup = int(capture_warmup)
        self.capture_hook = capture_hook          # called right before recording starts
        self._eager_steps = 0
        self._g = None
        if self.world > 1:
            self._sizes = [p.numel() for p in self.params]
            self.flat = torch.zeros(sum(self._sizes), device=dev, dtype=torch.float32)
            with torch.no_grad():   # identical start on every rank (what DDP's constructor does)
                for t in list(core.parameters()) + list(core.buffers()):
                    torch.distributed.broadcast(t.data, 0)

    # -- pieces of one step -------------------------------------------------------------------
    def _fwd_bwd(self, x, y):
        with torch.autocast("cuda", dtype=self.amp_dtype or torch.float32, enabled=self.amp_dtype is not None,
                            cache_enabled=not self.graphs):
            logits = self.model(x)
        if y.is_floating_point():   # soft targets from MixUp/CutMix (one_epoch_train.py:89-92)
            from .mix import soft_target_cross_entropy
            loss = soft_target_cross_entropy(logits.float(), y)
        else:
            loss = F.cross_entropy(logits.float(), y, label_smoothing=self.ls)
        loss.backward()
        return loss.detach()

    def _flatten(self):
        grads = [p.grad if p.grad is not None else torch.zeros_like(p) for p in self.params]
        torch.cat([g.reshape(-1) for g in grads], out=self.flat)
        self.flat.mul_(1.0 / self.world)

    def _unflatten(self):
        views = [v.view_as(p) for v, p in zip(self.flat.split(self._sizes), self.params)]
        for p, v in zip(self.params, views):
            if p.grad is None:
                p.grad = torch.empty_like(p)
        torch._foreach_copy_([p.grad for p in self.params], views)

    def _update(self):
        if self.clip is not None:
            torch.nn.utils.clip_grad_norm_(self.params, self.clip, foreach=True)
        self.opt.step()

    def _allreduce(self):
        torch.distributed.all_reduce(self.flat)

    def _eager(self, x, y):
        self.opt.zero_grad(set_to_none=True)
        loss = self._fwd_bwd(x, y)
        if self.world > 1:
            self._flatten()
            self._allreduce()
            self._unflatten()
        self._update()
        return loss

    def _capture(self, x, y):
        """This call's update runs eagerly on a side stream (allocator / library warm-up, as graph
        capture requires); then the step is recorded — recording executes nothing."""
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            loss = self._eager(x, y)
        torch.cuda.current_stream().wait_stream(side)
        loss = loss.clone()
        self.opt.zero_grad(set_to_none=True)
        self._x, self._y = x, y
        if self.capture_hook is not None:
            self.capture_hook()
        pool = torch.cuda.graph_pool_handle()
        self._g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self._g, pool=pool):
            self._loss = self._fwd_bwd(x, y)
            if self.world > 1:
                self._flatten()
            else:
                self._update()
        self.graph_grads = [p.grad for p in self.params]   # the tensors the replays write
        if self.world > 1:
            self._g2 = torch.cuda.CUDAGraph()
            with torch.cuda.graph(self._g2, pool=pool):
                self._unflatten()
                self._update()
        return loss

    def step(self, x: torch.Tensor, y: torch.Tensor) -> torch.Tensor:
        if not self.graphs or (self._g is None and self._eager_steps < self.capture_warmup):
            self._eager_steps += 1
            loss = self._eager(x, y)
        elif self._g is None:
            loss = self._capture(x, y)
        else:
            if x is not self._x or y is not self._y:
                self._x.copy_(x)
                self._y.copy_(y)
            self._g.replay()
            if self.world > 1:
                self._allreduce()
                self._g2.replay()
            loss = self._loss
        self.sched.step()
        return loss
