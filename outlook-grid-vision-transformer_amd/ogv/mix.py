"""MixUp / CutMix on the device — the tensor work of src/training/cutmix_mixup_aug.py:17-64 as two
native launches (ogv_mix_images, ogv_mix_targets).

The host side draws every random decision in the reference's order and from the same sources
(`random.random()` for the apply / cutmix coin flips, `torch.randperm(B, device=images.device)`,
`torch.distributions.Beta(a, a).sample().item()` for lam, `random.randint` for the box centre), so a
run seeded like the reference makes the same decisions.  `draw_mix_plan` is that host logic on its
own (CPU-testable); `apply_plan` launches the kernels.  No CPU fallback: a non-HIP tensor raises.
"""
from __future__ import annotations

import math
import random
from dataclasses import dataclass
from typing import Optional, Tuple

import torch
import torch.nn.functional as F

from . import _lib


@dataclass
class MixPlan:
    """One batch's decisions.  mix False => the reference's early returns (images, one_hot)."""
    mix: bool
    cutmix: bool = False
    perm: Optional[torch.Tensor] = None
    lam: float = 1.0                 # final lam (CutMix: 1 - box area / image area, :56-58)
    box: Tuple[int, int, int, int] = (0, 0, 0, 0)   # y1, y2, x1, x2 (CutMix only)


def draw_mix_plan(B: int, H: int, W: int, mixup_alpha: float = 0.0, cutmix_alpha: float = 0.0,
                  prob: float = 1.0, device="cpu") -> MixPlan:
    """Host draws of apply_mixup_cutmix (cutmix_mixup_aug.py:29-62), same order and sources."""
    if prob <= 0.0 or (mixup_alpha <= 0.0 and cutmix_alpha <= 0.0):
        return MixPlan(False)
    if random.random() > prob:
        return MixPlan(False)
    use_cutmix = (cutmix_alpha > 0.0) and (mixup_alpha <= 0.0 or random.random() < 0.5)
    perm = torch.randperm(B, device=device)
    if use_cutmix:
        lam = torch.distributions.Beta(cutmix_alpha, cutmix_alpha).sample().item()
        cut_w = int(W * math.sqrt(1.0 - lam))
        cut_h = int(H * math.sqrt(1.0 - lam))
        cx = random.randint(0, W - 1)
        cy = random.randint(0, H - 1)
        x1, x2 = max(cx - cut_w // 2, 0), min(cx + cut_w // 2, W)
        y1, y2 = max(cy - cut_h // 2, 0), min(cy + cut_h // 2, H)
        lam = 1.0 - (x2 - x1) * (y2 - y1) / float(W * H)
        return MixPlan(True, True, perm, lam, (y1, y2, x1, x2))
    lam = torch.distributions.Beta(mixup_alpha, mixup_alpha).sample().item()
    return MixPlan(True, False, perm, lam)


def _need_hip(t: torch.Tensor, what: str):
    if t.device.type != "cuda":
        raise RuntimeError(f"{what}: ogv kernels need a HIP device tensor (got {t.device})")


def one_hot(targets: torch.Tensor, num_classes: int) -> torch.Tensor:
    """F.one_hot(targets, K).float() (cutmix_mixup_aug.py:6-7) in one launch."""
    return _soft_targets(targets, None, num_classes, 1.0, 0.0)


def _soft_targets(targets, perm, K, lam_a, lam_b):
    """Soft targets on the device.  Divergence from the reference, on purpose (no host sync): a label
    outside [0, K) -- e.g. an ignore_index of -100 -- does not raise like F.one_hot
    (cutmix_mixup_aug.py:6-7); its row becomes NaN, so that batch's loss is non-finite and the
    Trainer's device guard skips the update and counts it in ``Trainer.nonfinite_steps`` (read it
    per epoch).  The non-mix CE path (F.cross_entropy) instead ignores -100 labels."""
    _need_hip(targets, "ogv mix targets")
    t = targets.to(torch.int64).contiguous()
    out = torch.empty(t.shape[0], K, device=t.device, dtype=torch.float32)
    p = perm.to(device=t.device, dtype=torch.int64).contiguous() if perm is not None else None
    _lib.check(_lib.load().ogv_mix_targets(t.data_ptr(), p.data_ptr() if p is not None else None, out.data_ptr(),
                                           t.shape[0], K, lam_a, lam_b, torch.cuda.current_stream().cuda_stream),
               "ogv_mix_targets")
    return out


def apply_plan(images: torch.Tensor, targets: torch.Tensor, num_classes: int, plan: MixPlan):
    """Run a MixPlan: (images_aug, targets_soft [B, K] fp32)."""
    if not plan.mix:
        return images, one_hot(targets, num_classes)
    _need_hip(images, "ogv_mix_images")
    if images.ndim != 4:
        raise ValueError(f"apply_mixup_cutmix expects [B, C, H, W] images, got {tuple(images.shape)}")
    B, C, H, W = images.shape
    if images.dtype not in (torch.float32, torch.bfloat16):
        raise NotImplementedError(f"ogv_mix_images: dtype {images.dtype}")
    if images.is_contiguous():
        cl = 0
    elif images.is_contiguous(memory_format=torch.channels_last):
        cl = 1
    else:
        images, cl = images.contiguous(), 0
    out = torch.empty_like(images)          # keeps the memory format
    perm = plan.perm.to(device=images.device, dtype=torch.int64).contiguous()
    lam = plan.lam
    # ATen's scalar ops take lam and (1 - lam) as fp32 opmath scalars (:53 and :64)
    lam_a, lam_b = lam, 1.0 - lam
    y1, y2, x1, x2 = plan.box
    dt = _lib.OGV_BF16 if images.dtype == torch.bfloat16 else _lib.OGV_F32
    _lib.check(_lib.load().ogv_mix_images(images.data_ptr(), out.data_ptr(), perm.data_ptr(), B, C, H, W, cl,
                                          1 if plan.cutmix else 0, lam_a, lam_b, y1, y2, x1, x2, dt,
                                          torch.cuda.current_stream().cuda_stream), "ogv_mix_images")
    return out, _soft_targets(targets, perm, num_classes, lam_a, lam_b)


def apply_mixup_cutmix(images: torch.Tensor, targets: torch.Tensor, num_classes: int, mixup_alpha: float = 0.0,
                       cutmix_alpha: float = 0.0, prob: float = 1.0):
    """Drop-in for apply_mixup_cutmix (cutmix_mixup_aug.py:17-64): (images_aug [B,3,H,W], targets_soft [B,K])."""
    B, _, H, W = images.shape
    plan = draw_mix_plan(B, H, W, mixup_alpha, cutmix_alpha, prob, device=images.device)
    return apply_plan(images, targets, num_classes, plan)


def soft_target_cross_entropy(logits: torch.Tensor, targets_soft: torch.Tensor) -> torch.Tensor:
    """-(targets_soft * log_softmax(logits)).sum(1).mean() (cutmix_mixup_aug.py:10-12)."""
    logp = F.log_softmax(logits, dim=1)
    return -(targets_soft * logp).sum(dim=1).mean()
