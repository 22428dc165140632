"""Drop-in for src/training/cutmix_mixup_aug.py: the same three functions, with the batch and
label mixing done by the native kernels (ogv/mix.py, ogv_mix_images / ogv_mix_targets)."""
import math  # noqa: F401  (the reference module exports these names)
import random  # noqa: F401

from ogv.mix import apply_mixup_cutmix, soft_target_cross_entropy  # noqa: F401
from ogv.mix import one_hot as _one_hot  # noqa: F401
