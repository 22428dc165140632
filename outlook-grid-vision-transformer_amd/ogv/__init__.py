"""ogv — MI355X-native host runtime for the OutGridViT hot path (OutGridBlock fwd/bwd).

    ogv._lib        ctypes binding of libogv_hip.so (C-ABI in include/ogv.h)
    ogv.functional  autograd Functions over the HIP kernels (no CPU path)
    ogv.layers      Conv1x1 / Linear / LayerNorm drop-ins (stock parameter layout)
    ogv.train       Model-A builder, AdamW/WarmupCosine step, data-parallel harness

The reference-compatible module tree lives beside this package in ``src/`` (same import paths
as pablo-reyes8/outlook-grid-vision-transformer's ``src/model``).
"""
from ._lib import LIB_PATH, load, version  # noqa: F401

__version__ = "0.1.0"
