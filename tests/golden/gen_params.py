"""Deterministic, order-independent parameter / input generator for the golden fixtures.

Used twice, with identical results:
  * by ``make_golden.py`` (run once in the survey container, where the reference imports) to
    fill the *reference* modules before recording outputs, and
  * by the tests, to fill *our* drop-in modules (same state_dict keys) before comparing.

Every tensor is drawn from its own ``numpy.random.RandomState`` whose seed is derived from
(base seed, state_dict key) with crc32, so the values do not depend on iteration order.
The legacy RandomState stream is frozen by numpy's compatibility policy, so no weight files
need to be committed.
"""
from __future__ import annotations

import zlib

import numpy as np


def _rs(key: str, seed: int) -> np.random.RandomState:
    return np.random.RandomState((zlib.crc32(key.encode()) ^ (seed * 2654435761)) & 0x7FFFFFFF)


def param_value(key: str, shape, seed: int = 0) -> np.ndarray:
    """Value for one state_dict entry (parameter or buffer)."""
    shape = tuple(int(s) for s in shape)
    rs = _rs(key, seed)
    leaf = key.rsplit(".", 1)[-1]
    if leaf == "num_batches_tracked":
        return np.zeros(shape, dtype=np.int64)
    if leaf == "running_mean":
        return (0.1 * rs.standard_normal(shape)).astype(np.float32)
    if leaf == "running_var":
        return (1.0 + 0.2 * rs.uniform(size=shape)).astype(np.float32)
    if leaf == "bias":
        return (0.1 * rs.standard_normal(shape)).astype(np.float32)
    if len(shape) >= 2:
        fan_in = int(np.prod(shape[1:]))
        return (rs.standard_normal(shape) / np.sqrt(fan_in)).astype(np.float32)
    # 1-d affine weights (LayerNorm / BatchNorm gamma)
    return (1.0 + 0.1 * rs.standard_normal(shape)).astype(np.float32)


def fill_module(module, seed: int = 0) -> None:
    """Overwrite every parameter and buffer of a torch module in place."""
    import torch

    sd = module.state_dict()
    new = {}
    for k, v in sd.items():
        arr = param_value(k, v.shape, seed)
        new[k] = torch.from_numpy(arr).to(v.dtype)
    module.load_state_dict(new, strict=True)


def tensor(name: str, shape, seed: int = 0, scale: float = 1.0) -> np.ndarray:
    """Input / upstream-gradient tensor."""
    return (scale * _rs("input:" + name, seed).standard_normal(tuple(shape))).astype(np.float32)


def labels(name: str, n: int, num_classes: int, seed: int = 0) -> np.ndarray:
    return _rs("labels:" + name, seed).randint(0, num_classes, size=(n,)).astype(np.int64)


def sketch_matrix(key: str, cols: int, k: int = 4) -> np.ndarray:
    """Fixed normal [cols, k] matrix used to sketch large weight gradients (G @ R)."""
    return _rs("sketch:" + key, 0).standard_normal((cols, k))


def input_from_spec(spec) -> np.ndarray:
    """spec = [name, shape, scale, offset] as recorded in a fixture's meta."""
    name, shape, scale, offset = spec
    return tensor(name, shape, scale=scale) + np.float32(offset)
