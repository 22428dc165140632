"""Strided grid partition — drop-in for src/model/grid_partition.py (:3-32).

Group (b, gi, gj) collects the pixels (ty*g + gi, tx*g + gj): a *dilated* partition with g*g
groups per image of (H/g)*(W/g) tokens each.  On the hot path this regrouping never happens as a
copy — the grid-attention kernel addresses the tokens in place — but the functions are kept for
analysis code that calls them (same errors, same output layout).
"""
import torch


def _check_bhwc(x: torch.Tensor, what: str):
    if x.ndim != 4:
        raise ValueError(f"Expected {what}.ndim==4{' (BHWC)' if what == 'x' else ''}. Got shape {tuple(x.shape)}")


def grid_partition(x: torch.Tensor, grid_size: int):
    _check_bhwc(x, "x")
    B, H, W, C = x.shape
    g = grid_size
    if g <= 0:
        raise ValueError("grid_size must be > 0")
    if H % g or W % g:
        raise ValueError(f"H and W must be divisible by grid_size. Got H={H}, W={W}, g={g}")
    grids = x.reshape(B, H // g, g, W // g, g, C).permute(0, 2, 4, 1, 3, 5).reshape(B * g * g, H // g, W // g, C)
    return grids, (B, H, W, C, g)


def grid_unpartition(grids: torch.Tensor, meta) -> torch.Tensor:
    _check_bhwc(grids, "grids")
    B, H, W, C, g = meta
    if grids.shape[0] != B * g * g:
        raise ValueError(f"grids.shape[0] must be B*g*g = {B*g*g}. Got {grids.shape[0]}")
    if tuple(grids.shape[1:]) != (H // g, W // g, C):
        raise ValueError(f"grids shape mismatch. Expected (*,{H // g},{W // g},{C}) got {tuple(grids.shape)}")
    return grids.reshape(B, g, g, H // g, W // g, C).permute(0, 3, 1, 4, 2, 5).reshape(B, H, W, C)
