"""Per-stage hyper-parameters consumed by OutGridBlock(cfg) and MaxOutNet.

Field-for-field the same dataclass as the reference's ``StageCfg``
(src/stage_config.py:4-34) so YAML ``model.stages`` entries and ``StageCfg(**d)`` calls keep
working.  ``window_size`` is accepted and ignored, as in the reference (grid mode only).
"""
from dataclasses import dataclass


@dataclass
class StageCfg:
    dim: int                      # channels C of the stage
    depth: int                    # number of OutGridBlocks
    num_heads: int                # grid-attention heads
    grid_size: int                # g: strided grid partition factor
    window_size: int = 8          # unused (kept for config compatibility)
    outlook_heads: int = 6
    outlook_kernel: int = 3
    outlook_mlp_ratio: float = 2.0
    mbconv_expand_ratio: float = 4.0
    mbconv_se_ratio: float = 0.25
    mbconv_act: str = "silu"
    use_bn: bool = True
    attn_drop: float = 0.0
    proj_drop: float = 0.0
    ffn_drop: float = 0.0
    drop_path: float = 0.0
    mlp_ratio: float = 4.0        # BHWC MLP expansion
    mlp_act: str = "gelu"
