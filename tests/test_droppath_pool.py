"""The batched DropPath draw (ogv.layers.draw_drop_path_scales) keeps the reference DropPath law
(src/model/Outlook_Block.py:15-22: per-sample Bernoulli(keep) / keep) and its consumption rules."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "outlook-grid-vision-transformer_amd"))


def test_pool_law_and_consumption():
    from ogv.layers import draw_drop_path_scales, drop_path_scale
    from src.model.Outlook_Block import DropPath
    torch.manual_seed(0)
    mods = [DropPath(0.1), DropPath(0.3), DropPath(0.0)]
    for m in mods:
        m.train()
    B = 200000
    x = torch.empty(B, 4)
    draw_drop_path_scales(mods, B, torch.device("cpu"))
    for m, p in zip(mods[:2], (0.1, 0.3)):
        s = drop_path_scale(m, x)
        keep = 1.0 - p
        vals = set(torch.unique(s).tolist())
        assert vals <= {0.0, 1.0 / keep} or all(abs(v - 0.0) < 1e-7 or abs(v - 1.0 / keep) < 1e-5 for v in vals)
        assert abs(float((s > 0).float().mean()) - keep) < 0.01       # Bernoulli(keep)
        assert abs(float(s.mean()) - 1.0) < 0.015                      # unbiased factor
        assert getattr(m, "_ogv_scale", None) is None                  # consumed once
    assert drop_path_scale(mods[2], x) is None                         # p = 0: identity
    # without a pooled draw, each call draws its own mask (reference behaviour)
    s = drop_path_scale(mods[0], x)
    assert s.shape == (B,) and abs(float(s.mean()) - 1.0) < 0.015
    # eval: identity, nothing drawn
    for m in mods:
        m.eval()
    draw_drop_path_scales(mods, B, torch.device("cpu"))
    assert drop_path_scale(mods[0], x) is None
