"""Diagnose NaN persistence after a non-finite batch (eager and graph modes)."""
import sys
sys.path.insert(0, "outlook-grid-vision-transformer_amd")
sys.path.insert(0, "tests")
import torch
import ogv
ogv.load()
from test_gpu_train import _model, _batch
from ogv.train import Trainer

for graphs in (False, True):
    m = _model(8)
    t = Trainer(m, total_steps=50, warmup_ratio=0.1, graphs=graphs, capture_warmup=1)
    for i in range(3):
        t.step(*_batch(8, 20 + i))
    x, y = _batch(8, 30)
    x[2, 1, 5, 7] = float("nan")
    t.step(x, y)
    nanbufs = [n for n, b in m.named_buffers() if b.is_floating_point() and not torch.isfinite(b).all()]
    nanpar = [n for n, p in m.named_parameters() if not torch.isfinite(p).all()]
    print("graphs", graphs, "nan buffers:", len(nanbufs), nanbufs[:5], "nan params:", nanpar[:5])
    l = t.step(*_batch(8, 31))
    print("  next loss", l.item())
    # reset the buffers to finite values and retry
    with torch.no_grad():
        for n, b in m.named_buffers():
            if b.is_floating_point():
                b.nan_to_num_(0.0)
    l = t.step(*_batch(8, 32))
    print("  after buffer reset loss", l.item())
    # eval-free forward check
    with torch.no_grad(), torch.autocast("cuda", dtype=torch.bfloat16):
        out = m(_batch(8, 33)[0])
    print("  plain forward finite:", torch.isfinite(out).all().item())
