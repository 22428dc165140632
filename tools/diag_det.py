"""Diagnostic: is the Model-A-7M train-mode forward reproducible call to call?  Prints the loss of
repeated grad-mode forwards with and without restoring the BatchNorm buffers in between."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "outlook-grid-vision-transformer_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

import ogv  # noqa: E402
from test_gpu_train import _batch, _model  # noqa: E402

ogv.load()
lib = ogv._lib.load()
for pg in (1, 0):
    assert lib.ogv_set_option(b"pgemm", pg) == 0
    m = _model(2)
    x, y = _batch(8, 5)
    bufs = [b.detach().clone() for b in m.buffers()]

    def fwd(grad):
        with torch.set_grad_enabled(grad), torch.autocast("cuda", dtype=torch.bfloat16):
            return F.cross_entropy(m(x).float(), y, label_smoothing=0.1).item()
    a = [fwd(True) for _ in range(3)]
    res = []
    for grad in (True, True, False):
        for b, s in zip(m.buffers(), bufs):
            b.data.copy_(s)
        res.append(fwd(grad))
    print(f"pgemm={pg} consecutive {a}  restored-buffers {res}")
