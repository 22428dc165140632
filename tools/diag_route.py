"""Diagnostic: GEMM routing of the grad-mode vs no-grad forward of Model-A-7M (B=8).  Run with
OGV_LOG_GEMM=1; prints the launches whose (shape, alignment, route) differ between the two."""
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
m = _model(2)
x, y = _batch(8, 5)
torch.cuda.synchronize()
print("=== grad", file=sys.stderr, flush=True)
with torch.autocast("cuda", dtype=torch.bfloat16):
    l1 = F.cross_entropy(m(x).float(), y, label_smoothing=0.1)
torch.cuda.synchronize()
print("=== nograd", file=sys.stderr, flush=True)
with torch.no_grad(), torch.autocast("cuda", dtype=torch.bfloat16):
    l2 = F.cross_entropy(m(x).float(), y, label_smoothing=0.1)
torch.cuda.synchronize()
print("=== end", file=sys.stderr, flush=True)
print("loss grad", l1.item(), "nograd", l2.item())
