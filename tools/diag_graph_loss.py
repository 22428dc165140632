"""Diagnostic: replayed-step loss vs eager forward loss (test_graph_replay_takes_new_inputs), split
into logits / loss-function differences.  argv: [sync] [stem=0] ..."""
import sys
import torch
import torch.nn.functional as F
sys.path.insert(0, "tests")
sys.path.insert(0, "outlook-grid-vision-transformer_amd")
from test_gpu_train import _model, _batch  # noqa: E402
from ogv.train import Trainer  # noqa: E402
from ogv.functional import cross_entropy_ls  # noqa: E402
from ogv._lib import load  # noqa: E402

args = sys.argv[1:]
for a in args:
    if "=" in a:
        k, v = a.split("=")
        assert load().ogv_set_option(k.encode(), int(v)) == 0
m = _model(2)
t = Trainer(m, total_steps=50, graphs=True, capture_warmup=0)
x0, y0 = _batch(8, 5)
t.step(x0, y0)
if "sync" in args:
    torch.cuda.synchronize()
for i in (6, 5):
    x, y = _batch(8, i)
    with torch.no_grad(), torch.autocast("cuda", dtype=torch.bfloat16):
        pass
    with torch.autocast("cuda", dtype=torch.bfloat16):
        z = m(x).float().detach()
    with torch.autocast("cuda", dtype=torch.bfloat16):
        z2 = m(x).float().detach()
    ref = F.cross_entropy(z, y, label_smoothing=0.1).item()
    loss = t.step(x, y).float().item()
    print(f"{args} batch {i}: torch CE {ref:.7f} replay {loss:.7f} eager repeat max|dz| {float((z2 - z).abs().max()):.3e}",
          flush=True)
