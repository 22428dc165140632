import sys
sys.path.insert(0, "outlook-grid-vision-transformer_amd"); sys.path.insert(0, "tests")
import torch, ogv
import torch.nn.functional as F
ogv.load()
from ogv.train import Trainer
import test_gpu_train as T
batches = [T._batch(8, 5), T._batch(8, 6)]
m = T._model(2)
def fwd(x, y, grad):
    with torch.set_grad_enabled(grad), torch.autocast("cuda", dtype=torch.bfloat16):
        return F.cross_entropy(m(x).float(), y, label_smoothing=0.1).item()
x, y = batches[1]
print("nograd", fwd(x, y, False), fwd(x, y, False), "grad", fwd(x, y, True), fwd(x, y, True))
m.eval(); print("eval nograd", fwd(x, y, False), fwd(x, y, False)); m.train()
# BN running stats change per train forward: check sensitivity
t = Trainer(m, total_steps=50, graphs=True, capture_warmup=0)
t.step(*batches[0])
print("after capture nograd", fwd(x, y, False), "grad", fwd(x, y, True))
print("replay", t.step(x, y).item())
