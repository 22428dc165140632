import sys
sys.path.insert(0, "outlook-grid-vision-transformer_amd"); sys.path.insert(0, "tests")
import torch, ogv
ogv.load()
from ogv.train import Trainer
import test_gpu_train as T
torch.backends.cudnn.benchmark = False
B = int(sys.argv[1]) if len(sys.argv) > 1 else 64
x, y = T._batch(B, 3)
ma, mb = T._model(11), T._model(11)
ta = Trainer(ma, total_steps=100, graphs=False)
tb = Trainer(mb, total_steps=100, graphs=True, capture_warmup=1)
for i in range(8):
    la = ta.step(x, y).item(); lb = tb.step(x, y).item()
    torch.cuda.synchronize()
    d = max(float((pa - pb).abs().max()) for pa, pb in zip(ma.parameters(), mb.parameters()))
    worst = max(((float((pa - pb).abs().max()), n) for (n, pa), pb in zip(ma.named_parameters(), mb.parameters())))
    p0 = next(iter(tb.opt.state))
    print(i, f"loss {la:.5f} {lb:.5f}  max|dparam| {d:.3e} worst {worst[1]}  lrA {ta.opt.param_groups[0]['lr']:.3e} "
          f"lrB {float(tb.opt.param_groups[0]['lr']):.3e} stepB {float(tb.opt.state[p0]['step'])} "
          f"stepA {float(ta.opt.state[next(iter(ta.opt.state))]['step'])}", flush=True)
