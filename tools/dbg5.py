import sys
sys.path.insert(0, "outlook-grid-vision-transformer_amd"); sys.path.insert(0, "tests")
import torch, ogv
ogv.load()
import test_gpu_train as T
x, y = T._batch(8, 6)
m = T._model(2)
outs = {}
def hook(name):
    def f(mod, inp, out):
        outs.setdefault(name, []).append(out.detach().float().clone())
    return f
for n, mod in m.named_modules():
    if n.count(".") <= 2 and n:
        mod.register_forward_hook(hook(n))
with torch.no_grad(), torch.autocast("cuda", dtype=torch.bfloat16):
    m(x); m(x)
for n, v in outs.items():
    if len(v) >= 2:
        d = float((v[0] - v[1]).abs().max()); s = float(v[0].abs().max())
        print(f"{n:40s} max|d|={d:.3e} scale={s:.3e}")
