"""Time the stem conv+BN+SiLU forward / backward (Model-A 7M: B=512, 32x32, 3 -> 64, bf16 train) on
the dedicated kernels for several workgroup counts (knob stem_wgs) and on the generic conv kernels."""
import sys
import torch
sys.path.insert(0, "tests")
sys.path.insert(0, "outlook-grid-vision-transformer_amd")
from test_gpu_convbn import _modules  # noqa: E402
from ogv import functional as OF  # noqa: E402
from ogv._lib import load  # noqa: E402

lib = load()
conv, bn = _modules(3, 64, 1, True, "silu", seed=4)
conv = conv.cuda().to(memory_format=torch.channels_last)
bn = bn.cuda().train()
x = torch.randn(512, 3, 32, 32, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
gy = torch.randn(512, 64, 32, 32, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
for stem, wgs in [(0, 512), (1, 256), (1, 512), (1, 1024), (1, 2048), (1, 4096)]:
    lib.ogv_set_option(b"stem", stem)
    lib.ogv_set_option(b"stem_wgs", wgs)
    for _ in range(3):
        y = OF.conv3x3_bn_act(x, conv, bn, "silu")
        y.backward(gy)
    torch.cuda.synchronize()
    e = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
    n = 20
    e[0].record()
    for _ in range(n):
        y = OF.conv3x3_bn_act(x, conv, bn, "silu")
    e[1].record()
    for _ in range(n):
        y = OF.conv3x3_bn_act(x, conv, bn, "silu")
        y.backward(gy)
    e[2].record()
    torch.cuda.synchronize()
    f = e[0].elapsed_time(e[1]) / n
    print(f"stem={stem} wgs={wgs}: fwd op {1e3 * f:.1f} us, fwd+bwd {1e3 * e[1].elapsed_time(e[2]) / n:.1f} us", flush=True)
