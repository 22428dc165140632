"""MaxOutNet stem / downsample / head on the native kernels vs an fp64 torch reference (CPU).

conv3x3(pad 1, stride 1|2) -> BatchNorm2d -> act  (ogv_convbn_fwd/bwd) and BatchNorm2d alone
(ogv_bn_act_fwd/bwd): outputs, running statistics, input / weight / bias / BN-affine gradients.
Tolerances: fp32 1e-3 * max(1, |ref|max) (north star), bf16 3e-2 * max(1, |ref|max) (bf16 storage
of activations and gradients, fp32 accumulation).
"""
import copy

import pytest
import torch
import torch.nn as nn

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True, scope="module")
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    import ogv
    ogv.load()


def _err(a, b):
    a, b = a.detach(), b.detach()
    return float((a.double().cpu() - b.double().cpu()).abs().max()), max(1.0, float(b.abs().max()))


def _modules(Cin, Cout, stride, use_bn, act, seed):
    torch.manual_seed(seed)
    conv = nn.Conv2d(Cin, Cout, 3, stride, 1, bias=not use_bn)
    bn = nn.BatchNorm2d(Cout) if use_bn else None
    if bn is not None:
        with torch.no_grad():
            bn.weight.uniform_(0.5, 1.5)
            bn.bias.uniform_(-0.3, 0.3)
            bn.running_mean.uniform_(-0.2, 0.2)
            bn.running_var.uniform_(0.5, 1.5)
    return conv, bn


ACTS = {"silu": nn.SiLU(), "gelu": nn.GELU(), "relu": nn.ReLU(), None: nn.Identity()}


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("case", [
    # B, Cin, Cout, H, W, stride, use_bn, train, act
    (4, 3, 64, 32, 32, 1, True, True, "silu"),       # stem
    (4, 48, 96, 32, 32, 2, True, True, "silu"),      # downsample s0 -> s1
    (2, 96, 192, 16, 16, 2, True, False, "silu"),    # eval BN
    (3, 16, 24, 9, 7, 2, True, True, "gelu"),        # odd sizes, ragged row tiles
    (2, 8, 40, 5, 6, 1, False, True, "relu"),        # use_bn=False: conv bias, no BN
    (2, 5, 12, 6, 6, 2, True, True, None),           # Cin % 8 != 0 on the strided path
    (3, 16, 24, 10, 6, 2, True, True, "gelu"),       # dgrad as 4 parity-class GEMMs, non-square
    # the dedicated stem kernels (bf16, C_in <= 3, C_out 32 / 64; fp32 and wider stems: generic path)
    (4, 3, 32, 10, 6, 1, True, True, "silu"),        # ragged 128-row tiles spanning images, C_out 32
    (2, 3, 64, 12, 12, 2, True, True, "silu"),       # stride 2
    (8, 1, 64, 9, 9, 1, False, True, "relu"),        # C_in 1, conv bias: dbias from the ones column
    (3, 3, 64, 10, 7, 1, True, True, "silu"),        # input not whole 16-B chunks: generic path
    (2, 2, 32, 8, 8, 1, True, False, "gelu"),        # C_in 2, eval BN
    (2, 3, 96, 8, 8, 1, True, True, "silu"),         # C_out 96: generic path
])
@pytest.mark.parametrize("wcl", [False, True], ids=["w_oihw", "w_channels_last"])
def test_conv_bn_act(case, dtype, wcl):
    """wcl: the conv weight in channels_last memory (as after model.to(channels_last)) -- the tap-major
    matrix the kernels use directly (w_layout 1: no transposes, the gradient written in place)."""
    from ogv import functional as OF
    B, Cin, Cout, H, W, stride, use_bn, train, act = case
    conv, bn = _modules(Cin, Cout, stride, use_bn, act, seed=Cin * 7 + Cout)
    g = torch.Generator().manual_seed(11)
    x = torch.randn(B, Cin, H, W, generator=g)
    # reference (fp64 CPU, stock modules)
    rconv, rbn = copy.deepcopy(conv).double(), copy.deepcopy(bn).double() if bn is not None else None
    if rbn is not None:
        rbn.train(train)
    xr = x.double().requires_grad_(True)
    yr = rconv(xr)
    if rbn is not None:
        yr = rbn(yr)
    yr = ACTS[act].double()(yr)
    gy = torch.randn(yr.shape, generator=g)
    yr.backward(gy.double())
    # ogv
    dconv = copy.deepcopy(conv).cuda()
    if wcl:
        dconv = dconv.to(memory_format=torch.channels_last)
        assert not dconv.weight.is_contiguous() or Cin == 1
    dbn = copy.deepcopy(bn).cuda() if bn is not None else None
    if dbn is not None:
        dbn.train(train)
    xd = x.cuda().to(dtype).contiguous(memory_format=torch.channels_last).requires_grad_(True)
    yd = OF.conv3x3_bn_act(xd, dconv, dbn, act)
    assert yd.shape == yr.shape and yd.dtype == dtype
    yd.backward(gy.cuda().to(dtype))
    tol = 1e-3 if dtype == torch.float32 else 3e-2
    names = ["out", "dx", "dw"] + (["dbias"] if conv.bias is not None else []) + \
        (["dgamma", "dbeta", "running_mean", "running_var"] if bn is not None else [])

    def results(c, b, xx, yy):
        r = {"out": yy, "dx": xx.grad, "dw": c.weight.grad, "dbias": c.bias.grad if c.bias is not None else None}
        if b is not None:
            r.update(dgamma=b.weight.grad, dbeta=b.bias.grad, running_mean=b.running_mean, running_var=b.running_var)
        return r

    got, ref = results(dconv, dbn, xd, yd), results(rconv, rbn, xr, yr)
    if bn is not None:
        assert int(dbn.num_batches_tracked) == int(rbn.num_batches_tracked)
    torch_err = {}
    if dtype == torch.bfloat16:
        # torch's own bf16 error on the same inputs (stock modules under autocast): a ReLU / SiLU
        # gate evaluated on bf16-rounded pre-activations flips near zero in both implementations
        tconv = copy.deepcopy(conv).cuda()
        tbn = copy.deepcopy(bn).cuda().train(train) if bn is not None else None
        xt = x.cuda().requires_grad_(True)
        with torch.autocast("cuda", dtype=torch.bfloat16):
            yt = tconv(xt)
            yt = tbn(yt) if tbn is not None else yt
            yt = ACTS[act].cuda()(yt)
        yt.backward(gy.cuda().to(yt.dtype))
        for n, t in results(tconv, tbn, xt, yt).items():
            if t is not None:
                torch_err[n] = _err(t, ref[n])[0]
    for name in names:
        e, scale = _err(got[name], ref[name])
        bound = max(tol * scale, 2.0 * torch_err.get(name, 0.0))
        assert e <= bound, f"{name}: max|d|={e:.3e} bound={bound:.3e} scale={scale:.3e} ({dtype}, {case})"


@pytest.mark.parametrize("case", [(512, 48, 96, 32, 32), (512, 96, 192, 16, 16), (512, 192, 256, 8, 8),
                                  (3, 16, 24, 10, 6), (2, 8, 16, 2, 2)])
def test_transposed_conv_merged_launch_bitwise(case):
    """The stride-2 conv's data gradient (a transposed conv) runs its four parity classes as ONE launch of the
    panel kernel (knob pg_tconv1, default; workgroup groups per class) -- the same tiles and arithmetic as the
    four launches it replaces, so dx (and every other gradient) is bit-identical to pg_tconv1 = 0; the 7M
    downsample shapes at bs 512 included."""
    from ogv import functional as OF
    from ogv._lib import load
    lib = load()
    B, Cin, Cout, H, W = case
    conv, bn = _modules(Cin, Cout, 2, True, "silu", seed=Cin + Cout)
    g = torch.Generator(device="cuda").manual_seed(5)
    x = torch.randn(B, Cin, H, W, device="cuda", generator=g).to(torch.bfloat16).contiguous(
        memory_format=torch.channels_last)
    outs = []
    try:
        for merged in (1, 0):
            assert lib.ogv_set_option(b"pg_tconv1", merged) == 0
            c, b = copy.deepcopy(conv).cuda().to(memory_format=torch.channels_last), copy.deepcopy(bn).cuda().train()
            xd = x.clone().requires_grad_(True)
            y = OF.conv3x3_bn_act(xd, c, b, "silu")
            y.backward(torch.ones_like(y))
            torch.cuda.synchronize()
            outs.append([y.detach(), xd.grad, c.weight.grad, b.weight.grad, b.bias.grad])
    finally:
        assert lib.ogv_set_option(b"pg_tconv1", 1) == 0
    for a, r in zip(*outs):
        assert torch.equal(a, r)


def test_stem_input_needs_no_grad():
    """The stem's input image has no gradient: the data-gradient GEMM is skipped."""
    from ogv import functional as OF
    conv, bn = _modules(3, 16, 1, True, "silu", seed=1)
    x = torch.randn(2, 3, 8, 8, device="cuda")
    y = OF.conv3x3_bn_act(x, conv.cuda(), bn.cuda(), "silu")
    y.sum().backward()
    assert x.grad is None and conv.weight.grad is not None


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("train", [True, False])
def test_head_batchnorm(dtype, train):
    from ogv.layers import BatchNorm2d
    torch.manual_seed(5)
    ref = nn.BatchNorm2d(256)
    with torch.no_grad():
        ref.weight.uniform_(0.5, 1.5)
        ref.bias.uniform_(-0.3, 0.3)
        ref.running_var.uniform_(0.5, 1.5)
    mod = BatchNorm2d(256)
    mod.load_state_dict(ref.state_dict())
    ref = ref.double().train(train)
    mod = mod.cuda().train(train)
    x = torch.randn(16, 256, 4, 4)
    xr = x.double().requires_grad_(True)
    yr = ref(xr)
    gy = torch.randn(yr.shape)
    yr.backward(gy.double())
    xd = x.cuda().to(dtype).contiguous(memory_format=torch.channels_last).requires_grad_(True)
    yd = mod(xd)
    yd.backward(gy.cuda().to(dtype))
    tol = 1e-3 if dtype == torch.float32 else 3e-2
    for name, got, want in [("out", yd, yr), ("dx", xd.grad, xr.grad), ("dgamma", mod.weight.grad, ref.weight.grad),
                            ("dbeta", mod.bias.grad, ref.bias.grad), ("rm", mod.running_mean, ref.running_mean),
                            ("rv", mod.running_var, ref.running_var)]:
        e, scale = _err(got, want)
        assert e <= tol * scale, f"{name}: {e:.3e} / {scale:.3e}"


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("train", [True, False])
@pytest.mark.parametrize("shape", [(512, 384, 4, 4), (16, 256, 4, 4), (8, 96, 7, 7), (3, 20, 5, 3), (5, 12, 1, 1)])
def test_head_bn_pool_matches_bn_then_mean(shape, dtype, train):
    """The classifier head's BatchNorm2d -> mean((2, 3)) as ONE op (ogv_head_bn_pool_*: BN of the per-image
    channel means) against the reference's order -- nn.BatchNorm2d then the mean -- in fp64 on the same (bf16-
    rounded) input: pooled features, running statistics, input and BN-affine gradients.  The op reads x in its
    storage type and computes in fp32 / fp64, so the bf16 bars are the fp32 ones except for dx (stored bf16)."""
    from ogv import functional as OF
    from ogv.layers import BatchNorm2d
    B, C, H, W = shape
    torch.manual_seed(B + C + H)
    ref = nn.BatchNorm2d(C)
    with torch.no_grad():
        ref.weight.uniform_(0.5, 1.5)
        ref.bias.uniform_(-0.3, 0.3)
        ref.running_mean.uniform_(-0.2, 0.2)
        ref.running_var.uniform_(0.5, 1.5)
    mod = BatchNorm2d(C)
    mod.load_state_dict(ref.state_dict())
    ref = ref.double().train(train)
    mod = mod.cuda().train(train)
    x = (1.5 * torch.randn(B, C, H, W) + 0.7).to(dtype)      # a mean far from the running mean: shifted sums
    xr = x.double().requires_grad_(True)
    pr = ref(xr).mean(dim=(2, 3))
    g = torch.randn(B, C)
    pr.backward(g.double())
    xd = x.cuda().contiguous(memory_format=torch.channels_last).requires_grad_(True)
    pd = OF.head_bn_pool(xd, mod)
    assert pd.dtype == torch.float32 and pd.shape == (B, C)
    pd.backward(g.cuda())
    assert int(mod.num_batches_tracked) == int(ref.num_batches_tracked)
    for name, got, want, tol in [("pooled", pd, pr, 1e-5), ("rm", mod.running_mean, ref.running_mean, 1e-6),
                                 ("rv", mod.running_var, ref.running_var, 1e-6),
                                 ("dgamma", mod.weight.grad, ref.weight.grad, 1e-5),
                                 ("dbeta", mod.bias.grad, ref.bias.grad, 1e-5),
                                 ("dx", xd.grad, xr.grad, 1e-5 if dtype == torch.float32 else 1e-2)]:
        e, scale = _err(got, want)
        assert e <= tol * scale, f"{name}: {e:.3e} / {scale:.3e}"


def test_model_head_uses_fused_bn_pool_unless_hooked():
    """MaxOutNet's head: head_norm + pool as ogv_head_bn_pool (the module's own forward never runs), the
    same logits as BatchNorm2d -> mean -> Linear; with a forward hook on head_norm the module runs (its
    output observable) and the logits agree."""
    from ogv.layers import BatchNorm2d
    from src.Model_A_OutGridNet import classifier_head
    torch.manual_seed(3)
    bn, lin = BatchNorm2d(64).cuda(), nn.Linear(64, 10).cuda()
    x = torch.randn(6, 64, 4, 4, device="cuda").contiguous(memory_format=torch.channels_last)
    calls = []
    y_fused = classifier_head(x, lin, bn)
    assert not calls
    bn2 = copy.deepcopy(bn)
    bn2.load_state_dict({**bn.state_dict(), "running_mean": torch.zeros(64), "running_var": torch.ones(64),
                         "num_batches_tracked": torch.tensor(0)})
    h = bn2.register_forward_hook(lambda m, i, o: calls.append(o.shape))
    y_hooked = classifier_head(x, lin, bn2)
    h.remove()
    assert calls == [(6, 64, 4, 4)]
    torch.testing.assert_close(y_fused, y_hooked, rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(bn.running_mean, bn2.running_mean, rtol=1e-6, atol=1e-6)


def test_convbn_full_size_stem_stats():
    """bs=512 stem (M = 524288 rows): BN batch statistics of the native path equal the
    mean/var of its own conv output recomputed by torch in fp64 (size-independent property)."""
    from ogv import functional as OF
    conv, bn = _modules(3, 64, 1, True, "silu", seed=2)
    conv, bn = conv.cuda(), bn.cuda().train()
    rm0 = bn.running_mean.clone()
    x = torch.randn(512, 3, 32, 32, device="cuda").contiguous(memory_format=torch.channels_last)
    with torch.no_grad():
        OF.conv3x3_bn_act(x, conv, bn, "silu")
        yconv = torch.nn.functional.conv2d(x.double(), conv.weight.double(), None, 1, 1)
        mean = yconv.mean(dim=(0, 2, 3))
    want = 0.9 * rm0.double() + 0.1 * mean
    e = float((bn.running_mean.double() - want).abs().max())
    assert e <= 1e-4, e


@pytest.mark.parametrize("B", [64, 512])
def test_stem_kernels_match_generic_conv(B):
    """Knob stem = 1 (dedicated stem kernels) against stem = 0 (the implicit-GEMM conv kernels) on the
    Model-A stem at 32 x 32, bf16 train mode: output, weight gradient, BN affine gradients and running
    statistics.  Both multiply by the split (hi + lo) weight with fp32 accumulation, so they differ only
    by the order of the 27-term sums, the bf16 rounding of the output that follows and the order of the
    row reductions (bounds: 1 bf16 ulp-scale on the output, 1e-3 relative on the reductions)."""
    from ogv import functional as OF
    from ogv._lib import load
    lib = load()
    conv, bn = _modules(3, 64, 1, True, "silu", seed=4)
    x = torch.randn(B, 3, 32, 32, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    gy = torch.randn(B, 64, 32, 32, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    res = []
    try:
        for knob in (0, 1):
            assert lib.ogv_set_option(b"stem", knob) == 0
            c = copy.deepcopy(conv).cuda().to(memory_format=torch.channels_last)
            b = copy.deepcopy(bn).cuda().train()
            y = OF.conv3x3_bn_act(x, c, b, "silu")
            y.backward(gy)
            res.append(dict(y=y.float(), dw=c.weight.grad, dg=b.weight.grad, db=b.bias.grad, rm=b.running_mean,
                            rv=b.running_var))
    finally:
        assert lib.ogv_set_option(b"stem", 1) == 0
    for k in res[0]:
        a, r = res[1][k], res[0][k]
        scale = max(1.0, float(r.abs().max()))
        tol = 1.6e-2 if k == "y" else 1e-3
        assert float((a - r).abs().max()) <= tol * scale, (k, float((a - r).abs().max()), scale)


def test_stem_kernel_output_independent_of_running_mean():
    """Train-mode BatchNorm output must not depend on the running mean used as the statistics' shift
    (it moves every step): the stem's fp64 per-lane statistics make it exact (tools/diag_stem.py
    measured one bf16 ulp of drift with fp32 partials, which a replayed step then amplified)."""
    from ogv import functional as OF
    conv, bn = _modules(3, 64, 1, True, "silu", seed=4)
    conv = conv.cuda().to(memory_format=torch.channels_last)
    bn = bn.cuda().train()
    x = torch.randn(8, 3, 32, 32, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    ys = [OF.conv3x3_bn_act(x, conv, bn, "silu").detach().clone() for _ in range(3)]   # running mean moves
    assert torch.equal(ys[0], ys[1]) and torch.equal(ys[0], ys[2])
