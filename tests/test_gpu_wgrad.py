"""bf16 weight gradient through the C ABI (ogv_gemm_wgrad): the split-M tiled kernel (ogv_gemm.hip),
the streaming kernel (ogv_swgrad.hip) and the pipelined kernel (ogv_wgrad2.hip, knob wg2, default 2) against
fp64 torch on the same seeded inputs.

    dW[n, k] = sum_m rs(m) dOut[m, n] * act(A[m, k]),   dbias[n] = sum_m rs(m) dOut[m, n]

Cases: the Model-A-7M step's own shapes (M = 32768 / 8192 / 131072 rows, the GELU prologue of fc2),
ragged rows (M not a multiple of the 64-row pipeline step, fewer rows than one step), output
widths that pad the 64 / 96 / 128 / 192 tile edges, the per-sample DropPath row scale, no bias;
every tile edge forced through wg2_tile; and whole bf16 module fixtures (the MBConv project's BN +
SiLU + SE-gate prologue form, which only the fused MBConv op issues) on the previous kernels
(wg2 = 0) against the reference's goldens.  Tolerance: bf16 operands (the prologue output rounded to bf16, as the kernel
does -- the fp64 reference rounds it the same way), fp32 accumulation -> 1e-2 * max|ref|.
"""
import ctypes

import pytest
import torch

import _fixtures as fx

pytestmark = pytest.mark.gpu
DEV = "cuda"
BF16, ACT = 1, {None: 0, "gelu": 1, "silu": 2}


@pytest.fixture(autouse=True, scope="module")
def _lib():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    import ogv
    ogv.load()


def _L():
    from ogv._lib import load
    return load()


def _opt(name, v):
    assert _L().ogv_set_option(name.encode(), int(v)) == 0


def _p(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else None


def _wgrad(d, x, s, rps, act, bias, M, N, K):
    dW = torch.full((N, K), float("nan"), device=DEV)
    db = torch.full((N,), float("nan"), device=DEV) if bias else None
    # sized after the knobs are set (the plan, hence the partial count, depends on them)
    ws = torch.empty(_L().ogv_gemm_wgrad_ws_bytes(M, N, K), device=DEV, dtype=torch.uint8)
    st = torch.cuda.current_stream().cuda_stream
    rc = _L().ogv_gemm_wgrad(_p(d), N, _p(x), K, _p(s), rps, _p(dW), _p(db), M, N, K, ACT[act], _p(ws), BF16,
                             ctypes.c_void_p(st))
    assert rc == 0
    torch.cuda.synchronize()
    return dW, db


def _ref(d, x, s, rps, act, M):
    f = {None: lambda t: t, "gelu": torch.nn.functional.gelu, "silu": torch.nn.functional.silu}[act]
    a = f(x.double())
    if act:
        a = a.to(torch.bfloat16).double()  # the kernel rounds the prologue's output to bf16
    g = d.double()
    if s is not None:
        # the kernel scales dOut by rs in fp32 and stages it as bf16
        g = (g.float() * s.float().repeat_interleave(rps)[:M, None]).to(torch.bfloat16).double()
    return g.t() @ a, g.sum(0)


CASES = [  # M, N, K, prologue act, bias, rowscale
    (32768, 192, 768, "gelu", True, True), (32768, 768, 192, None, True, False),
    (32768, 192, 192, None, True, False), (32768, 576, 192, None, False, True),
    (32768, 192, 384, "gelu", False, False), (8192, 256, 1024, "gelu", True, False),
    (8192, 1024, 256, None, True, True), (8192, 72, 256, None, True, False),
    (131072, 96, 384, "gelu", True, False), (1000, 200, 136, "gelu", True, True),
    (777, 96, 64, None, True, False), (40, 48, 24, None, True, False), (130, 328, 248, "silu", True, True),
]
MODES = [("default", {}), ("wg2=0", {"wg2": 0}), ("wg2=1", {"wg2": 1}),
         ("wg2_fuse=1", {"wg2_fuse": 1})]  # default = wg2 2, wg2_fuse 0
DEFAULTS = {"wg2": 2, "wg2_blocks": 512, "wg2_tile": 0, "wg2_fuse": 0}


def _inputs(M, N, K, rs, seed):
    g = torch.Generator().manual_seed(seed)
    x = torch.randn(M, K, generator=g).to(torch.bfloat16)
    d = torch.randn(M, N, generator=g).to(torch.bfloat16)
    rps = 64
    s = (torch.rand((M + rps - 1) // rps, generator=g) * 2).float() if rs else None
    return x, d, s, rps


def _check(case, knobs, seed=0):
    M, N, K, act, bias, rs = case
    x, d, s, rps = _inputs(M, N, K, rs, seed + M + N + K)
    ref_w, ref_b = _ref(d, x, s, rps, act, M)
    xd, dd = x.to(DEV), d.to(DEV)
    sd = s.to(DEV) if s is not None else None
    for k, v in knobs.items():
        _opt(k, v)
    try:
        dW, db = _wgrad(dd, xd, sd, rps, act, bias, M, N, K)
    finally:
        for k in knobs:
            _opt(k, DEFAULTS.get(k, 0))
    assert torch.isfinite(dW).all(), "unwritten / non-finite dW"
    assert fx.maxrel(dW, ref_w) <= 1e-2, (case, knobs, fx.maxrel(dW, ref_w))
    if bias:
        assert torch.isfinite(db).all()
        assert fx.maxrel(db, ref_b) <= 1e-2, (case, knobs, fx.maxrel(db, ref_b))
    return dW, db


@pytest.mark.parametrize("mode", MODES, ids=[m[0] for m in MODES])
@pytest.mark.parametrize("case", CASES, ids=lambda c: "x".join(str(v) for v in c[:3]) + f"-{c[3]}")
def test_wgrad_vs_fp64(case, mode):
    _check(case, mode[1])


@pytest.mark.parametrize("tile", [64, 96, 128, 192])
@pytest.mark.parametrize("case", [(32768, 192, 768, "gelu", True, True), (1000, 200, 136, None, True, False),
                                  (130, 328, 248, "silu", False, True)],
                         ids=lambda c: "x".join(str(v) for v in c[:3]))
def test_wgrad2_forced_tiles(case, tile):
    _check(case, {"wg2": 2, "wg2_tile": tile})


@pytest.mark.parametrize("blocks", [64, 4096])
def test_wgrad2_slab_counts(blocks):
    """Few long slabs (many pipeline steps per workgroup) and many short ones (one or two steps)."""
    _check((32768, 192, 768, "gelu", True, True), {"wg2": 2, "wg2_blocks": blocks})
    _check((8192, 256, 1024, "gelu", True, False), {"wg2": 2, "wg2_blocks": blocks})


def test_wgrad2_deterministic():
    case = (32768, 192, 768, "gelu", True, True)
    a = _check(case, {"wg2": 2})
    b = _check(case, {"wg2": 2})
    assert torch.equal(a[0], b[0]) and torch.equal(a[1], b[1])


@pytest.mark.parametrize("case", [(32768, 768, 192, None, True, False), (8192, 72, 256, None, True, False),
                                  (40, 48, 24, None, True, False), (130, 328, 248, "silu", True, True)],
                         ids=lambda c: "x".join(str(v) for v in c[:3]))
def test_wgrad2_fused_reduction(case):
    """The in-kernel last-workgroup reduction (wg2_fuse=1; off by default, slower): equal to the colreduce path
    within fp32 summation-order rounding, BIT-identical across repeated launches (slab order fixed,
    whichever workgroup arrives last; the arrival counters reset themselves -- a stale counter would
    skip or double a tile), also over more launches than the counter ring holds and with launches
    in flight on two streams at once."""
    M, N, K, act, bias, rs = case
    x, d, s, rps = _inputs(M, N, K, rs, 11)
    xd, dd = x.to(DEV), d.to(DEV)
    sd = s.to(DEV) if s is not None else None
    ref = _check(case, {"wg2_fuse": 0}, seed=11 - M - N - K)
    _opt("wg2_fuse", 1)
    try:
        _fused_repeats(case, dd, xd, sd, rps, ref)
    finally:
        _opt("wg2_fuse", 0)


def _fused_repeats(case, dd, xd, sd, rps, ref):
    M, N, K, act, bias, rs = case
    outs = [_wgrad(dd, xd, sd, rps, act, bias, M, N, K) for _ in range(3)]
    for w, b in outs:
        assert torch.isfinite(w).all()
        assert fx.maxrel(w, ref[0]) <= 1e-5
        if bias:
            assert fx.maxrel(b, ref[1]) <= 1e-5
        assert torch.equal(w, outs[0][0]) and (not bias or torch.equal(b, outs[0][1]))
    # many launches back to back (several trips round the counter ring) on two streams at once
    ws = [torch.empty(_L().ogv_gemm_wgrad_ws_bytes(M, N, K), device=DEV, dtype=torch.uint8) for _ in range(2)]
    res = [(torch.empty(N, K, device=DEV), torch.empty(N, device=DEV) if bias else None) for _ in range(2)]
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    for st in streams:
        st.wait_stream(torch.cuda.current_stream())
    for it in range(400):
        i = it & 1
        with torch.cuda.stream(streams[i]):
            rc = _L().ogv_gemm_wgrad(_p(dd), N, _p(xd), K, _p(sd), rps, _p(res[i][0]), _p(res[i][1]), M, N, K,
                                     ACT[act], _p(ws[i]), BF16, ctypes.c_void_p(streams[i].cuda_stream))
            assert rc == 0
    torch.cuda.synchronize()
    for w, b in res:
        assert torch.equal(w, outs[0][0]) and (not bias or torch.equal(b, outs[0][1]))


@pytest.mark.parametrize("name", fx.fixture_names("mbconv_") + fx.fixture_names("outgrid_block_")[:2])
def test_modules_bf16_legacy_wgrad(name):
    """Whole bf16 modules (fused MBConv: BN + SiLU + SE-gate prologue) with the weight gradients on
    the previous split-M / streaming kernels (wg2 = 0), against the reference's goldens
    (test_gpu_parity.test_golden_bf16 runs the same fixtures on the default, pipelined kernel)."""
    import test_gpu_parity as tp
    _opt("wg2", 0)
    try:
        tp.test_golden_bf16(name)
    finally:
        _opt("wg2", 2)


# ------------------------------------------------------------------------------------------------
# ogv_gemm_fwd_act: fc1 of a Linear -> act -> Linear pair writes Z and act(Z) in one launch; the MLPs
# then run fc2 and its weight gradient on act(Z) with no prologue (functional.materialise_act).
FWD_ACT_CASES = [  # M, N, K, act: streaming (large M), panel (M = 32768 / 8192), tiled (ragged / N % 8)
    (524288, 192, 48, "gelu"), (131072, 384, 96, "gelu"), (32768, 768, 192, "gelu"), (8192, 1024, 256, "silu"),
    (1000, 200, 136, "gelu"), (130, 54, 24, "gelu"),
]


@pytest.mark.parametrize("case", FWD_ACT_CASES, ids=lambda c: "x".join(str(v) for v in c[:3]) + f"-{c[3]}")
def test_gemm_fwd_act(case):
    """out is bit-identical to ogv_gemm_fwd's; aout = act(out) of the stored bf16 values within one
    bf16 rounding (the kernels' erf is the A&S 7.1.26 form, |err| <= 1.5e-7)."""
    M, N, K, act = case
    g = torch.Generator().manual_seed(M + N + K)
    x = torch.randn(M, K, generator=g).to(torch.bfloat16).to(DEV)
    w = (torch.randn(N, K, generator=g) / K ** 0.5).to(DEV)
    b = (0.1 * torch.randn(N, generator=g)).to(DEV)
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    ref = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
    assert _L().ogv_gemm_fwd(_p(x), K, _p(w), _p(b), None, None, 1, _p(ref), N, M, N, K, 0, BF16, st) == 0
    out = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
    aout = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
    assert _L().ogv_gemm_fwd_act(_p(x), K, _p(w), _p(b), _p(out), N, _p(aout), N, M, N, K, ACT[act], BF16, st) == 0
    torch.cuda.synchronize()
    assert torch.equal(out, ref)
    f = {"gelu": torch.nn.functional.gelu, "silu": torch.nn.functional.silu}[act]
    want = f(out.float())
    assert ((aout.float() - want).abs() <= 2 ** -7 * want.abs() + 1e-6).all()


def test_gemm_fwd_act_rejects():
    x = torch.zeros(64, 32, device=DEV)
    w = torch.zeros(16, 32, device=DEV)
    o = torch.zeros(64, 16, device=DEV)
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    assert _L().ogv_gemm_fwd_act(_p(x), 32, _p(w), None, _p(o), 16, _p(o), 16, 64, 16, 32, 1, 0, st) != 0  # fp32
    xb, ob = x.bfloat16(), o.bfloat16()
    assert _L().ogv_gemm_fwd_act(_p(xb), 32, _p(w), None, _p(ob), 16, _p(ob), 16, 64, 16, 32, 0, BF16, st) != 0


@pytest.mark.parametrize("which,C,H,B", [("mlp", 192, 8, 16), ("mlp", 48, 32, 4), ("mlp2d", 96, 16, 6),
                                         ("mlp2d", 256, 4, 8)])
def test_mlp_materialised_act_matches_prologue(which, C, H, B):
    """A bf16 MLP with the activation materialised by fc1 (default) against the same module with the
    activation as fc2's prologue (OGV_MAT_ACT=0 form): same bf16 operands everywhere, so outputs and
    the input gradient agree to bf16 rounding and the weight gradients to the fp32 summation order."""
    from ogv import functional as OF
    from src.model.Out_Grid_Block import MLP
    from src.model.outlook_attention import MLP2d
    torch.manual_seed(C + H)
    mod = (MLP(C, 4.0) if which == "mlp" else MLP2d(C, 2.0)).to(DEV)
    if which == "mlp":
        x = torch.randn(B, H, H, C, device=DEV)
        res = torch.randn(B, H, H, C, device=DEV).bfloat16()
    else:
        x = torch.randn(B, C, H, H, device=DEV).contiguous(memory_format=torch.channels_last)
        res = torch.randn(B, C, H, H, device=DEV).contiguous(memory_format=torch.channels_last).bfloat16()
    rs = (torch.rand(B, device=DEV) * 2)
    runs = []
    for mat in (True, False):
        OF._MAT_ACT = mat
        try:
            xi = x.clone().bfloat16().requires_grad_()
            for p in mod.parameters():
                p.grad = None
            with torch.autocast("cuda", dtype=torch.bfloat16):
                y = mod(xi, residual=res, row_scale=rs)
            y.float().square().sum().backward()
            runs.append((y.detach().float(), xi.grad.float(), [p.grad.clone() for p in mod.parameters()]))
        finally:
            OF._MAT_ACT = True
    (y0, dx0, g0), (y1, dx1, g1) = runs
    assert fx.maxrel(y0, y1) <= 1e-2
    assert fx.maxrel(dx0, dx1) <= 1e-2
    for a, b in zip(g0, g1):
        assert fx.maxrel(a, b) <= 1e-3
