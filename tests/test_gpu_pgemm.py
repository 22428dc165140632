"""Pipelined panel GEMM (csrc/ogv_pgemm.hip): the small-M bf16 forward / data-gradient path.

Called through the C ABI (ogv_gemm_fwd / ogv_gemm_dgrad) on seeded inputs and held against fp64
torch, and against the LDS-tiled kernel it replaces (knob pgemm=0) on the same inputs:
  * the step's own small-M shapes (Model-A-7M stages 2-3: M = 32768 / 8192 rows), incl. the GELU
    prologue of fc2 and the activation-derivative epilogue of the fc1 data gradient;
  * ragged rows (M not a multiple of the 64 / 128-row panel), output widths that pad the 64 / 128 /
    192-column tile (40, 248, 328, 576), reductions that are not a multiple of the 64-wide k-step
    (8, 200, 248, 328);
  * every compiled (rows, columns) tile forced through the pg_rs / pg_tn knobs.
Tolerance: bf16 output storage, fp32 accumulation -> 1e-2 * max|ref| (forward weights are split
hi + lo, data-gradient weights rounded to bf16: both far inside it).
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


def _fwd(x, w, b, r, s, rps, act, M, N, K):
    out = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
    st = torch.cuda.current_stream().cuda_stream
    rc = _L().ogv_gemm_fwd(_p(x), K, _p(w), _p(b), _p(r), _p(s), rps, _p(out), N, M, N, K, ACT[act], BF16,
                           ctypes.c_void_p(st))
    assert rc == 0
    return out


def _dgrad(d, w, z, s, rps, act, M, N, K):
    dA = torch.empty(M, K, device=DEV, dtype=torch.bfloat16)
    ws = torch.empty(1 << 16, device=DEV, dtype=torch.uint8)
    st = torch.cuda.current_stream().cuda_stream
    rc = _L().ogv_gemm_dgrad(_p(d), N, _p(w), _p(z), K, _p(s), rps, _p(dA), K, M, N, K, ACT[act], _p(ws), BF16,
                             ctypes.c_void_p(st))
    assert rc == 0
    return dA


def _inputs(M, N, K, seed):
    g = torch.Generator().manual_seed(seed)
    x = torch.randn(M, K, generator=g).to(torch.bfloat16)
    w = torch.randn(N, K, generator=g) / K ** 0.5
    b = 0.1 * torch.randn(N, generator=g)
    r = torch.randn(M, N, generator=g).to(torch.bfloat16)
    d = torch.randn(M, N, generator=g).to(torch.bfloat16)
    z = torch.randn(M, K, generator=g).to(torch.bfloat16)
    return x, w, b, r, d, z


def _ref_fwd(x, w, b, r, s, rps, act, M):
    f = {None: lambda t: t, "gelu": torch.nn.functional.gelu, "silu": torch.nn.functional.silu}[act]
    a = f(x.double())
    if act:
        a = a.to(torch.bfloat16).double()  # the kernel rounds the prologue's output to bf16
    y = a @ w.double().t() + (b.double() if b is not None else 0)
    if s is not None:
        y = y * s.double().repeat_interleave(rps)[:M, None]
    if r is not None:
        y = y + r.double()
    return y


def _ref_dgrad(d, w, z, s, rps, act, M):
    y = d.double() @ w.to(torch.bfloat16).double()
    if s is not None:
        y = y * s.double().repeat_interleave(rps)[:M, None]
    if act:
        zz = z.double().requires_grad_()
        f = {"gelu": torch.nn.functional.gelu, "silu": torch.nn.functional.silu}[act]
        gz, = torch.autograd.grad(f(zz).sum(), zz)
        y = y * gz
    return y


FWD_CASES = [  # M, N, K, prologue act, bias, residual, rowscale
    (32768, 768, 192, None, True, False, False), (32768, 192, 768, "gelu", True, True, True),
    (32768, 576, 192, None, True, False, False), (32768, 248, 192, None, True, True, False),
    (8192, 1024, 256, None, True, False, False), (8192, 256, 1024, "gelu", True, True, True),
    (8192, 328, 256, None, False, True, False), (8192, 512, 256, None, True, False, False),
    (1000, 40, 200, "silu", True, True, True), (777, 96, 8, None, True, False, False),
    (130, 200, 248, "gelu", False, False, True), (64, 1024, 256, None, True, True, False),
    (5000, 256, 328, None, True, False, False),
]


@pytest.mark.parametrize("case", FWD_CASES)
def test_pgemm_fwd_vs_fp64(case):
    M, N, K, act, hb, hr, hs = case
    x, w, b, r, _, _ = _inputs(M, N, K, M + 7 * N + 13 * K)
    rps = 16
    s = (torch.rand((M + rps - 1) // rps, generator=torch.Generator().manual_seed(K)) + 0.5) if hs else None
    ref = _ref_fwd(x, w, b if hb else None, r if hr else None, s, rps, act, M)
    args = [t.to(DEV) if t is not None else None for t in (x, w, b if hb else None, r if hr else None, s)]
    errs = {}
    for mode in (1, 0):
        _opt("pgemm", mode)
        y = _fwd(*args[:4], args[4], rps, act, M, N, K)
        torch.cuda.synchronize()
        errs[mode] = fx.maxrel(y.float(), ref)
    _opt("pgemm", 1)
    assert errs[1] <= 1e-2, errs
    assert errs[1] <= 1.5 * errs[0] + 2e-3, errs


DGRAD_CASES = [  # M, N (reduction), K (output columns), act derivative, rowscale
    (32768, 768, 192, "gelu", False), (32768, 192, 768, None, False), (32768, 576, 192, "silu", True),
    (8192, 1024, 256, "gelu", False), (8192, 256, 1024, None, True), (8192, 328, 256, None, False),
    (1000, 200, 40, "silu", True), (130, 248, 96, None, False), (64, 8, 1024, "gelu", False),
]


@pytest.mark.parametrize("case", DGRAD_CASES)
def test_pgemm_dgrad_vs_fp64(case):
    M, N, K, act, hs = case
    _, w, _, _, d, z = _inputs(M, N, K, 3 * M + N + K)
    rps = 16
    s = (torch.rand((M + rps - 1) // rps, generator=torch.Generator().manual_seed(N)) + 0.5) if hs else None
    ref = _ref_dgrad(d, w, z, s, rps, act, M)
    dd, wd, zd = d.to(DEV), w.to(DEV), z.to(DEV)
    sd = s.to(DEV) if s is not None else None
    errs = {}
    for mode in (1, 0):
        _opt("pgemm", mode)
        y = _dgrad(dd, wd, zd if act else None, sd, rps, act, M, N, K)
        torch.cuda.synchronize()
        errs[mode] = fx.maxrel(y.float(), ref)
    _opt("pgemm", 1)
    assert errs[1] <= 1e-2, errs
    assert errs[1] <= 1.5 * errs[0] + 2e-3, errs


@pytest.mark.parametrize("rs", [1, 2])  # pg_rs is ignored for tn=12 (64-row panels only)
@pytest.mark.parametrize("tn", [4, 8, 12])
def test_pgemm_forced_tiles(rs, tn):
    """Every compiled tile shape: forward with the GELU prologue + residual, and a data gradient with
    the SiLU derivative, at a ragged shape."""
    M, N, K = 3001, 200, 136
    x, w, b, r, d, z = _inputs(M, N, K, 11 * rs + tn)
    _opt("pg_rs", rs)
    _opt("pg_tn", tn)
    try:
        y = _fwd(x.to(DEV), w.to(DEV), b.to(DEV), r.to(DEV), None, 1, "gelu", M, N, K)
        dA = _dgrad(d.to(DEV), w.to(DEV), z.to(DEV), None, 1, "silu", M, N, K)
        torch.cuda.synchronize()
    finally:
        _opt("pg_rs", 0)
        _opt("pg_tn", 0)
    assert fx.maxrel(y.float(), _ref_fwd(x, w, b, r, None, 1, "gelu", M)) <= 1e-2
    assert fx.maxrel(dA.float(), _ref_dgrad(d, w, z, None, 1, "silu", M)) <= 1e-2


def test_pgemm_identity_exact():
    """W = I (hi = 1, lo = 0) passes bf16 inputs through bit-exactly; 2I + residual x gives 3x."""
    M, C = 8192, 256
    x = torch.randn(M, C, device=DEV).to(torch.bfloat16)
    eye = torch.eye(C, device=DEV)
    assert torch.equal(_fwd(x, eye, None, None, None, 1, None, M, C, C), x)
    assert torch.equal(_fwd(x, 2 * eye, None, x, None, 1, None, M, C, C), (3 * x.float()).to(torch.bfloat16))
    assert torch.equal(_dgrad(x, eye, None, None, 1, None, M, C, C), x)
