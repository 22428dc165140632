"""Autograd glue between the drop-in nn.Modules and the C-ABI of libogv_hip.so.

Every function here takes/returns device tensors and calls the HIP kernels through ctypes on
torch's current stream.  There is NO CPU path: a CPU tensor raises, so a test that passes can
only have passed through the native kernels.

Activations are handled as row-major [M, C] matrices, M = B*H*W: a channels_last NCHW tensor is
exactly that layout, so the reference's `.permute(...).contiguous()` copies
(src/model/outlook_attention.py:28-30, src/model/Out_Grid_Block.py:96,107) become free views.
"""
from __future__ import annotations

import ctypes
import os
import warnings

import torch

from . import _lib
from ._lib import ACT, OGV_BF16, OGV_F32, check

_vp = ctypes.c_void_p


def _ptr(t):
    return None if t is None else _vp(t.data_ptr())


def _stream():
    return _vp(torch.cuda.current_stream().cuda_stream)


def _dt(t: torch.Tensor) -> int:
    if t.dtype == torch.bfloat16:
        return OGV_BF16
    if t.dtype == torch.float32:
        return OGV_F32
    raise TypeError(f"ogv kernels support float32 and bfloat16 activations, got {t.dtype}")


_SIDE = {}
# Linear backward: weight gradient forked onto a side stream ("1") or after the data gradient on the
# current stream ("0", default since round 4).  Re-measured with the round-4 kernels (paired 40-step
# 7M runs, profiles/r04_side_streams.log): both forks 15.52-15.53 ms, neither (this and the MBConv
# library knob mb_side = 0) 15.13-15.14 ms -- concurrent kernels slow each other more than the
# overlap wins, and every cross-stream edge costs ~10 us in the graph.
_FORK = os.environ.get("OGV_FORK", "0") != "0"
# smallest M*(N+K) of a Linear backward whose weight gradient is forked onto the side stream
_FORK_MIN_WORK = int(os.environ.get("OGV_FORK_MIN_WORK", "0"))
# fork policy for the Linears whose dgrad applies an activation derivative (the MLP fc2 inputs):
# "1" = fork like the others, "0" = weight gradient after the data gradient on the current stream
_FORK_ACT = os.environ.get("OGV_FORK_ACT", "1") != "0"


def _side_stream(device):
    s = _SIDE.get(device.index)
    if s is None:
        s = _SIDE[device.index] = torch.cuda.Stream(device=device)
    return s


class _fork:
    """Context manager yielding the stream handle for the forked work: a side stream that waits on
    the current stream at entry and that the current stream waits on at exit (enabled), or the
    current stream itself (disabled).  Tensors touched on the side stream are recorded on it so the
    caching allocator does not hand their memory out early."""

    def __init__(self, enabled, *tensors):
        self.enabled = bool(enabled)
        self.tensors = [t for t in tensors if t is not None]

    def __enter__(self):
        self.main = torch.cuda.current_stream()
        if not self.enabled:
            return _vp(self.main.cuda_stream)
        self.side = _side_stream(self.main.device)
        self.side.wait_stream(self.main)
        for t in self.tensors:
            t.record_stream(self.side)
        return _vp(self.side.cuda_stream)

    def __exit__(self, *a):
        if self.enabled:
            self.main.wait_stream(self.side)
        return False


def require_device(*tensors, what="ogv"):
    for t in tensors:
        if t is not None and not t.is_cuda:
            raise RuntimeError(f"{what}: the MI355X kernels need HIP device tensors (got {t.device}); "
                               f"this framework has no CPU execution path")


def _ws(nbytes: int, device, deferrable: bool = False) -> torch.Tensor:
    """Scratch for one C-ABI call.  deferrable: the call's parameter-gradient reduction may be deferred
    (deferred_param_reductions), so its slab partials must stay allocated until the flush."""
    t = torch.empty(max(int(nbytes), 16), dtype=torch.uint8, device=device)
    if deferrable and _DEFER["on"]:
        _DEFER["keep"].append(t)
    return t


_DEFER = {"on": False, "keep": []}


class deferred_param_reductions:
    """Within this context the column reductions that produce parameter gradients (Linear weight /
    bias gradients through ogv_gemm_wgrad, LayerNorm gamma / beta, the fused MBConv's expand / project /
    SE weight gradients) are recorded, not launched; on exit they run as batched launches on the
    current stream (ogv_reduce_flush) -- ~110 fewer launches per Model-A-7M step.  Only for a backward whose parameter gradients nothing reads before the exit:
    every .grad None at entry (set_to_none) and no parameter used twice in the graph (autograd would
    add its two partial gradients before they exist), and no gradient hooks that read them (DP bucket
    hooks).  Every side stream the backward forked must be joined into the current one (ogv's forks
    are)."""

    def __init__(self, enabled=True):
        self.enabled = bool(enabled)

    def __enter__(self):
        if self.enabled:
            if _DEFER["on"]:
                raise RuntimeError("ogv.deferred_param_reductions: already active")
            _DEFER["on"], _DEFER["keep"] = True, []
            _lib.load().ogv_reduce_defer(1)
        return self

    def __exit__(self, *exc):
        if self.enabled:
            lib = _lib.load()
            lib.ogv_reduce_defer(0)
            _DEFER["on"] = False
            try:
                check(lib.ogv_reduce_flush(_stream()), "ogv_reduce_flush")
            finally:
                _DEFER["keep"] = []
        return False


def flush_deferred_reductions():
    """Run the parameter-gradient reductions recorded so far (deferral stays on for the rest of the
    backward): the gradients of every parameter whose AccumulateGrad already ran are final after this.
    The graph-mode DP buckets call it when a bucket's last gradient is in (Trainer(dp_overlap))."""
    if _DEFER["on"]:
        check(_lib.load().ogv_reduce_flush(_stream()), "ogv_reduce_flush")


_warned_fp16 = False

# ------------------------------------------------------------------------------------------------
# live kernel probe (bench.py): HIP events on the launching stream around EVERY launch of a named
# kernel while armed, each with the launch's algorithmic HBM bytes.  (ROCm graphs
# cannot hold timing events, so the probe is used on eager launches only.)
# ------------------------------------------------------------------------------------------------
_PROBE = {"target": None, "armed": False, "recs": []}


def probe_bytes(name: str, u: dict) -> int:
    """Algorithmic bytes of one launch: every operand read once, every result written once."""
    e = u["elem"]
    if name == "outlook_fwd":   # read v [M,C] + logits [M,k*k*h], write y [M,C]
        return e * u["M"] * (2 * u["C"] + u["k"] * u["k"] * u["heads"])
    if name == "outlook_vproj":  # read x [M,C] + fp32 W [ld,C] (+ bias), write y [M,C] (+ cat [M,ld] in training;
        # the fp32-logits form: v [M,C] + fp32 logits [M, 9h rounded to 4])
        if u.get("l32"):
            saved = (e * u["C"] + 4 * _l32_ld(u["heads"], u["k"])) if u["cat"] else 0
            return e * u["M"] * 2 * u["C"] + u["M"] * saved + 4 * u["ld"] * (u["C"] + 1)
        return e * u["M"] * (2 * u["C"] + (u["ld"] if u["cat"] else 0)) + 4 * u["ld"] * (u["C"] + 1)
    if name == "outlook_vproj_bwd":  # read x [M,C], dy [M,C] + fp32 W [ld,C] (+ bias), write dcat [M,ld]
        return e * u["M"] * (2 * u["C"] + u["ld"]) + 4 * u["ld"] * (u["C"] + 1)
    if name == "grid_fwd":     # read qkv [M,3C], write out [M,C] + fp32 lse [M,h]
        return e * u["M"] * 4 * u["C"] + 4 * u["M"] * u["heads"]
    if name == "outlook_bwd":   # read dy, v, logits; write dv, dlogits (the fp32-logits form reads fp32 logits)
        nl = u["k"] * u["k"] * u["heads"]
        return e * u["M"] * (3 * u["C"] + nl) + (4 if u.get("l32") else e) * u["M"] * nl
    if name == "wgrad":         # read G [M,N], X [M,K]; write fp32 dW [N,K] (+ dbias)
        return e * u["M"] * (u["N"] + u["K"]) + 4 * u["N"] * u["K"] + (4 * u["N"] if u["bias"] else 0)
    if name in ("gemm_fwd", "sgemm", "gemm_tiled", "gemm_panel") and u.get("kind", "fwd") == "fwd":
        # read A [M,K] (+ residual [M,N]) + fp32 W [N,K] (+ bias), write out [M,N] (+ act(out) [M,N]; + the next
        # LayerNorm's output [M,N], its fp32 mean / rstd and the fp32 gamma / beta with ogv_gemm_fwd_ln)
        return (e * u["M"] * (u["K"] + u["N"] * (2 if u["res"] else 1) + (u["N"] if u.get("aout") else 0))
                + 4 * u["N"] * u["K"] + (4 * u["N"] if u["bias"] else 0)
                + ((e * u["M"] * u["N"] + 8 * u["M"] + 8 * u["N"]) if u.get("ln") else 0))
    if name in ("sgemm", "gemm_tiled", "gemm_panel"):   # dgrad: read dOut [M,N] (+ Z [M,K]) + fp32 W [N,K], write dA [M,K]
        return e * u["M"] * (u["N"] + u["K"] * (2 if u["z"] else 1)) + 4 * u["N"] * u["K"]
    raise KeyError(name)


def probe_flops(name: str, u: dict) -> int:
    """Algorithmic flops of one launch: the GEMMs 2*M*N*K (the MFMA work)."""
    if name == "outlook_fwd":
        return 18 * u["M"] * u["C"] + 45 * u["M"] * u["heads"]
    if name == "outlook_bwd":
        return 36 * u["M"] * u["C"]
    if name == "outlook_vproj":   # the projection GEMM + the aggregation
        return 2 * u["M"] * u["ld"] * u["C"] + 18 * u["M"] * u["C"] + 45 * u["M"] * u["heads"]
    if name == "outlook_vproj_bwd":   # the recomputed projection + the aggregation backward
        return 2 * u["M"] * u["ld"] * u["C"] + 36 * u["M"] * u["C"] + 45 * u["M"] * u["heads"]
    if name == "grid_fwd":
        return 4 * u["M"] * u["N"] * u["C"]
    return 2 * u["M"] * u["N"] * u["K"]


def probe_arm(target: str):
    if torch.cuda.is_available() and torch.cuda.is_current_stream_capturing():
        raise RuntimeError("ogv probe: timing events cannot be recorded into a ROCm graph")
    _PROBE["target"], _PROBE["armed"] = target, True


def probe_disarm():
    _PROBE["armed"] = False


class _probe:
    """Events bracket the launch on its stream; a ~40 us device-side spin queued in front keeps the
    GPU behind the host, so the interval is the kernel's own duration, not host launch latency."""

    def __init__(self, name, units, when=True):
        self.on = _PROBE["armed"] and _PROBE["target"] == name and bool(when)
        if self.on:
            self.e0 = torch.cuda.Event(enable_timing=True)
            self.e1 = torch.cuda.Event(enable_timing=True)
            self.nbytes = probe_bytes(name, units)
            self.nflops = probe_flops(name, units)
            self.units = units

    def __enter__(self):
        if self.on:
            check(_lib.load().ogv_gpu_sleep(40, _stream()), "ogv_gpu_sleep")
            self.e0.record()
        return self

    def __exit__(self, *a):
        if self.on:
            self.e1.record()
            _PROBE["recs"].append((self.e0, self.e1, self.nbytes, self.nflops, self.units))
        return False


def _empty_pair_ms(reps: int = 16) -> float:
    """What an event pair adds around a device spin of KNOWN length (ogv_gpu_sleep: a wall-clock loop
    of 20 us, the same 40 us spin in front): median interval minus 20 us.  REPORTED ONLY, not
    subtracted: around a real kernel this cost overlaps the kernel, and the raw probe interval
    equals rocprofv3's kernel duration (27.67 vs 27.67 us per panel launch at HEAD, 27.58 vs 26.94 at
    the round-3 head pass), while subtracting it -- or the empty-pair interval of round 2 -- read
    10-14% under rocprof (profiles/r03_final_probe_vs_trace.txt).  The raw interval is therefore a
    conservative bound: achieved bytes / raw interval <= the kernel's true rate."""
    lib = _lib.load()
    pairs = []
    spin_us = 20
    for _ in range(reps):
        check(lib.ogv_gpu_sleep(40, _stream()), "ogv_gpu_sleep")
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        check(lib.ogv_gpu_sleep(spin_us, _stream()), "ogv_gpu_sleep")
        b.record()
        pairs.append((a, b))
    torch.cuda.synchronize()
    ms = sorted(a.elapsed_time(b) for a, b in pairs)
    return max(ms[len(ms) // 2] - spin_us * 1e-3, 0.0)


def probe_results():
    """{n, avg_ms, bytes_per_launch, achieved_GBs, event_overhead_ms} over the recorded launches
    (raw event intervals: see _empty_pair_ms), or None."""
    recs = _PROBE["recs"]
    if not recs:
        return None
    torch.cuda.synchronize()
    ovh = _empty_pair_ms()
    ms = [max(a.elapsed_time(b), 1e-6) for a, b, _, _, _ in recs]
    dump = os.environ.get("OGV_PROBE_DUMP")
    if dump:   # per-launch table: shape, algorithmic bytes, time, GB/s
        with open(dump, "a") as f:
            for (a, b, nb, nf, u), t in zip(recs, ms):
                f.write(f"{_PROBE['target']} {u.get('kind', 'fwd')} M={u.get('M')} N={u.get('N')} K={u.get('K')} "
                        f"z={int(bool(u.get('z')))} res={int(bool(u.get('res')))} bytes={nb} us={1e3 * t:.2f} "
                        f"GBs={nb / (t * 1e-3) / 1e9:.0f}\n")
    nbytes = sum(r[2] for r in recs)
    nflops = sum(r[3] for r in recs)
    tot = sum(ms)
    return {"n": len(recs), "avg_ms": tot / len(recs), "bytes_per_launch": nbytes / len(recs),
            "achieved_GBs": nbytes / (tot * 1e-3) / 1e9 if tot > 0 else None, "event_overhead_ms": ovh,
            "flops_per_launch": nflops / len(recs),
            "achieved_TFLOPs": nflops / (tot * 1e-3) / 1e12 if tot > 0 else None}


def probe_reset():
    _PROBE["recs"] = []


# ------------------------------------------------------------------------------------------------
# step census (bench.py roofline.step): HIP events around EVERY C-ABI op of one eager step, each
# with the algorithmic bytes / flops of the kernels it launches (each kernel reads its operands once
# and writes its results once: DESIGN.md §3), so Σ roofline time / Σ measured time
# can be reported over the whole step.  Forks are off while armed (every op on one stream, where
# its events are).
# ------------------------------------------------------------------------------------------------
_CENSUS = {"armed": False, "recs": []}


def _serial() -> bool:
    return _PROBE["armed"] or _CENSUS["armed"]


def op_cost(name: str, u: dict):
    """(algorithmic HBM bytes, flops) of one C-ABI op.  s = activation element size; M rows of C
    channels; weights are fp32 [N, K]."""
    s = u["elem"]
    M = u.get("M", 0)
    if name == "gemm_fwd":
        return probe_bytes("gemm_fwd", u), 2 * M * u["N"] * u["K"]
    if name == "gemm_dgrad":
        return probe_bytes("sgemm", dict(u, kind="dgrad")), 2 * M * u["N"] * u["K"]
    if name == "gemm_wgrad":
        return probe_bytes("wgrad", u), 2 * M * u["N"] * u["K"]
    C = u.get("C", 0)
    if name == "layernorm_fwd":      # read x, write y (+ fp32 mean / rstd)
        return s * 2 * M * C + 8 * M, 8 * M * C
    if name == "layernorm_bwd":      # read dy, x (+ dres), write dx (+ fp32 mean / rstd, gamma / beta partials)
        return s * M * C * (4 if u.get("dres") else 3) + 8 * M + 8 * C, 10 * M * C
    if name in ("outlook_fwd", "outlook_bwd", "outlook_vproj", "outlook_vproj_bwd", "grid_fwd"):
        return probe_bytes(name, u), probe_flops(name, u)
    if name == "grid_bwd":           # read dO, qkv, O (+ lse), write dqkv (+ delta)
        return s * M * 8 * C + 8 * M * u["heads"], 8 * M * u["N"] * C
    if name == "dwconv_fwd":         # read x, write y
        return s * (M + u["Mo"]) * C + 36 * C, 18 * u["Mo"] * C
    if name == "dwconv_bwd":         # dgrad: read dy, write dx; wgrad: read dy, x
        return s * 2 * (M + u["Mo"]) * C + 36 * C, 36 * u["Mo"] * C
    if name in ("mbconv_fwd", "mbconv_bwd"):
        m, se, B = u["mid"], u["se"], u["B"]
        w = 4 * (2 * m * C + 9 * m + 2 * m * se)                   # fp32 weights
        if name == "mbconv_fwd":     # expand (x -> e), dw (e -> d), SE pool (d), project (d -> p), BN3 + residual (p, x -> out)
            return s * M * (5 * C + 5 * m) + w, 2 * M * m * C * 2 + 18 * M * m
        # BN3 reduce + apply, project dgrad + wgrad, SE reduce, dw wgrad + dgrad with the BN2 backward in its
        # staging (reads dA3 and d: dd is never stored), BN1 apply, expand wgrad + dgrad (+ the residual)
        return s * M * (11 * C + 15 * m) + 2 * w, 2 * M * m * C * 4 + 36 * M * m
    if name in ("convbn_fwd", "convbn_bwd"):
        Mi, Mo, Ci, Co = M, u["Mo"], u["Cin"], u["Cout"]
        f = 2 * Mo * Co * 9 * Ci
        if name == "convbn_fwd":     # conv (x -> y), BN apply + act (y -> out)
            return s * (Mi * Ci + 3 * Mo * Co) + 4 * 9 * Ci * Co, f
        # BN reduce (dout, y), BN apply (dout, y -> dy), wgrad (dy, x), dgrad (dy -> dx)
        return s * (7 * Mo * Co + 2 * Mi * Ci) + 8 * 9 * Ci * Co, 2 * f
    if name in ("bn_act_fwd", "bn_act_bwd") and u.get("head"):   # the head's BN + pool: x once (+ dx)
        return (s * M * C + 8 * (M // max(1, u.get("hw", 1))) * C, 4 * M * C) if name == "bn_act_fwd" else \
            (2 * s * M * C, 6 * M * C)
    if name == "bn_act_fwd":         # (statistics pass over x when training) + apply
        return s * M * C * (3 if u.get("train") else 2), 4 * M * C
    if name == "bn_act_bwd":         # reduce (dout, x) + apply (dout, x -> dx)
        return s * M * C * 5, 8 * M * C
    if name == "ce_fwd":             # read fp32 logits + int64 labels, write the per-row logsumexp
        return 4 * u["B"] * u["K"] + 12 * u["B"], 4 * u["B"] * u["K"]
    if name == "ce_bwd":             # read logits, labels, logsumexp; write dlogits
        return 8 * u["B"] * u["K"] + 12 * u["B"], 4 * u["B"] * u["K"]
    raise KeyError(name)


def census_arm():
    if torch.cuda.is_available() and torch.cuda.is_current_stream_capturing():
        raise RuntimeError("ogv census: timing events cannot be recorded into a ROCm graph")
    _CENSUS["armed"] = True


def census_disarm():
    _CENSUS["armed"] = False


def census_reset():
    _CENSUS["recs"] = []


class _census:
    """One C-ABI op of the census: events around it on the current stream (same device spin in front
    as the probes), recorded with its name, algorithmic bytes and flops."""

    def __init__(self, name, units):
        self.on = _CENSUS["armed"]
        if self.on:
            self.name = name
            self.nbytes, self.nflops = op_cost(name, units)
            self.e0 = torch.cuda.Event(enable_timing=True)
            self.e1 = torch.cuda.Event(enable_timing=True)

    def __enter__(self):
        if self.on:
            check(_lib.load().ogv_gpu_sleep(40, _stream()), "ogv_gpu_sleep")
            self.e0.record()
        return self

    def __exit__(self, *a):
        if self.on:
            self.e1.record()
            _CENSUS["recs"].append((self.name, self.e0, self.e1, self.nbytes, self.nflops))
        return False


def census_results(hbm_gbs: float, mfma_tflops: float):
    """Per-op-family table and totals of the recorded ops: algorithmic bytes / flops, roofline time
    max(bytes / HBM peak, flops / MFMA peak), measured time (raw event intervals, see
    _empty_pair_ms)."""
    recs = _CENSUS["recs"]
    if not recs:
        return None
    torch.cuda.synchronize()
    ovh = _empty_pair_ms()
    fam = {}
    for name, a, b, nb, nf in recs:
        ms = max(a.elapsed_time(b), 1e-6)
        bound = max(nb / (hbm_gbs * 1e9), nf / (mfma_tflops * 1e12)) * 1e3
        d = fam.setdefault(name, {"launches": 0, "bytes": 0, "flops": 0, "bound_ms": 0.0, "measured_ms": 0.0})
        d["launches"] += 1
        d["bytes"] += nb
        d["flops"] += nf
        d["bound_ms"] += bound
        d["measured_ms"] += ms
    for d in fam.values():
        d["frac"] = round(d["bound_ms"] / d["measured_ms"], 4)
        d["bound_ms"] = round(d["bound_ms"], 4)
        d["measured_ms"] = round(d["measured_ms"], 4)
    tb = sum(d["bound_ms"] for d in fam.values())
    tm = sum(d["measured_ms"] for d in fam.values())
    return {"ops": len(recs), "bytes": sum(d["bytes"] for d in fam.values()),
            "flops": sum(d["flops"] for d in fam.values()), "bound_ms": round(tb, 4), "measured_ms": round(tm, 4),
            "frac": round(tb / tm, 4), "event_overhead_ms": round(ovh, 5),
            "families": dict(sorted(fam.items(), key=lambda kv: -kv[1]["measured_ms"]))}


def compute_dtype(x: torch.Tensor) -> torch.dtype:
    """Activation dtype for the kernels: the autocast dtype inside an autocast region (fp16 is
    computed as bf16 on MI355X), else the input dtype (fp32 or bf16)."""
    global _warned_fp16
    if x.is_cuda and torch.is_autocast_enabled("cuda"):
        d = torch.get_autocast_dtype("cuda")
    else:
        d = x.dtype
    if d == torch.float16:
        if not _warned_fp16:
            warnings.warn("ogv: fp16 autocast requested; the MI355X kernels compute in bf16 instead")
            _warned_fp16 = True
        d = torch.bfloat16
    if d not in (torch.float32, torch.bfloat16):
        raise TypeError(f"ogv: unsupported activation dtype {d}")
    return d


def f32(p):
    """Parameters go to the kernels as fp32 (the AMP master copy); differentiable cast if needed."""
    if p is None:
        return None
    return p if p.dtype == torch.float32 else p.float()


# ------------------------------------------------------------------------------------------------
# layout helpers
# ------------------------------------------------------------------------------------------------
def nchw_to_rows(x: torch.Tensor) -> torch.Tensor:
    """[B,C,H,W] -> [B*H*W, C] view (copies once into channels_last if the input is not)."""
    B, C, H, W = x.shape
    if not x.is_contiguous(memory_format=torch.channels_last):
        x = x.contiguous(memory_format=torch.channels_last)
    return x.permute(0, 2, 3, 1).reshape(B * H * W, C)


def rows_to_nchw(y: torch.Tensor, B: int, H: int, W: int) -> torch.Tensor:
    """[B*H*W, C] -> [B,C,H,W] channels_last view (no copy)."""
    return y.view(B, H, W, y.shape[-1]).permute(0, 3, 1, 2)


def _rows_contig(t: torch.Tensor) -> torch.Tensor:
    if t.stride(-1) != 1 or t.stride(0) < t.shape[-1] or t.data_ptr() % 16:
        t = t.contiguous()
    return t


# ------------------------------------------------------------------------------------------------
# Linear / 1x1 conv on rows:  out = res + rs[b] * (act_in(x) @ W^T + b)
# ------------------------------------------------------------------------------------------------
class _Linear(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x2d, w2d, bias, residual, row_scale, rps, act_in, x_act):
        # x_act (optional): act_in(x2d) already materialised by the producing GEMM (ogv_gemm_fwd_act):
        # the product and the weight gradient read it with no prologue; x2d (the pre-activation)
        # only feeds the data gradient's act'(x2d) epilogue
        lib = _lib.load()
        M, K = x2d.shape
        N = w2d.shape[0]
        out = torch.empty((M, N), dtype=x2d.dtype, device=x2d.device)
        a_in = x_act if x_act is not None else x2d
        act_fwd = None if x_act is not None else act_in
        units = dict(M=M, N=N, K=K, elem=x2d.element_size(), res=residual is not None, bias=bias is not None)
        route = lib.ogv_gemm_stream_route(0, M, N, K, ACT[act_fwd]) if _PROBE["armed"] else -1
        bf = x2d.dtype == torch.bfloat16
        with _probe("gemm_fwd", units), _probe("sgemm", units, when=bf and route == 1), \
                _probe("gemm_panel", units, when=bf and route == 2), _probe("gemm_tiled", units, when=bf and route == 0), \
                _census("gemm_fwd", units):
            check(lib.ogv_gemm_fwd(_ptr(a_in), a_in.stride(0), _ptr(w2d), _ptr(bias), _ptr(residual), _ptr(row_scale),
                                   int(rps), _ptr(out), N, M, N, K, ACT[act_fwd], _dt(x2d), _stream()), "ogv_gemm_fwd")
        ctx.save_for_backward(x2d, w2d, row_scale, x_act)
        ctx.meta = (M, N, K, int(rps), ACT[act_in], bias is not None, residual is not None)
        return out

    @staticmethod
    def backward(ctx, dout):
        x2d, w2d, rs, x_act = ctx.saved_tensors
        M, N, K, rps, act, has_bias, has_res = ctx.meta
        dout = dout.to(x2d.dtype).contiguous()
        want_dx = ctx.needs_input_grad[0]
        want_dw = ctx.needs_input_grad[1] or (has_bias and ctx.needs_input_grad[2])
        dx, dw, db = _linear_bwd(dout, x2d, w2d, rs, rps, act, has_bias, want_dx, want_dw, x_act)
        dres = dout if has_res and ctx.needs_input_grad[3] else None
        return dx, dw, db, dres, None, None, None, None


class _LinearAct(torch.autograd.Function):
    """First Linear of a Linear -> act -> Linear pair: (Z, act(Z)) from one GEMM launch
    (ogv_gemm_fwd_act).  act(Z) is a non-differentiable by-product: the second layer, given it as
    x_act, returns its input gradient with respect to Z (act'(Z) in its data-gradient epilogue)."""

    @staticmethod
    def forward(ctx, x2d, w2d, bias, act):
        lib = _lib.load()
        M, K = x2d.shape
        N = w2d.shape[0]
        out = torch.empty((M, N), dtype=x2d.dtype, device=x2d.device)
        aout = torch.empty((M, N), dtype=x2d.dtype, device=x2d.device)
        units = dict(M=M, N=N, K=K, elem=x2d.element_size(), res=False, bias=bias is not None, aout=True)
        with _probe("gemm_fwd", units), _census("gemm_fwd", units):
            check(lib.ogv_gemm_fwd_act(_ptr(x2d), x2d.stride(0), _ptr(w2d), _ptr(bias), _ptr(out), N, _ptr(aout), N,
                                       M, N, K, ACT[act], _dt(x2d), _stream()), "ogv_gemm_fwd_act")
        ctx.mark_non_differentiable(aout)
        ctx.set_materialize_grads(False)   # no zero-filled gradient for aout (an [M, N] fill per call)
        ctx.save_for_backward(x2d, w2d)
        ctx.meta = bias is not None
        return out, aout

    @staticmethod
    def backward(ctx, dout, _daout):
        x2d, w2d = ctx.saved_tensors
        has_bias = ctx.meta
        if dout is None:   # Z unused downstream (possible once grads are not materialised)
            return None, None, None, None
        dout = dout.to(x2d.dtype).contiguous()
        want_dx = ctx.needs_input_grad[0]
        want_dw = ctx.needs_input_grad[1] or (has_bias and ctx.needs_input_grad[2])
        dx, dw, db = _linear_bwd(dout, x2d, w2d, None, 1, 0, has_bias, want_dx, want_dw)
        return dx, dw, db, None


def _linear_bwd(dout, x2d, w2d, rs, rps, act, has_bias, want_dx, want_dw, x_act=None):
    """(dx, dW, dbias) of out = rs * (act(x) @ W^T + b) from dout; the weight gradient forks onto the
    side stream when both are wanted.  With x_act (= act(x) materialised) the weight gradient reads it
    with no prologue."""
    lib = _lib.load()
    M, K = x2d.shape
    N = w2d.shape[0]
    dt = _dt(x2d)
    dx = dw = db = None
    xw, wact = (x_act, 0) if x_act is not None else (x2d, act)
    if want_dx:
        dx = torch.empty((M, K), dtype=x2d.dtype, device=x2d.device)
        ws_d = _ws(lib.ogv_gemm_dgrad_ws_bytes(N, K), x2d.device)
    if want_dw:
        dw = torch.empty((N, K), dtype=torch.float32, device=x2d.device)
        db = torch.empty((N,), dtype=torch.float32, device=x2d.device) if has_bias else None
        ws_w = _ws(lib.ogv_gemm_wgrad_ws_bytes(M, N, K), x2d.device, deferrable=True)
    # dgrad and wgrad are independent: the weight gradient runs on a side stream (forked from and
    # joined back into the current one, also inside a captured graph) so the two latency-bound
    # GEMMs overlap.
    # (below ~_FORK_MIN_WORK the fork/join latency (~10 us per cross-stream edge) outweighs the overlap)
    # (while a probe is armed everything stays on the current stream, where its events are)
    fork = (_FORK and want_dx and want_dw and M * (N + K) >= _FORK_MIN_WORK and not _serial()
            and (_FORK_ACT or not act))
    with _fork(fork, dout, xw, rs, dw, db, ws_w if want_dw else None) as side:
        if want_dw:
            wu = dict(M=M, N=N, K=K, elem=x2d.element_size(), bias=has_bias)
            with _probe("wgrad", wu, when=x2d.dtype == torch.bfloat16), _census("gemm_wgrad", wu):
                check(lib.ogv_gemm_wgrad(_ptr(dout), N, _ptr(xw), xw.stride(0), _ptr(rs), rps, _ptr(dw), _ptr(db),
                                         M, N, K, wact, _ptr(ws_w), dt, side), "ogv_gemm_wgrad")
        if want_dx:
            route = lib.ogv_gemm_stream_route(1, M, N, K, act) if _PROBE["armed"] else -1
            du = dict(kind="dgrad", M=M, N=N, K=K, elem=x2d.element_size(), z=bool(act))
            bf = x2d.dtype == torch.bfloat16
            with _probe("sgemm", du, when=bf and route == 1), _probe("gemm_panel", du, when=bf and route == 2), \
                    _probe("gemm_tiled", du, when=bf and route == 0), _census("gemm_dgrad", du):
                check(lib.ogv_gemm_dgrad(_ptr(dout), N, _ptr(w2d), _ptr(x2d) if act else None, x2d.stride(0),
                                         _ptr(rs), rps, _ptr(dx), K, M, N, K, act, _ptr(ws_d), dt, _stream()),
                      "ogv_gemm_dgrad")
    return dx, dw, db


class _LinearLNPair(torch.autograd.Function):
    """(LN(out), out) with out = residual + rs * (x2d @ W^T + b): a pre-norm block's producing Linear and the
    residual stream's next LayerNorm (Outlook_Block.py:58-60, Out_Grid_Block.py:100-102) in ONE launch
    (ogv_gemm_fwd_ln: the LN in the GEMM epilogue; where the kernel declines, ogv_gemm_fwd + ogv_layernorm_fwd).
    out is the next block's residual (its gradient arrives here and is summed inside the LN backward, as
    _LayerNormPair does); the backward is the LN backward then the Linear's."""

    @staticmethod
    def forward(ctx, x2d, w2d, bias, residual, row_scale, rps, gamma, beta, eps):
        lib = _lib.load()
        M, K = x2d.shape
        N = w2d.shape[0]
        dt = _dt(x2d)
        out = torch.empty((M, N), dtype=x2d.dtype, device=x2d.device)
        y = torch.empty((M, N), dtype=x2d.dtype, device=x2d.device)
        mean = torch.empty((M,), dtype=torch.float32, device=x2d.device)
        rstd = torch.empty((M,), dtype=torch.float32, device=x2d.device)
        units = dict(M=M, N=N, K=K, elem=x2d.element_size(), res=residual is not None, bias=bias is not None, ln=True)
        with _census("gemm_fwd", units):
            rc = lib.ogv_gemm_fwd_ln(_ptr(x2d), x2d.stride(0), _ptr(w2d), _ptr(bias), _ptr(residual), _ptr(row_scale),
                                     int(rps), _ptr(out), N, _ptr(y), _ptr(gamma), _ptr(beta), float(eps), _ptr(mean),
                                     _ptr(rstd), M, N, K, dt, _stream())
        if rc == _lib.OGV_ERR_UNSUPPORTED:    # nothing launched: the two ops
            units["ln"] = False
            with _census("gemm_fwd", units):
                check(lib.ogv_gemm_fwd(_ptr(x2d), x2d.stride(0), _ptr(w2d), _ptr(bias), _ptr(residual), _ptr(row_scale),
                                       int(rps), _ptr(out), N, M, N, K, ACT[None], dt, _stream()), "ogv_gemm_fwd")
            with _census("layernorm_fwd", dict(M=M, C=N, elem=x2d.element_size())):
                check(lib.ogv_layernorm_fwd(_ptr(out), _ptr(gamma), _ptr(beta), _ptr(y), _ptr(mean), _ptr(rstd), M, N,
                                            float(eps), dt, _stream()), "ogv_layernorm_fwd")
        else:
            check(rc, "ogv_gemm_fwd_ln")
        ctx.save_for_backward(x2d, w2d, row_scale, out, gamma, mean, rstd)
        ctx.meta = (int(rps), bias is not None, residual is not None, beta is not None)
        return y, out

    @staticmethod
    def backward(ctx, dy, dres):
        lib = _lib.load()
        x2d, w2d, rs, out, gamma, mean, rstd = ctx.saved_tensors
        rps, has_bias, has_res, has_beta = ctx.meta
        M, N = out.shape
        dgamma = dbeta = None
        if dy is None:
            dtot = dres.to(x2d.dtype).contiguous()
        else:
            dy = dy.to(x2d.dtype).contiguous()
            if dres is not None:
                dres = dres.to(x2d.dtype).contiguous()
            dtot = torch.empty_like(out)
            dgamma = torch.empty((N,), dtype=torch.float32, device=x2d.device)
            dbeta = torch.empty((N,), dtype=torch.float32, device=x2d.device) if has_beta else None
            ws = _ws(lib.ogv_layernorm_bwd_ws_bytes(M, N), x2d.device, deferrable=True)
            with _census("layernorm_bwd", dict(M=M, C=N, elem=x2d.element_size(), dres=dres is not None)):
                check(lib.ogv_layernorm_bwd(_ptr(dy), _ptr(out), _ptr(gamma), _ptr(mean), _ptr(rstd), _ptr(dres),
                                            _ptr(dtot), _ptr(dgamma), _ptr(dbeta), _ptr(ws), M, N, _dt(x2d), _stream()),
                      "ogv_layernorm_bwd")
        want_dx = ctx.needs_input_grad[0]
        want_dw = ctx.needs_input_grad[1] or (has_bias and ctx.needs_input_grad[2])
        dx, dw, db = _linear_bwd(dtot, x2d, w2d, rs, rps, 0, has_bias, want_dx, want_dw)
        dresid = dtot if has_res and ctx.needs_input_grad[3] else None
        return dx, dw, db, dresid, None, None, dgamma, dbeta, None


def linear_rows_ln(x2d, weight, bias, residual, row_scale, rps, gamma, beta, eps):
    """(LN(out), out), out = residual + rs * (x2d @ W^T + b): see _LinearLNPair.  x2d [M, K] bf16 / fp32 rows,
    weight [N, K] (or [N, K, 1, 1]), gamma / beta [N] (the LayerNorm's affine, beta may be None)."""
    require_device(x2d, weight, bias, residual, row_scale, gamma, beta, what="ogv.linear_ln")
    x2d = _rows_contig(x2d)
    w2d = f32(weight).reshape(weight.shape[0], -1)
    if w2d.shape[1] != x2d.shape[1]:
        raise ValueError(f"ogv.linear_ln: weight in_features {w2d.shape[1]} != input features {x2d.shape[1]}")
    if residual is not None:
        residual = residual.to(x2d.dtype).contiguous()
        if residual.shape != (x2d.shape[0], w2d.shape[0]):
            raise ValueError("ogv.linear_ln: residual shape mismatch")
    if row_scale is not None:
        row_scale = row_scale.float().contiguous()
    g = f32(gamma).contiguous()
    b = f32(beta).contiguous() if beta is not None else torch.zeros_like(g)
    return _LinearLNPair.apply(x2d, w2d, f32(bias), residual, row_scale, int(rps), g, b, float(eps))


# knob: OGV_LN_EPI=1 runs the residual stream's next LayerNorm in the producing Linear's epilogue where the
# kernel takes the shape (opt-in: no step-time gain measured at 7M, profiles/r06k_ln_epi_ab.log; default off
# keeps every LayerNorm a launch of its own)
_LN_EPI = os.environ.get("OGV_LN_EPI", "0") == "1"


def ln_epilogue_params(norm, *mods):
    """(gamma, beta, eps) when `norm` -- the residual stream's next LayerNorm (ogv.layers.LayerNorm or
    LayerNorm2d) -- can run in the producing Linear's epilogue: no hooks on it or on the producing modules,
    a 1-D affine normalisation.  None otherwise (the caller runs the Linear, then norm.forward_pair)."""
    if not _LN_EPI or norm is None:
        return None
    ln = getattr(norm, "ln", norm)       # LayerNorm2d wraps an nn.LayerNorm as .ln
    for m in (norm, ln) + mods:
        if m._forward_hooks or m._forward_pre_hooks:
            return None
    if not isinstance(ln, torch.nn.LayerNorm) or len(ln.normalized_shape) != 1 or ln.weight is None:
        return None
    return ln.weight, ln.bias, ln.eps


# knob: OGV_MAT_ACT=0 keeps the activation between two Linears as the second GEMM's prologue
_MAT_ACT = os.environ.get("OGV_MAT_ACT", "1") != "0"


def materialise_act(x: torch.Tensor, *mods) -> bool:
    """Whether a Linear -> act -> Linear pair should run as ogv_gemm_fwd_act + a prologue-free second
    GEMM: bf16 compute, autograd recording (the materialised activation is kept for the weight
    gradient; inference keeps the prologue form and its smaller footprint), no hooks on either
    Linear (their outputs must stay the reference's single tensors)."""
    if not _MAT_ACT or not torch.is_grad_enabled() or compute_dtype(x) != torch.bfloat16:
        return False
    return not any(m._forward_hooks or m._forward_pre_hooks for m in mods)


def linear_rows(x2d, weight, bias=None, residual=None, row_scale=None, rps=1, act_in=None, x_act=None):
    """x2d [M,K] (row stride >= K), weight [N,K] (or [N,K,1,1]), residual [M,N].  x_act: act_in(x2d)
    as materialised by linear_rows_act (same shape)."""
    require_device(x2d, weight, bias, residual, row_scale, x_act, what="ogv.linear")
    x2d = _rows_contig(x2d)
    w2d = f32(weight).reshape(weight.shape[0], -1)
    if w2d.shape[1] != x2d.shape[1]:
        raise ValueError(f"ogv.linear: weight in_features {w2d.shape[1]} != input features {x2d.shape[1]}")
    if residual is not None:
        residual = residual.to(x2d.dtype).contiguous()
        if residual.shape != (x2d.shape[0], w2d.shape[0]):
            raise ValueError("ogv.linear: residual shape mismatch")
    if row_scale is not None:
        row_scale = row_scale.float().contiguous()
    if x_act is not None:
        if act_in is None or x_act.shape != x2d.shape or x_act.dtype != x2d.dtype:
            raise ValueError("ogv.linear: x_act must be act_in(x2d) with x2d's shape and dtype")
        x_act = _rows_contig(x_act)
    return _Linear.apply(x2d, w2d, f32(bias), residual, row_scale, int(rps), act_in, x_act)


def linear_rows_act(x2d, weight, bias, act):
    """(Z, act(Z)) = (x2d @ W^T + b, its activation), both [M, N] bf16, one launch.  act(Z) carries no
    gradient of its own: pass it to the next linear_rows as x_act with act_in=act and Z as x2d."""
    require_device(x2d, weight, bias, what="ogv.linear_act")
    x2d = _rows_contig(x2d)
    if x2d.dtype != torch.bfloat16:
        raise ValueError("ogv.linear_act: bf16 only")
    w2d = f32(weight).reshape(weight.shape[0], -1)
    if w2d.shape[1] != x2d.shape[1]:
        raise ValueError(f"ogv.linear_act: weight in_features {w2d.shape[1]} != input features {x2d.shape[1]}")
    return _LinearAct.apply(x2d, w2d, f32(bias), act)


# ------------------------------------------------------------------------------------------------
# Training loss: cross-entropy with label smoothing (src/training/one_epoch_train.py:96)
# ------------------------------------------------------------------------------------------------
class _CrossEntropyLS(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, target, ls, found, bad):
        lib = _lib.load()
        B, K = logits.shape
        loss = torch.empty((), dtype=torch.float32, device=logits.device)
        ws = torch.empty((lib.ogv_ce_ls_ws_bytes(B) // 4,), dtype=torch.float32, device=logits.device)
        with _census("ce_fwd", dict(B=B, K=K, elem=4)):
            check(lib.ogv_ce_ls_fwd(_ptr(logits), _ptr(target), B, K, float(ls), _ptr(loss), _ptr(ws),
                                    _ptr(found) if found is not None else None, _ptr(bad) if bad is not None else None,
                                    _stream()), "ogv_ce_ls_fwd")
        ctx.save_for_backward(logits, target, ws)
        ctx.ls = float(ls)
        return loss

    @staticmethod
    def backward(ctx, g):
        lib = _lib.load()
        logits, target, ws = ctx.saved_tensors
        B, K = logits.shape
        g = g.float().contiguous()
        dz = torch.empty_like(logits)
        with _census("ce_bwd", dict(B=B, K=K, elem=4)):
            check(lib.ogv_ce_ls_bwd(_ptr(logits), _ptr(target), _ptr(ws), _ptr(g), B, K, ctx.ls, _ptr(dz), _stream()),
                  "ogv_ce_ls_bwd")
        return dz, None, None, None, None


def cross_entropy_ls(logits, target, label_smoothing=0.0, found=None, bad_labels=None):
    """F.cross_entropy(logits.float(), target, label_smoothing=ls) (mean, ignore_index -100) on the
    native kernels: logits [B, K] (cast to contiguous fp32), target [B] int64 class indices.  found: an
    optional fp32 [1] device tensor that receives !isfinite(loss) from the same launch (the training
    step's found_inf guard).  A label outside [0, K) gives a NaN loss instead of torch's raise (a raise
    needs a device sync); bad_labels: an optional fp32 [1] device counter the same launch adds the number
    of such rows to, so the caller can raise when it next syncs (Trainer does)."""
    require_device(logits, target, found, bad_labels, what="ogv.cross_entropy")
    if logits.dim() != 2 or target.dim() != 1 or target.shape[0] != logits.shape[0]:
        raise ValueError(f"ogv.cross_entropy: logits [B, K] and target [B] expected, got {tuple(logits.shape)} "
                         f"and {tuple(target.shape)}")
    if target.dtype != torch.int64:
        raise ValueError("ogv.cross_entropy: class-index targets (int64) only")
    if not 0.0 <= label_smoothing <= 1.0:
        raise ValueError(f"ogv.cross_entropy: label_smoothing {label_smoothing} not in [0, 1]")
    return _CrossEntropyLS.apply(logits.float().contiguous(), target.contiguous(), float(label_smoothing), found,
                                 bad_labels)


# ------------------------------------------------------------------------------------------------
# LayerNorm over the last (contiguous) dim
# ------------------------------------------------------------------------------------------------
class _LayerNorm(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x2d, gamma, beta, eps):
        lib = _lib.load()
        M, C = x2d.shape
        y = torch.empty_like(x2d)
        mean = torch.empty((M,), dtype=torch.float32, device=x2d.device)
        rstd = torch.empty((M,), dtype=torch.float32, device=x2d.device)
        with _census("layernorm_fwd", dict(M=M, C=C, elem=x2d.element_size())):
            check(lib.ogv_layernorm_fwd(_ptr(x2d), _ptr(gamma), _ptr(beta), _ptr(y), _ptr(mean), _ptr(rstd), M, C,
                                        float(eps), _dt(x2d), _stream()), "ogv_layernorm_fwd")
        ctx.save_for_backward(x2d, gamma, mean, rstd)
        ctx.affine = (gamma is not None, beta is not None)
        return y

    @staticmethod
    def backward(ctx, dy):
        lib = _lib.load()
        x2d, gamma, mean, rstd = ctx.saved_tensors
        M, C = x2d.shape
        dy = dy.to(x2d.dtype).contiguous()
        dx = torch.empty_like(x2d)
        dgamma = torch.empty((C,), dtype=torch.float32, device=x2d.device) if ctx.affine[0] else None
        dbeta = torch.empty((C,), dtype=torch.float32, device=x2d.device) if ctx.affine[1] else None
        ws = _ws(lib.ogv_layernorm_bwd_ws_bytes(M, C), x2d.device, deferrable=True)
        with _census("layernorm_bwd", dict(M=M, C=C, elem=x2d.element_size(), dres=False)):
            check(lib.ogv_layernorm_bwd(_ptr(dy), _ptr(x2d), _ptr(gamma), _ptr(mean), _ptr(rstd), None, _ptr(dx),
                                        _ptr(dgamma), _ptr(dbeta), _ptr(ws), M, C, _dt(x2d), _stream()),
                  "ogv_layernorm_bwd")
        return dx, dgamma, dbeta, None


class _LayerNormPair(torch.autograd.Function):
    """(LN(x), x) for a pre-norm residual block x + f(LN(x)).  The second output is x itself (a
    view), used as the block's residual, so its gradient arrives HERE and is summed into dx inside
    the LN backward kernel instead of by a separate autograd accumulation add."""

    @staticmethod
    def forward(ctx, x2d, gamma, beta, eps):
        y = _LayerNorm.forward(ctx, x2d, gamma, beta, eps)
        return y, x2d.view_as(x2d)

    @staticmethod
    def backward(ctx, dy, dres):
        lib = _lib.load()
        x2d, gamma, mean, rstd = ctx.saved_tensors
        M, C = x2d.shape
        if dy is None:
            return dres, None, None, None
        dy = dy.to(x2d.dtype).contiguous()
        if dres is not None:
            dres = dres.to(x2d.dtype).contiguous()
        dx = torch.empty_like(x2d)
        dgamma = torch.empty((C,), dtype=torch.float32, device=x2d.device) if ctx.affine[0] else None
        dbeta = torch.empty((C,), dtype=torch.float32, device=x2d.device) if ctx.affine[1] else None
        ws = _ws(lib.ogv_layernorm_bwd_ws_bytes(M, C), x2d.device, deferrable=True)
        with _census("layernorm_bwd", dict(M=M, C=C, elem=x2d.element_size(), dres=dres is not None)):
            check(lib.ogv_layernorm_bwd(_ptr(dy), _ptr(x2d), _ptr(gamma), _ptr(mean), _ptr(rstd), _ptr(dres), _ptr(dx),
                                        _ptr(dgamma), _ptr(dbeta), _ptr(ws), M, C, _dt(x2d), _stream()),
                  "ogv_layernorm_bwd")
        return dx, dgamma, dbeta, None


def layer_norm_rows(x2d, gamma, beta, eps):
    require_device(x2d, gamma, beta, what="ogv.layer_norm")
    x2d = x2d.contiguous()
    return _LayerNorm.apply(x2d, f32(gamma), f32(beta), float(eps))


def layer_norm_rows_pair(x2d, gamma, beta, eps):
    """(LN(x2d), x2d-as-residual): see _LayerNormPair."""
    require_device(x2d, gamma, beta, what="ogv.layer_norm")
    x2d = x2d.contiguous()
    return _LayerNormPair.apply(x2d, f32(gamma), f32(beta), float(eps))


# ------------------------------------------------------------------------------------------------
# Outlook aggregation (softmax over k*k + zero-padded neighbourhood gather)
# ------------------------------------------------------------------------------------------------
def _outlook_bwd(dy, v2d, ldv, logits2d, ldl, dv, lddv, dlogits, lddl, dl_cols, B, H, W, C, heads, k):
    lib = _lib.load()
    M = B * H * W
    dt = _dt(dy)
    nws = lib.ogv_outlook_bwd_ws_bytes(B, H, W, C, heads, k, dt)
    probs = torch.empty(max(nws // 4, 1), dtype=torch.float32, device=dy.device) if nws else None
    ou = dict(M=M, C=C, heads=heads, k=k, elem=dy.element_size())
    with _probe("outlook_bwd", ou), _census("outlook_bwd", ou):
        check(lib.ogv_outlook_agg_bwd(_ptr(dy), _vp(v2d), _vp(logits2d), _vp(dv), _vp(dlogits), _ptr(probs), B, H, W,
                                      C, heads, k, ldl, ldv, lddv, lddl, dl_cols, dt, _stream()), "ogv_outlook_agg_bwd")


class _OutlookAgg(torch.autograd.Function):
    """v [M, C] (row stride >= C) and logits [M, heads*k*k] as separate tensors."""

    @staticmethod
    def forward(ctx, v2d, logits2d, B, H, W, heads, k):
        lib = _lib.load()
        M, C = v2d.shape
        y = torch.empty((M, C), dtype=v2d.dtype, device=v2d.device)
        ou = dict(M=M, C=C, heads=heads, k=k, elem=v2d.element_size())
        with _probe("outlook_fwd", ou), _census("outlook_fwd", ou):
            check(lib.ogv_outlook_agg_fwd(_ptr(v2d), _ptr(logits2d), _ptr(y), B, H, W, C, heads, k,
                                          logits2d.stride(0), v2d.stride(0), _dt(v2d), _stream()),
                  "ogv_outlook_agg_fwd")
        ctx.save_for_backward(v2d, logits2d)
        ctx.meta = (B, H, W, C, heads, k)
        return y

    @staticmethod
    def backward(ctx, dy):
        v2d, logits2d = ctx.saved_tensors
        B, H, W, C, heads, k = ctx.meta
        kk = k * k
        dy = dy.to(v2d.dtype).contiguous()
        M = v2d.shape[0]
        dv = torch.empty((M, C), dtype=v2d.dtype, device=v2d.device)
        ld = logits2d.stride(0)
        dlogits = torch.empty((M, ld), dtype=v2d.dtype, device=v2d.device)[:, : heads * kk]
        _outlook_bwd(dy, v2d.data_ptr(), v2d.stride(0), logits2d.data_ptr(), ld, dv.data_ptr(), C, dlogits.data_ptr(),
                     ld, heads * kk, B, H, W, C, heads, k)
        return dv, dlogits, None, None, None, None, None


class _OutlookAggCat(torch.autograd.Function):
    """The fused v / attn projection output cat = [v | logits | zero pad] of shape [M, ld]
    (OutlookAttention2d with no hooks): the kernels read both column ranges in place, and the
    backward writes ONE gradient [dv | dlogits | 0] of the same layout, which the single
    concatenated GEMM's backward consumes (one dgrad + one wgrad, no autograd add)."""

    @staticmethod
    def forward(ctx, cat, C, B, H, W, heads, k):
        lib = _lib.load()
        M, ld = cat.shape
        y = torch.empty((M, C), dtype=cat.dtype, device=cat.device)
        es = cat.element_size()
        ou = dict(M=M, C=C, heads=heads, k=k, elem=es)
        with _probe("outlook_fwd", ou), _census("outlook_fwd", ou):
            check(lib.ogv_outlook_agg_fwd(_ptr(cat), _vp(cat.data_ptr() + C * es), _ptr(y), B, H, W, C, heads, k, ld, ld,
                                          _dt(cat), _stream()), "ogv_outlook_agg_fwd")
        ctx.save_for_backward(cat)
        ctx.meta = (B, H, W, C, heads, k)
        return y

    @staticmethod
    def backward(ctx, dy):
        cat, = ctx.saved_tensors
        B, H, W, C, heads, k = ctx.meta
        M, ld = cat.shape
        es = cat.element_size()
        dy = dy.to(cat.dtype).contiguous()
        dcat = torch.empty_like(cat)
        _outlook_bwd(dy, cat.data_ptr(), ld, cat.data_ptr() + C * es, ld, dcat.data_ptr(), ld, dcat.data_ptr() + C * es,
                     ld, ld - C, B, H, W, C, heads, k)
        return dcat, None, None, None, None, None, None


def _l32_ld(heads, k):
    return (heads * k * k + 3) // 4 * 4


class _OutlookVProj(torch.autograd.Function):
    """Outlooker forward fused with its v / attn 1x1 projections (ogv_outlook_vproj_fwd): x [M, C]
    -> y [M, C].  mode 0: inference (nothing saved); 1: training with the fused backward
    (ogv_outlook_vproj_bwd recomputes [v | logits] from x in LDS, so the forward writes only y);
    2: training that saves cat = [v | logits | 0] [M, ld] for the LDS-tiled aggregation backward.
    l32 (the default where ogv_outlook_vproj_l32_supported): the fp32-logits form -- the forward's softmax
    reads the logits unrounded, mode 2 saves v [M, C] bf16 and the logits [M, 9 heads rounded to 4] fp32
    (ogv_outlook_vproj_fwd_l32), and the tiled backward recomputes the softmax from them
    (ogv_outlook_agg_bwd_l32).  Either backward yields ONE dcat = [dv | dlogits | 0], then ONE dgrad +
    ONE wgrad of the concatenated weight (as _OutlookAggCat + _Linear)."""

    @staticmethod
    def forward(ctx, x2d, w, b, C, B, H, W, heads, k, mode, l32):
        lib = _lib.load()
        M = x2d.shape[0]
        ld = w.shape[0]
        y = torch.empty((M, C), dtype=x2d.dtype, device=x2d.device)
        ou = dict(M=M, C=C, ld=ld, heads=heads, k=k, cat=mode == 2, elem=x2d.element_size(), l32=l32)
        lg = None
        if l32:
            lld = _l32_ld(heads, k)
            cat = torch.empty((M, C), dtype=x2d.dtype, device=x2d.device) if mode == 2 else None
            lg = torch.empty((M, lld), dtype=torch.float32, device=x2d.device) if mode == 2 else None
            with _probe("outlook_vproj", ou), _census("outlook_vproj", ou):
                check(lib.ogv_outlook_vproj_fwd_l32(_ptr(x2d), x2d.stride(0), _ptr(w), _ptr(b), _ptr(cat), C, _ptr(lg),
                                                    lld, _ptr(y), B, H, W, C, heads, k, _dt(x2d), _stream()),
                      "ogv_outlook_vproj_fwd_l32")
        else:
            cat = torch.empty((M, ld), dtype=x2d.dtype, device=x2d.device) if mode == 2 else None
            with _probe("outlook_vproj", ou), _census("outlook_vproj", ou):
                check(lib.ogv_outlook_vproj_fwd(_ptr(x2d), x2d.stride(0), _ptr(w), _ptr(b), _ptr(cat), ld, _ptr(y), B, H,
                                                W, C, heads, k, _dt(x2d), _stream()), "ogv_outlook_vproj_fwd")
        ctx.save_for_backward(x2d, w, b, cat, lg)
        ctx.meta = (B, H, W, C, heads, k, b is not None, mode)
        return y

    @staticmethod
    def backward(ctx, dy):
        x2d, w, b, cat, lg = ctx.saved_tensors
        B, H, W, C, heads, k, has_bias, mode = ctx.meta
        M, ld = x2d.shape[0], w.shape[0]
        dy = dy.to(x2d.dtype).contiguous()
        dcat = torch.empty((M, ld), dtype=x2d.dtype, device=x2d.device)
        if mode == 1:
            ou = dict(M=M, C=C, ld=ld, heads=heads, k=k, elem=x2d.element_size())
            with _probe("outlook_vproj_bwd", ou), _census("outlook_vproj_bwd", ou):
                check(_lib.load().ogv_outlook_vproj_bwd(_ptr(x2d), x2d.stride(0), _ptr(w), _ptr(b), _ptr(dy), _ptr(dcat),
                                                        ld, B, H, W, C, heads, k, _dt(x2d), _stream()),
                      "ogv_outlook_vproj_bwd")
        elif lg is not None:
            es = dcat.element_size()
            ou = dict(M=M, C=C, heads=heads, k=k, elem=es, l32=True)
            with _probe("outlook_bwd", ou), _census("outlook_bwd", ou):
                check(_lib.load().ogv_outlook_agg_bwd_l32(_ptr(dy), _ptr(cat), _ptr(lg), _ptr(dcat),
                                                          _vp(dcat.data_ptr() + C * es), B, H, W, C, heads, k,
                                                          lg.stride(0), cat.stride(0), ld, ld, ld - C, _dt(dy), _stream()),
                      "ogv_outlook_agg_bwd_l32")
        else:
            es = cat.element_size()
            _outlook_bwd(dy, cat.data_ptr(), ld, cat.data_ptr() + C * es, ld, dcat.data_ptr(), ld,
                         dcat.data_ptr() + C * es, ld, ld - C, B, H, W, C, heads, k)
        want_dw = ctx.needs_input_grad[1] or (has_bias and ctx.needs_input_grad[2])
        dx, dw, db = _linear_bwd(dcat, x2d, w, None, 1, 0, has_bias, ctx.needs_input_grad[0], want_dw)
        return dx, dw, db, None, None, None, None, None, None, None, None


class _AliasedConcat(torch.autograd.Function):
    """torch.cat along rows for parts that already ARE row blocks of `full` (views of one buffer,
    e.g. parameters re-pointed into it; part i starts at row offsets[i]): returns `full` itself --
    no copy launch -- and hands each part the matching row block of the incoming gradient (views
    that AccumulateGrad steals: nothing is copied on the way back either).  Rows of `full` outside
    the parts carry no gradient."""

    @staticmethod
    def forward(ctx, full, offsets, *parts):
        ctx.meta = [(int(o), p.shape) for o, p in zip(offsets, parts)]
        return full.view(full.shape)

    @staticmethod
    def backward(ctx, g):
        return (None, None) + tuple(g[o:o + shp[0]].view(shp) for o, shp in ctx.meta)


def aliased_concat(full, offsets, *parts):
    return _AliasedConcat.apply(full, tuple(offsets), *parts)


def outlook_vproj_supported(B, H, W, C, heads, k, ld, dtype, train) -> bool:
    """Whether OutlookAttention2d takes the fused projection + aggregation forward for this shape
    (knob "outlook_vproj": 0 never, 1 inference only, 2 also in training -- the default --, 3 training
    with the recompute backward)."""
    if dtype != torch.bfloat16:
        return False
    return bool(_lib.load().ogv_outlook_vproj_supported(B, H, W, C, heads, k, ld, int(bool(train)), OGV_BF16))


def outlook_vproj(x2d, w, b, C, B, H, W, heads, k, save_cat=None):
    """y [M, C] = outlook aggregation of (x2d @ [Wv; Wattn; 0]^T + b) without materialising the
    projection for the forward's own use (x2d bf16 rows, w fp32 [ld, C], b fp32 [ld] or None).
    When a gradient will be wanted: save_cat=True writes cat = [v | logits | 0] [M, ld] in the same
    launch for the LDS-tiled aggregation backward; False keeps only x and recomputes [v | logits]
    in the backward (ogv_outlook_vproj_bwd); None follows the knob (outlook_vproj 3 -> recompute)."""
    require_device(x2d, w, b, what="ogv.outlook_vproj")
    x2d = _rows_contig(x2d)
    train = torch.is_grad_enabled() and any(t is not None and t.requires_grad for t in (x2d, w, b))
    if train and save_cat is None:
        save_cat = _lib.load().ogv_outlook_vproj_supported(int(B), int(H), int(W), int(C), int(heads), int(k),
                                                           int(w.shape[0]), 1, OGV_BF16) != 2
    elif train and not save_cat and not _lib.load().ogv_outlook_vproj_bwd_supported(
            int(B), int(H), int(W), int(C), int(heads), int(k), int(w.shape[0]), OGV_BF16):
        raise ValueError(f"ogv.outlook_vproj: no recompute backward at C={C} (wide stages save cat)")
    mode = 0 if not train else (2 if save_cat else 1)
    # the fp32-logits form wherever it applies (not with the recompute backward, mode 1)
    l32 = mode != 1 and bool(_lib.load().ogv_outlook_vproj_l32_supported(int(B), int(H), int(W), int(C), int(heads),
                                                                          int(k), int(train), OGV_BF16))
    return _OutlookVProj.apply(x2d, w.contiguous(), None if b is None else b.contiguous(), int(C), int(B), int(H),
                               int(W), int(heads), int(k), mode, l32)


def outlook_aggregate_rows(v2d, logits2d, B, H, W, heads, k):
    require_device(v2d, logits2d, what="ogv.outlook_aggregate")
    v2d = _rows_contig(v2d)
    if logits2d.stride(-1) != 1 or logits2d.data_ptr() % 4:
        logits2d = logits2d.contiguous()
    if logits2d.dtype != v2d.dtype:
        logits2d = logits2d.to(v2d.dtype)
    return _OutlookAgg.apply(v2d, logits2d, int(B), int(H), int(W), int(heads), int(k))


def outlook_aggregate_cat(cat, C, B, H, W, heads, k):
    """cat [M, ld] = [v (C columns) | logits (heads*k*k) | padding] -> y [M, C]."""
    require_device(cat, what="ogv.outlook_aggregate")
    if cat.stride(-1) != 1 or cat.stride(0) != cat.shape[1] or cat.shape[1] < C + heads * k * k:
        raise ValueError("ogv.outlook_aggregate_cat: expects a contiguous [M, >= C + heads*k*k] tensor")
    return _OutlookAggCat.apply(cat, int(C), int(B), int(H), int(W), int(heads), int(k))


# ------------------------------------------------------------------------------------------------
# Grid attention core (partition folded into addressing)
# ------------------------------------------------------------------------------------------------
class _GridAttn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, qkv2d, B, H, W, heads, g, scale, want_probs):
        lib = _lib.load()
        M = qkv2d.shape[0]
        C = qkv2d.shape[1] // 3
        out = torch.empty((M, C), dtype=qkv2d.dtype, device=qkv2d.device)
        lse = torch.empty((M, heads), dtype=torch.float32, device=qkv2d.device)
        N = (H // g) * (W // g)
        probs = (torch.empty((B * g * g, heads, N, N), dtype=torch.float32, device=qkv2d.device)
                 if want_probs else None)
        gu = dict(M=M, C=C, heads=heads, N=N, elem=qkv2d.element_size())
        with _probe("grid_fwd", gu), _census("grid_fwd", gu):
            check(lib.ogv_grid_attn_fwd(_ptr(qkv2d), _ptr(out), _ptr(lse), _ptr(probs), B, H, W, C, heads, g,
                                        float(scale), _dt(qkv2d), _stream()), "ogv_grid_attn_fwd")
        ctx.save_for_backward(qkv2d, out, lse)
        ctx.meta = (B, H, W, C, heads, g, float(scale))
        if probs is None:
            probs = torch.empty(0, device=qkv2d.device)
        ctx.mark_non_differentiable(probs)
        return out, probs

    @staticmethod
    def backward(ctx, dout, _dprobs):
        lib = _lib.load()
        qkv2d, out, lse = ctx.saved_tensors
        B, H, W, C, heads, g, scale = ctx.meta
        dout = dout.to(qkv2d.dtype).contiguous()
        dqkv = torch.empty_like(qkv2d)
        delta = torch.empty((qkv2d.shape[0], heads), dtype=torch.float32, device=qkv2d.device)
        gu = dict(M=qkv2d.shape[0], C=C, heads=heads, N=(H // g) * (W // g), elem=qkv2d.element_size())
        with _census("grid_bwd", gu):
            check(lib.ogv_grid_attn_bwd(_ptr(dout), _ptr(qkv2d), _ptr(out), _ptr(lse), _ptr(dqkv), _ptr(delta), B, H, W,
                                        C, heads, g, scale, _dt(qkv2d), _stream()), "ogv_grid_attn_bwd")
        return dqkv, None, None, None, None, None, None, None


def grid_attention_rows(qkv2d, B, H, W, heads, g, scale, want_probs=False):
    """qkv2d [B*H*W, 3C] -> (out [B*H*W, C], probs [B*g*g, heads, N, N] or empty)."""
    require_device(qkv2d, what="ogv.grid_attention")
    qkv2d = qkv2d.contiguous()
    return _GridAttn.apply(qkv2d, int(B), int(H), int(W), int(heads), int(g), float(scale), bool(want_probs))


# ------------------------------------------------------------------------------------------------
# Depthwise 3x3 conv (MBConv.depthwise)
# ------------------------------------------------------------------------------------------------
class _DwConv3x3(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x2d, w, bias, B, H, W, stride):
        lib = _lib.load()
        C = x2d.shape[1]
        Ho, Wo = (H - 1) // stride + 1, (W - 1) // stride + 1
        y = torch.empty((B * Ho * Wo, C), dtype=x2d.dtype, device=x2d.device)
        ws = _ws(lib.ogv_dwconv_fwd_ws_bytes(C), x2d.device)
        with _census("dwconv_fwd", dict(M=x2d.shape[0], Mo=y.shape[0], C=C, elem=x2d.element_size())):
            check(lib.ogv_dwconv3x3_fwd(_ptr(x2d), _ptr(w), _ptr(bias), _ptr(y), B, H, W, C, stride, _ptr(ws), _dt(x2d),
                                        _stream()), "ogv_dwconv3x3_fwd")
        ctx.save_for_backward(x2d, w)
        ctx.meta = (B, H, W, C, stride, bias is not None)
        return y

    @staticmethod
    def backward(ctx, dy):
        lib = _lib.load()
        x2d, w = ctx.saved_tensors
        B, H, W, C, stride, has_bias = ctx.meta
        dy = dy.to(x2d.dtype).contiguous()
        dx = torch.empty_like(x2d) if ctx.needs_input_grad[0] else None
        dw = torch.empty_like(w) if ctx.needs_input_grad[1] else None
        db = torch.empty((C,), dtype=torch.float32, device=x2d.device) if (has_bias and ctx.needs_input_grad[2]) else None
        ws = _ws(lib.ogv_dwconv_bwd_ws_bytes(B, H, W, C, stride), x2d.device)
        with _census("dwconv_bwd", dict(M=x2d.shape[0], Mo=dy.shape[0], C=C, elem=x2d.element_size())):
            check(lib.ogv_dwconv3x3_bwd(_ptr(dy), _ptr(x2d), _ptr(w), _ptr(dx), _ptr(dw), _ptr(db), B, H, W, C, stride,
                                        _ptr(ws), _dt(x2d), _stream()), "ogv_dwconv3x3_bwd")
        return dx, dw, db, None, None, None, None


def dwconv3x3_nchw(x, weight, bias=None, stride=1):
    """Depthwise 3x3 conv (padding 1) on an NCHW (channels_last) tensor -> channels_last NCHW."""
    require_device(x, weight, bias, what="ogv.dwconv3x3")
    B, C, H, W = x.shape
    x2d = _rows_contig(nchw_to_rows(x))
    y = _DwConv3x3.apply(x2d, f32(weight).contiguous(), f32(bias), B, H, W, int(stride))
    return rows_to_nchw(y, B, (H - 1) // stride + 1, (W - 1) // stride + 1)


# ------------------------------------------------------------------------------------------------
# Fused MBConv (expand+BN1+act -> dw3x3+BN2+act -> SE -> project+BN3 -> +x)
# ------------------------------------------------------------------------------------------------
def _mb_units(geom, x2d):
    B, H, W, C, mid, se = geom[:6]
    return dict(M=B * H * W, B=B, C=C, mid=mid, se=se, elem=x2d.element_size())


class _MBConv(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x2d, geom, buffers, *params):
        lib = _lib.load()
        dt = _dt(x2d)
        desc = _lib.MBConvDesc(*geom, -1)
        # pin the saved-data variant (knob mb_a3) now: the backward reads `saved` with this same desc
        desc.a3 = lib.ogv_mbconv_a3_mode(ctypes.byref(desc), dt)
        w = dict(zip(_lib.MBCONV_GRAD_FIELDS, params))
        w.update(buffers)
        P = _lib.MBConvParams(*[_vp(w[n].data_ptr()) for n in _lib.MBCONV_PARAM_FIELDS])
        saved = torch.empty(lib.ogv_mbconv_saved_bytes(ctypes.byref(desc), dt), dtype=torch.uint8, device=x2d.device)
        ws = _ws(lib.ogv_mbconv_ws_bytes(ctypes.byref(desc), dt), x2d.device)
        out = torch.empty_like(x2d)
        with _census("mbconv_fwd", _mb_units(geom, x2d)):
            check(lib.ogv_mbconv_fwd(_ptr(x2d), _ptr(out), _ptr(saved), _ptr(ws), ctypes.byref(desc), ctypes.byref(P),
                                     dt, _stream()), "ogv_mbconv_fwd")
        ctx.save_for_backward(x2d, saved, *params)
        ctx.geom, ctx.buffers = geom + (int(desc.a3),), buffers
        return out

    @staticmethod
    def backward(ctx, dout):
        lib = _lib.load()
        x2d, saved, *params = ctx.saved_tensors
        desc = _lib.MBConvDesc(*ctx.geom)
        w = dict(zip(_lib.MBCONV_GRAD_FIELDS, params))
        w.update(ctx.buffers)
        P = _lib.MBConvParams(*[_vp(w[n].data_ptr()) for n in _lib.MBCONV_PARAM_FIELDS])
        grads = [torch.empty_like(t) for t in params]
        G = _lib.MBConvGrads(*[_vp(g.data_ptr()) for g in grads])
        dt = _dt(x2d)
        dout = dout.to(x2d.dtype).contiguous()
        dx = torch.empty_like(x2d)
        ws = _ws(lib.ogv_mbconv_ws_bytes(ctypes.byref(desc), dt), x2d.device)
        pws = _ws(lib.ogv_mbconv_param_ws_bytes(ctypes.byref(desc)), x2d.device, deferrable=True)
        with _census("mbconv_bwd", _mb_units(ctx.geom, x2d)):
            check(lib.ogv_mbconv_bwd(_ptr(dout), _ptr(x2d), _ptr(saved), _ptr(dx), ctypes.byref(G), _ptr(ws),
                                     _ptr(pws), ctypes.byref(desc), ctypes.byref(P), dt, _stream()), "ogv_mbconv_bwd")
        return (dx, None, None, *grads)


def mbconv_fused(x, B, H, W, mid, se, train, eps, momentum, act, params, buffers):
    """x: NCHW (channels_last); params: 13 fp32 tensors in MBCONV_GRAD_FIELDS order;
    buffers: {'bn1_rm', 'bn1_rv', ...} running statistics (updated in place when train)."""
    require_device(x, *params, what="ogv.mbconv")
    C = x.shape[1]
    x2d = _rows_contig(nchw_to_rows(x))
    geom = (int(B), int(H), int(W), int(C), int(mid), int(se), int(bool(train)), float(eps), float(momentum),
            ACT[act])
    y = _MBConv.apply(x2d, geom, buffers, *[f32(t).contiguous() for t in params])
    return rows_to_nchw(y, B, H, W)


# ------------------------------------------------------------------------------------------------
# MaxOutNet around the blocks: conv3x3 -> BatchNorm2d -> act (stem, downsample), BatchNorm alone
# (head).  src/model/stem_head.py:23-32, src/model/downsampling.py:28-65, Model_A_OutGridNet.py:66
# ------------------------------------------------------------------------------------------------
def _bn_args(bn):
    """(has_bn, train, eps, momentum, running_mean, running_var) of an nn.BatchNorm2d or None."""
    if bn is None:
        return 0, 0, 1e-5, 0.1, None, None
    if not bn.track_running_stats or bn.running_mean is None or bn.momentum is None:
        raise NotImplementedError("ogv BatchNorm: needs track_running_stats=True and a float momentum "
                                  "(the reference's nn.BatchNorm2d defaults)")
    return 1, int(bool(bn.training)), float(bn.eps), float(bn.momentum), bn.running_mean, bn.running_var


class _ConvBN(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x2d, geom, rm, rv, w, bias, bn_w, bn_b):
        lib = _lib.load()
        B, H, W, Cin, Cout, stride = geom[:6]
        desc = _lib.ConvBNDesc(*geom)
        P = _lib.ConvBNParams(_ptr(w), _ptr(bias), _ptr(bn_w), _ptr(bn_b), _ptr(rm), _ptr(rv))
        dt = _dt(x2d)
        Ho, Wo = (H - 1) // stride + 1, (W - 1) // stride + 1
        out = torch.empty((B * Ho * Wo, Cout), dtype=x2d.dtype, device=x2d.device)
        saved = torch.empty(lib.ogv_convbn_saved_bytes(ctypes.byref(desc), dt), dtype=torch.uint8, device=x2d.device)
        ws = _ws(lib.ogv_convbn_ws_bytes(ctypes.byref(desc), dt), x2d.device)
        cu = dict(M=x2d.shape[0], Mo=out.shape[0], Cin=Cin, Cout=Cout, elem=x2d.element_size())
        with _census("convbn_fwd", cu):
            check(lib.ogv_convbn_fwd(_ptr(x2d), _ptr(out), _ptr(saved), _ptr(ws), ctypes.byref(desc), ctypes.byref(P),
                                     dt, _stream()), "ogv_convbn_fwd")
        ctx.save_for_backward(x2d, saved, w, bias, bn_w, bn_b)
        ctx.geom = geom
        return out

    @staticmethod
    def backward(ctx, dout):
        lib = _lib.load()
        x2d, saved, w, bias, bn_w, bn_b = ctx.saved_tensors
        desc = _lib.ConvBNDesc(*ctx.geom)
        P = _lib.ConvBNParams(_ptr(w), _ptr(bias), _ptr(bn_w), _ptr(bn_b), None, None)
        dt = _dt(x2d)
        dout = dout.to(x2d.dtype).contiguous()
        dx = torch.empty_like(x2d) if ctx.needs_input_grad[0] else None
        dw = torch.empty_like(w)
        db = torch.empty_like(bias) if bias is not None else None
        dg = torch.empty_like(bn_w) if bn_w is not None else None
        dbb = torch.empty_like(bn_b) if bn_b is not None else None
        ws = _ws(lib.ogv_convbn_ws_bytes(ctypes.byref(desc), dt), x2d.device)
        B, H, W, Cin, Cout = ctx.geom[:5]
        cu = dict(M=x2d.shape[0], Mo=dout.shape[0], Cin=Cin, Cout=Cout, elem=x2d.element_size())
        with _census("convbn_bwd", cu):
            check(lib.ogv_convbn_bwd(_ptr(dout), _ptr(x2d), _ptr(saved), _ptr(dx), _ptr(dw), _ptr(db), _ptr(dg),
                                     _ptr(dbb), _ptr(ws), ctypes.byref(desc), ctypes.byref(P), dt, _stream()),
                  "ogv_convbn_bwd")
        return dx, None, None, None, dw, db, dg, dbb


def conv3x3_bn_act(x, conv, bn=None, act=None):
    """act(BN(conv(x))) for an nn.Conv2d(Cin, Cout, 3, stride 1|2, padding 1) and an optional
    nn.BatchNorm2d(Cout); x NCHW (any memory format) -> channels_last NCHW."""
    require_device(x, conv.weight, what="ogv.conv3x3_bn_act")
    if (tuple(conv.kernel_size) != (3, 3) or tuple(conv.padding) != (1, 1) or conv.groups != 1
            or tuple(conv.dilation) != (1, 1) or conv.stride[0] != conv.stride[1] or conv.stride[0] not in (1, 2)):
        raise NotImplementedError("ogv.conv3x3_bn_act: needs a dense 3x3 conv, padding 1, stride 1 or 2")
    B, Cin, H, W = x.shape
    Cout, stride = conv.out_channels, conv.stride[0]
    has_bn, train, eps, mom, rm, rv = _bn_args(bn)
    x2d = _rows_contig(nchw_to_rows(x.to(compute_dtype(x))))
    w = f32(conv.weight)
    # a channels_last weight (the model moved to channels_last) IS the tap-major [Cout, 3, 3, Cin]
    # matrix the kernels multiply by: passed as is (no copy here, no transpose launches, and its
    # gradient comes back in the same layout, so AccumulateGrad copies nothing)
    tap_major = not w.is_contiguous() and w.is_contiguous(memory_format=torch.channels_last)
    if not tap_major:
        w = w.contiguous()
    geom = (int(B), int(H), int(W), int(Cin), int(Cout), int(stride), has_bn, train, eps, mom, ACT[act], int(tap_major))
    y = _ConvBN.apply(x2d, geom, rm, rv, w, f32(conv.bias),
                      f32(bn.weight) if has_bn else None, f32(bn.bias) if has_bn else None)
    if has_bn and train and not getattr(bn, "_ogv_nbt_pooled", False):
        bn.num_batches_tracked.add_(1)
    return rows_to_nchw(y, B, (H - 1) // stride + 1, (W - 1) // stride + 1)


class _BNAct(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x2d, meta, rm, rv, bn_w, bn_b):
        lib = _lib.load()
        train, eps, mom, act = meta
        M, C = x2d.shape
        dt = _dt(x2d)
        out = torch.empty_like(x2d)
        saved = torch.empty(lib.ogv_bn_act_saved_bytes(C) // 4, dtype=torch.float32, device=x2d.device)
        ws = _ws(lib.ogv_bn_act_ws_bytes(M, C), x2d.device)
        with _census("bn_act_fwd", dict(M=M, C=C, train=train, elem=x2d.element_size())):
            check(lib.ogv_bn_act_fwd(_ptr(x2d), _ptr(out), _ptr(saved), _ptr(ws), _ptr(bn_w), _ptr(bn_b), _ptr(rm),
                                     _ptr(rv), M, C, train, eps, mom, act, dt, _stream()), "ogv_bn_act_fwd")
        ctx.save_for_backward(x2d, saved, bn_w, bn_b)
        ctx.meta = meta
        return out

    @staticmethod
    def backward(ctx, dout):
        lib = _lib.load()
        x2d, saved, bn_w, bn_b = ctx.saved_tensors
        train, eps, mom, act = ctx.meta
        M, C = x2d.shape
        dt = _dt(x2d)
        dout = dout.to(x2d.dtype).contiguous()
        dx = torch.empty_like(x2d)
        dg = torch.empty_like(bn_w) if bn_w is not None else None
        dbb = torch.empty_like(bn_b) if bn_b is not None else None
        ws = _ws(lib.ogv_bn_act_ws_bytes(M, C), x2d.device)
        with _census("bn_act_bwd", dict(M=M, C=C, elem=x2d.element_size())):
            check(lib.ogv_bn_act_bwd(_ptr(dout), _ptr(x2d), _ptr(saved), _ptr(dx), _ptr(dg), _ptr(dbb), _ptr(ws),
                                     _ptr(bn_w), M, C, train, act, dt, _stream()), "ogv_bn_act_bwd")
        return dx, None, None, None, dg, dbb


class _HeadBNPool(torch.autograd.Function):
    """mean_p(BatchNorm2d(x)) as BN(mean_p(x)) from one read of x (ogv_head_bn_pool_fwd/bwd): the classifier
    head of MaxOutNet / OutlookerFrontGridNet (Model_A_OutGridNet.py:64-66).  Returns fp32 [B, C]."""

    @staticmethod
    def forward(ctx, x2d, meta, rm, rv, bn_w, bn_b):
        lib = _lib.load()
        B, HW, train, eps, mom = meta
        C = x2d.shape[1]
        dt = _dt(x2d)
        raw = torch.empty((B, C), dtype=torch.float32, device=x2d.device)
        pooled = torch.empty((B, C), dtype=torch.float32, device=x2d.device)
        saved = torch.empty(lib.ogv_bn_act_saved_bytes(C) // 4, dtype=torch.float32, device=x2d.device)
        ws = _ws(lib.ogv_head_bn_pool_ws_bytes(B, C), x2d.device)
        with _census("bn_act_fwd", dict(M=B * HW, C=C, train=train, elem=x2d.element_size(), head=True, hw=HW)):
            check(lib.ogv_head_bn_pool_fwd(_ptr(x2d), _ptr(raw), _ptr(pooled), _ptr(saved), _ptr(ws), _ptr(bn_w),
                                           _ptr(bn_b), _ptr(rm), _ptr(rv), B, HW, C, train, eps, mom, dt, _stream()),
                  "ogv_head_bn_pool_fwd")
        ctx.save_for_backward(x2d, raw, saved, bn_w)
        ctx.meta = meta
        return pooled

    @staticmethod
    def backward(ctx, dpooled):
        lib = _lib.load()
        x2d, raw, saved, bn_w = ctx.saved_tensors
        B, HW, train, _, _ = ctx.meta
        C = x2d.shape[1]
        dpooled = dpooled.float().contiguous()
        dx = torch.empty_like(x2d)
        dg = torch.empty_like(bn_w) if bn_w is not None else None
        dbb = torch.empty((C,), dtype=torch.float32, device=x2d.device) if ctx.needs_input_grad[5] else None
        ws = _ws(lib.ogv_head_bn_pool_ws_bytes(B, C), x2d.device)
        with _census("bn_act_bwd", dict(M=B * HW, C=C, elem=x2d.element_size(), head=True, hw=HW)):
            check(lib.ogv_head_bn_pool_bwd(_ptr(dpooled), _ptr(x2d), _ptr(raw), _ptr(saved), _ptr(dx), _ptr(dg),
                                           _ptr(dbb), _ptr(ws), _ptr(bn_w), B, HW, C, train, _dt(x2d), _stream()),
                  "ogv_head_bn_pool_bwd")
        return dx, None, None, None, dg, dbb


def head_bn_pool(x, bn):
    """BatchNorm2d(x).mean((2, 3)) in fp32 [B, C] (nn.BatchNorm2d semantics incl. the running-stat update),
    computed as BN of the per-image channel means (BN is per-channel affine): one pass over x each way."""
    require_device(x, what="ogv.head_bn_pool")
    has_bn, train, eps, mom, rm, rv = _bn_args(bn)
    B, C, H, W = x.shape
    x2d = _rows_contig(nchw_to_rows(x.to(compute_dtype(x))))
    y = _HeadBNPool.apply(x2d, (int(B), int(H * W), train, eps, mom), rm, rv,
                          f32(bn.weight) if bn.affine else None, f32(bn.bias) if bn.affine else None)
    if train and not getattr(bn, "_ogv_nbt_pooled", False):
        bn.num_batches_tracked.add_(1)
    return y


def batchnorm_act_nchw(x, bn, act=None):
    """act(BatchNorm2d(x)) on a channels_last view of x (nn.BatchNorm2d semantics)."""
    require_device(x, what="ogv.batchnorm")
    has_bn, train, eps, mom, rm, rv = _bn_args(bn)
    B, C, H, W = x.shape
    x2d = _rows_contig(nchw_to_rows(x.to(compute_dtype(x))))
    y = _BNAct.apply(x2d, (train, eps, mom, ACT[act]), rm, rv, f32(bn.weight) if bn.affine else None,
                     f32(bn.bias) if bn.affine else None)
    if train and not getattr(bn, "_ogv_nbt_pooled", False):
        bn.num_batches_tracked.add_(1)
    return rows_to_nchw(y, B, H, W)
