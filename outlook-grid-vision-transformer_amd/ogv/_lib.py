"""ctypes binding of libogv_hip.so (the C-ABI declared in include/ogv.h).

The library is loaded AFTER ``import torch`` so that its ``libamdhip64.so.7`` dependency resolves
to the HIP runtime torch already mapped (same SONAME); device pointers and streams are then
shared with PyTorch's caching allocator and stream pool.  There is no fallback: if the shared
object is missing or a symbol is absent, the import raises.
"""
from __future__ import annotations

import ctypes
import os

import torch  # noqa: F401  (must precede the CDLL: binds to torch's HIP runtime)

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("OGV_LIB", os.path.join(_HERE, "libogv_hip.so"))

_p = ctypes.c_void_p
_i = ctypes.c_int
_f = ctypes.c_float
_sz = ctypes.c_size_t

class MBConvDesc(ctypes.Structure):
    _fields_ = [("B", _i), ("H", _i), ("W", _i), ("C", _i), ("mid", _i), ("se", _i), ("train", _i),
                ("bn_eps", _f), ("bn_momentum", _f), ("act", _i), ("a3", _i)]


MBCONV_PARAM_FIELDS = ["w_expand", "bn1_w", "bn1_b", "bn1_rm", "bn1_rv", "w_dw", "bn2_w", "bn2_b", "bn2_rm", "bn2_rv",
                       "se_w1", "se_b1", "se_w2", "se_b2", "w_proj", "bn3_w", "bn3_b", "bn3_rm", "bn3_rv"]
MBCONV_GRAD_FIELDS = ["w_expand", "bn1_w", "bn1_b", "w_dw", "bn2_w", "bn2_b", "se_w1", "se_b1", "se_w2", "se_b2",
                      "w_proj", "bn3_w", "bn3_b"]


class MBConvParams(ctypes.Structure):
    _fields_ = [(n, _p) for n in MBCONV_PARAM_FIELDS]


class MBConvGrads(ctypes.Structure):
    _fields_ = [(n, _p) for n in MBCONV_GRAD_FIELDS]


class ConvBNDesc(ctypes.Structure):
    _fields_ = [("B", _i), ("H", _i), ("W", _i), ("Cin", _i), ("Cout", _i), ("stride", _i), ("has_bn", _i),
                ("train", _i), ("bn_eps", _f), ("bn_momentum", _f), ("act", _i), ("w_layout", _i)]


class ConvBNParams(ctypes.Structure):
    _fields_ = [(n, _p) for n in ("w", "bias", "bn_w", "bn_b", "bn_rm", "bn_rv")]


class AdamWTensor(ctypes.Structure):
    _fields_ = [("param", _p), ("grad", _p), ("exp_avg", _p), ("exp_avg_sq", _p), ("step", _p),
                ("numel", ctypes.c_longlong), ("group", _i)]


class AdamWGroup(ctypes.Structure):
    _fields_ = [("lr", _p), ("weight_decay", _f), ("beta1", _f), ("beta2", _f), ("eps", _f),
                ("one_minus_beta1", _f), ("one_minus_beta2", _f)]


class CopySeg(ctypes.Structure):
    _fields_ = [("src", _p), ("dst", _p), ("numel", ctypes.c_longlong)]


_PD = ctypes.POINTER(MBConvDesc)
_PCD = ctypes.POINTER(ConvBNDesc)
_PCP = ctypes.POINTER(ConvBNParams)
_PP = ctypes.POINTER(MBConvParams)
_PG = ctypes.POINTER(MBConvGrads)

# name -> (restype, argtypes); must match include/ogv.h exactly
SIGNATURES = {
    "ogv_version": (ctypes.c_char_p, []),
    "ogv_last_error": (ctypes.c_char_p, []),
    "ogv_set_option": (_i, [ctypes.c_char_p, _i]),
    "ogv_gemm_stream_route": (_i, [_i, _i, _i, _i, _i]),
    "ogv_gpu_sleep": (_i, [_i, _p]),
    "ogv_reduce_defer": (_i, [_i]),
    "ogv_reduce_flush": (_i, [_p]),
    "ogv_outlook_agg_fwd": (_i, [_p, _p, _p, _i, _i, _i, _i, _i, _i, _i, _i, _i, _p]),
    "ogv_outlook_bwd_ws_bytes": (_sz, [_i, _i, _i, _i, _i, _i, _i]),
    "ogv_outlook_vproj_supported": (_i, [_i, _i, _i, _i, _i, _i, _i, _i, _i]),
    "ogv_outlook_vproj_bwd_supported": (_i, [_i, _i, _i, _i, _i, _i, _i, _i]),
    "ogv_outlook_vproj_fwd": (_i, [_p, _i, _p, _p, _p, _i, _p, _i, _i, _i, _i, _i, _i, _i, _p]),
    "ogv_gemm_fwd_ln": (_i, [_p, _i, _p, _p, _p, _p, _i, _p, _i, _p, _p, _p, _f, _p, _p, _i, _i, _i, _i, _p]),
    "ogv_outlook_vproj_l32_supported": (_i, [_i, _i, _i, _i, _i, _i, _i, _i]),
    "ogv_outlook_vproj_fwd_l32": (_i, [_p, _i, _p, _p, _p, _i, _p, _i, _p, _i, _i, _i, _i, _i, _i, _i, _p]),
    "ogv_outlook_agg_bwd_l32": (_i, [_p, _p, _p, _p, _p, _i, _i, _i, _i, _i, _i, _i, _i, _i, _i, _i, _i, _p]),
    "ogv_outlook_vproj_bwd": (_i, [_p, _i, _p, _p, _p, _p, _i, _i, _i, _i, _i, _i, _i, _i, _p]),
    "ogv_outlook_agg_bwd": (_i, [_p, _p, _p, _p, _p, _p, _i, _i, _i, _i, _i, _i, _i, _i, _i, _i, _i, _i, _p]),
    "ogv_grid_attn_fwd": (_i, [_p, _p, _p, _p, _i, _i, _i, _i, _i, _i, _f, _i, _p]),
    "ogv_grid_attn_bwd": (_i, [_p, _p, _p, _p, _p, _p, _i, _i, _i, _i, _i, _i, _f, _i, _p]),
    "ogv_layernorm_fwd": (_i, [_p, _p, _p, _p, _p, _p, _i, _i, _f, _i, _p]),
    "ogv_layernorm_bwd_ws_bytes": (_sz, [_i, _i]),
    "ogv_layernorm_bwd": (_i, [_p, _p, _p, _p, _p, _p, _p, _p, _p, _p, _i, _i, _i, _p]),
    "ogv_gemm_fwd": (_i, [_p, _i, _p, _p, _p, _p, _i, _p, _i, _i, _i, _i, _i, _i, _p]),
    "ogv_gemm_fwd_act": (_i, [_p, _i, _p, _p, _p, _i, _p, _i, _i, _i, _i, _i, _i, _p]),
    "ogv_gemm_dgrad_ws_bytes": (_sz, [_i, _i]),
    "ogv_gemm_dgrad": (_i, [_p, _i, _p, _p, _i, _p, _i, _p, _i, _i, _i, _i, _i, _p, _i, _p]),
    "ogv_gemm_wgrad_ws_bytes": (_sz, [_i, _i, _i]),
    "ogv_gemm_wgrad": (_i, [_p, _i, _p, _i, _p, _i, _p, _p, _i, _i, _i, _i, _p, _i, _p]),
    "ogv_dwconv_fwd_ws_bytes": (_sz, [_i]),
    "ogv_dwconv3x3_fwd": (_i, [_p, _p, _p, _p, _i, _i, _i, _i, _i, _p, _i, _p]),
    "ogv_dwconv_bwd_ws_bytes": (_sz, [_i, _i, _i, _i, _i]),
    "ogv_dwconv3x3_bwd": (_i, [_p, _p, _p, _p, _p, _p, _i, _i, _i, _i, _i, _p, _i, _p]),
    "ogv_mbconv_a3_mode": (_i, [_PD, _i]),
    "ogv_mbconv_saved_bytes": (_sz, [_PD, _i]),
    "ogv_mbconv_ws_bytes": (_sz, [_PD, _i]),
    "ogv_mbconv_fwd": (_i, [_p, _p, _p, _p, _PD, _PP, _i, _p]),
    "ogv_mbconv_param_ws_bytes": (_sz, [_PD]),
    "ogv_mbconv_bwd": (_i, [_p, _p, _p, _p, _PG, _p, _p, _PD, _PP, _i, _p]),
    "ogv_convbn_saved_bytes": (_sz, [_PCD, _i]),
    "ogv_convbn_ws_bytes": (_sz, [_PCD, _i]),
    "ogv_convbn_fwd": (_i, [_p, _p, _p, _p, _PCD, _PCP, _i, _p]),
    "ogv_convbn_bwd": (_i, [_p, _p, _p, _p, _p, _p, _p, _p, _p, _PCD, _PCP, _i, _p]),
    "ogv_bn_act_saved_bytes": (_sz, [_i]),
    "ogv_bn_act_ws_bytes": (_sz, [_i, _i]),
    "ogv_bn_act_fwd": (_i, [_p, _p, _p, _p, _p, _p, _p, _p, _i, _i, _i, _f, _f, _i, _i, _p]),
    "ogv_bn_act_bwd": (_i, [_p, _p, _p, _p, _p, _p, _p, _p, _i, _i, _i, _i, _i, _p]),
    "ogv_head_bn_pool_ws_bytes": (_sz, [_i, _i]),
    "ogv_head_bn_pool_fwd": (_i, [_p, _p, _p, _p, _p, _p, _p, _p, _p, _i, _i, _i, _i, _f, _f, _i, _p]),
    "ogv_head_bn_pool_bwd": (_i, [_p, _p, _p, _p, _p, _p, _p, _p, _p, _i, _i, _i, _i, _i, _p]),
    "ogv_mix_images": (_i, [_p, _p, _p, _i, _i, _i, _i, _i, _i, _f, _f, _i, _i, _i, _i, _i, _p]),
    "ogv_mix_targets": (_i, [_p, _p, _p, _i, _i, _f, _f, _p]),
    "ogv_cast": (_i, [_p, _i, _p, _i, _sz, _p]),
    "ogv_step_flag": (_i, [_p, _i, _p, _p]),
    "ogv_ce_ls_ws_bytes": (_sz, [_i]),
    "ogv_ce_ls_fwd": (_i, [_p, _p, _i, _i, _f, _p, _p, _p, _p, _p]),
    "ogv_ce_ls_bwd": (_i, [_p, _p, _p, _p, _i, _i, _f, _p, _p]),
    "ogv_clip_adamw_ws_bytes": (_sz, [ctypes.POINTER(AdamWTensor), _i]),
    "ogv_clip_adamw": (_i, [ctypes.POINTER(AdamWTensor), _i, ctypes.POINTER(AdamWGroup), _i, _p, _f, _p, _p]),
    "ogv_schedule_step": (_i, [_p, _p, _p, ctypes.POINTER(_p), ctypes.POINTER(_f), _i, _i, _i, _f, _p]),
    "ogv_copy_batch_f32": (_i, [ctypes.POINTER(CopySeg), _i, _f, _p]),
}

OGV_F32, OGV_BF16 = 0, 1
OGV_OK, OGV_ERR_ARG, OGV_ERR_UNSUPPORTED, OGV_ERR_LAUNCH = 0, 1, 2, 3   # include/ogv.h status codes
ACT = {None: 0, "none": 0, "gelu": 1, "silu": 2, "relu": 3}

_lib = None


def load() -> ctypes.CDLL:
    """Load (once) and return the library; raises OSError / AttributeError loudly on failure."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise OSError(f"libogv_hip.so not found at {LIB_PATH}: build it with "
                      f"`python -c 'import __graft_entry__ as g; g.build()'` (or make -C .../csrc)")
    lib = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)  # AttributeError if the symbol is missing
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


class OgvError(RuntimeError):
    pass


def check(rc: int, what: str) -> None:
    if rc != 0:
        msg = load().ogv_last_error().decode(errors="replace")
        raise OgvError(f"{what} failed (code {rc}): {msg}")


def version() -> str:
    return load().ogv_version().decode()
