// Shared device/host helpers for libogv_hip.so (gfx950 only).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>
#include <stdarg.h>

#include "../../include/ogv.h"

typedef __bf16 bf16;
typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) __bf16 bf16x4;
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(4))) short s16x4;

namespace ogv {
int skip_mask();   // knob "skip" (ogv_gemm.hip): what-if timing experiments only

// BatchNorm batch statistics are accumulated as sums shifted by the running mean (fp64).  A
// non-finite running mean (a NaN batch poisons it, exactly as in torch's BatchNorm2d) must not
// leak into the train-mode output, which torch computes from the batch alone: such a shift is 0.
__device__ __forceinline__ float bn_shift(float v) { return __builtin_isfinite(v) ? v : 0.f; }

// ---------------------------------------------------------------- host-side error plumbing
void set_error(const char* fmt, ...);
int check_launch(const char* what);
// Dynamic LDS above the 64 KB default needs the kernel's grant raised (to 160 KB) once per kernel and
// DEVICE; returns false when the runtime refuses it (or bytes > 160 KB), so callers can plan around it.
bool lds_grant(const void* kern, size_t bytes);
// The current device lets one workgroup opt in to 160 KB of LDS (cached per device).  The *_supported
// queries of the kernels that need more than 64 KB answer 0 without it, so callers take the unfused path.
// With no device at all it answers true: the queries stay pure shape questions (nothing can launch).
bool lds_160k();
// lds_grant for a launch site with no fallback: on refusal the caller skips the launch and the next
// check_launch reports OGV_ERR_LAUNCH naming kname (never a silent skipped kernel).
bool lds_ok(const void* kern, size_t bytes, const char* kname);

#define OGV_REQUIRE(cond, ...)                 \
  do {                                         \
    if (!(cond)) {                             \
      ::ogv::set_error(__VA_ARGS__);           \
      return OGV_ERR_ARG;                      \
    }                                          \
  } while (0)

// deterministic "sum the rows of an fp32 slab" (ogv_dwconv.hip)
size_t colreduce_tmp_floats(long R, long n);
// dst[j] = sum_r src[r*ld + j] for j < n; with dst2, columns j >= n1 go to dst2[j - n1] instead.
void colreduce(const float* src, float* dst, long R, long n, long ld, float* tmp, hipStream_t s,
               float* dst2 = nullptr, long n1 = 0);
// fp64 variant (BatchNorm batch statistics); tmp needs colreduce_tmp_floats(R, n) doubles
void colreduce(const double* src, double* dst, long R, long n, long ld, double* tmp, hipStream_t s);
// The same reduction for a PARAMETER GRADIENT (dst read by nothing before the optimizer): while the
// caller has deferral on (ogv_reduce_defer), recorded instead of launched and run later by
// ogv_reduce_flush as ONE batched launch with every other deferred reduction (same arithmetic as the
// single-pass colreduce4 kernel); otherwise identical to colreduce.
void colreduce_param(const float* src, float* dst, long R, long n, long ld, float* tmp, hipStream_t s,
                     float* dst2 = nullptr, long n1 = 0);
// Deferred tap-major -> channel-major reduction (the depthwise weight gradient: src columns tap*C + c,
// dst[c*9 + tap]); returns false (nothing recorded) when deferral is off or the shape does not fit
bool colreduce_param_tap(const float* src, float* dst, long R, long C, long ld);

static inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }
static inline unsigned cdiv(long a, long b) { return (unsigned)((a + b - 1) / b); }

// ---------------------------------------------------------------- element conversion
__device__ __forceinline__ float to_f(float x) { return x; }
__device__ __forceinline__ float to_f(bf16 x) { return (float)x; }
template <typename T> __device__ __forceinline__ T from_f(float x);
template <> __device__ __forceinline__ float from_f<float>(float x) { return x; }
template <> __device__ __forceinline__ bf16 from_f<bf16>(float x) { return (bf16)x; }

// Vector load/store of V consecutive elements (V*sizeof(T) must be 4, 8 or 16 bytes aligned).
template <typename T, int V> struct VecT;
template <> struct VecT<float, 1> { typedef float type; };
template <> struct VecT<float, 2> { typedef float2 type; };
template <> struct VecT<float, 4> { typedef float4 type; };
template <> struct VecT<float, 8> { typedef float4 type; };  // two loads
template <> struct VecT<bf16, 1> { typedef bf16 type; };
template <> struct VecT<bf16, 2> { typedef uint32_t type; };
template <> struct VecT<bf16, 4> { typedef uint2 type; };
template <> struct VecT<bf16, 8> { typedef uint4 type; };

template <typename T, int V>
__device__ __forceinline__ void load_vec(const T* __restrict__ p, float* out) {
  if constexpr (sizeof(T) == 4 && V == 8) {
    float4 a = *reinterpret_cast<const float4*>(p);
    float4 b = *reinterpret_cast<const float4*>(p + 4);
    out[0] = a.x; out[1] = a.y; out[2] = a.z; out[3] = a.w;
    out[4] = b.x; out[5] = b.y; out[6] = b.z; out[7] = b.w;
  } else if constexpr (V == 1) {
    out[0] = to_f(p[0]);
  } else {
    typedef typename VecT<T, V>::type VT;
    VT v = *reinterpret_cast<const VT*>(p);
    const T* e = reinterpret_cast<const T*>(&v);
#pragma unroll
    for (int i = 0; i < V; ++i) out[i] = to_f(e[i]);
  }
}

template <typename T, int V>
__device__ __forceinline__ void store_vec(T* __restrict__ p, const float* in) {
  if constexpr (sizeof(T) == 4 && V == 8) {
    *reinterpret_cast<float4*>(p) = make_float4(in[0], in[1], in[2], in[3]);
    *reinterpret_cast<float4*>(p + 4) = make_float4(in[4], in[5], in[6], in[7]);
  } else if constexpr (V == 1) {
    p[0] = from_f<T>(in[0]);
  } else {
    typedef typename VecT<T, V>::type VT;
    VT v;
    T* e = reinterpret_cast<T*>(&v);
#pragma unroll
    for (int i = 0; i < V; ++i) e[i] = from_f<T>(in[i]);
    *reinterpret_cast<VT*>(p) = v;
  }
}

// V consecutive elements kept as the raw loaded bits (bf16 pairs / fp32) until they are used, so a
// prefetch need not retire before the next use of any LATER load (vmcnt retires in issue order), and a
// load under a (uniform) branch is not converted -- hence waited for -- inside the branch.
template <typename T, int V>
struct RawVec {
  static constexpr int NV = (sizeof(T) == 4 && V == 8) ? 2 : 1;
  typedef typename VecT<T, V>::type VT;
  VT v[NV];
  __device__ __forceinline__ void load(const T* __restrict__ p) {
#pragma unroll
    for (int k = 0; k < NV; ++k) v[k] = *reinterpret_cast<const VT*>(p + k * (V / NV));
  }
  __device__ __forceinline__ void unpack(float* out) const {
    const T* e = reinterpret_cast<const T*>(v);
#pragma unroll
    for (int i = 0; i < V; ++i) out[i] = to_f(e[i]);
  }
};

// ---------------------------------------------------------------- XCD-aware block order
// Hardware block i runs on XCD i % 8.  Logical block id = (i % 8) * per + i / 8 hands each XCD a
// contiguous range of logical ids, so blocks that differ only in the fastest index (e.g. the
// channel tiles of one row slice of an NHWC tensor, which read the same cache lines) share one
// L2.  Launch xcd_grid(nb) blocks; xcd_block() returns false for the padding blocks.
static inline unsigned xcd_grid(long nb) { return (unsigned)(((nb + 7) / 8) * 8); }
__device__ __forceinline__ bool xcd_block(long nb, long& id) {
  const long per = (nb + 7) / 8;
  id = (long)(blockIdx.x & 7) * per + (blockIdx.x >> 3);
  return id < nb;
}

// ---------------------------------------------------------------- activations (exact erf GELU)
// logistic sigmoid with the hardware reciprocal (v_rcp_f32, 1 ulp) instead of an IEEE division
__device__ __forceinline__ float fast_sigmoid(float x) { return __builtin_amdgcn_rcpf(1.0f + __expf(-x)); }

// Phi(x) = 0.5 (1 + erf(x / sqrt 2)) for the exact (erf) GELU of nn.GELU().  erf from
// Abramowitz & Stegun 7.1.26 (|abs err| <= 1.5e-7, i.e. fp32-level): branch-free, one v_rcp and
// one v_exp, where the library erff evaluates two divergent polynomial branches.  Also returns
// e = exp(-x^2 / 2), which the derivative's pdf term reuses.
__device__ __forceinline__ float gelu_cdf(float x, float& e) {
  const float u = fabsf(x) * 0.70710678118654752f;
  const float t = __builtin_amdgcn_rcpf(fmaf(0.3275911f, u, 1.0f));
  float p = fmaf(t, 1.061405429f, -1.453152027f);
  p = fmaf(t, p, 1.421413741f);
  p = fmaf(t, p, -0.284496736f);
  p = fmaf(t, p, 0.254829592f);
  e = __expf(-u * u);
  const float h = 0.5f * (p * t) * e;  // 0.5 * erfc(u)
  return x >= 0.f ? 1.0f - h : h;
}

__device__ __forceinline__ float act_fwd(int act, float x) {
  switch (act) {
    case OGV_ACT_GELU: {
      float e;
      return x * gelu_cdf(x, e);
    }
    case OGV_ACT_SILU: return x * fast_sigmoid(x);
    case OGV_ACT_RELU: return x > 0.f ? x : 0.f;
    default: return x;
  }
}
// d act / dx evaluated at the pre-activation x
__device__ __forceinline__ float act_grad(int act, float x) {
  switch (act) {
    case OGV_ACT_GELU: {
      float e;
      const float cdf = gelu_cdf(x, e);
      return fmaf(x * 0.39894228040143268f, e, cdf);
    }
    case OGV_ACT_SILU: {
      const float s = fast_sigmoid(x);
      return s * (1.0f + x * (1.0f - s));
    }
    case OGV_ACT_RELU: return x > 0.f ? 1.f : 0.f;
    default: return 1.f;
  }
}
// act(x) and act'(x) with their shared transcendental evaluated once (bit-identical to act_fwd / act_grad:
// the same expressions on the same values; the compiler does not always merge the two when registers are tight)
__device__ __forceinline__ void act_both(int act, float x, float& f, float& g) {
  switch (act) {
    case OGV_ACT_GELU: {
      float e;
      const float cdf = gelu_cdf(x, e);
      f = x * cdf;
      g = fmaf(x * 0.39894228040143268f, e, cdf);
      return;
    }
    case OGV_ACT_SILU: {
      const float s = fast_sigmoid(x);
      f = x * s;
      g = s * (1.0f + x * (1.0f - s));
      return;
    }
    default:
      f = act_fwd(act, x);
      g = act_grad(act, x);
  }
}

// ---------------------------------------------------------------- wave reductions (wave64)
// Exchanges inside a row of 16 lanes go through DPP (an operand modifier of a VALU instruction);
// __shfl_xor lowers to ds_bpermute, an LDS round trip per call.  Butterfly partners: xor 1 and
// xor 2 (quad_perm), then the mirrored lane of the other quad (row_half_mirror) and of the other
// half-row (row_mirror): after those four steps every lane of a row holds the row total, the same
// value in all 16 lanes (a + b == b + a).  The steps across rows (16, 32) stay shuffles.
template <int CTRL>
__device__ __forceinline__ float dpp_mov(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), CTRL, 0xF, 0xF, false));
}
constexpr int DPP_XOR1 = 0xB1, DPP_XOR2 = 0x4E, DPP_HALF_MIRROR = 0x141, DPP_MIRROR = 0x140;

template <int G>
__device__ __forceinline__ float group_sum(float v) {  // sum within aligned groups of G lanes
  static_assert(G == 1 || G == 2 || G == 4 || G == 8 || G == 16 || G == 32 || G == 64, "power of two <= 64");
  if constexpr (G >= 2) v += dpp_mov<DPP_XOR1>(v);
  if constexpr (G >= 4) v += dpp_mov<DPP_XOR2>(v);
  if constexpr (G >= 8) v += dpp_mov<DPP_HALF_MIRROR>(v);
  if constexpr (G >= 16) v += dpp_mov<DPP_MIRROR>(v);
  if constexpr (G >= 32) v += __shfl_xor(v, 16, 64);
  if constexpr (G >= 64) v += __shfl_xor(v, 32, 64);
  return v;
}
template <int G>
__device__ __forceinline__ float group_max(float v) {
  static_assert(G == 1 || G == 2 || G == 4 || G == 8 || G == 16 || G == 32 || G == 64, "power of two <= 64");
  if constexpr (G >= 2) v = fmaxf(v, dpp_mov<DPP_XOR1>(v));
  if constexpr (G >= 4) v = fmaxf(v, dpp_mov<DPP_XOR2>(v));
  if constexpr (G >= 8) v = fmaxf(v, dpp_mov<DPP_HALF_MIRROR>(v));
  if constexpr (G >= 16) v = fmaxf(v, dpp_mov<DPP_MIRROR>(v));
  if constexpr (G >= 32) v = fmaxf(v, __shfl_xor(v, 16, 64));
  if constexpr (G >= 64) v = fmaxf(v, __shfl_xor(v, 32, 64));
  return v;
}
__device__ __forceinline__ float wave_sum(float v) { return group_sum<64>(v); }

}  // namespace ogv
