// LayerNorm over the contiguous channel dim of [M, C] rows (NHWC activations).
// Replaces nn.LayerNorm in LayerNorm2d (src/model/outlook_attention.py:24-31; the two permute+
// contiguous copies disappear because the activation is already channel-last) and
// OutGridBlock.norm2/norm3 (src/model/Out_Grid_Block.py:69,84,98,102).
// A row is owned by G lanes of one wave (G = pow2 >= C/VEC); two-pass mean/variance in registers.
#include "ogv_common.h"

namespace ogv {

template <typename T, int G, int NV, int VEC, int RPI = 2>
__global__ __launch_bounds__(256) void ln_fwd_kernel(const T* __restrict__ x, const float* __restrict__ gamma,
                                                     const float* __restrict__ beta, T* __restrict__ y,
                                                     float* __restrict__ mean_out, float* __restrict__ rstd_out,
                                                     long M, int C, float eps) {
  constexpr int E = NV * VEC;
  const int lane_g = threadIdx.x % G;
  const long rows_per_block = blockDim.x / G;
  float gw[E], bw[E];
  bool valid[NV];
#pragma unroll
  for (int v = 0; v < NV; ++v) {
    const int c = (v * G + lane_g) * VEC;
    valid[v] = c < C;
    // unconditional loads at a clamped column (a lane without a column stores nothing): a per-lane guard
    // put each of these loads in a branch of its own and the rows' loads waited behind all of them
    const int cc = valid[v] ? c : 0;
#pragma unroll
    for (int i = 0; i < VEC; ++i) {
      gw[v * VEC + i] = gamma ? gamma[cc + i] : 1.f;
      bw[v * VEC + i] = beta ? beta[cc + i] : 0.f;
    }
  }
  const float invC = 1.f / (float)C;
  // RPI rows per iteration, every load issued before any use (RPI independent reduction chains)
  const long stride = (long)gridDim.x * rows_per_block;
  for (long row0 = blockIdx.x * rows_per_block + threadIdx.x / G; row0 < M; row0 += RPI * stride) {
    float xv[RPI][E];
    // raw bits of every row first, converted once all are in flight (converting next to each load let the
    // scheduler put the next row's load behind the first row's wait: one round trip per row)
    RawVec<T, VEC> rx[RPI][NV];
#pragma unroll
    for (int q = 0; q < RPI; ++q) {
      const long row = min(row0 + q * stride, M - 1);
#pragma unroll
      for (int v = 0; v < NV; ++v) rx[q][v].load(x + row * C + min((v * G + lane_g) * VEC, C - VEC));
    }
    __builtin_amdgcn_sched_barrier(0);   // (the machine scheduler would otherwise still interleave them)
#pragma unroll
    for (int q = 0; q < RPI; ++q)
#pragma unroll
      for (int v = 0; v < NV; ++v) rx[q][v].unpack(xv[q] + v * VEC);
#pragma unroll
    for (int q = 0; q < RPI; ++q) {
      const long row = row0 + q * stride;
      if (row >= M) break;
      float s = 0.f;
#pragma unroll
      for (int v = 0; v < NV; ++v)
#pragma unroll
        for (int i = 0; i < VEC; ++i) s += valid[v] ? xv[q][v * VEC + i] : 0.f;
      const float mu = group_sum<G>(s) * invC;
      float ss = 0.f;
#pragma unroll
      for (int v = 0; v < NV; ++v)
#pragma unroll
        for (int i = 0; i < VEC; ++i) {
          const float d = valid[v] ? xv[q][v * VEC + i] - mu : 0.f;
          ss = fmaf(d, d, ss);
        }
      const float rs = rsqrtf(group_sum<G>(ss) * invC + eps);
      T* yr = y + row * C;
#pragma unroll
      for (int v = 0; v < NV; ++v) {
        const int c = (v * G + lane_g) * VEC;
        if (valid[v]) {
          float o[VEC];
#pragma unroll
          for (int i = 0; i < VEC; ++i) o[i] = (xv[q][v * VEC + i] - mu) * rs * gw[v * VEC + i] + bw[v * VEC + i];
          store_vec<T, VEC>(yr + c, o);
        }
      }
      if (lane_g == 0) {
        if (mean_out) mean_out[row] = mu;
        if (rstd_out) rstd_out[row] = rs;
      }
    }
  }
}

// dx = rstd * (g - mean(g) - xhat * mean(g * xhat)),  g = dy * gamma
// per-block partial dgamma = sum dy*xhat, dbeta = sum dy  -> part[block][2][C]
template <typename T, int G, int NV, int VEC, int RPI = 2>
__global__ __launch_bounds__(256) void ln_bwd_kernel(const T* __restrict__ dy, const T* __restrict__ x,
                                                     const float* __restrict__ gamma, const float* __restrict__ mean,
                                                     const float* __restrict__ rstd, const T* __restrict__ dres,
                                                     T* __restrict__ dx, float* __restrict__ part, long M, int C) {
  constexpr int E = NV * VEC;
  const int lane_g = threadIdx.x % G;
  const long rows_per_block = blockDim.x / G;
  float gw[E], dgam[E], dbet[E];
  bool valid[NV];
#pragma unroll
  for (int v = 0; v < NV; ++v) {
    const int c = (v * G + lane_g) * VEC;
    valid[v] = c < C;
    const int cc = valid[v] ? c : 0;   // (clamped, unconditional: as in the forward; d = 0 on such lanes)
#pragma unroll
    for (int i = 0; i < VEC; ++i) {
      gw[v * VEC + i] = gamma ? gamma[cc + i] : 1.f;
      dgam[v * VEC + i] = 0.f;
      dbet[v * VEC + i] = 0.f;
    }
  }
  const float invC = 1.f / (float)C;
  // RPI rows per iteration, every load of all of them (x, dy, dres, mean, rstd) issued before any use
  const long stride = (long)gridDim.x * rows_per_block;
  for (long row0 = blockIdx.x * rows_per_block + threadIdx.x / G; row0 < M; row0 += RPI * stride) {
    float xv[RPI][E], dv[RPI][E], rv[RPI][E], mu[RPI], rs[RPI];
    // raw bits first, converted after every load of both rows is in flight (a conversion next to a
    // load under the dres branch made the compiler wait for each of those loads in turn)
    RawVec<T, VEC> rx[RPI][NV], rd[RPI][NV], rr[RPI][NV];
#pragma unroll
    for (int q = 0; q < RPI; ++q) {
      const long row = min(row0 + q * stride, M - 1);
      mu[q] = mean[row];
      rs[q] = rstd[row];
#pragma unroll
      for (int v = 0; v < NV; ++v) {
        const int c = min((v * G + lane_g) * VEC, C - VEC);
        rx[q][v].load(x + row * C + c);
        rd[q][v].load(dy + row * C + c);
      }
    }
    if (dres) {
#pragma unroll
      for (int q = 0; q < RPI; ++q) {
        const long row = min(row0 + q * stride, M - 1);
#pragma unroll
        for (int v = 0; v < NV; ++v) rr[q][v].load(dres + row * C + min((v * G + lane_g) * VEC, C - VEC));
      }
    }
#pragma unroll
    for (int q = 0; q < RPI; ++q)
#pragma unroll
      for (int v = 0; v < NV; ++v) {
        rx[q][v].unpack(xv[q] + v * VEC);
        rd[q][v].unpack(dv[q] + v * VEC);
        if (dres) rr[q][v].unpack(rv[q] + v * VEC);
      }
#pragma unroll
    for (int q = 0; q < RPI; ++q) {
      const long row = row0 + q * stride;
      if (row >= M) break;
      float xh[E], gv[E];
      float s1 = 0.f, s2 = 0.f;
#pragma unroll
      for (int v = 0; v < NV; ++v) {
#pragma unroll
        for (int i = 0; i < VEC; ++i) {
          const int e = v * VEC + i;
          const float d = valid[v] ? dv[q][e] : 0.f;
          xh[e] = valid[v] ? (xv[q][e] - mu[q]) * rs[q] : 0.f;
          gv[e] = d * gw[e];
          s1 += gv[e];
          s2 = fmaf(gv[e], xh[e], s2);
          dgam[e] = fmaf(d, xh[e], dgam[e]);
          dbet[e] += d;
        }
      }
      const float m1 = group_sum<G>(s1) * invC;
      const float m2 = group_sum<G>(s2) * invC;
#pragma unroll
      for (int v = 0; v < NV; ++v) {
        const int c = (v * G + lane_g) * VEC;
        if (valid[v]) {
          float o[VEC];
#pragma unroll
          for (int i = 0; i < VEC; ++i) {
            o[i] = rs[q] * (gv[v * VEC + i] - m1 - xh[v * VEC + i] * m2);
            if (dres) o[i] += rv[q][v * VEC + i];  // gradient of the residual branch that reused x
          }
          store_vec<T, VEC>(dx + row * C + c, o);
        }
      }
    }
  }
  // reduce the per-lane partials of the (256/G) row slots of this block: across a wave's 64/G slots with
  // xor shuffles (every value at once), then the 4 waves through LDS, ONE barrier (was 2 x 2E barriers and
  // a serial 256/G-long LDS walk per value)
  float* out = part + (long)blockIdx.x * 2 * C;
#pragma unroll
  for (int e = 0; e < E; ++e)
    for (int o = G; o < 64; o <<= 1) {
      dgam[e] += __shfl_xor(dgam[e], o, 64);
      dbet[e] += __shfl_xor(dbet[e], o, 64);
    }
  __shared__ float red[4][E * G];   // <= 32 KB (E * G <= 2048)
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
  for (int which = 0; which < 2; ++which) {
    if (which) __syncthreads();   // the first pass's readers are done
    if (lane < G) {
#pragma unroll
      for (int e = 0; e < E; ++e) red[wave][e * G + lane] = which ? dbet[e] : dgam[e];
    }
    __syncthreads();
    for (int r = threadIdx.x; r < E * G; r += blockDim.x) {
      const float acc = ((red[0][r] + red[1][r]) + red[2][r]) + red[3][r];
      const int e = r / G, lg = r - e * G, v = e / VEC, i = e - v * VEC;
      const int c = (v * G + lg) * VEC + i;
      if (c < C) out[which * C + c] = acc;
    }
  }
}

struct LnPlan {
  int G, NV, VEC;
};

static int ln_plan(int C, LnPlan& p) {
  if (C % 8 == 0) p.VEC = 8;
  else if (C % 4 == 0) p.VEC = 4;
  else return OGV_ERR_UNSUPPORTED;
  const int nvec = C / p.VEC;
  int G = 1;
  while (G < nvec && G < 64) G <<= 1;
  p.G = G < 2 ? 2 : G;
  p.NV = (nvec + p.G - 1) / p.G;
  if (p.NV > 4) return OGV_ERR_UNSUPPORTED;
  if (p.NV == 3) p.NV = 4;
  return OGV_OK;
}

static long ln_blocks(long M, int G) {
  const long rows_per_block = 256 / G;
  long nb = (M + rows_per_block - 1) / rows_per_block;
  return nb < 2048 ? nb : 2048;
}

#define OGV_LN_CASE_NV(T, G, VEC, FN, ...)                 \
  switch (p.NV) {                                          \
    case 1: FN<T, G, 1, VEC>(__VA_ARGS__); break;          \
    case 2: FN<T, G, 2, VEC>(__VA_ARGS__); break;          \
    default: FN<T, G, 4, VEC>(__VA_ARGS__); break;         \
  }
#define OGV_LN_CASE_G(T, VEC, FN, ...)                     \
  switch (p.G) {                                           \
    case 2: OGV_LN_CASE_NV(T, 2, VEC, FN, __VA_ARGS__) break;   \
    case 4: OGV_LN_CASE_NV(T, 4, VEC, FN, __VA_ARGS__) break;   \
    case 8: OGV_LN_CASE_NV(T, 8, VEC, FN, __VA_ARGS__) break;   \
    case 16: OGV_LN_CASE_NV(T, 16, VEC, FN, __VA_ARGS__) break; \
    case 32: OGV_LN_CASE_NV(T, 32, VEC, FN, __VA_ARGS__) break; \
    default: OGV_LN_CASE_NV(T, 64, VEC, FN, __VA_ARGS__) break; \
  }
#define OGV_LN_DISPATCH(FN, ...)                                               \
  do {                                                                         \
    if (dt == OGV_BF16) {                                                      \
      if (p.VEC == 8) { OGV_LN_CASE_G(bf16, 8, FN, __VA_ARGS__) }              \
      else { OGV_LN_CASE_G(bf16, 4, FN, __VA_ARGS__) }                         \
    } else {                                                                   \
      if (p.VEC == 8) { OGV_LN_CASE_G(float, 8, FN, __VA_ARGS__) }             \
      else { OGV_LN_CASE_G(float, 4, FN, __VA_ARGS__) }                        \
    }                                                                          \
  } while (0)

// knob "ln_rpi": rows per iteration of the LayerNorm kernels (2 or 4, default 2): 4 measured slower on the
// 7M step (backward 0.60 -> 0.66 ms: 168 VGPRs, 3 waves per SIMD; forward unchanged), profiles/r05j_ln.log
static int g_ln_rpi = 2;
void set_ln_rpi(int v) { g_ln_rpi = v >= 4 ? 4 : 2; }

template <typename T, int G, int NV, int VEC>
static void ln_fwd_launch(const void* x, const float* gamma, const float* beta, void* y, float* mean, float* rstd,
                          long M, int C, float eps, hipStream_t s) {
  if (g_ln_rpi == 4 && NV <= 2)
    ln_fwd_kernel<T, G, NV, VEC, 4><<<(unsigned)ln_blocks(M, G), 256, 0, s>>>((const T*)x, gamma, beta, (T*)y, mean,
                                                                              rstd, M, C, eps);
  else
    ln_fwd_kernel<T, G, NV, VEC, 2><<<(unsigned)ln_blocks(M, G), 256, 0, s>>>((const T*)x, gamma, beta, (T*)y, mean,
                                                                              rstd, M, C, eps);
}

template <typename T, int G, int NV, int VEC>
static void ln_bwd_launch(const void* dy, const void* x, const float* gamma, const float* mean, const float* rstd,
                          const void* dres, void* dx, float* part, long nb, long M, int C, hipStream_t s) {
  if (g_ln_rpi == 4 && NV <= 2)
    ln_bwd_kernel<T, G, NV, VEC, 4><<<(unsigned)nb, 256, 0, s>>>((const T*)dy, (const T*)x, gamma, mean, rstd,
                                                                 (const T*)dres, (T*)dx, part, M, C);
  else
    ln_bwd_kernel<T, G, NV, VEC, 2><<<(unsigned)nb, 256, 0, s>>>((const T*)dy, (const T*)x, gamma, mean, rstd,
                                                                 (const T*)dres, (T*)dx, part, M, C);
}

}  // namespace ogv

using namespace ogv;

extern "C" int ogv_layernorm_fwd(const void* x, const float* gamma, const float* beta, void* y, float* mean,
                                 float* rstd, int M, int C, float eps, ogv_dtype dt, void* stream) {
  if (skip_mask() & 16) return OGV_OK;
  OGV_REQUIRE(x && y, "ogv_layernorm_fwd: null pointer");
  OGV_REQUIRE(M >= 0 && C > 0, "ogv_layernorm_fwd: bad shape M=%d C=%d", M, C);
  LnPlan p;
  OGV_REQUIRE(ln_plan(C, p) == OGV_OK, "ogv_layernorm_fwd: C=%d unsupported (need C%%4==0, C<=2048)", C);
  if (M == 0) return OGV_OK;
  OGV_LN_DISPATCH(ln_fwd_launch, x, gamma, beta, y, mean, rstd, (long)M, C, eps, as_stream(stream));
  return check_launch("ogv_layernorm_fwd");
}

// tuning knob "ln_bwd_blocks": grid cap of the backward (each block's dgamma/dbeta partial is a row
// of the slab, summed by one colreduce pass up to 2048 rows)
static long g_ln_bwd_cap = 1024;
namespace ogv {
void set_ln_bwd_blocks(int v) { g_ln_bwd_cap = v > 0 ? v : 1024; }
}
static long ln_bwd_blocks(long M, int G) {
  const long rows_per_block = 256 / G;
  long nb = (M + rows_per_block - 1) / rows_per_block;
  return nb < g_ln_bwd_cap ? nb : g_ln_bwd_cap;
}

extern "C" size_t ogv_layernorm_bwd_ws_bytes(int M, int C) {
  LnPlan p;
  if (ln_plan(C, p) != OGV_OK) return 0;
  const long nb = ln_bwd_blocks(M > 0 ? M : 1, p.G);
  return ((size_t)nb * 2 * C + colreduce_tmp_floats(nb, 2L * C) + 2 * (size_t)C) * sizeof(float);
}

extern "C" int ogv_layernorm_bwd(const void* dy, const void* x, const float* gamma, const float* mean,
                                 const float* rstd, const void* dres, void* dx, float* dgamma, float* dbeta, void* ws,
                                 int M, int C, ogv_dtype dt, void* stream) {
  if (skip_mask() & 16) return OGV_OK;
  OGV_REQUIRE(dy && x && mean && rstd && dx && ws, "ogv_layernorm_bwd: null pointer");
  OGV_REQUIRE(M > 0 && C > 0, "ogv_layernorm_bwd: bad shape M=%d C=%d", M, C);
  LnPlan p;
  OGV_REQUIRE(ln_plan(C, p) == OGV_OK, "ogv_layernorm_bwd: C=%d unsupported", C);
  const long nb = ln_bwd_blocks(M, p.G);
  hipStream_t s = as_stream(stream);
  float* part = (float*)ws;
  float* tmp = part + (size_t)nb * 2 * C;
  OGV_LN_DISPATCH(ln_bwd_launch, dy, x, gamma, mean, rstd, dres, dx, part, nb, (long)M, C, s);
  // partials are [nb][dgamma(C) | dbeta(C)]: reduced straight into the caller's buffers
  if (dgamma && dbeta) colreduce_param(part, dgamma, nb, 2L * C, 2L * C, tmp, s, dbeta, C);
  else if (dgamma) colreduce_param(part, dgamma, nb, C, 2L * C, tmp, s);
  else if (dbeta) colreduce_param(part + C, dbeta, nb, C, 2L * C, tmp, s);
  return check_launch("ogv_layernorm_bwd");
}
