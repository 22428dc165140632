// Streaming weight gradient for the large-M projections (gfx950).
//
//   dW[n, k] = sum_m rs(m) G[m, n] * pro(X)[m, k],   dbias[n] = sum_m rs(m) G[m, n]
//
// At the large-M stages (M = B*H*W = 131k-524k rows) with N, K <= 384 the reduction runs over a
// very long M and the output tile is small, so instead of a block-cooperative tile loop:
//   * a workgroup owns one BN x BK output tile over one M slab; each of its 4 waves walks its
//     own 16-row chunks of the slab with NO workgroup barrier: it loads the chunk's G and X row
//     segments (16-B vector loads), applies the row scale / X prologue in registers, stages them
//     in a wave-private LDS slab [16 rows][cols], and reads MFMA fragments back with
//     ds_read_b64_tr_b16 (the transpose that puts the reduction index m into the fragment's k),
//   * v_mfma_f32_16x16x16_bf16 accumulates the whole BN x BK tile in registers across the
//     wave's chunks (no per-chunk partial traffic),
//   * at the end the 4 waves' tiles are summed in a fixed order through LDS and the workgroup
//     writes one fp32 partial row [slab][N*K + N] (same layout as the tiled kernel, reduced by
//     the caller's colreduce).  Deterministic: fixed chunk order per wave, fixed wave order.
// Tiles of one slab are mapped to one XCD so their re-reads of the slab's G / X rows hit that L2.
#include "ogv_gemm.h"

namespace ogv {

constexpr int SW_NW = 4;   // waves per workgroup
constexpr int SW_CH = 16;  // rows per chunk (= MFMA k of 16x16x16)

// LDS row pitch (elements): 16 * odd, which keeps the transposed 64-bit reads conflict-free
template <int B>
__host__ __device__ constexpr int sw_pitch() { return ((B / 16) % 2 == 0) ? B + 16 : B + 32; }

template <int BN, int BK, int PA>
__global__ __launch_bounds__(SW_NW * 64) void swgrad_bf16_kernel(const bf16* __restrict__ G, int ldg,
                                                                 const bf16* __restrict__ X, int ldx, Pro pro,
                                                                 const float* __restrict__ rs, int rps,
                                                                 float* __restrict__ part, long ldp, int want_bias,
                                                                 int M, int N, int K, int nNt, int tiles, int S,
                                                                 int rows_per_slab) {
  constexpr int GP = sw_pitch<BN>(), XP = sw_pitch<BK>();
  constexpr int GC = BN / 8, XC = BK / 8;                // 16-B chunks per staged row (4, 6 or 8)
  constexpr int GCP = GC == 4 ? 4 : 8, XCP = XC == 4 ? 4 : 8;  // lanes per row (a lane keeps one chunk)
  constexpr int GL = SW_CH * GCP / 64, XL = SW_CH * XCP / 64;  // loads per lane per chunk
  constexpr int TN = BN / 16, TK = BK / 16;
  constexpr int WAVE_LDS = SW_CH * (GP + XP);            // bf16 elements
  constexpr int RED_FLOATS = BN * BK + SW_NW * BN;
  constexpr int LDS_BYTES = (SW_NW * WAVE_LDS * 2 > RED_FLOATS * 4) ? SW_NW * WAVE_LDS * 2 : RED_FLOATS * 4;
  __shared__ __attribute__((aligned(16))) char smem[LDS_BYTES];

  const int b = blockIdx.x, xcd = b & 7, local = b >> 3;
  const int tile = local % tiles, s = (local / tiles) * 8 + xcd;
  if (s >= S) return;
  const int nt = tile % nNt, kt = tile / nNt;
  const int n0 = nt * BN, k0 = kt * BK;
  const int mbeg = s * rows_per_slab;
  const int mend = min(M, mbeg + rows_per_slab);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const bool do_bias = want_bias && kt == 0;

  bf16* Gs = reinterpret_cast<bf16*>(smem) + wave * WAVE_LDS;
  bf16* Xs = Gs + SW_CH * GP;

  // this lane's fixed 8-column chunk of the G / X row segments
  const int gcc = lane % GCP, grow = lane / GCP, xcc = lane % XCP, xrow = lane / XCP;
  const int gn = n0 + gcc * 8, xk = k0 + xcc * 8;
  const bool gact = gcc < GC && gn < N, xact = xcc < XC && xk < K;

  f32x4 acc[TN][TK];
#pragma unroll
  for (int i = 0; i < TN; ++i)
#pragma unroll
    for (int j = 0; j < TK; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  float bacc[8];
#pragma unroll
  for (int q = 0; q < 8; ++q) bacc[q] = 0.f;
  // prologue scale / shift of this lane's X columns (loop-invariant; the SiLU form only)
  float psc[8], psh[8];
#pragma unroll
  for (int q = 0; q < 8; ++q) { psc[q] = 1.f; psh[q] = 0.f; }
  if constexpr (PA == OGV_ACT_SILU) {
    if (xact) {
      load_vec<float, 8>(pro.sc + xk, psc);
      load_vec<float, 8>(pro.sh + xk, psh);
    }
  }

  const int g = lane >> 4, c16 = lane & 15, qd = c16 >> 2, p4 = (c16 & 3) * 4;
  typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

  // Chunk loads use clamped (always valid) addresses and zero-select afterwards, so they are
  // unconditional: the next chunk's loads are in flight while this chunk is staged and multiplied
  // (only loads are in flight in this loop, so the in-order vmcnt wait is exact).
  constexpr bool use_gate = PA == OGV_ACT_SILU;  // MBConv project: BN2 scale/shift + SiLU + SE gate
  const int gcol = gact ? gn : 0, xcol = xact ? xk : 0;
  uint4 gr[GL], xr[XL], gn2[GL], xn2[XL];
  float rsv[GL], rsn[GL];
  float gtv[use_gate ? XL : 1][8], gtn[use_gate ? XL : 1][8];
  auto load_chunk = [&](int c, uint4 (&gd)[GL], uint4 (&xd)[XL], float (&rd)[GL], auto& td) {
#pragma unroll
    for (int t = 0; t < GL; ++t) {
      const int m = min(c + grow + t * (64 / GCP), mend - 1);
      gd[t] = *reinterpret_cast<const uint4*>(G + (long)m * ldg + gcol);
      rd[t] = rs ? rs[m / rps] : 1.f;
    }
#pragma unroll
    for (int t = 0; t < XL; ++t) {
      const int m = min(c + xrow + t * (64 / XCP), mend - 1);
      xd[t] = *reinterpret_cast<const uint4*>(X + (long)m * ldx + xcol);
      if constexpr (use_gate) load_vec<float, 8>(pro.gate + (long)(m / pro.rps) * pro.gld + xcol, td[t]);
    }
  };
  const int step = SW_NW * SW_CH;
  int c = mbeg + wave * SW_CH;
  if (c < mend) load_chunk(c, gr, xr, rsv, gtv);
  for (; c < mend; c += step) {
    const bool more = c + step < mend;
    if (more) load_chunk(c + step, gn2, xn2, rsn, gtn);
#pragma unroll
    for (int t = 0; t < GL; ++t) {
      const int r = grow + t * (64 / GCP), m = c + r;
      const bool ok = gact && m < mend;
      uint4 v = ok ? gr[t] : uint4{0u, 0u, 0u, 0u};
      bf16* e = reinterpret_cast<bf16*>(&v);
      if (rs) {
#pragma unroll
        for (int q = 0; q < 8; ++q) e[q] = (bf16)((float)e[q] * rsv[t]);
      }
      if (do_bias) {
#pragma unroll
        for (int q = 0; q < 8; ++q) bacc[q] += (float)e[q];
      }
      if (gcc < GC) *reinterpret_cast<uint4*>(Gs + r * GP + gcc * 8) = v;
    }
#pragma unroll
    for (int t = 0; t < XL; ++t) {
      const int r = xrow + t * (64 / XCP), m = c + r;
      const bool ok = xact && m < mend;
      uint4 v = ok ? xr[t] : uint4{0u, 0u, 0u, 0u};
      if constexpr (PA >= 0) {
        if (ok) {
          bf16* e = reinterpret_cast<bf16*>(&v);
          float f[8];
#pragma unroll
          for (int q = 0; q < 8; ++q)
            f[q] = act_fwd(PA, PA == OGV_ACT_SILU ? fmaf((float)e[q], psc[q], psh[q]) : (float)e[q]);
          if constexpr (use_gate) {
#pragma unroll
            for (int q = 0; q < 8; ++q) f[q] *= gtv[t][q];
          }
#pragma unroll
          for (int q = 0; q < 8; ++q) e[q] = (bf16)f[q];
        }
      }
      if (xcc < XC) *reinterpret_cast<uint4*>(Xs + r * XP + xcc * 8) = v;
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    s16x4 af[TN], xf[TK];
#pragma unroll
    for (int i = 0; i < TN; ++i)
      af[i] = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(Gs + (4 * g + qd) * GP + i * 16 + p4));
#pragma unroll
    for (int j = 0; j < TK; ++j)
      xf[j] = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(Xs + (4 * g + qd) * XP + j * 16 + p4));
#pragma unroll
    for (int i = 0; i < TN; ++i)
#pragma unroll
      for (int j = 0; j < TK; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(af[i], xf[j], acc[i][j], 0, 0, 0);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    if (more) {
#pragma unroll
      for (int t = 0; t < GL; ++t) { gr[t] = gn2[t]; rsv[t] = rsn[t]; }
#pragma unroll
      for (int t = 0; t < XL; ++t) {
        xr[t] = xn2[t];
        if constexpr (use_gate) {
#pragma unroll
          for (int q = 0; q < 8; ++q) gtv[t][q] = gtn[t][q];
        }
      }
    }
  }

  // ---- fixed-order reduction of the 4 waves' tiles (and bias sums) through LDS
  float* red = reinterpret_cast<float*>(smem);
  float* bred = red + BN * BK;  // [wave][BN]
  if (do_bias) {  // lanes sharing a chunk: xor tree over the row groups (deterministic)
#pragma unroll
    for (int q = 0; q < 8; ++q)
#pragma unroll
      for (int o = GCP; o < 64; o <<= 1) bacc[q] += __shfl_xor(bacc[q], o, 64);
  }
  __syncthreads();  // staging slabs are dead
  if (do_bias && lane < GC) {
#pragma unroll
    for (int q = 0; q < 8; ++q) bred[wave * BN + lane * 8 + q] = bacc[q];
  }
#pragma unroll 1
  for (int w = 0; w < SW_NW; ++w) {
    if (wave == w) {
#pragma unroll
      for (int i = 0; i < TN; ++i)
#pragma unroll
        for (int j = 0; j < TK; ++j)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            float* d = red + (i * 16 + 4 * g + r) * BK + j * 16 + c16;
            *d = (w == 0 ? 0.f : *d) + acc[i][j][r];
          }
    }
    __syncthreads();
  }
  float* dst = part + (long)s * ldp;
  for (int e = tid; e < BN * BK; e += SW_NW * 64) {
    const int n = n0 + e / BK, k = k0 + e % BK;
    if (n < N && k < K) dst[(long)n * K + k] = red[e];
  }
  if (do_bias) {
    for (int e = tid; e < BN; e += SW_NW * 64) {
      float t = 0.f;
#pragma unroll
      for (int w = 0; w < SW_NW; ++w) t += bred[w * BN + e];
      if (n0 + e < N) dst[(long)N * K + n0 + e] = t;
    }
  }
}

// ------------------------------------------------------------------------------------------------
struct SwPlan {
  int ok = 0, BN = 0, BK = 0, nNt = 0, nKt = 0, S = 0, rows = 0;
};

static int sw_tile(int D) {  // tile edge for an output dim: multiple of 16 in {32, 48, 64}, little padding
  if (D <= 32) return 32;
  if (D <= 48) return 48;
  if (D <= 64) return 64;
  if (D % 64 == 0) return 64;
  if (D % 48 == 0) return 48;
  return 64;
}

// knob "swg_min_m": smallest M routed to the streaming weight gradient (0 = sgemm_min_m)
static int g_swg_min_m = 0;
void set_swg_min_m(int v) { g_swg_min_m = v < 0 ? 0 : v; }

static SwPlan swgrad_plan(int M, int N, int K) {
  SwPlan p;
  if (M < (g_swg_min_m ? g_swg_min_m : sgemm_min_m()) || (N & 7) || (K & 7)) return p;
  p.BN = sw_tile(N);
  p.BK = sw_tile(K);
  p.nNt = (N + p.BN - 1) / p.BN;
  p.nKt = (K + p.BK - 1) / p.BK;
  const int tiles = p.nNt * p.nKt;
  // ~1536 workgroups (6 per CU), >= 4 chunks per wave; partial rows <= 512
  long S = (1536 + tiles - 1) / tiles;
  S = std::min<long>(S, M / (SW_NW * SW_CH * 4));
  S = std::max<long>(1, std::min<long>(S, 512));
  int rows = (int)((M + S - 1) / S);
  rows = (rows + SW_CH - 1) / SW_CH * SW_CH;
  p.S = (M + rows - 1) / rows;
  p.rows = rows;
  p.ok = 1;
  return p;
}

size_t swgrad_ws_floats(int M, int N, int K) {
  const SwPlan p = swgrad_plan(M, N, K);
  if (!p.ok) return 0;
  const long ld = (long)N * K + N;
  return (size_t)p.S * ld + colreduce_tmp_floats(p.S, ld);
}

template <int BN, int BK, int PA>
static void sw_launch(const SwPlan& p, const bf16* G, int ldg, const bf16* X, int ldx, const Pro& pro, const float* rs,
                      int rps, float* part, long ldp, bool bias, int M, int N, int K, hipStream_t s) {
  const int tiles = p.nNt * p.nKt;
  const unsigned grid = (unsigned)(((p.S + 7) / 8) * 8 * tiles);
  swgrad_bf16_kernel<BN, BK, PA><<<grid, SW_NW * 64, 0, s>>>(G, ldg, X, ldx, pro, rs, rps, part, ldp, bias ? 1 : 0, M,
                                                             N, K, p.nNt, tiles, p.S, p.rows);
}

template <int PA>
static void sw_dispatch_tile(const SwPlan& p, const bf16* G, int ldg, const bf16* X, int ldx, const Pro& pro,
                             const float* rs, int rps, float* part, long ldp, bool bias, int M, int N, int K,
                             hipStream_t s) {
#define OGV_SW_K(BN_)                                                                                  \
  do {                                                                                                 \
    if (p.BK == 32) sw_launch<BN_, 32, PA>(p, G, ldg, X, ldx, pro, rs, rps, part, ldp, bias, M, N, K, s); \
    else if (p.BK == 48) sw_launch<BN_, 48, PA>(p, G, ldg, X, ldx, pro, rs, rps, part, ldp, bias, M, N, K, s); \
    else sw_launch<BN_, 64, PA>(p, G, ldg, X, ldx, pro, rs, rps, part, ldp, bias, M, N, K, s);          \
  } while (0)
  if (p.BN == 32) OGV_SW_K(32);
  else if (p.BN == 48) OGV_SW_K(48);
  else OGV_SW_K(64);
#undef OGV_SW_K
}

// Returns the number of partial rows written into part (layout [S][N*K + N]), 0 if not handled.
int swgrad_try(const void* G, int ldg, const void* X, int ldx, const Pro& pro, const float* rs, int rps, float* part,
               bool bias, int M, int N, int K, hipStream_t s) {
  if (!sgemm_mode()) return 0;
  if ((ldg & 7) || (ldx & 7) || (reinterpret_cast<uintptr_t>(G) & 15) || (reinterpret_cast<uintptr_t>(X) & 15))
    return 0;
  // prologue forms compiled here: GELU alone (MLP fc2) or BN scale/shift + SiLU + SE gate (MBConv project)
  const bool gelu_only = pro.act == OGV_ACT_GELU && !pro.sc && !pro.sh && !pro.gate;
  const bool bn_silu_gate = pro.act == OGV_ACT_SILU && pro.sc && pro.sh && pro.gate && !(pro.gld & 7);
  if (pro.any() && !gelu_only && !bn_silu_gate) return 0;
  const SwPlan p = swgrad_plan(M, N, K);
  if (!p.ok) return 0;
  const long ldp = (long)N * K + N;
  const bf16* g = static_cast<const bf16*>(G);
  const bf16* x = static_cast<const bf16*>(X);
  if (!pro.any()) sw_dispatch_tile<-1>(p, g, ldg, x, ldx, pro, rs, rps, part, ldp, bias, M, N, K, s);
  else if (pro.act == OGV_ACT_GELU) sw_dispatch_tile<OGV_ACT_GELU>(p, g, ldg, x, ldx, pro, rs, rps, part, ldp, bias, M, N, K, s);
  else sw_dispatch_tile<OGV_ACT_SILU>(p, g, ldg, x, ldx, pro, rs, rps, part, ldp, bias, M, N, K, s);
  return p.S;
}

}  // namespace ogv
