// Grid multi-head self-attention on MFMA (bf16, N >= 16 tokens per grid group).
//
// Same semantics and addressing as ogv_grid.hip (strided grid partition folded into the pixel
// index, qkv channel s*C + head*hd + d, out channel head*hd + d, fp32 LSE saved per (pixel, head)),
// but the QK^T / PV products run on v_mfma_f32_16x16x32_bf16 / 16x16x16_bf16 in flash-attention
// form: one wave owns a 16-row block of one (group, head) and walks the other side in 16-token
// chunks with an online softmax, so it scales to the N = 196 / 784 groups of the 64^2 / 224^2
// configurations (the thread-per-query kernel is VALU-bound there).
//
// Fragment layouts (lane = 16*fg + fr):
//   16x16x32 A operand: row fr, k = 8*fg..8*fg+7 (one 16-B load of a token's head slice)
//   16x16x32 B operand: col fr, k = 8*fg..8*fg+7 (same load shape)
//   16x16x16 A operand: row fr, k = 4*fg..4*fg+3 -- exactly what a lane holds of a 16x16 C tile
//            computed TRANSPOSED (C[4*fg+r][fr]), so softmax probabilities feed the next MFMA
//            from registers
//   16x16x16 B operand: k = 4*fg..4*fg+3, col fr -- ds_read_b64_tr_b16 of a [token][dim] LDS tile
//   C / D:   C[4*fg + r][fr], r = 0..3
// Forward: S^T = K Q^T per key chunk; P^T (registers) -> O += P V (V chunk through LDS).
// dQ:      S^T, dP^T = V dO^T; dS^T -> dQ += dS K (K chunk through LDS).
// dK, dV:  S = Q K^T, dP = dO V^T per query chunk; dV += P^T dO, dK += dS^T Q (dO, Q through LDS).
#include "ogv_common.h"

namespace ogv {

struct GridGeomM {
  int B, H, W, C, heads, g, Hg, Wg, N, hd;
  __device__ __forceinline__ long pixel(long grp, int tok) const {
    const int gj = (int)(grp % g);
    const long r = grp / g;
    const int gi = (int)(r % g);
    const long b = r / g;
    const int ty = tok / Wg, tx = tok - ty * Wg;
    return (b * H + (long)ty * g + gi) * W + (long)tx * g + gj;
  }
};

typedef __attribute__((ext_vector_type(4))) short gm_s16x4;
typedef __attribute__((address_space(3))) gm_s16x4 gm_lds_s16x4;

template <int HDP>
__host__ __device__ constexpr int gm_pitch() { return HDP == 32 ? 48 : 80; }  // 16 * odd elements

// 8 consecutive head dims of one token (zero past hd / for invalid tokens)
__device__ __forceinline__ bf16x8 gm_load8(const bf16* __restrict__ p, bool ok) {
  bf16x8 v = {};
  if (ok) v = *reinterpret_cast<const bf16x8*>(p);
  return v;
}

__device__ __forceinline__ gm_s16x4 pack4(const float (&x)[4]) {
  gm_s16x4 r;
  bf16* e = reinterpret_cast<bf16*>(&r);
#pragma unroll
  for (int i = 0; i < 4; ++i) e[i] = (bf16)x[i];
  return r;
}

// Stage 16 tokens x HDP dims (token rows of a chunk) into a wave-private [16][PITCH] LDS tile.
template <int HDP>
__device__ __forceinline__ void gm_stage(bf16* tile, const bf16* __restrict__ base, const GridGeomM& G, long grp,
                                         int tok0, long rowstride, int lane) {
  constexpr int PIECES = HDP / 8;  // 16-B pieces per token row
  constexpr int PITCH = gm_pitch<HDP>();
#pragma unroll
  for (int t = 0; t < (16 * PIECES + 63) / 64; ++t) {
    const int idx = lane + 64 * t;
    if (idx < 16 * PIECES) {
      const int row = idx / PIECES, pc = idx - row * PIECES;
      const int tok = tok0 + row;
      const bool ok = tok < G.N && pc * 8 < G.hd;
      const bf16x8 v = gm_load8(base + (ok ? G.pixel(grp, tok) : 0) * rowstride + pc * 8, ok);
      *reinterpret_cast<bf16x8*>(tile + row * PITCH + pc * 8) = v;
    }
  }
}

__device__ __forceinline__ void wave_sync_lds() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Store a 16-token x hd output tile held in C layout (rows 4*fg + r, dim j*16 + fr, times mul[r])
// through the wave's LDS tile, as 16-B row pieces at base + pixel(tok0 + row) * rowstride.
template <int HDP>
__device__ __forceinline__ void gm_store(bf16* tile, const f32x4 (&acc)[HDP / 16], const float (&mul)[4],
                                         bf16* __restrict__ base, const GridGeomM& G, long grp, int tok0,
                                         long rowstride, int lane) {
  constexpr int ND = HDP / 16, PIECES = HDP / 8, PITCH = gm_pitch<HDP>();
  const int fr = lane & 15, fg = lane >> 4;
#pragma unroll
  for (int j = 0; j < ND; ++j)
#pragma unroll
    for (int r = 0; r < 4; ++r) tile[(4 * fg + r) * PITCH + j * 16 + fr] = (bf16)(acc[j][r] * mul[r]);
  wave_sync_lds();
#pragma unroll
  for (int t = 0; t < (16 * PIECES + 63) / 64; ++t) {
    const int idx = lane + 64 * t;
    if (idx < 16 * PIECES) {
      const int row = idx / PIECES, pc = idx - row * PIECES;
      const int tok = tok0 + row;
      if (tok < G.N && pc * 8 < G.hd)
        *reinterpret_cast<bf16x8*>(base + G.pixel(grp, tok) * rowstride + pc * 8) =
            *reinterpret_cast<const bf16x8*>(tile + row * PITCH + pc * 8);
    }
  }
  wave_sync_lds();
}

// ---------------------------------------------------------------------------------------------- fwd
template <int HDP>
__global__ __launch_bounds__(256) void grid_mfma_fwd_kernel(const bf16* __restrict__ qkv, bf16* __restrict__ out,
                                                            float* __restrict__ lse, GridGeomM G, float scale,
                                                            long units) {
  constexpr int KK = HDP / 32, ND = HDP / 16, PITCH = gm_pitch<HDP>();
  __shared__ __attribute__((aligned(16))) bf16 lds[4][16 * PITCH];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const long unit = (long)blockIdx.x * 4 + wave;
  if (unit >= units) return;
  const int nqb = (G.N + 15) / 16;
  const int qb = (int)(unit % nqb);
  const long gh = unit / nqb;
  const int h = (int)(gh % G.heads);
  const long grp = gh / G.heads;
  const int fr = lane & 15, fg = lane >> 4;
  const long C3 = 3L * G.C;
  const bf16* qbase = qkv + h * G.hd;
  const bf16* kbase = qkv + G.C + h * G.hd;
  const bf16* vbase = qkv + 2 * G.C + h * G.hd;
  bf16* tile = lds[wave];

  // Q^T as the B operand: query q0 + fr, dims 8*fg (+32*kk)
  const int qtok = qb * 16 + fr;
  const bool qok = qtok < G.N;
  const long qpix = qok ? G.pixel(grp, qtok) : 0;
  bf16x8 qf[KK];
#pragma unroll
  for (int kk = 0; kk < KK; ++kk) {
    const int d = kk * 32 + fg * 8;
    qf[kk] = gm_load8(qbase + qpix * C3 + d, qok && d < G.hd);
  }
  f32x4 o[ND];
#pragma unroll
  for (int j = 0; j < ND; ++j) o[j] = f32x4{0.f, 0.f, 0.f, 0.f};
  float m = -INFINITY, l = 0.f;  // running max / sum of query fr (replicated over fg)

  for (int k0 = 0; k0 < G.N; k0 += 16) {
    // S^T[key 4fg+r][query fr] = K Q^T
    const int ktok = k0 + fr;
    const bool kok = ktok < G.N;
    const long kpix = kok ? G.pixel(grp, ktok) : 0;
    f32x4 s = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kk = 0; kk < KK; ++kk) {
      const int d = kk * 32 + fg * 8;
      const bf16x8 kf = gm_load8(kbase + kpix * C3 + d, kok && d < G.hd);
      s = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kf, qf[kk], s, 0, 0, 0);
    }
    // V chunk -> LDS (B operand of P V through transposed reads)
    gm_stage<HDP>(tile, vbase, G, grp, k0, C3, lane);
    // online softmax over the chunk's keys for query fr
    float x[4], mc = -INFINITY;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      x[r] = (k0 + 4 * fg + r < G.N) ? s[r] * scale : -INFINITY;
      mc = fmaxf(mc, x[r]);
    }
    mc = fmaxf(mc, __shfl_xor(mc, 16, 64));
    mc = fmaxf(mc, __shfl_xor(mc, 32, 64));
    const float mn = fmaxf(m, mc);
    const float corr = __expf(m - mn);  // 0 on the first chunk (m = -inf)
    float p[4], ps = 0.f;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      p[r] = __expf(x[r] - mn);
      ps += p[r];
    }
    ps += __shfl_xor(ps, 16, 64);
    ps += __shfl_xor(ps, 32, 64);
    l = l * corr + ps;
    m = mn;
    // O rows are queries 4fg+r: their correction factors live in lanes 4fg+r
    float cr[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) cr[r] = __shfl(corr, 4 * fg + r, 64);
#pragma unroll
    for (int j = 0; j < ND; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) o[j][r] *= cr[r];
    const gm_s16x4 pa = pack4(p);  // A operand: P[query fr][keys 4fg..4fg+3]
    wave_sync_lds();
#pragma unroll
    for (int j = 0; j < ND; ++j) {
      const gm_s16x4 vb =
          __builtin_amdgcn_ds_read_tr16_b64_v4i16((gm_lds_s16x4*)(tile + (4 * fg + (fr >> 2)) * PITCH + j * 16 + (fr & 3) * 4));
      o[j] = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(pa, vb, o[j], 0, 0, 0);
    }
    wave_sync_lds();
  }
  // normalise rows 4fg+r and store; LSE of query fr
  float inv[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) inv[r] = 1.f / __shfl(l, 4 * fg + r, 64);
  gm_store<HDP>(tile, o, inv, out + h * G.hd, G, grp, qb * 16, G.C, lane);
  if (fg == 0 && qok) lse[qpix * G.heads + h] = m + __logf(l);
}

// ----------------------------------------------------------------------------------------- dQ
template <int HDP>
__global__ __launch_bounds__(256) void grid_mfma_dq_kernel(const bf16* __restrict__ dout, const bf16* __restrict__ qkv,
                                                           const float* __restrict__ lse,
                                                           const float* __restrict__ delta, bf16* __restrict__ dqkv,
                                                           GridGeomM G, float scale, long units) {
  constexpr int KK = HDP / 32, ND = HDP / 16, PITCH = gm_pitch<HDP>();
  __shared__ __attribute__((aligned(16))) bf16 lds[4][16 * PITCH];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const long unit = (long)blockIdx.x * 4 + wave;
  if (unit >= units) return;
  const int nqb = (G.N + 15) / 16;
  const int qb = (int)(unit % nqb);
  const long gh = unit / nqb;
  const int h = (int)(gh % G.heads);
  const long grp = gh / G.heads;
  const int fr = lane & 15, fg = lane >> 4;
  const long C3 = 3L * G.C;
  const bf16* qbase = qkv + h * G.hd;
  const bf16* kbase = qkv + G.C + h * G.hd;
  const bf16* vbase = qkv + 2 * G.C + h * G.hd;
  bf16* tile = lds[wave];

  const int qtok = qb * 16 + fr;
  const bool qok = qtok < G.N;
  const long qpix = qok ? G.pixel(grp, qtok) : 0;
  bf16x8 qf[KK], gf[KK];  // Q^T and dO^T as B operands (query fr)
#pragma unroll
  for (int kk = 0; kk < KK; ++kk) {
    const int d = kk * 32 + fg * 8;
    qf[kk] = gm_load8(qbase + qpix * C3 + d, qok && d < G.hd);
    gf[kk] = gm_load8(dout + qpix * G.C + h * G.hd + d, qok && d < G.hd);
  }
  const float lq = qok ? lse[qpix * G.heads + h] : INFINITY;
  const float dl = qok ? delta[qpix * G.heads + h] : 0.f;
  f32x4 dq[ND];
#pragma unroll
  for (int j = 0; j < ND; ++j) dq[j] = f32x4{0.f, 0.f, 0.f, 0.f};

  for (int k0 = 0; k0 < G.N; k0 += 16) {
    const int ktok = k0 + fr;
    const bool kok = ktok < G.N;
    const long kpix = kok ? G.pixel(grp, ktok) : 0;
    f32x4 s = f32x4{0.f, 0.f, 0.f, 0.f}, dp = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kk = 0; kk < KK; ++kk) {
      const int d = kk * 32 + fg * 8;
      const bf16x8 kf = gm_load8(kbase + kpix * C3 + d, kok && d < G.hd);
      const bf16x8 vf = gm_load8(vbase + kpix * C3 + d, kok && d < G.hd);
      s = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kf, qf[kk], s, 0, 0, 0);    // S^T
      dp = __builtin_amdgcn_mfma_f32_16x16x32_bf16(vf, gf[kk], dp, 0, 0, 0);  // dP^T
    }
    gm_stage<HDP>(tile, kbase, G, grp, k0, C3, lane);  // K chunk: B operand of dS K
    float ds[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const bool ok = k0 + 4 * fg + r < G.N;
      const float pw = ok ? __expf(s[r] * scale - lq) : 0.f;
      ds[r] = pw * (dp[r] - dl);
    }
    const gm_s16x4 da = pack4(ds);  // A operand: dS[query fr][keys 4fg..]
    wave_sync_lds();
#pragma unroll
    for (int j = 0; j < ND; ++j) {
      const gm_s16x4 kb =
          __builtin_amdgcn_ds_read_tr16_b64_v4i16((gm_lds_s16x4*)(tile + (4 * fg + (fr >> 2)) * PITCH + j * 16 + (fr & 3) * 4));
      dq[j] = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(da, kb, dq[j], 0, 0, 0);
    }
    wave_sync_lds();
  }
  const float sc4[4] = {scale, scale, scale, scale};
  gm_store<HDP>(tile, dq, sc4, dqkv + h * G.hd, G, grp, qb * 16, C3, lane);
}

// --------------------------------------------------------------------------------------- dK, dV
template <int HDP>
__global__ __launch_bounds__(256) void grid_mfma_dkv_kernel(const bf16* __restrict__ dout, const bf16* __restrict__ qkv,
                                                            const float* __restrict__ lse,
                                                            const float* __restrict__ delta, bf16* __restrict__ dqkv,
                                                            GridGeomM G, float scale, long units) {
  constexpr int KK = HDP / 32, ND = HDP / 16, PITCH = gm_pitch<HDP>();
  __shared__ __attribute__((aligned(16))) bf16 lds[4][2][16 * PITCH];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const long unit = (long)blockIdx.x * 4 + wave;
  if (unit >= units) return;
  const int nkb = (G.N + 15) / 16;
  const int kb = (int)(unit % nkb);
  const long gh = unit / nkb;
  const int h = (int)(gh % G.heads);
  const long grp = gh / G.heads;
  const int fr = lane & 15, fg = lane >> 4;
  const long C3 = 3L * G.C;
  const bf16* qbase = qkv + h * G.hd;
  const bf16* kbase = qkv + G.C + h * G.hd;
  const bf16* vbase = qkv + 2 * G.C + h * G.hd;
  bf16* qt = lds[wave][0];
  bf16* gt = lds[wave][1];

  const int ktok = kb * 16 + fr;
  const bool kok = ktok < G.N;
  const long kpix = kok ? G.pixel(grp, ktok) : 0;
  bf16x8 kf[KK], vf[KK];  // K^T, V^T as B operands (key fr)
#pragma unroll
  for (int kk = 0; kk < KK; ++kk) {
    const int d = kk * 32 + fg * 8;
    kf[kk] = gm_load8(kbase + kpix * C3 + d, kok && d < G.hd);
    vf[kk] = gm_load8(vbase + kpix * C3 + d, kok && d < G.hd);
  }
  f32x4 dk[ND], dv[ND];
#pragma unroll
  for (int j = 0; j < ND; ++j) {
    dk[j] = f32x4{0.f, 0.f, 0.f, 0.f};
    dv[j] = f32x4{0.f, 0.f, 0.f, 0.f};
  }
  for (int q0 = 0; q0 < G.N; q0 += 16) {
    // S[query 4fg+r][key fr] = Q K^T ; dP = dO V^T  (query rows of the A operand = q0 + fr)
    const int qtok = q0 + fr;
    const bool qok = qtok < G.N;
    const long qpix = qok ? G.pixel(grp, qtok) : 0;
    f32x4 s = f32x4{0.f, 0.f, 0.f, 0.f}, dp = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kk = 0; kk < KK; ++kk) {
      const int d = kk * 32 + fg * 8;
      const bf16x8 qa = gm_load8(qbase + qpix * C3 + d, qok && d < G.hd);
      const bf16x8 ga = gm_load8(dout + qpix * G.C + h * G.hd + d, qok && d < G.hd);
      s = __builtin_amdgcn_mfma_f32_16x16x32_bf16(qa, kf[kk], s, 0, 0, 0);
      dp = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ga, vf[kk], dp, 0, 0, 0);
    }
    gm_stage<HDP>(qt, qbase, G, grp, q0, C3, lane);              // Q chunk  (B operand of dS^T Q)
    gm_stage<HDP>(gt, dout + h * G.hd, G, grp, q0, G.C, lane);   // dO chunk (B operand of P^T dO)
    // lse / delta of the C-tile rows (queries 4fg+r)
    float pw[4], ds[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int tok = q0 + 4 * fg + r;
      float lq = INFINITY, dl = 0.f;
      if (tok < G.N) {
        const long pq = G.pixel(grp, tok);
        lq = lse[pq * G.heads + h];
        dl = delta[pq * G.heads + h];
      }
      pw[r] = kok ? __expf(s[r] * scale - lq) : 0.f;
      ds[r] = pw[r] * (dp[r] - dl);
    }
    // C layout holds [query 4fg+r][key fr] = the A operand [key fr][queries 4fg..] of the
    // key-row products below
    const gm_s16x4 pa = pack4(pw), da = pack4(ds);
    wave_sync_lds();
#pragma unroll
    for (int j = 0; j < ND; ++j) {
      const int off = (4 * fg + (fr >> 2)) * PITCH + j * 16 + (fr & 3) * 4;
      const gm_s16x4 gb = __builtin_amdgcn_ds_read_tr16_b64_v4i16((gm_lds_s16x4*)(gt + off));
      const gm_s16x4 qb2 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((gm_lds_s16x4*)(qt + off));
      dv[j] = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(pa, gb, dv[j], 0, 0, 0);
      dk[j] = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(da, qb2, dk[j], 0, 0, 0);
    }
    wave_sync_lds();
  }
  // rows of dK / dV are keys kb*16 + 4fg + r
  const float sc4[4] = {scale, scale, scale, scale}, one4[4] = {1.f, 1.f, 1.f, 1.f};
  gm_store<HDP>(qt, dk, sc4, dqkv + G.C + h * G.hd, G, grp, kb * 16, C3, lane);
  gm_store<HDP>(gt, dv, one4, dqkv + 2 * G.C + h * G.hd, G, grp, kb * 16, C3, lane);
}

// ------------------------------------------------------------------------------------------------
// LDS-resident variants: a block owns PP (group, head) pairs and first stages the pair's whole
// K/V (fwd, dQ) or Q/dO (+ lse, delta: dK/dV) into LDS once; its 4 waves then walk the pair's
// 16-row blocks against it.  The per-row-block kernels above re-read those operands from global
// memory for every row block and every 16-token chunk (a global-latency chain per chunk); here the
// chunk loop runs entirely out of LDS.  Used when the tiles fit in 64 KB (N <= ~300 for hd <= 32).
struct GmLds {
  int PP, nrb, Np;      // pairs per block, 16-row blocks per pair, padded tokens
  long pairs, blocks;
  size_t tile_elems;    // one [Np][PITCH] tile
};
template <int HDP>
static GmLds gm_lds_plan(const GridGeomM& G) {
  GmLds p;
  p.nrb = (G.N + 15) / 16;
  p.Np = p.nrb * 16;
  p.PP = p.nrb >= 4 ? 1 : 4 / p.nrb;
  p.pairs = (long)G.B * G.g * G.g * G.heads;
  p.blocks = (p.pairs + p.PP - 1) / p.PP;
  p.tile_elems = (size_t)p.Np * gm_pitch<HDP>();
  return p;
}
template <int HDP>
static size_t gm_lds_bytes(const GmLds& p, bool stats) {
  return (size_t)p.PP * (2 * p.tile_elems * sizeof(bf16) + (stats ? 2 * p.Np * sizeof(float) : 0)) +
         4 * 16 * gm_pitch<HDP>() * sizeof(bf16);
}

// all 256 threads: tokens [0, Np) x head dims of one pair from base (row stride ld) into tile
template <int HDP>
__device__ __forceinline__ void gm_stage_pair(bf16* tile, const bf16* __restrict__ base, long ld, const GridGeomM& G,
                                              long grp, int Np) {
  constexpr int PIECES = HDP / 8, PITCH = gm_pitch<HDP>();
  for (int idx = threadIdx.x; idx < Np * PIECES; idx += 256) {
    const int row = idx / PIECES, pc = idx - row * PIECES;
    const bool ok = row < G.N && pc * 8 < G.hd;
    const bf16x8 v = gm_load8(base + (ok ? G.pixel(grp, row) : 0) * ld + pc * 8, ok);
    *reinterpret_cast<bf16x8*>(tile + row * PITCH + pc * 8) = v;
  }
}

template <int HDP>
__global__ __launch_bounds__(256) void grid_lds_fwd_kernel(const bf16* __restrict__ qkv, bf16* __restrict__ out,
                                                           float* __restrict__ lse, GridGeomM G, float scale, GmLds L) {
  constexpr int KK = HDP / 32, ND = HDP / 16, PITCH = gm_pitch<HDP>();
  extern __shared__ __attribute__((aligned(16))) bf16 gsm[];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int fr = lane & 15, fg = lane >> 4;
  const long C3 = 3L * G.C;
  const long pair0 = (long)blockIdx.x * L.PP;
  for (int p = 0; p < L.PP; ++p) {
    const long pr = pair0 + p;
    if (pr >= L.pairs) break;
    const int h = (int)(pr % G.heads);
    const long grp = pr / G.heads;
    bf16* Ks = gsm + (size_t)p * 2 * L.tile_elems;
    gm_stage_pair<HDP>(Ks, qkv + G.C + h * G.hd, C3, G, grp, L.Np);
    gm_stage_pair<HDP>(Ks + L.tile_elems, qkv + 2 * G.C + h * G.hd, C3, G, grp, L.Np);
  }
  __syncthreads();
  bf16* tile = gsm + (size_t)L.PP * 2 * L.tile_elems + wave * 16 * PITCH;
  for (int it = wave; it < L.PP * L.nrb; it += 4) {
    const int p = it / L.nrb, qb = it - p * L.nrb;
    const long pr = pair0 + p;
    if (pr >= L.pairs) break;
    const int h = (int)(pr % G.heads);
    const long grp = pr / G.heads;
    const bf16* Ks = gsm + (size_t)p * 2 * L.tile_elems;
    const bf16* Vs = Ks + L.tile_elems;
    const int qtok = qb * 16 + fr;
    const bool qok = qtok < G.N;
    const long qpix = qok ? G.pixel(grp, qtok) : 0;
    bf16x8 qf[KK];
#pragma unroll
    for (int kk = 0; kk < KK; ++kk) {
      const int d = kk * 32 + fg * 8;
      qf[kk] = gm_load8(qkv + h * G.hd + qpix * C3 + d, qok && d < G.hd);
    }
    f32x4 o[ND];
#pragma unroll
    for (int j = 0; j < ND; ++j) o[j] = f32x4{0.f, 0.f, 0.f, 0.f};
    float m = -INFINITY, l = 0.f;
    for (int k0 = 0; k0 < G.N; k0 += 16) {
      f32x4 s = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kk = 0; kk < KK; ++kk) {
        const bf16x8 kf = *reinterpret_cast<const bf16x8*>(Ks + (k0 + fr) * PITCH + kk * 32 + fg * 8);
        s = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kf, qf[kk], s, 0, 0, 0);
      }
      float x[4], mc = -INFINITY;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        x[r] = (k0 + 4 * fg + r < G.N) ? s[r] * scale : -INFINITY;
        mc = fmaxf(mc, x[r]);
      }
      mc = fmaxf(mc, __shfl_xor(mc, 16, 64));
      mc = fmaxf(mc, __shfl_xor(mc, 32, 64));
      const float mn = fmaxf(m, mc);
      const float corr = __expf(m - mn);
      float pw[4], ps = 0.f;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        pw[r] = __expf(x[r] - mn);
        ps += pw[r];
      }
      ps += __shfl_xor(ps, 16, 64);
      ps += __shfl_xor(ps, 32, 64);
      l = l * corr + ps;
      m = mn;
      float cr[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) cr[r] = __shfl(corr, 4 * fg + r, 64);
#pragma unroll
      for (int j = 0; j < ND; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) o[j][r] *= cr[r];
      const gm_s16x4 pa = pack4(pw);
#pragma unroll
      for (int j = 0; j < ND; ++j) {
        const gm_s16x4 vb = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
            (gm_lds_s16x4*)(Vs + (k0 + 4 * fg + (fr >> 2)) * PITCH + j * 16 + (fr & 3) * 4));
        o[j] = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(pa, vb, o[j], 0, 0, 0);
      }
    }
    float inv[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) inv[r] = 1.f / __shfl(l, 4 * fg + r, 64);
    gm_store<HDP>(tile, o, inv, out + h * G.hd, G, grp, qb * 16, G.C, lane);
    if (fg == 0 && qok) lse[qpix * G.heads + h] = m + __logf(l);
  }
}

template <int HDP>
__global__ __launch_bounds__(256) void grid_lds_dq_kernel(const bf16* __restrict__ dout, const bf16* __restrict__ qkv,
                                                          const float* __restrict__ lse, const float* __restrict__ delta,
                                                          bf16* __restrict__ dqkv, GridGeomM G, float scale, GmLds L) {
  constexpr int KK = HDP / 32, ND = HDP / 16, PITCH = gm_pitch<HDP>();
  extern __shared__ __attribute__((aligned(16))) bf16 gsm[];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int fr = lane & 15, fg = lane >> 4;
  const long C3 = 3L * G.C;
  const long pair0 = (long)blockIdx.x * L.PP;
  for (int p = 0; p < L.PP; ++p) {
    const long pr = pair0 + p;
    if (pr >= L.pairs) break;
    const int h = (int)(pr % G.heads);
    const long grp = pr / G.heads;
    bf16* Ks = gsm + (size_t)p * 2 * L.tile_elems;
    gm_stage_pair<HDP>(Ks, qkv + G.C + h * G.hd, C3, G, grp, L.Np);
    gm_stage_pair<HDP>(Ks + L.tile_elems, qkv + 2 * G.C + h * G.hd, C3, G, grp, L.Np);
  }
  __syncthreads();
  bf16* tile = gsm + (size_t)L.PP * 2 * L.tile_elems + wave * 16 * PITCH;
  for (int it = wave; it < L.PP * L.nrb; it += 4) {
    const int p = it / L.nrb, qb = it - p * L.nrb;
    const long pr = pair0 + p;
    if (pr >= L.pairs) break;
    const int h = (int)(pr % G.heads);
    const long grp = pr / G.heads;
    const bf16* Ks = gsm + (size_t)p * 2 * L.tile_elems;
    const bf16* Vs = Ks + L.tile_elems;
    const int qtok = qb * 16 + fr;
    const bool qok = qtok < G.N;
    const long qpix = qok ? G.pixel(grp, qtok) : 0;
    bf16x8 qf[KK], gf[KK];
#pragma unroll
    for (int kk = 0; kk < KK; ++kk) {
      const int d = kk * 32 + fg * 8;
      qf[kk] = gm_load8(qkv + h * G.hd + qpix * C3 + d, qok && d < G.hd);
      gf[kk] = gm_load8(dout + qpix * G.C + h * G.hd + d, qok && d < G.hd);
    }
    const float lq = qok ? lse[qpix * G.heads + h] : INFINITY;
    const float dl = qok ? delta[qpix * G.heads + h] : 0.f;
    f32x4 dq[ND];
#pragma unroll
    for (int j = 0; j < ND; ++j) dq[j] = f32x4{0.f, 0.f, 0.f, 0.f};
    for (int k0 = 0; k0 < G.N; k0 += 16) {
      f32x4 s = f32x4{0.f, 0.f, 0.f, 0.f}, dp = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kk = 0; kk < KK; ++kk) {
        const int off = (k0 + fr) * PITCH + kk * 32 + fg * 8;
        const bf16x8 kf = *reinterpret_cast<const bf16x8*>(Ks + off);
        const bf16x8 vf = *reinterpret_cast<const bf16x8*>(Vs + off);
        s = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kf, qf[kk], s, 0, 0, 0);
        dp = __builtin_amdgcn_mfma_f32_16x16x32_bf16(vf, gf[kk], dp, 0, 0, 0);
      }
      float ds[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const bool ok = k0 + 4 * fg + r < G.N;
        const float pw = ok ? __expf(s[r] * scale - lq) : 0.f;
        ds[r] = pw * (dp[r] - dl);
      }
      const gm_s16x4 da = pack4(ds);
#pragma unroll
      for (int j = 0; j < ND; ++j) {
        const gm_s16x4 kb = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
            (gm_lds_s16x4*)(Ks + (k0 + 4 * fg + (fr >> 2)) * PITCH + j * 16 + (fr & 3) * 4));
        dq[j] = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(da, kb, dq[j], 0, 0, 0);
      }
    }
    const float sc4[4] = {scale, scale, scale, scale};
    gm_store<HDP>(tile, dq, sc4, dqkv + h * G.hd, G, grp, qb * 16, C3, lane);
  }
}

template <int HDP>
__global__ __launch_bounds__(256) void grid_lds_dkv_kernel(const bf16* __restrict__ dout, const bf16* __restrict__ qkv,
                                                           const float* __restrict__ lse,
                                                           const float* __restrict__ delta, bf16* __restrict__ dqkv,
                                                           GridGeomM G, float scale, GmLds L) {
  constexpr int KK = HDP / 32, ND = HDP / 16, PITCH = gm_pitch<HDP>();
  extern __shared__ __attribute__((aligned(16))) bf16 gsm[];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int fr = lane & 15, fg = lane >> 4;
  const long C3 = 3L * G.C;
  const long pair0 = (long)blockIdx.x * L.PP;
  float* stats = reinterpret_cast<float*>(gsm + (size_t)L.PP * 2 * L.tile_elems);  // [PP][2][Np]
  for (int p = 0; p < L.PP; ++p) {
    const long pr = pair0 + p;
    if (pr >= L.pairs) break;
    const int h = (int)(pr % G.heads);
    const long grp = pr / G.heads;
    bf16* Qs = gsm + (size_t)p * 2 * L.tile_elems;
    gm_stage_pair<HDP>(Qs, qkv + h * G.hd, C3, G, grp, L.Np);
    gm_stage_pair<HDP>(Qs + L.tile_elems, dout + h * G.hd, G.C, G, grp, L.Np);
    for (int t = threadIdx.x; t < L.Np; t += 256) {
      const bool ok = t < G.N;
      const long pq = ok ? G.pixel(grp, t) : 0;
      stats[(p * 2 + 0) * L.Np + t] = ok ? lse[pq * G.heads + h] : INFINITY;
      stats[(p * 2 + 1) * L.Np + t] = ok ? delta[pq * G.heads + h] : 0.f;
    }
  }
  __syncthreads();
  bf16* tile = reinterpret_cast<bf16*>(stats + (size_t)L.PP * 2 * L.Np) + wave * 16 * PITCH;
  for (int it = wave; it < L.PP * L.nrb; it += 4) {
    const int p = it / L.nrb, kb = it - p * L.nrb;
    const long pr = pair0 + p;
    if (pr >= L.pairs) break;
    const int h = (int)(pr % G.heads);
    const long grp = pr / G.heads;
    const bf16* Qs = gsm + (size_t)p * 2 * L.tile_elems;
    const bf16* Gs = Qs + L.tile_elems;
    const float* lq_s = stats + (p * 2 + 0) * L.Np;
    const float* dl_s = stats + (p * 2 + 1) * L.Np;
    const int ktok = kb * 16 + fr;
    const bool kok = ktok < G.N;
    const long kpix = kok ? G.pixel(grp, ktok) : 0;
    bf16x8 kf[KK], vf[KK];
#pragma unroll
    for (int kk = 0; kk < KK; ++kk) {
      const int d = kk * 32 + fg * 8;
      kf[kk] = gm_load8(qkv + G.C + h * G.hd + kpix * C3 + d, kok && d < G.hd);
      vf[kk] = gm_load8(qkv + 2 * G.C + h * G.hd + kpix * C3 + d, kok && d < G.hd);
    }
    f32x4 dk[ND], dv[ND];
#pragma unroll
    for (int j = 0; j < ND; ++j) {
      dk[j] = f32x4{0.f, 0.f, 0.f, 0.f};
      dv[j] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
    for (int q0 = 0; q0 < G.N; q0 += 16) {
      f32x4 s = f32x4{0.f, 0.f, 0.f, 0.f}, dp = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kk = 0; kk < KK; ++kk) {
        const int off = (q0 + fr) * PITCH + kk * 32 + fg * 8;
        const bf16x8 qa = *reinterpret_cast<const bf16x8*>(Qs + off);
        const bf16x8 ga = *reinterpret_cast<const bf16x8*>(Gs + off);
        s = __builtin_amdgcn_mfma_f32_16x16x32_bf16(qa, kf[kk], s, 0, 0, 0);
        dp = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ga, vf[kk], dp, 0, 0, 0);
      }
      float pw[4], ds[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int tok = q0 + 4 * fg + r;  // < Np: padded rows hold lse = inf -> pw = 0
        pw[r] = kok ? __expf(s[r] * scale - lq_s[tok]) : 0.f;
        ds[r] = pw[r] * (dp[r] - dl_s[tok]);
      }
      const gm_s16x4 pa = pack4(pw), da = pack4(ds);
#pragma unroll
      for (int j = 0; j < ND; ++j) {
        const int off = (q0 + 4 * fg + (fr >> 2)) * PITCH + j * 16 + (fr & 3) * 4;
        const gm_s16x4 gb = __builtin_amdgcn_ds_read_tr16_b64_v4i16((gm_lds_s16x4*)(Gs + off));
        const gm_s16x4 qb2 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((gm_lds_s16x4*)(Qs + off));
        dv[j] = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(pa, gb, dv[j], 0, 0, 0);
        dk[j] = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(da, qb2, dk[j], 0, 0, 0);
      }
    }
    const float sc4[4] = {scale, scale, scale, scale}, one4[4] = {1.f, 1.f, 1.f, 1.f};
    gm_store<HDP>(tile, dk, sc4, dqkv + G.C + h * G.hd, G, grp, kb * 16, C3, lane);
    gm_store<HDP>(tile, dv, one4, dqkv + 2 * G.C + h * G.hd, G, grp, kb * 16, C3, lane);
  }
}

// ------------------------------------------------------------------------------------------------
// Large groups (N = 784 at 224^2 stage 0): one (group, head) pair per block of 16 waves, its whole
// K and V (2 x N x PITCH bf16, up to 150 KB for head_dim 32) resident in LDS, staged once with
// batched 16-B loads.  Each wave walks query blocks of 16 against it 64 keys at a time: four
// S^T = K Q^T MFMAs, ONE running-max / rescale step for the 64 keys (the per-16-key kernels pay the
// cross-lane max, the exp of the correction and the O rescale four times as often), then 4 x ND
// P V MFMAs.  The output leaves straight from the accumulators (2-byte stores; the LDS is full).
constexpr int GB_NW = 16;
template <int HDP>
__global__ __launch_bounds__(GB_NW * 64) void grid_big_fwd_kernel(const bf16* __restrict__ qkv, bf16* __restrict__ out,
                                                                 float* __restrict__ lse, GridGeomM G, float scale,
                                                                 int Np) {
  constexpr int KK = HDP / 32, ND = HDP / 16, PITCH = gm_pitch<HDP>(), PIECES = HDP / 8;
  extern __shared__ __attribute__((aligned(16))) bf16 gsm[];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int fr = lane & 15, fg = lane >> 4;
  const long C3 = 3L * G.C;
  const long pr = blockIdx.x;
  const int h = (int)(pr % G.heads);
  const long grp = pr / G.heads;
  bf16* Ks = gsm;
  bf16* Vs = gsm + (size_t)Np * PITCH;
  // stage K and V: 8 independent 16-B loads per thread in flight before any LDS store
  {
    const int total = 2 * Np * PIECES;
    for (int base = threadIdx.x; base < total; base += 8 * GB_NW * 64) {
      bf16x8 v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int idx = base + u * GB_NW * 64;
        const int t = idx / (Np * PIECES), r = idx - t * Np * PIECES;
        const int row = r / PIECES, pc = r - row * PIECES;
        const bool ok = idx < total && row < G.N && pc * 8 < G.hd;
        v[u] = gm_load8(qkv + (t + 1) * G.C + h * G.hd + (ok ? G.pixel(grp, row) : 0) * C3 + pc * 8, ok);
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int idx = base + u * GB_NW * 64;
        if (idx < total) {
          const int t = idx / (Np * PIECES), r = idx - t * Np * PIECES;
          const int row = r / PIECES, pc = r - row * PIECES;
          *reinterpret_cast<bf16x8*>(gsm + (size_t)t * Np * PITCH + row * PITCH + pc * 8) = v[u];
        }
      }
    }
  }
  __syncthreads();
  const int nrb = Np / 16;
  for (int qb = wave; qb < nrb; qb += GB_NW) {
    const int qtok = qb * 16 + fr;
    const bool qok = qtok < G.N;
    const long qpix = qok ? G.pixel(grp, qtok) : 0;
    bf16x8 qf[KK];
#pragma unroll
    for (int kk = 0; kk < KK; ++kk) {
      const int d = kk * 32 + fg * 8;
      qf[kk] = gm_load8(qkv + h * G.hd + qpix * C3 + d, qok && d < G.hd);
    }
    f32x4 o[ND];
#pragma unroll
    for (int j = 0; j < ND; ++j) o[j] = f32x4{0.f, 0.f, 0.f, 0.f};
    float m = -INFINITY, l = 0.f;
    for (int k0 = 0; k0 < Np; k0 += 64) {
      const int nc = (Np - k0) >= 64 ? 4 : (Np - k0) / 16;   // 16-key chunks in this step
      f32x4 sc[4];
      float mc = -INFINITY;
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        sc[c] = f32x4{0.f, 0.f, 0.f, 0.f};
        if (c < nc) {
#pragma unroll
          for (int kk = 0; kk < KK; ++kk) {
            const bf16x8 kf = *reinterpret_cast<const bf16x8*>(Ks + (k0 + 16 * c + fr) * PITCH + kk * 32 + fg * 8);
            sc[c] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kf, qf[kk], sc[c], 0, 0, 0);
          }
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int key = k0 + 16 * c + 4 * fg + r;
          sc[c][r] = (c < nc && key < G.N) ? sc[c][r] * scale : -INFINITY;
          mc = fmaxf(mc, sc[c][r]);
        }
      }
      mc = fmaxf(mc, __shfl_xor(mc, 16, 64));
      mc = fmaxf(mc, __shfl_xor(mc, 32, 64));
      const float mn = fmaxf(m, mc);
      const float corr = __expf(m - mn);   // 0 on the first step (m = -inf)
      float ps = 0.f;
#pragma unroll
      for (int c = 0; c < 4; ++c)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          sc[c][r] = __expf(sc[c][r] - mn);
          ps += sc[c][r];
        }
      ps += __shfl_xor(ps, 16, 64);
      ps += __shfl_xor(ps, 32, 64);
      l = l * corr + ps;
      m = mn;
      float cr[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) cr[r] = __shfl(corr, 4 * fg + r, 64);
#pragma unroll
      for (int j = 0; j < ND; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) o[j][r] *= cr[r];
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        if (c >= nc) break;
        float pw[4] = {sc[c][0], sc[c][1], sc[c][2], sc[c][3]};
        const gm_s16x4 pa = pack4(pw);
#pragma unroll
        for (int j = 0; j < ND; ++j) {
          const gm_s16x4 vb = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
              (gm_lds_s16x4*)(Vs + (k0 + 16 * c + 4 * fg + (fr >> 2)) * PITCH + j * 16 + (fr & 3) * 4));
          o[j] = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(pa, vb, o[j], 0, 0, 0);
        }
      }
    }
    // rows 4fg + r of the C layout are queries qb*16 + 4fg + r
    float inv[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) inv[r] = 1.f / __shfl(l, 4 * fg + r, 64);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int tok = qb * 16 + 4 * fg + r;
      if (tok >= G.N) continue;
      bf16* dst = out + G.pixel(grp, tok) * G.C + h * G.hd;
#pragma unroll
      for (int j = 0; j < ND; ++j)
        if (j * 16 + fr < G.hd) dst[j * 16 + fr] = (bf16)(o[j][r] * inv[r]);
    }
    if (fg == 0 && qok) lse[qpix * G.heads + h] = m + __logf(l);
  }
}

// Stage tokens [0, Np) x head dims of tensors (base_t, row stride ld_t) t = 0, 1 of one pair into
// [2][Np][PITCH] LDS (zeros past N / hd), 8 independent 16-B loads per thread in flight.
template <int HDP>
__device__ __forceinline__ void gb_stage2(bf16* lds, const bf16* __restrict__ b0, long ld0, const bf16* __restrict__ b1,
                                          long ld1, const GridGeomM& G, long grp, int Np) {
  constexpr int PITCH = gm_pitch<HDP>(), PIECES = HDP / 8;
  const int total = 2 * Np * PIECES;
  for (int base = threadIdx.x; base < total; base += 8 * GB_NW * 64) {
    bf16x8 v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int idx = base + u * GB_NW * 64;
      const int t = idx / (Np * PIECES), r = idx - t * Np * PIECES;
      const int row = r / PIECES, pc = r - row * PIECES;
      const bool ok = idx < total && row < G.N && pc * 8 < G.hd;
      const long pix = ok ? G.pixel(grp, row) : 0;
      v[u] = gm_load8((t ? b1 + pix * ld1 : b0 + pix * ld0) + pc * 8, ok);
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int idx = base + u * GB_NW * 64;
      if (idx < total) {
        const int t = idx / (Np * PIECES), r = idx - t * Np * PIECES;
        const int row = r / PIECES, pc = r - row * PIECES;
        *reinterpret_cast<bf16x8*>(lds + (size_t)t * Np * PITCH + row * PITCH + pc * 8) = v[u];
      }
    }
  }
}

// rows 4fg + r of a C-layout accumulator (times mul[r]) -> base + pixel(tok0 + 4fg + r) * ld, dims j*16 + fr
template <int HDP>
__device__ __forceinline__ void gb_store(const f32x4 (&acc)[HDP / 16], const float (&mul)[4], bf16* __restrict__ base,
                                         long ld, const GridGeomM& G, long grp, int tok0, int lane) {
  const int fr = lane & 15, fg = lane >> 4;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int tok = tok0 + 4 * fg + r;
    if (tok >= G.N) continue;
    bf16* dst = base + G.pixel(grp, tok) * ld;
#pragma unroll
    for (int j = 0; j < HDP / 16; ++j)
      if (j * 16 + fr < G.hd) dst[j * 16 + fr] = (bf16)(acc[j][r] * mul[r]);
  }
}

// dQ of large groups: K and V of the pair resident in LDS; a wave per 16-query block walks all keys.
template <int HDP>
__global__ __launch_bounds__(GB_NW * 64) void grid_big_dq_kernel(const bf16* __restrict__ dout,
                                                                const bf16* __restrict__ qkv,
                                                                const float* __restrict__ lse,
                                                                const float* __restrict__ delta,
                                                                bf16* __restrict__ dqkv, GridGeomM G, float scale,
                                                                int Np) {
  constexpr int KK = HDP / 32, ND = HDP / 16, PITCH = gm_pitch<HDP>();
  extern __shared__ __attribute__((aligned(16))) bf16 gsm[];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int fr = lane & 15, fg = lane >> 4;
  const long C3 = 3L * G.C;
  const long pr = blockIdx.x;
  const int h = (int)(pr % G.heads);
  const long grp = pr / G.heads;
  const bf16* Ks = gsm;
  const bf16* Vs = gsm + (size_t)Np * PITCH;
  gb_stage2<HDP>(gsm, qkv + G.C + h * G.hd, C3, qkv + 2 * G.C + h * G.hd, C3, G, grp, Np);
  __syncthreads();
  for (int qb = wave; qb < Np / 16; qb += GB_NW) {
    const int qtok = qb * 16 + fr;
    const bool qok = qtok < G.N;
    const long qpix = qok ? G.pixel(grp, qtok) : 0;
    bf16x8 qf[KK], gf[KK];  // Q^T and dO^T as B operands (query fr)
#pragma unroll
    for (int kk = 0; kk < KK; ++kk) {
      const int d = kk * 32 + fg * 8;
      qf[kk] = gm_load8(qkv + h * G.hd + qpix * C3 + d, qok && d < G.hd);
      gf[kk] = gm_load8(dout + qpix * G.C + h * G.hd + d, qok && d < G.hd);
    }
    const float lq = qok ? lse[qpix * G.heads + h] : INFINITY;
    const float dl = qok ? delta[qpix * G.heads + h] : 0.f;
    f32x4 dq[ND];
#pragma unroll
    for (int j = 0; j < ND; ++j) dq[j] = f32x4{0.f, 0.f, 0.f, 0.f};
    for (int k0 = 0; k0 < Np; k0 += 16) {
      f32x4 sv = f32x4{0.f, 0.f, 0.f, 0.f}, dp = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kk = 0; kk < KK; ++kk) {
        const bf16x8 kf = *reinterpret_cast<const bf16x8*>(Ks + (k0 + fr) * PITCH + kk * 32 + fg * 8);
        const bf16x8 vf = *reinterpret_cast<const bf16x8*>(Vs + (k0 + fr) * PITCH + kk * 32 + fg * 8);
        sv = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kf, qf[kk], sv, 0, 0, 0);    // S^T
        dp = __builtin_amdgcn_mfma_f32_16x16x32_bf16(vf, gf[kk], dp, 0, 0, 0);    // dP^T
      }
      float ds[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const bool ok = k0 + 4 * fg + r < G.N;
        const float pw = ok ? __expf(sv[r] * scale - lq) : 0.f;
        ds[r] = pw * (dp[r] - dl);
      }
      const gm_s16x4 da = pack4(ds);  // A operand: dS[query fr][keys 4fg..]
#pragma unroll
      for (int j = 0; j < ND; ++j) {
        const gm_s16x4 kb = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
            (gm_lds_s16x4*)(Ks + (k0 + 4 * fg + (fr >> 2)) * PITCH + j * 16 + (fr & 3) * 4));
        dq[j] = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(da, kb, dq[j], 0, 0, 0);
      }
    }
    const float sc4[4] = {scale, scale, scale, scale};
    gb_store<HDP>(dq, sc4, dqkv + h * G.hd, C3, G, grp, qb * 16, lane);
  }
}

// dK, dV of large groups: Q, dO (+ lse, delta) of the pair resident in LDS; a wave per 16-key block.
template <int HDP>
__global__ __launch_bounds__(GB_NW * 64) void grid_big_dkv_kernel(const bf16* __restrict__ dout,
                                                                 const bf16* __restrict__ qkv,
                                                                 const float* __restrict__ lse,
                                                                 const float* __restrict__ delta,
                                                                 bf16* __restrict__ dqkv, GridGeomM G, float scale,
                                                                 int Np) {
  constexpr int KK = HDP / 32, ND = HDP / 16, PITCH = gm_pitch<HDP>();
  extern __shared__ __attribute__((aligned(16))) bf16 gsm[];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int fr = lane & 15, fg = lane >> 4;
  const long C3 = 3L * G.C;
  const long pr = blockIdx.x;
  const int h = (int)(pr % G.heads);
  const long grp = pr / G.heads;
  const bf16* Qs = gsm;
  const bf16* Gs = gsm + (size_t)Np * PITCH;
  float* lq_s = reinterpret_cast<float*>(gsm + 2 * (size_t)Np * PITCH);
  float* dl_s = lq_s + Np;
  gb_stage2<HDP>(gsm, qkv + h * G.hd, C3, dout + h * G.hd, G.C, G, grp, Np);
  for (int t = threadIdx.x; t < Np; t += GB_NW * 64) {   // padded rows: lse = inf -> P = 0
    const bool ok = t < G.N;
    const long pq = ok ? G.pixel(grp, t) : 0;
    lq_s[t] = ok ? lse[pq * G.heads + h] : INFINITY;
    dl_s[t] = ok ? delta[pq * G.heads + h] : 0.f;
  }
  __syncthreads();
  for (int kb = wave; kb < Np / 16; kb += GB_NW) {
    const int ktok = kb * 16 + fr;
    const bool kok = ktok < G.N;
    const long kpix = kok ? G.pixel(grp, ktok) : 0;
    bf16x8 kf[KK], vf[KK];  // K^T, V^T as B operands (key fr)
#pragma unroll
    for (int kk = 0; kk < KK; ++kk) {
      const int d = kk * 32 + fg * 8;
      kf[kk] = gm_load8(qkv + G.C + h * G.hd + kpix * C3 + d, kok && d < G.hd);
      vf[kk] = gm_load8(qkv + 2 * G.C + h * G.hd + kpix * C3 + d, kok && d < G.hd);
    }
    f32x4 dk[ND], dv[ND];
#pragma unroll
    for (int j = 0; j < ND; ++j) {
      dk[j] = f32x4{0.f, 0.f, 0.f, 0.f};
      dv[j] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
    for (int q0 = 0; q0 < Np; q0 += 16) {
      // S[query 4fg+r][key fr] = Q K^T ; dP = dO V^T
      f32x4 sv = f32x4{0.f, 0.f, 0.f, 0.f}, dp = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kk = 0; kk < KK; ++kk) {
        const bf16x8 qa = *reinterpret_cast<const bf16x8*>(Qs + (q0 + fr) * PITCH + kk * 32 + fg * 8);
        const bf16x8 ga = *reinterpret_cast<const bf16x8*>(Gs + (q0 + fr) * PITCH + kk * 32 + fg * 8);
        sv = __builtin_amdgcn_mfma_f32_16x16x32_bf16(qa, kf[kk], sv, 0, 0, 0);
        dp = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ga, vf[kk], dp, 0, 0, 0);
      }
      float pw[4], ds[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int tok = q0 + 4 * fg + r;   // < Np: padded rows hold lse = inf -> pw = 0
        pw[r] = kok ? __expf(sv[r] * scale - lq_s[tok]) : 0.f;
        ds[r] = pw[r] * (dp[r] - dl_s[tok]);
      }
      const gm_s16x4 pa = pack4(pw), da = pack4(ds);
#pragma unroll
      for (int j = 0; j < ND; ++j) {
        const int off = (q0 + 4 * fg + (fr >> 2)) * PITCH + j * 16 + (fr & 3) * 4;
        const gm_s16x4 gb = __builtin_amdgcn_ds_read_tr16_b64_v4i16((gm_lds_s16x4*)(Gs + off));
        const gm_s16x4 qb2 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((gm_lds_s16x4*)(Qs + off));
        dv[j] = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(pa, gb, dv[j], 0, 0, 0);
        dk[j] = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(da, qb2, dk[j], 0, 0, 0);
      }
    }
    const float sc4[4] = {scale, scale, scale, scale}, one4[4] = {1.f, 1.f, 1.f, 1.f};
    gb_store<HDP>(dk, sc4, dqkv + G.C + h * G.hd, C3, G, grp, kb * 16, lane);
    gb_store<HDP>(dv, one4, dqkv + 2 * G.C + h * G.hd, C3, G, grp, kb * 16, lane);
  }
}

// ------------------------------------------------------------------------------------------------
// Large groups, second generation (knob grid_big = 2, the default).  The kernels above spend most
// of their time on the VALU, not the MFMA: per score they pay a scale multiply, a mask select, the
// max, a subtract, the log2(e) multiply inside __expf and a cross-lane row sum, and the probability
// products run on the 16x16x16 MFMA (half the 16x16x32 rate on gfx950).  Here:
//   * exp(s * scale - m) = exp2(s * scale*log2(e) - m2): one FMA + v_exp_f32 per score, the max is
//     taken on the raw scores (scale > 0) and scaled once per row;
//   * masks only on the ragged last step (N % 64 / % 32 / % 16 keys);
//   * lazy rescale: the running max m2 only moves (O and the row sum rescaled, 4 cross-lane reads)
//     when some row's chunk max exceeds it by more than 2^8, decided wave-uniformly; between
//     rescales P <= 2^8, exact in fp32 and bf16 (same 8-bit exponent);
//   * the row sum is kept per lane (its 4 keys of each chunk) and reduced over the 4 lane groups
//     once at the end;
//   * two 16-key chunks are paired into one 16x16x32 MFMA for P V, dS K, P^T dO and dS^T Q: the
//     A operand is [pack4(chunk c) | pack4(chunk c+1)], the B operand the two transposed LDS reads
//     of the same key rows, so k index i < 4 <-> key 16c + 4fg + i and i >= 4 <-> 16(c+1) + 4fg + i-4
//     on both sides.
constexpr float GB_LOG2E = 1.4426950408889634f, GB_LN2 = 0.6931471805599453f;
constexpr float GB_RESCALE = 8.f;  // log2 units

__device__ __forceinline__ float gb_exp2(float x) { return __builtin_amdgcn_exp2f(x); }

__device__ __forceinline__ bf16x8 gb_cat8(gm_s16x4 a, gm_s16x4 b) {
  typedef __attribute__((ext_vector_type(8))) short s16x8;
  const s16x8 t = __builtin_shufflevector(a, b, 0, 1, 2, 3, 4, 5, 6, 7);
  return __builtin_bit_cast(bf16x8, t);
}

// transposed 16x16x16-B-operand read of key rows row0 + 4fg + (fr >> 2), dims j*16 + (fr & 3)*4
__device__ __forceinline__ gm_s16x4 gb_tr(const bf16* tile, int row0, int pitch, int j, int lane) {
  const int fr = lane & 15, fg = lane >> 4;
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (gm_lds_s16x4*)(tile + (row0 + 4 * fg + (fr >> 2)) * pitch + j * 16 + (fr & 3) * 4));
}

template <int HDP>
__global__ __launch_bounds__(GB_NW * 64) void grid_big_fwd2_kernel(const bf16* __restrict__ qkv, bf16* __restrict__ out,
                                                                  float* __restrict__ lse, GridGeomM G, float scale,
                                                                  int Np) {
  constexpr int KK = HDP / 32, ND = HDP / 16, PITCH = gm_pitch<HDP>();
  extern __shared__ __attribute__((aligned(16))) bf16 gsm[];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int fr = lane & 15, fg = lane >> 4;
  const long C3 = 3L * G.C;
  const long pr = blockIdx.x;
  const int h = (int)(pr % G.heads);
  const long grp = pr / G.heads;
  const bf16* Ks = gsm;
  const bf16* Vs = gsm + (size_t)Np * PITCH;
  gb_stage2<HDP>(gsm, qkv + G.C + h * G.hd, C3, qkv + 2 * G.C + h * G.hd, C3, G, grp, Np);
  __syncthreads();
  const float sl2 = scale * GB_LOG2E;
  const int kfull = G.N & ~63;   // keys of the unmasked 64-key steps
  for (int qb = wave; qb < Np / 16; qb += GB_NW) {
    const int qtok = qb * 16 + fr;
    const bool qok = qtok < G.N;
    const long qpix = qok ? G.pixel(grp, qtok) : 0;
    bf16x8 qf[KK];
#pragma unroll
    for (int kk = 0; kk < KK; ++kk) {
      const int d = kk * 32 + fg * 8;
      qf[kk] = gm_load8(qkv + h * G.hd + qpix * C3 + d, qok && d < G.hd);
    }
    f32x4 o[ND];
#pragma unroll
    for (int j = 0; j < ND; ++j) o[j] = f32x4{0.f, 0.f, 0.f, 0.f};
    float m = -INFINITY, lp = 0.f;  // running max (log2 units, replicated over fg); this lane's row-sum part
    auto step = [&](const int k0, const int nc, const bool tail) {
      f32x4 sc[4];
      float mc = -INFINITY;
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        sc[c] = f32x4{0.f, 0.f, 0.f, 0.f};
        if (c < nc) {
#pragma unroll
          for (int kk = 0; kk < KK; ++kk) {
            const bf16x8 kf = *reinterpret_cast<const bf16x8*>(Ks + (k0 + 16 * c + fr) * PITCH + kk * 32 + fg * 8);
            sc[c] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kf, qf[kk], sc[c], 0, 0, 0);
          }
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          if (tail && !(c < nc && k0 + 16 * c + 4 * fg + r < G.N)) sc[c][r] = -INFINITY;
          mc = fmaxf(mc, sc[c][r]);
        }
      }
      mc = fmaxf(mc, __shfl_xor(mc, 16, 64));
      mc = fmaxf(mc, __shfl_xor(mc, 32, 64));
      const float mc2 = mc * sl2;
      if (__any(mc2 > m + GB_RESCALE)) {   // always on the first step (m = -inf)
        const float mn = fmaxf(m, mc2);
        const float corr = gb_exp2(m - mn);
        lp *= corr;
        float cr[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) cr[r] = __shfl(corr, 4 * fg + r, 64);
#pragma unroll
        for (int j = 0; j < ND; ++j)
#pragma unroll
          for (int r = 0; r < 4; ++r) o[j][r] *= cr[r];
        m = mn;
      }
#pragma unroll
      for (int c = 0; c < 4; ++c)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          sc[c][r] = gb_exp2(fmaf(sc[c][r], sl2, -m));   // masked: exp2(-inf) = 0
          lp += sc[c][r];
        }
#pragma unroll
      for (int cp = 0; cp < 2; ++cp) {
        if (2 * cp >= nc) break;
        const bool two = 2 * cp + 1 < nc;
        const float p0[4] = {sc[2 * cp][0], sc[2 * cp][1], sc[2 * cp][2], sc[2 * cp][3]};
        const float p1[4] = {sc[2 * cp + 1][0], sc[2 * cp + 1][1], sc[2 * cp + 1][2], sc[2 * cp + 1][3]};
        const bf16x8 pa = gb_cat8(pack4(p0), pack4(p1));
#pragma unroll
        for (int j = 0; j < ND; ++j) {
          const gm_s16x4 v0 = gb_tr(Vs, k0 + 32 * cp, PITCH, j, lane);
          const gm_s16x4 v1 = two ? gb_tr(Vs, k0 + 32 * cp + 16, PITCH, j, lane) : gm_s16x4{0, 0, 0, 0};
          o[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(pa, gb_cat8(v0, v1), o[j], 0, 0, 0);
        }
      }
    };
    int k0 = 0;
    for (; k0 < kfull; k0 += 64) step(k0, 4, false);
    if (k0 < Np) step(k0, (Np - k0) / 16, true);
    float l = lp + __shfl_xor(lp, 16, 64);
    l += __shfl_xor(l, 32, 64);
    float inv[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) inv[r] = 1.f / __shfl(l, 4 * fg + r, 64);
    gb_store<HDP>(o, inv, out + h * G.hd, G.C, G, grp, qb * 16, lane);
    if (fg == 0 && qok) lse[qpix * G.heads + h] = m * GB_LN2 + __logf(l);
  }
}

// dQ, second generation: K and V resident; 32 keys (two S^T / dP^T chunks) per 16x16x32 dS K MFMA.
template <int HDP>
__global__ __launch_bounds__(GB_NW * 64) void grid_big_dq2_kernel(const bf16* __restrict__ dout,
                                                                 const bf16* __restrict__ qkv,
                                                                 const float* __restrict__ lse,
                                                                 const float* __restrict__ delta,
                                                                 bf16* __restrict__ dqkv, GridGeomM G, float scale,
                                                                 int Np) {
  constexpr int KK = HDP / 32, ND = HDP / 16, PITCH = gm_pitch<HDP>();
  extern __shared__ __attribute__((aligned(16))) bf16 gsm[];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int fr = lane & 15, fg = lane >> 4;
  const long C3 = 3L * G.C;
  const long pr = blockIdx.x;
  const int h = (int)(pr % G.heads);
  const long grp = pr / G.heads;
  const bf16* Ks = gsm;
  const bf16* Vs = gsm + (size_t)Np * PITCH;
  gb_stage2<HDP>(gsm, qkv + G.C + h * G.hd, C3, qkv + 2 * G.C + h * G.hd, C3, G, grp, Np);
  __syncthreads();
  const float sl2 = scale * GB_LOG2E;
  const int kfull = G.N & ~31;
  for (int qb = wave; qb < Np / 16; qb += GB_NW) {
    const int qtok = qb * 16 + fr;
    const bool qok = qtok < G.N;
    const long qpix = qok ? G.pixel(grp, qtok) : 0;
    bf16x8 qf[KK], gf[KK];  // Q^T and dO^T as B operands (query fr)
#pragma unroll
    for (int kk = 0; kk < KK; ++kk) {
      const int d = kk * 32 + fg * 8;
      qf[kk] = gm_load8(qkv + h * G.hd + qpix * C3 + d, qok && d < G.hd);
      gf[kk] = gm_load8(dout + qpix * G.C + h * G.hd + d, qok && d < G.hd);
    }
    const float lq2 = qok ? lse[qpix * G.heads + h] * GB_LOG2E : INFINITY;   // invalid query: P = 0
    const float dl = qok ? delta[qpix * G.heads + h] : 0.f;
    f32x4 dq[ND];
#pragma unroll
    for (int j = 0; j < ND; ++j) dq[j] = f32x4{0.f, 0.f, 0.f, 0.f};
    auto chunk = [&](const int k0, const bool tail, float (&ds)[4]) {
      f32x4 sv = f32x4{0.f, 0.f, 0.f, 0.f}, dp = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kk = 0; kk < KK; ++kk) {
        const bf16x8 kf = *reinterpret_cast<const bf16x8*>(Ks + (k0 + fr) * PITCH + kk * 32 + fg * 8);
        const bf16x8 vf = *reinterpret_cast<const bf16x8*>(Vs + (k0 + fr) * PITCH + kk * 32 + fg * 8);
        sv = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kf, qf[kk], sv, 0, 0, 0);    // S^T
        dp = __builtin_amdgcn_mfma_f32_16x16x32_bf16(vf, gf[kk], dp, 0, 0, 0);    // dP^T
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float pw = gb_exp2(fmaf(sv[r], sl2, -lq2));
        if (tail && k0 + 4 * fg + r >= G.N) pw = 0.f;
        ds[r] = pw * (dp[r] - dl);
      }
    };
    auto pair = [&](const int k0, const bool tail) {
      const bool two = k0 + 16 < Np;
      float d0[4], d1[4] = {0.f, 0.f, 0.f, 0.f};
      chunk(k0, tail, d0);
      if (two) chunk(k0 + 16, tail, d1);
      const bf16x8 da = gb_cat8(pack4(d0), pack4(d1));   // A operand: dS[query fr][32 keys]
#pragma unroll
      for (int j = 0; j < ND; ++j) {
        const gm_s16x4 k0b = gb_tr(Ks, k0, PITCH, j, lane);
        const gm_s16x4 k1b = two ? gb_tr(Ks, k0 + 16, PITCH, j, lane) : gm_s16x4{0, 0, 0, 0};
        dq[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(da, gb_cat8(k0b, k1b), dq[j], 0, 0, 0);
      }
    };
    int k0 = 0;
    for (; k0 < kfull; k0 += 32) pair(k0, false);
    if (k0 < Np) pair(k0, true);
    const float sc4[4] = {scale, scale, scale, scale};
    gb_store<HDP>(dq, sc4, dqkv + h * G.hd, C3, G, grp, qb * 16, lane);
  }
}

// dK, dV, second generation: Q, dO, lse*log2(e), delta resident; 32 queries per 16x16x32 MFMA pair.
template <int HDP>
__global__ __launch_bounds__(GB_NW * 64) void grid_big_dkv2_kernel(const bf16* __restrict__ dout,
                                                                  const bf16* __restrict__ qkv,
                                                                  const float* __restrict__ lse,
                                                                  const float* __restrict__ delta,
                                                                  bf16* __restrict__ dqkv, GridGeomM G, float scale,
                                                                  int Np) {
  constexpr int KK = HDP / 32, ND = HDP / 16, PITCH = gm_pitch<HDP>();
  extern __shared__ __attribute__((aligned(16))) bf16 gsm[];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int fr = lane & 15, fg = lane >> 4;
  const long C3 = 3L * G.C;
  const long pr = blockIdx.x;
  const int h = (int)(pr % G.heads);
  const long grp = pr / G.heads;
  const bf16* Qs = gsm;
  const bf16* Gs = gsm + (size_t)Np * PITCH;
  float* lq_s = reinterpret_cast<float*>(gsm + 2 * (size_t)Np * PITCH);
  float* dl_s = lq_s + Np;
  gb_stage2<HDP>(gsm, qkv + h * G.hd, C3, dout + h * G.hd, G.C, G, grp, Np);
  for (int t = threadIdx.x; t < Np; t += GB_NW * 64) {   // padded rows: lse = inf -> P = 0
    const bool ok = t < G.N;
    const long pq = ok ? G.pixel(grp, t) : 0;
    lq_s[t] = ok ? lse[pq * G.heads + h] * GB_LOG2E : INFINITY;
    dl_s[t] = ok ? delta[pq * G.heads + h] : 0.f;
  }
  __syncthreads();
  const float sl2 = scale * GB_LOG2E;
  for (int kb = wave; kb < Np / 16; kb += GB_NW) {
    const int ktok = kb * 16 + fr;
    const bool kok = ktok < G.N;
    const long kpix = kok ? G.pixel(grp, ktok) : 0;
    bf16x8 kf[KK], vf[KK];  // K^T, V^T as B operands (key fr)
#pragma unroll
    for (int kk = 0; kk < KK; ++kk) {
      const int d = kk * 32 + fg * 8;
      kf[kk] = gm_load8(qkv + G.C + h * G.hd + kpix * C3 + d, kok && d < G.hd);
      vf[kk] = gm_load8(qkv + 2 * G.C + h * G.hd + kpix * C3 + d, kok && d < G.hd);
    }
    f32x4 dk[ND], dv[ND];
#pragma unroll
    for (int j = 0; j < ND; ++j) {
      dk[j] = f32x4{0.f, 0.f, 0.f, 0.f};
      dv[j] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
    auto chunk = [&](const int q0, float (&pw)[4], float (&ds)[4]) {
      // S[query 4fg+r][key fr] = Q K^T ; dP = dO V^T
      f32x4 sv = f32x4{0.f, 0.f, 0.f, 0.f}, dp = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kk = 0; kk < KK; ++kk) {
        const bf16x8 qa = *reinterpret_cast<const bf16x8*>(Qs + (q0 + fr) * PITCH + kk * 32 + fg * 8);
        const bf16x8 ga = *reinterpret_cast<const bf16x8*>(Gs + (q0 + fr) * PITCH + kk * 32 + fg * 8);
        sv = __builtin_amdgcn_mfma_f32_16x16x32_bf16(qa, kf[kk], sv, 0, 0, 0);
        dp = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ga, vf[kk], dp, 0, 0, 0);
      }
      const float4 lq4 = *reinterpret_cast<const float4*>(lq_s + q0 + 4 * fg);
      const float4 dl4 = *reinterpret_cast<const float4*>(dl_s + q0 + 4 * fg);
      const float lq[4] = {lq4.x, lq4.y, lq4.z, lq4.w}, dl[4] = {dl4.x, dl4.y, dl4.z, dl4.w};
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        pw[r] = kok ? gb_exp2(fmaf(sv[r], sl2, -lq[r])) : 0.f;
        ds[r] = pw[r] * (dp[r] - dl[r]);
      }
    };
    for (int q0 = 0; q0 < Np; q0 += 32) {
      const bool two = q0 + 16 < Np;
      float p0[4], d0[4], p1[4] = {0.f, 0.f, 0.f, 0.f}, d1[4] = {0.f, 0.f, 0.f, 0.f};
      chunk(q0, p0, d0);
      if (two) chunk(q0 + 16, p1, d1);
      const bf16x8 pa = gb_cat8(pack4(p0), pack4(p1)), da = gb_cat8(pack4(d0), pack4(d1));
#pragma unroll
      for (int j = 0; j < ND; ++j) {
        const gm_s16x4 g0 = gb_tr(Gs, q0, PITCH, j, lane), q0b = gb_tr(Qs, q0, PITCH, j, lane);
        const gm_s16x4 g1 = two ? gb_tr(Gs, q0 + 16, PITCH, j, lane) : gm_s16x4{0, 0, 0, 0};
        const gm_s16x4 q1b = two ? gb_tr(Qs, q0 + 16, PITCH, j, lane) : gm_s16x4{0, 0, 0, 0};
        dv[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(pa, gb_cat8(g0, g1), dv[j], 0, 0, 0);
        dk[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(da, gb_cat8(q0b, q1b), dk[j], 0, 0, 0);
      }
    }
    const float sc4[4] = {scale, scale, scale, scale}, one4[4] = {1.f, 1.f, 1.f, 1.f};
    gb_store<HDP>(dk, sc4, dqkv + G.C + h * G.hd, C3, G, grp, kb * 16, lane);
    gb_store<HDP>(dv, one4, dqkv + 2 * G.C + h * G.hd, C3, G, grp, kb * 16, lane);
  }
}

template <int HDP>
static bool grid_big_bwd_try(const GridGeomM& G, const void* dout, const void* qkv, const float* lse,
                             const float* delta, void* dqkv, float scale, hipStream_t s);

// tuning knob "grid_big": one-pair-per-block LDS kernels for large groups (0 off, 1 first
// generation, 2 exp2/lazy-rescale/16x16x32 second generation)
static int g_grid_big = 2;
void set_grid_big(int v) { g_grid_big = v < 0 ? 0 : (v > 2 ? 2 : v); }
constexpr size_t GB_LDS_MAX = 160 * 1024;

template <int HDP>
static bool grid_big_fwd_try(const GridGeomM& G, const void* qkv, void* out, float* lse, float scale, hipStream_t s) {
  const int Np = (G.N + 15) / 16 * 16;
  const size_t lds = 2 * (size_t)Np * gm_pitch<HDP>() * sizeof(bf16);
  if (!g_grid_big || lds > GB_LDS_MAX) return false;
  if (!lds_grant(reinterpret_cast<const void*>(grid_big_fwd_kernel<HDP>), GB_LDS_MAX) ||
      !lds_grant(reinterpret_cast<const void*>(grid_big_fwd2_kernel<HDP>), GB_LDS_MAX))
    return false;   // the caller takes the unfused path
  const long pairs = (long)G.B * G.g * G.g * G.heads;
  if (g_grid_big == 2)
    grid_big_fwd2_kernel<HDP><<<(unsigned)pairs, GB_NW * 64, lds, s>>>((const bf16*)qkv, (bf16*)out, lse, G, scale, Np);
  else
    grid_big_fwd_kernel<HDP><<<(unsigned)pairs, GB_NW * 64, lds, s>>>((const bf16*)qkv, (bf16*)out, lse, G, scale, Np);
  return true;
}

template <int HDP>
static bool grid_big_bwd_try(const GridGeomM& G, const void* dout, const void* qkv, const float* lse,
                             const float* delta, void* dqkv, float scale, hipStream_t s) {
  const int Np = (G.N + 15) / 16 * 16;
  const size_t l1 = 2 * (size_t)Np * gm_pitch<HDP>() * sizeof(bf16), l2 = l1 + 2 * (size_t)Np * sizeof(float);
  if (!g_grid_big || l2 > GB_LDS_MAX) return false;
  for (const void* k : {reinterpret_cast<const void*>(grid_big_dq_kernel<HDP>),
                        reinterpret_cast<const void*>(grid_big_dkv_kernel<HDP>),
                        reinterpret_cast<const void*>(grid_big_dq2_kernel<HDP>),
                        reinterpret_cast<const void*>(grid_big_dkv2_kernel<HDP>)})
    if (!lds_grant(k, GB_LDS_MAX)) return false;
  const long pairs = (long)G.B * G.g * G.g * G.heads;
  if (g_grid_big == 2) {
    grid_big_dq2_kernel<HDP><<<(unsigned)pairs, GB_NW * 64, l1, s>>>((const bf16*)dout, (const bf16*)qkv, lse, delta,
                                                                     (bf16*)dqkv, G, scale, Np);
    grid_big_dkv2_kernel<HDP><<<(unsigned)pairs, GB_NW * 64, l2, s>>>((const bf16*)dout, (const bf16*)qkv, lse, delta,
                                                                      (bf16*)dqkv, G, scale, Np);
    return true;
  }
  grid_big_dq_kernel<HDP><<<(unsigned)pairs, GB_NW * 64, l1, s>>>((const bf16*)dout, (const bf16*)qkv, lse, delta,
                                                                  (bf16*)dqkv, G, scale, Np);
  grid_big_dkv_kernel<HDP><<<(unsigned)pairs, GB_NW * 64, l2, s>>>((const bf16*)dout, (const bf16*)qkv, lse, delta,
                                                                   (bf16*)dqkv, G, scale, Np);
  return true;
}

static int g_grid_lds = 1;  // tuning knob "grid_lds": LDS-resident pairs when they fit
void set_grid_lds(int v) { g_grid_lds = v; }
constexpr size_t GM_LDS_MAX = 64 * 1024;

// ------------------------------------------------------------------------------------------------
static bool gm_ok(const GridGeomM& G) { return G.N >= 16 && G.hd % 8 == 0 && G.hd <= 64; }

bool grid_mfma_fwd(const void* qkv, void* out, float* lse, int B, int H, int W, int C, int heads, int g, float scale,
                   hipStream_t s) {
  GridGeomM G{B, H, W, C, heads, g, H / g, W / g, (H / g) * (W / g), C / heads};
  if (!gm_ok(G)) return false;
  if (g_grid_lds && G.N > 16) {
    if (G.hd <= 32) {
      const GmLds L = gm_lds_plan<32>(G);
      const size_t lds = gm_lds_bytes<32>(L, false);
      if (lds <= GM_LDS_MAX) {
        grid_lds_fwd_kernel<32><<<(unsigned)L.blocks, 256, lds, s>>>((const bf16*)qkv, (bf16*)out, lse, G, scale, L);
        return true;
      }
    } else {
      const GmLds L = gm_lds_plan<64>(G);
      const size_t lds = gm_lds_bytes<64>(L, false);
      if (lds <= GM_LDS_MAX) {
        grid_lds_fwd_kernel<64><<<(unsigned)L.blocks, 256, lds, s>>>((const bf16*)qkv, (bf16*)out, lse, G, scale, L);
        return true;
      }
    }
  }
  if (G.N > 16 && (G.hd <= 32 ? grid_big_fwd_try<32>(G, qkv, out, lse, scale, s)
                                : grid_big_fwd_try<64>(G, qkv, out, lse, scale, s)))
    return true;
  const long units = (long)B * g * g * heads * ((G.N + 15) / 16);
  const unsigned grid = cdiv(units, 4);
  if (G.hd <= 32)
    grid_mfma_fwd_kernel<32><<<grid, 256, 0, s>>>((const bf16*)qkv, (bf16*)out, lse, G, scale, units);
  else
    grid_mfma_fwd_kernel<64><<<grid, 256, 0, s>>>((const bf16*)qkv, (bf16*)out, lse, G, scale, units);
  return true;
}

// delta must already hold rowsum(dO * O) per (pixel, head)
bool grid_mfma_bwd(const void* dout, const void* qkv, const float* lse, const float* delta, void* dqkv, int B, int H,
                   int W, int C, int heads, int g, float scale, hipStream_t s) {
  GridGeomM G{B, H, W, C, heads, g, H / g, W / g, (H / g) * (W / g), C / heads};
  if (!gm_ok(G)) return false;
  if (g_grid_lds && G.N > 16) {
#define OGV_GRID_LDS_BWD(HD)                                                                                          \
  {                                                                                                                   \
    const GmLds L = gm_lds_plan<HD>(G);                                                                               \
    const size_t l1 = gm_lds_bytes<HD>(L, false), l2 = gm_lds_bytes<HD>(L, true);                                     \
    if (l2 <= GM_LDS_MAX) {                                                                                           \
      grid_lds_dq_kernel<HD><<<(unsigned)L.blocks, 256, l1, s>>>((const bf16*)dout, (const bf16*)qkv, lse, delta,     \
                                                                 (bf16*)dqkv, G, scale, L);                          \
      grid_lds_dkv_kernel<HD><<<(unsigned)L.blocks, 256, l2, s>>>((const bf16*)dout, (const bf16*)qkv, lse, delta,    \
                                                                  (bf16*)dqkv, G, scale, L);                         \
      return true;                                                                                                    \
    }                                                                                                                 \
  }
    if (G.hd <= 32) OGV_GRID_LDS_BWD(32) else OGV_GRID_LDS_BWD(64)
#undef OGV_GRID_LDS_BWD
  }
  if (G.N > 16 && (G.hd <= 32 ? grid_big_bwd_try<32>(G, dout, qkv, lse, delta, dqkv, scale, s)
                              : grid_big_bwd_try<64>(G, dout, qkv, lse, delta, dqkv, scale, s)))
    return true;
  const long units = (long)B * g * g * heads * ((G.N + 15) / 16);
  const unsigned grid = cdiv(units, 4);
  if (G.hd <= 32) {
    grid_mfma_dq_kernel<32><<<grid, 256, 0, s>>>((const bf16*)dout, (const bf16*)qkv, lse, delta, (bf16*)dqkv, G, scale,
                                                 units);
    grid_mfma_dkv_kernel<32><<<grid, 256, 0, s>>>((const bf16*)dout, (const bf16*)qkv, lse, delta, (bf16*)dqkv, G,
                                                  scale, units);
  } else {
    grid_mfma_dq_kernel<64><<<grid, 256, 0, s>>>((const bf16*)dout, (const bf16*)qkv, lse, delta, (bf16*)dqkv, G, scale,
                                                 units);
    grid_mfma_dkv_kernel<64><<<grid, 256, 0, s>>>((const bf16*)dout, (const bf16*)qkv, lse, delta, (bf16*)dqkv, G,
                                                  scale, units);
  }
  return true;
}

}  // namespace ogv
