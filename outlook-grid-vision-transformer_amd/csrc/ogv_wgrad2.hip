// Pipelined bf16 weight gradient (gfx950) for the mid-M projections (M = 8k-131k rows).
//
//   dW[n, k] = sum_m rs(m) G[m, n] * pro(X)[m, k],   dbias[n] = sum_m rs(m) G[m, n]
//
// The split-M tiled kernel of ogv_gemm.hip stages 32 rows per step behind two barriers with the
// next step's loads one short MFMA phase ahead: at these shapes a workgroup's step is a few dozen
// MFMAs, so every step waits out an L2/HBM round trip, and its X prologue (GELU of MLP fc2, BN +
// SiLU + SE gate of MBConv project) runs in that serial staging phase, once per N tile (measured
// isolated, M=32768 N=192 K=768: 156 us with the GELU prologue vs 50 us without it).  Here:
//   * 64 rows per step (two 32-deep MFMA k-blocks), two LDS buffers, ONE barrier per step;
//   * two register sets: step t+1 is staged from registers while step t+2's loads are in flight,
//     so each load has two compute phases to land;
//   * the prologue form is a template parameter (no runtime switch per element), and the tile
//     edge may cover all of N (BN = 192), so the prologue runs once per X element;
//   * loads use clamped, always-valid addresses and select zero afterwards (no branch per load).
// Output: fp32 partials [S][N*K + N] (the tiled kernel's layout) and, with an arrival counter per
// output tile (knob wg2_fuse = 1), dW / dbias themselves: the LAST workgroup of a tile to finish (arrival
// counted by one agent-scope atomic ticket behind write-through partial stores) sums that tile's S
// partials in slab order 0..S-1 -- deterministic, whichever workgroup arrives last -- and resets
// the counter, so no separate column-reduce launch follows (slower at these slab counts: see the knob).
// Fragment reads: ds_read_b64_tr_b16 with the same m-permutation as the tiled kernel (rows 4g+q and
// 16+4g+q of each 32-row block; an odd multiple of 16 as pitch keeps them conflict-free).
#include "ogv_gemm.h"

namespace ogv {

constexpr int W2_MS = 64;   // rows per pipeline step
constexpr int W2_NT = 256;  // 4 waves, 2 x 2 over the output tile

// prologue forms: -1 none; OGV_ACT_GELU: gelu(x); OGV_ACT_SILU: silu(x * sc + sh) * gate; 99: any (runtime)
constexpr int W2_GENERIC = 99;

// arrival counters of the fused reduction: zero at module load, each used window reset to zero by
// its last workgroup; the host hands every launch its own window of a ring (w2_counters)
constexpr int W2_CNT = 1 << 16;
__device__ unsigned g_w2_cnt[W2_CNT];
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

// CV: X is the implicit-GEMM gather of a 3x3 convolution's input (ConvG cv; row m = output pixel,
// column k = tap * Cs + channel, 8 | Cs so an 8-column chunk never straddles a tap; zero padding)
template <int BN, int BK, int PA, bool CV = false>
__global__ __launch_bounds__(W2_NT) void wgrad2_bf16_kernel(const bf16* __restrict__ G, int ldg,
                                                            const bf16* __restrict__ X, int ldx, Pro pro,
                                                            const float* __restrict__ rs, int rps,
                                                            float* __restrict__ part, long ldp, int want_bias, int M,
                                                            int N, int K, int mchunk, int nNt, int tiles, int S,
                                                            int cnt0, float* __restrict__ dW, float* __restrict__ dbias,
                                                            ConvG cv) {
  constexpr int MS = W2_MS;
  constexpr int GP = BN + 16, XP = BK + 16;      // odd multiples of 16 for BN in {64, 96, 128, 192}, BK in {64, 128}
  constexpr int GC = BN / 8, XC = BK / 8;        // 16-B chunks per staged row
  constexpr int GV = MS * GC / W2_NT, XV = MS * XC / W2_NT;
  static_assert(GV * W2_NT == MS * GC && XV * W2_NT == MS * XC, "tile edge must make whole chunk passes");
  constexpr int TN = BN / 32, TK = BK / 32;      // 16-wide fragments per wave (wave tile BN/2 x BK/2)
  constexpr int BUF = MS * (GP + XP);            // bf16 elements per LDS buffer
  __shared__ __attribute__((aligned(16))) bf16 smem[2 * BUF];

  const int b = blockIdx.x, xcd = b & 7, local = b >> 3;
  const int tile = local % tiles, s = (local / tiles) * 8 + xcd;
  if (s >= S) return;
  const int nt = tile % nNt, kt = tile / nNt;
  const int n0 = nt * BN, k0 = kt * BK;
  const int mbeg = s * mchunk, mend = min(M, mbeg + mchunk);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wn = wave >> 1, wk = wave & 1;

  f32x4 acc[TN][TK];
#pragma unroll
  for (int i = 0; i < TN; ++i)
#pragma unroll
    for (int j = 0; j < TK; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // per-chunk coordinates (chunk id = tid + v * 256 -> row id / GC, column chunk id % GC).  XC
  // divides 256, so a thread's X chunks all sit in one column chunk (its BN scale / shift and column
  // guard are loop-invariant scalars); G chunks may not (BN = 96 / 192).
  int grow[GV], gcol[GV];
  bool gok[GV];
#pragma unroll
  for (int v = 0; v < GV; ++v) {
    const int id = tid + v * W2_NT;
    grow[v] = id / GC;
    gcol[v] = (id % GC) * 8;
    gok[v] = n0 + gcol[v] < N;
  }
  static_assert(W2_NT % XC == 0, "X chunk columns must be thread-invariant");
  const int xrow0 = tid / XC, xcol = (tid % XC) * 8;
  constexpr int XRP = W2_NT / XC;  // X rows per chunk pass
  const bool xok = k0 + xcol < K;
  const int xk = xok ? k0 + xcol : 0;
  // dbias[n] = sum_m G[m, n] rides on the MFMA: the waves of the first K tile with wk == 0 multiply
  // their G fragments by a ones fragment as well (+1/TK MFMAs, no per-thread bias registers)
  const bool bias_wave = want_bias && kt == 0 && wk == 0;
  f32x4 bacc[TN];
#pragma unroll
  for (int i = 0; i < TN; ++i) bacc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  // loop-invariant BN scale / shift of the X columns (SiLU form)
  constexpr bool SG = PA == OGV_ACT_SILU;
  float psc[8], psh[8];
#pragma unroll
  for (int t = 0; t < 8; ++t) { psc[t] = 1.f; psh[t] = 0.f; }
  if constexpr (SG) {
    load_vec<float, 8>(pro.sc + xk, psc);
    load_vec<float, 8>(pro.sh + xk, psh);
  }

  struct Regs {
    uint4 g[GV], x[XV];
    float r[GV];
    float gt[SG ? XV : 1][8];
  };
  auto load = [&](Regs& R, int m0) {
#pragma unroll
    for (int v = 0; v < GV; ++v) {
      const int m = min(m0 + grow[v], mend - 1);
      R.g[v] = *reinterpret_cast<const uint4*>(G + (long)m * ldg + (gok[v] ? n0 + gcol[v] : 0));
      R.r[v] = rs ? rs[m / rps] : 1.f;
    }
#pragma unroll
    for (int v = 0; v < XV; ++v) {
      const int m = min(m0 + xrow0 + v * XRP, mend - 1);
      if constexpr (CV) {
        const int tap = xk / cv.Cs;
        const long off = conv_src(cv, conv_row(cv, m), tap);
        // unconditional load at a valid address (element 0 for a zero tap), zero selected after: the
        // guarded form made the compiler wait for each of these loads in turn
        const uint4 xv = *reinterpret_cast<const uint4*>(X + (off >= 0 ? off + (xk - tap * cv.Cs) : 0));
        R.x[v] = off >= 0 ? xv : uint4{0u, 0u, 0u, 0u};
      } else {
        R.x[v] = *reinterpret_cast<const uint4*>(X + (long)m * ldx + xk);
      }
      if constexpr (SG) load_vec<float, 8>(pro.gate + (long)(m / pro.rps) * pro.gld + xk, R.gt[v]);
    }
  };
  auto stage = [&](Regs& R, int m0, bf16* buf) {
    bf16* Gs = buf;
    bf16* Xs = buf + MS * GP;
#pragma unroll
    for (int v = 0; v < GV; ++v) {
      const bool ok = gok[v] && m0 + grow[v] < mend;
      uint4 u = ok ? R.g[v] : uint4{0u, 0u, 0u, 0u};
      bf16* e = reinterpret_cast<bf16*>(&u);
      if (rs) {
#pragma unroll
        for (int t = 0; t < 8; ++t) e[t] = (bf16)((float)e[t] * R.r[v]);
      }
      *reinterpret_cast<uint4*>(Gs + grow[v] * GP + gcol[v]) = u;
    }
#pragma unroll
    for (int v = 0; v < XV; ++v) {
      const int m = m0 + xrow0 + v * XRP;
      const bool ok = xok && m < mend;
      uint4 u = ok ? R.x[v] : uint4{0u, 0u, 0u, 0u};
      if constexpr (PA >= 0) {
        bf16* e = reinterpret_cast<bf16*>(&u);
        float f[8];
#pragma unroll
        for (int t = 0; t < 8; ++t) f[t] = (float)e[t];
        if constexpr (PA == W2_GENERIC) {
          if (ok) pro_apply_run<8>(pro, f, m, k0 + xcol, K);
        } else if constexpr (SG) {
#pragma unroll
          for (int t = 0; t < 8; ++t) f[t] = act_fwd(OGV_ACT_SILU, fmaf(f[t], psc[t], psh[t])) * R.gt[v][t];
        } else {
#pragma unroll
          for (int t = 0; t < 8; ++t) f[t] = act_fwd(PA, f[t]);
        }
#pragma unroll
        for (int t = 0; t < 8; ++t) e[t] = ok ? (bf16)f[t] : (bf16)0.f;
      }
      *reinterpret_cast<uint4*>(Xs + (xrow0 + v * XRP) * XP + xcol) = u;
    }
  };
  const int g = lane >> 4, c16 = lane & 15, q = c16 >> 2, p4 = (c16 & 3) * 4;
  typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
  typedef __attribute__((ext_vector_type(8))) short s16x8;
  auto compute = [&](const bf16* buf) {
    const bf16* Gs = buf;
    const bf16* Xs = buf + MS * GP;
#pragma unroll
    for (int kb = 0; kb < MS / 32; ++kb) {
      const int r0 = kb * 32 + 4 * g + q;
      bf16x8 af[TN], xf[TK];
#pragma unroll
      for (int i = 0; i < TN; ++i) {
        const int col = wn * (BN / 2) + i * 16 + p4;
        s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(Gs + r0 * GP + col));
        s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(Gs + (r0 + 16) * GP + col));
        s16x8 a8 = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        af[i] = __builtin_bit_cast(bf16x8, a8);
      }
#pragma unroll
      for (int j = 0; j < TK; ++j) {
        const int col = wk * (BK / 2) + j * 16 + p4;
        s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(Xs + r0 * XP + col));
        s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(Xs + (r0 + 16) * XP + col));
        s16x8 x8 = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        xf[j] = __builtin_bit_cast(bf16x8, x8);
      }
#pragma unroll
      for (int i = 0; i < TN; ++i)
#pragma unroll
        for (int j = 0; j < TK; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], xf[j], acc[i][j], 0, 0, 0);
      if (bias_wave) {
        const s16x8 one8 = {0x3F80, 0x3F80, 0x3F80, 0x3F80, 0x3F80, 0x3F80, 0x3F80, 0x3F80};  // bf16 1.0
        const bf16x8 ones = __builtin_bit_cast(bf16x8, one8);
#pragma unroll
        for (int i = 0; i < TN; ++i) bacc[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], ones, bacc[i], 0, 0, 0);
      }
    }
  };

  // ---- pipeline: LDS buffers 0/1 alternate; register sets A/B hold steps t+1 / t+2
  const int nsteps = (mend - mbeg + MS - 1) / MS;
  bf16* buf0 = smem;
  bf16* buf1 = smem + BUF;
  Regs RA, RB;
  load(RA, mbeg);
  if (nsteps > 1) load(RB, mbeg + MS);
  stage(RA, mbeg, buf0);
  if (nsteps > 2) load(RA, mbeg + 2 * MS);
  __syncthreads();
  for (int t = 0; t < nsteps; t += 2) {
    compute(buf0);
    if (t + 1 < nsteps) {
      stage(RB, mbeg + (t + 1) * MS, buf1);
      if (t + 3 < nsteps) load(RB, mbeg + (t + 3) * MS);
    }
    __syncthreads();
    if (t + 1 >= nsteps) break;
    compute(buf1);
    if (t + 2 < nsteps) {
      stage(RA, mbeg + (t + 2) * MS, buf0);
      if (t + 4 < nsteps) load(RA, mbeg + (t + 4) * MS);
    }
    __syncthreads();
  }

  if (cnt0 < 0) {   // partials only: the caller's colreduce sums them
    float* dst = part + (long)s * ldp;
#pragma unroll
    for (int i = 0; i < TN; ++i)
#pragma unroll
      for (int j = 0; j < TK; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int n = n0 + wn * (BN / 2) + i * 16 + 4 * g + r;
          const int k = k0 + wk * (BK / 2) + j * 16 + c16;
          if (n < N && k < K) dst[(long)n * K + k] = acc[i][j][r];
        }
    if (bias_wave && c16 == 0) {  // every column of the ones product holds the row sum
#pragma unroll
      for (int i = 0; i < TN; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int n = n0 + wn * (BN / 2) + i * 16 + 4 * g + r;
          if (n < N) dst[(long)N * K + n] = bacc[i][r];
        }
    }
    return;
  }
  // ---- fused reduction (cdna_hip_programming.md §5 "In-launch split-K reduction", sc1 form): the
  // partial tile goes out as 16-B WRITE-THROUGH (sc1) stores, staged through LDS into whole rows;
  // every wave drains them (vmcnt 0) before the workgroup barrier, then ONE lane takes a ticket
  // (relaxed agent-scope add); the workgroup that draws S - 1 reads all S partial tiles with sc1
  // loads (never an L2 writeback / invalidate: no __threadfence) in slab order 0..S-1.
  constexpr int TP = BK + 4;                         // fp32 tile pitch: conflict-free fragment writes
  float* T = reinterpret_cast<float*>(smem);         // [BN][TP] partial tile, then [BN] bias, then a flag
  float* Tb = T + BN * TP;
  unsigned* flag = reinterpret_cast<unsigned*>(Tb + BN);
  static_assert((BN * TP + BN + 1) * 4 <= 2 * BUF * 2, "fp32 tile must fit the staging LDS");
  __syncthreads();                                   // every wave's last fragment reads are done
#pragma unroll
  for (int i = 0; i < TN; ++i)
#pragma unroll
    for (int j = 0; j < TK; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        T[(wn * (BN / 2) + i * 16 + 4 * g + r) * TP + wk * (BK / 2) + j * 16 + c16] = acc[i][j][r];
  if (bias_wave && c16 == 0) {
#pragma unroll
    for (int i = 0; i < TN; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) Tb[wn * (BN / 2) + i * 16 + 4 * g + r] = bacc[i][r];
  }
  __syncthreads();
  const __amdgpu_buffer_rsrc_t prs = __builtin_amdgcn_make_buffer_rsrc(part, (short)0, (int)(S * ldp * 4), 0x00020000);
  constexpr int C4 = BK / 4;   // 16-B chunks per tile row
  const bool bias_tile = want_bias && kt == 0;
  for (int e = tid; e < BN * C4; e += W2_NT) {
    const int nl = e / C4, kl = (e % C4) * 4, n = n0 + nl, k = k0 + kl;
    if (n >= N || k >= K) continue;
    const float4 v = *reinterpret_cast<const float4*>(T + nl * TP + kl);
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), prs, (int)(((long)s * ldp + (long)n * K + k) * 4), 0,
                                           16);
  }
  if (bias_tile) {
    for (int e = tid; e < BN / 4; e += W2_NT) {
      const int n = n0 + 4 * e;
      if (n >= N) continue;
      const float4 v = *reinterpret_cast<const float4*>(Tb + 4 * e);
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), prs, (int)(((long)s * ldp + (long)N * K + n) * 4),
                                             0, 16);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // EVERY storing wave drains its sc1 stores
  __syncthreads();
  if (tid == 0)
    flag[0] = __hip_atomic_fetch_add(&g_w2_cnt[cnt0 + tile], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ==
              (unsigned)(S - 1);
  __syncthreads();
  if (!flag[0]) return;
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");   // (compiler ordering only: every load below is sc1)
  for (int e = tid; e < BN * C4; e += W2_NT) {
    const int n = n0 + e / C4, k = k0 + (e % C4) * 4;
    if (n >= N || k >= K) continue;
    const int off = (int)(((long)n * K + k) * 4), step = (int)(ldp * 4);
    float4 a = make_float4(0.f, 0.f, 0.f, 0.f);
    int r = 0;
    for (; r + 8 <= S; r += 8) {
      float4 v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u)
        v[u] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(prs, off + (r + u) * step, 0, 16));
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        a.x += v[u].x; a.y += v[u].y; a.z += v[u].z; a.w += v[u].w;
      }
    }
    for (; r < S; ++r) {
      const float4 v = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(prs, off + r * step, 0, 16));
      a.x += v.x; a.y += v.y; a.z += v.z; a.w += v.w;
    }
    *reinterpret_cast<float4*>(dW + (long)n * K + k) = a;
  }
  if (bias_tile && dbias) {
    for (int e = tid; e < BN / 4; e += W2_NT) {
      const int n = n0 + 4 * e;
      if (n >= N) continue;
      const int off = (int)(((long)N * K + n) * 4), step = (int)(ldp * 4);
      float4 a = make_float4(0.f, 0.f, 0.f, 0.f);
      for (int r = 0; r < S; ++r) {
        const float4 v = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(prs, off + r * step, 0, 16));
        a.x += v.x; a.y += v.y; a.z += v.z; a.w += v.w;
      }
      *reinterpret_cast<float4*>(dbias + n) = a;
    }
  }
  if (tid == 0) __hip_atomic_store(&g_w2_cnt[cnt0 + tile], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// ------------------------------------------------------------------------------------------------
static int g_wg2 = 2;          // knob "wg2": 0 off, 1 = this kernel below the streaming-wgrad M, 2 = at every M (default: measured faster than both other kernels at every 7M shape but one, which ties)
static int g_wg2_blocks = 512;   // knob "wg2_blocks": workgroups the split-M plan aims for (round 4, 7M step, 30 steps: 512 16.32, 768 16.29, 1024 16.36-16.37, 1536 16.41 ms; round-6 re-sweep at 14.36 ms, three paired rounds: 512 14.308-14.326, 768 14.358-14.365, 1024 14.416-14.459 ms — profiles/r06_sweep.txt)
static int g_wg2_tile = 0;     // knob "wg2_tile": force the N edge (64 / 96 / 128 / 192; K edge 64 / 128)
static int g_wg2_conv = 1;     // knob "wg2_conv": 3x3 conv weight gradients (8 | C_in) on this kernel (0: tiled kernel)
void set_wg2_conv(int v) { g_wg2_conv = v ? 1 : 0; }
// knob "wg2_fuse": 1 = last-workgroup reduction in the kernel, 0 = the caller's colreduce (default).
// Measured and rejected as the default (tools/bench_wgrad.py, profiles/r03_wgrad_fuse.log, 7M step
// shapes): the split-M plan aims at ~1024 workgroups, so a tile has S = 29-1024 slabs and its last
// workgroup reads S x 16 KB serially -- per-step total 5.69 ms with colreduce vs 16.6 ms fused
// (10.2 ms at 256 workgroups); e.g. M = 524288, N = K = 48: 27 vs 402 us.  (A __threadfence()
// release / acquire in every workgroup, the first form tried, took the 7M step from 17.0 to 32.3 ms.)
static int g_wg2_fuse = 0;
void set_wg2_fuse(int v) { g_wg2_fuse = v ? 1 : 0; }

// A window of `tiles` arrival counters for one launch.  Windows are handed out round the ring in
// launch order, per device; a window is reused only W2_CNT counters later, by which time its
// previous user has finished (a step launches far fewer than W2_CNT tiles, and every launch that
// could still be running -- side streams, the branches of one captured graph -- holds a distinct
// window).  Returns -1 (no fused reduction) when a launch has more tiles than a ring share.
static int w2_counters(int tiles) {
  static long pos[64];
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64 || tiles > W2_CNT / 16) return -1;
  if (pos[dev] + tiles > W2_CNT) pos[dev] = 0;
  const int c = (int)pos[dev];
  pos[dev] += tiles;
  return c;
}
int wg2_mode() { return g_wg2; }
void set_wg2(int v) { g_wg2 = v < 0 ? 0 : (v > 2 ? 2 : v); }
void set_wg2_blocks(int v) { g_wg2_blocks = v < 64 ? 64 : v; }
void set_wg2_tile(int v) { g_wg2_tile = (v == 64 || v == 96 || v == 128 || v == 192) ? v : 0; }
// knob "wg2_pbeta" (percent; 0 = off): cap the slab count so the fp32 slab partials (written here, read back
// by the column reduction: S * (N*K + N) * 4 bytes each way) stay below beta x the launch's algorithmic
// operand bytes M * (N + K) * 2 -- at small M and wide layers (7M stage 3: M = 8192, N = K = 384) the ~768-
// workgroup target makes the partials 2x the operands; never below one workgroup per CU
static int g_wg2_pbeta = 0;
void set_wg2_pbeta(int v) { g_wg2_pbeta = v < 0 ? 0 : v; }

struct W2Plan {
  int ok = 0, BN = 0, BK = 0, nNt = 0, nKt = 0, S = 0, mchunk = 0;
};

// Tile edges (measured, tools/bench_wgrad.py over the 7M step's shapes, profiles/r03_wgrad_isolated.txt):
// 64 x 64 everywhere (3 workgroups per CU, the most tiles in flight), except a prologue operand
// with N <= 192, where one N tile covers all of G's columns so the X prologue runs once per element
// (N edge 96 / 128 / 192; X edge 64).
static void w2_tiles(int N, bool pro, int& BN, int& BK) {
  BN = BK = 64;
  if (pro && N > 64 && N <= 192) BN = N <= 96 ? 96 : (N <= 128 ? 128 : 192);
}

static W2Plan wgrad2_plan(int M, int N, int K, bool pro) {
  W2Plan p;
  if ((N & 7) || (K & 7) || M <= 0) return p;
  w2_tiles(N, pro, p.BN, p.BK);
  if (g_wg2_tile) {
    p.BN = g_wg2_tile;
    p.BK = g_wg2_tile == 128 ? 128 : 64;  // (N edges 96 / 192 pair with a 64-wide X edge)
  }
  p.nNt = (N + p.BN - 1) / p.BN;
  p.nKt = (K + p.BK - 1) / p.BK;
  const long tiles = (long)p.nNt * p.nKt;
  long S = (g_wg2_blocks + tiles - 1) / tiles;
  S = std::min<long>(S, ((long)M + 4 * W2_MS - 1) / (4 * W2_MS));  // >= 4 steps per workgroup
  if (g_wg2_pbeta > 0) {
    const double cap = g_wg2_pbeta * 0.01 * (double)M * (N + K) * 2.0 / (4.0 * ((double)N * K + N));
    const long floor_s = (256 + tiles - 1) / tiles;
    S = std::min<long>(S, std::max<long>((long)cap, floor_s));
  }
  S = std::max<long>(1, S);
  int mchunk = (int)((M + S - 1) / S);
  mchunk = (mchunk + W2_MS - 1) / W2_MS * W2_MS;
  p.S = (M + mchunk - 1) / mchunk;
  p.mchunk = mchunk;
  p.ok = 1;
  return p;
}

size_t wgrad2_ws_floats(int M, int N, int K) {
  // sized for the larger of the two tile plans (with / without a prologue), knob-independent of "wg2"
  size_t best = 0;
  for (bool pro : {false, true}) {
    const W2Plan p = wgrad2_plan(M, N, K, pro);
    if (!p.ok) continue;
    const long ld = (long)N * K + N;
    best = std::max(best, (size_t)p.S * ld + colreduce_tmp_floats(p.S, ld));
  }
  return best;
}

struct W2Out {
  float* part;
  long ldp;
  int cnt0;          // counter window, -1 = partials only
  float *dW, *dbias;
};

template <int BN, int BK, int PA, bool CV = false>
static void w2_launch(const W2Plan& p, const bf16* G, int ldg, const bf16* X, int ldx, const Pro& pro, const float* rs,
                      int rps, const W2Out& o, bool bias, int M, int N, int K, hipStream_t s, const ConvG& cv = ConvG()) {
  const int tiles = p.nNt * p.nKt;
  const unsigned grid = (unsigned)(((p.S + 7) / 8) * 8 * tiles);
  wgrad2_bf16_kernel<BN, BK, PA, CV><<<grid, W2_NT, 0, s>>>(G, ldg, X, ldx, pro, rs, rps, o.part, o.ldp, bias ? 1 : 0, M,
                                                            N, K, p.mchunk, p.nNt, tiles, p.S, o.cnt0, o.dW, o.dbias, cv);
}

template <int PA>
static void w2_dispatch(const W2Plan& p, const bf16* G, int ldg, const bf16* X, int ldx, const Pro& pro,
                        const float* rs, int rps, const W2Out& o, bool bias, int M, int N, int K, hipStream_t s) {
  // instantiated: 64 x 64, 96 x 64, 128 x 64, 192 x 64 and 128 x 128 (forced by wg2_tile=128 only)
  if (p.BN == 128 && p.BK == 128) w2_launch<128, 128, PA>(p, G, ldg, X, ldx, pro, rs, rps, o, bias, M, N, K, s);
  else if (p.BN == 64) w2_launch<64, 64, PA>(p, G, ldg, X, ldx, pro, rs, rps, o, bias, M, N, K, s);
  else if (p.BN == 96) w2_launch<96, 64, PA>(p, G, ldg, X, ldx, pro, rs, rps, o, bias, M, N, K, s);
  else if (p.BN == 128) w2_launch<128, 64, PA>(p, G, ldg, X, ldx, pro, rs, rps, o, bias, M, N, K, s);
  else w2_launch<192, 64, PA>(p, G, ldg, X, ldx, pro, rs, rps, o, bias, M, N, K, s);
}

// Returns the number of partial rows written into part (layout [S][N*K + N]), 0 if not handled.
// *reduced = true when the kernel also wrote dW (and dbias, when bias) itself: no colreduce needed.
// xc: X is a 3x3 convolution's gathered input (forward convs with 8 | Cs; 64 x 64 tiles, no prologue).
int wgrad2_try(const void* G, int ldg, const void* X, int ldx, const Pro& pro, const float* rs, int rps, float* part,
               float* dW, float* dbias, bool bias, int M, int N, int K, hipStream_t s, bool* reduced, const ConvG* xc) {
  *reduced = false;
  if (!g_wg2) return 0;
  if (xc) {
    if (!g_wg2_conv || xc->transposed || xc->par >= 0 || (xc->Cs & 7) || pro.any() || rs || (ldg & 7) ||
        (reinterpret_cast<uintptr_t>(G) & 15) || (reinterpret_cast<uintptr_t>(X) & 15) || (N & 7) || (K & 7))
      return 0;
    W2Plan p = wgrad2_plan(M, N, K, false);
    if (!p.ok || p.BN != 64 || p.BK != 64) return 0;
    const W2Out o{part, (long)N * K + N, -1, dW, dbias};
    w2_launch<64, 64, -1, true>(p, static_cast<const bf16*>(G), ldg, static_cast<const bf16*>(X), 0, pro, nullptr, 1, o,
                                bias, M, N, K, s, *xc);
    return p.S;
  }
  if ((ldg & 7) || (ldx & 7) || (reinterpret_cast<uintptr_t>(G) & 15) || (reinterpret_cast<uintptr_t>(X) & 15))
    return 0;
  W2Plan p = wgrad2_plan(M, N, K, pro.any());
  if (!p.ok) return 0;
  W2Out o{part, (long)N * K + N, -1, dW, dbias};
  if (g_wg2_fuse && dW && !(reinterpret_cast<uintptr_t>(dW) & 15) && !(reinterpret_cast<uintptr_t>(part) & 15) &&
      (!dbias || !(reinterpret_cast<uintptr_t>(dbias) & 15)) && (long)p.S * o.ldp * 4 < (1L << 31))
    o.cnt0 = w2_counters(p.nNt * p.nKt);
  const bf16* g = static_cast<const bf16*>(G);
  const bf16* x = static_cast<const bf16*>(X);
  const bool gelu_only = pro.act == OGV_ACT_GELU && !pro.sc && !pro.sh && !pro.gate;
  const bool bn_silu_gate = pro.act == OGV_ACT_SILU && pro.sc && pro.sh && pro.gate && !(pro.gld & 3);
  if (!pro.any()) w2_dispatch<-1>(p, g, ldg, x, ldx, pro, rs, rps, o, bias, M, N, K, s);
  else if (gelu_only) w2_dispatch<OGV_ACT_GELU>(p, g, ldg, x, ldx, pro, rs, rps, o, bias, M, N, K, s);
  else if (bn_silu_gate) w2_dispatch<OGV_ACT_SILU>(p, g, ldg, x, ldx, pro, rs, rps, o, bias, M, N, K, s);
  else w2_dispatch<W2_GENERIC>(p, g, ldg, x, ldx, pro, rs, rps, o, bias, M, N, K, s);
  *reduced = o.cnt0 >= 0;
  return p.S;
}

}  // namespace ogv
