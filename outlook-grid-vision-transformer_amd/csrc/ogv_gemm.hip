// Dense projection GEMMs of the hot path on MFMA (gfx950).
//
// Every 1x1 Conv2d / nn.Linear on the OutGridBlock path is out = A[M,K] . W[N,K]^T with M = B*H*W
// (hundreds of thousands of rows) and K, N <= 1024: tall-skinny and HBM-bound, so the kernel's
// job is to stream A once with full-width loads and to fuse what the reference does in separate
// ATen passes (bias, DropPath scale, residual add, activation of the producer's output, and the
// activation derivative in backward).
//
//   fwd   : out = res + rs[m/rps] * (act_in(A) . W^T + bias)
//   dgrad : dA  = act_in'(Z) * rs[m/rps] * (dOut . W)      (W^T staged once into the workspace)
//   wgrad : dW  = (rs*dOut)^T . act_in(A),  dbias = colsum(rs*dOut)   (split over M, fp32 slabs)
//
// bf16 operands use v_mfma_f32_16x16x32_bf16, fp32 operands the exact-f32 v_mfma_f32_16x16x4_f32.
// Block = 256 threads (4 waves in 2x2), tile BM x BN, BK = 32 (bf16) / 16 (fp32); the tile -> block
// map keeps all N-tiles of an M-panel on one XCD (blocks b and b+8 share an XCD) so the A panel is
// fetched from HBM once and re-read from that XCD's L2.
#include "ogv_common.h"

namespace ogv {

// ------------------------------------------------------------------------------------------------
// fwd / dgrad kernel, bf16
// ------------------------------------------------------------------------------------------------
template <int BM, int BN, int ACT>
__global__ __launch_bounds__(256) void gemm_bf16_kernel(const bf16* __restrict__ A, int lda,
                                                        const float* __restrict__ Wt, int ldw,
                                                        const float* __restrict__ bias, const bf16* __restrict__ res,
                                                        const float* __restrict__ rs, int rps,
                                                        const bf16* __restrict__ Z, int ldz, int zact,
                                                        bf16* __restrict__ out, int ldo, int M, int N, int K,
                                                        int Ka, int Kb, int nMt, int nNt) {
  // K: reduction length; Ka / Kb: valid reduction columns of A / W (zero beyond)
  constexpr int BK = 32;
  constexpr int PITCH = BK + 8;  // 80-byte rows: 16-B aligned fragment reads
  constexpr int WM = BM / 2, WN = BN / 2, TM = WM / 16, TN = WN / 16;
  constexpr int A_VECS = BM * BK / 8 / 256;
  constexpr int B_F4 = BN * BK / 4 / 256;
  __shared__ __attribute__((aligned(16))) bf16 As[BM * PITCH];
  __shared__ __attribute__((aligned(16))) bf16 Bs[BN * PITCH];

  const int bid = blockIdx.x;
  const int xcd = bid & 7, local = bid >> 3;
  const int mt = (local / nNt) * 8 + xcd, nt = local % nNt;
  if (mt >= nMt) return;
  const int m0 = mt * BM, n0 = nt * BN;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  uint4 ra[A_VECS];
  float4 rb[B_F4];
  const bool a_vec = ((lda & 7) == 0) && ((reinterpret_cast<uintptr_t>(A) & 15) == 0);
  const bool b_vec = ((ldw & 3) == 0) && ((reinterpret_cast<uintptr_t>(Wt) & 15) == 0);
  auto load_tile = [&](int k0) {
#pragma unroll
    for (int i = 0; i < A_VECS; ++i) {
      const int idx = tid + i * 256, row = idx / (BK / 8), kv = idx % (BK / 8);
      const int gm = m0 + row, gk = k0 + kv * 8;
      ra[i] = uint4{0u, 0u, 0u, 0u};
      if (gm < M) {
        const bf16* src = A + (long)gm * lda + gk;
        if (a_vec && gk + 8 <= Ka) {
          ra[i] = *reinterpret_cast<const uint4*>(src);
        } else {
          bf16* e = reinterpret_cast<bf16*>(&ra[i]);
#pragma unroll
          for (int q = 0; q < 8; ++q) e[q] = (gk + q < Ka) ? src[q] : (bf16)0.f;
        }
      }
    }
#pragma unroll
    for (int i = 0; i < B_F4; ++i) {
      const int idx = tid + i * 256, row = idx / (BK / 4), kq = idx % (BK / 4);
      const int gn = n0 + row, gk = k0 + kq * 4;
      rb[i] = float4{0.f, 0.f, 0.f, 0.f};
      if (gn < N) {
        const float* src = Wt + (long)gn * ldw + gk;
        if (b_vec && gk + 4 <= Kb) {
          rb[i] = *reinterpret_cast<const float4*>(src);
        } else {
          rb[i].x = gk < Kb ? src[0] : 0.f;
          rb[i].y = gk + 1 < Kb ? src[1] : 0.f;
          rb[i].z = gk + 2 < Kb ? src[2] : 0.f;
          rb[i].w = gk + 3 < Kb ? src[3] : 0.f;
        }
      }
    }
  };
  auto store_tile = [&]() {
#pragma unroll
    for (int i = 0; i < A_VECS; ++i) {
      const int idx = tid + i * 256, row = idx / (BK / 8), kv = idx % (BK / 8);
      uint4 v = ra[i];
      if constexpr (ACT != OGV_ACT_NONE) {
        bf16* e = reinterpret_cast<bf16*>(&v);
#pragma unroll
        for (int q = 0; q < 8; ++q) e[q] = (bf16)act_fwd(ACT, (float)e[q]);
      }
      *reinterpret_cast<uint4*>(As + row * PITCH + kv * 8) = v;
    }
#pragma unroll
    for (int i = 0; i < B_F4; ++i) {
      const int idx = tid + i * 256, row = idx / (BK / 4), kq = idx % (BK / 4);
      bf16x4 b = {(bf16)rb[i].x, (bf16)rb[i].y, (bf16)rb[i].z, (bf16)rb[i].w};
      *reinterpret_cast<bf16x4*>(Bs + row * PITCH + kq * 4) = b;
    }
  };

  load_tile(0);
  for (int k0 = 0; k0 < K; k0 += BK) {
    store_tile();
    __syncthreads();
    if (k0 + BK < K) load_tile(k0 + BK);  // next tile's HBM latency hides under this tile's MFMAs
    bf16x8 af[TM], bfg[TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
      af[i] = *reinterpret_cast<const bf16x8*>(As + (wm * WM + i * 16 + (lane & 15)) * PITCH + 8 * (lane >> 4));
#pragma unroll
    for (int j = 0; j < TN; ++j)
      bfg[j] = *reinterpret_cast<const bf16x8*>(Bs + (wn * WN + j * 16 + (lane & 15)) * PITCH + 8 * (lane >> 4));
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfg[j], acc[i][j], 0, 0, 0);
    __syncthreads();
  }

#pragma unroll
  for (int i = 0; i < TM; ++i) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int m = m0 + wm * WM + i * 16 + 4 * (lane >> 4) + r;
      if (m >= M) continue;
      const float sc = rs ? rs[m / rps] : 1.f;
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int n = n0 + wn * WN + j * 16 + (lane & 15);
        if (n >= N) continue;
        float v = acc[i][j][r];
        if (bias) v += bias[n];
        v *= sc;
        if (res) v += (float)res[(long)m * ldo + n];
        if (zact) v *= act_grad(zact, (float)Z[(long)m * ldz + n]);
        out[(long)m * ldo + n] = (bf16)v;
      }
    }
  }
}

// ------------------------------------------------------------------------------------------------
// fwd / dgrad kernel, fp32 (exact-f32 MFMA 16x16x4)
// ------------------------------------------------------------------------------------------------
template <int BM, int BN, int ACT>
__global__ __launch_bounds__(256) void gemm_f32_kernel(const float* __restrict__ A, int lda,
                                                       const float* __restrict__ Wt, int ldw,
                                                       const float* __restrict__ bias, const float* __restrict__ res,
                                                       const float* __restrict__ rs, int rps,
                                                       const float* __restrict__ Z, int ldz, int zact,
                                                       float* __restrict__ out, int ldo, int M, int N, int K,
                                                       int Ka, int Kb, int nMt, int nNt) {
  constexpr int BK = 16;
  constexpr int PITCH = BK + 1;
  constexpr int WM = BM / 2, WN = BN / 2, TM = WM / 16, TN = WN / 16;
  constexpr int A_F4 = BM * BK / 4 / 256;
  constexpr int B_F4 = BN * BK / 4 / 256;
  __shared__ float As[BM * PITCH];
  __shared__ float Bs[BN * PITCH];

  const int bid = blockIdx.x;
  const int xcd = bid & 7, local = bid >> 3;
  const int mt = (local / nNt) * 8 + xcd, nt = local % nNt;
  if (mt >= nMt) return;
  const int m0 = mt * BM, n0 = nt * BN;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  float4 ra[A_F4], rb[B_F4];
  const bool a_vec = ((lda & 3) == 0) && ((reinterpret_cast<uintptr_t>(A) & 15) == 0);
  const bool b_vec = ((ldw & 3) == 0) && ((reinterpret_cast<uintptr_t>(Wt) & 15) == 0);
  auto ld4 = [](const float* src, int gk, int lim, bool vec) {
    if (vec && gk + 4 <= lim) return *reinterpret_cast<const float4*>(src);
    float4 r;
    r.x = gk < lim ? src[0] : 0.f;
    r.y = gk + 1 < lim ? src[1] : 0.f;
    r.z = gk + 2 < lim ? src[2] : 0.f;
    r.w = gk + 3 < lim ? src[3] : 0.f;
    return r;
  };
  auto load_tile = [&](int k0) {
#pragma unroll
    for (int i = 0; i < A_F4; ++i) {
      const int idx = tid + i * 256, row = idx / (BK / 4), kq = idx % (BK / 4);
      const int gm = m0 + row, gk = k0 + kq * 4;
      ra[i] = float4{0.f, 0.f, 0.f, 0.f};
      if (gm < M) ra[i] = ld4(A + (long)gm * lda + gk, gk, Ka, a_vec);
    }
#pragma unroll
    for (int i = 0; i < B_F4; ++i) {
      const int idx = tid + i * 256, row = idx / (BK / 4), kq = idx % (BK / 4);
      const int gn = n0 + row, gk = k0 + kq * 4;
      rb[i] = float4{0.f, 0.f, 0.f, 0.f};
      if (gn < N) rb[i] = ld4(Wt + (long)gn * ldw + gk, gk, Kb, b_vec);
    }
  };
  auto store_tile = [&]() {
#pragma unroll
    for (int i = 0; i < A_F4; ++i) {
      const int idx = tid + i * 256, row = idx / (BK / 4), kq = idx % (BK / 4);
      float* d = As + row * PITCH + kq * 4;
      d[0] = act_fwd(ACT, ra[i].x); d[1] = act_fwd(ACT, ra[i].y);
      d[2] = act_fwd(ACT, ra[i].z); d[3] = act_fwd(ACT, ra[i].w);
    }
#pragma unroll
    for (int i = 0; i < B_F4; ++i) {
      const int idx = tid + i * 256, row = idx / (BK / 4), kq = idx % (BK / 4);
      float* d = Bs + row * PITCH + kq * 4;
      d[0] = rb[i].x; d[1] = rb[i].y; d[2] = rb[i].z; d[3] = rb[i].w;
    }
  };

  load_tile(0);
  for (int k0 = 0; k0 < K; k0 += BK) {
    store_tile();
    __syncthreads();
    if (k0 + BK < K) load_tile(k0 + BK);
#pragma unroll
    for (int ks = 0; ks < BK; ks += 4) {
      float af[TM], bfg[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) af[i] = As[(wm * WM + i * 16 + (lane & 15)) * PITCH + ks + (lane >> 4)];
#pragma unroll
      for (int j = 0; j < TN; ++j) bfg[j] = Bs[(wn * WN + j * 16 + (lane & 15)) * PITCH + ks + (lane >> 4)];
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(af[i], bfg[j], acc[i][j], 0, 0, 0);
    }
    __syncthreads();
  }

#pragma unroll
  for (int i = 0; i < TM; ++i) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int m = m0 + wm * WM + i * 16 + 4 * (lane >> 4) + r;
      if (m >= M) continue;
      const float sc = rs ? rs[m / rps] : 1.f;
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int n = n0 + wn * WN + j * 16 + (lane & 15);
        if (n >= N) continue;
        float v = acc[i][j][r];
        if (bias) v += bias[n];
        v *= sc;
        if (res) v += res[(long)m * ldo + n];
        if (zact) v *= act_grad(zact, Z[(long)m * ldz + n]);
        out[(long)m * ldo + n] = v;
      }
    }
  }
}

// ------------------------------------------------------------------------------------------------
// wgrad, bf16: part[s][n][k] = sum_{m in chunk s} G[m,n] * act(X[m,k])   (G pre-scaled by rs)
// Tiles staged [m][col] as loaded; MFMA fragments (reduction index = m) come from
// ds_read_b64_tr_b16 transposed reads.  The m -> fragment-k map is permuted (j<4: m = 4g+j,
// j>=4: m = 16+4g+j-4) identically for both operands, which makes each 32-lane half read 8
// distinct rows: with an 80-element pitch the reads are bank-conflict free.
// ------------------------------------------------------------------------------------------------
template <int ACT>
__global__ __launch_bounds__(256) void wgrad_bf16_kernel(const bf16* __restrict__ G, int ldg, const bf16* __restrict__ X,
                                                         int ldx, const float* __restrict__ rs, int rps,
                                                         float* __restrict__ part, float* __restrict__ dbias_part,
                                                         int M, int N, int K, int mchunk, int nNt) {
  constexpr int BN = 64, BKK = 64, MS = 32, PITCH = 80;
  __shared__ __attribute__((aligned(16))) bf16 Gs[MS * PITCH];
  __shared__ __attribute__((aligned(16))) bf16 Xs[MS * PITCH];
  const int nt = blockIdx.x % nNt, kt = blockIdx.x / nNt;
  const int s = blockIdx.y;
  const int n0 = nt * BN, k0 = kt * BKK;
  const int mbeg = s * mchunk;
  const int mend = min(M, mbeg + mchunk);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wn = wave >> 1, wk = wave & 1;
  const bool do_bias = dbias_part != nullptr && kt == 0;

  f32x4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  float bsum = 0.f;

  const int srow = tid >> 3, scol = (tid & 7) * 8;
  const int g = lane >> 4, c16 = lane & 15, q = c16 >> 2, p4 = (c16 & 3) * 4;
  const bool g_vec = ((ldg & 7) == 0) && ((reinterpret_cast<uintptr_t>(G) & 15) == 0);
  const bool x_vec = ((ldx & 7) == 0) && ((reinterpret_cast<uintptr_t>(X) & 15) == 0);
  for (int m0 = mbeg; m0 < mend; m0 += MS) {
    {
      const int gm = m0 + srow;
      uint4 gv = uint4{0u, 0u, 0u, 0u}, xv = uint4{0u, 0u, 0u, 0u};
      if (gm < mend) {
        const bf16* gsrc = G + (long)gm * ldg + n0 + scol;
        const bf16* xsrc = X + (long)gm * ldx + k0 + scol;
        if (g_vec && n0 + scol + 8 <= N) gv = *reinterpret_cast<const uint4*>(gsrc);
        else {
          bf16* e = reinterpret_cast<bf16*>(&gv);
#pragma unroll
          for (int t = 0; t < 8; ++t) e[t] = (n0 + scol + t < N) ? gsrc[t] : (bf16)0.f;
        }
        if (x_vec && k0 + scol + 8 <= K) xv = *reinterpret_cast<const uint4*>(xsrc);
        else {
          bf16* e = reinterpret_cast<bf16*>(&xv);
#pragma unroll
          for (int t = 0; t < 8; ++t) e[t] = (k0 + scol + t < K) ? xsrc[t] : (bf16)0.f;
        }
        if (rs) {
          const float sc = rs[gm / rps];
          bf16* e = reinterpret_cast<bf16*>(&gv);
#pragma unroll
          for (int t = 0; t < 8; ++t) e[t] = (bf16)((float)e[t] * sc);
        }
        if constexpr (ACT != OGV_ACT_NONE) {
          bf16* e = reinterpret_cast<bf16*>(&xv);
#pragma unroll
          for (int t = 0; t < 8; ++t) e[t] = (bf16)act_fwd(ACT, (float)e[t]);
        }
      }
      *reinterpret_cast<uint4*>(Gs + srow * PITCH + scol) = gv;
      *reinterpret_cast<uint4*>(Xs + srow * PITCH + scol) = xv;
    }
    __syncthreads();
    if (do_bias && tid < BN) {
#pragma unroll 8
      for (int r = 0; r < MS; ++r) bsum += (float)Gs[r * PITCH + tid];
    }
    bf16x8 af[2], xf[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int col = wn * 32 + i * 16 + p4;
      typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
      s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(Gs + (4 * g + q) * PITCH + col));
      s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(Gs + (16 + 4 * g + q) * PITCH + col));
      const int colx = wk * 32 + i * 16 + p4;
      s16x4 xlo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(Xs + (4 * g + q) * PITCH + colx));
      s16x4 xhi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(Xs + (16 + 4 * g + q) * PITCH + colx));
      typedef __attribute__((ext_vector_type(8))) short s16x8;
      s16x8 a8 = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      s16x8 x8 = {xlo[0], xlo[1], xlo[2], xlo[3], xhi[0], xhi[1], xhi[2], xhi[3]};
      af[i] = __builtin_bit_cast(bf16x8, a8);
      xf[i] = __builtin_bit_cast(bf16x8, x8);
    }
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], xf[j], acc[i][j], 0, 0, 0);
    __syncthreads();
  }
  float* dst = part + (long)s * N * K;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int n = n0 + wn * 32 + i * 16 + 4 * g + r;
        const int k = k0 + wk * 32 + j * 16 + c16;
        if (n < N && k < K) dst[(long)n * K + k] = acc[i][j][r];
      }
  if (do_bias && tid < BN && n0 + tid < N) dbias_part[(long)s * N + n0 + tid] = bsum;
}

// wgrad, fp32: f32 MFMA fragments read straight from the [m][col] tiles (k = lane>>4 layout).
template <int ACT>
__global__ __launch_bounds__(256) void wgrad_f32_kernel(const float* __restrict__ G, int ldg, const float* __restrict__ X,
                                                        int ldx, const float* __restrict__ rs, int rps,
                                                        float* __restrict__ part, float* __restrict__ dbias_part,
                                                        int M, int N, int K, int mchunk, int nNt) {
  constexpr int BN = 64, BKK = 64, MS = 16, PITCH = 68;
  __shared__ __attribute__((aligned(16))) float Gs[MS * PITCH];
  __shared__ __attribute__((aligned(16))) float Xs[MS * PITCH];
  const int nt = blockIdx.x % nNt, kt = blockIdx.x / nNt;
  const int s = blockIdx.y;
  const int n0 = nt * BN, k0 = kt * BKK;
  const int mbeg = s * mchunk;
  const int mend = min(M, mbeg + mchunk);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wn = wave >> 1, wk = wave & 1;
  const bool do_bias = dbias_part != nullptr && kt == 0;

  f32x4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  float bsum = 0.f;
  const int srow = tid >> 4, scol = (tid & 15) * 4;
  const bool g_vec = ((ldg & 3) == 0) && ((reinterpret_cast<uintptr_t>(G) & 15) == 0);
  const bool x_vec = ((ldx & 3) == 0) && ((reinterpret_cast<uintptr_t>(X) & 15) == 0);
  for (int m0 = mbeg; m0 < mend; m0 += MS) {
    {
      const int gm = m0 + srow;
      float4 gv = float4{0.f, 0.f, 0.f, 0.f}, xv = float4{0.f, 0.f, 0.f, 0.f};
      if (gm < mend) {
        const float* gsrc = G + (long)gm * ldg + n0 + scol;
        const float* xsrc = X + (long)gm * ldx + k0 + scol;
        if (g_vec && n0 + scol + 4 <= N) gv = *reinterpret_cast<const float4*>(gsrc);
        else {
          gv.x = n0 + scol < N ? gsrc[0] : 0.f; gv.y = n0 + scol + 1 < N ? gsrc[1] : 0.f;
          gv.z = n0 + scol + 2 < N ? gsrc[2] : 0.f; gv.w = n0 + scol + 3 < N ? gsrc[3] : 0.f;
        }
        if (x_vec && k0 + scol + 4 <= K) xv = *reinterpret_cast<const float4*>(xsrc);
        else {
          xv.x = k0 + scol < K ? xsrc[0] : 0.f; xv.y = k0 + scol + 1 < K ? xsrc[1] : 0.f;
          xv.z = k0 + scol + 2 < K ? xsrc[2] : 0.f; xv.w = k0 + scol + 3 < K ? xsrc[3] : 0.f;
        }
        if (rs) {
          const float sc = rs[gm / rps];
          gv.x *= sc; gv.y *= sc; gv.z *= sc; gv.w *= sc;
        }
        xv.x = act_fwd(ACT, xv.x); xv.y = act_fwd(ACT, xv.y);
        xv.z = act_fwd(ACT, xv.z); xv.w = act_fwd(ACT, xv.w);
      }
      *reinterpret_cast<float4*>(Gs + srow * PITCH + scol) = gv;
      *reinterpret_cast<float4*>(Xs + srow * PITCH + scol) = xv;
    }
    __syncthreads();
    if (do_bias && tid < BN) {
#pragma unroll
      for (int r = 0; r < MS; ++r) bsum += Gs[r * PITCH + tid];
    }
#pragma unroll
    for (int ks = 0; ks < MS; ks += 4) {
      float af[2], xf[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        af[i] = Gs[(ks + (lane >> 4)) * PITCH + wn * 32 + i * 16 + (lane & 15)];
        xf[i] = Xs[(ks + (lane >> 4)) * PITCH + wk * 32 + i * 16 + (lane & 15)];
      }
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(af[i], xf[j], acc[i][j], 0, 0, 0);
    }
    __syncthreads();
  }
  float* dst = part + (long)s * N * K;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int n = n0 + wn * 32 + i * 16 + 4 * (lane >> 4) + r;
        const int k = k0 + wk * 32 + j * 16 + (lane & 15);
        if (n < N && k < K) dst[(long)n * K + k] = acc[i][j][r];
      }
  if (do_bias && tid < BN && n0 + tid < N) dbias_part[(long)s * N + n0 + tid] = bsum;
}

// WT[k][n] = W[n][k]  (fp32, 32x32 tiles through LDS)
__global__ __launch_bounds__(256) void transpose_f32_kernel(const float* __restrict__ W, float* __restrict__ WT, int N,
                                                            int K, int ldt) {
  __shared__ float t[32][33];
  const int kb = blockIdx.x * 32, nb = blockIdx.y * 32;
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;
  for (int r = ty; r < 32; r += 8) {
    const int n = nb + r, k = kb + tx;
    t[r][tx] = (n < N && k < K) ? W[(long)n * K + k] : 0.f;
  }
  __syncthreads();
  for (int r = ty; r < 32; r += 8) {
    const int k = kb + r, n = nb + tx;
    if (k < K && n < ldt) WT[(long)k * ldt + n] = t[tx][r];
  }
}

// ------------------------------------------------------------------------------------------------
// host dispatch
// ------------------------------------------------------------------------------------------------
template <typename T, int BM, int BN, int ACT>
static void launch_mm(const void* A, int lda, const float* Wt, int ldw, const float* bias, const void* res,
                      const float* rs, int rps, const void* Z, int ldz, int zact, void* out, int ldo, int M, int N,
                      int K, int Ka, int Kb, hipStream_t s) {
  const int nMt = (M + BM - 1) / BM, nNt = (N + BN - 1) / BN;
  const unsigned grid = (unsigned)(((nMt + 7) / 8) * 8 * nNt);
  if constexpr (sizeof(T) == 2)
    gemm_bf16_kernel<BM, BN, ACT><<<grid, 256, 0, s>>>((const bf16*)A, lda, Wt, ldw, bias, (const bf16*)res, rs, rps,
                                                       (const bf16*)Z, ldz, zact, (bf16*)out, ldo, M, N, K, Ka, Kb, nMt, nNt);
  else
    gemm_f32_kernel<BM, BN, ACT><<<grid, 256, 0, s>>>((const float*)A, lda, Wt, ldw, bias, (const float*)res, rs, rps,
                                                      (const float*)Z, ldz, zact, (float*)out, ldo, M, N, K, Ka, Kb, nMt, nNt);
}

template <typename T, int ACT>
static void launch_mm_tiles(const void* A, int lda, const float* Wt, int ldw, const float* bias, const void* res,
                            const float* rs, int rps, const void* Z, int ldz, int zact, void* out, int ldo, int M,
                            int N, int K, hipStream_t s, int Ka = -1, int Kb = -1) {
  if (Ka < 0) Ka = K;
  if (Kb < 0) Kb = K;
  if (N > 64)
    launch_mm<T, 128, 128, ACT>(A, lda, Wt, ldw, bias, res, rs, rps, Z, ldz, zact, out, ldo, M, N, K, Ka, Kb, s);
  else
    launch_mm<T, 128, 64, ACT>(A, lda, Wt, ldw, bias, res, rs, rps, Z, ldz, zact, out, ldo, M, N, K, Ka, Kb, s);
}

template <typename T>
static void launch_mm_act(int act, const void* A, int lda, const float* Wt, int ldw, const float* bias,
                          const void* res, const float* rs, int rps, const void* Z, int ldz, int zact, void* out,
                          int ldo, int M, int N, int K, hipStream_t s) {
  switch (act) {
    case OGV_ACT_GELU:
      launch_mm_tiles<T, OGV_ACT_GELU>(A, lda, Wt, ldw, bias, res, rs, rps, Z, ldz, zact, out, ldo, M, N, K, s);
      break;
    case OGV_ACT_SILU:
      launch_mm_tiles<T, OGV_ACT_SILU>(A, lda, Wt, ldw, bias, res, rs, rps, Z, ldz, zact, out, ldo, M, N, K, s);
      break;
    case OGV_ACT_RELU:
      launch_mm_tiles<T, OGV_ACT_RELU>(A, lda, Wt, ldw, bias, res, rs, rps, Z, ldz, zact, out, ldo, M, N, K, s);
      break;
    default:
      launch_mm_tiles<T, OGV_ACT_NONE>(A, lda, Wt, ldw, bias, res, rs, rps, Z, ldz, zact, out, ldo, M, N, K, s);
  }
}

struct WgradPlan {
  int nNt, nKt, S, mchunk;
};
static WgradPlan wgrad_plan(int M, int N, int K, int ms) {
  WgradPlan p;
  p.nNt = (N + 63) / 64;
  p.nKt = (K + 63) / 64;
  const int tiles = p.nNt * p.nKt;
  int S = (1024 + tiles - 1) / tiles;
  const int max_s = (M + 1023) / 1024;  // keep >= ~1024 rows per chunk so the slab pass stays small
  if (S > max_s) S = max_s;
  if (S < 1) S = 1;
  int mchunk = (M + S - 1) / S;
  mchunk = (mchunk + ms - 1) / ms * ms;
  p.S = (M + mchunk - 1) / mchunk;
  p.mchunk = mchunk;
  return p;
}

static int check_common(int M, int N, int K, ogv_act act, ogv_dtype dt, const char* who) {
  OGV_REQUIRE(M >= 0 && N > 0 && K > 0, "%s: bad shape M=%d N=%d K=%d", who, M, N, K);
  OGV_REQUIRE(dt == OGV_F32 || dt == OGV_BF16, "%s: bad dtype", who);
  OGV_REQUIRE(act >= OGV_ACT_NONE && act <= OGV_ACT_RELU, "%s: bad activation", who);
  return OGV_OK;
}

}  // namespace ogv

using namespace ogv;

extern "C" int ogv_gemm_fwd(const void* A, int lda, const float* W, const float* bias, const void* res,
                            const float* rs, int rps, void* out, int ldo, int M, int N, int K, ogv_act act_in,
                            ogv_dtype dt, void* stream) {
  int rc = check_common(M, N, K, act_in, dt, "ogv_gemm_fwd");
  if (rc) return rc;
  OGV_REQUIRE(A && W && out, "ogv_gemm_fwd: null pointer");
  OGV_REQUIRE(lda >= K, "ogv_gemm_fwd: lda %d < K %d", lda, K);
  OGV_REQUIRE(ldo >= N, "ogv_gemm_fwd: ldo %d < N %d", ldo, N);
  OGV_REQUIRE(!rs || rps > 0, "ogv_gemm_fwd: rows-per-sample must be > 0 with a row scale");
  if (M == 0) return OGV_OK;
  hipStream_t s = as_stream(stream);
  if (dt == OGV_BF16)
    launch_mm_act<bf16>(act_in, A, lda, W, K, bias, res, rs, rps, nullptr, 0, 0, out, ldo, M, N, K, s);
  else
    launch_mm_act<float>(act_in, A, lda, W, K, bias, res, rs, rps, nullptr, 0, 0, out, ldo, M, N, K, s);
  return check_launch("ogv_gemm_fwd");
}

static inline int pad8(int n) { return (n + 7) / 8 * 8; }
extern "C" size_t ogv_gemm_dgrad_ws_bytes(int N, int K) { return (size_t)pad8(N) * K * sizeof(float); }

extern "C" int ogv_gemm_dgrad(const void* dout, int ldd, const float* W, const void* Z, int ldz, const float* rs,
                              int rps, void* dA, int lda, int M, int N, int K, ogv_act act_in, void* ws, ogv_dtype dt,
                              void* stream) {
  int rc = check_common(M, N, K, act_in, dt, "ogv_gemm_dgrad");
  if (rc) return rc;
  OGV_REQUIRE(dout && W && dA && ws, "ogv_gemm_dgrad: null pointer");
  OGV_REQUIRE(act_in == OGV_ACT_NONE || Z, "ogv_gemm_dgrad: activation derivative needs Z");
  OGV_REQUIRE(ldd >= N, "ogv_gemm_dgrad: ldd %d < N %d", ldd, N);
  OGV_REQUIRE(lda >= K, "ogv_gemm_dgrad: lda %d < K %d", lda, K);
  OGV_REQUIRE(!rs || rps > 0, "ogv_gemm_dgrad: rows-per-sample must be > 0 with a row scale");
  if (M == 0) return OGV_OK;
  hipStream_t s = as_stream(stream);
  float* WT = (float*)ws;  // [K][Np], zero beyond N
  const int Np = pad8(N);
  dim3 tg(cdiv(K, 32), cdiv(Np, 32));
  transpose_f32_kernel<<<tg, 256, 0, s>>>(W, WT, N, K, Np);
  // dA[M,K] = dout[M,N] . WT[K,N]^T, epilogue: * rs, * act'(Z)
  if (dt == OGV_BF16)
    launch_mm_tiles<bf16, OGV_ACT_NONE>(dout, ldd, WT, Np, nullptr, nullptr, rs, rps, Z, ldz, (int)act_in, dA, lda, M,
                                        K, Np, s, N, Np);
  else
    launch_mm_tiles<float, OGV_ACT_NONE>(dout, ldd, WT, Np, nullptr, nullptr, rs, rps, Z, ldz, (int)act_in, dA, lda,
                                         M, K, Np, s, N, Np);
  return check_launch("ogv_gemm_dgrad");
}

extern "C" size_t ogv_gemm_wgrad_ws_bytes(int M, int N, int K) {
  WgradPlan p = wgrad_plan(M > 0 ? M : 1, N, K, 32);
  const size_t t1 = colreduce_tmp_floats(p.S, (long)N * K), t2 = colreduce_tmp_floats(p.S, N);
  return ((size_t)p.S * ((size_t)N * K + N) + (t1 > t2 ? t1 : t2)) * sizeof(float);
}

extern "C" int ogv_gemm_wgrad(const void* dout, int ldd, const void* A, int lda, const float* rs, int rps, float* dW,
                              float* dbias, int M, int N, int K, ogv_act act_in, void* ws, ogv_dtype dt,
                              void* stream) {
  int rc = check_common(M, N, K, act_in, dt, "ogv_gemm_wgrad");
  if (rc) return rc;
  OGV_REQUIRE(dout && A && dW && ws, "ogv_gemm_wgrad: null pointer");
  OGV_REQUIRE(ldd >= N && lda >= K, "ogv_gemm_wgrad: ldd/lda smaller than N/K");
  OGV_REQUIRE(!rs || rps > 0, "ogv_gemm_wgrad: rows-per-sample must be > 0 with a row scale");
  hipStream_t s = as_stream(stream);
  if (M == 0) {
    (void)hipMemsetAsync(dW, 0, (size_t)N * K * sizeof(float), s);
    if (dbias) (void)hipMemsetAsync(dbias, 0, (size_t)N * sizeof(float), s);
    return check_launch("ogv_gemm_wgrad");
  }
  // plan with the same row granularity used by the size query (32)
  WgradPlan p = wgrad_plan(M, N, K, 32);
  float* part = (float*)ws;
  float* bpart = part + (size_t)p.S * N * K;
  dim3 grid(p.nNt * p.nKt, p.S);
  if (dt == OGV_BF16) {
    switch (act_in) {
      case OGV_ACT_GELU:
        wgrad_bf16_kernel<OGV_ACT_GELU><<<grid, 256, 0, s>>>((const bf16*)dout, ldd, (const bf16*)A, lda, rs, rps, part,
                                                             dbias ? bpart : nullptr, M, N, K, p.mchunk, p.nNt);
        break;
      case OGV_ACT_SILU:
        wgrad_bf16_kernel<OGV_ACT_SILU><<<grid, 256, 0, s>>>((const bf16*)dout, ldd, (const bf16*)A, lda, rs, rps, part,
                                                             dbias ? bpart : nullptr, M, N, K, p.mchunk, p.nNt);
        break;
      case OGV_ACT_RELU:
        wgrad_bf16_kernel<OGV_ACT_RELU><<<grid, 256, 0, s>>>((const bf16*)dout, ldd, (const bf16*)A, lda, rs, rps, part,
                                                             dbias ? bpart : nullptr, M, N, K, p.mchunk, p.nNt);
        break;
      default:
        wgrad_bf16_kernel<OGV_ACT_NONE><<<grid, 256, 0, s>>>((const bf16*)dout, ldd, (const bf16*)A, lda, rs, rps, part,
                                                             dbias ? bpart : nullptr, M, N, K, p.mchunk, p.nNt);
    }
  } else {
    switch (act_in) {
      case OGV_ACT_GELU:
        wgrad_f32_kernel<OGV_ACT_GELU><<<grid, 256, 0, s>>>((const float*)dout, ldd, (const float*)A, lda, rs, rps, part,
                                                            dbias ? bpart : nullptr, M, N, K, p.mchunk, p.nNt);
        break;
      case OGV_ACT_SILU:
        wgrad_f32_kernel<OGV_ACT_SILU><<<grid, 256, 0, s>>>((const float*)dout, ldd, (const float*)A, lda, rs, rps, part,
                                                            dbias ? bpart : nullptr, M, N, K, p.mchunk, p.nNt);
        break;
      case OGV_ACT_RELU:
        wgrad_f32_kernel<OGV_ACT_RELU><<<grid, 256, 0, s>>>((const float*)dout, ldd, (const float*)A, lda, rs, rps, part,
                                                            dbias ? bpart : nullptr, M, N, K, p.mchunk, p.nNt);
        break;
      default:
        wgrad_f32_kernel<OGV_ACT_NONE><<<grid, 256, 0, s>>>((const float*)dout, ldd, (const float*)A, lda, rs, rps, part,
                                                            dbias ? bpart : nullptr, M, N, K, p.mchunk, p.nNt);
    }
  }
  const long len = (long)N * K;
  float* tmp = bpart + (size_t)p.S * N;
  colreduce(part, dW, p.S, len, len, tmp, s);
  if (dbias) colreduce(bpart, dbias, p.S, N, N, tmp, s);
  return check_launch("ogv_gemm_wgrad");
}
