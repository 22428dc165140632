// Dense projection GEMMs of the hot path on MFMA (gfx950).
//
// Every 1x1 Conv2d / nn.Linear on the OutGridBlock path is out = A[M,K] . W[N,K]^T with M = B*H*W
// (hundreds of thousands of rows) and K, N <= 1024: tall-skinny and HBM-bound, so the kernel's
// job is to stream A once with full-width loads and to fuse what the reference does in separate
// ATen passes: bias, DropPath scale and residual add in the epilogue; the activation of the
// producer's output (and, for MBConv, BatchNorm-apply + SiLU + the SE gate) in the A prologue;
// the activation derivative in the backward epilogue; BatchNorm batch statistics of the output.
//
//   fwd   : out = res + rs[m/rps] * (pro(A) . W^T + bias)      [+ per-column stats of out]
//   dgrad : dA  = act'(Z) * rs[m/rps] * (dOut . W) (+ res)     (W^T staged once into the workspace)
//   wgrad : dW  = (rs*dOut)^T . pro(X),  dbias = colsum(rs*dOut)  (split over M, fp32 slabs)
//
// bf16 operands use v_mfma_f32_16x16x32_bf16, fp32 operands the exact-f32 v_mfma_f32_16x16x4_f32.
// Block = 256 threads (4 waves in 2x2), tile 128 x BN, BK = 32 (bf16) / 16 (fp32); the tile ->
// block map keeps all N-tiles of an M-panel on one XCD (blocks b and b+8 share an XCD) so the A
// panel is fetched from HBM once and re-read from that XCD's L2.
#include "ogv_gemm.h"

namespace ogv {

// Column statistics of a wave's accumulator tile -> per-panel partials (deterministic).
// Each thread holds rows 4*(lane>>4)+r (+16*i) of columns (lane&15) (+16*j); sums over its rows,
// then across the 4 lane groups (xor 16, 32), then across the two M-waves through LDS.
template <int TN, int WN, int BN>
__device__ __forceinline__ void stats_store(double (&s1)[TN], double (&s2)[TN], double* lds, int wm, int wn,
                                            int lane, double* stat, int mt, int n0, int N) {
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    s1[j] += __shfl_xor(s1[j], 16, 64);
    s1[j] += __shfl_xor(s1[j], 32, 64);
    s2[j] += __shfl_xor(s2[j], 16, 64);
    s2[j] += __shfl_xor(s2[j], 32, 64);
  }
  __syncthreads();  // LDS tiles are dead: reuse them
  if (lane < 16) {
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int c = wn * WN + j * 16 + lane;
      lds[(wm * 2 + 0) * BN + c] = s1[j];
      lds[(wm * 2 + 1) * BN + c] = s2[j];
    }
  }
  __syncthreads();
  if (wm == 0 && lane < 16) {
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int c = wn * WN + j * 16 + lane;
      const int n = n0 + c;
      if (n < N) {
        stat[((long)mt * 2 + 0) * N + n] = lds[0 * BN + c] + lds[2 * BN + c];
        stat[((long)mt * 2 + 1) * N + n] = lds[1 * BN + c] + lds[3 * BN + c];
      }
    }
  }
}

// Row-contiguous epilogue for the bf16 kernels.  The MFMA C fragment gives each lane one column
// of 4 rows, so storing straight from registers means 2-byte scattered stores (and 2-byte
// residual / Z loads).  Instead each wave stages its accumulator 16 rows at a time through LDS
// (fp32, pitch WN+4) and re-reads it as 8-column runs: LPR = WN/8 lanes per row, 16-byte loads of
// res / Z and 16-byte stores of out.  Per-column batch statistics follow the same mapping
// (8 columns per lane), reduced over lanes sharing columns, then over the two M-waves.
template <int TM, int TN, int WM, int WN, bool STATS>
__device__ __forceinline__ void gemm_epilogue_bf16(f32x4 (&acc)[TM][TN], float* stage_all, const Epi& epi,
                                                   bf16* __restrict__ out, int ldo, int M, int N, int m0, int n0,
                                                   int mt, int wm, int wn, int wave, int lane) {
  constexpr int SP = WN + 4, LPR = WN / 8, RPP = 64 / LPR, PASSES = 16 / RPP;
  float* stage = stage_all + wave * 16 * SP;
  const bf16* res = static_cast<const bf16*>(epi.res);
  const bf16* Z = static_cast<const bf16*>(epi.Z);
  const int c8 = (lane % LPR) * 8, rr0 = lane / LPR;
  const int n = n0 + wn * WN + c8;
  const bool full = n + 8 <= N;
  const bool vec = full && (ldo & 7) == 0 && (reinterpret_cast<uintptr_t>(out) & 15) == 0 &&
                   (!res || (reinterpret_cast<uintptr_t>(res) & 15) == 0) &&
                   (!epi.zact || ((epi.ldz & 7) == 0 && (reinterpret_cast<uintptr_t>(Z) & 15) == 0));
  float bias[8], shift[8];
  double s1[8], s2[8];
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    bias[q] = (epi.bias && n + q < N) ? epi.bias[n + q] : 0.f;
    shift[q] = (STATS && epi.stat_shift && n + q < N) ? bn_shift(epi.stat_shift[n + q]) : 0.f;
    s1[q] = 0.0;
    s2[q] = 0.0;
  }
  __syncthreads();  // main-loop LDS tiles are dead
#pragma unroll
  for (int i = 0; i < TM; ++i) {
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) stage[(4 * (lane >> 4) + r) * SP + j * 16 + (lane & 15)] = acc[i][j][r];
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
    for (int ps = 0; ps < PASSES; ++ps) {
      const int rr = rr0 + ps * RPP;
      const int m = m0 + wm * (TM * 16) + i * 16 + rr;
      if (m < M && n < N) {
        float v[8];
        const float4 lo = *reinterpret_cast<const float4*>(stage + rr * SP + c8);
        const float4 hi = *reinterpret_cast<const float4*>(stage + rr * SP + c8 + 4);
        v[0] = lo.x; v[1] = lo.y; v[2] = lo.z; v[3] = lo.w;
        v[4] = hi.x; v[5] = hi.y; v[6] = hi.z; v[7] = hi.w;
        const float sc = epi.rs ? epi.rs[m / epi.rps] : 1.f;
#pragma unroll
        for (int q = 0; q < 8; ++q) v[q] = (v[q] + bias[q]) * sc;
        const long o = (long)m * ldo + n;
        bf16 ob[8];
        if (vec) {
          if (res) {
            float t[8];
            load_vec<bf16, 8>(res + o, t);
#pragma unroll
            for (int q = 0; q < 8; ++q) v[q] += t[q];
          }
          if (epi.zact) {
            float t[8];
            load_vec<bf16, 8>(Z + (long)m * epi.ldz + n, t);
#pragma unroll
            for (int q = 0; q < 8; ++q) v[q] *= act_grad(epi.zact, t[q]);
          }
#pragma unroll
          for (int q = 0; q < 8; ++q) {
            ob[q] = (bf16)v[q];
            v[q] = (float)ob[q];
          }
          store_vec<bf16, 8>(out + o, v);
          if (epi.aout) {
            float a[8];
#pragma unroll
            for (int q = 0; q < 8; ++q) a[q] = act_fwd(epi.aact, v[q]);
            store_vec<bf16, 8>(static_cast<bf16*>(epi.aout) + (long)m * epi.ldao + n, a);
          }
        } else {
#pragma unroll
          for (int q = 0; q < 8; ++q) {
            if (n + q >= N) { ob[q] = (bf16)0.f; continue; }
            if (res) v[q] += (float)res[o + q];
            if (epi.zact) v[q] *= act_grad(epi.zact, (float)Z[(long)m * epi.ldz + n + q]);
            ob[q] = (bf16)v[q];
            out[o + q] = ob[q];
            if (epi.aout)
              static_cast<bf16*>(epi.aout)[(long)m * epi.ldao + n + q] = (bf16)act_fwd(epi.aact, (float)ob[q]);
          }
        }
        if constexpr (STATS) {
#pragma unroll
          for (int q = 0; q < 8; ++q) {
            const double d = n + q < N ? (double)(float)ob[q] - (double)shift[q] : 0.0;
            s1[q] += d;
            s2[q] = fma(d, d, s2[q]);
          }
        }
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  }
  if constexpr (STATS) {
#pragma unroll
    for (int q = 0; q < 8; ++q) {
#pragma unroll
      for (int o = LPR; o < 64; o <<= 1) {
        s1[q] += __shfl_xor(s1[q], o, 64);
        s2[q] += __shfl_xor(s2[q], o, 64);
      }
    }
    __syncthreads();
    // [wm][2][BN] partials; lanes < LPR hold their wave's column sums
    constexpr int BN = 2 * WN;
    double* red = reinterpret_cast<double*>(stage_all);  // 4 x BN doubles
    if (lane < LPR) {
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        red[(wm * 2 + 0) * BN + wn * WN + c8 + q] = s1[q];
        red[(wm * 2 + 1) * BN + wn * WN + c8 + q] = s2[q];
      }
    }
    __syncthreads();
    if (wm == 0 && lane < LPR) {
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const int c = wn * WN + c8 + q;
        if (n + q < N) {
          epi.stat[((long)mt * 2 + 0) * N + n + q] = red[0 * BN + c] + red[2 * BN + c];
          epi.stat[((long)mt * 2 + 1) * N + n + q] = red[1 * BN + c] + red[3 * BN + c];
        }
      }
    }
  }
}

// ------------------------------------------------------------------------------------------------
// fwd / dgrad kernel, bf16
// ------------------------------------------------------------------------------------------------
// BK = 32 or 64 reduction columns per k-step (64 halves the serial chain of dependent slab loads
// and barriers: the small-M shapes, whose K loop is latency-bound, use it).
// SW (split weights): the fp32 weight w is staged as two bf16 tiles, hi = bf16(w) and
// lo = bf16(w - hi), and every A fragment meets both (two MFMAs): the product carries ~16
// mantissa bits of the weight instead of 8, so the only bf16 rounding left on a projection is
// the activation's own storage.  The GEMMs are far below the MFMA ridge (HBM-bound), so the
// doubled matrix work is nearly free; it halves the bf16 model's logit error.
template <int BM, int BN, bool PRO, bool STATS, int AM = 0, bool BT = false, int BK = 32, bool SW = false>
__global__ __launch_bounds__(256) void gemm_bf16_kernel(const bf16* __restrict__ A, int lda, Pro pro,
                                                        const float* __restrict__ Wt, int ldw, Epi epi,
                                                        bf16* __restrict__ out, int ldo, int M, int N, int K, int Ka,
                                                        int Kb, int nMt, int nNt, ConvG cv) {
  constexpr int PITCH = BK + 8;  // 80 / 144-byte rows: 16-B aligned fragment reads
  constexpr int WM = BM / 2, WN = BN / 2, TM = WM / 16, TN = WN / 16;
  constexpr int A_VECS = BM * BK / 8 / 256;
  constexpr int B_F4 = BN * BK / 4 / 256;
  constexpr int SP = WN + 4;  // epilogue staging pitch (floats)
  constexpr int B_ELEMS = (BT && BK * (BN + 16) > BN * PITCH) ? BK * (BN + 16) : BN * PITCH;
  constexpr int MAIN_BYTES = (BM * PITCH + B_ELEMS * (SW ? 2 : 1)) * 2, EPI_BYTES = 4 * 16 * SP * 4;
  __shared__ __attribute__((aligned(16))) char smem[MAIN_BYTES > EPI_BYTES ? MAIN_BYTES : EPI_BYTES];
  bf16* As = reinterpret_cast<bf16*>(smem);
  bf16* Bs = As + BM * PITCH;
  bf16* Bl = Bs + B_ELEMS;  // SW: the lo tile, same layout

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
  // prologue parameters of the staged A chunks, fetched with the tile (not by the staging pass,
  // whose own loads would wait behind the next tile's prefetch): this thread's k chunk is the same
  // for all its A_VECS rows (256 % (BK/8) == 0)
  constexpr bool PV = PRO && AM == 0;
  float psc[PV ? 8 : 1], psh[PV ? 8 : 1], pgt[PV ? A_VECS : 1][8];
  bool pvec = false;
  const bool a_vec = ((lda & 7) == 0) && ((reinterpret_cast<uintptr_t>(A) & 15) == 0);
  const bool b_vec = ((ldw & 3) == 0) && ((reinterpret_cast<uintptr_t>(Wt) & 15) == 0);
  ConvRow crow[AM ? A_VECS : 1];
  const bool c_vec = AM && (cv.Cs & 7) == 0 && ((reinterpret_cast<uintptr_t>(A) & 15) == 0);
  if constexpr (AM != 0) {
#pragma unroll
    for (int i = 0; i < A_VECS; ++i) {
      const int gm = m0 + (tid + i * 256) / (BK / 8);
      crow[i] = conv_row(cv, gm < M ? gm : 0);  // rows are fixed per thread across the K loop
    }
  }
  auto load_tile = [&](int k0) {
#pragma unroll
    for (int i = 0; i < A_VECS; ++i) {
      const int idx = tid + i * 256, row = idx / (BK / 8), kv = idx % (BK / 8);
      const int gm = m0 + row, gk = k0 + kv * 8;
      ra[i] = uint4{0u, 0u, 0u, 0u};
      if constexpr (AM != 0) {
        if (gm < M && gk < Ka) {
          if (c_vec) {
            const int tap = gk / cv.Cs;
            const long off = conv_src(cv, crow[i], tap);
            if (off >= 0) ra[i] = *reinterpret_cast<const uint4*>(A + off + (gk - tap * cv.Cs));
          } else {
            bf16* e = reinterpret_cast<bf16*>(&ra[i]);
#pragma unroll
            for (int q = 0; q < 8; ++q) {
              const int k = gk + q, tap = k / cv.Cs;
              const long off = k < Ka ? conv_src(cv, crow[i], tap) : -1;
              e[q] = off >= 0 ? A[off + (k - tap * cv.Cs)] : (bf16)0.f;
            }
          }
        }
        continue;
      }
      if constexpr (PV) {
        if (i == 0) {
          pvec = gk + 8 <= Ka && (gk & 3) == 0 && (pro.gld & 3) == 0;
#pragma unroll
          for (int t = 0; t < 8; ++t) { psc[t] = 1.f; psh[t] = 0.f; }
          if (pvec && pro.sc) load_vec<float, 8>(pro.sc + gk, psc);
          if (pvec && pro.sh) load_vec<float, 8>(pro.sh + gk, psh);
        }
        if (pvec && pro.gate && gm < M) load_vec<float, 8>(pro.gate + (long)(gm / pro.rps) * pro.gld + gk, pgt[i]);
      }
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
      if constexpr (BT) {  // W stored [reduction][output]: 4 consecutive output columns of one row
        const int idx = tid + i * 256, kr = idx / (BN / 4), nq = idx % (BN / 4);
        const int gk = k0 + kr, gn = n0 + nq * 4;
        rb[i] = float4{0.f, 0.f, 0.f, 0.f};
        if (gk < Kb) {
          const float* src = Wt + (long)gk * ldw + gn;
          if (b_vec && gn + 4 <= N) {
            rb[i] = *reinterpret_cast<const float4*>(src);
          } else {
            rb[i].x = gn < N ? src[0] : 0.f;
            rb[i].y = gn + 1 < N ? src[1] : 0.f;
            rb[i].z = gn + 2 < N ? src[2] : 0.f;
            rb[i].w = gn + 3 < N ? src[3] : 0.f;
          }
        }
        continue;
      }
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
  auto store_tile = [&](int k0) {
#pragma unroll
    for (int i = 0; i < A_VECS; ++i) {
      const int idx = tid + i * 256, row = idx / (BK / 8), kv = idx % (BK / 8);
      uint4 v = ra[i];
      if constexpr (PRO) {
        const int gm = m0 + row, gk = k0 + kv * 8;
        bf16* e = reinterpret_cast<bf16*>(&v);
        if (gm < M) {
          float f[8];
#pragma unroll
          for (int q = 0; q < 8; ++q) f[q] = (float)e[q];
          if constexpr (PV) {
            if (pvec) {
#pragma unroll
              for (int q = 0; q < 8; ++q) {
                f[q] = act_fwd(pro.act, fmaf(f[q], psc[q], psh[q]));
                if (pro.gate) f[q] *= pgt[i][q];
              }
            } else {
              pro_apply_run<8>(pro, f, gm, gk, Ka);
            }
          } else {
            pro_apply_run<8>(pro, f, gm, gk, Ka);
          }
#pragma unroll
          for (int q = 0; q < 8; ++q) e[q] = gk + q < Ka ? (bf16)f[q] : (bf16)0.f;
        }
      }
      *reinterpret_cast<uint4*>(As + row * PITCH + kv * 8) = v;
    }
#pragma unroll
    for (int i = 0; i < B_F4; ++i) {
      const int idx = tid + i * 256;
      // BT: stage as loaded, Bs[kr][n] (pitch BN+16), read back with transposed LDS reads
      const int off = BT ? (idx / (BN / 4)) * (BN + 16) + (idx % (BN / 4)) * 4
                         : (idx / (BK / 4)) * PITCH + (idx % (BK / 4)) * 4;
      bf16x4 b = {(bf16)rb[i].x, (bf16)rb[i].y, (bf16)rb[i].z, (bf16)rb[i].w};
      *reinterpret_cast<bf16x4*>(Bs + off) = b;
      if constexpr (SW) {
        bf16x4 l = {(bf16)(rb[i].x - (float)b[0]), (bf16)(rb[i].y - (float)b[1]), (bf16)(rb[i].z - (float)b[2]),
                    (bf16)(rb[i].w - (float)b[3])};
        *reinterpret_cast<bf16x4*>(Bl + off) = l;
      }
    }
  };

  load_tile(0);
  for (int k0 = 0; k0 < K; k0 += BK) {
    store_tile(k0);
    __syncthreads();
    if (k0 + BK < K) load_tile(k0 + BK);  // next tile's HBM latency hides under this tile's MFMAs
#pragma unroll
    for (int ks = 0; ks < BK; ks += 32) {
      bf16x8 af[TM], bfg[TN];
      if constexpr (BT) {
        // B fragments from the [k][n] tile via ds_read_b64_tr_b16: lane (g = lane>>4, c = lane&15) gets
        // column c at k = {4g..4g+3, 16+4g..16+4g+3}; A fragments are read in that same k order.
        typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
        typedef __attribute__((ext_vector_type(8))) short s16x8;
        const int g = lane >> 4, c16 = lane & 15, q = c16 >> 2, p4 = (c16 & 3) * 4;
#pragma unroll
        for (int i = 0; i < TM; ++i) {
          const bf16* arow = As + (wm * WM + i * 16 + c16) * PITCH + ks;
          const s16x4 lo = *reinterpret_cast<const s16x4*>(arow + 4 * g);
          const s16x4 hi = *reinterpret_cast<const s16x4*>(arow + 16 + 4 * g);
          const s16x8 a8 = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
          af[i] = __builtin_bit_cast(bf16x8, a8);
        }
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          const int col = wn * WN + j * 16 + p4;
          const s16x4 lo =
              __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(Bs + (ks + 4 * g + q) * (BN + 16) + col));
          const s16x4 hi =
              __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(Bs + (ks + 16 + 4 * g + q) * (BN + 16) + col));
          const s16x8 b8 = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
          bfg[j] = __builtin_bit_cast(bf16x8, b8);
        }
      } else {
#pragma unroll
        for (int i = 0; i < TM; ++i)
          af[i] = *reinterpret_cast<const bf16x8*>(As + (wm * WM + i * 16 + (lane & 15)) * PITCH + ks + 8 * (lane >> 4));
#pragma unroll
        for (int j = 0; j < TN; ++j)
          bfg[j] = *reinterpret_cast<const bf16x8*>(Bs + (wn * WN + j * 16 + (lane & 15)) * PITCH + ks + 8 * (lane >> 4));
      }
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfg[j], acc[i][j], 0, 0, 0);
      if constexpr (SW) {  // the lo tile: same fragment addresses, second MFMA per (i, j)
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          if constexpr (BT) {
            typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
            typedef __attribute__((ext_vector_type(8))) short s16x8;
            const int g = lane >> 4, c16 = lane & 15, q = c16 >> 2, p4 = (c16 & 3) * 4;
            const int col = wn * WN + j * 16 + p4;
            const s16x4 lo =
                __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(Bl + (ks + 4 * g + q) * (BN + 16) + col));
            const s16x4 hi =
                __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(Bl + (ks + 16 + 4 * g + q) * (BN + 16) + col));
            const s16x8 b8 = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
            bfg[j] = __builtin_bit_cast(bf16x8, b8);
          } else {
            bfg[j] = *reinterpret_cast<const bf16x8*>(Bl + (wn * WN + j * 16 + (lane & 15)) * PITCH + ks + 8 * (lane >> 4));
          }
        }
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfg[j], acc[i][j], 0, 0, 0);
      }
    }
    __syncthreads();
  }

  gemm_epilogue_bf16<TM, TN, WM, WN, STATS>(acc, reinterpret_cast<float*>(smem), epi, out, ldo, M, N, m0, n0, mt, wm,
                                             wn, wave, lane);
}

// ------------------------------------------------------------------------------------------------
// fwd / dgrad kernel, fp32 (exact-f32 MFMA 16x16x4)
// ------------------------------------------------------------------------------------------------
template <int BM, int BN, bool PRO, bool STATS, int AM = 0, bool BT = false>
__global__ __launch_bounds__(256) void gemm_f32_kernel(const float* __restrict__ A, int lda, Pro pro,
                                                       const float* __restrict__ Wt, int ldw, Epi epi,
                                                       float* __restrict__ out, int ldo, int M, int N, int K, int Ka,
                                                       int Kb, int nMt, int nNt, ConvG cv, int kc = 0) {
  if (kc > 0) {  // split-K: blockIdx.y owns columns [y*kc, y*kc + kc); raw partial to out[y]
    const int ofs = blockIdx.y * kc;
    A += ofs;
    Wt += BT ? (long)ofs * ldw : ofs;  // BT: the reduction index is W's row
    Ka = min(Ka - ofs, kc);
    Kb = min(Kb - ofs, kc);
    if (pro.sc) pro.sc += ofs;
    if (pro.sh) pro.sh += ofs;
    if (pro.gate) pro.gate += ofs;
    out += (long)blockIdx.y * M * ldo;
    K = kc;
  }
  constexpr int BK = 16;
  constexpr int PITCH = BK + 1;
  constexpr int WM = BM / 2, WN = BN / 2, TM = WM / 16, TN = WN / 16;
  constexpr int A_F4 = BM * BK / 4 / 256;
  constexpr int B_F4 = BN * BK / 4 / 256;
  constexpr int B_FLOATS = (BT && BK * (BN + 16) > BN * PITCH) ? BK * (BN + 16) : BN * PITCH;
  __shared__ __attribute__((aligned(16))) float As[BM * PITCH];
  __shared__ __attribute__((aligned(16))) float Bs[B_FLOATS];

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
  ConvRow crow[AM ? A_F4 : 1];
  const bool c_vec = AM && (cv.Cs & 3) == 0 && ((reinterpret_cast<uintptr_t>(A) & 15) == 0);
  if constexpr (AM != 0) {
#pragma unroll
    for (int i = 0; i < A_F4; ++i) {
      const int gm = m0 + (tid + i * 256) / (BK / 4);
      crow[i] = conv_row(cv, gm < M ? gm : 0);
    }
  }
  auto load_tile = [&](int k0) {
#pragma unroll
    for (int i = 0; i < A_F4; ++i) {
      const int idx = tid + i * 256, row = idx / (BK / 4), kq = idx % (BK / 4);
      const int gm = m0 + row, gk = k0 + kq * 4;
      ra[i] = float4{0.f, 0.f, 0.f, 0.f};
      if constexpr (AM != 0) {
        if (gm < M && gk < Ka) {
          if (c_vec) {
            const int tap = gk / cv.Cs;
            const long off = conv_src(cv, crow[i], tap);
            if (off >= 0) ra[i] = *reinterpret_cast<const float4*>(A + off + (gk - tap * cv.Cs));
          } else {
            float e[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) {
              const int k = gk + q, tap = k / cv.Cs;
              const long off = k < Ka ? conv_src(cv, crow[i], tap) : -1;
              e[q] = off >= 0 ? A[off + (k - tap * cv.Cs)] : 0.f;
            }
            ra[i] = make_float4(e[0], e[1], e[2], e[3]);
          }
        }
        continue;
      }
      if (gm < M) ra[i] = ld4(A + (long)gm * lda + gk, gk, Ka, a_vec);
    }
#pragma unroll
    for (int i = 0; i < B_F4; ++i) {
      if constexpr (BT) {  // W stored [reduction][output]
        const int idx = tid + i * 256, kr = idx / (BN / 4), nq = idx % (BN / 4);
        const int gk = k0 + kr, gn = n0 + nq * 4;
        rb[i] = float4{0.f, 0.f, 0.f, 0.f};
        if (gk < Kb) rb[i] = ld4(Wt + (long)gk * ldw + gn, gn, N, b_vec);
        continue;
      }
      const int idx = tid + i * 256, row = idx / (BK / 4), kq = idx % (BK / 4);
      const int gn = n0 + row, gk = k0 + kq * 4;
      rb[i] = float4{0.f, 0.f, 0.f, 0.f};
      if (gn < N) rb[i] = ld4(Wt + (long)gn * ldw + gk, gk, Kb, b_vec);
    }
  };
  auto store_tile = [&](int k0) {
#pragma unroll
    for (int i = 0; i < A_F4; ++i) {
      const int idx = tid + i * 256, row = idx / (BK / 4), kq = idx % (BK / 4);
      float v[4] = {ra[i].x, ra[i].y, ra[i].z, ra[i].w};
      if constexpr (PRO) {
        const int gm = m0 + row, gk = k0 + kq * 4;
        if (gm < M) {
          pro_apply_run<4>(pro, v, gm, gk, Ka);
#pragma unroll
          for (int q = 0; q < 4; ++q) v[q] = gk + q < Ka ? v[q] : 0.f;
        }
      }
      float* d = As + row * PITCH + kq * 4;
      d[0] = v[0]; d[1] = v[1]; d[2] = v[2]; d[3] = v[3];
    }
#pragma unroll
    for (int i = 0; i < B_F4; ++i) {
      if constexpr (BT) {  // Bs[kr][n], pitch BN+16 (the 16x16x4 B fragment reads [k][n] directly)
        const int idx = tid + i * 256, kr = idx / (BN / 4), nq = idx % (BN / 4);
        *reinterpret_cast<float4*>(Bs + kr * (BN + 16) + nq * 4) = rb[i];
        continue;
      }
      const int idx = tid + i * 256, row = idx / (BK / 4), kq = idx % (BK / 4);
      float* d = Bs + row * PITCH + kq * 4;
      d[0] = rb[i].x; d[1] = rb[i].y; d[2] = rb[i].z; d[3] = rb[i].w;
    }
  };

  load_tile(0);
  for (int k0 = 0; k0 < K; k0 += BK) {
    store_tile(k0);
    __syncthreads();
    if (k0 + BK < K) load_tile(k0 + BK);
#pragma unroll
    for (int ks = 0; ks < BK; ks += 4) {
      float af[TM], bfg[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) af[i] = As[(wm * WM + i * 16 + (lane & 15)) * PITCH + ks + (lane >> 4)];
#pragma unroll
      for (int j = 0; j < TN; ++j)
        bfg[j] = BT ? Bs[(ks + (lane >> 4)) * (BN + 16) + wn * WN + j * 16 + (lane & 15)]
                    : Bs[(wn * WN + j * 16 + (lane & 15)) * PITCH + ks + (lane >> 4)];
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(af[i], bfg[j], acc[i][j], 0, 0, 0);
    }
    __syncthreads();
  }

  const float* res = static_cast<const float*>(epi.res);
  const float* Z = static_cast<const float*>(epi.Z);
  double s1[TN], s2[TN];
#pragma unroll
  for (int j = 0; j < TN; ++j) { s1[j] = 0.0; s2[j] = 0.0; }
#pragma unroll
  for (int i = 0; i < TM; ++i) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int m = m0 + wm * WM + i * 16 + 4 * (lane >> 4) + r;
      if (m >= M) continue;
      const float sc = epi.rs ? epi.rs[m / epi.rps] : 1.f;
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int n = n0 + wn * WN + j * 16 + (lane & 15);
        if (n >= N) continue;
        float v = acc[i][j][r];
        if (epi.bias) v += epi.bias[n];
        v *= sc;
        if (res) v += res[(long)m * ldo + n];
        if (epi.zact) v *= act_grad(epi.zact, Z[(long)m * epi.ldz + n]);
        out[(long)m * ldo + n] = v;
        if constexpr (STATS) {
          const double d = (double)v - (double)(epi.stat_shift ? bn_shift(epi.stat_shift[n]) : 0.f);
          s1[j] += d;
          s2[j] = fma(d, d, s2[j]);
        }
      }
    }
  }
  if constexpr (STATS)
    stats_store<TN, WN, BN>(s1, s2, reinterpret_cast<double*>(As), wm, wn, lane, epi.stat, mt, n0, N);
}

// ------------------------------------------------------------------------------------------------
// wgrad, bf16: part[s][n][k] = sum_{m in chunk s} G[m,n] * pro(X)[m,k]   (G pre-scaled by rs)
// Tiles staged [m][col] as loaded; MFMA fragments (reduction index = m) come from
// ds_read_b64_tr_b16 transposed reads.  The m -> fragment-k map is permuted (j<4: m = 4g+j,
// j>=4: m = 16+4g+j-4) identically for both operands, which makes each 32-lane half read 8
// distinct rows: with an 80-element pitch the reads are bank-conflict free.
// ------------------------------------------------------------------------------------------------
template <int BN, int BK, bool PRO, int AM = 0>
__global__ __launch_bounds__(256) void wgrad_bf16_kernel(const bf16* __restrict__ G, int ldg, const bf16* __restrict__ X,
                                                         int ldx, Pro pro, const float* __restrict__ rs, int rps,
                                                         float* __restrict__ part, long ldp, int want_bias, int M, int N,
                                                         int K, int mchunk, int nNt, int tiles, int S, ConvG cv) {
  constexpr int MS = 32;
  constexpr int GP = BN + 16, XP = BK + 16;  // 16 * odd elements: conflict-free transposed reads
  constexpr int GV = MS * BN / 8 / 256, XV = MS * BK / 8 / 256;
  constexpr int GC = BN / 8, XC = BK / 8;  // 8-element chunks per staged row
  constexpr int TN = BN / 32, TK = BK / 32;
  __shared__ __attribute__((aligned(16))) bf16 Gs[MS * GP];
  __shared__ __attribute__((aligned(16))) bf16 Xs[MS * XP];
  // slab-major XCD map: all tiles of slab s run on XCD s % 8, so their re-reads of the slab's
  // G / X rows come from that XCD's L2
  const int b = blockIdx.x, xcd = b & 7, local = b >> 3;
  const int tile = local % tiles, s = (local / tiles) * 8 + xcd;
  if (s >= S) return;
  const int nt = tile % nNt, kt = tile / nNt;
  const int n0 = nt * BN, k0 = kt * BK;
  const int mbeg = s * mchunk;
  const int mend = min(M, mbeg + mchunk);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wn = wave >> 1, wk = wave & 1;
  const bool do_bias = want_bias && kt == 0;

  f32x4 acc[TN][TK];
#pragma unroll
  for (int i = 0; i < TN; ++i)
#pragma unroll
    for (int j = 0; j < TK; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  float bacc[8];
#pragma unroll
  for (int t = 0; t < 8; ++t) bacc[t] = 0.f;

  const int gc8 = (tid % GC) * 8, grow = tid / GC;
  const int xc8 = (tid % XC) * 8, xrow = tid / XC;
  const bool g_vec = ((ldg & 7) == 0) && ((reinterpret_cast<uintptr_t>(G) & 15) == 0) && n0 + gc8 + 8 <= N;
  const bool x_vec = ((ldx & 7) == 0) && ((reinterpret_cast<uintptr_t>(X) & 15) == 0) && k0 + xc8 + 8 <= K;
  uint4 gr[GV], xr[XV];
  // Everything the staging pass multiplies in is fetched with the tile (row scales, SE gate) or once
  // per block (per-column BN scale / shift): the staging pass issues no global load of its own, which
  // would otherwise wait behind the next tile's prefetch (vmcnt retires in issue order).
  float rsv[GV];
  const int pk = k0 + xc8;
  const bool pvec = PRO && pk + 8 <= K && (pk & 3) == 0 && (pro.gld & 3) == 0;
  float psc[8], psh[8], gtv[PRO ? XV : 1][8];
#pragma unroll
  for (int t = 0; t < 8; ++t) { psc[t] = 1.f; psh[t] = 0.f; }
  if constexpr (PRO) {
    if (pvec && pro.sc) load_vec<float, 8>(pro.sc + pk, psc);
    if (pvec && pro.sh) load_vec<float, 8>(pro.sh + pk, psh);
  }
  auto load = [&](int m0) {
#pragma unroll
    for (int i = 0; i < GV; ++i) {
      const int gm = m0 + grow + i * (256 / GC);
      gr[i] = uint4{0u, 0u, 0u, 0u};
      rsv[i] = 1.f;
      if (rs && gm < mend) rsv[i] = rs[gm / rps];
      if (gm < mend) {
        const bf16* src = G + (long)gm * ldg + n0 + gc8;
        if (g_vec) gr[i] = *reinterpret_cast<const uint4*>(src);
        else {
          bf16* e = reinterpret_cast<bf16*>(&gr[i]);
#pragma unroll
          for (int t = 0; t < 8; ++t) e[t] = (n0 + gc8 + t < N) ? src[t] : (bf16)0.f;
        }
      }
    }
#pragma unroll
    for (int i = 0; i < XV; ++i) {
      const int gm = m0 + xrow + i * (256 / XC);
      xr[i] = uint4{0u, 0u, 0u, 0u};
      if constexpr (AM != 0) {  // implicit-GEMM conv: X = gather(x), tap-major columns
        const int k = k0 + xc8;
        if (gm < mend && k < K) {
          const ConvRow cr = conv_row(cv, gm);
          if ((cv.Cs & 7) == 0 && ((reinterpret_cast<uintptr_t>(X) & 15) == 0)) {
            const int tap = k / cv.Cs;
            const long off = conv_src(cv, cr, tap);
            if (off >= 0) xr[i] = *reinterpret_cast<const uint4*>(X + off + (k - tap * cv.Cs));
          } else {
            bf16* e = reinterpret_cast<bf16*>(&xr[i]);
#pragma unroll
            for (int t = 0; t < 8; ++t) {
              const int kk = k + t, tap = kk / cv.Cs;
              const long off = kk < K ? conv_src(cv, cr, tap) : -1;
              e[t] = off >= 0 ? X[off + (kk - tap * cv.Cs)] : (bf16)0.f;
            }
          }
        }
        continue;
      }
      if constexpr (PRO) {
        if (pvec && pro.gate && gm < mend) load_vec<float, 8>(pro.gate + (long)(gm / pro.rps) * pro.gld + pk, gtv[i]);
      }
      if (gm < mend) {
        const bf16* src = X + (long)gm * ldx + k0 + xc8;
        if (x_vec) xr[i] = *reinterpret_cast<const uint4*>(src);
        else {
          bf16* e = reinterpret_cast<bf16*>(&xr[i]);
#pragma unroll
          for (int t = 0; t < 8; ++t) e[t] = (k0 + xc8 + t < K) ? src[t] : (bf16)0.f;
        }
      }
    }
  };
  auto stage = [&](int m0) {
#pragma unroll
    for (int i = 0; i < GV; ++i) {
      const int r = grow + i * (256 / GC);
      uint4 v = gr[i];
      bf16* e = reinterpret_cast<bf16*>(&v);
      if (rs && m0 + r < mend) {
#pragma unroll
        for (int t = 0; t < 8; ++t) e[t] = (bf16)((float)e[t] * rsv[i]);
      }
      if (do_bias) {
#pragma unroll
        for (int t = 0; t < 8; ++t) bacc[t] += (float)e[t];
      }
      *reinterpret_cast<uint4*>(Gs + r * GP + gc8) = v;
    }
#pragma unroll
    for (int i = 0; i < XV; ++i) {
      const int r = xrow + i * (256 / XC);
      uint4 v = xr[i];
      if constexpr (PRO) {
        const int gm = m0 + r;
        if (gm < mend) {
          bf16* e = reinterpret_cast<bf16*>(&v);
          float f[8];
#pragma unroll
          for (int t = 0; t < 8; ++t) f[t] = (float)e[t];
          if (pvec) {
#pragma unroll
            for (int t = 0; t < 8; ++t) {
              f[t] = act_fwd(pro.act, fmaf(f[t], psc[t], psh[t]));
              if (pro.gate) f[t] *= gtv[i][t];
            }
          } else {
            pro_apply_run<8>(pro, f, gm, k0 + xc8, K);
          }
#pragma unroll
          for (int t = 0; t < 8; ++t) e[t] = k0 + xc8 + t < K ? (bf16)f[t] : (bf16)0.f;
        }
      }
      *reinterpret_cast<uint4*>(Xs + r * XP + xc8) = v;
    }
  };

  const int g = lane >> 4, c16 = lane & 15, q = c16 >> 2, p4 = (c16 & 3) * 4;
  typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
  typedef __attribute__((ext_vector_type(8))) short s16x8;
  load(mbeg);
  for (int m0 = mbeg; m0 < mend; m0 += MS) {
    stage(m0);
    __syncthreads();
    if (m0 + MS < mend) load(m0 + MS);  // next rows' HBM latency hides under this step's MFMAs
    bf16x8 af[TN], xf[TK];
#pragma unroll
    for (int i = 0; i < TN; ++i) {
      const int col = wn * (BN / 2) + i * 16 + p4;
      s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(Gs + (4 * g + q) * GP + col));
      s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(Gs + (16 + 4 * g + q) * GP + col));
      s16x8 a8 = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      af[i] = __builtin_bit_cast(bf16x8, a8);
    }
#pragma unroll
    for (int j = 0; j < TK; ++j) {
      const int col = wk * (BK / 2) + j * 16 + p4;
      s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(Xs + (4 * g + q) * XP + col));
      s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(Xs + (16 + 4 * g + q) * XP + col));
      s16x8 x8 = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      xf[j] = __builtin_bit_cast(bf16x8, x8);
    }
#pragma unroll
    for (int i = 0; i < TN; ++i)
#pragma unroll
      for (int j = 0; j < TK; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], xf[j], acc[i][j], 0, 0, 0);
    __syncthreads();
  }
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
  if (do_bias) {
    // lanes sharing gc8 within the wave, then the 4 waves through LDS (Gs is free after the loop)
#pragma unroll
    for (int t = 0; t < 8; ++t)
#pragma unroll
      for (int o = GC; o < 64; o <<= 1) bacc[t] += __shfl_xor(bacc[t], o, 64);
    float* red = reinterpret_cast<float*>(Gs);  // 4 x BN floats <= MS * GP * 2 bytes
    if (lane < GC) {
#pragma unroll
      for (int t = 0; t < 8; ++t) red[wave * BN + gc8 + t] = bacc[t];
    }
    __syncthreads();
    if (tid < BN && n0 + tid < N)
      dst[(long)N * K + n0 + tid] = (red[tid] + red[BN + tid]) + (red[2 * BN + tid] + red[3 * BN + tid]);
  }
}

// wgrad, fp32: f32 MFMA fragments read straight from the [m][col] tiles (k = lane>>4 layout).
template <bool PRO, int AM = 0>
__global__ __launch_bounds__(256) void wgrad_f32_kernel(const float* __restrict__ G, int ldg, const float* __restrict__ X,
                                                        int ldx, Pro pro, const float* __restrict__ rs, int rps,
                                                        float* __restrict__ part, long ldp, int want_bias, int M,
                                                        int N, int K, int mchunk, int nNt, ConvG cv) {
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
  const bool do_bias = want_bias && kt == 0;

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
      float gv[4] = {0.f, 0.f, 0.f, 0.f}, xv[4] = {0.f, 0.f, 0.f, 0.f};
      if (gm < mend) {
        const float* gsrc = G + (long)gm * ldg + n0 + scol;
        const float* xsrc = X + (long)gm * ldx + k0 + scol;
        if (g_vec && n0 + scol + 4 <= N) {
          const float4 t = *reinterpret_cast<const float4*>(gsrc);
          gv[0] = t.x; gv[1] = t.y; gv[2] = t.z; gv[3] = t.w;
        } else {
#pragma unroll
          for (int t = 0; t < 4; ++t) gv[t] = n0 + scol + t < N ? gsrc[t] : 0.f;
        }
        if constexpr (AM != 0) {  // implicit-GEMM conv: X = gather(x), tap-major columns
          const ConvRow cr = conv_row(cv, gm);
#pragma unroll
          for (int t = 0; t < 4; ++t) {
            const int kk = k0 + scol + t, tap = kk / cv.Cs;
            const long off = kk < K ? conv_src(cv, cr, tap) : -1;
            xv[t] = off >= 0 ? X[off + (kk - tap * cv.Cs)] : 0.f;
          }
        } else if (x_vec && k0 + scol + 4 <= K) {
          const float4 t = *reinterpret_cast<const float4*>(xsrc);
          xv[0] = t.x; xv[1] = t.y; xv[2] = t.z; xv[3] = t.w;
        } else {
#pragma unroll
          for (int t = 0; t < 4; ++t) xv[t] = k0 + scol + t < K ? xsrc[t] : 0.f;
        }
        if (rs) {
          const float sc = rs[gm / rps];
#pragma unroll
          for (int t = 0; t < 4; ++t) gv[t] *= sc;
        }
        if constexpr (PRO) {
          pro_apply_run<4>(pro, xv, gm, k0 + scol, K);
#pragma unroll
          for (int t = 0; t < 4; ++t) xv[t] = k0 + scol + t < K ? xv[t] : 0.f;
        }
      }
      *reinterpret_cast<float4*>(Gs + srow * PITCH + scol) = make_float4(gv[0], gv[1], gv[2], gv[3]);
      *reinterpret_cast<float4*>(Xs + srow * PITCH + scol) = make_float4(xv[0], xv[1], xv[2], xv[3]);
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
  float* dst = part + (long)s * ldp;
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
  if (do_bias && tid < BN && n0 + tid < N) dst[(long)N * K + n0 + tid] = bsum;
}

// ------------------------------------------------------------------------------------------------
// Tiny GEMMs (the SE MLP: M = batch rows, fp32).  The MFMA kernels would launch a handful of
// 128-row blocks for these and run latency-bound.
// ------------------------------------------------------------------------------------------------
// Groups of G lanes per output (G = 4 / 16 / 64 chosen from K): the group reads one A row and
// one W row with coalesced loads, reduces with shuffles; lane 0 of the group runs the epilogue.
template <int G>
__global__ __launch_bounds__(256) void small_fwd_kernel(const float* __restrict__ A, int lda, Pro pro,
                                                        const float* __restrict__ Wt, int ldw, Epi epi,
                                                        float* __restrict__ out, int ldo, int M, int N, int Ka,
                                                        int Kb) {
  const long gid = ((long)blockIdx.x * blockDim.x + threadIdx.x) / G;
  const int j = threadIdx.x & (G - 1);
  const bool live = gid < (long)M * N;
  const int n = live ? (int)(gid % N) : 0, m = live ? (int)(gid / N) : 0;
  const int K = Ka < Kb ? Ka : Kb;
  const float* a = A + (long)m * lda;
  const float* w = Wt + (long)n * ldw;
  const bool p = pro.act != OGV_ACT_NONE || pro.sc || pro.sh || pro.gate;
  float acc0 = 0.f, acc1 = 0.f;
  int k = j;
  if (live) {
    for (; k + G < K; k += 2 * G) {
      const float x0 = a[k], x1 = a[k + G];
      acc0 = fmaf(p ? pro_apply(pro, x0, m, k) : x0, w[k], acc0);
      acc1 = fmaf(p ? pro_apply(pro, x1, m, k + G) : x1, w[k + G], acc1);
    }
    if (k < K) acc0 = fmaf(p ? pro_apply(pro, a[k], m, k) : a[k], w[k], acc0);
  }
  float v = group_sum<G>(acc0 + acc1);
  if (!live || j != 0) return;
  const float* res = static_cast<const float*>(epi.res);
  const float* Z = static_cast<const float*>(epi.Z);
  if (epi.bias) v += epi.bias[n];
  if (epi.rs) v *= epi.rs[m / epi.rps];
  if (res) v += res[(long)m * ldo + n];
  if (epi.zact) v *= act_grad(epi.zact, Z[(long)m * epi.ldz + n]);
  out[(long)m * ldo + n] = v;
}

// WT[k][n] = W[n][k]  (fp32, 32x32 tiles through LDS), zero for n in [N, ldt)
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
// internal launchers
// ------------------------------------------------------------------------------------------------
static int g_bm64_max_m = 16384;  // tuning knob "bm64_max_m": largest M using 64-row tiles
void set_bm64_max_m(int v) { g_bm64_max_m = v; }
static int g_bk64_max_m = 32768;  // tuning knob "bk64_max_m": largest M using 64-wide k-steps (0 = off)
void set_bk64_max_m(int v) { g_bk64_max_m = v; }
// Measured (tools/bench_sgemm.py, stages 2-3): 64-wide k-steps win for long reductions without a
// prologue / activation-derivative epilogue, and at the last stage for narrow outputs.
static bool use_bk64(int M, int K, int ncols, bool pro, bool zact) {
  if (M > g_bk64_max_m || pro || zact) return false;
  return K >= 512 || (M <= 8192 && K >= 256 && ncols <= 512);
}

// knob "split_w" (bit mask, default 1): bf16 GEMMs multiply by the weight's hi + lo bf16 halves
// (SW above) in the forward products (bit 0: projections, implicit-GEMM convs) and / or the data
// gradients (bit 1)
static int g_split_w = 1;
void set_split_w(int v) { g_split_w = v & 3; }
int split_w() { return g_split_w; }
// knob "skip" (timing what-if experiments only -- outputs are left unwritten): bit 1 panel GEMMs,
// 2 streaming GEMMs, 4 weight gradients (wgrad / swgrad launches), 8 MBConv depthwise kernels,
// 16 LayerNorm, 32 grid attention, 64 Outlooker aggregation
static int g_skip = 0;
int skip_mask() { return g_skip; }
void set_skip(int v) { g_skip = v; }
#define OGV_SW_LAUNCH(COND, KERN, grid, s, ...)  \
  do {                                           \
    if (COND) {                                  \
      constexpr bool SW_ = true;                 \
      auto k_ = KERN;                            \
      k_<<<(grid), 256, 0, (s)>>>(__VA_ARGS__);  \
    } else {                                     \
      constexpr bool SW_ = false;                \
      auto k_ = KERN;                            \
      k_<<<(grid), 256, 0, (s)>>>(__VA_ARGS__);  \
    }                                            \
  } while (0)

template <typename T, int BN, bool PRO, bool STATS, int BM = GEMM_BM>
static void launch_mm(const void* A, int lda, const Pro& pro, const float* Wt, int ldw, void* out, int ldo, int M,
                      int N, int K, int Ka, int Kb, const Epi& epi, hipStream_t s) {
  if constexpr (!STATS && BM == GEMM_BM) {
    // small M (the last stage, M = 8192): 64-row tiles double the blocks and the K-slabs in flight
    // (measured: a loss already at M = 32768, where W-tile reloads dominate)
    if (M <= g_bm64_max_m) {
      launch_mm<T, BN, PRO, STATS, 64>(A, lda, pro, Wt, ldw, out, ldo, M, N, K, Ka, Kb, epi, s);
      return;
    }
  }
  const int nMt = (M + BM - 1) / BM, nNt = (N + BN - 1) / BN;
  const unsigned grid = (unsigned)(((nMt + 7) / 8) * 8 * nNt);
  if constexpr (sizeof(T) == 2) {
    if constexpr (!PRO) {
      if (use_bk64(M, K, N, false, false)) {
        OGV_SW_LAUNCH(g_split_w & 1, (gemm_bf16_kernel<BM, BN, PRO, STATS, 0, false, 64, SW_>), grid, s,
                      (const bf16*)A, lda, pro, Wt, ldw, epi, (bf16*)out, ldo, M, N, K, Ka, Kb, nMt, nNt, ConvG());
        return;
      }
    }
    OGV_SW_LAUNCH(g_split_w & 1, (gemm_bf16_kernel<BM, BN, PRO, STATS, 0, false, 32, SW_>), grid, s, (const bf16*)A, lda, pro, Wt, ldw,
                  epi, (bf16*)out, ldo, M, N, K, Ka, Kb, nMt, nNt, ConvG());
  } else
    gemm_f32_kernel<BM, BN, PRO, STATS><<<grid, 256, 0, s>>>((const float*)A, lda, pro, Wt, ldw, epi, (float*)out, ldo,
                                                             M, N, K, Ka, Kb, nMt, nNt, ConvG());
}

// 128-wide column tiles unless that leaves a half-empty last tile (N = 192, 576: 64-wide tiles
// waste nothing and give more blocks).  Knob "gemm_bn64" (default 1) turns the rule off.
static int g_gemm_bn64 = 1;
void set_gemm_bn64(int v) { g_gemm_bn64 = v; }
static bool wide_cols(int N) { return N > 64 && !(g_gemm_bn64 && N % 128 != 0 && N % 128 <= 64); }

template <typename T, bool PRO, bool STATS>
static void launch_mm_bn(const void* A, int lda, const Pro& pro, const float* Wt, int ldw, void* out, int ldo, int M,
                         int N, int K, int Ka, int Kb, const Epi& epi, hipStream_t s) {
  if (wide_cols(N))
    launch_mm<T, 128, PRO, STATS>(A, lda, pro, Wt, ldw, out, ldo, M, N, K, Ka, Kb, epi, s);
  else
    launch_mm<T, 64, PRO, STATS>(A, lda, pro, Wt, ldw, out, ldo, M, N, K, Ka, Kb, epi, s);
}

template <typename T>
static void launch_mm_any(const void* A, int lda, const Pro& pro, const float* Wt, int ldw, void* out, int ldo, int M,
                          int N, int K, int Ka, int Kb, const Epi& epi, hipStream_t s) {
  const bool p = pro.any(), st = epi.stat != nullptr;
  if (p && st) launch_mm_bn<T, true, true>(A, lda, pro, Wt, ldw, out, ldo, M, N, K, Ka, Kb, epi, s);
  else if (p) launch_mm_bn<T, true, false>(A, lda, pro, Wt, ldw, out, ldo, M, N, K, Ka, Kb, epi, s);
  else if (st) launch_mm_bn<T, false, true>(A, lda, pro, Wt, ldw, out, ldo, M, N, K, Ka, Kb, epi, s);
  else launch_mm_bn<T, false, false>(A, lda, pro, Wt, ldw, out, ldo, M, N, K, Ka, Kb, epi, s);
}

static bool tiny(int M, int N, ogv_dtype dt, const Epi& epi) {
  return dt == OGV_F32 && epi.stat == nullptr && M <= 2048 && (long)M * N <= (1L << 20);
}

// OGV_LOG_GEMM=1: one stderr line per GEMM launch (kind, shape, prologue/epilogue flags) for tuning
static bool log_gemm() {
  static const int on = [] {
    const char* e = getenv("OGV_LOG_GEMM");
    return e && *e == '1' ? 1 : 0;
  }();
  return on != 0;
}

int gemm_fwd_launch(ogv_dtype dt, const void* A, int lda, const Pro& pro, const float* W, int ldw, void* out, int ldo,
                    int M, int N, int K, int Ka, int Kb, const Epi& epi, hipStream_t s) {
  if (M <= 0) return 0;
  if (log_gemm())
    fprintf(stderr, "OGVGEMM fwd dt=%d M=%d N=%d K=%d Ka=%d Kb=%d pro=%d stats=%d res=%d lda=%d ldo=%d al=%d%d%d\n",
            (int)dt, M, N, K, Ka, Kb, (int)pro.any(), epi.stat != nullptr, epi.res != nullptr, lda, ldo,
            (int)(reinterpret_cast<uintptr_t>(A) & 15), (int)(reinterpret_cast<uintptr_t>(out) & 15),
            (int)(reinterpret_cast<uintptr_t>(epi.res) & 15));
  if (dt == OGV_BF16 && Ka == K && Kb == K) {
    const int r = sgemm_fwd_try(A, lda, pro, W, ldw, out, ldo, M, N, K, epi, s);
    if (r > 0) {
      if (log_gemm()) fprintf(stderr, "OGVROUTE fwd stream\n");
      return r;
    }
    const int r2 = pgemm_fwd_try(A, lda, pro, W, ldw, out, ldo, M, N, K, epi, s);
    if (r2 > 0) {
      if (log_gemm()) fprintf(stderr, "OGVROUTE fwd panel\n");
      return r2;
    }
  }
  if (log_gemm()) fprintf(stderr, "OGVROUTE fwd tiled\n");
  if (tiny(M, N, dt, epi)) {
    const int K0 = Ka < Kb ? Ka : Kb;
    const long outs = (long)M * N;
    if (K0 >= 256)
      small_fwd_kernel<64><<<cdiv(outs * 64, 256), 256, 0, s>>>((const float*)A, lda, pro, W, ldw, epi, (float*)out,
                                                                 ldo, M, N, Ka, Kb);
    else if (K0 >= 48)
      small_fwd_kernel<16><<<cdiv(outs * 16, 256), 256, 0, s>>>((const float*)A, lda, pro, W, ldw, epi, (float*)out,
                                                                 ldo, M, N, Ka, Kb);
    else
      small_fwd_kernel<4><<<cdiv(outs * 4, 256), 256, 0, s>>>((const float*)A, lda, pro, W, ldw, epi, (float*)out, ldo,
                                                               M, N, Ka, Kb);
    return 1;
  }
  if (dt == OGV_BF16) launch_mm_any<bf16>(A, lda, pro, W, ldw, out, ldo, M, N, K, Ka, Kb, epi, s);
  else launch_mm_any<float>(A, lda, pro, W, ldw, out, ldo, M, N, K, Ka, Kb, epi, s);
  return gemm_stat_rows(M);
}

template <typename T, bool STATS>
static void launch_conv_mm(const void* A, const ConvG& cv, const float* Wt, void* out, int M, int N, int K,
                           const Epi& epi, hipStream_t s) {
  constexpr int BM = GEMM_BM;
  const int nMt = (M + BM - 1) / BM;
  const int Kp = (K + 31) / 32 * 32;  // loop bound: whole BK slabs, zero-filled past K
  if (N > 64) {
    const int nNt = (N + 127) / 128;
    const unsigned grid = (unsigned)(((nMt + 7) / 8) * 8 * nNt);
    if constexpr (sizeof(T) == 2)
      OGV_SW_LAUNCH(g_split_w & (cv.transposed ? 2 : 1), (gemm_bf16_kernel<BM, 128, false, STATS, 1, false, 32, SW_>), grid, s, (const bf16*)A, 0, Pro(), Wt,
                    K, epi, (bf16*)out, N, M, N, Kp, K, K, nMt, nNt, cv);
    else
      gemm_f32_kernel<BM, 128, false, STATS, 1><<<grid, 256, 0, s>>>((const float*)A, 0, Pro(), Wt, K, epi,
                                                                     (float*)out, N, M, N, Kp, K, K, nMt, nNt, cv);
  } else {
    const int nNt = (N + 63) / 64;
    const unsigned grid = (unsigned)(((nMt + 7) / 8) * 8 * nNt);
    if constexpr (sizeof(T) == 2)
      OGV_SW_LAUNCH(g_split_w & (cv.transposed ? 2 : 1), (gemm_bf16_kernel<BM, 64, false, STATS, 1, false, 32, SW_>), grid, s, (const bf16*)A, 0, Pro(), Wt,
                    K, epi, (bf16*)out, N, M, N, Kp, K, K, nMt, nNt, cv);
    else
      gemm_f32_kernel<BM, 64, false, STATS, 1><<<grid, 256, 0, s>>>((const float*)A, 0, Pro(), Wt, K, epi,
                                                                    (float*)out, N, M, N, Kp, K, K, nMt, nNt, cv);
  }
}

int conv_gemm_launch(ogv_dtype dt, const void* A, const ConvG& cv, const float* Wt, void* out, int M, int N,
                     const Epi& epi, hipStream_t s) {
  if (M <= 0) return 1;
  const int K = 9 * cv.Cs;
  const bool st = epi.stat != nullptr;
  // the pipelined panel kernel with implicit-conv A fragments (8 | Cs): BN partial rows per 128-row panel
  // (or per 64-row panel on small M, knob pg_conv_rs1: at most conv_stat_rows(M)), the count returned
  if (dt == OGV_BF16) {
    const int rows = pgemm_conv_try(A, cv, Wt, out, M, N, epi, s);
    if (rows) return rows;
  }
  if (dt == OGV_BF16 && !epi.stat && !epi.res && !epi.zact && !epi.bias && !epi.rs &&
      pgemm_tconv_try(A, cv, Wt, out, M, N, s))
    return 1;
  if (dt == OGV_BF16) {
    if (st) launch_conv_mm<bf16, true>(A, cv, Wt, out, M, N, K, epi, s);
    else launch_conv_mm<bf16, false>(A, cv, Wt, out, M, N, K, epi, s);
  } else {
    if (st) launch_conv_mm<float, true>(A, cv, Wt, out, M, N, K, epi, s);
    else launch_conv_mm<float, false>(A, cv, Wt, out, M, N, K, epi, s);
  }
  return gemm_stat_rows(M);
}

// ------------------------------------------------------------------ small-M fp32 GEMMs (SE MLP)
// M = batch rows (512), K up to 1024: one K-serial block per 128-row tile would be latency-bound,
// so K is split over blockIdx.y (exact-f32 MFMA, raw partials), then one pass sums the partials in
// a fixed order and applies the epilogue.
struct SplitPlan {
  int S, kc, nNt, BN;
};
static int g_splitk_max = 32;  // knob "splitk_max": cap on the K slabs of the fp32 split-K GEMM (SE MLP)
void set_splitk_max(int v) { g_splitk_max = v < 1 ? 1 : (v > 32 ? 32 : v); }

static SplitPlan splitk_plan(int M, int N, int K) {
  SplitPlan p;
  p.BN = N > 64 ? 128 : 64;
  p.nNt = (N + p.BN - 1) / p.BN;
  const long tiles = (long)((M + GEMM_BM - 1) / GEMM_BM) * p.nNt;
  long S = (256 + tiles - 1) / tiles;
  S = std::min(S, (long)((K + 31) / 32));                          // >= 2 MFMA K-steps per chunk
  S = std::min(S, std::max(1L, (4L << 20) / ((long)M * N)));       // partials <= 16 MB
  S = std::max(1L, std::min(S, (long)g_splitk_max));
  p.kc = (int)(((K + S - 1) / S + 15) / 16 * 16);
  p.S = (K + p.kc - 1) / p.kc;
  return p;
}

size_t splitk_ws_bytes(int M, int N, int K) {
  const SplitPlan p = splitk_plan(M > 0 ? M : 1, N, K);
  return (size_t)p.S * (M > 0 ? M : 1) * N * sizeof(float) + 256;
}

__global__ __launch_bounds__(256) void splitk_reduce_kernel(const float* __restrict__ part, int S, int M, int N,
                                                            Epi epi, float* __restrict__ out, int ldo,
                                                            float* __restrict__ sig_out) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (long)M * N) return;
  const int m = (int)(i / N), n = (int)(i - (long)m * N);
  const long MN = (long)M * N;
  float a[4] = {0.f, 0.f, 0.f, 0.f};   // four slices' loads in flight per trip
  int s = 0;
  for (; s + 3 < S; s += 4) {
#pragma unroll
    for (int u = 0; u < 4; ++u) a[u] += part[(long)(s + u) * MN + i];
  }
  for (; s < S; ++s) a[0] += part[(long)s * MN + i];
  float v = (a[0] + a[1]) + (a[2] + a[3]);
  if (epi.bias) v += epi.bias[n];
  if (epi.rs) v *= epi.rs[m / epi.rps];
  if (epi.res) v += static_cast<const float*>(epi.res)[(long)m * ldo + n];
  if (epi.zact) v *= act_grad(epi.zact, static_cast<const float*>(epi.Z)[(long)m * epi.ldz + n]);
  out[(long)m * ldo + n] = v;
  if (sig_out) sig_out[(long)m * ldo + n] = fast_sigmoid(v);  // the SE gate, fused (was its own launch)
}

void gemm_fwd_splitk_f32(const float* A, int lda, const Pro& pro, const float* W, int ldw, float* out, int ldo, int M,
                         int N, int K, const Epi& epi, void* ws, hipStream_t s, bool bt, float* sig_out) {
  if (M <= 0) return;
  const SplitPlan p = splitk_plan(M, N, K);
  float* part = (float*)ws;
  const int nMt = (M + GEMM_BM - 1) / GEMM_BM;
  dim3 grid((unsigned)(((nMt + 7) / 8) * 8 * p.nNt), (unsigned)p.S);
  const bool pr = pro.any();
  if (bt) {  // W stored [K][ldw] (reduction-major): the data-gradient of a [N'][K'] weight, no transpose
    if (p.BN == 128)
      gemm_f32_kernel<GEMM_BM, 128, false, false, 0, true><<<grid, 256, 0, s>>>(A, lda, pro, W, ldw, Epi(), part, N, M,
                                                                                N, p.kc, K, K, nMt, p.nNt, ConvG(), p.kc);
    else
      gemm_f32_kernel<GEMM_BM, 64, false, false, 0, true><<<grid, 256, 0, s>>>(A, lda, pro, W, ldw, Epi(), part, N, M,
                                                                               N, p.kc, K, K, nMt, p.nNt, ConvG(), p.kc);
  } else if (p.BN == 128) {
    if (pr) gemm_f32_kernel<GEMM_BM, 128, true, false><<<grid, 256, 0, s>>>(A, lda, pro, W, ldw, Epi(), part, N, M, N,
                                                                           p.kc, K, K, nMt, p.nNt, ConvG(), p.kc);
    else gemm_f32_kernel<GEMM_BM, 128, false, false><<<grid, 256, 0, s>>>(A, lda, pro, W, ldw, Epi(), part, N, M, N,
                                                                          p.kc, K, K, nMt, p.nNt, ConvG(), p.kc);
  } else {
    if (pr) gemm_f32_kernel<GEMM_BM, 64, true, false><<<grid, 256, 0, s>>>(A, lda, pro, W, ldw, Epi(), part, N, M, N,
                                                                          p.kc, K, K, nMt, p.nNt, ConvG(), p.kc);
    else gemm_f32_kernel<GEMM_BM, 64, false, false><<<grid, 256, 0, s>>>(A, lda, pro, W, ldw, Epi(), part, N, M, N,
                                                                         p.kc, K, K, nMt, p.nNt, ConvG(), p.kc);
  }
  splitk_reduce_kernel<<<cdiv((long)M * N, 256), 256, 0, s>>>(part, p.S, M, N, epi, out, ldo, sig_out);
}

void transpose_f32_launch(const float* W, float* WT, int N, int K, int ldt, hipStream_t s) {
  dim3 tg(cdiv(K, 32), cdiv(ldt, 32));
  transpose_f32_kernel<<<tg, 256, 0, s>>>(W, WT, N, K, ldt);
}

size_t dgrad_ws_bytes(int N, int K) { return 256; }

template <typename T, int BN, int BM = GEMM_BM>
static void launch_mm_bt(const void* A, int lda, const float* W, int ldw, void* out, int ldo, int M, int N, int K,
                         const Epi& epi, hipStream_t s) {
  if constexpr (BM == GEMM_BM) {
    if (M <= g_bm64_max_m) {
      launch_mm_bt<T, BN, 64>(A, lda, W, ldw, out, ldo, M, N, K, epi, s);
      return;
    }
  }
  const int nMt = (M + BM - 1) / BM, nNt = (N + BN - 1) / BN;
  const unsigned grid = (unsigned)(((nMt + 7) / 8) * 8 * nNt);
  const int Kp = (K + 31) / 32 * 32;
  if constexpr (sizeof(T) == 2) {
    if (use_bk64(M, K, N, false, epi.zact != 0))
      OGV_SW_LAUNCH(g_split_w & 2, (gemm_bf16_kernel<BM, BN, false, false, 0, true, 64, SW_>), grid, s, (const bf16*)A, lda, Pro(), W,
                    ldw, epi, (bf16*)out, ldo, M, N, (K + 63) / 64 * 64, K, K, nMt, nNt, ConvG());
    else
      OGV_SW_LAUNCH(g_split_w & 2, (gemm_bf16_kernel<BM, BN, false, false, 0, true, 32, SW_>), grid, s, (const bf16*)A, lda, Pro(), W,
                    ldw, epi, (bf16*)out, ldo, M, N, Kp, K, K, nMt, nNt, ConvG());
  } else
    gemm_f32_kernel<BM, BN, false, false, 0, true><<<grid, 256, 0, s>>>((const float*)A, lda, Pro(), W, ldw, epi,
                                                                        (float*)out, ldo, M, N, Kp, K, K, nMt, nNt,
                                                                        ConvG());
}

void gemm_dgrad_launch(ogv_dtype dt, const void* dout, int ldd, const float* W, const void* Z, int ldz, int zact,
                       const float* rs, int rps, const void* res, void* dA, int lda, int M, int N, int K, void* ws,
                       hipStream_t s) {
  if (M <= 0) return;
  if (log_gemm())
    fprintf(stderr, "OGVGEMM dgrad dt=%d M=%d N=%d K=%d zact=%d res=%d\n", (int)dt, M, N, K, zact, res != nullptr);
  Epi e;
  e.rs = rs;
  e.rps = rps;
  e.Z = Z;
  e.ldz = ldz;
  e.zact = zact;
  e.res = res;
  // dA[M,K] = dout[M,N] . W[N,K]: W read as [reduction N][output K] (no transposed copy)
  if (dt == OGV_BF16 && sgemm_dgrad_try(dout, ldd, W, dA, lda, M, N, K, e, s)) return;
  if (dt == OGV_BF16 && pgemm_dgrad_try(dout, ldd, W, dA, lda, M, N, K, e, s)) return;
  if (dt == OGV_BF16) {
    if (wide_cols(K)) launch_mm_bt<bf16, 128>(dout, ldd, W, K, dA, lda, M, K, N, e, s);
    else launch_mm_bt<bf16, 64>(dout, ldd, W, K, dA, lda, M, K, N, e, s);
  } else {
    if (wide_cols(K)) launch_mm_bt<float, 128>(dout, ldd, W, K, dA, lda, M, K, N, e, s);
    else launch_mm_bt<float, 64>(dout, ldd, W, K, dA, lda, M, K, N, e, s);
  }
}

// Split-M plan.  bf16: tiles of BN x BK in {64,128}^2, slab partials [S][N*K + N] (dW then
// dbias) summed by one colreduce.  S is sized to put ~1024 blocks on the chip with >= 256 rows per
// slab, while keeping the partial traffic under max(data / 4, 16 MB).
struct WgradPlan {
  int BN, BK, nNt, nKt, S, mchunk;
};
static int g_wg_blocks = 2048;  // knob "wg_blocks": workgroups the bf16 split-M plan aims for (measured: 1024 18.87, 2048 18.84, 4096 18.82-18.85 ms/step)
static int g_wg_tile = 0;       // knob "wg_tile": force BN = BK = 64 (64) or 128 (128); 0 = by shape
void set_wg_blocks(int v) { g_wg_blocks = v < 64 ? 64 : v; }
void set_wg_tile(int v) { g_wg_tile = (v == 64 || v == 128) ? v : 0; }
static WgradPlan wgrad_plan(ogv_dtype dt, int M, int N, int K) {
  WgradPlan p;
  // bf16: 64 x 64 tiles (more tiles in flight, no half-empty 128-wide tile at K or N = 192),
  // except the large M = 32768 projections of 147k-weight layers where 128 x 128 measured faster
  // (tools/gpu_pgemm_sweep.sh KINDS=wgrad: 7M census 4.35 -> 3.79 ms)
  p.BN = p.BK = 64;
  if (dt == OGV_BF16 && M >= 32768 && (long)N * K >= 147456 && std::max(N, K) <= 768) {
    p.BN = N > 64 ? 128 : 64;
    p.BK = K > 64 ? 128 : 64;
  }
  if (dt == OGV_BF16 && g_wg_tile) p.BN = p.BK = g_wg_tile;
  p.nNt = (N + p.BN - 1) / p.BN;
  p.nKt = (K + p.BK - 1) / p.BK;
  const long tiles = (long)p.nNt * p.nKt;
  long S = ((dt == OGV_BF16 ? g_wg_blocks : 1024) + tiles - 1) / tiles;
  S = std::min(S, ((long)M + (M <= 4096 ? 31 : 255)) / (M <= 4096 ? 32 : 256));  // small M (SE): 32-row slabs
  const double data = 2.0 * M * (N + K) * (dt == OGV_BF16 ? 2 : 4);
  const long cap = (long)(std::max(data / 4, 16.0 * (1 << 20)) / (4.0 * ((double)N * K + N)));
  S = std::max(1L, std::min(S, cap));
  int mchunk = (int)((M + S - 1) / S);
  mchunk = (mchunk + 31) / 32 * 32;
  p.S = (M + mchunk - 1) / mchunk;
  p.mchunk = mchunk;
  return p;
}

size_t wgrad_ws_bytes(int M, int N, int K) {
  // the larger of the bf16 and fp32 plans (the C ABI sizes the workspace without the dtype)
  size_t best = 0;
  for (ogv_dtype dt : {OGV_BF16, OGV_F32}) {
    WgradPlan p = wgrad_plan(dt, M > 0 ? M : 1, N, K);
    const long ld = (long)N * K + N;
    best = std::max(best, ((size_t)p.S * ld + colreduce_tmp_floats(p.S, ld)) * sizeof(float));
  }
  best = std::max(best, wgrad2_ws_floats(M > 0 ? M : 1, N, K) * sizeof(float));
  return std::max(best, swgrad_ws_floats(M > 0 ? M : 1, N, K) * sizeof(float));
}

template <int BN, int BK>
static void launch_wgrad_bf16(const WgradPlan& p, const void* G, int ldg, const void* X, int ldx, const Pro& pro,
                              const float* rs, int rps, float* part, long ldp, bool bias, int M, int N, int K,
                              hipStream_t s, const ConvG* xc) {
  const int tiles = p.nNt * p.nKt;
  const unsigned grid = (unsigned)(((p.S + 7) / 8) * 8 * tiles);
  const ConvG cv = xc ? *xc : ConvG();
  if (xc)
    wgrad_bf16_kernel<BN, BK, false, 1><<<grid, 256, 0, s>>>((const bf16*)G, ldg, (const bf16*)X, ldx, pro, rs, rps,
                                                             part, ldp, bias, M, N, K, p.mchunk, p.nNt, tiles, p.S, cv);
  else if (pro.any())
    wgrad_bf16_kernel<BN, BK, true><<<grid, 256, 0, s>>>((const bf16*)G, ldg, (const bf16*)X, ldx, pro, rs, rps, part,
                                                         ldp, bias, M, N, K, p.mchunk, p.nNt, tiles, p.S, cv);
  else
    wgrad_bf16_kernel<BN, BK, false><<<grid, 256, 0, s>>>((const bf16*)G, ldg, (const bf16*)X, ldx, pro, rs, rps, part,
                                                          ldp, bias, M, N, K, p.mchunk, p.nNt, tiles, p.S, cv);
}

void gemm_wgrad_launch(ogv_dtype dt, const void* G, int ldg, const void* X, int ldx, const Pro& pro, const float* rs,
                       int rps, float* dW, float* dbias, int M, int N, int K, void* ws, hipStream_t s,
                       const ConvG* xc, bool param_grad) {
  // param_grad: dW / dbias are final parameter gradients (read by nothing but the optimizer), so
  // their slab reduction may be deferred (colreduce_param)
  auto reduce = param_grad ? colreduce_param : static_cast<void (*)(const float*, float*, long, long, long, float*,
                                                                    hipStream_t, float*, long)>(colreduce);
  if (skip_mask() & 4) return;
  if (M <= 0) {
    (void)hipMemsetAsync(dW, 0, (size_t)N * K * sizeof(float), s);
    if (dbias) (void)hipMemsetAsync(dbias, 0, (size_t)N * sizeof(float), s);
    return;
  }
  if (log_gemm())
    fprintf(stderr, "OGVGEMM wgrad dt=%d M=%d N=%d K=%d pro=%d conv=%d bias=%d\n", (int)dt, M, N, K, (int)pro.any(),
            xc != nullptr, dbias != nullptr);
  const long ldp = (long)N * K + N;
  float* part = (float*)ws;
  if (dt == OGV_BF16 && xc) {   // 3x3 conv weight gradient: pipelined kernel with the gather (8 | C_in)
    bool reduced = false;
    const int S = wgrad2_try(G, ldg, X, ldx, pro, rs, rps, part, dW, dbias, dbias != nullptr, M, N, K, s, &reduced, xc);
    if (S > 0) {
      reduce(part, dW, S, dbias ? ldp : (long)N * K, ldp, part + (size_t)S * ldp, s, dbias, (long)N * K);
      return;
    }
  }
  if (dt == OGV_BF16 && !xc) {
    const bool b = dbias != nullptr;
    bool reduced = false;
    int S = wg2_mode() == 2 ? wgrad2_try(G, ldg, X, ldx, pro, rs, rps, part, dW, dbias, b, M, N, K, s, &reduced) : 0;
    if (S == 0) S = swgrad_try(G, ldg, X, ldx, pro, rs, rps, part, b, M, N, K, s);
    if (S == 0 && wg2_mode() == 1) S = wgrad2_try(G, ldg, X, ldx, pro, rs, rps, part, dW, dbias, b, M, N, K, s, &reduced);
    if (S > 0) {
      if (!reduced)
        reduce(part, dW, S, dbias ? ldp : (long)N * K, ldp, part + (size_t)S * ldp, s, dbias, (long)N * K);
      return;
    }
  }
  const WgradPlan p = wgrad_plan(dt, M, N, K);
  float* tmp = part + (size_t)p.S * ldp;
  if (dt == OGV_BF16) {
    const bool b = dbias != nullptr;
    if (p.BN == 128 && p.BK == 128)
      launch_wgrad_bf16<128, 128>(p, G, ldg, X, ldx, pro, rs, rps, part, ldp, b, M, N, K, s, xc);
    else if (p.BN == 128) launch_wgrad_bf16<128, 64>(p, G, ldg, X, ldx, pro, rs, rps, part, ldp, b, M, N, K, s, xc);
    else if (p.BK == 128) launch_wgrad_bf16<64, 128>(p, G, ldg, X, ldx, pro, rs, rps, part, ldp, b, M, N, K, s, xc);
    else launch_wgrad_bf16<64, 64>(p, G, ldg, X, ldx, pro, rs, rps, part, ldp, b, M, N, K, s, xc);
  } else {
    dim3 grid(p.nNt * p.nKt, p.S);
    const ConvG cv = xc ? *xc : ConvG();
    if (xc)
      wgrad_f32_kernel<false, 1><<<grid, 256, 0, s>>>((const float*)G, ldg, (const float*)X, ldx, pro, rs, rps, part,
                                                      ldp, dbias != nullptr, M, N, K, p.mchunk, p.nNt, cv);
    else if (pro.any())
      wgrad_f32_kernel<true><<<grid, 256, 0, s>>>((const float*)G, ldg, (const float*)X, ldx, pro, rs, rps, part, ldp,
                                                  dbias != nullptr, M, N, K, p.mchunk, p.nNt, cv);
    else
      wgrad_f32_kernel<false><<<grid, 256, 0, s>>>((const float*)G, ldg, (const float*)X, ldx, pro, rs, rps, part, ldp,
                                                   dbias != nullptr, M, N, K, p.mchunk, p.nNt, cv);
  }
  reduce(part, dW, p.S, dbias ? ldp : (long)N * K, ldp, tmp, s, dbias, (long)N * K);
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
  Pro pro;
  pro.act = act_in;
  Epi epi;
  epi.bias = bias;
  epi.res = res;
  epi.rs = rs;
  epi.rps = rps > 0 ? rps : 1;
  gemm_fwd_launch(dt, A, lda, pro, W, K, out, ldo, M, N, K, K, K, epi, as_stream(stream));
  return check_launch("ogv_gemm_fwd");
}

// knob "ln_epi": the next LayerNorm in the producing GEMM's epilogue (ogv_gemm_fwd_ln) -- 0 never; 1 (default)
// where the panel kernel is the route anyway (M below sgemm_min_m); 2 at every M (the panel kernel then replaces
// the streaming one)
static int g_ln_epi = 1;
namespace ogv {
void set_ln_epi(int v) { g_ln_epi = v < 0 ? 0 : (v > 2 ? 2 : v); }
}  // namespace ogv

// out = res + rs * (A . W^T + bias) (bf16, stored rounded) and the next LayerNorm of those rows, one launch:
// ln_out = (out - mean) * rstd * gamma + beta (row stride ldo), mean / rstd [M] for the LN backward.
// OGV_ERR_UNSUPPORTED, with nothing launched, where the panel kernel does not take it.
extern "C" int ogv_gemm_fwd_ln(const void* A, int lda, const float* W, const float* bias, const void* res,
                               const float* rs, int rps, void* out, int ldo, void* ln_out, const float* gamma,
                               const float* beta, float eps, float* mean, float* rstd, int M, int N, int K,
                               ogv_dtype dt, void* stream) {
  int rc = check_common(M, N, K, OGV_ACT_NONE, dt, "ogv_gemm_fwd_ln");
  if (rc) return rc;
  OGV_REQUIRE(A && W && out && ln_out && gamma && beta && mean && rstd, "ogv_gemm_fwd_ln: null pointer");
  OGV_REQUIRE(lda >= K && ldo >= N, "ogv_gemm_fwd_ln: lda %d / ldo %d too small", lda, ldo);
  OGV_REQUIRE(!rs || rps > 0, "ogv_gemm_fwd_ln: rows-per-sample must be > 0 with a row scale");
  if (dt != OGV_BF16 || !g_ln_epi || (g_ln_epi == 1 && M >= sgemm_min_m())) {
    set_error("ogv_gemm_fwd_ln: unsupported here (bf16 panel-kernel shapes only, knob ln_epi)");
    return OGV_ERR_UNSUPPORTED;
  }
  Epi epi;
  epi.bias = bias;
  epi.res = res;
  epi.rs = rs;
  epi.rps = rps > 0 ? rps : 1;
  epi.ln_out = ln_out;
  epi.ln_g = gamma;
  epi.ln_b = beta;
  epi.ln_mean = mean;
  epi.ln_rstd = rstd;
  epi.ln_eps = eps;
  if (!pgemm_fwd_ln_try(A, lda, W, K, out, ldo, M, N, K, epi, as_stream(stream))) {
    set_error("ogv_gemm_fwd_ln: unsupported shape (N <= 192, 8 | N, 8 | K, 16-B aligned rows)");
    return OGV_ERR_UNSUPPORTED;
  }
  return check_launch("ogv_gemm_fwd_ln");
}

// out = A . W^T + bias (bf16, stored rounded) and aout = act(out) of the stored values, one launch:
// the pre-activation for the next layer's data gradient (act'(Z)) and the activation for its
// forward and weight gradient, so neither recomputes the activation per element.
extern "C" int ogv_gemm_fwd_act(const void* A, int lda, const float* W, const float* bias, void* out, int ldo,
                                void* aout, int ldao, int M, int N, int K, ogv_act act_out, ogv_dtype dt,
                                void* stream) {
  int rc = check_common(M, N, K, act_out, dt, "ogv_gemm_fwd_act");
  if (rc) return rc;
  OGV_REQUIRE(dt == OGV_BF16, "ogv_gemm_fwd_act: bf16 only");
  OGV_REQUIRE(A && W && out && aout, "ogv_gemm_fwd_act: null pointer");
  OGV_REQUIRE(act_out != OGV_ACT_NONE, "ogv_gemm_fwd_act: needs an activation");
  OGV_REQUIRE(lda >= K, "ogv_gemm_fwd_act: lda %d < K %d", lda, K);
  OGV_REQUIRE(ldo >= N && ldao >= N, "ogv_gemm_fwd_act: ldo %d / ldao %d < N %d", ldo, ldao, N);
  Epi epi;
  epi.bias = bias;
  epi.aout = aout;
  epi.ldao = ldao;
  epi.aact = (int)act_out;
  gemm_fwd_launch(dt, A, lda, Pro(), W, K, out, ldo, M, N, K, K, K, epi, as_stream(stream));
  return check_launch("ogv_gemm_fwd_act");
}

extern "C" size_t ogv_gemm_dgrad_ws_bytes(int N, int K) { return dgrad_ws_bytes(N, K); }

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
  gemm_dgrad_launch(dt, dout, ldd, W, Z, ldz, (int)act_in, rs, rps > 0 ? rps : 1, nullptr, dA, lda, M, N, K, ws,
                    as_stream(stream));
  return check_launch("ogv_gemm_dgrad");
}

extern "C" size_t ogv_gemm_wgrad_ws_bytes(int M, int N, int K) { return wgrad_ws_bytes(M, N, K); }

extern "C" int ogv_gemm_wgrad(const void* dout, int ldd, const void* A, int lda, const float* rs, int rps, float* dW,
                              float* dbias, int M, int N, int K, ogv_act act_in, void* ws, ogv_dtype dt,
                              void* stream) {
  int rc = check_common(M, N, K, act_in, dt, "ogv_gemm_wgrad");
  if (rc) return rc;
  OGV_REQUIRE(dout && A && dW && ws, "ogv_gemm_wgrad: null pointer");
  OGV_REQUIRE(ldd >= N && lda >= K, "ogv_gemm_wgrad: ldd/lda smaller than N/K");
  OGV_REQUIRE(!rs || rps > 0, "ogv_gemm_wgrad: rows-per-sample must be > 0 with a row scale");
  Pro pro;
  pro.act = act_in;
  gemm_wgrad_launch(dt, dout, ldd, A, lda, pro, rs, rps > 0 ? rps : 1, dW, dbias, M, N, K, ws, as_stream(stream),
                    nullptr, true);
  return check_launch("ogv_gemm_wgrad");
}
