// Pipelined panel GEMM for the small-M projections (stages 2-3 of Model-A-7M, M <= 32768).
//
// At M = 8192 - 32768 rows the whole GEMM is a few hundred 128-row panels: every workgroup does
// a handful of k-steps and leaves, so what bounds the classic LDS-tiled kernel (ogv_gemm.hip) is
// the serial chain of "load slab -> barrier -> MFMA -> barrier" round trips, not bandwidth or the
// matrix cores.  This kernel keeps more bytes in flight per CU and shortens that chain:
//   * A (activations) never goes through LDS: each wave owns 16*RS rows and loads its MFMA
//     fragments straight from HBM into registers (16 B per lane, a whole 128-B line per row per
//     64-wide k-step), TWO k-steps ahead of the MFMAs;
//   * only the weight slab [BN x 64] is shared: staged through registers (fp32 -> bf16 hi / lo) into
//     a double-buffered LDS tile one k-step ahead, ONE workgroup barrier per k-step;
//   * the product is computed transposed (D[n][m] = W-slab . A^T, the weight fragment as the MFMA
//     A operand), so a lane's accumulator holds 4 consecutive output columns of one row and the
//     epilogue (bias, DropPath row scale, residual, activation derivative, BatchNorm column
//     statistics) runs from registers with 8-B loads / stores, as in the streaming kernel
//     (ogv_sgemm.hip), which covers M >= 65536;
//   * the A prologue (GELU of fc2, or MBConv's BatchNorm-apply + SiLU + SE gate) is applied to the
//     fragments in registers, once per element and N-tile.
// Forward: B[n][k] = W[n*ldw + k].  Data gradient (BT): the forward weight [Nf][Kf] read as
// [reduction][output]; the slab is staged [k][n] as loaded and the fragments come from
// ds_read_b64_tr_b16 transposed reads, with the slab's rows permuted so the reads are
// bank-conflict free and each lane still receives 8 CONSECUTIVE k (so the A fragment stays one
// 16-B load).
#include "ogv_gemm.h"

namespace ogv {

constexpr int PG_NW = 4;           // waves per workgroup
constexpr int PG_KB = 64;          // reduction columns per k-step (two 32-wide MFMA sub-steps)
constexpr int PG_KP = PG_KB;       // [n][k] slab pitch (elements): 128-B rows, 16-B chunks rotated by the row
// data gradients (BT) with their slab columns permuted like the forward's rows (16-B epilogue
// accesses of dX, Z and the residual) instead of 8-B ones
constexpr bool PG_BT16 = true;
// (chunk c of row r stored at (c + r) & 7): conflict-free 16-B fragment reads and 8-B staging writes

template <int TN, bool BT>
__host__ __device__ constexpr int pg_slab_elems() {
  return BT ? PG_KB * (TN * 16 + 16) : TN * 16 * PG_KP;
}

// logical k (0..31 inside a 32-wide sub-step) -> physical slab row for the BT layout: bits 2 and 3
// swapped, so the rows one tr-read instruction touches (k = 8g + 4h + q over g = 0,1) are 8
// consecutive rows (conflict-free with a pitch of 8 mod 64 dwords)
__device__ __forceinline__ int pg_perm(int k) { return (k & ~12) | ((k & 4) << 1) | ((k & 8) >> 1); }

// forward slab row of tile column c (see store_w) and its inverse
__device__ __forceinline__ int pg_col_slot(int c) {
  const int cc = c & 31;
  return (c & ~31) | (((cc >> 2) & 1) << 4) | ((cc >> 3) << 2) | (cc & 3);
}
__device__ __forceinline__ int pg_slot_col(int r) {
  const int rr = r & 31;
  return (r & ~31) | (((rr >> 2) & 3) << 3) | (((rr >> 4) & 1) << 2) | (rr & 3);
}

// RS: 16-row fragments per wave (rows per tile = 64 * RS); TN: 16-column fragments per tile
// (BN = 16 * TN).  PA: -1 = no prologue, else its activation (sc / sh optional, staged in LDS);
// GT: the prologue has an SE gate.  ZA: activation derivative at Z in the epilogue.
//
// Persistent: workgroup b walks the virtual tiles vb = b, b + G, b + 2G, ... (G = gridDim.x, a
// multiple of 8, so vb keeps b's XCD) and the (tile, k-step) pairs form ONE pipeline: the loads of
// the next tile's first k-steps are in flight while the current tile's epilogue runs.
// CV: implicit-GEMM 3x3 convolution (stem / downsample convs, their data gradients as transposed
// convs): row m = output pixel, column k = tap * Cs + channel (tap-major weight), A fragments
// gathered from the NHWC source (cv, conv_src; zero outside the image); lda unused.
// LNO: the residual stream's next LayerNorm in the epilogue (Epi::ln_*): the tile holds whole rows (one column
// tile), so each row's mean / variance of the stored (rounded) outputs is a register sum over the lane's 8 * TN / 2
// columns plus two xor shuffles across the four lanes sharing the row -- the LayerNorm kernel's read of the row and
// its launch are gone
template <int RS, int TN, int PA, bool GT, int ZA, bool STATS, bool BT, bool SW, bool CV = false, bool LNO = false>
__global__ __launch_bounds__(PG_NW * 64, 2) void pgemm_bf16_kernel(const bf16* __restrict__ A, int lda, Pro pro,
                                                                const float* __restrict__ W, int ldw, Epi epi,
                                                                bf16* __restrict__ out, int ldo, int M, int N, int K,
                                                                int nMt, int nNt, int dbg, ConvG cv) {
  // the merged transposed-conv launch (cv.par == 4): this workgroup's parity class, its index within the
  // class's workgroups and the class's taps / reduction length
  int bid = blockIdx.x, G = gridDim.x;
  if constexpr (CV) {
    if (cv.par == 4) {
      const int c = blockIdx.x / cv.cls_G;
      bid = blockIdx.x - c * cv.cls_G;
      G = cv.cls_G;
      cv.par = c;
      cv.ntap = tconv_ntap(c);
#pragma unroll
      for (int t = 0; t < 4; ++t) cv.tap[t] = tconv_tap(c, t);
      K = cv.ntap * cv.Cs;
    }
  }
  constexpr int BN = TN * 16;
  constexpr int BM = PG_NW * 16 * RS;
  constexpr int SLAB = pg_slab_elems<TN, BT>();
  constexpr int NSLAB = SW ? 2 : 1;          // hi (+ lo) weight halves
  constexpr int WF4 = BN * PG_KB / 4 / 256;  // float4 weight loads per thread and k-step (= TN)
  constexpr int BP = BN + 16;                // BT slab pitch
  extern __shared__ __attribute__((aligned(16))) char smem[];
  bf16* slab = reinterpret_cast<bf16*>(smem);                                    // [2][NSLAB][SLAB]
  float* cvec = reinterpret_cast<float*>(smem + (size_t)2 * NSLAB * SLAB * 2);  // [2 tiles][bias | shift]
  double* red = reinterpret_cast<double*>(cvec + 4 * BN);                        // STATS: [wave][2][BN]
  bf16* stg = reinterpret_cast<bf16*>(red + (STATS ? PG_NW * 2 * BN : 0));        // STATS: [wave][16][16]
  float* pvec = reinterpret_cast<float*>(stg + (STATS ? PG_NW * 256 : 0));       // [sc | sh], PA >= 0

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int fr = lane & 15, fg = lane >> 4;
  const int xcd = bid & 7;
  // tiles of this workgroup: vb = bid + G * j; M-panel index is non-decreasing in j
  auto tile_mt = [&](int j) { return (((bid + G * j) >> 3) / nNt) * 8 + xcd; };
  auto tile_nt = [&](int j) { return ((bid + G * j) >> 3) % nNt; };
  int ntiles = 0;
  while (tile_mt(ntiles) < nMt) ++ntiles;
  if (ntiles == 0) return;
  const int nsteps = (K + PG_KB - 1) / PG_KB;
  const int total = ntiles * nsteps;

  if constexpr (PA >= 0) {
    for (int k = tid; k < K; k += PG_NW * 64) {
      pvec[k] = pro.sc ? pro.sc[k] : 1.f;
      pvec[K + k] = pro.sh ? pro.sh[k] : 0.f;
    }
  }

  // ---- weight slab of global step g (registers), staging (bf16 hi / lo -> LDS)
  float4 wr[WF4];
  auto load_w = [&](int g) {
    const int j = g / nsteps, k0 = (g - j * nsteps) * PG_KB, n0 = tile_nt(j) * BN;
#pragma unroll
    for (int i = 0; i < WF4; ++i) {
      const int idx = tid + i * 256;
      wr[i] = float4{0.f, 0.f, 0.f, 0.f};
      if constexpr (!BT) {
        const int r = idx / (PG_KB / 4), k = k0 + (idx % (PG_KB / 4)) * 4;
        int kc = k;
        if constexpr (CV) {
          if (cv.par >= 0) {   // the class's tap t -> the weight's full tap-major column block
            const int t = k / cv.Cs;
            kc = conv_tap(cv, t) * cv.Cs + (k - t * cv.Cs);
          }
        }
        if (n0 + r < N && k < K) wr[i] = *reinterpret_cast<const float4*>(W + (long)(n0 + r) * ldw + kc);
      } else {
        const int kr = idx / (BN / 4), c = (idx % (BN / 4)) * 4;
        if (k0 + kr < K && n0 + c < N) wr[i] = *reinterpret_cast<const float4*>(W + (long)(k0 + kr) * ldw + n0 + c);
      }
    }
  };
  auto store_w = [&](int buf) {
    bf16* hi = slab + (size_t)buf * NSLAB * SLAB;
#pragma unroll
    for (int i = 0; i < WF4; ++i) {
      const int idx = tid + i * 256;
      int off;
      if constexpr (!BT) {
        // weight row (tile column) c -> slab row pg_col_slot(c): fragment pair (2q, 2q+1) holds
        // columns 32q + 8g + 4h + r' at fragment 2q+h, row 4g + r', so a lane's accumulators of the
        // pair are 8 CONSECUTIVE output columns (16-B epilogue loads / stores)
        const int r = pg_col_slot(idx / (PG_KB / 4)), kq = idx % (PG_KB / 4);
        off = r * PG_KP + (((kq >> 1) + r) & 7) * 8 + (kq & 1) * 4;
      } else {
        // column c of the [k][n] slab stored at pg_col_slot(c) (groups of 4 stay contiguous): the
        // transposed reads then hand a lane's fragment pair 8 consecutive output columns, as in the
        // forward (16-B epilogue accesses)
        const int kr = idx / (BN / 4);
        const int c = (idx % (BN / 4)) * 4;
        off = ((kr & ~31) | pg_perm(kr & 31)) * BP + (PG_BT16 ? pg_col_slot(c) : c);
      }
      const bf16x4 h = {(bf16)wr[i].x, (bf16)wr[i].y, (bf16)wr[i].z, (bf16)wr[i].w};
      *reinterpret_cast<bf16x4*>(hi + off) = h;
      if constexpr (SW) {
        const bf16x4 l = {(bf16)(wr[i].x - (float)h[0]), (bf16)(wr[i].y - (float)h[1]),
                          (bf16)(wr[i].z - (float)h[2]), (bf16)(wr[i].w - (float)h[3])};
        *reinterpret_cast<bf16x4*>(hi + SLAB + off) = l;
      }
    }
  };

  // ---- A fragments of global step g: lane (fr, fg) holds row mw + 16 i + fr, k = k0 + 32 kt + 8 fg
  auto load_a = [&](int g, bf16x8 (&a)[RS][2]) {
    const int j = g / nsteps, k0 = (g - j * nsteps) * PG_KB;
    const int mw = tile_mt(j) * BM + wave * 16 * RS;
#pragma unroll
    for (int i = 0; i < RS; ++i) {
      const int m = mw + i * 16 + fr;
      if constexpr (CV) {
        if (cv.par >= 0) {   // parity class of a stride-2 transposed conv
          const int h2 = cv.Hr >> 1, w2 = cv.Wr >> 1, mm = m < M ? m : 0;
          const int b = mm / (h2 * w2), rem = mm - b * h2 * w2, Y = rem / w2;
          const int ry = 2 * Y + (cv.par >> 1), rx = 2 * (rem - Y * w2) + (cv.par & 1);
          // (offsets first, then both loads unconditionally at a valid address -- element 0 for a zero
          // tap -- and the zeros selected after: a guarded load here made the compiler wait for each)
          long offs[2];
#pragma unroll
          for (int kt = 0; kt < 2; ++kt) {
            const int k = k0 + kt * 32 + fg * 8;
            offs[kt] = -1;
            if (m < M && k < K) {
              const int t = k / cv.Cs, tp = conv_tap(cv, t);
              const int ky = tp / 3, kx = tp - 3 * ky;
              const int sy = (ry + 1 - ky) >> 1, sx = (rx + 1 - kx) >> 1;   // even by the class
              if (sy >= 0 && sy < cv.Hs && sx >= 0 && sx < cv.Ws)
                offs[kt] = ((long)(b * cv.Hs + sy) * cv.Ws + sx) * cv.Cs + (k - t * cv.Cs);
            }
          }
#pragma unroll
          for (int kt = 0; kt < 2; ++kt) {
            const bf16x8 v = *reinterpret_cast<const bf16x8*>(A + (offs[kt] >= 0 ? offs[kt] : 0));
            a[i][kt] = offs[kt] >= 0 ? v : bf16x8{};
          }
          continue;
        }
        const ConvRow cr = conv_row(cv, m < M ? m : 0);
        long offs[2];
#pragma unroll
        for (int kt = 0; kt < 2; ++kt) {
          const int k = k0 + kt * 32 + fg * 8;
          offs[kt] = -1;
          if (m < M && k < K) {
            const int tap = k / cv.Cs;            // 8 | Cs: the 8 columns share one tap
            const long off = conv_src(cv, cr, tap);
            if (off >= 0) offs[kt] = off + (k - tap * cv.Cs);
          }
        }
#pragma unroll
        for (int kt = 0; kt < 2; ++kt) {
          const bf16x8 v = *reinterpret_cast<const bf16x8*>(A + (offs[kt] >= 0 ? offs[kt] : 0));
          a[i][kt] = offs[kt] >= 0 ? v : bf16x8{};
        }
      } else {
#pragma unroll
        for (int kt = 0; kt < 2; ++kt) {
          const int k = k0 + kt * 32 + fg * 8;
          const bool ok = m < M && k < K;
          const bf16x8 v = *reinterpret_cast<const bf16x8*>(A + (ok ? (long)m * lda + k : 0));
          a[i][kt] = ok ? v : bf16x8{};
        }
      }
    }
  };
  // SE gate of step g (prologue with a gate): loaded one k-step ahead, with the weight slab
  float4 gr[GT ? RS : 1][GT ? 2 : 1][2];
  auto load_g = [&](int g) {
    if constexpr (GT) {
      const int j = g / nsteps, k0 = (g - j * nsteps) * PG_KB;
      const int mw = tile_mt(j) * BM + wave * 16 * RS;
#pragma unroll
      for (int i = 0; i < RS; ++i) {
        const int m = mw + i * 16 + fr;
#pragma unroll
        for (int kt = 0; kt < 2; ++kt) {
          const int k = k0 + kt * 32 + fg * 8;
          gr[i][kt][0] = gr[i][kt][1] = float4{1.f, 1.f, 1.f, 1.f};
          if (m < M && k < K) {
            const float* gp = pro.gate + (long)(m / pro.rps) * pro.gld + k;
            gr[i][kt][0] = *reinterpret_cast<const float4*>(gp);
            gr[i][kt][1] = *reinterpret_cast<const float4*>(gp + 4);
          }
        }
      }
    }
  };

  f32x4 acc[RS][TN];
#pragma unroll
  for (int i = 0; i < RS; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
  typedef __attribute__((ext_vector_type(8))) short s16x8;
  const int q = fr >> 2, p4 = (fr & 3) * 4;

  auto compute = [&](int k0, bf16x8 (&a)[RS][2], int buf) {
    if constexpr (PA >= 0) {
#pragma unroll
      for (int i = 0; i < RS; ++i) {
#pragma unroll
        for (int kt = 0; kt < 2; ++kt) {
          const int k = k0 + kt * 32 + fg * 8;
          if (k < K) {
            float g8[8];
            if constexpr (GT) {
              g8[0] = gr[i][kt][0].x; g8[1] = gr[i][kt][0].y; g8[2] = gr[i][kt][0].z; g8[3] = gr[i][kt][0].w;
              g8[4] = gr[i][kt][1].x; g8[5] = gr[i][kt][1].y; g8[6] = gr[i][kt][1].z; g8[7] = gr[i][kt][1].w;
            }
            const float4 sc0 = *reinterpret_cast<const float4*>(pvec + k);
            const float4 sc1 = *reinterpret_cast<const float4*>(pvec + k + 4);
            const float4 sh0 = *reinterpret_cast<const float4*>(pvec + K + k);
            const float4 sh1 = *reinterpret_cast<const float4*>(pvec + K + k + 4);
            const float sc[8] = {sc0.x, sc0.y, sc0.z, sc0.w, sc1.x, sc1.y, sc1.z, sc1.w};
            const float sh[8] = {sh0.x, sh0.y, sh0.z, sh0.w, sh1.x, sh1.y, sh1.z, sh1.w};
#pragma unroll
            for (int e = 0; e < 8; ++e) {
              float f = act_fwd(PA, fmaf((float)a[i][kt][e], sc[e], sh[e]));
              if constexpr (GT) f *= g8[e];
              a[i][kt][e] = (bf16)f;
            }
          }
        }
      }
    }
    const bf16* hi = slab + (size_t)buf * NSLAB * SLAB;
#pragma unroll
    for (int kt = 0; kt < 2; ++kt) {
#pragma unroll
      for (int j = 0; j < TN; ++j) {
#pragma unroll
        for (int h = 0; h < NSLAB; ++h) {
          const bf16* t = hi + h * SLAB;
          bf16x8 wf;
          if constexpr (!BT) {
            const int r = j * 16 + fr;
            wf = *reinterpret_cast<const bf16x8*>(t + r * PG_KP + ((kt * 4 + fg + r) & 7) * 8);
          } else {
            const int r = kt * 32 + 16 * (fg >> 1) + 4 * (fg & 1) + q;  // pg_perm(8 fg + q)
            const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(t + r * BP + j * 16 + p4));
            const s16x4 up = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(t + (r + 8) * BP + j * 16 + p4));
            const s16x8 w8 = {lo[0], lo[1], lo[2], lo[3], up[0], up[1], up[2], up[3]};
            wf = __builtin_bit_cast(bf16x8, w8);
          }
#pragma unroll
          for (int i = 0; i < RS; ++i) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf, a[i][kt], acc[i][j], 0, 0, 0);
        }
      }
    }
  };

  // ---- epilogue of tile j: lane holds out[m = mw + 16 i + fr][n = n0 + 16 jj + 4 fg + r], r = 0..3
  const bf16* res = static_cast<const bf16*>(epi.res);
  const bf16* Z = static_cast<const bf16*>(epi.Z);
  constexpr int JC = TN <= 8 ? TN : TN / 2;  // column fragments per residual / Z round trip
  // output row of GEMM row m: the pixel itself, except for a parity class (its strided pixels)
  auto orow = [&](int m) -> long {
    if constexpr (CV) {
      if (cv.par >= 0) {
        const int h2 = cv.Hr >> 1, w2 = cv.Wr >> 1;
        const int b = m / (h2 * w2), rem = m - b * h2 * w2, Y = rem / w2;
        return ((long)b * cv.Hr + 2 * Y + (cv.par >> 1)) * cv.Wr + 2 * (rem - Y * w2) + (cv.par & 1);
      }
    }
    return m;
  };
  auto epilogue = [&](int j) {
    const int mt = tile_mt(j), n0 = tile_nt(j) * BN, mw = mt * BM + wave * 16 * RS;
    const float* cv = cvec + (j & 1) * 2 * BN;
    if constexpr (LNO) {   // (n0 = 0: the plan has one column tile)
      bf16* lno = static_cast<bf16*>(epi.ln_out);
      const float invN = 1.f / (float)N;
#pragma unroll
      for (int i = 0; i < RS; ++i) {
        const int m = mw + i * 16 + fr;
        const bool mok = m < M;
        const long mc = mok ? m : M - 1;
        const float rsc = epi.rs ? epi.rs[mc / epi.rps] : 1.f;
        uint4 rv[TN / 2];
#pragma unroll
        for (int q = 0; q < TN / 2; ++q) {
          rv[q] = uint4{0u, 0u, 0u, 0u};
          if (res) rv[q] = *reinterpret_cast<const uint4*>(res + mc * ldo + min(32 * q + 8 * fg, N - 8));
        }
        // the stored (rounded) row values replace the accumulators (dead after the epilogue): no extra registers
        float s = 0.f;
#pragma unroll
        for (int q = 0; q < TN / 2; ++q) {
          const int n = 32 * q + 8 * fg;
          const bool ok = mok && n < N;
          const float4 b0 = *reinterpret_cast<const float4*>(cv + n);
          const float4 b1 = *reinterpret_cast<const float4*>(cv + n + 4);
          const float bias[8] = {b0.x, b0.y, b0.z, b0.w, b1.x, b1.y, b1.z, b1.w};
          const bf16* rb = reinterpret_cast<const bf16*>(&rv[q]);
          uint4 ov;
          bf16* ob = reinterpret_cast<bf16*>(&ov);
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            ob[e] = (bf16)((acc[i][2 * q + (e >> 2)][e & 3] + bias[e]) * rsc + (float)rb[e]);
            const float vr = n < N ? (float)ob[e] : 0.f;
            acc[i][2 * q + (e >> 2)][e & 3] = vr;
            s += vr;
          }
          if (ok && !(dbg & 4)) *reinterpret_cast<uint4*>(out + (long)m * ldo + n) = ov;
        }
        s += __shfl_xor(s, 16, 64);
        s += __shfl_xor(s, 32, 64);
        const float mu = s * invN;
        float ss = 0.f;
#pragma unroll
        for (int q = 0; q < TN / 2; ++q) {
          const bool nok = 32 * q + 8 * fg < N;
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            const float d = nok ? acc[i][2 * q + (e >> 2)][e & 3] - mu : 0.f;
            ss = fmaf(d, d, ss);
          }
        }
        ss += __shfl_xor(ss, 16, 64);
        ss += __shfl_xor(ss, 32, 64);
        const float rstd = rsqrtf(ss * invN + epi.ln_eps);
#pragma unroll
        for (int q = 0; q < TN / 2; ++q) {
          const int n = 32 * q + 8 * fg, nc = min(n, N - 8);
          const float4 g0 = *reinterpret_cast<const float4*>(epi.ln_g + nc);
          const float4 g1 = *reinterpret_cast<const float4*>(epi.ln_g + nc + 4);
          const float4 h0 = *reinterpret_cast<const float4*>(epi.ln_b + nc);
          const float4 h1 = *reinterpret_cast<const float4*>(epi.ln_b + nc + 4);
          const float gw[8] = {g0.x, g0.y, g0.z, g0.w, g1.x, g1.y, g1.z, g1.w};
          const float bw[8] = {h0.x, h0.y, h0.z, h0.w, h1.x, h1.y, h1.z, h1.w};
          float o[8];
#pragma unroll
          for (int e = 0; e < 8; ++e) o[e] = (acc[i][2 * q + (e >> 2)][e & 3] - mu) * rstd * gw[e] + bw[e];
          if (mok && n < N) store_vec<bf16, 8>(lno + (long)m * ldo + n, o);
        }
        if (fg == 0 && mok) {
          epi.ln_mean[m] = mu;
          epi.ln_rstd[m] = rstd;
        }
      }
    } else if constexpr (!BT || PG_BT16) {
      // lane: row m, columns 32 q + 8 fg .. + 7 of every fragment pair q (pg_col_slot)
#pragma unroll
      for (int i = 0; i < RS; ++i) {
        const int m = mw + i * 16 + fr;
        const bool mok = m < M;
        // residual / Z / row-scale loads at CLAMPED (always valid) addresses, issued unconditionally under
        // a uniform branch: the compiler then keeps them in flight together (one wait), where per-lane
        // guards made it wait after each load (one HBM round trip per 16-B load, 8 per RS = 2 tile)
        const long mc = mok ? m : M - 1;
        const float rsc = epi.rs ? epi.rs[mc / epi.rps] : 1.f;
        constexpr int QC = (ZA != 0 && TN > 8) ? TN / 4 : TN / 2;   // fragment pairs per residual / Z round trip
#pragma unroll
        for (int q0 = 0; q0 < TN / 2; q0 += QC) {
        uint4 rv[QC], zv[QC];
#pragma unroll
        for (int u = 0; u < QC; ++u) rv[u] = zv[u] = uint4{0u, 0u, 0u, 0u};
        if (res) {
#pragma unroll
          for (int u = 0; u < QC; ++u) {
            const int n = min(n0 + 32 * (q0 + u) + 8 * fg, N - 8);
            rv[u] = *reinterpret_cast<const uint4*>(res + mc * ldo + n);
          }
        }
        if constexpr (ZA != 0) {
#pragma unroll
          for (int u = 0; u < QC; ++u) {
            const int n = min(n0 + 32 * (q0 + u) + 8 * fg, N - 8);
            zv[u] = *reinterpret_cast<const uint4*>(Z + mc * epi.ldz + n);
          }
        }
#pragma unroll
        for (int u = 0; u < QC; ++u) {
          const int q = q0 + u;
          const int c = 32 * q + 8 * fg, n = n0 + c;
          const bool ok = mok && n < N;
          const float4 b0 = *reinterpret_cast<const float4*>(cv + c);
          const float4 b1 = *reinterpret_cast<const float4*>(cv + c + 4);
          const float bias[8] = {b0.x, b0.y, b0.z, b0.w, b1.x, b1.y, b1.z, b1.w};
          const bf16* rb = reinterpret_cast<const bf16*>(&rv[u]);
          const bf16* zb = reinterpret_cast<const bf16*>(&zv[u]);
          uint4 ov;
          bf16* ob = reinterpret_cast<bf16*>(&ov);
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            float x = (acc[i][2 * q + (e >> 2)][e & 3] + bias[e]) * rsc + (float)rb[e];
            if constexpr (ZA != 0) x *= act_grad(ZA, (float)zb[e]);
            ob[e] = (bf16)x;
          }
          if (ok && !(dbg & 4)) *reinterpret_cast<uint4*>(out + orow(m) * ldo + n) = ov;
          if (epi.aout && ok) {
            uint4 av;
            bf16* ab = reinterpret_cast<bf16*>(&av);
#pragma unroll
            for (int e = 0; e < 8; ++e) ab[e] = (bf16)act_fwd(epi.aact, (float)ob[e]);
            *reinterpret_cast<uint4*>(static_cast<bf16*>(epi.aout) + orow(m) * epi.ldao + n) = av;
          }
          if constexpr (STATS) {
#pragma unroll
            for (int h = 0; h < 2; ++h) {   // fragment 2q + h: the same wave-private 16 x 16 pass as below
              const int jj = 2 * q + h;
              bf16* st = stg + wave * 256;
              *reinterpret_cast<uint2*>(st + fr * 16 + 4 * fg) = reinterpret_cast<const uint2*>(&ov)[h];
              __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
              __builtin_amdgcn_wave_barrier();
              __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
              const int cc = pg_slot_col(jj * 16 + fr), nc = n0 + cc;   // this lane's column
              const double sh = (double)cv[BN + cc];
              double t1 = 0.0, t2 = 0.0;
#pragma unroll
              for (int e = 0; e < 4; ++e) {
                const int row = 4 * fg + e;
                if (mw + i * 16 + row < M && nc < N) {
                  const double d = (double)(float)st[row * 16 + fr] - sh;
                  t1 += d;
                  t2 = fma(d, d, t2);
                }
              }
              t1 += __shfl_xor(t1, 16, 64);
              t2 += __shfl_xor(t2, 16, 64);
              t1 += __shfl_xor(t1, 32, 64);
              t2 += __shfl_xor(t2, 32, 64);
              if (fg == 0) {
                double* r1 = red + (wave * 2 + 0) * BN + cc;
                double* r2 = red + (wave * 2 + 1) * BN + cc;
                *r1 = i == 0 ? t1 : *r1 + t1;
                *r2 = i == 0 ? t2 : *r2 + t2;
              }
              __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
              __builtin_amdgcn_wave_barrier();
              __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            }
          }
        }
        }   // q0
      }
    } else {
#pragma unroll
    for (int i = 0; i < RS; ++i) {
      const int m = mw + i * 16 + fr;
      const bool mok = m < M;
      const float rsc = (epi.rs && mok) ? epi.rs[m / epi.rps] : 1.f;
#pragma unroll
      for (int jc = 0; jc < TN; jc += JC) {
        uint2 rv[JC], zv[JC];
#pragma unroll
        for (int u = 0; u < JC; ++u) {  // residual / Z of the chunk first: one round trip
          const int n = n0 + (jc + u) * 16 + 4 * fg;
          rv[u] = uint2{0u, 0u};
          zv[u] = uint2{0u, 0u};
          if (mok && n < N) {
            if (res) rv[u] = *reinterpret_cast<const uint2*>(res + (long)m * ldo + n);
            if constexpr (ZA != 0) zv[u] = *reinterpret_cast<const uint2*>(Z + (long)m * epi.ldz + n);
          }
        }
#pragma unroll
        for (int u = 0; u < JC; ++u) {
          const int jj = jc + u, c = jj * 16 + 4 * fg, n = n0 + c;
          const bool ok = mok && n < N;
          const float4 bs = *reinterpret_cast<const float4*>(cv + c);
          const float bias[4] = {bs.x, bs.y, bs.z, bs.w};
          const bf16* rb = reinterpret_cast<const bf16*>(&rv[u]);
          const bf16* zb = reinterpret_cast<const bf16*>(&zv[u]);
          uint2 ov;
          bf16* ob = reinterpret_cast<bf16*>(&ov);
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            float x = (acc[i][jj][r] + bias[r]) * rsc + (float)rb[r];
            if constexpr (ZA != 0) x *= act_grad(ZA, (float)zb[r]);
            ob[r] = (bf16)x;
          }
          if (ok && !(dbg & 4)) *reinterpret_cast<uint2*>(out + (long)m * ldo + n) = ov;
          if constexpr (STATS) {
            // BatchNorm column sums of the stored values, fp64 from the first add (d = out - shift
            // is exact in fp64), so they do not depend on the shift's value: the 16 x 16 fragment
            // goes through a wave-private LDS tile and comes back one column per lane
            bf16* st = stg + wave * 256;
            *reinterpret_cast<uint2*>(st + fr * 16 + 4 * fg) = ov;
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            const int cc = jj * 16 + fr, nc = n0 + cc;  // this lane's column, rows 4 fg .. 4 fg + 3
            const double sh = (double)cv[BN + cc];
            double t1 = 0.0, t2 = 0.0;
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              const int row = 4 * fg + e;
              if (mw + i * 16 + row < M && nc < N) {
                const double d = (double)(float)st[row * 16 + fr] - sh;
                t1 += d;
                t2 = fma(d, d, t2);
              }
            }
            t1 += __shfl_xor(t1, 16, 64);
            t2 += __shfl_xor(t2, 16, 64);
            t1 += __shfl_xor(t1, 32, 64);
            t2 += __shfl_xor(t2, 32, 64);
            if (fg == 0) {
              double* r1 = red + (wave * 2 + 0) * BN + cc;
              double* r2 = red + (wave * 2 + 1) * BN + cc;
              *r1 = i == 0 ? t1 : *r1 + t1;
              *r2 = i == 0 ? t2 : *r2 + t2;
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
          }
        }
      }
    }
    }   // BT
#pragma unroll
    for (int i = 0; i < RS; ++i)
#pragma unroll
      for (int jj = 0; jj < TN; ++jj) acc[i][jj] = f32x4{0.f, 0.f, 0.f, 0.f};
    if constexpr (STATS) {
      __syncthreads();  // (the previous tile's readers of red passed this tile's k-step barriers)
      for (int c = tid; c < BN; c += PG_NW * 64) {
        if (n0 + c >= N) continue;
        double t1 = 0.0, t2 = 0.0;
#pragma unroll
        for (int w = 0; w < PG_NW; ++w) {  // across the waves, fixed order
          t1 += red[(w * 2 + 0) * BN + c];
          t2 += red[(w * 2 + 1) * BN + c];
        }
        epi.stat[((long)mt * 2 + 0) * N + n0 + c] = t1;
        epi.stat[((long)mt * 2 + 1) * N + n0 + c] = t2;
      }
    }
  };

  // bias / BatchNorm shift of tile j into its parity slot (read by tile j's epilogue only; the slot
  // is rewritten by tile j + 2, after tile j + 1's k-step barriers)
  auto tile_consts = [&](int j) {
    const int n0 = tile_nt(j) * BN;
    float* cv = cvec + (j & 1) * 2 * BN;
    for (int c = tid; c < BN; c += PG_NW * 64) {
      const int n = n0 + c;
      cv[c] = (epi.bias && n < N) ? epi.bias[n] : 0.f;
      cv[BN + c] = (STATS && epi.stat_shift && n < N) ? bn_shift(epi.stat_shift[n]) : 0.f;
    }
  };

  bf16x8 a0[RS][2], a1[RS][2];
  load_w(0);
  load_g(0);
  load_a(0, a0);
  if (total > 1) load_a(1, a1);
  // one barrier per k-step: step g writes buffer g & 1, whose last readers (step g - 2's MFMAs)
  // all passed step g - 1's barrier
  auto step = [&](int g, bf16x8 (&a)[RS][2]) {
    const int j = g / nsteps, s = g - j * nsteps;
    if (s == 0) tile_consts(j);
    store_w(g & 1);
    if (g + 1 < total && !(dbg & 1)) load_w(g + 1);
    __syncthreads();
    compute(s * PG_KB, a, g & 1);
    if constexpr (GT) {
      if (g + 1 < total) load_g(g + 1);
    }
    if (g + 2 < total && !(dbg & 2)) load_a(g + 2, a);
    if (s == nsteps - 1) epilogue(j);
  };
  for (int g = 0; g < total; g += 2) {
    step(g, a0);
    if (g + 1 < total) step(g + 1, a1);
  }
}

// ------------------------------------------------------------------------------------------------
// plan + dispatch
// ------------------------------------------------------------------------------------------------
static int g_pgemm = 1;   // knob "pgemm": route small-M bf16 fwd / dgrad here (0 = tiled kernel)
// knob "pg_split" (bit mask, default 15 = all four bits): bit 1 lets the panel kernel's forward
// launches use the split (hi + lo) weights (when split_w is on), bit 2 its implicit-conv launches,
// bit 4 runs the stride-2 transposed convs as parity classes (pgemm_tconv_try), bit 8 keeps the split
// weights on the launches with an A prologue.
// Bit 8 off (pg_split=7: the launches with an A prologue -- GELU fc2, MBConv project -- multiply by the
// single bf16 weight) measured 18.75-18.77 -> 18.62-18.67 ms/step with the Model-A-7M logits error
// 0.48% -> 0.57% of |ref|, but the 224^2 stage-0 OutGridBlock eval fixture then misses the 1e-2
// bound, so the default keeps every forward split.
static int g_pg_split = 15;  // bit 4: stride-2 transposed convs as parity classes (pgemm_tconv_try);
                             // bit 8: split weights also on the launches with an A prologue
void set_pg_split(int v) { g_pg_split = v & 15; }
static int g_pg_rs = 0;   // knobs "pg_rs" / "pg_tn": force the tile (0 = planner)
static int g_pg_tn = 0;
// knob "pg_per_cu": workgroups per CU the grid is capped at (measured: 8, i.e. one tile per workgroup
// on these shapes, beats 1-2 resident persistent workgroups: the hardware's dynamic dispatch
// balances the tail better than the static tile walk)
static int g_pg_per_cu = 8;
static long g_pg_tn4_max_m = 262144;
static int g_pg_pa_wide = 0;
void set_pg_pa_wide(int v) { g_pg_pa_wide = v ? 1 : 0; }
void set_pg_tn4_max_m(int v) { g_pg_tn4_max_m = v > 0 ? v : 262144; }
void set_pgemm(int v) { g_pgemm = v; }
static int g_pg_lds_kb = 80;  // knob "pg_lds_kb": LDS cap per workgroup the planner allows (80: two per CU)
void set_pg_lds_kb(int v) { g_pg_lds_kb = v < 16 ? 16 : (v > 160 ? 160 : v); }
static int g_pg_dbg = 0;  // knob "pg_dbg" (timing experiments only, wrong results): 1 no weight reloads, 2 no A reloads, 4 no stores
void set_pg_dbg(int v) { g_pg_dbg = v; }
void set_pg_per_cu(int v) { g_pg_per_cu = v < 1 ? 1 : (v > 8 ? 8 : v); }
static int pg_cus() {
  static int cus = 0;
  if (!cus) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
      cus = 256;
  }
  return cus;
}
void set_pg_rs(int v) { g_pg_rs = v; }
void set_pg_tn(int v) { g_pg_tn = v; }

struct PgPlan {
  int ok = 0, RS = 2, TN = 8, nMt = 0, nNt = 0;
  size_t lds = 0;
};

static size_t pg_lds(int TN, bool bt, bool sw, int K, bool pa, bool stats) {
  const size_t slab = bt ? (size_t)PG_KB * (TN * 16 + 16) : (size_t)TN * 16 * PG_KP;
  return 2 * (sw ? 2 : 1) * slab * 2 + 4 * TN * 16 * 4 + (stats ? (size_t)PG_NW * (2 * TN * 16 * 8 + 512) : 0) +
         (pa ? 2 * (size_t)K * 4 : 0);
}

static bool al16p(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

// N = output columns, K = reduction.  Picks (RS, TN): 128-column tiles unless they pad N by more
// than 1/16 (then 192, then 64),
// then enough workgroups (>= 2 per CU) by halving the rows; BatchNorm statistics need the 128-row
// panel (one partial row per gemm_stat_rows panel).
// knob "pg_conv_rs1": 1 (default) lets the implicit-conv forward WITH BatchNorm statistics take 64-row panels
// when 128-row ones would leave fewer than 512 tiles (the caller sizes the partial rows for M / 64): the 7M
// stage-3 downsample (M = 8192, K = 1728) gets two workgroups per CU; 7M 14.751 / 14.769 -> 14.722 / 14.747 ms,
// 14M unchanged (profiles/r05u_pg_conv_rs1.log)
static int g_pg_conv_rs1 = 1;
void set_pg_conv_rs1(int v) { g_pg_conv_rs1 = v ? 1 : 0; }
static PgPlan pg_plan(int M, int N, int K, bool stats, bool sw, bool bt, bool pa, bool gate, bool stats_rs1 = false) {
  PgPlan p;
  if (!g_pgemm || M <= 0 || (N & 7) || (K & 7)) return p;
  // 64-column tiles first at every shape: round 4 re-measured on the whole 7M step (paired 30-step
  // runs on one box, profiles/r04_pgsweep.log): forcing them 15.49-15.52 vs 15.69-15.72 ms with the round-2 rule
  // (64 columns only at M <= 16384 and N < 1024, tools/gpu_pgemm_sweep.sh census) -- the 128 / 192-
  // column tiles need 220-256 VGPRs (two workgroups per CU), the 64-column ones 100-160
  // (knob "pg_tn4_max_m": above it the 128-column tiles come first -- 22M@224's large-M data
  // gradients: 343.6 ms forced 128 vs 347.0 with 64-column tiles)
  // an A prologue (MBConv BN + SiLU + SE gate, GELU) is recomputed for every column tile, so with
  // one there the 128-column tiles come first (knob "pg_pa_wide")
  const bool tn4 = M <= g_pg_tn4_max_m && !(pa && g_pg_pa_wide);
  const int tns[3] = {tn4 ? 4 : 8, tn4 ? 8 : 12, tn4 ? 12 : 4};
  int best_tn = 0;
  for (int t : tns) {
    if (g_pg_tn && t != g_pg_tn) continue;
    // 192-column tiles only as 64-row panels (the 128-row one spills at two waves per SIMD), so
    // never with BatchNorm statistics (128-row partials) or an SE gate (registers)
    if (t == 12 && (gate || stats || N <= 128)) continue;
    const int bn = 16 * t, nnt = (N + bn - 1) / bn;
    if ((long)nnt * bn - N > N / 16 && t != 4 && !g_pg_tn) continue;
    if (pg_lds(t, bt, sw, K, pa, stats) > (size_t)g_pg_lds_kb * 1024) continue;  // two workgroups per CU
    best_tn = t;
    break;
  }
  if (!best_tn) return p;
  p.TN = best_tn;
  p.nNt = (N + 16 * p.TN - 1) / (16 * p.TN);
  p.RS = 2;
  if (p.TN == 12) p.RS = 1;
  else if ((!stats || stats_rs1) && !g_pg_rs) {
    const long wg2 = (long)((M + 127) / 128) * p.nNt;
    if (wg2 < 512) p.RS = 1;
  }
  if (g_pg_rs && !stats && p.TN != 12) p.RS = g_pg_rs;
  p.nMt = (M + 64 * p.RS - 1) / (64 * p.RS);
  p.lds = pg_lds(p.TN, bt, sw, K, pa, stats);
  p.ok = 1;
  return p;
}

// persistent: at most pg_per_cu workgroups per CU (shared by `parts` class groups), a multiple of 8 (keeps
// each one's XCD)
static unsigned pg_grid(const PgPlan& p, int parts = 1) {
  const long vb = (long)((p.nMt + 7) / 8) * 8 * p.nNt;
  return (unsigned)std::max<long>(8, std::min<long>(vb, (long)pg_cus() * g_pg_per_cu / parts / 8 * 8));
}
template <int RS, int TN, int PA, bool GT, int ZA, bool STATS, bool BT, bool SW, bool CV, bool LNO = false>
static void pg_launch(const PgPlan& p, const bf16* A, int lda, const Pro& pro, const float* W, int ldw,
                      const Epi& epi, bf16* out, int ldo, int M, int N, int K, const ConvG& cv, hipStream_t s) {
  if (skip_mask() & 1) return;
  auto kern = pgemm_bf16_kernel<RS, TN, PA, GT, ZA, STATS, BT, SW, CV, LNO>;
  if (!lds_ok(reinterpret_cast<const void*>(kern), p.lds, "pgemm_bf16_kernel")) return;
  // the merged transposed-conv launch: four class groups of cv.cls_G workgroups
  const unsigned grid = (CV && cv.par == 4) ? (unsigned)(4 * cv.cls_G) : pg_grid(p);
  kern<<<grid, PG_NW * 64, p.lds, s>>>(A, lda, pro, W, ldw, epi, out, ldo, M, N, K, p.nMt, p.nNt, g_pg_dbg, cv);
}

template <int PA, bool GT, int ZA, bool STATS, bool BT, bool SW, bool CV = false>
static void pg_tiles(const PgPlan& p, const bf16* A, int lda, const Pro& pro, const float* W, int ldw,
                     const Epi& epi, bf16* out, int ldo, int M, int N, int K, hipStream_t s,
                     const ConvG& cv = ConvG()) {
#define OGV_PG(RS_, TN_) pg_launch<RS_, TN_, PA, GT, ZA, STATS, BT, SW, CV>(p, A, lda, pro, W, ldw, epi, out, ldo, M, N, K, cv, s)
  if (p.RS == 2) {
    if (p.TN == 8) OGV_PG(2, 8);
    else OGV_PG(2, 4);
  } else {
    if constexpr (!STATS) {
      if (p.TN == 12) {
        if constexpr (!GT) OGV_PG(1, 12);
      } else if (p.TN == 8) OGV_PG(1, 8);
      else OGV_PG(1, 4);
    } else if constexpr (CV) {   // 64-row panels with statistics: the implicit-conv forward only
      if (p.TN == 8) OGV_PG(1, 8);
      else OGV_PG(1, 4);
    }
  }
#undef OGV_PG
}

// Returns the BatchNorm partial rows written (>= 1) when handled, 0 otherwise (caller falls back).
int pgemm_fwd_try(const void* A, int lda, const Pro& pro, const float* W, int ldw, void* out, int ldo, int M, int N,
                  int K, const Epi& epi, hipStream_t s) {
  if (!g_pgemm || epi.zact || !al16p(A) || (lda & 7) || !al16p(out) || (ldo & 7) || (ldw & 3) || !al16p(W)) return 0;
  if (epi.res && !al16p(epi.res)) return 0;
  const bool pa = pro.any();
  if (pa && pro.act != OGV_ACT_GELU && pro.act != OGV_ACT_SILU) return 0;
  if (pro.gate && ((pro.gld & 3) || !al16p(pro.gate))) return 0;
  const bool st = epi.stat != nullptr;
  const bool sw = (split_w() & 1) != 0 && (g_pg_split & 1) && (!pa || (g_pg_split & 8));
  const PgPlan p = pg_plan(M, N, K, st, sw, false, pa, pro.gate != nullptr);
  if (!p.ok) return 0;
  const bf16* a = static_cast<const bf16*>(A);
  bf16* o = static_cast<bf16*>(out);
#define OGV_PGF(PA_, GT_, ST_)                                                                           \
  do {                                                                                                   \
    if (sw) pg_tiles<PA_, GT_, 0, ST_, false, true>(p, a, lda, pro, W, ldw, epi, o, ldo, M, N, K, s);   \
    else pg_tiles<PA_, GT_, 0, ST_, false, false>(p, a, lda, pro, W, ldw, epi, o, ldo, M, N, K, s);     \
  } while (0)
  if (!pa) {
    if (st) OGV_PGF(-1, false, true);
    else OGV_PGF(-1, false, false);
  } else if (pro.act == OGV_ACT_GELU && !pro.gate) {
    if (st) OGV_PGF(OGV_ACT_GELU, false, true);
    else OGV_PGF(OGV_ACT_GELU, false, false);
  } else if (pro.act == OGV_ACT_SILU && pro.gate) {
    if (st) OGV_PGF(OGV_ACT_SILU, true, true);
    else OGV_PGF(OGV_ACT_SILU, true, false);
  } else {
    return 0;
  }
#undef OGV_PGF
  return st ? p.nMt : 1;
}

// out = epi(A . W^T) with the next LayerNorm in the epilogue (epi.ln_*): the panel kernel with ONE column tile of
// 64 / 128 / 192 columns holding whole rows (N <= 192), no A prologue, no statistics.  Returns false (nothing
// launched) for a shape it does not take.
bool pgemm_fwd_ln_try(const void* A, int lda, const float* W, int ldw, void* out, int ldo, int M, int N, int K,
                      const Epi& epi, hipStream_t s) {
  if (!g_pgemm || M <= 0 || N > 192 || (N & 7) || (K & 7) || epi.zact || epi.stat || epi.aout || !epi.ln_out ||
      !epi.ln_g || !epi.ln_b || !epi.ln_mean || !epi.ln_rstd)
    return false;
  if (!al16p(A) || (lda & 7) || !al16p(out) || (ldo & 7) || (ldw & 3) || !al16p(W) || !al16p(epi.ln_out) ||
      !al16p(epi.ln_g) || !al16p(epi.ln_b) || (epi.res && !al16p(epi.res)))
    return false;
  const bool sw = (split_w() & 1) != 0 && (g_pg_split & 1);
  PgPlan p;
  p.TN = N <= 64 ? 4 : (N <= 128 ? 8 : 12);
  p.nNt = 1;
  p.RS = (p.TN == 12 || (long)((M + 127) / 128) < 512) ? 1 : 2;
  p.nMt = (M + 64 * p.RS - 1) / (64 * p.RS);
  p.lds = pg_lds(p.TN, false, sw, K, false, false);
  if (p.lds > (size_t)g_pg_lds_kb * 1024) return false;
  p.ok = 1;
  const bf16* a = static_cast<const bf16*>(A);
  bf16* o = static_cast<bf16*>(out);
#define OGV_PGL(RS_, TN_)                                                                                          \
  do {                                                                                                             \
    if (sw) pg_launch<RS_, TN_, -1, false, 0, false, false, true, false, true>(p, a, lda, Pro(), W, ldw, epi, o, ldo, M, N, K, ConvG(), s); \
    else pg_launch<RS_, TN_, -1, false, 0, false, false, false, false, true>(p, a, lda, Pro(), W, ldw, epi, o, ldo, M, N, K, ConvG(), s); \
  } while (0)
  if (p.TN == 12) OGV_PGL(1, 12);
  else if (p.TN == 8) { if (p.RS == 2) OGV_PGL(2, 8); else OGV_PGL(1, 8); }
  else { if (p.RS == 2) OGV_PGL(2, 4); else OGV_PGL(1, 4); }
#undef OGV_PGL
  return true;
}

// dA[M, Kf] = epi(dOut[M, Nf] . W[Nf, Kf]): reduction Nf, output columns Kf.
bool pgemm_dgrad_try(const void* dout, int ldd, const float* W, void* dA, int lda, int M, int Nf, int Kf,
                     const Epi& epi, hipStream_t s) {
  if (!g_pgemm || epi.stat || !al16p(dout) || (ldd & 7) || !al16p(dA) || (lda & 7) || (Kf & 3) || !al16p(W))
    return false;
  if (epi.res && !al16p(epi.res)) return false;
  if (epi.zact && (!epi.Z || !al16p(epi.Z) || (epi.ldz & 7))) return false;
  if (epi.zact != OGV_ACT_NONE && epi.zact != OGV_ACT_GELU && epi.zact != OGV_ACT_SILU) return false;
  const bool sw = (split_w() & 2) != 0;
  const PgPlan p = pg_plan(M, Kf, Nf, false, sw, true, false, false);
  if (!p.ok) return false;
  const bf16* a = static_cast<const bf16*>(dout);
  bf16* o = static_cast<bf16*>(dA);
#define OGV_PGD(ZA_)                                                                                      \
  do {                                                                                                    \
    if (sw) pg_tiles<-1, false, ZA_, false, true, true>(p, a, ldd, Pro(), W, Kf, epi, o, lda, M, Kf, Nf, s); \
    else pg_tiles<-1, false, ZA_, false, true, false>(p, a, ldd, Pro(), W, Kf, epi, o, lda, M, Kf, Nf, s);  \
  } while (0)
  if (epi.zact == OGV_ACT_GELU) OGV_PGD(OGV_ACT_GELU);
  else if (epi.zact == OGV_ACT_SILU) OGV_PGD(OGV_ACT_SILU);
  else OGV_PGD(0);
#undef OGV_PGD
  return true;
}

// Stride-2 transposed conv (a downsample's data gradient) as four parity-class GEMMs: output pixel
// (y, x) only receives taps with ky = y + 1 (mod 2), kx = x + 1 (mod 2), i.e. 1, 2, 2 or 4 of the 9
// (K / 2.25 on average, no zero taps staged or multiplied).  Returns false (nothing launched) when
// a class does not fit the panel kernel.
// knob "pg_tconv1" 1 (default) / 0: the four parity classes as ONE launch (workgroup groups per class) / four
static int g_pg_tconv1 = 1;
void set_pg_tconv1(int v) { g_pg_tconv1 = v ? 1 : 0; }
bool pgemm_tconv_try(const void* A, const ConvG& cv, const float* Wt, void* out, int M, int N, hipStream_t s) {
  if (!g_pgemm || !(g_pg_split & 4) || !cv.transposed || cv.stride != 2 || (cv.Hr & 1) || (cv.Wr & 1) || (cv.Cs & 7) ||
      !al16p(A) || !al16p(out) || !al16p(Wt) || M % (cv.Hr * cv.Wr))
    return false;
  const bool sw = (split_w() & 2) != 0;
  const int Mc = M / 4;
  ConvG g[4];
  PgPlan p[4];
  for (int par = 0; par < 4; ++par) {
    g[par] = cv;
    g[par].par = par;
    const int kys[2][2] = {{1, -1}, {0, 2}};
    int nt = 0;
    for (int a = 0; a < 2; ++a)
      for (int b = 0; b < 2; ++b) {
        const int ky = kys[par >> 1][a], kx = kys[par & 1][b];
        if (ky >= 0 && kx >= 0) g[par].tap[nt++] = ky * 3 + kx;
      }
    g[par].ntap = nt;
    p[par] = pg_plan(Mc, N, nt * cv.Cs, false, sw, false, false, false);
    if (!p[par].ok) return false;
  }
  const bf16* a = static_cast<const bf16*>(A);
  bf16* o = static_cast<bf16*>(out);
  if (g_pg_tconv1 && p[0].RS == p[3].RS && p[0].TN == p[3].TN) {
    // one launch for the four classes (same tile plan: the plan depends on the rows and columns only)
    ConvG g4 = cv;
    g4.par = 4;
    g4.cls_G = (int)pg_grid(p[3], 4);
    PgPlan p4 = p[3];
    for (int par = 0; par < 4; ++par) p4.lds = std::max(p4.lds, p[par].lds);
    const int K4 = 4 * cv.Cs;   // (each class group uses its own K)
    if (sw) pg_tiles<-1, false, 0, false, false, true, true>(p4, a, 0, Pro(), Wt, 9 * cv.Cs, Epi(), o, N, Mc, N, K4, s, g4);
    else pg_tiles<-1, false, 0, false, false, false, true>(p4, a, 0, Pro(), Wt, 9 * cv.Cs, Epi(), o, N, Mc, N, K4, s, g4);
    return true;
  }
  for (int par = 0; par < 4; ++par) {
    const int K = g[par].ntap * cv.Cs;
    if (sw) pg_tiles<-1, false, 0, false, false, true, true>(p[par], a, 0, Pro(), Wt, 9 * cv.Cs, Epi(), o, N, Mc, N, K, s, g[par]);
    else pg_tiles<-1, false, 0, false, false, false, true>(p[par], a, 0, Pro(), Wt, 9 * cv.Cs, Epi(), o, N, Mc, N, K, s, g[par]);
  }
  return true;
}

// Implicit-GEMM 3x3 conv (ogv_convbn forward): out[M, N] = epi(gather(A; cv)[M, 9 Cs] . Wt[N, 9 Cs]^T).
// Returns the BatchNorm partial rows written (>= 1) when handled, 0 otherwise (caller falls back).
int pgemm_conv_try(const void* A, const ConvG& cv, const float* Wt, void* out, int M, int N, const Epi& epi,
                   hipStream_t s) {
  const int K = 9 * cv.Cs;
  // forward convs only: measured (7M step, rocprofv3) downsample fwd + BN stats 113 -> 67 us, but the
  // stride-2 transposed convs of the data gradient (3 of 4 taps empty per output) 144 -> 225 us
  if (!g_pgemm || cv.transposed || (cv.Cs & 7) || !al16p(A) || !al16p(out) || !al16p(Wt) || epi.zact || epi.res)
    return 0;
  const bool st = epi.stat != nullptr;
  const bool sw = (split_w() & (cv.transposed ? 2 : 1)) != 0 && (g_pg_split & 2);
  const PgPlan p = pg_plan(M, N, K, st, sw, false, false, false, g_pg_conv_rs1 != 0);
  if (!p.ok) return 0;
  const bf16* a = static_cast<const bf16*>(A);
  bf16* o = static_cast<bf16*>(out);
  if (st) {
    if (sw) pg_tiles<-1, false, 0, true, false, true, true>(p, a, 0, Pro(), Wt, K, epi, o, N, M, N, K, s, cv);
    else pg_tiles<-1, false, 0, true, false, false, true>(p, a, 0, Pro(), Wt, K, epi, o, N, M, N, K, s, cv);
  } else {
    if (sw) pg_tiles<-1, false, 0, false, false, true, true>(p, a, 0, Pro(), Wt, K, epi, o, N, M, N, K, s, cv);
    else pg_tiles<-1, false, 0, false, false, false, true>(p, a, 0, Pro(), Wt, K, epi, o, N, M, N, K, s, cv);
  }
  return st ? p.nMt : 1;
}

bool pgemm_route(int kind, int M, int N, int K, int act) {
  if (kind == 0) {
    if (act != OGV_ACT_NONE && act != OGV_ACT_GELU && act != OGV_ACT_SILU) return false;
    return pg_plan(M, N, K, false, (split_w() & 1) != 0 && (g_pg_split & 1) && (act == OGV_ACT_NONE || (g_pg_split & 8)),
                   false, act != OGV_ACT_NONE, false).ok;
  }
  return pg_plan(M, K, N, false, (split_w() & 2) != 0, true, false, false).ok;  // dgrad: output K
}

}  // namespace ogv
