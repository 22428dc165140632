// The stem convolution of MaxOutNet (Conv2d(3, stem, 3, 1, 1) -> BN -> SiLU, src/model/stem_head.py:23-32)
// on dedicated kernels: with C_in = 3 the implicit GEMM has a 27-column reduction, so the generic
// conv kernels (8 | C_in gathers, or the LDS-tiled kernel's per-element gather over 32-wide k
// slabs) spend their time on addressing, not on the 67 MB output stream.  Here one 128-pixel tile
// builds its whole im2col block [128][32] in LDS once -- gathered per pixel (forward, StemCols) or
// from the input rows staged with 16-B loads (weight gradient, StemPatch) -- (k = tap * C_in + c,
// zero padding; k = 27 is a column of ones in the weight gradient, giving the bias gradient from
// the same MFMAs), and:
//   forward:  y = im2col . W^T (+ bias) on v_mfma_f32_16x16x32_bf16 with the weight held in
//             registers as bf16 hi + lo for the whole tile (the split-weight forward of the other
//             projections), transposed product so a lane stores 4 consecutive channels; BatchNorm
//             batch statistics of the rounded output (shifted by the running mean, the GEMM
//             epilogues' convention), one fp64 partial row per workgroup of up to 8 tiles;
//   weight gradient: split-M, each workgroup walks its rows in 128-row steps with the im2col block
//             and the dy block staged TRANSPOSED in LDS ([k][m], [n][m]: the MFMA operands are then
//             16-B row reads), the next step's raw loads in registers while the current one is
//             multiplied, one [N*K9 | N] partial row per workgroup, summed by one colreduce.
#include "ogv_gemm.h"

namespace ogv {

constexpr int ST_BM = 128;        // pixels per tile (= GEMM_BM: one BN partial row per tile)
constexpr int ST_AP = 40;         // forward im2col pitch [m][k] (bf16): 80-B rows
constexpr int ST_TP = ST_BM + 8;  // transposed pitch [k][m] / [n][m] (bf16)

struct StemG {
  int B, H, W, Ho, Wo, stride;
};

// Forward: the 16 im2col values of pixel p = tid >> 1, columns [16 h, 16 h + 16) (h = tid & 1), of the
// tile starting at output row m0, gathered straight from HBM / L2 at clamped (always valid) addresses,
// zeros selected after (measured faster for the forward than the LDS patch: 90.7 vs 99.9 us per
// stem op, tools/bench_stem.py, profiles/r04_stem_bench.log; the weight gradient is faster with it)
template <int CIN>
struct StemCols {
  bf16 raw[16];
  __device__ __forceinline__ void load(const bf16* __restrict__ x, const StemG& g, long m0, long M) {
    constexpr int K9 = 9 * CIN;
    const int p = threadIdx.x >> 1, h = threadIdx.x & 1;
    const long m = m0 + p < M ? m0 + p : M - 1;
    const int hw = g.Ho * g.Wo;
    const int b = (int)(m / hw), rem = (int)(m - (long)b * hw), oy = rem / g.Wo, ox = rem - oy * g.Wo;
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      const int k = 16 * h + j;
      const int tap = k / CIN, c = k - tap * CIN, ky = tap / 3, kx = tap - 3 * ky;
      const int sy = oy * g.stride - 1 + ky, sx = ox * g.stride - 1 + kx;
      const bool ok = k < K9 && sy >= 0 && sy < g.H && sx >= 0 && sx < g.W;
      raw[j] = x[ok ? (((long)b * g.H + sy) * g.W + sx) * CIN + c : 0];
      ok_[j] = ok;
    }
  }
  bool ok_[16];
  // value j after the zero padding (ONES: column K9 = 1 for the bias gradient)
  template <bool ONES>
  __device__ __forceinline__ bf16 value(int j) const {
    const int k = 16 * (threadIdx.x & 1) + j;
    return ok_[j] ? raw[j] : (ONES && k == 9 * CIN ? (bf16)1.f : (bf16)0.f);
  }
};

// The input a tile needs, staged in LDS: the contiguous range of source rows (flattened b * H + y,
// NHWC rows are contiguous, so a tile spanning images is still one range) from the row above its
// first output row to the row below its last, fetched with 16-B loads (SP_CH per thread, issued a
// tile ahead into registers) -- instead of 27 two-byte gathers per output pixel, which made the
// load-instruction rate the bound (60 us for the 7M stem forward).  The host checks that a tile's
// range fits SP_CH * 256 chunks and that the tensor is a whole number of 16-B chunks.
constexpr int SP_CH = 2;
constexpr int SP_ELEMS = SP_CH * 256 * 8;
template <int CIN>
struct StemPatch {
  uint4 raw[SP_CH];
  long base = 0;   // first staged element (a multiple of 8)
  int nchunk = 0;
  __device__ __forceinline__ void load(const bf16* __restrict__ x, const StemG& g, long m0, long M) {
    const long ml = m0 + ST_BM - 1 < M ? m0 + ST_BM - 1 : M - 1;
    const int hw = g.Ho * g.Wo;
    const long b0 = m0 / hw, b1 = ml / hw;
    const int oy0 = (int)((m0 - b0 * hw) / g.Wo), oy1 = (int)((ml - b1 * hw) / g.Wo);
    const long rlo = b0 * g.H + max(oy0 * g.stride - 1, 0), rhi = b1 * g.H + min(oy1 * g.stride + 1, g.H - 1);
    base = (rlo * g.W * CIN) & ~7L;
    nchunk = (int)(((rhi + 1) * g.W * CIN - base + 7) >> 3);
#pragma unroll
    for (int c = 0; c < SP_CH; ++c) {
      const int idx = min((int)threadIdx.x + c * 256, nchunk - 1);
      raw[c] = *reinterpret_cast<const uint4*>(x + base + (long)idx * 8);
    }
  }
  __device__ __forceinline__ void store(bf16* P) const {
#pragma unroll
    for (int c = 0; c < SP_CH; ++c) {
      const int idx = (int)threadIdx.x + c * 256;
      if (idx < nchunk) *reinterpret_cast<uint4*>(P + idx * 8) = raw[c];
    }
  }
  // im2col values of pixel p = tid >> 1 of the tile at m0, columns [16 h, 16 h + 16) (h = tid & 1),
  // from the staged patch (zero padding; ONES: column K9 = 1 for the bias gradient, valid pixels)
  template <bool ONES>
  __device__ __forceinline__ void cols(const bf16* P, const StemG& g, long m0, long M, bf16 (&v)[16]) const {
    constexpr int K9 = 9 * CIN;
    const int p = threadIdx.x >> 1, h = threadIdx.x & 1;
    const bool mok = m0 + p < M;
    const long m = mok ? m0 + p : M - 1;
    const int hw = g.Ho * g.Wo;
    const long b = m / hw;
    const int rem = (int)(m - b * hw), oy = rem / g.Wo, ox = rem - oy * g.Wo;
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      const int k = 16 * h + j;
      const int tap = k / CIN, c = k - tap * CIN, ky = tap / 3, kx = tap - 3 * ky;
      const int sy = oy * g.stride - 1 + ky, sx = ox * g.stride - 1 + kx;
      const bool ok = mok && k < K9 && sy >= 0 && sy < g.H && sx >= 0 && sx < g.W;
      const long off = ok ? ((b * g.H + sy) * g.W + sx) * CIN + c - base : 0;
      const bf16 e = P[off];
      v[j] = ok ? e : (ONES && mok && k == K9 ? (bf16)1.f : (bf16)0.f);
    }
  }
};

// A workgroup walks tpb consecutive 128-pixel tiles (the next tile's im2col gathers in flight while
// the current one is multiplied and stored); BN statistics accumulate per lane over its tiles and
// are reduced once per workgroup into partial row blockIdx.x.
template <int CIN, int NJ, bool STATS>
__global__ __launch_bounds__(256) void stem_fwd_kernel(const bf16* __restrict__ x, const float* __restrict__ wt,
                                                       const float* __restrict__ bias, bf16* __restrict__ out,
                                                       double* __restrict__ stat, const float* __restrict__ shift,
                                                       StemG g, long M, int tpb) {
  constexpr int K9 = 9 * CIN, N = 16 * NJ;
  __shared__ __attribute__((aligned(16))) bf16 A[ST_BM * ST_AP];
  __shared__ double red[STATS ? 4 : 1][2][N];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, fr = lane & 15, fg = lane >> 4;
  const long t0 = (long)blockIdx.x * tpb;
  // weight fragments (A operand): n-block j, lane (fr, fg) = W[16 j + fr][8 fg .. 8 fg + 7], hi + lo
  bf16x8 whi[NJ], wlo[NJ];
  float bv[NJ][4], sft[NJ][4];
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int k = 8 * fg + e;
      const float w = wt[(16 * j + fr) * K9 + (k < K9 ? k : 0)];
      const float wv = k < K9 ? w : 0.f;
      const bf16 hi = (bf16)wv;
      whi[j][e] = hi;
      wlo[j][e] = (bf16)(wv - (float)hi);
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      bv[j][r] = bias ? bias[16 * j + 4 * fg + r] : 0.f;
      sft[j][r] = STATS ? bn_shift(shift[16 * j + 4 * fg + r]) : 0.f;
    }
  }
  // fp64 per lane from the first term on: y - shift is exact in fp64 (a bf16 minus an fp32), so the
  // statistics -- and through them the rounded output -- do not move with the running-mean shift
  // (an fp32 per-lane partial did, by one bf16 ulp of the output: measured, tools/diag_stem.py)
  double s1[STATS ? NJ : 1][4], s2[STATS ? NJ : 1][4];
#pragma unroll
  for (int j = 0; j < (STATS ? NJ : 1); ++j)
#pragma unroll
    for (int r = 0; r < 4; ++r) { s1[j][r] = 0.0; s2[j][r] = 0.0; }
  StemCols<CIN> cols;
  cols.load(x, g, t0 * ST_BM, M);
  for (int t = 0; t < tpb; ++t) {
    const long m0 = (t0 + t) * ST_BM;
    if (m0 >= M) break;
    {
      bf16x8 v0, v1;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        v0[j] = cols.template value<false>(j);
        v1[j] = cols.template value<false>(8 + j);
      }
      bf16* d = A + (threadIdx.x >> 1) * ST_AP + 16 * (threadIdx.x & 1);
      *reinterpret_cast<bf16x8*>(d) = v0;
      *reinterpret_cast<bf16x8*>(d + 8) = v1;
    }
    __syncthreads();
    if (t + 1 < tpb && m0 + ST_BM < M) cols.load(x, g, m0 + ST_BM, M);   // next tile's gathers in flight
    bf16x8 a[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) a[i] = *reinterpret_cast<const bf16x8*>(A + (wave * 32 + 16 * i + fr) * ST_AP + 8 * fg);
    __syncthreads();   // A is restaged by the next tile
    f32x4 acc[2][NJ];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(whi[j], a[i], f32x4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wlo[j], a[i], acc[i][j], 0, 0, 0);
      }
    // lane holds y[m = m0 + 32 wave + 16 i + fr][n = 16 j + 4 fg + r]
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const long m = m0 + wave * 32 + 16 * i + fr;
      const bool mok = m < M;
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        bf16x4 o;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          o[r] = (bf16)(acc[i][j][r] + bv[j][r]);
          if constexpr (STATS) {
            const double dl = mok ? (double)(float)o[r] - (double)sft[j][r] : 0.0;
            s1[j][r] += dl;
            s2[j][r] = fma(dl, dl, s2[j][r]);
          }
        }
        if (mok) *reinterpret_cast<bf16x4*>(out + m * N + 16 * j + 4 * fg) = o;
      }
    }
  }
  if constexpr (STATS) {
    // per-lane partials -> across the 16 lanes of a column group, then the 4 waves
#pragma unroll
    for (int j = 0; j < NJ; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        double d1 = s1[j][r], d2 = s2[j][r];
#pragma unroll
        for (int o = 1; o < 16; o <<= 1) {
          d1 += __shfl_xor(d1, o, 64);
          d2 += __shfl_xor(d2, o, 64);
        }
        if (fr == 0) {
          red[wave][0][16 * j + 4 * fg + r] = d1;
          red[wave][1][16 * j + 4 * fg + r] = d2;
        }
      }
    __syncthreads();
    for (int t = threadIdx.x; t < 2 * N; t += 256) {
      const int q = t / N, n = t - q * N;
      stat[((long)blockIdx.x * 2 + q) * N + n] = ((red[0][q][n] + red[1][q][n]) + red[2][q][n]) + red[3][q][n];
    }
  }
}

// dW[n][k] (+ dbias[n] via the ones column k = K9) over rows [blk * rpb, (blk + 1) * rpb)
template <int CIN, int NJ>
__global__ __launch_bounds__(256) void stem_wgrad_kernel(const bf16* __restrict__ x, const bf16* __restrict__ dy,
                                                         float* __restrict__ part, long ldp, bool has_bias, StemG g,
                                                         long M, long rpb) {
  constexpr int K9 = 9 * CIN, N = 16 * NJ;
  constexpr int NT = 2 * NJ;                // 16 x 16 output tiles: NJ n-blocks x 2 k-blocks
  constexpr int TPW = (NT + 3) / 4;         // tiles per wave
  constexpr int DL = ST_BM * N / 8 / 256;   // 16-B dy loads per thread and step
  __shared__ __attribute__((aligned(16))) bf16 AT[32 * ST_TP];
  __shared__ __attribute__((aligned(16))) bf16 DT[N * ST_TP];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, fr = lane & 15, fg = lane >> 4;
  const long r0 = (long)blockIdx.x * rpb, r1 = r0 + rpb < M ? r0 + rpb : M;
  f32x4 acc[TPW];
#pragma unroll
  for (int t = 0; t < TPW; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
  __shared__ __attribute__((aligned(16))) bf16 P[SP_ELEMS];
  StemPatch<CIN> patch;
  uint4 dr[DL];
  auto load = [&](long s0) {
    patch.load(x, g, s0, M);
#pragma unroll
    for (int u = 0; u < DL; ++u) {
      const int idx = threadIdx.x + u * 256, p = idx / (N / 8), c8 = (idx - p * (N / 8)) * 8;
      const long m = s0 + p < M ? s0 + p : M - 1;
      dr[u] = *reinterpret_cast<const uint4*>(dy + m * N + c8);
    }
  };
  load(r0);
  for (long s0 = r0; s0 < r1; s0 += ST_BM) {
    // stage step s0 transposed (rows past the range / the tensor: zeros in both operands)
    patch.store(P);
    __syncthreads();
    {
      const int p = threadIdx.x >> 1, h = threadIdx.x & 1;
      const bool pok = s0 + p < r1;
      bf16 v[16];
      patch.template cols<true>(P, g, s0, M, v);
#pragma unroll
      for (int j = 0; j < 16; ++j) AT[(16 * h + j) * ST_TP + p] = pok ? v[j] : (bf16)0.f;
#pragma unroll
      for (int u = 0; u < DL; ++u) {
        const int idx = threadIdx.x + u * 256, q = idx / (N / 8), c8 = (idx - q * (N / 8)) * 8;
        const bool qok = s0 + q < r1;
        const bf16* e = reinterpret_cast<const bf16*>(&dr[u]);
#pragma unroll
        for (int i = 0; i < 8; ++i) DT[(c8 + i) * ST_TP + q] = qok ? e[i] : (bf16)0.f;
      }
    }
    __syncthreads();
    if (s0 + ST_BM < r1) load(s0 + ST_BM);   // next step's raw loads in flight during the MFMAs
#pragma unroll
    for (int t = 0; t < TPW; ++t) {
      const int tile = wave + 4 * t;
      if (tile < NT) {
        const int j = tile >> 1, kb = tile & 1;
#pragma unroll
        for (int mc = 0; mc < ST_BM / 32; ++mc) {
          const bf16x8 da = *reinterpret_cast<const bf16x8*>(DT + (16 * j + fr) * ST_TP + 32 * mc + 8 * fg);
          const bf16x8 xb = *reinterpret_cast<const bf16x8*>(AT + (16 * kb + fr) * ST_TP + 32 * mc + 8 * fg);
          acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(da, xb, acc[t], 0, 0, 0);
        }
      }
    }
    __syncthreads();
  }
  // lane holds dW[n = 16 j + 4 fg + r][k = 16 kb + fr]
  float* row = part + (long)blockIdx.x * ldp;
#pragma unroll
  for (int t = 0; t < TPW; ++t) {
    const int tile = wave + 4 * t;
    if (tile < NT) {
      const int j = tile >> 1, kb = tile & 1, k = 16 * kb + fr;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int n = 16 * j + 4 * fg + r;
        if (k < K9) row[n * K9 + k] = acc[t][r];
        else if (k == K9 && has_bias) row[N * K9 + n] = acc[t][r];
      }
    }
  }
}

static int g_stem = 1;   // knob "stem": 1 (default) = the dedicated stem kernels where they apply
void set_stem(int v) { g_stem = v; }

// 32 or 64 output channels (the Model-A / B stems are 64 wide; wider stems take the generic conv
// kernels: the fp64 statistics accumulators of NJ > 4 column blocks do not fit the register budget)
static bool stem_ok(int Cin, int N) { return g_stem && Cin >= 1 && Cin <= 3 && (N == 32 || N == 64); }

// the staged input range of any tile fits the LDS patch, and the tensor is whole 16-B chunks
static bool stem_patch_ok(const void* x, const ConvG& cv, long M) {
  const long B = M / ((long)cv.Hr * cv.Wr);
  const long total = B * cv.Hs * cv.Ws * cv.Cs;
  const long rows_out = (ST_BM + cv.Wr - 1) / cv.Wr + 1;
  const long rows_in = rows_out * cv.stride + 3;
  return (reinterpret_cast<uintptr_t>(x) & 15) == 0 && total % 8 == 0 &&
         rows_in * cv.Ws * cv.Cs + 8 <= SP_ELEMS;
}

static StemG stem_geom(const ConvG& cv) {
  return StemG{0, cv.Hs, cv.Ws, cv.Hr, cv.Wr, cv.stride};
}

// tiles per forward workgroup: ~g_stem_wgs workgroups, at most 8 tiles each (knob "stem_wgs")
static int g_stem_wgs = 512;
void set_stem_wgs(int v) { g_stem_wgs = v > 0 ? v : 512; }
static int stem_tpb(long M) {
  const long tiles = (M + ST_BM - 1) / ST_BM;
  long t = tiles / g_stem_wgs;
  return (int)(t < 1 ? 1 : (t > 8 ? 8 : t));
}
int stem_fwd_stat_rows(long M) {
  const long tiles = (M + ST_BM - 1) / ST_BM, tpb = stem_tpb(M);
  return (int)((tiles + tpb - 1) / tpb);
}

bool stem_fwd_try(const void* x, const ConvG& cv, const float* wt, void* out, int M, int N, const Epi& epi,
                  hipStream_t s, int* stat_rows) {
  if (!stem_ok(cv.Cs, N) || cv.transposed || epi.res || epi.rs || epi.zact || epi.Z) return false;
  const StemG g = stem_geom(cv);
  const int tpb = stem_tpb(M);
  const unsigned grid = (unsigned)stem_fwd_stat_rows(M);
  if (stat_rows) *stat_rows = (int)grid;
  const bool st = epi.stat != nullptr;
#define OGV_STEM_F(CIN, NJ)                                                                                       \
  if (st) stem_fwd_kernel<CIN, NJ, true><<<grid, 256, 0, s>>>((const bf16*)x, wt, epi.bias, (bf16*)out, epi.stat, \
                                                              epi.stat_shift, g, M, tpb);                         \
  else stem_fwd_kernel<CIN, NJ, false><<<grid, 256, 0, s>>>((const bf16*)x, wt, epi.bias, (bf16*)out, nullptr,   \
                                                            nullptr, g, M, tpb);
#define OGV_STEM_NJ(CIN)                   \
  switch (N / 16) {                        \
    case 2: OGV_STEM_F(CIN, 2) break;      \
    case 4: OGV_STEM_F(CIN, 4) break;      \
    default: return false;                 \
  }
  switch (cv.Cs) {
    case 1: OGV_STEM_NJ(1) break;
    case 2: OGV_STEM_NJ(2) break;
    default: OGV_STEM_NJ(3) break;
  }
#undef OGV_STEM_NJ
#undef OGV_STEM_F
  return true;
}

// workgroups of the weight gradient: ~2 per CU, >= 4 steps of 128 rows each
static long stem_wg_blocks(long M) {
  long S = 512;
  while (S > 1 && M / S < 4 * ST_BM) S >>= 1;
  return S;
}
size_t stem_wgrad_ws_bytes(long M, int N, int Cin) {
  const long S = stem_wg_blocks(M), ld = (long)N * 9 * Cin + N;
  return ((size_t)S * ld + colreduce_tmp_floats(S, ld) + 64) * sizeof(float);
}

bool stem_wgrad_try(const void* x, const ConvG& cv, const void* dy, float* dw, float* dbias, int M, int N, void* ws,
                    hipStream_t s) {
  if (!stem_ok(cv.Cs, N) || cv.transposed || !stem_patch_ok(x, cv, M)) return false;
  const StemG g = stem_geom(cv);
  const int K9 = 9 * cv.Cs;
  const long S = stem_wg_blocks(M), ld = (long)N * K9 + N;
  const long rpb = ((M + S - 1) / S + ST_BM - 1) / ST_BM * ST_BM;
  const long nb = (M + rpb - 1) / rpb;
  float* part = static_cast<float*>(ws);
  float* tmp = part + S * ld;
  const bool hb = dbias != nullptr;
#define OGV_STEM_W(CIN, NJ) \
  stem_wgrad_kernel<CIN, NJ><<<(unsigned)nb, 256, 0, s>>>((const bf16*)x, (const bf16*)dy, part, ld, hb, g, M, rpb);
#define OGV_STEM_WNJ(CIN)                  \
  switch (N / 16) {                        \
    case 2: OGV_STEM_W(CIN, 2) break;      \
    case 4: OGV_STEM_W(CIN, 4) break;      \
    default: return false;                 \
  }
  switch (cv.Cs) {
    case 1: OGV_STEM_WNJ(1) break;
    case 2: OGV_STEM_WNJ(2) break;
    default: OGV_STEM_WNJ(3) break;
  }
#undef OGV_STEM_WNJ
#undef OGV_STEM_W
  colreduce(part, dw, nb, hb ? ld : (long)N * K9, ld, tmp, s, hb ? dbias : nullptr, (long)N * K9);
  return true;
}

}  // namespace ogv
