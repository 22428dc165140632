// Internal (C++) GEMM launchers shared by the C-ABI wrappers and the fused MBConv.
#pragma once
#include "ogv_common.h"

namespace ogv {

// A-operand prologue, applied while staging A (fwd) or X (wgrad) tiles:
//   a' = act(a * sc[k] + sh[k]) * gate[(m / rps) * gld + k]      (each factor optional)
// Elements outside [0, M) x [0, Ka) stay exactly zero.
struct Pro {
  int act = OGV_ACT_NONE;
  const float* sc = nullptr;
  const float* sh = nullptr;
  const float* gate = nullptr;
  int rps = 1, gld = 0;
  bool any() const { return act != OGV_ACT_NONE || sc || sh || gate; }
};

__device__ __forceinline__ float pro_apply(const Pro& p, float v, int m, int k) {
  if (p.sc) v *= p.sc[k];
  if (p.sh) v += p.sh[k];
  v = act_fwd(p.act, v);
  if (p.gate) v *= p.gate[(long)(m / p.rps) * p.gld + k];
  return v;
}

// E consecutive columns k..k+E-1 of row m; per-column parameters fetched as vectors when the
// run is full and 16-B aligned (k % 4 == 0, gld % 4 == 0), element-wise otherwise.
template <int E>
__device__ __forceinline__ void pro_apply_run(const Pro& p, float (&v)[E], int m, int k, int Ka) {
  if (k + E <= Ka && (k & 3) == 0 && (p.gld & 3) == 0) {
    if (p.sc) {
      float t[E];
      load_vec<float, E>(p.sc + k, t);
#pragma unroll
      for (int i = 0; i < E; ++i) v[i] *= t[i];
    }
    if (p.sh) {
      float t[E];
      load_vec<float, E>(p.sh + k, t);
#pragma unroll
      for (int i = 0; i < E; ++i) v[i] += t[i];
    }
#pragma unroll
    for (int i = 0; i < E; ++i) v[i] = act_fwd(p.act, v[i]);
    if (p.gate) {
      float t[E];
      load_vec<float, E>(p.gate + (long)(m / p.rps) * p.gld + k, t);
#pragma unroll
      for (int i = 0; i < E; ++i) v[i] *= t[i];
    }
  } else {
#pragma unroll
    for (int i = 0; i < E; ++i)
      if (k + i < Ka) v[i] = pro_apply(p, v[i], m, k + i);
  }
}

// Epilogue: out = res + rs[m/rps] * (acc + bias[n]);  out *= act'(Z[m,n]) (zact);
// optional per-column batch statistics of the stored (rounded) output, accumulated in fp64:
//   stat[mt][0][n] = sum_rows (out - shift[n]),  stat[mt][1][n] = sum_rows (out - shift[n])^2
// for each 128-row panel mt (deterministic partials; reduce with the fp64 colreduce).
struct Epi {
  const float* bias = nullptr;
  const void* res = nullptr;
  const float* rs = nullptr;
  int rps = 1;
  const void* Z = nullptr;
  int ldz = 0, zact = 0;
  double* stat = nullptr;
  const float* stat_shift = nullptr;
  // second output (bf16 forward kernels): aout[m, n] = aact(out[m, n]) of the stored (rounded) value,
  // e.g. GELU(fc1) materialised for the next GEMM and its weight gradient (ogv_gemm_fwd_act)
  void* aout = nullptr;
  int ldao = 0, aact = 0;
  // LayerNorm of the stored output rows (panel kernel, one column tile holding whole rows; ogv_gemm_fwd_ln):
  // ln_out[m, :] = (out[m, :] - mean) * rstd * ln_g + ln_b, ln_mean / ln_rstd [M] for the LN backward
  void* ln_out = nullptr;
  const float *ln_g = nullptr, *ln_b = nullptr;
  float *ln_mean = nullptr, *ln_rstd = nullptr;
  float ln_eps = 0.f;
};

// Implicit-GEMM gather for 3x3 / pad-1 convolutions.  The A operand (or the wgrad X operand) is
// not a dense matrix but rows m = (b*Hr + ry)*Wr + rx of a row grid, and tap-major columns
// k = tap*Cs + c (tap = 3*ky + kx) that read source pixel (sy, sx) channel c:
//   forward   (transposed = 0): sy = ry*stride - 1 + ky                       (conv fwd)
//   transposed(transposed = 1): sy = (ry + 1 - ky) / stride when exact         (conv dgrad)
// and zero outside the source image.  With Cs % 8 == 0 an 8-wide k chunk is one 16-B load.
struct ConvG {
  int Hr = 0, Wr = 0;          // row grid
  int Hs = 0, Ws = 0, Cs = 0;  // source grid / channels
  int stride = 1, transposed = 0;
  // parity class of a stride-2 transposed conv (panel kernel only; -1 = off): rows are the output
  // pixels (2Y + (par >> 1), 2X + (par & 1)) and the reduction runs over the ntap taps that can hit
  // them (tap[0..ntap), tap-major columns k = t * Cs + c)
  int par = -1, ntap = 9;
  int tap[4] = {0, 0, 0, 0};
  // par == 4: ALL four parity classes in one launch (panel kernel): workgroups [c G4, (c + 1) G4) run class c
  // (G4 a multiple of 8, so a workgroup keeps its XCD); each class's taps follow from its parity
  int cls_G = 0;
};
// the taps of parity class c of a stride-2 transposed 3x3 conv: output pixel parity (y & 1, x & 1) = (c >> 1, c & 1)
// receives ky = 1 (even y) or {0, 2} (odd y), kx likewise
__host__ __device__ constexpr int tconv_ntap(int c) { return c == 0 ? 1 : (c == 3 ? 4 : 2); }
__host__ __device__ constexpr int tconv_tap(int c, int t) {
  return c == 0 ? 4 : c == 1 ? (t == 0 ? 3 : 5) : c == 2 ? (t == 0 ? 1 : 7) : (t == 0 ? 0 : t == 1 ? 2 : t == 2 ? 6 : 8);
}
// tap[t] of a parity class through selects on the (uniform) kernel-argument values: a dynamic index
// into the by-value argument struct makes the compiler re-load it from the kernarg segment and wait
// for that load at every use
__device__ __forceinline__ int conv_tap(const ConvG& g, int t) {
  // (readfirstlane pins each value in a register: a plain select chain is folded back into a load
  // through a selected kernarg address)
  const int t0 = __builtin_amdgcn_readfirstlane(g.tap[0]), t1 = __builtin_amdgcn_readfirstlane(g.tap[1]);
  const int t2 = __builtin_amdgcn_readfirstlane(g.tap[2]), t3 = __builtin_amdgcn_readfirstlane(g.tap[3]);
  return t <= 0 ? t0 : t == 1 ? t1 : t == 2 ? t2 : t3;
}
struct ConvRow {
  int b, ry, rx;
};
__device__ __forceinline__ ConvRow conv_row(const ConvG& g, int m) {
  ConvRow r;
  const int hw = g.Hr * g.Wr;
  r.b = m / hw;
  const int rem = m - r.b * hw;
  r.ry = rem / g.Wr;
  r.rx = rem - r.ry * g.Wr;
  return r;
}
// element offset of source pixel for (row, tap), or -1 when it is padding / not hit by the stride
__device__ __forceinline__ long conv_src(const ConvG& g, const ConvRow& r, int tap) {
  const int ky = tap / 3, kx = tap - 3 * ky;
  int sy, sx;
  if (!g.transposed) {
    sy = r.ry * g.stride - 1 + ky;
    sx = r.rx * g.stride - 1 + kx;
  } else {
    const int ny = r.ry + 1 - ky, nx = r.rx + 1 - kx;
    if (ny < 0 || nx < 0) return -1;
    sy = ny / g.stride;
    sx = nx / g.stride;
    if (sy * g.stride != ny || sx * g.stride != nx) return -1;
  }
  if (sy < 0 || sy >= g.Hs || sx < 0 || sx >= g.Ws) return -1;
  return ((long)(r.b * g.Hs + sy) * g.Ws + sx) * g.Cs;
}

constexpr int GEMM_BM = 128;
inline int gemm_stat_rows(int M) { return (M + GEMM_BM - 1) / GEMM_BM; }
// BatchNorm partial rows an implicit-conv forward may write (conv_gemm_launch: 64-row panels on small M)
inline int conv_stat_rows(int M) { return (M + 63) / 64; }

// out[M,N] = epi( pro(A)[M,K] . W[N,K]^T );  Ka / Kb = valid reduction columns of A / W.
// Returns the number of BatchNorm partial rows written to epi.stat (<= gemm_stat_rows(M)); the
// caller reduces exactly that many.
int gemm_fwd_launch(ogv_dtype dt, const void* A, int lda, const Pro& pro, const float* W, int ldw, void* out,
                     int ldo, int M, int N, int K, int Ka, int Kb, const Epi& epi, hipStream_t s);

// dA[M,K] = act'(Z) * rs * (dOut[M,N] . W[N,K]);  ws >= dgrad_ws_bytes(N, K); res added if given
size_t dgrad_ws_bytes(int N, int K);
void gemm_dgrad_launch(ogv_dtype dt, const void* dout, int ldd, const float* W, const void* Z, int ldz, int zact,
                       const float* rs, int rps, const void* res, void* dA, int lda, int M, int N, int K, void* ws,
                       hipStream_t s);

// dW[N,K] = sum_m rs*G[m,n] * pro(X)[m,k];  dbias[n] = sum_m rs*G[m,n]
size_t wgrad_ws_bytes(int M, int N, int K);
void gemm_wgrad_launch(ogv_dtype dt, const void* G, int ldg, const void* X, int ldx, const Pro& pro, const float* rs,
                       int rps, float* dW, float* dbias, int M, int N, int K, void* ws, hipStream_t s,
                       const ConvG* xconv = nullptr, bool param_grad = false);

// Small-M fp32 GEMM with split-K (SE MLP: M = batch rows): out = epi(pro(A)[M,K] . W[N,K]^T);
// ws >= splitk_ws_bytes(M, N, K).  Epilogue: bias, rs, res, zact (no stats).
size_t splitk_ws_bytes(int M, int N, int K);
void gemm_fwd_splitk_f32(const float* A, int lda, const Pro& pro, const float* W, int ldw, float* out, int ldo, int M,
                         int N, int K, const Epi& epi, void* ws, hipStream_t s, bool bt = false,
                         float* sig_out = nullptr);
// WT[k][n] = W[n][k] (fp32), zero for n in [N, ldt)
void transpose_f32_launch(const float* W, float* WT, int N, int K, int ldt, hipStream_t s);

// Implicit-GEMM 3x3 conv:  out[M, N] = epi( gather(A)[M, 9*Cs] . Wt[N, 9*Cs]^T ),  M = B*Hr*Wr.
// Wt is tap-major ([N][tap][Cs]).  Used for the conv forward (cv.transposed = 0) and its data
// gradient (cv.transposed = 1, Wt = the tap-major transposed weights).
int conv_gemm_launch(ogv_dtype dt, const void* A, const ConvG& cv, const float* Wt, void* out, int M, int N,
                      const Epi& epi, hipStream_t s);

// Persistent streaming GEMM (ogv_sgemm.hip) for tall-skinny bf16 shapes; 0 / false = not handled.
int sgemm_fwd_try(const void* A, int lda, const Pro& pro, const float* W, int ldw, void* out, int ldo, int M,
                  int N, int K, const Epi& epi, hipStream_t s);
bool sgemm_dgrad_try(const void* dout, int ldd, const float* W, void* dA, int lda, int M, int Nf, int Kf,
                     const Epi& epi, hipStream_t s);
// Pipelined panel GEMM (ogv_pgemm.hip) for small-M bf16 shapes; 0 / false = not handled.
int pgemm_fwd_try(const void* A, int lda, const Pro& pro, const float* W, int ldw, void* out, int ldo, int M,
                  int N, int K, const Epi& epi, hipStream_t s);
bool pgemm_fwd_ln_try(const void* A, int lda, const float* W, int ldw, void* out, int ldo, int M, int N, int K,
                      const Epi& epi, hipStream_t s);
void set_ln_epi(int v);
bool pgemm_dgrad_try(const void* dout, int ldd, const float* W, void* dA, int lda, int M, int Nf, int Kf,
                     const Epi& epi, hipStream_t s);
bool pgemm_route(int kind, int M, int N, int K, int act);
int pgemm_conv_try(const void* A, const ConvG& cv, const float* Wt, void* out, int M, int N, const Epi& epi,
                   hipStream_t s);
bool pgemm_tconv_try(const void* A, const ConvG& cv, const float* Wt, void* out, int M, int N, hipStream_t s);
void set_pgemm(int v);
void set_pg_rs(int v);
void set_pg_tn(int v);
void set_pg_per_cu(int v);
void set_pg_dbg(int v);
void set_pg_lds_kb(int v);
void set_wg_blocks(int v);
void set_wg_tile(int v);
// Streaming weight gradient (ogv_swgrad.hip) for large-M bf16 shapes: writes [S][N*K + N] fp32
// partials into part and returns S (0 = not handled); swgrad_ws_floats sizes part + colreduce tmp.
int swgrad_try(const void* G, int ldg, const void* X, int ldx, const Pro& pro, const float* rs, int rps, float* part,
               bool bias, int M, int N, int K, hipStream_t s);
size_t swgrad_ws_floats(int M, int N, int K);
// Pipelined split-M weight gradient (ogv_wgrad2.hip), same partial layout; knob "wg2": 0 off,
// 1 = where the streaming kernel does not apply, 2 = ahead of it as well.
int wgrad2_try(const void* G, int ldg, const void* X, int ldx, const Pro& pro, const float* rs, int rps, float* part,
               float* dW, float* dbias, bool bias, int M, int N, int K, hipStream_t s, bool* reduced,
               const ConvG* xc = nullptr);
void set_wg2_conv(int v);
void set_wg2_fuse(int v);
size_t wgrad2_ws_floats(int M, int N, int K);
int wg2_mode();
void set_wg2(int v);
void set_wg2_blocks(int v);
void set_wg2_tile(int v);
void set_wg2_pbeta(int v);
int sgemm_mode();
void set_sgemm_mode(int v);
int sgemm_min_m();
void set_sgemm_min_m(int v);
void set_sg_per_cu(int v);
void set_sg_prefetch(int v);
void set_sg_wgs(int v);
void set_splitk_max(int v);
void set_bk64_max_m(int v);
void set_bm64_max_m(int v);
void set_grid_mfma(int v);
void set_dw_blocks(int v);
void set_mb_side(int v);
void set_ln_bwd_blocks(int v);
void set_gemm_bn64(int v);
void set_grid_lds(int v);
void set_grid_big(int v);
void set_split_w(int v);
void set_outlook_tile(int v);
void set_outlook_vproj(int v);
void set_vp_dbg(int v);
void set_vp_tile(int v);
void set_vp_big(int v);
void set_dw_tw(int v);
void set_ln_rpi(int v);
void set_vp_head(int v);
void set_vph_rows(int v);
void set_vph_wgs(int v);
void set_vph_halo(int v);
void set_vp_l32(int v);
void set_vph_tile(int v);
void set_vph_dbg(int v);
// Squeeze-Excite GEMVs (ogv_se.hip); knob "se_gemv" (1 default, 0 = the split-K tiled GEMM + reduce)
void se_gemv_launch(const float* in, int ldi, int pro_act, const float* W, int ldw, const float* bias,
                    const float* Z, int ldz, int zact, float* out, int ldo, float* sig_out, int B, int N, int K,
                    bool rm, hipStream_t s);
bool se_gemv_on();
void set_se_gemv(int v);
void set_dw_fuse(int v);
void set_dw_bn2(int v);
void set_dw_fwd_r(int v);
void set_bn_slices(int v);
void set_pg_conv_rs1(int v);
void set_dw_bwd_r(int v);
void set_stem(int v);
void set_pg_tn4_max_m(int v);
void set_pg_pa_wide(int v);
void set_stem_wgs(int v);
// the stem convolution (C_in <= 3, ogv_stem.hip): false = not taken (the caller runs the generic path)
bool stem_fwd_try(const void* x, const ConvG& cv, const float* wt, void* out, int M, int N, const Epi& epi,
                  hipStream_t s, int* stat_rows);
int stem_fwd_stat_rows(long M);   // BN partial rows the stem forward writes (<= gemm_stat_rows(M))
bool stem_wgrad_try(const void* x, const ConvG& cv, const void* dy, float* dw, float* dbias, int M, int N, void* ws,
                    hipStream_t s);
size_t stem_wgrad_ws_bytes(long M, int N, int Cin);
void set_swg_min_m(int v);
void set_pg_split(int v);
void set_pg_tconv1(int v);
int split_w();
int skip_mask();
void set_skip(int v);

}  // namespace ogv
