// Stem / downsample / head of MaxOutNet on the MI355X: 3x3 convolution (pad 1, stride 1|2) as an
// implicit GEMM on the MFMA kernels, BatchNorm2d (train batch statistics or eval running
// statistics) and the activation, on NHWC rows.
//
//   stem:        Conv2d(in, stem, 3, 1, 1, bias=!bn) -> BN -> SiLU    src/model/stem_head.py:23-32
//   downsample:  Conv2d(C, C', 3, 2, 1, bias=!bn)    -> BN -> SiLU    src/model/downsampling.py:28-65
//   head:        BatchNorm2d(C) (no activation)                       src/Model_A_OutGridNet.py:52,66
//
// Forward: the conv GEMM's epilogue writes the conv output y and per-128-row-panel shifted BN
// sums (shift = running mean), a deterministic column reduction + finalize turn them into
// mean / invstd / apply coefficients (and update the running statistics), and one elementwise
// pass writes act(y*sc + sh).  Backward recomputes dz = da*act'(y*sc + sh) inside its two passes
// (reduction, apply), then the conv weight gradient (slab wgrad with the same gather on x) and,
// when the input needs it, the data gradient as a transposed-gather implicit GEMM.
#include "ogv_bn.h"
#include "ogv_gemm.h"

namespace ogv {

// ------------------------------------------------------------------ weight layout kernels
// wt[n][tap*Cin + c] = w[n][c][tap]   (tap-major K for the forward gather)
__global__ void conv_w_fwd_kernel(const float* __restrict__ w, float* __restrict__ wt, int Cout, int Cin) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (long)Cout * Cin * 9) return;
  const int n = (int)(i / (9L * Cin)), r = (int)(i - (long)n * 9 * Cin);
  const int tap = r / Cin, c = r - tap * Cin;
  wt[i] = w[((long)n * Cin + c) * 9 + tap];
}
// wd[c][tap*Cout + n] = w[n][c][tap]   (the data gradient's GEMM weights; tm: w stored tap-major
// [n][tap][c], a channels_last weight)
__global__ void conv_w_dgrad_kernel(const float* __restrict__ w, float* __restrict__ wd, int Cout, int Cin, int tm) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (long)Cout * Cin * 9) return;
  const int c = (int)(i / (9L * Cout)), r = (int)(i - (long)c * 9 * Cout);
  const int tap = r / Cout, n = r - tap * Cout;
  wd[i] = tm ? w[((long)n * 9 + tap) * Cin + c] : w[((long)n * Cin + c) * 9 + tap];
}
// dw[n][c][tap] = dwt[n][tap*Cin + c]
__global__ void conv_dw_untranspose_kernel(const float* __restrict__ dwt, float* __restrict__ dw, int Cout, int Cin) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (long)Cout * Cin * 9) return;
  const int n = (int)(i / (9L * Cin)), r = (int)(i - (long)n * 9 * Cin);
  const int c = r / 9, tap = r - c * 9;
  dw[i] = dwt[(long)n * 9 * Cin + tap * Cin + c];
}

// BatchNorm off (use_bn=False): identity coefficients mean 0, invstd 1, sc 1, sh 0 / coef (1, 0, 0)
__global__ void bn_identity_kernel(float* __restrict__ mean, float* __restrict__ invstd, float* __restrict__ sc,
                                   float* __restrict__ sh, float* __restrict__ coef, int K) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= K) return;
  if (mean) { mean[c] = 0.f; invstd[c] = 1.f; sc[c] = 1.f; sh[c] = 0.f; }
  if (coef) { coef[c] = 1.f; coef[K + c] = 0.f; coef[2 * K + c] = 0.f; }
}

// ------------------------------------------------------------------ BatchNorm(+act) passes
// Block = (4 chunks of V channels) x (64 row slots) for one (channel tile, row slice), XCD-aware
// order (xcd_block); partials go to stat[slice][q][C] and a colreduce sums the slices in a fixed
// order (deterministic).

// stat = [sum (x - shift), sum (x - shift)^2]   (BatchNorm batch statistics, fp64)
template <typename T, int V>
__global__ __launch_bounds__(256) void bn_stats_kernel(const T* __restrict__ x, const float* __restrict__ shift,
                                                       double* __restrict__ stat, long M, int C, long per) {
  __shared__ double lds[4 * 2 * 4 * 8];
  const int gx = (C + 4 * V - 1) / (4 * V);
  long lid;
  if (!xcd_block((long)gx * ((M + per - 1) / per), lid)) return;
  const int bx = (int)(lid % gx);
  const long by = lid / gx;
  const int chunk = threadIdx.x & 3, slot = threadIdx.x >> 2;
  const int c0 = (bx * 4 + chunk) * V;
  const long r0 = by * per, r1 = r0 + per < M ? r0 + per : M;
  double q[2][V];
#pragma unroll
  for (int i = 0; i < V; ++i) { q[0][i] = 0.0; q[1][i] = 0.0; }
  if (c0 < C) {
    float sf[V];
    load_vec<float, V>(shift + c0, sf);
#pragma unroll
    for (int i = 0; i < V; ++i) sf[i] = bn_shift(sf[i]);
    for (long r = r0 + slot; r < r1; r += 64) {
      float v[V];
      load_vec<T, V>(x + r * C + c0, v);
#pragma unroll
      for (int i = 0; i < V; ++i) {
        const double d = (double)v[i] - (double)sf[i];
        q[0][i] += d;
        q[1][i] = fma(d, d, q[1][i]);
      }
    }
  }
  chunk_reduce_store<2, V, double>(q, lds, stat + by * 2 * C, C, C, bx * 4 * V);
}

// out = act(y*sc + sh)
template <typename T, int V>
__global__ __launch_bounds__(256) void bn_act_apply_kernel(const T* __restrict__ y, const float* __restrict__ sc,
                                                           const float* __restrict__ sh, int act, T* __restrict__ out,
                                                           long M, int C) {
  const int nch = C / V;
  const long tid = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (tid >= M * nch) return;
  const int c0 = (int)(tid % nch) * V;
  const long m = tid / nch;
  float v[V], s[V], h[V];
  load_vec<T, V>(y + m * C + c0, v);
  load_vec<float, V>(sc + c0, s);
  load_vec<float, V>(sh + c0, h);
#pragma unroll
  for (int i = 0; i < V; ++i) v[i] = act_fwd(act, fmaf(v[i], s[i], h[i]));
  store_vec<T, V>(out + m * C + c0, v);
}

// dz = da * act'(y*sc + sh);  stat = [sum dz, sum dz*(y - mean)*invstd]
template <typename T, int V>
__global__ __launch_bounds__(256) void bn_act_bwd_reduce_kernel(const T* __restrict__ da, const T* __restrict__ y,
                                                                const float* __restrict__ sc,
                                                                const float* __restrict__ sh, int act,
                                                                const float* __restrict__ mean,
                                                                const float* __restrict__ invstd,
                                                                float* __restrict__ stat, long M, int C, long per) {
  __shared__ float lds[4 * 2 * 4 * 8];
  const int gx = (C + 4 * V - 1) / (4 * V);
  long lid;
  if (!xcd_block((long)gx * ((M + per - 1) / per), lid)) return;
  const int bx = (int)(lid % gx);
  const long by = lid / gx;
  const int chunk = threadIdx.x & 3, slot = threadIdx.x >> 2;
  const int c0 = (bx * 4 + chunk) * V;
  const long r0 = by * per, r1 = r0 + per < M ? r0 + per : M;
  float q[2][V];
#pragma unroll
  for (int i = 0; i < V; ++i) { q[0][i] = 0.f; q[1][i] = 0.f; }
  if (c0 < C) {
    float s[V], h[V], mu[V], is[V];
    load_vec<float, V>(sc + c0, s);
    load_vec<float, V>(sh + c0, h);
    load_vec<float, V>(mean + c0, mu);
    load_vec<float, V>(invstd + c0, is);
    for (long r = r0 + slot; r < r1; r += 64) {
      float g[V], v[V];
      load_vec<T, V>(da + r * C + c0, g);
      load_vec<T, V>(y + r * C + c0, v);
#pragma unroll
      for (int i = 0; i < V; ++i) {
        const float dz = act == OGV_ACT_NONE ? g[i] : g[i] * act_grad(act, fmaf(v[i], s[i], h[i]));
        q[0][i] += dz;
        q[1][i] = fmaf(dz, (v[i] - mu[i]) * is[i], q[1][i]);
      }
    }
  }
  chunk_reduce_store<2, V>(q, lds, stat + by * 2 * C, C, C, bx * 4 * V);
}

// out = coef0*(dz - coef1 - (y - mean)*invstd*coef2),  dz = da*act'(y*sc + sh)
template <typename T, int V>
__global__ __launch_bounds__(256) void bn_act_bwd_apply_kernel(const T* __restrict__ da, const T* __restrict__ y,
                                                               const float* __restrict__ sc,
                                                               const float* __restrict__ sh, int act,
                                                               const float* __restrict__ mean,
                                                               const float* __restrict__ invstd,
                                                               const float* __restrict__ coef, T* __restrict__ out,
                                                               long M, int C) {
  const int nch = C / V;
  const long tid = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (tid >= M * nch) return;
  const int c0 = (int)(tid % nch) * V;
  const long m = tid / nch;
  float g[V], v[V], s[V], h[V], mu[V], is[V], ca[V], cb[V], cc[V];
  load_vec<T, V>(da + m * C + c0, g);
  load_vec<T, V>(y + m * C + c0, v);
  load_vec<float, V>(sc + c0, s);
  load_vec<float, V>(sh + c0, h);
  load_vec<float, V>(mean + c0, mu);
  load_vec<float, V>(invstd + c0, is);
  load_vec<float, V>(coef + c0, ca);
  load_vec<float, V>(coef + C + c0, cb);
  load_vec<float, V>(coef + 2 * C + c0, cc);
#pragma unroll
  for (int i = 0; i < V; ++i) {
    const float dz = act == OGV_ACT_NONE ? g[i] : g[i] * act_grad(act, fmaf(v[i], s[i], h[i]));
    g[i] = ca[i] * (dz - cb[i] - (v[i] - mu[i]) * is[i] * cc[i]);
  }
  store_vec<T, V>(out + m * C + c0, g);
}

// ------------------------------------------------------------------ host plumbing
static int vec_width(int C) { return (C % 8 == 0) ? 8 : (C % 4 == 0) ? 4 : 1; }

struct RowSlices {
  long S, per;
};
// knob "bn_slices": the cap on row slices (blocks per channel group) of the BatchNorm statistics / backward
// reductions (default 1024; each slice >= 1024 rows): 7M step, 30 steps, 256 -> 14.79 / 14.82 ms, 512 -> 14.78,
// 1024 -> 14.76 / 14.77, 2048 -> 14.80 (profiles/r05r_bn_slices.log)
static long g_bn_slices = 1024;
void set_bn_slices(int v) { g_bn_slices = v < 16 ? 16 : (v > 4096 ? 4096 : v); }
static RowSlices row_slices(long M) {
  RowSlices r;
  r.S = (M + 1023) / 1024;
  if (r.S > g_bn_slices) r.S = g_bn_slices;
  if (r.S < 1) r.S = 1;
  r.per = (M + r.S - 1) / r.S;
  r.S = (M + r.per - 1) / r.per;
  return r;
}

template <typename T, int V>
static void bn_stats_run(const void* x, const float* shift, double* stat, long M, int C, const RowSlices& rs,
                         hipStream_t s) {
  bn_stats_kernel<T, V><<<xcd_grid((long)cdiv(C, 4 * V) * rs.S), 256, 0, s>>>((const T*)x, shift, stat, M, C, rs.per);
}
template <typename T, int V>
static void bn_apply_run(const void* y, const float* sc, const float* sh, int act, void* out, long M, int C,
                         hipStream_t s) {
  bn_act_apply_kernel<T, V><<<cdiv(M * (C / V), 256), 256, 0, s>>>((const T*)y, sc, sh, act, (T*)out, M, C);
}
template <typename T, int V>
static void bn_bwd_reduce_run(const void* da, const void* y, const float* sc, const float* sh, int act,
                              const float* mean, const float* invstd, float* stat, long M, int C, const RowSlices& rs,
                              hipStream_t s) {
  bn_act_bwd_reduce_kernel<T, V><<<xcd_grid((long)cdiv(C, 4 * V) * rs.S), 256, 0, s>>>((const T*)da, (const T*)y, sc, sh, act, mean, invstd, stat, M, C,
                                                   rs.per);
}
template <typename T, int V>
static void bn_bwd_apply_run(const void* da, const void* y, const float* sc, const float* sh, int act,
                             const float* mean, const float* invstd, const float* coef, void* out, long M, int C,
                             hipStream_t s) {
  bn_act_bwd_apply_kernel<T, V><<<cdiv(M * (C / V), 256), 256, 0, s>>>((const T*)da, (const T*)y, sc, sh, act, mean,
                                                                       invstd, coef, (T*)out, M, C);
}

#define OGV_CB_DISPATCH(dt, V, FN, ...)                        \
  do {                                                         \
    if ((dt) == OGV_BF16) {                                    \
      if ((V) == 8) FN<bf16, 8>(__VA_ARGS__);                  \
      else if ((V) == 4) FN<bf16, 4>(__VA_ARGS__);             \
      else FN<bf16, 1>(__VA_ARGS__);                           \
    } else {                                                   \
      if ((V) == 8) FN<float, 8>(__VA_ARGS__);                 \
      else if ((V) == 4) FN<float, 4>(__VA_ARGS__);            \
      else FN<float, 1>(__VA_ARGS__);                          \
    }                                                          \
  } while (0)

struct Carve {
  char* base;
  size_t off = 0;
  explicit Carve(void* b) : base((char*)b) {}
  template <typename P>
  P* take(size_t n) {
    off = (off + 255) & ~(size_t)255;
    P* r = reinterpret_cast<P*>(base ? base + off : nullptr);
    off += n * sizeof(P);
    return r;
  }
};

// BN per-channel vectors kept from forward to backward
struct BnSaved {
  float *mean, *invstd, *sc, *sh;
};
static BnSaved take_bn_saved(Carve& c, int C) {
  BnSaved b;
  b.mean = c.take<float>(C);
  b.invstd = c.take<float>(C);
  b.sc = c.take<float>(C);
  b.sh = c.take<float>(C);
  return b;
}

static size_t esize(ogv_dtype dt) { return dt == OGV_BF16 ? 2 : 4; }

// ------------------------------------------------------------------ conv3x3 -> BN -> act
struct CbGeom {
  int Ho, Wo;
  long M, Mo;
  ConvG fwd, bwd;
};
static CbGeom cb_geom(const ogv_convbn_desc& d) {
  CbGeom g;
  g.Ho = (d.H - 1) / d.stride + 1;
  g.Wo = (d.W - 1) / d.stride + 1;
  g.M = (long)d.B * d.H * d.W;
  g.Mo = (long)d.B * g.Ho * g.Wo;
  g.fwd.Hr = g.Ho; g.fwd.Wr = g.Wo; g.fwd.Hs = d.H; g.fwd.Ws = d.W; g.fwd.Cs = d.Cin;
  g.fwd.stride = d.stride; g.fwd.transposed = 0;
  g.bwd.Hr = d.H; g.bwd.Wr = d.W; g.bwd.Hs = g.Ho; g.bwd.Ws = g.Wo; g.bwd.Cs = d.Cout;
  g.bwd.stride = d.stride; g.bwd.transposed = 1;
  return g;
}

static int cb_check(const ogv_convbn_desc* d, ogv_dtype dt, const char* fn) {
  OGV_REQUIRE(d, "%s: null desc", fn);
  OGV_REQUIRE(dt == OGV_F32 || dt == OGV_BF16, "%s: bad dtype %d", fn, (int)dt);
  OGV_REQUIRE(d->B > 0 && d->H > 0 && d->W > 0 && d->Cin > 0 && d->Cout > 0, "%s: bad shape", fn);
  OGV_REQUIRE(d->stride == 1 || d->stride == 2, "%s: stride %d unsupported", fn, d->stride);
  OGV_REQUIRE(d->act >= OGV_ACT_NONE && d->act <= OGV_ACT_RELU, "%s: bad act %d", fn, d->act);
  OGV_REQUIRE((long)d->B * d->H * d->W < (1L << 31), "%s: too many rows", fn);
  return OGV_OK;
}

// saved = [y (conv output) Mo x Cout][mean, invstd, sc, sh]
static void cb_saved(const ogv_convbn_desc& d, ogv_dtype dt, void* base, void** y, BnSaved& b, size_t* bytes) {
  const CbGeom g = cb_geom(d);
  Carve c(base);
  char* yp = c.take<char>((size_t)g.Mo * d.Cout * esize(dt));
  b = take_bn_saved(c, d.Cout);
  if (y) *y = yp;
  if (bytes) *bytes = c.off;
}

struct CbWs {
  float* wt;      // tap-major weights (fwd) / transposed weights (dgrad)
  double* dstat;  // fwd BN statistics partials (fp64) ...
  double* dsums;  // ... reduced [2][Cout]
  double* dtmp;
  float* stat;    // bwd BN partials
  float* sums;    // reduced [2][Cout]
  float* tmp;     // colreduce scratch
  float* coef;    // [3][Cout]
  char* dy;       // conv-output gradient Mo x Cout
  float* dwt;     // tap-major dW
  char* gemm;     // wgrad slabs
  char* stem;     // the stem weight gradient's partial rows + colreduce scratch (C_in <= 3)
  size_t bytes;
};
static CbWs cb_ws(const ogv_convbn_desc& d, ogv_dtype dt, void* base) {
  const CbGeom g = cb_geom(d);
  const int K9 = 9 * d.Cin;
  const long nMt = conv_stat_rows((int)g.Mo);
  const RowSlices rs = row_slices(g.Mo);
  const long srows = nMt > rs.S ? nMt : rs.S;
  Carve c(base);
  CbWs w;
  w.wt = c.take<float>((size_t)d.Cout * K9);
  w.dstat = c.take<double>((size_t)srows * 2 * d.Cout);
  w.dsums = c.take<double>(2 * (size_t)d.Cout);
  w.dtmp = c.take<double>(colreduce_tmp_floats(srows, 2L * d.Cout));
  w.stat = c.take<float>((size_t)srows * 2 * d.Cout);
  w.sums = c.take<float>(2 * (size_t)d.Cout);
  w.tmp = c.take<float>(colreduce_tmp_floats(srows, 2L * d.Cout));
  w.coef = c.take<float>(3 * (size_t)d.Cout);
  w.dy = c.take<char>((size_t)g.Mo * d.Cout * esize(dt));
  w.dwt = c.take<float>((size_t)d.Cout * K9);
  w.gemm = c.take<char>(wgrad_ws_bytes((int)g.Mo, d.Cout, K9));
  w.stem = c.take<char>(d.Cin <= 3 ? stem_wgrad_ws_bytes(g.Mo, d.Cout, d.Cin) : 16);
  w.bytes = c.off;
  return w;
}

}  // namespace ogv

using namespace ogv;

extern "C" size_t ogv_convbn_saved_bytes(const ogv_convbn_desc* d, ogv_dtype dt) {
  if (cb_check(d, dt, "ogv_convbn_saved_bytes")) return 0;
  size_t n = 0;
  BnSaved b;
  cb_saved(*d, dt, nullptr, nullptr, b, &n);
  return n;
}

extern "C" size_t ogv_convbn_ws_bytes(const ogv_convbn_desc* d, ogv_dtype dt) {
  if (cb_check(d, dt, "ogv_convbn_ws_bytes")) return 0;
  return cb_ws(*d, dt, nullptr).bytes;
}

extern "C" int ogv_convbn_fwd(const void* x, void* out, void* saved, void* ws, const ogv_convbn_desc* d,
                              const ogv_convbn_params* p, ogv_dtype dt, void* stream) {
  int rc = cb_check(d, dt, "ogv_convbn_fwd");
  if (rc) return rc;
  OGV_REQUIRE(x && out && saved && ws && p && p->w, "ogv_convbn_fwd: null pointer");
  OGV_REQUIRE(!d->has_bn || (p->bn_rm && p->bn_rv), "ogv_convbn_fwd: BatchNorm needs running statistics");
  hipStream_t s = as_stream(stream);
  const CbGeom g = cb_geom(*d);
  void* y;
  BnSaved b;
  cb_saved(*d, dt, saved, &y, b, nullptr);
  const CbWs w = cb_ws(*d, dt, ws);
  const long nw = (long)d->Cout * d->Cin * 9;
  const float* wt = p->w;   // w_layout 1: already the tap-major matrix
  if (!d->w_layout) {
    conv_w_fwd_kernel<<<cdiv(nw, 256), 256, 0, s>>>(p->w, w.wt, d->Cout, d->Cin);
    wt = w.wt;
  }
  Epi e;
  e.bias = p->bias;
  const bool stats = d->has_bn && d->train;
  if (stats) {
    e.stat = w.dstat;
    e.stat_shift = p->bn_rm;
  }
  // the stem (C_in <= 3): dedicated kernel (ogv_stem.hip); everything else: implicit-GEMM conv kernels
  int srows = gemm_stat_rows((int)g.Mo);
  if (!(dt == OGV_BF16 && stem_fwd_try(x, g.fwd, wt, y, (int)g.Mo, d->Cout, e, s, &srows)))
    srows = conv_gemm_launch(dt, x, g.fwd, wt, y, (int)g.Mo, d->Cout, e, s);
  if (d->has_bn) {
    if (stats)   // partial rows -> batch statistics, running stats, apply coefficients: one launch
      bn_reduce_finalize_launch(w.dstat, srows, 2L * d->Cout, d->Cout, (double)g.Mo, p->bn_w,
                                p->bn_b, d->bn_eps, d->bn_momentum, p->bn_rm, p->bn_rv, b.mean, b.invstd, b.sc, b.sh, s);
    else
      bn_finalize_launch(w.dsums, d->Cout, (double)g.Mo, p->bn_w, p->bn_b, d->bn_eps, d->bn_momentum, p->bn_rm,
                         p->bn_rv, b.mean, b.invstd, b.sc, b.sh, d->train, s);
  } else {
    bn_identity_kernel<<<cdiv(d->Cout, 256), 256, 0, s>>>(b.mean, b.invstd, b.sc, b.sh, nullptr, d->Cout);
  }
  OGV_CB_DISPATCH(dt, vec_width(d->Cout), bn_apply_run, y, b.sc, b.sh, d->act, out, g.Mo, d->Cout, s);
  return check_launch("ogv_convbn_fwd");
}

extern "C" int ogv_convbn_bwd(const void* dout, const void* x, const void* saved, void* dx, float* dw, float* dbias,
                              float* dbn_w, float* dbn_b, void* ws, const ogv_convbn_desc* d,
                              const ogv_convbn_params* p, ogv_dtype dt, void* stream) {
  int rc = cb_check(d, dt, "ogv_convbn_bwd");
  if (rc) return rc;
  OGV_REQUIRE(dout && x && saved && ws && p && p->w && dw, "ogv_convbn_bwd: null pointer");
  hipStream_t s = as_stream(stream);
  const CbGeom g = cb_geom(*d);
  void* y;
  BnSaved b;
  cb_saved(*d, dt, const_cast<void*>(saved), &y, b, nullptr);
  const CbWs w = cb_ws(*d, dt, ws);
  const int V = vec_width(d->Cout);
  // 1) BatchNorm + activation backward -> gradient of the conv output
  if (d->has_bn) {
    const RowSlices rs = row_slices(g.Mo);
    OGV_CB_DISPATCH(dt, V, bn_bwd_reduce_run, dout, y, b.sc, b.sh, d->act, b.mean, b.invstd, w.stat, g.Mo, d->Cout, rs,
                    s);
    bn_reduce_coeffs_launch(w.stat, rs.S, 2L * d->Cout, d->Cout, (float)g.Mo, p->bn_w, b.invstd, dbn_w, dbn_b, w.coef,
                            d->train, s);
  } else {
    bn_identity_kernel<<<cdiv(d->Cout, 256), 256, 0, s>>>(nullptr, nullptr, nullptr, nullptr, w.coef, d->Cout);
  }
  OGV_CB_DISPATCH(dt, V, bn_bwd_apply_run, dout, y, b.sc, b.sh, d->act, b.mean, b.invstd, w.coef, w.dy, g.Mo, d->Cout,
                  s);
  // 2) weight (+bias) gradient: dW[n][tap*Cin+c] = sum_m dy[m,n] * gather(x)[m, tap*Cin+c]
  const int K9 = 9 * d->Cin;
  if (!(dt == OGV_BF16 && stem_wgrad_try(x, g.fwd, w.dy, d->w_layout ? dw : w.dwt, dbias, (int)g.Mo, d->Cout, w.stem,
                                         s)))
    gemm_wgrad_launch(dt, w.dy, d->Cout, x, 0, Pro(), nullptr, 1, d->w_layout ? dw : w.dwt, dbias, (int)g.Mo, d->Cout,
                      K9, w.gemm, s, &g.fwd);
  const long nw = (long)d->Cout * d->Cin * 9;
  if (!d->w_layout) conv_dw_untranspose_kernel<<<cdiv(nw, 256), 256, 0, s>>>(w.dwt, dw, d->Cout, d->Cin);
  // 3) data gradient: transposed gather of dy against the (Cin x 9*Cout) weight matrix
  if (dx) {
    conv_w_dgrad_kernel<<<cdiv(nw, 256), 256, 0, s>>>(p->w, w.wt, d->Cout, d->Cin, d->w_layout);
    conv_gemm_launch(dt, w.dy, g.bwd, w.wt, dx, (int)g.M, d->Cin, Epi(), s);
  }
  return check_launch("ogv_convbn_bwd");
}

// ------------------------------------------------------------------ BatchNorm(+act) alone
static int bn_check(int M, int C, int act, ogv_dtype dt, const char* fn) {
  OGV_REQUIRE(M > 0 && C > 0, "%s: bad shape M=%d C=%d", fn, M, C);
  OGV_REQUIRE(dt == OGV_F32 || dt == OGV_BF16, "%s: bad dtype %d", fn, (int)dt);
  OGV_REQUIRE(act >= OGV_ACT_NONE && act <= OGV_ACT_RELU, "%s: bad act %d", fn, act);
  return OGV_OK;
}

extern "C" size_t ogv_bn_act_saved_bytes(int C) { return 4 * (size_t)(C > 0 ? C : 0) * sizeof(float) + 1024; }

extern "C" size_t ogv_bn_act_ws_bytes(int M, int C) {
  if (M <= 0 || C <= 0) return 0;
  const RowSlices rs = row_slices(M);
  Carve c(nullptr);  // sized for the fp64 forward layout (>= the fp32 backward one)
  c.take<double>((size_t)rs.S * 2 * C);
  c.take<double>(2 * (size_t)C);
  c.take<double>(colreduce_tmp_floats(rs.S, 2L * C));
  c.take<float>(3 * (size_t)C);
  return c.off;
}

extern "C" int ogv_bn_act_fwd(const void* x, void* out, float* saved, void* ws, const float* bn_w, const float* bn_b,
                              float* rm, float* rv, int M, int C, int train, float eps, float momentum, int act,
                              ogv_dtype dt, void* stream) {
  int rc = bn_check(M, C, act, dt, "ogv_bn_act_fwd");
  if (rc) return rc;
  OGV_REQUIRE(x && out && saved && ws && rm && rv, "ogv_bn_act_fwd: null pointer");
  hipStream_t s = as_stream(stream);
  Carve cs(saved);
  const BnSaved b = take_bn_saved(cs, C);
  const RowSlices rs = row_slices(M);
  Carve cw(ws);
  double* stat = cw.take<double>((size_t)rs.S * 2 * C);
  double* sums = cw.take<double>(2 * (size_t)C);
  double* tmp = cw.take<double>(colreduce_tmp_floats(rs.S, 2L * C));
  const int V = vec_width(C);
  if (train) {
    OGV_CB_DISPATCH(dt, V, bn_stats_run, x, rm, stat, (long)M, C, rs, s);
    bn_reduce_finalize_launch(stat, rs.S, 2L * C, C, (double)M, bn_w, bn_b, eps, momentum, rm, rv, b.mean, b.invstd,
                              b.sc, b.sh, s);
  } else {
    bn_finalize_launch(sums, C, (double)M, bn_w, bn_b, eps, momentum, rm, rv, b.mean, b.invstd, b.sc, b.sh, train, s);
  }
  OGV_CB_DISPATCH(dt, V, bn_apply_run, x, b.sc, b.sh, act, out, (long)M, C, s);
  return check_launch("ogv_bn_act_fwd");
}

extern "C" int ogv_bn_act_bwd(const void* dout, const void* x, const float* saved, void* dx, float* dbn_w,
                              float* dbn_b, void* ws, const float* bn_w, int M, int C, int train, int act,
                              ogv_dtype dt, void* stream) {
  int rc = bn_check(M, C, act, dt, "ogv_bn_act_bwd");
  if (rc) return rc;
  OGV_REQUIRE(dout && x && saved && ws && dx, "ogv_bn_act_bwd: null pointer");
  hipStream_t s = as_stream(stream);
  Carve cs(const_cast<float*>(saved));
  const BnSaved b = take_bn_saved(cs, C);
  const RowSlices rs = row_slices(M);
  Carve cw(ws);
  float* stat = cw.take<float>((size_t)rs.S * 2 * C);
  float* sums = cw.take<float>(2 * (size_t)C);
  float* tmp = cw.take<float>(colreduce_tmp_floats(rs.S, 2L * C));
  float* coef = cw.take<float>(3 * (size_t)C);
  const int V = vec_width(C);
  OGV_CB_DISPATCH(dt, V, bn_bwd_reduce_run, dout, x, b.sc, b.sh, act, b.mean, b.invstd, stat, (long)M, C, rs, s);
  bn_reduce_coeffs_launch(stat, rs.S, 2L * C, C, (float)M, bn_w, b.invstd, dbn_w, dbn_b, coef, train, s);
  OGV_CB_DISPATCH(dt, V, bn_bwd_apply_run, dout, x, b.sc, b.sh, act, b.mean, b.invstd, coef, dx, (long)M, C, s);
  return check_launch("ogv_bn_act_bwd");
}

namespace ogv {

// ------------------------------------------------------------------ head: BatchNorm2d + global average pool
// Block = 4 channel chunks of V x 64 images: each thread walks its image's HW rows for its chunk (the image's
// channel sums stay in the thread: pooled_raw = sum / HW is written directly), and the fp64 shifted BatchNorm
// sums of the block's 64 images are reduced into one partial row ([blk][0..C) and [blk][C..2C), the layout
// bn_reduce_finalize reads).  One read of x; ceil(B / 64) partial rows.
constexpr int HP_IMG = 64;
template <typename T, int V>
__global__ __launch_bounds__(256) void head_pool_stats_kernel(const T* __restrict__ x, const float* __restrict__ shift,
                                                              double* __restrict__ stat, float* __restrict__ raw, int B,
                                                              int HW, int C) {
  __shared__ double lds[2 * 4 * 4 * 8];
  const int gx = (C + 4 * V - 1) / (4 * V);
  const int bx = (int)(blockIdx.x % gx), by = (int)(blockIdx.x / gx);
  const int chunk = threadIdx.x & 3, im = threadIdx.x >> 2;
  const int c0 = (bx * 4 + chunk) * V;
  const int b = by * HP_IMG + im;
  double q[2][V];
#pragma unroll
  for (int i = 0; i < V; ++i) { q[0][i] = 0.0; q[1][i] = 0.0; }
  if (c0 < C && b < B) {
    float sf[V];
    load_vec<float, V>(shift + c0, sf);
    double sx[V];
#pragma unroll
    for (int i = 0; i < V; ++i) { sf[i] = bn_shift(sf[i]); sx[i] = 0.0; }
    const T* xb = x + (long)b * HW * C + c0;
    int r = 0;
    for (; r + 4 <= HW; r += 4) {
      float v[4][V];
#pragma unroll
      for (int u = 0; u < 4; ++u) load_vec<T, V>(xb + (long)(r + u) * C, v[u]);
#pragma unroll
      for (int u = 0; u < 4; ++u)
#pragma unroll
        for (int i = 0; i < V; ++i) {
          const double d = (double)v[u][i] - (double)sf[i];
          q[0][i] += d;
          q[1][i] = fma(d, d, q[1][i]);
          sx[i] += (double)v[u][i];
        }
    }
    for (; r < HW; ++r) {
      float v[V];
      load_vec<T, V>(xb + (long)r * C, v);
#pragma unroll
      for (int i = 0; i < V; ++i) {
        const double d = (double)v[i] - (double)sf[i];
        q[0][i] += d;
        q[1][i] = fma(d, d, q[1][i]);
        sx[i] += (double)v[i];
      }
    }
    float m[V];
#pragma unroll
    for (int i = 0; i < V; ++i) m[i] = (float)(sx[i] / (double)HW);
    store_vec<float, V>(raw + (long)b * C + c0, m);
  }
  chunk_reduce_store<2, V, double>(q, lds, stat + (long)by * 2 * C, C, C, bx * 4 * V);
}

// pooled = pooled_raw * sc + sh   ([B, C], thread per element)
__global__ void head_pool_apply_kernel(const float* __restrict__ raw, const float* __restrict__ sc,
                                       const float* __restrict__ sh, float* __restrict__ pooled, int B, int C) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (long)B * C) return;
  const int c = (int)(i % C);
  pooled[i] = fmaf(raw[i], sc[c], sh[c]);
}

// backward partial rows, one per image: [g, g * xhat_b] with xhat_b = (pooled_raw - mean) * invstd -- the
// image's sum over its pixels of dz = g / HW and of dz * xhat
__global__ void head_pool_bwd_stats_kernel(const float* __restrict__ g, const float* __restrict__ raw,
                                           const float* __restrict__ mean, const float* __restrict__ invstd,
                                           float* __restrict__ stat, int B, int C) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (long)B * C) return;
  const int b = (int)(i / C), c = (int)(i - (long)b * C);
  const float gv = g[i];
  stat[(long)b * 2 * C + c] = gv;
  stat[(long)b * 2 * C + C + c] = gv * ((raw[i] - mean[c]) * invstd[c]);
}

// dx = coef0 * (g[b] / HW - coef1 - (x - mean) * invstd * coef2)
template <typename T, int V>
__global__ __launch_bounds__(256) void head_pool_dx_kernel(const float* __restrict__ g, const T* __restrict__ x,
                                                           const float* __restrict__ mean,
                                                           const float* __restrict__ invstd,
                                                           const float* __restrict__ coef, T* __restrict__ dx, int HW,
                                                           long M, int C) {
  const int nch = C / V;
  const long tid = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (tid >= M * nch) return;
  const int c0 = (int)(tid % nch) * V;
  const long m = tid / nch, b = m / HW;
  const float ihw = 1.f / (float)HW;
  float v[V], gv[V], mu[V], is[V], ca[V], cb[V], cc[V];
  load_vec<T, V>(x + m * C + c0, v);
  load_vec<float, V>(g + b * C + c0, gv);
  load_vec<float, V>(mean + c0, mu);
  load_vec<float, V>(invstd + c0, is);
  load_vec<float, V>(coef + c0, ca);
  load_vec<float, V>(coef + C + c0, cb);
  load_vec<float, V>(coef + 2 * C + c0, cc);
#pragma unroll
  for (int i = 0; i < V; ++i) v[i] = ca[i] * (gv[i] * ihw - cb[i] - (v[i] - mu[i]) * is[i] * cc[i]);
  store_vec<T, V>(dx + m * C + c0, v);
}

template <typename T, int V>
static void head_stats_run(const void* x, const float* shift, double* stat, float* raw, int B, int HW, int C,
                           hipStream_t s) {
  head_pool_stats_kernel<T, V><<<cdiv(C, 4 * V) * cdiv(B, HP_IMG), 256, 0, s>>>((const T*)x, shift, stat, raw, B, HW, C);
}
template <typename T, int V>
static void head_dx_run(const float* g, const void* x, const float* mean, const float* invstd, const float* coef, void* dx,
                        int HW, long M, int C, hipStream_t s) {
  head_pool_dx_kernel<T, V><<<cdiv(M * (C / V), 256), 256, 0, s>>>(g, (const T*)x, mean, invstd, coef, (T*)dx, HW, M, C);
}

static int head_check(int B, int HW, int C, ogv_dtype dt, const char* fn) {
  OGV_REQUIRE(B > 0 && HW > 0 && C > 0 && (long)B * HW <= INT32_MAX, "%s: bad shape B=%d HW=%d C=%d", fn, B, HW, C);
  OGV_REQUIRE(dt == OGV_F32 || dt == OGV_BF16, "%s: bad dtype %d", fn, (int)dt);
  return OGV_OK;
}

}  // namespace ogv

using namespace ogv;

extern "C" size_t ogv_head_bn_pool_ws_bytes(int B, int C) {
  if (B <= 0 || C <= 0) return 0;
  Carve c(nullptr);   // forward: fp64 [ceil(B / 64)][2C] + finalize scratch; backward: fp32 [B][2C] + coef [3C]
  const size_t fwd = (size_t)cdiv(B, HP_IMG) * 2 * C * sizeof(double) + 2 * (size_t)C * sizeof(double);
  const size_t bwd = ((size_t)B * 2 * C + 3 * (size_t)C) * sizeof(float);
  c.take<char>((fwd > bwd ? fwd : bwd) + 256);
  return c.off;
}

extern "C" int ogv_head_bn_pool_fwd(const void* x, float* pooled_raw, float* pooled, float* saved, void* ws,
                                    const float* bn_w, const float* bn_b, float* rm, float* rv, int B, int HW, int C,
                                    int train, float eps, float momentum, ogv_dtype dt, void* stream) {
  int rc = head_check(B, HW, C, dt, "ogv_head_bn_pool_fwd");
  if (rc) return rc;
  OGV_REQUIRE(x && pooled_raw && pooled && saved && ws && rm && rv, "ogv_head_bn_pool_fwd: null pointer");
  hipStream_t s = as_stream(stream);
  Carve cs(saved);
  const BnSaved b = take_bn_saved(cs, C);
  Carve cw(ws);
  const int R = cdiv(B, HP_IMG);
  double* stat = cw.take<double>((size_t)R * 2 * C);
  double* sums = cw.take<double>(2 * (size_t)C);
  const int V = vec_width(C);
  OGV_CB_DISPATCH(dt, V, head_stats_run, x, rm, stat, pooled_raw, B, HW, C, s);
  if (train)
    bn_reduce_finalize_launch(stat, R, 2L * C, C, (double)B * HW, bn_w, bn_b, eps, momentum, rm, rv, b.mean, b.invstd,
                              b.sc, b.sh, s);
  else
    bn_finalize_launch(sums, C, (double)B * HW, bn_w, bn_b, eps, momentum, rm, rv, b.mean, b.invstd, b.sc, b.sh, 0, s);
  head_pool_apply_kernel<<<cdiv((long)B * C, 256), 256, 0, s>>>(pooled_raw, b.sc, b.sh, pooled, B, C);
  return check_launch("ogv_head_bn_pool_fwd");
}

extern "C" int ogv_head_bn_pool_bwd(const float* dpooled, const void* x, const float* pooled_raw, const float* saved,
                                    void* dx, float* dbn_w, float* dbn_b, void* ws, const float* bn_w, int B, int HW,
                                    int C, int train, ogv_dtype dt, void* stream) {
  int rc = head_check(B, HW, C, dt, "ogv_head_bn_pool_bwd");
  if (rc) return rc;
  OGV_REQUIRE(dpooled && x && pooled_raw && saved && ws && dx, "ogv_head_bn_pool_bwd: null pointer");
  hipStream_t s = as_stream(stream);
  Carve cs(const_cast<float*>(saved));
  const BnSaved b = take_bn_saved(cs, C);
  Carve cw(ws);
  float* stat = cw.take<float>((size_t)B * 2 * C);
  float* coef = cw.take<float>(3 * (size_t)C);
  head_pool_bwd_stats_kernel<<<cdiv((long)B * C, 256), 256, 0, s>>>(dpooled, pooled_raw, b.mean, b.invstd, stat, B, C);
  bn_reduce_coeffs_launch(stat, B, 2L * C, C, (float)((double)B * HW), bn_w, b.invstd, dbn_w, dbn_b, coef, train, s);
  const int V = vec_width(C);
  OGV_CB_DISPATCH(dt, V, head_dx_run, dpooled, x, b.mean, b.invstd, coef, dx, HW, (long)B * HW, C, s);
  return check_launch("ogv_head_bn_pool_bwd");
}
