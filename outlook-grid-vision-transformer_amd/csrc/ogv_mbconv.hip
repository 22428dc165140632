// Fused MBConv (src/model/mbc_conv.py:44-98) for the OutGridBlock path:
//   e  = x . We^T                      expand 1x1, no bias   (+ BN1 batch stats in the GEMM epilogue)
//   a1 = act(BN1(e))                   applied on the fly by the depthwise conv's loads
//   d  = dw3x3(a1)                     (+ BN2 batch stats in the conv epilogue)
//   a2 = act(BN2(d))
//   g  = sigmoid(W2 act(W1 mean_hw(a2) + b1) + b2)        SqueezeExcite (:22-27), B rows only
//   p  = (a2 * g) . Wp^T               project 1x1: BN2-apply, act and the SE gate in the A prologue
//                                      (+ BN3 batch stats in the epilogue)
//   out = x + BN3(p)
// BatchNorm2d semantics (train): normalise with the biased batch variance, update running_mean /
// running_var (unbiased) with momentum 0.1; eval: running statistics.  Batch statistics are
// accumulated as per-panel sums of (v - running_mean) and (v - running_mean)^2 (shifted sums: no
// cancellation once the running mean tracks the batch mean) and reduced deterministically.
//
// Backward is hand-scheduled: the five per-(image, channel) reductions the SE and BN2 backward
// need are taken in ONE pass over (dA3, d); BN1's reductions ride in the depthwise-dgrad epilogue.
// HBM passes over the [M, mid] tensors: fwd 4 (e write, e read+d write, d read for the pool, d
// read for project), bwd 9.
#include "ogv_gemm.h"
#include "ogv_bn.h"

namespace ogv {

struct RowPlan {
  int V, nch, nchb, lanes, ctiles;
};
static RowPlan row_plan(int K) {
  RowPlan p;
  p.V = K % 8 == 0 ? 8 : (K % 4 == 0 ? 4 : 1);
  p.nch = K / p.V;
  p.nchb = p.nch < 64 ? p.nch : 64;
  p.lanes = 256 / p.nchb;
  p.ctiles = (p.nch + p.nchb - 1) / p.nchb;
  return p;
}

// ------------------------------------------------------------------ BN finalize / coefficients
// train: mean = shift + S1/n, var = S2/n - (S1/n)^2; running stats updated (unbiased var).
// eval : mean/var = running stats.  Emits invstd, sc = gamma*invstd, sh = beta - mean*sc.
__global__ void bn_finalize_kernel(const double* __restrict__ sums, int K, double n, const float* __restrict__ gamma,
                                   const float* __restrict__ beta, float eps, float momentum, float* rm, float* rv,
                                   float* __restrict__ mean_out, float* __restrict__ invstd_out, float* __restrict__ sc,
                                   float* __restrict__ sh, int train) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= K) return;
  float mean, var;
  if (train) {
    const double s1 = sums[c] / n, s2 = sums[K + c] / n;
    const double shift = bn_shift(rm[c]);
    mean = (float)(shift + s1);
    double v = s2 - s1 * s1;
    var = (float)(v > 0.0 ? v : 0.0);
    rm[c] = (1.f - momentum) * rm[c] + momentum * mean;
    rv[c] = (1.f - momentum) * rv[c] + momentum * (float)(var * (n / (n > 1.0 ? n - 1.0 : 1.0)));
  } else {
    mean = rm[c];
    var = rv[c];
  }
  const float is = rsqrtf(var + eps);
  const float g = gamma ? gamma[c] : 1.f, b = beta ? beta[c] : 0.f;
  mean_out[c] = mean;
  invstd_out[c] = is;
  sc[c] = g * is;
  sh[c] = b - mean * g * is;
}

// From S = [sum dy, sum dy*xhat]: dgamma, dbeta and the apply coefficients
// dx = ca*(dy - cb - xhat*cc),  ca = gamma*invstd, (cb, cc) = (S0, S1)/n in train, 0 in eval.
__global__ void bn_coeffs_kernel(const float* __restrict__ S, int K, float n, const float* __restrict__ gamma,
                                 const float* __restrict__ invstd, float* __restrict__ dgamma, float* __restrict__ dbeta,
                                 float* __restrict__ coef, int train) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= K) return;
  const float sdy = S[c], sdyx = S[K + c];
  if (dgamma) dgamma[c] = sdyx;
  if (dbeta) dbeta[c] = sdy;
  coef[c] = (gamma ? gamma[c] : 1.f) * invstd[c];
  coef[K + c] = train ? sdy / n : 0.f;
  coef[2 * K + c] = train ? sdyx / n : 0.f;
}

// Fused column reduction + finalize / coefficients: a block owns 16 channels, its RG row groups walk
// the [R][ld] partial rows (columns c and K + c) in a fixed order, combined in a fixed order in LDS;
// one launch instead of colreduce + bn_finalize / bn_coeffs.  The walk is latency-bound (a few dozen
// blocks, thousands of partial rows): knob "bn_red_rg" (16 or 64, default 64) sets the row groups, i.e.
// the loads in flight per channel (16 x RG threads per block): 7M step, 30 steps x 2, 16 -> 14.743 / 14.757 ms,
// 64 -> 14.733 / 14.714 (profiles/r05s_bn_red_rg.log)
static int g_bn_red_rg = 64;
void set_bn_red_rg(int v) { g_bn_red_rg = v >= 64 ? 64 : 16; }
template <int RG>
__global__ __launch_bounds__(16 * RG) void bn_reduce_finalize_kernel(const double* __restrict__ part, long R, long ld, int K,
                                                                 double n, const float* __restrict__ gamma,
                                                                 const float* __restrict__ beta, float eps,
                                                                 float momentum, float* rm, float* rv,
                                                                 float* __restrict__ mean_out,
                                                                 float* __restrict__ invstd_out, float* __restrict__ sc,
                                                                 float* __restrict__ sh) {
  __shared__ double red[2][RG][16];
  const int cl = threadIdx.x & 15, rg = threadIdx.x >> 4;
  const int c = blockIdx.x * 16 + cl;
  double s1 = 0.0, s2 = 0.0;
  if (c < K) {   // four row groups' loads in flight per trip (the loop is latency-bound otherwise)
    double a1[4] = {0.0, 0.0, 0.0, 0.0}, a2[4] = {0.0, 0.0, 0.0, 0.0};
    long r = rg;
    for (; r + 3 * RG < R; r += 4 * RG) {
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        a1[u] += part[(r + RG * u) * ld + c];
        a2[u] += part[(r + RG * u) * ld + K + c];
      }
    }
    for (; r < R; r += RG) {
      a1[0] += part[r * ld + c];
      a2[0] += part[r * ld + K + c];
    }
    s1 = (a1[0] + a1[1]) + (a1[2] + a1[3]);
    s2 = (a2[0] + a2[1]) + (a2[2] + a2[3]);
  }
  red[0][rg][cl] = s1;
  red[1][rg][cl] = s2;
  __syncthreads();
  if (rg != 0 || c >= K) return;
  double t1 = 0.0, t2 = 0.0;
#pragma unroll 16
  for (int g = 0; g < RG; ++g) {
    t1 += red[0][g][cl];
    t2 += red[1][g][cl];
  }
  const double m1 = t1 / n, m2 = t2 / n;
  const float mean = (float)((double)bn_shift(rm[c]) + m1);
  const double v = m2 - m1 * m1;
  const float var = (float)(v > 0.0 ? v : 0.0);
  rm[c] = (1.f - momentum) * rm[c] + momentum * mean;
  rv[c] = (1.f - momentum) * rv[c] + momentum * (float)(var * (n / (n > 1.0 ? n - 1.0 : 1.0)));
  const float is = rsqrtf(var + eps);
  const float gm = gamma ? gamma[c] : 1.f, bt = beta ? beta[c] : 0.f;
  mean_out[c] = mean;
  invstd_out[c] = is;
  sc[c] = gm * is;
  sh[c] = bt - mean * gm * is;
}

// BN2 (TERMS): the partial rows are not stored -- row b is formed from the SE reduce's per-image sums
// R[5][B][K], the gate and dpool/HW.  dy2 = (dA3*gate + dpool/HW) * s', so
//   sum dy2 = sum_b gate*R1 + dpool/HW*R2,  sum dy2*dh = sum_b gate*R3 + dpool/HW*R4
struct Bn2Terms {
  const float *R, *gate, *dpool;
  int HW;
};
template <bool TERMS, int RG>
__global__ __launch_bounds__(16 * RG) void bn_reduce_coeffs_kernel(const float* __restrict__ part, long R, long ld, int K,
                                                               float n, const float* __restrict__ gamma,
                                                               const float* __restrict__ invstd,
                                                               float* __restrict__ dgamma, float* __restrict__ dbeta,
                                                               float* __restrict__ coef, int train, Bn2Terms bt = {}) {
  __shared__ float red[2][RG][16];
  const int cl = threadIdx.x & 15, rg = threadIdx.x >> 4;
  const int c = blockIdx.x * 16 + cl;
  float s1 = 0.f, s2 = 0.f;
  // row r's two partials: stored ([R][ld]), or the BN2 terms of image r
  const long BK = R * K;
  const float ihw = TERMS ? 1.f / (float)bt.HW : 0.f;
  auto row = [&](long r, float& v1, float& v2) {
    if constexpr (TERMS) {
      const long i = r * K + c;
      const float gg = bt.gate[i], dp = bt.dpool[i] * ihw;
      v1 = gg * bt.R[1 * BK + i] + dp * bt.R[2 * BK + i];
      v2 = gg * bt.R[3 * BK + i] + dp * bt.R[4 * BK + i];
    } else {
      v1 = part[r * ld + c];
      v2 = part[r * ld + K + c];
    }
  };
  if (c < K) {   // four row groups' loads in flight per trip
    float a1[4] = {0.f, 0.f, 0.f, 0.f}, a2[4] = {0.f, 0.f, 0.f, 0.f};
    long r = rg;
    for (; r + 3 * RG < R; r += 4 * RG) {
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        float v1, v2;
        row(r + RG * u, v1, v2);
        a1[u] += v1;
        a2[u] += v2;
      }
    }
    for (; r < R; r += RG) {
      float v1, v2;
      row(r, v1, v2);
      a1[0] += v1;
      a2[0] += v2;
    }
    s1 = (a1[0] + a1[1]) + (a1[2] + a1[3]);
    s2 = (a2[0] + a2[1]) + (a2[2] + a2[3]);
  }
  red[0][rg][cl] = s1;
  red[1][rg][cl] = s2;
  __syncthreads();
  if (rg != 0 || c >= K) return;
  float sdy = 0.f, sdyx = 0.f;
#pragma unroll 16
  for (int g = 0; g < RG; ++g) {
    sdy += red[0][g][cl];
    sdyx += red[1][g][cl];
  }
  if (dgamma) dgamma[c] = sdyx;
  if (dbeta) dbeta[c] = sdy;
  coef[c] = (gamma ? gamma[c] : 1.f) * invstd[c];
  coef[K + c] = train ? sdy / n : 0.f;
  coef[2 * K + c] = train ? sdyx / n : 0.f;
}

void bn_reduce_finalize_launch(const double* part, long R, long ld, int K, double n, const float* gamma,
                               const float* beta, float eps, float momentum, float* rm, float* rv, float* mean,
                               float* invstd, float* sc, float* sh, hipStream_t s) {
  if (g_bn_red_rg == 64)
    bn_reduce_finalize_kernel<64><<<cdiv(K, 16), 16 * 64, 0, s>>>(part, R, ld, K, n, gamma, beta, eps, momentum, rm, rv,
                                                                   mean, invstd, sc, sh);
  else
    bn_reduce_finalize_kernel<16><<<cdiv(K, 16), 16 * 16, 0, s>>>(part, R, ld, K, n, gamma, beta, eps, momentum, rm, rv,
                                                                   mean, invstd, sc, sh);
}
template <bool TERMS = false>
void bn_reduce_coeffs_run(const float* part, long R, long ld, int K, float n, const float* gamma, const float* invstd,
                          float* dgamma, float* dbeta, float* coef, int train, hipStream_t s, Bn2Terms bt = {}) {
  if (g_bn_red_rg == 64)
    bn_reduce_coeffs_kernel<TERMS, 64><<<cdiv(K, 16), 16 * 64, 0, s>>>(part, R, ld, K, n, gamma, invstd, dgamma, dbeta,
                                                                       coef, train, bt);
  else
    bn_reduce_coeffs_kernel<TERMS, 16><<<cdiv(K, 16), 16 * 16, 0, s>>>(part, R, ld, K, n, gamma, invstd, dgamma, dbeta,
                                                                       coef, train, bt);
}
void bn_reduce_coeffs_launch(const float* part, long R, long ld, int K, float n, const float* gamma,
                             const float* invstd, float* dgamma, float* dbeta, float* coef, int train, hipStream_t s) {
  bn_reduce_coeffs_run(part, R, ld, K, n, gamma, invstd, dgamma, dbeta, coef, train, s);
}
void bn_finalize_launch(const double* sums, int K, double n, const float* gamma, const float* beta, float eps,
                        float momentum, float* rm, float* rv, float* mean, float* invstd, float* sc, float* sh, int train,
                        hipStream_t s) {
  bn_finalize_kernel<<<cdiv(K, 256), 256, 0, s>>>(sums, K, n, gamma, beta, eps, momentum, rm, rv, mean, invstd, sc, sh,
                                                   train);
}
void bn_coeffs_launch(const float* S, int K, float n, const float* gamma, const float* invstd, float* dgamma,
                      float* dbeta, float* coef, int train, hipStream_t s) {
  bn_coeffs_kernel<<<cdiv(K, 256), 256, 0, s>>>(S, K, n, gamma, invstd, dgamma, dbeta, coef, train);
}

// ------------------------------------------------------------------ depthwise conv with BN fusion
// ---- row-streaming depthwise kernels -------------------------------------------------------
// Block = (group of G images, column strip of TW <= 32 pixels, channel tile of CT = chunks*V
// channels), XCD-aware order with the channel tile fastest.  The block walks its images stacked into
// one tall strip of "virtual rows" (H rows per image plus one zero row between images, so the 3x3
// halo never mixes images), DW_R output rows per step: a (DW_R+2)-row ring in LDS holds input rows
// u-1 .. u+DW_R (TW+2 pixels with the column halo, zero outside the image, the producer's BatchNorm
// + activation applied once per element as it is staged) and the next DW_R rows are loaded into
// registers while the current ones are computed, so every input element is read from HBM once,
// ~DW_R rows per block are in flight, and the pipeline runs on across image seams (one prologue and
// one weight load per block, G chosen for ~one wave of resident blocks).  chunks is chosen so that
// one output row is ~256 (pixel, V-channel chunk) items: one per thread per row.  Statistics /
// weight-gradient partials are reduced once per block into row rid = group*ncolt + colt of a
// [rows][Q][C] slab.
constexpr int DW_R = 4;   // the data / weight-gradient kernels (two sources + per-pixel loads: VGPR-bound)
// the forward kernel's rows per step, knob "dw_fwd_r" (4 or 8): 8 rows per step (one source, ~124 VGPRs:
// room for the deeper row pipeline) measured 16.14-16.16 vs 16.08-16.13 ms/step at 4 (7M, paired,
// profiles/r04_dw_fwd_r.log): the kernel is not bound by loads in flight, so 4 stays the default
static int g_dw_fwd_r = 4;
void set_dw_fwd_r(int v) { g_dw_fwd_r = v == 4 ? 4 : 8; }
// tuning knob "dw_blocks": > 0 = target block count of the depthwise kernels; 0 (default) = images
// per block chosen for ~32 output rows per block (many short blocks balance best over the CUs)
static int g_dw_blocks = 0;
void set_dw_blocks(int v) { g_dw_blocks = v > 0 ? v : 0; }
// knob "dw_tw": the column strip width (pixels, 8 / 16 / 32; default 32): a narrower strip widens the
// channel tile (~256 (pixel, 4-channel) items per row), i.e. more contiguous bytes per pixel per load
static int g_dw_tw = 32;
void set_dw_tw(int v) { g_dw_tw = v <= 8 ? 8 : (v <= 16 ? 16 : 32); }
struct DwTile {
  int B, H, W, C, TW, ncolt, chunks, CT, nct, PP, ldq, G, ngroups;
  __host__ __device__ long rows() const { return (long)ngroups * ncolt; }
  long rows_max() const { return (long)B * ncolt; }  // workspace sizing: any G
  __host__ __device__ long nblocks() const { return rows() * nct; }
  size_t ring_bytes(int R = DW_R) const { return (size_t)(R + 2) * (TW + 2) * PP * sizeof(float); }
  size_t lds_bytes(int nq, int V, size_t asz, int R = DW_R) const {
    const size_t red = (size_t)4 * chunks * nq * V * asz;
    return ring_bytes(R) > red ? ring_bytes(R) : red;
  }
};
static DwTile dw_tile_plan(int B, int H, int W, int C, int V) {
  DwTile t;
  t.B = B; t.H = H; t.W = W; t.C = C;
  t.TW = W < g_dw_tw ? W : g_dw_tw;
  t.ncolt = (W + t.TW - 1) / t.TW;
  int ch = 1;
  while (ch * 2 * t.TW <= 256 && ch < 64) ch *= 2;            // ~256 items per output row
  while (ch > 1 && (ch / 2) * V >= C) ch /= 2;                // do not exceed the channel count
  t.chunks = ch;
  t.CT = ch * V;
  t.nct = (C + t.CT - 1) / t.CT;
  t.PP = t.CT;  // unpadded: conflict-free ds_read_b128 lane groups for the tap reads (chunks >= 8)
  t.ldq = ((t.TW + 2) * ch + 255) / 256;                      // row-load items per thread (<= 3)
  long G;
  if (g_dw_blocks > 0) {
    const long tiles = (long)B * t.ncolt * t.nct;
    G = (tiles + g_dw_blocks - 1) / g_dw_blocks;
  } else {
    G = 32 / H;
  }
  G = G < 1 ? 1 : (G > B ? B : G);
  t.G = (int)G;
  t.ngroups = (int)((B + G - 1) / G);
  return t;
}
static unsigned dw_grid(const DwTile& t) { return xcd_grid(t.nblocks()); }

struct TileIdx {
  int ct, colt, x0, tw, nimg;
  long b0, rid;
};
__device__ __forceinline__ bool tile_idx(const DwTile& t, TileIdx& i) {
  long id;
  if (!xcd_block(t.nblocks(), id)) return false;
  i.ct = (int)(id % t.nct); id /= t.nct;
  i.colt = (int)(id % t.ncolt);
  const long g = id / t.ncolt;
  i.rid = g * t.ncolt + i.colt;
  i.b0 = g * t.G;
  i.nimg = (int)(t.B - i.b0 < t.G ? t.B - i.b0 : t.G);
  i.x0 = i.colt * t.TW;
  i.tw = t.W - i.x0 < t.TW ? t.W - i.x0 : t.TW;
  return true;
}
// virtual row u (>= -1) = (image im of the block's group, row y); y == H is the zero seam row.
// Walked one row at a time (no division).
struct VRow {
  int u, im, y;
};
__device__ __forceinline__ VRow vnext(const DwTile& t, VRow p) {
  ++p.u;
  if (++p.y > t.H) {
    p.y = 0;
    ++p.im;
  }
  return p;
}
template <int K>
__device__ __forceinline__ VRow vadv(const DwTile& t, VRow p) {
#pragma unroll
  for (int k = 0; k < K; ++k) p = vnext(t, p);
  return p;
}

template <int R = DW_R>
__device__ __forceinline__ int ring_slot(int r) { return (r + R + 2) % (R + 2); }
template <int R = DW_R>
__device__ __forceinline__ const float* ring_px(const float* ring, const DwTile& t, int r, int px) {
  return ring + ((size_t)ring_slot<R>(r) * (t.TW + 2) + px) * t.PP;
}


// Up to DW_R input rows (TW+2 pixels incl. halo) of the block's channel tile, in registers.  The
// loads are unconditional (addresses clamped into the tensor); the zero padding, the producer's
// transform (stage(v, v2, image): BatchNorm + activation forward, or the whole BN2 backward from
// the two sources (dA3, d) when TWO) and the conversion to fp32 are applied as the rows enter the
// LDS ring.
template <typename T, int V, int LDQ, bool TWO = false, int R = DW_R>
struct RowPipe {
  RawVec<T, V> raw[R][LDQ];
  RawVec<T, V> raw2[TWO ? R : 1][TWO ? LDQ : 1];
  template <int NR>
  __device__ __forceinline__ void load(const T* __restrict__ src, const T* __restrict__ src2, const DwTile& t,
                                       const TileIdx& ti, VRow p, int cc) {
#pragma unroll
    for (int r = 0; r < NR; ++r) {
      const long b = ti.b0 + min(max(p.im, 0), ti.nimg - 1);
      const int y = min(p.y, t.H - 1);
#pragma unroll
      for (int j = 0; j < LDQ; ++j) {
        const int i = threadIdx.x + j * 256;
        const int x = min(max(ti.x0 - 1 + i / t.chunks, 0), t.W - 1);
        const long off = ((b * t.H + y) * t.W + x) * t.C + cc;
        raw[r][j].load(src + off);
        if constexpr (TWO) raw2[r][j].load(src2 + off);
      }
      p = vnext(t, p);
    }
  }
  template <typename Stage>
  __device__ __forceinline__ void store(float* ring, const DwTile& t, const TileIdx& ti, VRow p, int nr, int chunk,
                                        bool cok, Stage&& stage) const {
    const int n = (ti.tw + 2) * t.chunks;
#pragma unroll
    for (int r = 0; r < R; ++r, p = vnext(t, p)) {
      if (r >= nr) break;
      const bool rok = cok && p.im >= 0 && p.im < ti.nimg && p.y < t.H;
      const int im = min(max(p.im, 0), ti.nimg - 1);
      float* slot = ring + (size_t)ring_slot<R>(p.u) * (t.TW + 2) * t.PP;
#pragma unroll
      for (int j = 0; j < LDQ; ++j) {
        const int i = threadIdx.x + j * 256;
        if (i < n) {
          const int x = ti.x0 - 1 + i / t.chunks;
          const bool ok = rok && x >= 0 && x < t.W;
          float v[V];
          raw[r][j].unpack(v);
          if constexpr (TWO) {
            float v2[V];
            raw2[r][j].unpack(v2);
            stage(v, v2, im);
          } else {
            stage(v, v, im);
          }
#pragma unroll
          for (int k = 0; k < V; ++k) v[k] = ok ? v[k] : 0.f;
          float* d = slot + (i / t.chunks) * t.PP + chunk * V;
#pragma unroll
          for (int k = 0; k < V; k += 4)
            *reinterpret_cast<float4*>(d + k) = make_float4(v[k], v[k + 1], v[k + 2], v[k + 3]);
        }
      }
    }
  }
};

// Sum the per-thread q[NQ][V] over the threads sharing a channel chunk (chunk = tid % chunks):
// xor-shuffles inside each wave, then the 4 waves through LDS (reused ring).  out[k*qstride + c].
template <int NQ, int V, typename A>
__device__ __forceinline__ void dw_reduce_store(A (&q)[NQ][V], float* lds_raw, int chunks, A* out, long qstride,
                                                int C, int c0, const float* gate = nullptr, float* dz = nullptr) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
  for (int k = 0; k < NQ; ++k)
#pragma unroll
    for (int i = 0; i < V; ++i)
      for (int o = chunks; o < 64; o <<= 1) q[k][i] += __shfl_xor(q[k][i], o, 64);
  A* lds = reinterpret_cast<A*>(lds_raw);
  __syncthreads();
  if (lane < chunks) {
#pragma unroll
    for (int k = 0; k < NQ; ++k)
#pragma unroll
      for (int i = 0; i < V; ++i) lds[((wave * chunks + lane) * NQ + k) * V + i] = q[k][i];
  }
  __syncthreads();
  for (int idx = threadIdx.x; idx < chunks * NQ * V; idx += 256) {
    const int ch = idx / (NQ * V), r = idx - ch * NQ * V, k = r / V, i = r - k * V;
    A sum = 0;
#pragma unroll
    for (int w = 0; w < 4; ++w) sum += lds[((w * chunks + ch) * NQ + k) * V + i];
    const int c = c0 + ch * V + i;
    if (c < C) {
      out[(long)k * qstride + c] = sum;
      if (dz && k == 0) dz[c] = (float)sum * gate[c] * (1.f - gate[c]);  // SE sigmoid backward, fused
    }
  }
}

// The shared row walk over the block's virtual rows: ring <- rows -1, 0; regs <- rows 1..R; per
// step: store regs (rows u+1..u+R), issue the prefetch of rows u+R+1..u+2R (always: past the end it
// re-reads a clamped row), then pre(u+R, px, slot') issues the body's own per-pixel loads for the NEXT
// step's output rows into the other buffer, then the output rows among u..u+R-1 (not seam rows) are
// computed through body(r, u+r, image, y, px, slot), one item (pixel, V channels) per thread and row, from
// the per-pixel data loaded one step earlier.  Issue order = retire order, so nothing the bodies read is
// behind the prefetch in flight.
template <int S>
struct DwSlot {
  static constexpr int v = S;
};
template <typename T, int V, int LDQ, bool TWO, int R, bool PRE = true, typename Stage, typename Pre, typename Body>
__device__ __forceinline__ void dw_walk(float* ring, const T* __restrict__ src, const T* __restrict__ src2,
                                        const DwTile& t, const TileIdx& ti, int cc, int chunk, bool cok,
                                        Stage&& stage, Pre&& pre, Body&& body) {
  RowPipe<T, V, LDQ, TWO, R> rp;
  VRow p = {-1, -1, t.H};
  rp.template load<2>(src, src2, t, ti, p, cc);
  rp.store(ring, t, ti, p, 2, chunk, cok, stage);
  rp.template load<R>(src, src2, t, ti, vadv<2>(t, p), cc);
  const int nitems = ti.tw * t.chunks;  // <= 256 (dw_tile_plan)
  const bool item = cok && (int)threadIdx.x < nitems;
  const int px = min((int)threadIdx.x, nitems - 1) / t.chunks;
  const int nv = ti.nimg * (t.H + 1) - 1;  // virtual rows incl. the seams between images
  p = vnext(t, p);
  pre(p, px, DwSlot<0>());   // the first step's per-pixel loads
  // steps alternate between the two per-pixel buffers (unrolled in pairs: no register copy, so nothing
  // waits for the stores of a step before the next one starts)
  auto step = [&](auto slot) {
    constexpr int S = decltype(slot)::v;
    rp.store(ring, t, ti, vnext(t, p), R, chunk, cok, stage);
    __syncthreads();
    rp.template load<R>(src, src2, t, ti, vadv<R + 1>(t, p), cc);
    // the body's own per-pixel loads run one step ahead as well, issued right behind the prefetch: loads
    // retire in issue order, and loaded in the same step (the compiler sank them below the prefetch) the
    // first body waited for the whole prefetch (vmcnt(0)), exposing the next rows' latency every step
    pre(vadv<R>(t, p), px, DwSlot<1 - S>());
    if (item) {
      VRow q = p;
#pragma unroll
      for (int r = 0; r < R; ++r, q = vnext(t, q))
        if (q.u < nv && q.y < t.H) body(r, q.u, ti.b0 + q.im, q.y, px, DwSlot<S>());
    }
    __syncthreads();
    p = vadv<R>(t, p);
  };
  if constexpr (PRE) {
    while (p.u < nv) {
      step(DwSlot<0>());
      if (p.u >= nv) break;
      step(DwSlot<1>());
    }
  } else {   // no per-pixel loads: one buffer, no unrolled pair (fewer registers)
    while (p.u < nv) step(DwSlot<0>());
  }
}
// pre-load helper: V elements of src at this thread's pixel of virtual row u (clamped into the tensor)
template <typename T, int V>
__device__ __forceinline__ void dw_pixel_load(RawVec<T, V>& rv, const T* __restrict__ src, const DwTile& t,
                                              const TileIdx& ti, VRow q, int px, int cc) {
  const long b = ti.b0 + min(q.im, ti.nimg - 1);
  const int y = min(q.y, t.H - 1);
  rv.load(src + ((b * t.H + y) * t.W + ti.x0 + px) * t.C + cc);
}

// d = dw3x3(act(e*sc1 + sh1)) (+ fp64 stats of the rounded output minus shift)
template <typename T, int V, int LDQ, int ACT, int R>
__global__ __launch_bounds__(256) void dw_fwd_tile_kernel(const T* __restrict__ e, const float* __restrict__ wdw,
                                                          const float* __restrict__ sc, const float* __restrict__ sh,
                                                          int act, T* __restrict__ out, double* __restrict__ stat,
                                                          const float* __restrict__ shift, DwTile t) {
  extern __shared__ __attribute__((aligned(16))) float ring[];
  TileIdx ti;
  if (!tile_idx(t, ti)) return;
  const int chunk = threadIdx.x % t.chunks;
  const int c = ti.ct * t.CT + chunk * V;
  const bool cok = c < t.C;
  float w[9][V], s[V], h[V], sft[V];
#pragma unroll
  for (int i = 0; i < V; ++i) {
#pragma unroll
    for (int k = 0; k < 9; ++k) w[k][i] = cok ? wdw[(c + i) * 9 + k] : 0.f;
    s[i] = cok ? sc[c + i] : 0.f;
    h[i] = cok ? sh[c + i] : 0.f;
    sft[i] = (cok && shift) ? bn_shift(shift[c + i]) : 0.f;
  }
  double q[2][V];  // BN batch statistics in fp64 (shifted sums: fp32 cancels visibly when the
                   // running-mean shift is far from the batch mean)
#pragma unroll
  for (int i = 0; i < V; ++i) { q[0][i] = 0.0; q[1][i] = 0.0; }
  const int cc = cok ? c : 0;
  auto stage = [&](float (&v)[V], const float (&)[V], int) {
#pragma unroll
    for (int k = 0; k < V; ++k) v[k] = act_fwd(ACT, fmaf(v[k], s[k], h[k]));
  };
  dw_walk<T, V, LDQ, false, R, false>(ring, e, e, t, ti, cc, chunk, cok, stage, [&](VRow, int, auto) {},
                           [&](int, int u, long b, int y, int px, auto) {
    float acc[V];
#pragma unroll
    for (int i = 0; i < V; ++i) acc[i] = 0.f;
#pragma unroll
    for (int ki = 0; ki < 3; ++ki)
#pragma unroll
      for (int kj = 0; kj < 3; ++kj) {
        const float* src = ring_px<R>(ring, t, u - 1 + ki, px + kj) + chunk * V;
#pragma unroll
        for (int i = 0; i < V; i += 4) {
          const float4 a = *reinterpret_cast<const float4*>(src + i);
          acc[i] = fmaf(w[ki * 3 + kj][i], a.x, acc[i]);
          acc[i + 1] = fmaf(w[ki * 3 + kj][i + 1], a.y, acc[i + 1]);
          acc[i + 2] = fmaf(w[ki * 3 + kj][i + 2], a.z, acc[i + 2]);
          acc[i + 3] = fmaf(w[ki * 3 + kj][i + 3], a.w, acc[i + 3]);
        }
      }
    float of[V];
#pragma unroll
    for (int i = 0; i < V; ++i) {
      of[i] = to_f(from_f<T>(acc[i]));
      const double dl = (double)of[i] - (double)sft[i];
      q[0][i] += dl;
      q[1][i] = fma(dl, dl, q[1][i]);
    }
    store_vec<T, V>(out + ((b * t.H + y) * t.W + ti.x0 + px) * t.C + c, of);
  });
  if (stat) dw_reduce_store<2, V, double>(q, ring, t.chunks, stat + ti.rid * 2 * t.C, t.C, t.C, ti.ct * t.CT);
}

// dy1 = (dw3x3^T dd) * act'(e*sc1 + sh1) -> out; stats: sum dy1, sum dy1*(e - mean1)*invstd1.
// WG: the weight gradient in the same pass -- dW[tap] = sum_p dd[p] a[p + tap] = sum_q a[q] dd[q - tap]
// with a = act(e*sc1 + sh1): the transposed conv already reads dd[q - tap] for every tap of output
// pixel q and loads e[q], so the 9 partial sums cost 9 FMAs per element and no second pass over dd
// and e (part[rid][tap][c], as dw_wgrad_tile_kernel writes them)
// BN2: dd is not materialised -- the ring stages dd = BN2-backward(dA3, d) (bn2_apply_kernel's
// arithmetic, rounded to T as the stored dd would be) from the two [M, C] sources, the per-image
// SE gate and dpool/HW of the block's images staged once in LDS behind the ring.
template <typename T>
struct Bn2In {
  const T* d;
  const float *sc, *sh, *mean, *inv, *gate, *dpool, *coef;
  int HW;
};
template <typename T, int V, int LDQ, int ACT, bool WG = false, bool BN2 = false, int R = DW_R>
__global__ __launch_bounds__(256) void dw_dgrad_tile_kernel(const T* __restrict__ dd, const float* __restrict__ wdw,
                                                            const T* __restrict__ e, const float* __restrict__ sc,
                                                            const float* __restrict__ sh,
                                                            const float* __restrict__ mean,
                                                            const float* __restrict__ invstd, int act,
                                                            T* __restrict__ out, float* __restrict__ stat, DwTile t,
                                                            float* __restrict__ part, Bn2In<T> b2, int tab_off) {
  extern __shared__ __attribute__((aligned(16))) float ring[];
  TileIdx ti;
  if (!tile_idx(t, ti)) return;
  const int chunk = threadIdx.x % t.chunks;
  const int c = ti.ct * t.CT + chunk * V;
  const bool cok = c < t.C;
  float w[9][V], s[V], h[V], mu[V], is[V];
#pragma unroll
  for (int i = 0; i < V; ++i) {
#pragma unroll
    for (int k = 0; k < 9; ++k) w[k][i] = cok ? wdw[(c + i) * 9 + k] : 0.f;
    s[i] = cok ? sc[c + i] : 0.f;
    h[i] = cok ? sh[c + i] : 0.f;
    mu[i] = cok ? mean[c + i] : 0.f;
    is[i] = cok ? invstd[c + i] : 0.f;
  }
  float s2[BN2 ? V : 1], h2[BN2 ? V : 1], mu2[BN2 ? V : 1], is2[BN2 ? V : 1], ca[BN2 ? V : 1], cb[BN2 ? V : 1],
      cc2[BN2 ? V : 1];
  float* tab = ring + tab_off;  // [G][2][CT]: gate, dpool/HW of the block's images
  if constexpr (BN2) {
#pragma unroll
    for (int i = 0; i < V; ++i) {
      s2[i] = cok ? b2.sc[c + i] : 0.f;
      h2[i] = cok ? b2.sh[c + i] : 0.f;
      mu2[i] = cok ? b2.mean[c + i] : 0.f;
      is2[i] = cok ? b2.inv[c + i] : 0.f;
      ca[i] = cok ? b2.coef[c + i] : 0.f;
      cb[i] = cok ? b2.coef[t.C + c + i] : 0.f;
      cc2[i] = cok ? b2.coef[2 * t.C + c + i] : 0.f;
    }
    const float ihw = 1.f / (float)b2.HW;
    for (int idx = threadIdx.x; idx < t.G * t.CT; idx += 256) {
      const int im = idx / t.CT, cl = idx - im * t.CT, ch = ti.ct * t.CT + cl;
      const bool ok = im < ti.nimg && ch < t.C;
      const long gi = ok ? (ti.b0 + im) * t.C + ch : 0;
      const float g = b2.gate[gi], dp = b2.dpool[gi];
      tab[im * 2 * t.CT + cl] = ok ? g : 0.f;
      tab[(im * 2 + 1) * t.CT + cl] = ok ? dp * ihw : 0.f;
    }
    __syncthreads();
  }
  float q[2][V];
#pragma unroll
  for (int i = 0; i < V; ++i) { q[0][i] = 0.f; q[1][i] = 0.f; }
  float q9[WG ? 9 : 1][V];
#pragma unroll
  for (int k = 0; k < (WG ? 9 : 1); ++k)
#pragma unroll
    for (int i = 0; i < V; ++i) q9[k][i] = 0.f;
  const int cc = cok ? c : 0;
  RawVec<T, V> ce[2][R];  // e at this thread's output pixel of a step's rows (two steps in flight)
  auto pre = [&](VRow q, int px, auto slot) {
#pragma unroll
    for (int r = 0; r < R; ++r, q = vnext(t, q)) dw_pixel_load(ce[decltype(slot)::v][r], e, t, ti, q, px, cc);
  };
  auto stage = [&](float (&v)[V], const float (&dv)[V], int im) {
    if constexpr (BN2) {
      const float* gp = tab + im * 2 * t.CT + chunk * V;
      float gt[V], dpi[V];
#pragma unroll
      for (int k = 0; k < V; k += 4) {
        const float4 g4 = *reinterpret_cast<const float4*>(gp + k);
        const float4 p4 = *reinterpret_cast<const float4*>(gp + t.CT + k);
        gt[k] = g4.x; gt[k + 1] = g4.y; gt[k + 2] = g4.z; gt[k + 3] = g4.w;
        dpi[k] = p4.x; dpi[k + 1] = p4.y; dpi[k + 2] = p4.z; dpi[k + 3] = p4.w;
      }
#pragma unroll
      for (int k = 0; k < V; ++k) {
        const float y = fmaf(dv[k], s2[k], h2[k]);
        const float dy2 = fmaf(v[k], gt[k], dpi[k]) * act_grad(ACT, y);
        const float dh = (dv[k] - mu2[k]) * is2[k];
        v[k] = to_f(from_f<T>(ca[k] * (dy2 - cb[k] - dh * cc2[k])));
      }
    }
  };
  dw_walk<T, V, LDQ, BN2, R>(ring, dd, b2.d, t, ti, cc, chunk, cok, stage, pre, [&](int r, int u, long b, int y, int px,
                                                                                   auto slot) {
    const long off = ((b * t.H + y) * t.W + ti.x0 + px) * t.C + c;
    float ev[V];
    ce[decltype(slot)::v][r].unpack(ev);
    // act(BN1(e)) for the weight gradient and act'(BN1(e)) for the output from one transcendental pair
    float acc[V], av[V], ag[V];
#pragma unroll
    for (int i = 0; i < V; ++i) {
      acc[i] = 0.f;
      if constexpr (WG) act_both(ACT, fmaf(ev[i], s[i], h[i]), av[i], ag[i]);
      else ag[i] = act_grad(ACT, fmaf(ev[i], s[i], h[i]));
    }
#pragma unroll
    for (int ki = 0; ki < 3; ++ki)
#pragma unroll
      for (int kj = 0; kj < 3; ++kj) {
        // transposed conv: dd row y+1-ki, column x+1-kj  (ring pixel px + 2 - kj)
        const float* src = ring_px<R>(ring, t, u + 1 - ki, px + 2 - kj) + chunk * V;
#pragma unroll
        for (int i = 0; i < V; i += 4) {
          const float4 a = *reinterpret_cast<const float4*>(src + i);
          acc[i] = fmaf(w[ki * 3 + kj][i], a.x, acc[i]);
          acc[i + 1] = fmaf(w[ki * 3 + kj][i + 1], a.y, acc[i + 1]);
          acc[i + 2] = fmaf(w[ki * 3 + kj][i + 2], a.z, acc[i + 2]);
          acc[i + 3] = fmaf(w[ki * 3 + kj][i + 3], a.w, acc[i + 3]);
          if constexpr (WG) {
            q9[ki * 3 + kj][i] = fmaf(av[i], a.x, q9[ki * 3 + kj][i]);
            q9[ki * 3 + kj][i + 1] = fmaf(av[i + 1], a.y, q9[ki * 3 + kj][i + 1]);
            q9[ki * 3 + kj][i + 2] = fmaf(av[i + 2], a.z, q9[ki * 3 + kj][i + 2]);
            q9[ki * 3 + kj][i + 3] = fmaf(av[i + 3], a.w, q9[ki * 3 + kj][i + 3]);
          }
        }
      }
    float o2[V];
#pragma unroll
    for (int i = 0; i < V; ++i) {
      o2[i] = to_f(from_f<T>(acc[i] * ag[i]));
      q[0][i] += o2[i];
      q[1][i] = fmaf(o2[i], (ev[i] - mu[i]) * is[i], q[1][i]);
    }
    store_vec<T, V>(out + off, o2);
  });
  dw_reduce_store<2, V, float>(q, ring, t.chunks, stat + ti.rid * 2 * t.C, t.C, t.C, ti.ct * t.CT);
  if constexpr (WG) dw_reduce_store<9, V, float>(q9, ring, t.chunks, part + ti.rid * 9 * t.C, t.C, t.C, ti.ct * t.CT);
}

// dWdw partials: part[rid][tap][c] = sum over the block's pixels dd[p,c] * act(e*sc1+sh1)[p+tap, c]
template <typename T, int V, int LDQ, int ACT>
__global__ __launch_bounds__(256) void dw_wgrad_tile_kernel(const T* __restrict__ dd, const T* __restrict__ e,
                                                            const float* __restrict__ sc, const float* __restrict__ sh,
                                                            int act, float* __restrict__ part, DwTile t) {
  extern __shared__ __attribute__((aligned(16))) float ring[];
  TileIdx ti;
  if (!tile_idx(t, ti)) return;
  const int chunk = threadIdx.x % t.chunks;
  const int c = ti.ct * t.CT + chunk * V;
  const bool cok = c < t.C;
  float s[V], h[V];
#pragma unroll
  for (int i = 0; i < V; ++i) {
    s[i] = cok ? sc[c + i] : 0.f;
    h[i] = cok ? sh[c + i] : 0.f;
  }
  float q[9][V];
#pragma unroll
  for (int k = 0; k < 9; ++k)
#pragma unroll
    for (int i = 0; i < V; ++i) q[k][i] = 0.f;
  const int cc = cok ? c : 0;
  RawVec<T, V> cg[2][DW_R];  // dd at this thread's output pixel of a step's rows (two steps in flight)
  auto pre = [&](VRow q, int px, auto slot) {
#pragma unroll
    for (int r = 0; r < DW_R; ++r, q = vnext(t, q)) dw_pixel_load(cg[decltype(slot)::v][r], dd, t, ti, q, px, cc);
  };
  auto stage = [&](float (&v)[V], const float (&)[V], int) {
#pragma unroll
    for (int k = 0; k < V; ++k) v[k] = act_fwd(ACT, fmaf(v[k], s[k], h[k]));
  };
  dw_walk<T, V, LDQ, false, DW_R>(ring, e, e, t, ti, cc, chunk, cok, stage, pre, [&](int r, int u, long, int, int px,
                                                                                   auto slot) {
    float g[V];
    cg[decltype(slot)::v][r].unpack(g);
#pragma unroll
    for (int ki = 0; ki < 3; ++ki)
#pragma unroll
      for (int kj = 0; kj < 3; ++kj) {
        const float* src = ring_px(ring, t, u - 1 + ki, px + kj) + chunk * V;
#pragma unroll
        for (int i = 0; i < V; i += 4) {
          const float4 a = *reinterpret_cast<const float4*>(src + i);
          q[ki * 3 + kj][i] = fmaf(g[i], a.x, q[ki * 3 + kj][i]);
          q[ki * 3 + kj][i + 1] = fmaf(g[i + 1], a.y, q[ki * 3 + kj][i + 1]);
          q[ki * 3 + kj][i + 2] = fmaf(g[i + 2], a.z, q[ki * 3 + kj][i + 2]);
          q[ki * 3 + kj][i + 3] = fmaf(g[i + 3], a.w, q[ki * 3 + kj][i + 3]);
        }
      }
  });
  dw_reduce_store<9, V, float>(q, ring, t.chunks, part + ti.rid * 9 * t.C, t.C, t.C, ti.ct * t.CT);
}

// dw[c*9 + tap] = s[tap*C + c]
__global__ void tapmajor_to_chan_kernel(const float* __restrict__ s, float* __restrict__ dw, int C) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= 9 * C) return;
  const int c = i / 9, tap = i - c * 9;
  dw[i] = s[tap * C + c];
}

// ------------------------------------------------------------------ Squeeze-Excite
// Per-image channel reductions over [B, HW, K] rows: block = (image b, group of chunks*V channels),
// thread = (chunk = tid % chunks, pixel slot = tid / chunks) striding over the image's pixels.
// chunks is picked per shape so every thread takes >= ~4 pixels (small images: wide channel groups
// instead of idle slots), then the slots are summed in a fixed order (dw_reduce_store).
struct ImgPlan {
  int chunks, ngx;
};
static ImgPlan img_plan(int HW, int K, int V) {
  int slots = 8;
  while (slots < 64 && slots * 2 * 4 <= HW) slots *= 2;  // >= 4 pixels per slot
  int ch = 256 / slots;
  while (ch > 1 && (ch / 2) * V >= K) ch /= 2;
  ImgPlan p;
  p.chunks = ch;
  p.ngx = (K + ch * V - 1) / (ch * V);
  return p;
}
constexpr int IMG_MAX_CHUNKS = 32;  // img_plan: >= 8 slots

// pooled[b, c] = mean over the image's pixels of act(d*sc + sh)
template <typename T, int V, int ACT>
__global__ __launch_bounds__(256) void se_pool_kernel(const T* __restrict__ d, const float* __restrict__ sc,
                                                      const float* __restrict__ sh, float* __restrict__ pooled,
                                                      int HW, int K, int B, int chunks, int ngx) {
  __shared__ __attribute__((aligned(16))) float lds[4 * IMG_MAX_CHUNKS * 1 * V];  // dw_reduce_store scratch
  long lid;
  if (!xcd_block((long)ngx * B, lid)) return;
  const int bx = (int)(lid % ngx);
  const long b = lid / ngx;
  const int chunk = threadIdx.x % chunks, slot = threadIdx.x / chunks, nslots = 256 / chunks;
  const int c0 = (bx * chunks + chunk) * V;
  float q[1][V];
#pragma unroll
  for (int i = 0; i < V; ++i) q[0][i] = 0.f;
  if (c0 < K) {
    float s[V], h[V];
    load_vec<float, V>(sc + c0, s);
    load_vec<float, V>(sh + c0, h);
#pragma unroll 2
    for (int p = slot; p < HW; p += nslots) {
      float v[V];
      load_vec<T, V>(d + (b * HW + p) * K + c0, v);
#pragma unroll
      for (int i = 0; i < V; ++i) q[0][i] += act_fwd(ACT, fmaf(v[i], s[i], h[i]));
    }
    const float inv = 1.f / (float)HW;
#pragma unroll
    for (int i = 0; i < V; ++i) q[0][i] *= inv;
  }
  dw_reduce_store<1, V, float>(q, lds, chunks, pooled + b * K, K, K, bx * chunks * V);
}

__global__ void sigmoid_kernel(const float* __restrict__ z, float* __restrict__ g, long n) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) g[i] = fast_sigmoid(z[i]);
}

// dz2 = dgate * g * (1 - g)
__global__ void sigmoid_bwd_kernel(const float* __restrict__ dgate, const float* __restrict__ g, float* __restrict__ dz,
                                   long n) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) dz[i] = dgate[i] * g[i] * (1.f - g[i]);
}

// pooled[b, c] = mean over the image's pixels of act(d*sc + sh)   large images: 4 chunks x 64 pixel slots
template <typename T, int V>
__global__ __launch_bounds__(256) void se_pool_wide_kernel(const T* __restrict__ d, const float* __restrict__ sc,
                                                      const float* __restrict__ sh, int act, float* __restrict__ pooled,
                                                      int HW, int K, int B) {
  __shared__ float lds[4 * 1 * 4 * 8];
  const int gx = (K + 4 * V - 1) / (4 * V);
  long lid;
  if (!xcd_block((long)gx * B, lid)) return;
  const int bx = (int)(lid % gx);
  const int chunk = threadIdx.x & 3, slot = threadIdx.x >> 2;
  const int c0 = (bx * 4 + chunk) * V;
  const long b = lid / gx;
  float q[1][V];
#pragma unroll
  for (int i = 0; i < V; ++i) q[0][i] = 0.f;
  if (c0 < K) {
    float s[V], h[V];
    load_vec<float, V>(sc + c0, s);
    load_vec<float, V>(sh + c0, h);
    for (int p = slot; p < HW; p += 64) {
      float v[V];
      load_vec<T, V>(d + (b * HW + p) * K + c0, v);
#pragma unroll
      for (int i = 0; i < V; ++i) q[0][i] += act_fwd(act, fmaf(v[i], s[i], h[i]));
    }
    const float inv = 1.f / (float)HW;
#pragma unroll
    for (int i = 0; i < V; ++i) q[0][i] *= inv;
  }
  chunk_reduce_store<1, V>(q, lds, pooled + b * K, K, K, bx * 4 * V);
}

template <typename T, int V>
__global__ __launch_bounds__(256) void se_bwd_reduce_wide_kernel(const T* __restrict__ dA3, const T* __restrict__ d,
                                                            const float* __restrict__ sc, const float* __restrict__ sh,
                                                            const float* __restrict__ mean,
                                                            const float* __restrict__ invstd, int act,
                                                            float* __restrict__ R, int B, int HW, int K,
                                                            const float* __restrict__ gate, float* __restrict__ dz2) {
  __shared__ float lds[4 * 5 * 4 * 8];
  const int gx = (K + 4 * V - 1) / (4 * V);
  long lid;
  if (!xcd_block((long)gx * B, lid)) return;
  const int bx = (int)(lid % gx);
  const int chunk = threadIdx.x & 3, slot = threadIdx.x >> 2;
  const int c0 = (bx * 4 + chunk) * V;
  const long b = lid / gx;
  float q[5][V];
#pragma unroll
  for (int k = 0; k < 5; ++k)
#pragma unroll
    for (int i = 0; i < V; ++i) q[k][i] = 0.f;
  if (c0 < K) {
    float s[V], h[V], mu[V], is[V];
    load_vec<float, V>(sc + c0, s);
    load_vec<float, V>(sh + c0, h);
    load_vec<float, V>(mean + c0, mu);
    load_vec<float, V>(invstd + c0, is);
    for (int p = slot; p < HW; p += 64) {
      float ga[V], dv[V];
      load_vec<T, V>(dA3 + (b * HW + p) * K + c0, ga);
      load_vec<T, V>(d + (b * HW + p) * K + c0, dv);
#pragma unroll
      for (int i = 0; i < V; ++i) {
        const float y = fmaf(dv[i], s[i], h[i]);
        const float sg = fast_sigmoid(y);
        float a, sp;
        if (act == OGV_ACT_SILU) {
          a = y * sg;
          sp = sg * (1.0f + y * (1.0f - sg));
        } else {
          a = act_fwd(act, y);
          sp = act_grad(act, y);
        }
        const float dh = (dv[i] - mu[i]) * is[i];
        q[0][i] = fmaf(ga[i], a, q[0][i]);
        q[1][i] = fmaf(ga[i], sp, q[1][i]);
        q[2][i] += sp;
        q[3][i] = fmaf(ga[i] * sp, dh, q[3][i]);
        q[4][i] = fmaf(sp, dh, q[4][i]);
      }
    }
  }
  chunk_reduce_store<5, V>(q, lds, R + b * K, (long)B * K, K, bx * 4 * V, gate + b * K, dz2 + b * K);
}

// One pass over (dA3, d) per image: R[q][b][c] for
//   q0 = sum dA3*a2 (-> dgate), q1 = sum dA3*s', q2 = sum s', q3 = sum dA3*s'*dh, q4 = sum s'*dh
// with y2 = d*sc2+sh2, a2 = act(y2), s' = act'(y2), dh = (d-mean2)*invstd2.
template <typename T, int V, int ACT>
__global__ __launch_bounds__(256) void se_bwd_reduce_kernel(const T* __restrict__ dA3, const T* __restrict__ d,
                                                            const float* __restrict__ sc, const float* __restrict__ sh,
                                                            const float* __restrict__ mean,
                                                            const float* __restrict__ invstd, float* __restrict__ R,
                                                            int B, int HW, int K, int chunks, int ngx,
                                                            const float* __restrict__ gate, float* __restrict__ dz2) {
  __shared__ __attribute__((aligned(16))) float lds[4 * IMG_MAX_CHUNKS * 5 * V];  // dw_reduce_store scratch
  long lid;
  if (!xcd_block((long)ngx * B, lid)) return;
  const int bx = (int)(lid % ngx);
  const long b = lid / ngx;
  const int chunk = threadIdx.x % chunks, slot = threadIdx.x / chunks, nslots = 256 / chunks;
  const int c0 = (bx * chunks + chunk) * V;
  float q[5][V];
#pragma unroll
  for (int k = 0; k < 5; ++k)
#pragma unroll
    for (int i = 0; i < V; ++i) q[k][i] = 0.f;
  if (c0 < K) {
    float s[V], h[V], mu[V], is[V];
    load_vec<float, V>(sc + c0, s);
    load_vec<float, V>(sh + c0, h);
    load_vec<float, V>(mean + c0, mu);
    load_vec<float, V>(invstd + c0, is);
#pragma unroll 2
    for (int p = slot; p < HW; p += nslots) {
      float ga[V], dv[V];
      load_vec<T, V>(dA3 + (b * HW + p) * K + c0, ga);
      load_vec<T, V>(d + (b * HW + p) * K + c0, dv);
#pragma unroll
      for (int i = 0; i < V; ++i) {
        const float y = fmaf(dv[i], s[i], h[i]);
        float a, sp;
        if constexpr (ACT == OGV_ACT_SILU) {
          const float sg = fast_sigmoid(y);
          a = y * sg;
          sp = sg * (1.0f + y * (1.0f - sg));
        } else {
          a = act_fwd(ACT, y);
          sp = act_grad(ACT, y);
        }
        const float dh = (dv[i] - mu[i]) * is[i];
        q[0][i] = fmaf(ga[i], a, q[0][i]);
        q[1][i] = fmaf(ga[i], sp, q[1][i]);
        q[2][i] += sp;
        q[3][i] = fmaf(ga[i] * sp, dh, q[3][i]);
        q[4][i] = fmaf(sp, dh, q[4][i]);
      }
    }
  }
  dw_reduce_store<5, V, float>(q, lds, chunks, R + b * K, (long)B * K, K, bx * chunks * V, gate + b * K, dz2 + b * K);
}

// ---- row-tiled elementwise kernels: thread = (channel chunk, row slot), EW_RPT rows per thread, so
// the per-channel coefficients are loaded once per EW_RPT rows; rows are clamped (loads of all
// EW_RPT rows are issued up front), stores guarded.
constexpr int EW_RPT = 4;
struct EwPlan {
  int nch, CG, RB, ncg;
  long nrb;
  unsigned grid() const { return xcd_grid((long)ncg * nrb); }
};
static EwPlan ew_plan(long M, int K, int V) {
  EwPlan p;
  p.nch = K / V;
  p.CG = p.nch < 64 ? p.nch : 64;
  p.RB = 256 / p.CG;
  p.ncg = (p.nch + p.CG - 1) / p.CG;
  p.nrb = (M + (long)p.RB * EW_RPT - 1) / ((long)p.RB * EW_RPT);
  return p;
}
__device__ __forceinline__ bool ew_idx(const EwPlan& p, int V, int& c0, long& m0) {
  long id;
  if (!xcd_block((long)p.ncg * p.nrb, id)) return false;
  const int cg = (int)(id % p.ncg);
  const long rb = id / p.ncg;
  const int cc = threadIdx.x % p.CG, rr = threadIdx.x / p.CG;
  const int ch = cg * p.CG + cc;
  if (rr >= p.RB || ch >= p.nch) return false;
  c0 = ch * V;
  m0 = rb * p.RB * EW_RPT + rr;
  return true;
}

// A3 = act(d*sc2 + sh2) * gate, rounded to T once: the project GEMM's input with exactly the arithmetic
// of the GEMM kernels' A prologue (knob mb_a3), so the GEMM and its weight gradient run prologue-free
template <typename T, int V, int ACT>
__global__ __launch_bounds__(256) void a3_kernel(const T* __restrict__ d, const float* __restrict__ sc,
                                                 const float* __restrict__ sh, const float* __restrict__ gate,
                                                 T* __restrict__ out, long M, int HW, int K, EwPlan ep) {
  int c0;
  long m0;
  if (!ew_idx(ep, V, c0, m0)) return;
  float s[V], h[V];
  load_vec<float, V>(sc + c0, s);
  load_vec<float, V>(sh + c0, h);
  float dv[EW_RPT][V];
#pragma unroll
  for (int j = 0; j < EW_RPT; ++j) {
    const long m = min(m0 + (long)j * ep.RB, M - 1);
    load_vec<T, V>(d + m * K + c0, dv[j]);
  }
#pragma unroll
  for (int j = 0; j < EW_RPT; ++j) {
    const long m = m0 + (long)j * ep.RB;
    if (m >= M) break;
    float gt[V], o[V];
    load_vec<float, V>(gate + (m / HW) * K + c0, gt);
#pragma unroll
    for (int i = 0; i < V; ++i) {
      o[i] = act_fwd(ACT, fmaf(dv[j][i], s[i], h[i]));
      o[i] *= gt[i];
    }
    store_vec<T, V>(out + m * K + c0, o);
  }
}

// dd = ca*(dy2 - cb - dh*cc), dy2 = (dA3*gate + dpool/HW) * act'(d*sc2+sh2)
template <typename T, int V, int ACT>
__global__ __launch_bounds__(256) void bn2_apply_kernel(const T* __restrict__ dA3, const T* __restrict__ d,
                                                        const float* __restrict__ sc, const float* __restrict__ sh,
                                                        const float* __restrict__ mean, const float* __restrict__ invstd,
                                                        const float* __restrict__ gate, const float* __restrict__ dpool,
                                                        const float* __restrict__ coef, T* __restrict__ out,
                                                        long M, int HW, int K, EwPlan ep) {
  int c0;
  long m0;
  if (!ew_idx(ep, V, c0, m0)) return;
  float s[V], h[V], mu[V], is[V], ca[V], cb[V], cc[V];
  load_vec<float, V>(sc + c0, s);
  load_vec<float, V>(sh + c0, h);
  load_vec<float, V>(mean + c0, mu);
  load_vec<float, V>(invstd + c0, is);
  load_vec<float, V>(coef + c0, ca);
  load_vec<float, V>(coef + K + c0, cb);
  load_vec<float, V>(coef + 2 * K + c0, cc);
  const float inv = 1.f / (float)HW;
  float ga[EW_RPT][V], dv[EW_RPT][V];
#pragma unroll
  for (int j = 0; j < EW_RPT; ++j) {
    const long m = min(m0 + (long)j * ep.RB, M - 1);
    load_vec<T, V>(dA3 + m * K + c0, ga[j]);
    load_vec<T, V>(d + m * K + c0, dv[j]);
  }
#pragma unroll
  for (int j = 0; j < EW_RPT; ++j) {
    const long m = m0 + (long)j * ep.RB;
    if (m >= M) break;
    const long b = m / HW;
    float gt[V], dp[V], o[V];
    load_vec<float, V>(gate + b * K + c0, gt);
    load_vec<float, V>(dpool + b * K + c0, dp);
#pragma unroll
    for (int i = 0; i < V; ++i) {
      const float y = fmaf(dv[j][i], s[i], h[i]);
      const float dy2 = fmaf(ga[j][i], gt[i], dp[i] * inv) * act_grad(ACT, y);
      const float dh = (dv[j][i] - mu[i]) * is[i];
      o[i] = ca[i] * (dy2 - cb[i] - dh * cc[i]);
    }
    store_vec<T, V>(out + m * K + c0, o);
  }
}

// generic BN backward reduction over rows: stat[slice] = [sum dy, sum dy*(x-mean)*invstd]
template <typename T, int V>
__global__ __launch_bounds__(256) void bn_bwd_reduce_kernel(const T* __restrict__ dy, const T* __restrict__ x,
                                                            const float* __restrict__ mean,
                                                            const float* __restrict__ invstd, float* __restrict__ stat,
                                                            long M, int K, long rows_per_slice) {
  __shared__ float lds[4 * 2 * 4 * 8];
  const int gx = (K + 4 * V - 1) / (4 * V);
  long lid;
  if (!xcd_block((long)gx * ((M + rows_per_slice - 1) / rows_per_slice), lid)) return;
  const int bx = (int)(lid % gx);
  const long by = lid / gx;
  const int chunk = threadIdx.x & 3, slot = threadIdx.x >> 2;
  const int c0 = (bx * 4 + chunk) * V;
  const long r0 = by * rows_per_slice;
  const long r1 = r0 + rows_per_slice < M ? r0 + rows_per_slice : M;
  float q[2][V];
#pragma unroll
  for (int i = 0; i < V; ++i) { q[0][i] = 0.f; q[1][i] = 0.f; }
  if (c0 < K) {
    float mu[V], is[V];
    load_vec<float, V>(mean + c0, mu);
    load_vec<float, V>(invstd + c0, is);
    for (long r = r0 + slot; r < r1; r += 64) {
      float g[V], xv[V];
      load_vec<T, V>(dy + r * K + c0, g);
      load_vec<T, V>(x + r * K + c0, xv);
#pragma unroll
      for (int i = 0; i < V; ++i) {
        q[0][i] += g[i];
        q[1][i] = fmaf(g[i], (xv[i] - mu[i]) * is[i], q[1][i]);
      }
    }
  }
  chunk_reduce_store<2, V>(q, lds, stat + by * 2 * K, K, K, bx * 4 * V);
}

// out = ca*(dy - cb - (x-mean)*invstd*cc)
template <typename T, int V>
__global__ __launch_bounds__(256) void bn_bwd_apply_kernel(const T* __restrict__ dy, const T* __restrict__ x,
                                                           const float* __restrict__ mean,
                                                           const float* __restrict__ invstd,
                                                           const float* __restrict__ coef, T* __restrict__ out, long M,
                                                           int K, EwPlan ep) {
  int c0;
  long m0;
  if (!ew_idx(ep, V, c0, m0)) return;
  float mu[V], is[V], ca[V], cb[V], cc[V];
  load_vec<float, V>(mean + c0, mu);
  load_vec<float, V>(invstd + c0, is);
  load_vec<float, V>(coef + c0, ca);
  load_vec<float, V>(coef + K + c0, cb);
  load_vec<float, V>(coef + 2 * K + c0, cc);
  float g[EW_RPT][V], xv[EW_RPT][V];
#pragma unroll
  for (int j = 0; j < EW_RPT; ++j) {
    const long m = min(m0 + (long)j * ep.RB, M - 1);
    load_vec<T, V>(dy + m * K + c0, g[j]);
    load_vec<T, V>(x + m * K + c0, xv[j]);
  }
#pragma unroll
  for (int j = 0; j < EW_RPT; ++j) {
    const long m = m0 + (long)j * ep.RB;
    if (m >= M) break;
    float o[V];
#pragma unroll
    for (int i = 0; i < V; ++i) o[i] = ca[i] * (g[j][i] - cb[i] - (xv[j][i] - mu[i]) * is[i] * cc[i]);
    store_vec<T, V>(out + m * K + c0, o);
  }
}

// out = res + p*sc + sh
template <typename T, int V>
__global__ __launch_bounds__(256) void affine_residual_kernel(const T* __restrict__ res, const T* __restrict__ p,
                                                              const float* __restrict__ sc,
                                                              const float* __restrict__ sh, T* __restrict__ out, long M,
                                                              int K, EwPlan ep) {
  int c0;
  long m0;
  if (!ew_idx(ep, V, c0, m0)) return;
  float s[V], h[V];
  load_vec<float, V>(sc + c0, s);
  load_vec<float, V>(sh + c0, h);
  float a[EW_RPT][V], pv[EW_RPT][V];
#pragma unroll
  for (int j = 0; j < EW_RPT; ++j) {
    const long m = min(m0 + (long)j * ep.RB, M - 1);
    load_vec<T, V>(res + m * K + c0, a[j]);
    load_vec<T, V>(p + m * K + c0, pv[j]);
  }
#pragma unroll
  for (int j = 0; j < EW_RPT; ++j) {
    const long m = m0 + (long)j * ep.RB;
    if (m >= M) break;
#pragma unroll
    for (int i = 0; i < V; ++i) a[j][i] += fmaf(pv[j][i], s[i], h[i]);
    store_vec<T, V>(out + m * K + c0, a[j]);
  }
}

// ------------------------------------------------------------------ orchestration
struct Buf {
  char* base;
  size_t off = 0;
  explicit Buf(void* b) : base((char*)b) {}
  template <typename P>
  P* take(size_t n) {
    off = (off + 255) & ~(size_t)255;
    P* r = reinterpret_cast<P*>(base ? base + off : nullptr);
    off += n * sizeof(P);
    return r;
  }
};

// Saved-for-backward layout (lives in the caller's `saved` buffer).
// knob "mb_a3": once the SE gate is known, one elementwise pass writes the project GEMM's input
// A3 = act(BN2(d)) * gate (the GEMM prologue's arithmetic), and the project GEMM runs without an A prologue
// (recomputed per element -- and per column tile -- the SiLU's exp / rcp made it 0.42-0.47 ms of the 7M step,
// profiles/r05x_mb_a3_rejected.txt).  Modes: 0: the prologue form everywhere; 1: A3 lives in the forward
// workspace (no extra memory: the backward's workspace is larger), the weight gradient keeps its prologue;
// 2: A3 is saved for the backward too (+1 [M, 4C] activation per MBConv -- Model-A-22M at 224^2, bs 128 then
// no longer fits 288 GB), the weight gradient prologue-free as well; 3 (the knob's default): 2 for an MBConv
// whose A3 takes at most 512 MB, else 1 (7M, 30 steps: 0 -> 14.76-14.79 ms, 1 -> 14.69-14.70,
// 2 -> 14.60-14.63; 22M 339.5 -> 338.9 ms with 1; profiles/r05ac_mb_a3.log).
// The mode is part of the saved data's contract: desc.a3 pins it (ogv_mbconv_a3_mode resolves the knob once,
// the caller keeps the desc for the backward), and the optional A3 slab sits AFTER every fixed field, so a
// knob change between a forward and its backward can neither shift the statistics nor read past the buffer.
static int g_mb_a3 = 3;
void set_mb_a3(int v) { g_mb_a3 = v < 0 ? 0 : (v > 3 ? 3 : v); }
static int a3_resolve(const ogv_mbconv_desc& s, size_t esz) {
  if (g_mb_a3 != 3) return g_mb_a3;
  return (size_t)s.B * s.H * s.W * s.mid * esz <= (512u << 20) ? 2 : 1;
}
static int a3_mode(const ogv_mbconv_desc& s, size_t esz) { return s.a3 >= 0 ? s.a3 : a3_resolve(s, esz); }
struct Saved {
  void *e, *d, *p;                             // [M,mid], [M,mid], [M,C] activation dtype
  void* a3;                                    // [M,mid] act(BN2(d)) * gate (A3 mode 2 only; stored last)
  float *mean1, *inv1, *sc1, *sh1;             // [mid]
  float *mean2, *inv2, *sc2, *sh2;             // [mid]
  float *mean3, *inv3, *sc3, *sh3;             // [C]
  float *pooled, *z1, *z2, *gate;              // [B,mid], [B,se], [B,mid], [B,mid]
};
static Saved saved_layout(void* base, const ogv_mbconv_desc& s, size_t esz, size_t* total) {
  Buf b(base);
  const long M = (long)s.B * s.H * s.W;
  Saved v;
  v.e = b.take<char>(M * s.mid * esz);
  v.d = b.take<char>(M * s.mid * esz);
  v.p = b.take<char>(M * s.C * esz);
  v.mean1 = b.take<float>(s.mid); v.inv1 = b.take<float>(s.mid); v.sc1 = b.take<float>(s.mid); v.sh1 = b.take<float>(s.mid);
  v.mean2 = b.take<float>(s.mid); v.inv2 = b.take<float>(s.mid); v.sc2 = b.take<float>(s.mid); v.sh2 = b.take<float>(s.mid);
  v.mean3 = b.take<float>(s.C); v.inv3 = b.take<float>(s.C); v.sc3 = b.take<float>(s.C); v.sh3 = b.take<float>(s.C);
  v.pooled = b.take<float>((size_t)s.B * s.mid);
  v.z1 = b.take<float>((size_t)s.B * s.se);
  v.z2 = b.take<float>((size_t)s.B * s.mid);
  v.gate = b.take<float>((size_t)s.B * s.mid);
  v.a3 = a3_mode(s, esz) == 2 ? b.take<char>(M * s.mid * esz) : nullptr;   // last: the fixed fields never move
  if (total) *total = b.off + 256;
  return v;
}

static long dw_slices(long P, const RowPlan& rp) {   // row slices for the global BN reductions
  const long ct = (rp.nch + 3) / 4;
  long S = (2048 + ct - 1) / ct;
  const long maxS = (P + 511) / 512;                    // >= 8 rows per slot
  if (S > maxS) S = maxS;
  return S < 1 ? 1 : S;
}

struct FwdWs {
  double *stat1, *stat2, *stat3, *sums, *tmp;  // fp64 BatchNorm batch statistics
  float* split;                                // SE split-K partials
  char* gemm;
  void* a3;                                    // mb_a3 = 1: [M,mid] A3 (within the backward's workspace size)
};
static FwdWs fwd_ws_layout(void* base, const ogv_mbconv_desc& s, size_t esz, size_t* total) {
  Buf b(base);
  const long M = (long)s.B * s.H * s.W;
  RowPlan rp = row_plan(s.mid);
  const long S2 = dw_tile_plan(s.B, s.H, s.W, s.mid, 4).rows_max();
  const long R1 = gemm_stat_rows((int)M);
  FwdWs w;
  w.stat1 = b.take<double>(R1 * 2 * s.mid);
  w.stat2 = b.take<double>(S2 * 2 * s.mid);
  w.stat3 = b.take<double>(R1 * 2 * s.C);
  w.sums = b.take<double>(2 * (size_t)(s.mid > s.C ? s.mid : s.C));
  long Rmax = R1 > S2 ? R1 : S2;
  w.tmp = b.take<double>(colreduce_tmp_floats(Rmax, 2L * (s.mid > s.C ? s.mid : s.C)) + 16);
  w.split = b.take<float>(std::max(splitk_ws_bytes(s.B, s.se, s.mid), splitk_ws_bytes(s.B, s.mid, s.se)) / 4 + 64);
  w.gemm = b.take<char>(64);
  w.a3 = a3_mode(s, esz) == 1 ? b.take<char>(M * s.mid * esz) : nullptr;
  if (total) *total = b.off + 256;
  return w;
}

struct BwdWs {
  void *dp, *bufA, *bufB;
  float *stat, *S, *coef, *R, *dgate, *dz2, *dh, *dz1, *dpool, *part9, *tmp, *sums9;
  float *wtse, *split;  // transposed SE weight, split-K partials
  float* tmp2;          // colreduce scratch of the side stream
  char *gemm, *gemm2;   // GEMM workspaces: current stream, side stream
  // slab partials of the four parameter weight gradients, one region each, and the depthwise weight
  // gradient's [rows][9][mid] partials: their column reductions may be deferred to the end of the
  // backward (colreduce_param / colreduce_param_tap), so no later phase may reuse them
  char *wg_proj, *wg_expand, *wg_se2, *wg_se1;
};
static size_t max3(size_t a, size_t b, size_t c) { return a > b ? (a > c ? a : c) : (b > c ? b : c); }
static BwdWs bwd_ws_layout(void* base, const ogv_mbconv_desc& s, size_t esz, size_t* total) {
  Buf b(base);
  const long M = (long)s.B * s.H * s.W;
  RowPlan rp = row_plan(s.mid), rc = row_plan(s.C);
  const long S2 = dw_tile_plan(s.B, s.H, s.W, s.mid, 4).rows_max(), S3 = dw_slices(M, rc);
  const long K2 = s.mid > s.C ? s.mid : s.C;
  BwdWs w;
  w.dp = b.take<char>(M * s.C * esz);
  w.bufA = b.take<char>(M * s.mid * esz);
  w.bufB = b.take<char>(M * s.mid * esz);
  const long Smax = S2 > S3 ? S2 : S3;
  w.stat = b.take<float>(Smax * 2 * K2);
  w.S = b.take<float>(2 * K2);
  w.coef = b.take<float>(3 * K2);
  w.R = b.take<float>((size_t)5 * s.B * s.mid);
  w.dgate = b.take<float>((size_t)s.B * s.mid);
  w.dz2 = b.take<float>((size_t)s.B * s.mid);
  w.dh = b.take<float>((size_t)s.B * s.se);
  w.dz1 = b.take<float>((size_t)s.B * s.se);
  w.dpool = b.take<float>((size_t)s.B * s.mid);
  w.tmp = b.take<float>(max3(max3(colreduce_tmp_floats(Smax, 2 * K2), colreduce_tmp_floats(S2, 9L * s.mid), 16),
                             colreduce_tmp_floats(s.B, 2L * s.mid), 16));
  w.sums9 = b.take<float>(9 * (size_t)s.mid);
  w.wtse = b.take<float>((size_t)s.mid * s.se);
  w.split = b.take<float>(std::max(splitk_ws_bytes(s.B, s.se, s.mid), splitk_ws_bytes(s.B, s.mid, s.se)) / 4 + 64);
  const size_t g = max3(max3(dgrad_ws_bytes(s.C, s.mid), dgrad_ws_bytes(s.mid, s.C), wgrad_ws_bytes((int)M, s.C, s.mid)),
                        max3(wgrad_ws_bytes((int)M, s.mid, s.C), wgrad_ws_bytes(s.B, s.mid, s.se),
                             wgrad_ws_bytes(s.B, s.se, s.mid)),
                        max3(dgrad_ws_bytes(s.mid, s.se), dgrad_ws_bytes(s.se, s.mid), 64));
  w.gemm = b.take<char>(g);
  w.tmp2 = b.take<float>(colreduce_tmp_floats(S2, 9L * s.mid) + 16);
  w.gemm2 = b.take<char>(g);
  w.wg_proj = w.wg_expand = w.wg_se2 = w.wg_se1 = nullptr;   // bwd_param_ws_layout
  w.part9 = nullptr;
  if (total) *total = b.off + 256;
  return w;
}
// the four parameter weight gradients' slab partials, one region each (a separate buffer: it stays
// allocated until a deferred reduction has read it, the big workspace above need not)
static void bwd_param_ws_layout(void* base, const ogv_mbconv_desc& s, BwdWs* w, size_t* total) {
  Buf b(base);
  const long M = (long)s.B * s.H * s.W;
  char* p0 = b.take<char>(wgrad_ws_bytes((int)M, s.C, s.mid));
  char* p1 = b.take<char>(wgrad_ws_bytes((int)M, s.mid, s.C));
  char* p2 = b.take<char>(wgrad_ws_bytes(s.B, s.mid, s.se));
  char* p3 = b.take<char>(wgrad_ws_bytes(s.B, s.se, s.mid));
  float* p9 = b.take<float>(dw_tile_plan(s.B, s.H, s.W, s.mid, 4).rows_max() * 9 * s.mid);
  if (w) {
    w->wg_proj = p0;
    w->wg_expand = p1;
    w->wg_se2 = p2;
    w->wg_se1 = p3;
    w->part9 = p9;
  }
  if (total) *total = b.off + 256;
}

// Side stream for the weight-gradient work of the fused backward (independent of the data-gradient
// chain): forked from / joined back into the caller's stream with events, which also works inside a
// captured hipGraph (the side stream joins the capture).  Knob "mb_side": default 0 since round 4 --
// with the round-4 kernels the concurrent weight gradients slowed the data-gradient chain more than
// they overlapped it (7M, paired: 15.52-15.53 ms with it, 15.38-15.41 without; 15.13-15.14 with the
// Linear fork off too, profiles/r04_side_streams.log)
static int g_mb_side = 0;
void set_mb_side(int v) { g_mb_side = v; }
// knob "dw_fuse": 1 (default) = the depthwise data and weight gradients in one pass over (dd, e)
static int g_dw_fuse = 1;
void set_dw_fuse(int v) { g_dw_fuse = v; }
// knob "dw_bn2": 1 (default) = the BN2 backward computed in the depthwise backward's staging (dd never
// written to HBM: one [M, mid] write + read and the bn2_apply launch saved); needs dw_fuse
static int g_dw_bn2 = 1;
void set_dw_bn2(int v) { g_dw_bn2 = v; }
// (default 2 since the per-pixel loads run a step ahead: 7M 14.42 / 14.38 ms with 4 rows per step, 14.35 / 14.35
// with 2, profiles/r06t_knobs.log; fewer live registers, 228 vs 252 VGPRs)
static int g_dw_bwd_r = 2;
void set_dw_bwd_r(int v) { g_dw_bwd_r = v == 2 ? 2 : 4; }
// dynamic LDS of dw_dgrad_tile_kernel: the staged tile (+ the 9-tap partials with part) and, BN2-staged
// (b2), the per-image gate / dpool table
static size_t dw_dgrad_lds(const DwTile& t, bool part, bool b2) {
  size_t lds = t.lds_bytes(part ? 9 : 2, 4, sizeof(float), b2 ? g_dw_bwd_r : DW_R);
  if (b2) lds += (size_t)t.G * 2 * t.CT * sizeof(float);
  return lds;
}
struct SideStream {
  hipStream_t s = nullptr;
  hipEvent_t fork = nullptr, join = nullptr;
};
static SideStream* side_stream() {
  static SideStream ss[64];
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return nullptr;
  SideStream& x = ss[dev];
  if (!x.s) {
    if (hipStreamCreateWithFlags(&x.s, hipStreamNonBlocking) != hipSuccess) return nullptr;
    (void)hipEventCreateWithFlags(&x.fork, hipEventDisableTiming);
    (void)hipEventCreateWithFlags(&x.join, hipEventDisableTiming);
  }
  return &x;
}
// returns the stream side work goes to (the caller's when the side stream is off / unavailable)
static hipStream_t fork_side(hipStream_t st) {
  SideStream* x = g_mb_side ? side_stream() : nullptr;
  if (!x) return st;
  (void)hipEventRecord(x->fork, st);
  (void)hipStreamWaitEvent(x->s, x->fork, 0);
  return x->s;
}
static void join_side(hipStream_t st, hipStream_t side) {
  if (side == st) return;
  SideStream* x = side_stream();
  (void)hipEventRecord(x->join, side);
  (void)hipStreamWaitEvent(st, x->join, 0);
}

#define OGV_V_DISPATCH(V, FN, ...)      \
  do {                                  \
    if ((V) == 8) FN<8>(__VA_ARGS__);   \
    else if ((V) == 4) FN<4>(__VA_ARGS__); \
    else FN<1>(__VA_ARGS__);            \
  } while (0)
#define OGV_V84_DISPATCH(V, FN, ...)    \
  do {                                  \
    if ((V) == 8) FN<8>(__VA_ARGS__);   \
    else FN<4>(__VA_ARGS__);            \
  } while (0)

template <typename T>
struct Ops {
  // runtime activation -> compile-time ACT (the staging / derivative code is then branch-free)
#define OGV_DW_ACT(act, ...)                                   \
  switch (act) {                                               \
    case OGV_ACT_GELU: { constexpr int A = OGV_ACT_GELU; __VA_ARGS__; } break; \
    case OGV_ACT_SILU: { constexpr int A = OGV_ACT_SILU; __VA_ARGS__; } break; \
    case OGV_ACT_RELU: { constexpr int A = OGV_ACT_RELU; __VA_ARGS__; } break; \
    default: { constexpr int A = OGV_ACT_NONE; __VA_ARGS__; } break;           \
  }
  static void dw_fwd(const void* e, const float* w, const float* sc, const float* sh, int act, void* out, double* stat,
                     const float* shift, const DwTile& t, hipStream_t st) {
    if (skip_mask() & 8) return;
    constexpr int V = 4;
    const size_t lds = t.lds_bytes(2, V, sizeof(double), g_dw_fwd_r);
#define OGV_DWF(R_)                                                                                  \
    OGV_DW_ACT(act, if (t.ldq <= 1) dw_fwd_tile_kernel<T, V, 1, A, R_><<<dw_grid(t), 256, lds, st>>>( \
                        (const T*)e, w, sc, sh, act, (T*)out, stat, shift, t);                        \
               else if (t.ldq <= 2) dw_fwd_tile_kernel<T, V, 2, A, R_><<<dw_grid(t), 256, lds, st>>>( \
                        (const T*)e, w, sc, sh, act, (T*)out, stat, shift, t);                        \
               else dw_fwd_tile_kernel<T, V, 3, A, R_><<<dw_grid(t), 256, lds, st>>>(                  \
                        (const T*)e, w, sc, sh, act, (T*)out, stat, shift, t))
    if (g_dw_fwd_r == 8) { OGV_DWF(8) }
    else { OGV_DWF(4) }
#undef OGV_DWF
  }
  // part != nullptr: the weight-gradient partials in the same pass (dw_dgrad_tile_kernel<.., WG>)
  // b2 != nullptr: dd is BN2-backward(dA3 = dd, b2->d), computed as the rows are staged.  Rows per
  // step: knob "dw_bwd_r" for the BN2-staged kernel (2 or 4)
  static void dw_dgrad(const void* dd, const float* w, const void* e, const float* sc, const float* sh,
                       const float* mean, const float* inv, int act, void* out, float* stat, const DwTile& t,
                       hipStream_t st, float* part = nullptr, const Bn2In<T>* b2 = nullptr) {
    if (skip_mask() & 8) return;
    constexpr int V = 4;
    const int R = b2 ? g_dw_bwd_r : DW_R;
    const size_t lds = dw_dgrad_lds(t, part != nullptr, b2 != nullptr);
    const int tab_off = (int)(t.lds_bytes(part ? 9 : 2, V, sizeof(float), R) / sizeof(float));
    const Bn2In<T> bi = b2 ? *b2 : Bn2In<T>{};
#define OGV_DWD(WG_, B2_, R_)                                                                                        \
    OGV_DW_ACT(act, if (t.ldq <= 1) dw_dgrad_tile_kernel<T, V, 1, A, WG_, B2_, R_><<<dw_grid(t), 256, lds, st>>>(    \
                        (const T*)dd, w, (const T*)e, sc, sh, mean, inv, act, (T*)out, stat, t, part, bi, tab_off);  \
               else if (t.ldq <= 2) dw_dgrad_tile_kernel<T, V, 2, A, WG_, B2_, R_><<<dw_grid(t), 256, lds, st>>>(    \
                        (const T*)dd, w, (const T*)e, sc, sh, mean, inv, act, (T*)out, stat, t, part, bi, tab_off);  \
               else dw_dgrad_tile_kernel<T, V, 3, A, WG_, B2_, R_><<<dw_grid(t), 256, lds, st>>>(                     \
                        (const T*)dd, w, (const T*)e, sc, sh, mean, inv, act, (T*)out, stat, t, part, bi, tab_off))
    if (part && b2 && R == 2) { OGV_DWD(true, true, 2) }
    else if (part && b2) { OGV_DWD(true, true, DW_R) }
    else if (part) { OGV_DWD(true, false, DW_R) }
    else { OGV_DWD(false, false, DW_R) }
#undef OGV_DWD
  }
  static void dw_wgrad(const void* dd, const void* e, const float* sc, const float* sh, int act, float* part,
                       const DwTile& t, hipStream_t st) {
    if (skip_mask() & 8) return;
    constexpr int V = 4;
    const size_t lds = t.lds_bytes(9, V, sizeof(float));
    OGV_DW_ACT(act, if (t.ldq <= 1) dw_wgrad_tile_kernel<T, V, 1, A><<<dw_grid(t), 256, lds, st>>>(
                        (const T*)dd, (const T*)e, sc, sh, act, part, t);
               else if (t.ldq <= 2) dw_wgrad_tile_kernel<T, V, 2, A><<<dw_grid(t), 256, lds, st>>>(
                        (const T*)dd, (const T*)e, sc, sh, act, part, t);
               else dw_wgrad_tile_kernel<T, V, 3, A><<<dw_grid(t), 256, lds, st>>>(
                        (const T*)dd, (const T*)e, sc, sh, act, part, t))
  }
#undef OGV_DW_ACT
  template <int V>
  static void pool(const void* d, const float* sc, const float* sh, int act, float* pooled, int B, int HW, int K,
                   const RowPlan& rp, hipStream_t st) {
    if (HW >= 256) {  // measured: the fixed 4-chunk kernel is faster for large images
      se_pool_wide_kernel<T, V><<<xcd_grid((long)cdiv(K, 4 * V) * B), 256, 0, st>>>((const T*)d, sc, sh, act, pooled,
                                                                                   HW, K, B);
      return;
    }
    const ImgPlan ip = img_plan(HW, K, V);
    const unsigned g = xcd_grid((long)ip.ngx * B);
    switch (act) {
      case OGV_ACT_SILU:
        se_pool_kernel<T, V, OGV_ACT_SILU><<<g, 256, 0, st>>>((const T*)d, sc, sh, pooled, HW, K, B, ip.chunks, ip.ngx);
        break;
      case OGV_ACT_GELU:
        se_pool_kernel<T, V, OGV_ACT_GELU><<<g, 256, 0, st>>>((const T*)d, sc, sh, pooled, HW, K, B, ip.chunks, ip.ngx);
        break;
      case OGV_ACT_RELU:
        se_pool_kernel<T, V, OGV_ACT_RELU><<<g, 256, 0, st>>>((const T*)d, sc, sh, pooled, HW, K, B, ip.chunks, ip.ngx);
        break;
      default:
        se_pool_kernel<T, V, OGV_ACT_NONE><<<g, 256, 0, st>>>((const T*)d, sc, sh, pooled, HW, K, B, ip.chunks, ip.ngx);
    }
  }
  template <int V>
  static void se_reduce(const void* dA3, const void* d, const float* sc, const float* sh, const float* mean,
                        const float* inv, int act, float* R, int B, int HW, int K, const RowPlan& rp, hipStream_t st,
                        const float* gate, float* dz2) {
    if (HW >= 256) {
      se_bwd_reduce_wide_kernel<T, V><<<xcd_grid((long)cdiv(K, 4 * V) * B), 256, 0, st>>>(
          (const T*)dA3, (const T*)d, sc, sh, mean, inv, act, R, B, HW, K, gate, dz2);
      return;
    }
    const ImgPlan ip = img_plan(HW, K, V);
    const unsigned g = xcd_grid((long)ip.ngx * B);
#define OGV_SE_RED(A)                                                                                            \
  se_bwd_reduce_kernel<T, V, A><<<g, 256, 0, st>>>((const T*)dA3, (const T*)d, sc, sh, mean, inv, R, B, HW, K, \
                                                   ip.chunks, ip.ngx, gate, dz2)
    switch (act) {
      case OGV_ACT_SILU: OGV_SE_RED(OGV_ACT_SILU); break;
      case OGV_ACT_GELU: OGV_SE_RED(OGV_ACT_GELU); break;
      case OGV_ACT_RELU: OGV_SE_RED(OGV_ACT_RELU); break;
      default: OGV_SE_RED(OGV_ACT_NONE);
    }
#undef OGV_SE_RED
  }
  template <int V>
  static void bn2_apply(const void* dA3, const void* d, const float* sc, const float* sh, const float* mean,
                        const float* inv, const float* gate, const float* dpool, const float* coef, int act, void* out,
                        long M, int HW, int K, hipStream_t st) {
    const EwPlan ep = ew_plan(M, K, V);
#define OGV_BN2(A)                                                                                             \
  bn2_apply_kernel<T, V, A><<<ep.grid(), 256, 0, st>>>((const T*)dA3, (const T*)d, sc, sh, mean, inv, gate, dpool, \
                                                       coef, (T*)out, M, HW, K, ep)
    switch (act) {
      case OGV_ACT_SILU: OGV_BN2(OGV_ACT_SILU); break;
      case OGV_ACT_GELU: OGV_BN2(OGV_ACT_GELU); break;
      case OGV_ACT_RELU: OGV_BN2(OGV_ACT_RELU); break;
      default: OGV_BN2(OGV_ACT_NONE);
    }
#undef OGV_BN2
  }
  template <int V>
  static void a3(const void* d, const float* sc, const float* sh, const float* gate, int act, void* out, long M, int HW,
                 int K, hipStream_t st) {
    const EwPlan ep = ew_plan(M, K, V);
#define OGV_A3(A) a3_kernel<T, V, A><<<ep.grid(), 256, 0, st>>>((const T*)d, sc, sh, gate, (T*)out, M, HW, K, ep)
    switch (act) {
      case OGV_ACT_SILU: OGV_A3(OGV_ACT_SILU); break;
      case OGV_ACT_GELU: OGV_A3(OGV_ACT_GELU); break;
      case OGV_ACT_RELU: OGV_A3(OGV_ACT_RELU); break;
      default: OGV_A3(OGV_ACT_NONE);
    }
#undef OGV_A3
  }
  template <int V>
  static void bn_reduce(const void* dy, const void* x, const float* mean, const float* inv, float* stat, long M, int K,
                        const RowPlan& rp, long S, long per, hipStream_t st) {
    bn_bwd_reduce_kernel<T, V><<<xcd_grid((long)cdiv(K, 4 * V) * S), 256, 0, st>>>((const T*)dy, (const T*)x, mean, inv, stat, M,
                                                                        K, per);
  }
  template <int V>
  static void bn_apply(const void* dy, const void* x, const float* mean, const float* inv, const float* coef, void* out,
                       long M, int K, hipStream_t st) {
    const EwPlan ep = ew_plan(M, K, V);
    bn_bwd_apply_kernel<T, V><<<ep.grid(), 256, 0, st>>>((const T*)dy, (const T*)x, mean, inv, coef, (T*)out, M, K, ep);
  }
  template <int V>
  static void affine_res(const void* res, const void* p, const float* sc, const float* sh, void* out, long M, int K,
                         hipStream_t st) {
    const EwPlan ep = ew_plan(M, K, V);
    affine_residual_kernel<T, V><<<ep.grid(), 256, 0, st>>>((const T*)res, (const T*)p, sc, sh, (T*)out, M, K, ep);
  }
};

template <typename T>
static void mbconv_fwd_impl(const void* x, void* out, const Saved& sv, const FwdWs& w, const ogv_mbconv_desc& s,
                            const ogv_mbconv_params& P, ogv_dtype dt, hipStream_t st) {
  using O = Ops<T>;
  const long M = (long)s.B * s.H * s.W;
  const int HW = s.H * s.W;
  const bool tr = s.train != 0;
  RowPlan rp = row_plan(s.mid), rc = row_plan(s.C);
  // 1) expand GEMM (+ BN1 stats)
  {
    Epi e;
    if (tr) { e.stat = w.stat1; e.stat_shift = P.bn1_rm; }
    const int R = gemm_fwd_launch(dt, x, s.C, Pro(), P.w_expand, s.C, sv.e, s.mid, (int)M, s.mid, s.C, s.C, s.C, e, st);
    if (tr)
      bn_reduce_finalize_launch(w.stat1, R, 2L * s.mid, s.mid, (double)M, P.bn1_w, P.bn1_b,
                                                        s.bn_eps, s.bn_momentum, P.bn1_rm, P.bn1_rv, sv.mean1, sv.inv1, sv.sc1, sv.sh1, st);
    else
      bn_finalize_kernel<<<cdiv(s.mid, 256), 256, 0, st>>>(w.sums, s.mid, (double)M, P.bn1_w, P.bn1_b, s.bn_eps, s.bn_momentum,
                                                         P.bn1_rm, P.bn1_rv, sv.mean1, sv.inv1, sv.sc1, sv.sh1, 0);
  }
  // 2) depthwise conv on act(BN1(e)) (+ BN2 stats)
  {
    const DwTile t = dw_tile_plan(s.B, s.H, s.W, s.mid, 4);
    O::dw_fwd(sv.e, P.w_dw, sv.sc1, sv.sh1, s.act, sv.d, tr ? w.stat2 : nullptr,
                     tr ? P.bn2_rm : nullptr, t, st);
    if (tr)
      bn_reduce_finalize_launch(w.stat2, t.rows(), 2L * s.mid, s.mid, (double)M, P.bn2_w, P.bn2_b,
                                                        s.bn_eps, s.bn_momentum, P.bn2_rm, P.bn2_rv, sv.mean2, sv.inv2, sv.sc2, sv.sh2, st);
    else
      bn_finalize_kernel<<<cdiv(s.mid, 256), 256, 0, st>>>(w.sums, s.mid, (double)M, P.bn2_w, P.bn2_b, s.bn_eps, s.bn_momentum,
                                                         P.bn2_rm, P.bn2_rv, sv.mean2, sv.inv2, sv.sc2, sv.sh2, 0);
  }
  // 3) Squeeze-Excite gate (B rows)
  {
    OGV_V_DISPATCH(rp.V, O::template pool, sv.d, sv.sc2, sv.sh2, s.act, sv.pooled, s.B, HW, s.mid, rp, st);
    Epi e1;
    e1.bias = P.se_b1;
    if (se_gemv_on())
      se_gemv_launch(sv.pooled, s.mid, OGV_ACT_NONE, P.se_w1, s.mid, P.se_b1, nullptr, 0, 0, sv.z1, s.se, nullptr, s.B,
                     s.se, s.mid, false, st);
    else
      gemm_fwd_splitk_f32(sv.pooled, s.mid, Pro(), P.se_w1, s.mid, sv.z1, s.se, s.B, s.se, s.mid, e1, w.split, st);
    Pro p2;
    p2.act = s.act;
    Epi e2;
    e2.bias = P.se_b2;
    if (se_gemv_on())   // gate = sigmoid(z2) written by the same launch
      se_gemv_launch(sv.z1, s.se, s.act, P.se_w2, s.se, P.se_b2, nullptr, 0, 0, sv.z2, s.mid, sv.gate, s.B, s.mid,
                     s.se, false, st);
    else
      gemm_fwd_splitk_f32(sv.z1, s.se, p2, P.se_w2, s.se, sv.z2, s.mid, s.B, s.mid, s.se, e2, w.split, st, false,
                          sv.gate);  // gate = sigmoid(z2) written by the split-K reduce
  }
  // 4) project GEMM on act(BN2(d)) * gate (+ BN3 stats), then out = x + BN3(p)
  {
    Pro pr;
    pr.act = s.act;
    pr.sc = sv.sc2;
    pr.sh = sv.sh2;
    pr.gate = sv.gate;
    pr.rps = HW;
    pr.gld = s.mid;
    const void* a = sv.d;
    const int am = a3_mode(s, sizeof(T));
    if (am) {   // A3 materialised (kept for the backward in mode 2): a prologue-free GEMM
      void* a3 = am == 2 ? sv.a3 : w.a3;
      OGV_V_DISPATCH(rp.V, O::template a3, sv.d, sv.sc2, sv.sh2, sv.gate, s.act, a3, M, HW, s.mid, st);
      pr = Pro();
      a = a3;
    }
    Epi e;
    if (tr) { e.stat = w.stat3; e.stat_shift = P.bn3_rm; }
    const int R = gemm_fwd_launch(dt, a, s.mid, pr, P.w_proj, s.mid, sv.p, s.C, (int)M, s.C, s.mid, s.mid, s.mid, e, st);
    if (tr)
      bn_reduce_finalize_launch(w.stat3, R, 2L * s.C, s.C, (double)M, P.bn3_w, P.bn3_b,
                                                        s.bn_eps, s.bn_momentum, P.bn3_rm, P.bn3_rv, sv.mean3, sv.inv3, sv.sc3, sv.sh3, st);
    else
      bn_finalize_kernel<<<cdiv(s.C, 256), 256, 0, st>>>(w.sums, s.C, (double)M, P.bn3_w, P.bn3_b, s.bn_eps, s.bn_momentum,
                                                         P.bn3_rm, P.bn3_rv, sv.mean3, sv.inv3, sv.sc3, sv.sh3, 0);
    OGV_V_DISPATCH(rc.V, O::template affine_res, x, sv.p, sv.sc3, sv.sh3, out, M, s.C, st);
  }
}

template <typename T>
static void mbconv_bwd_impl(const void* dout, const void* x, const Saved& sv, void* dx, const ogv_mbconv_grads& G,
                            const BwdWs& w, const ogv_mbconv_desc& s, const ogv_mbconv_params& P, ogv_dtype dt,
                            hipStream_t st) {
  using O = Ops<T>;
  const long M = (long)s.B * s.H * s.W;
  const int HW = s.H * s.W;
  RowPlan rp = row_plan(s.mid), rc = row_plan(s.C);
  // B1) BN3 backward: dp = ca*(dout - cb - phat*cc)
  {
    const long S = dw_slices(M, rc), per = (M + S - 1) / S;
    OGV_V_DISPATCH(rc.V, O::template bn_reduce, dout, sv.p, sv.mean3, sv.inv3, w.stat, M, s.C, rc, S, per, st);
    bn_reduce_coeffs_run(w.stat, S, 2L * s.C, s.C, (float)M, P.bn3_w, sv.inv3, G.bn3_w, G.bn3_b, w.coef, s.train, st);
    OGV_V_DISPATCH(rc.V, O::template bn_apply, dout, sv.p, sv.mean3, sv.inv3, w.coef, w.dp, M, s.C, st);
  }
  // B2) project: dA3 = dp . Wp ; dWp = dp^T . (act(BN2(d)) * gate)   (dWp on the side stream)
  hipStream_t sd = fork_side(st);
  {
    gemm_dgrad_launch(dt, w.dp, s.C, P.w_proj, nullptr, 0, 0, nullptr, 1, nullptr, w.bufA, s.mid, (int)M, s.C, s.mid,
                      w.gemm, st);
    Pro pr;
    pr.act = s.act;
    pr.sc = sv.sc2;
    pr.sh = sv.sh2;
    pr.gate = sv.gate;
    pr.rps = HW;
    pr.gld = s.mid;
    const bool a3 = a3_mode(s, sizeof(T)) == 2 && sv.a3;   // the forward's A3 (the prologue's values)
    if (a3) pr = Pro();
    gemm_wgrad_launch(dt, w.dp, s.C, a3 ? sv.a3 : sv.d, s.mid, pr, nullptr, 1, G.w_proj, nullptr, (int)M, s.C, s.mid,
                      w.wg_proj, sd, nullptr, true);
  }
  // B3) one pass over (dA3, d): SE gate grads + BN2 partial sums per image
  // (+ dz2 = dgate * g * (1 - g), the gate's sigmoid backward, written by the same reduce)
  OGV_V_DISPATCH(rp.V, O::template se_reduce, w.bufA, sv.d, sv.sc2, sv.sh2, sv.mean2, sv.inv2, s.act, w.R, s.B, HW,
                 s.mid, rp, st, sv.gate, w.dz2);
  // B4) SE MLP backward (fp32, B rows): dgate = R0 -> dz2 -> (W2, b2) -> dz1 (act') -> (W1, b1) -> dpooled
  // (the two weight gradients go to the side stream, behind the project weight gradient, as soon
  // as their inputs exist; joined before B6, ahead of the next use of w.gemm in B8)
  {
    Pro p2;
    p2.act = s.act;
    gemm_wgrad_launch(OGV_F32, w.dz2, s.mid, sv.z1, s.se, p2, nullptr, 1, G.se_w2, G.se_b2, s.B, s.mid, s.se, w.wg_se2,
                      fork_side(st), nullptr, true);
    {  // dz1 = act'(z1) * (dz2 . W2):  W2 [mid, se] read reduction-major (no transpose launch)
      Epi e;
      e.Z = sv.z1;
      e.ldz = s.se;
      e.zact = s.act;
      if (se_gemv_on())
        se_gemv_launch(w.dz2, s.mid, OGV_ACT_NONE, P.se_w2, s.se, nullptr, sv.z1, s.se, s.act, w.dz1, s.se, nullptr,
                       s.B, s.se, s.mid, true, st);
      else
        gemm_fwd_splitk_f32(w.dz2, s.mid, Pro(), P.se_w2, s.se, w.dz1, s.se, s.B, s.se, s.mid, e, w.split, st, true);
    }
    gemm_wgrad_launch(OGV_F32, w.dz1, s.se, sv.pooled, s.mid, Pro(), nullptr, 1, G.se_w1, G.se_b1, s.B, s.se, s.mid,
                      w.wg_se1, fork_side(st), nullptr, true);
    {  // dpool = dz1 . W1:  W1 [se, mid] read reduction-major
      if (se_gemv_on())
        se_gemv_launch(w.dz1, s.se, OGV_ACT_NONE, P.se_w1, s.mid, nullptr, nullptr, 0, 0, w.dpool, s.mid, nullptr, s.B,
                       s.mid, s.se, true, st);
      else
        gemm_fwd_splitk_f32(w.dz1, s.se, Pro(), P.se_w1, s.mid, w.dpool, s.mid, s.B, s.mid, s.se, Epi(), w.split, st,
                            true);
    }
  }
  // B5) BN2 backward: dd = ca*(dy2 - cb - dhat*cc)  -> bufB  (with dw_bn2: computed inside B6's staging)
  // The BN2-staged kernel adds a per-image (gate, dpool) table of G x 2 x CT floats to the tile's LDS; a
  // plan whose total would pass the 64 KB default grant takes the unfused bn2_apply path instead.
  const DwTile t6 = dw_tile_plan(s.B, s.H, s.W, s.mid, 4);
  const bool bn2f = g_dw_fuse && g_dw_bn2 && dw_dgrad_lds(t6, true, true) <= 64 * 1024;
  {
    // BN2's column sums over the images, the per-image terms formed on the fly (no terms launch)
    bn_reduce_coeffs_run<true>(nullptr, s.B, 2L * s.mid, s.mid, (float)M, P.bn2_w, sv.inv2, G.bn2_w, G.bn2_b, w.coef,
                               s.train, st, Bn2Terms{w.R, sv.gate, w.dpool, HW});
    if (!bn2f)
      OGV_V_DISPATCH(rp.V, O::template bn2_apply, w.bufA, sv.d, sv.sc2, sv.sh2, sv.mean2, sv.inv2, sv.gate, w.dpool,
                     w.coef, s.act, w.bufB, M, HW, s.mid, st);
  }
  // B6) depthwise backward: dy1 = dgrad(dd) * act'(BN1(e)) -> dy1 (+ BN1 sums); dWdw from (dd, act(BN1(e)))
  // dy1 = bufA (dd in bufB), or bufB when dd is staged from (dA3 = bufA, d)
  void* dy1 = bn2f ? w.bufB : w.bufA;
  void* de = bn2f ? w.bufA : w.bufB;
  {
    const DwTile& t = t6;
    join_side(st, sd);
    if (bn2f) {  // one pass over (dA3, d, e): BN2 backward + data gradient + BN1 sums + dWdw partials
      const Bn2In<T> b2 = {(const T*)sv.d, sv.sc2, sv.sh2, sv.mean2, sv.inv2, sv.gate, w.dpool, w.coef, HW};
      O::dw_dgrad(w.bufA, P.w_dw, sv.e, sv.sc1, sv.sh1, sv.mean1, sv.inv1, s.act, dy1, w.stat, t, st, w.part9, &b2);
      sd = fork_side(st);
      // dWdw: deferred into the batched flush (written channel-major there), or reduced here
      if (!colreduce_param_tap(w.part9, G.w_dw, t.rows(), s.mid, 9L * s.mid)) {
        colreduce(w.part9, w.sums9, t.rows(), 9L * s.mid, 9L * s.mid, w.tmp2, sd);
        tapmajor_to_chan_kernel<<<cdiv(9 * s.mid, 256), 256, 0, sd>>>(w.sums9, G.w_dw, s.mid);
      }
    } else if (g_dw_fuse) {   // one pass over (dd, e): data gradient + BN1 sums + dWdw partials
      O::dw_dgrad(w.bufB, P.w_dw, sv.e, sv.sc1, sv.sh1, sv.mean1, sv.inv1, s.act, w.bufA, w.stat, t, st, w.part9);
      sd = fork_side(st);  // the partials' reduction overlaps the BN1 backward
      colreduce(w.part9, w.sums9, t.rows(), 9L * s.mid, 9L * s.mid, w.tmp2, sd);
      tapmajor_to_chan_kernel<<<cdiv(9 * s.mid, 256), 256, 0, sd>>>(w.sums9, G.w_dw, s.mid);
    } else {
      sd = fork_side(st);  // bufB (dd) complete: dWdw on the side stream overlaps the data gradient
      O::dw_wgrad(w.bufB, sv.e, sv.sc1, sv.sh1, s.act, w.part9, t, sd);
      colreduce(w.part9, w.sums9, t.rows(), 9L * s.mid, 9L * s.mid, w.tmp2, sd);
      tapmajor_to_chan_kernel<<<cdiv(9 * s.mid, 256), 256, 0, sd>>>(w.sums9, G.w_dw, s.mid);
      O::dw_dgrad(w.bufB, P.w_dw, sv.e, sv.sc1, sv.sh1, sv.mean1, sv.inv1, s.act,
                       w.bufA, w.stat, t, st);
    }
  }
  join_side(st, sd);  // B7 overwrites de
  // B7) BN1 backward: de = ca*(dy1 - cb - ehat*cc)
  {
    const long R1 = dw_tile_plan(s.B, s.H, s.W, s.mid, 4).rows();
    bn_reduce_coeffs_run(w.stat, R1, 2L * s.mid, s.mid, (float)M, P.bn1_w, sv.inv1, G.bn1_w, G.bn1_b, w.coef, s.train,
                         st);
  }
  OGV_V_DISPATCH(rp.V, O::template bn_apply, dy1, sv.e, sv.mean1, sv.inv1, w.coef, de, M, s.mid, st);
  // B8) expand: dx = de . We + dout (residual) ; dWe = de^T . x
  sd = fork_side(st);  // dWe on the side stream, overlapping dx
  gemm_wgrad_launch(dt, de, s.mid, x, s.C, Pro(), nullptr, 1, G.w_expand, nullptr, (int)M, s.mid, s.C, w.wg_expand,
                    sd, nullptr, true);
  gemm_dgrad_launch(dt, de, s.mid, P.w_expand, nullptr, 0, 0, nullptr, 1, dout, dx, s.C, (int)M, s.mid, s.C,
                    w.gemm, st);
  join_side(st, sd);
}

static int mb_check(const ogv_mbconv_desc* s, ogv_dtype dt, const char* who) {
  OGV_REQUIRE(s, "%s: null desc", who);
  OGV_REQUIRE(s->B > 0 && s->H > 0 && s->W > 0 && s->C > 0 && s->mid > 0 && s->se > 0, "%s: bad shape", who);
  OGV_REQUIRE(s->C % 4 == 0 && s->mid % 4 == 0, "%s: channels must be multiples of 4 (C=%d, mid=%d)", who, s->C,
              s->mid);
  OGV_REQUIRE(dt == OGV_F32 || dt == OGV_BF16, "%s: bad dtype", who);
  OGV_REQUIRE(s->act >= OGV_ACT_NONE && s->act <= OGV_ACT_RELU, "%s: bad activation", who);
  OGV_REQUIRE(s->a3 >= -1 && s->a3 <= 2, "%s: bad A3 mode %d (-1, 0, 1 or 2)", who, s->a3);
  return OGV_OK;
}

}  // namespace ogv

using namespace ogv;

extern "C" size_t ogv_mbconv_saved_bytes(const ogv_mbconv_desc* s, ogv_dtype dt) {
  if (!s) return 0;
  size_t t = 0;
  saved_layout(nullptr, *s, dt == OGV_BF16 ? 2 : 4, &t);
  return t;
}

extern "C" int ogv_mbconv_a3_mode(const ogv_mbconv_desc* s, ogv_dtype dt) {
  if (!s) return -1;
  return a3_resolve(*s, dt == OGV_BF16 ? 2 : 4);
}

extern "C" size_t ogv_mbconv_ws_bytes(const ogv_mbconv_desc* s, ogv_dtype dt) {
  if (!s) return 0;
  size_t a = 0, b = 0;
  fwd_ws_layout(nullptr, *s, dt == OGV_BF16 ? 2 : 4, &a);
  bwd_ws_layout(nullptr, *s, dt == OGV_BF16 ? 2 : 4, &b);
  return a > b ? a : b;
}

extern "C" int ogv_mbconv_fwd(const void* x, void* out, void* saved, void* ws, const ogv_mbconv_desc* s,
                              const ogv_mbconv_params* P, ogv_dtype dt, void* stream) {
  int rc = mb_check(s, dt, "ogv_mbconv_fwd");
  if (rc) return rc;
  OGV_REQUIRE(x && out && saved && ws && P, "ogv_mbconv_fwd: null pointer");
  OGV_REQUIRE(P->w_expand && P->w_dw && P->se_w1 && P->se_b1 && P->se_w2 && P->se_b2 && P->w_proj,
              "ogv_mbconv_fwd: missing weight");
  OGV_REQUIRE(P->bn1_rm && P->bn1_rv && P->bn2_rm && P->bn2_rv && P->bn3_rm && P->bn3_rv,
              "ogv_mbconv_fwd: missing BatchNorm running statistics");
  Saved sv = saved_layout(saved, *s, dt == OGV_BF16 ? 2 : 4, nullptr);
  FwdWs w = fwd_ws_layout(ws, *s, dt == OGV_BF16 ? 2 : 4, nullptr);
  if (dt == OGV_BF16) mbconv_fwd_impl<bf16>(x, out, sv, w, *s, *P, dt, as_stream(stream));
  else mbconv_fwd_impl<float>(x, out, sv, w, *s, *P, dt, as_stream(stream));
  return check_launch("ogv_mbconv_fwd");
}

extern "C" size_t ogv_mbconv_param_ws_bytes(const ogv_mbconv_desc* s) {
  if (!s) return 0;
  size_t t = 0;
  bwd_param_ws_layout(nullptr, *s, nullptr, &t);
  return t;
}

extern "C" int ogv_mbconv_bwd(const void* dout, const void* x, const void* saved, void* dx,
                              const ogv_mbconv_grads* G, void* ws, void* param_ws, const ogv_mbconv_desc* s,
                              const ogv_mbconv_params* P, ogv_dtype dt, void* stream) {
  int rc = mb_check(s, dt, "ogv_mbconv_bwd");
  if (rc) return rc;
  OGV_REQUIRE(dout && x && saved && dx && G && ws && param_ws && P, "ogv_mbconv_bwd: null pointer");
  OGV_REQUIRE(G->w_expand && G->bn1_w && G->bn1_b && G->w_dw && G->bn2_w && G->bn2_b && G->se_w1 && G->se_b1 &&
                  G->se_w2 && G->se_b2 && G->w_proj && G->bn3_w && G->bn3_b,
              "ogv_mbconv_bwd: every gradient output must be given");
  Saved sv = saved_layout(const_cast<void*>(saved), *s, dt == OGV_BF16 ? 2 : 4, nullptr);
  BwdWs w = bwd_ws_layout(ws, *s, dt == OGV_BF16 ? 2 : 4, nullptr);
  bwd_param_ws_layout(param_ws, *s, &w, nullptr);
  if (dt == OGV_BF16) mbconv_bwd_impl<bf16>(dout, x, sv, dx, *G, w, *s, *P, dt, as_stream(stream));
  else mbconv_bwd_impl<float>(dout, x, sv, dx, *G, w, *s, *P, dt, as_stream(stream));
  return check_launch("ogv_mbconv_bwd");
}
