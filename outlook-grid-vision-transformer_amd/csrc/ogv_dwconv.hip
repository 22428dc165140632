// Depthwise 3x3 convolution on NHWC rows (MBConv.depthwise, src/model/mbc_conv.py:75-79:
// Conv2d(mid, mid, 3, stride, padding=1, groups=mid)), plus the deterministic column reducer
// shared by every "sum over the M rows" gradient (LN gamma/beta, conv weights, GEMM slabs).
//
// fwd  : out[b,oy,ox,c] = sum_{ki,kj} w[c,ki,kj] * in[b, oy*s+ki-1, ox*s+kj-1, c]   (+ bias[c])
// dgrad: din[b,y,x,c]   = sum_{ki,kj: (y+1-ki)%s==0 ...} w[c,ki,kj] * dout[b,(y+1-ki)/s,(x+1-kj)/s,c]
// wgrad: dw[c,ki,kj]    = sum_{b,oy,ox} dout[b,oy,ox,c] * in[b, oy*s+ki-1, ox*s+kj-1, c]
//        (per-block partials [S][9][C] -> column reducer; dbias = sum dout)
// Channels are vectorised V-wide per thread (16-B loads for bf16 at V=8); weights are staged as
// wt[tap][C] fp32 so a thread's 9 taps x V channels are contiguous.
#include <vector>

#include "ogv_common.h"

namespace ogv {

// ------------------------------------------------------------------ column reducer
// dst[j] (+)= sum_r src[r*ld + j], j < n.  Block = 64 columns x 4 row lanes; grid.y splits rows.
template <typename T>
__global__ __launch_bounds__(256) void colreduce_kernel(const T* __restrict__ src, T* __restrict__ dst, long R, long n,
                                                        long ld, long rows_per_chunk, T* __restrict__ dst2, long n1) {
  __shared__ T red[4][64];
  const int cx = threadIdx.x & 63, ry = threadIdx.x >> 6;
  const long j = (long)blockIdx.x * 64 + cx;
  const long r0 = (long)blockIdx.y * rows_per_chunk;
  const long r1 = r0 + rows_per_chunk < R ? r0 + rows_per_chunk : R;
  T acc = 0;
  if (j < n) {
    long r = r0 + ry;
    for (; r + 12 < r1; r += 16) {
      const T a = src[r * ld + j], b = src[(r + 4) * ld + j], c = src[(r + 8) * ld + j], d = src[(r + 12) * ld + j];
      acc += (a + b) + (c + d);
    }
    for (; r < r1; r += 4) acc += src[r * ld + j];
  }
  red[ry][cx] = acc;
  __syncthreads();
  if (ry == 0 && j < n) {
    const T s = (red[0][cx] + red[1][cx]) + (red[2][cx] + red[3][cx]);
    if (dst2 && j >= n1) dst2[j - n1] = s;  // single-pass split destination (gridDim.y == 1)
    else dst[(long)blockIdx.y * n + j] = s;
  }
}

// Single-pass form for up to 2048 rows (one launch instead of two): block = CR4_CQ column quads
// (16-B loads) x CR4_RG row groups; each thread keeps 8 rows' loads in flight, then the row-group
// sums are combined in a fixed order through LDS.  Needs n, ld % 4 == 0 and 16-B alignment (fp32
// only); split destination as in colreduce_kernel.  Round 4: 64 quads x 4 row groups (1 KB of each
// slab row per block, was 256 B: the partial slabs are rows ~100 KB-600 KB apart, and the wider
// contiguous run per row keeps the HBM bursts full -- the batched parameter-gradient flush below
// uses the same block body, so deferred and immediate reductions stay bit-identical).
constexpr int CR4_CQ = 64, CR4_RG = 256 / CR4_CQ;
__device__ __forceinline__ void colreduce4_block(const float* __restrict__ src, float* __restrict__ dst, long R,
                                                 long n, long ld, float* __restrict__ dst2, long n1, long colblk,
                                                 long tapC) {
  __shared__ float4 red[CR4_RG][CR4_CQ];
  const int cq = threadIdx.x % CR4_CQ, rg = threadIdx.x / CR4_CQ;
  const long j = (colblk * CR4_CQ + cq) * 4;
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  if (j < n) {
    long r = rg;
    for (; r + 7 * CR4_RG < R; r += 8 * CR4_RG) {
      float4 v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = *reinterpret_cast<const float4*>(src + (r + u * CR4_RG) * ld + j);
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        acc.x += v[u].x; acc.y += v[u].y; acc.z += v[u].z; acc.w += v[u].w;
      }
    }
    for (; r < R; r += CR4_RG) {
      const float4 v = *reinterpret_cast<const float4*>(src + r * ld + j);
      acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
    }
  }
  red[rg][cq] = acc;
  __syncthreads();
  if (rg == 0 && j < n) {
    float4 t = red[0][cq];
#pragma unroll
    for (int g = 1; g < CR4_RG; ++g) {
      const float4 v = red[g][cq];
      t.x += v.x; t.y += v.y; t.z += v.z; t.w += v.w;
    }
    const float o[4] = {t.x, t.y, t.z, t.w};
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const long c = j + q;
      if (c >= n) break;
      if (dst2 && c >= n1) dst2[c - n1] = o[q];
      else if (tapC > 0) dst[(c % tapC) * 9 + c / tapC] = o[q];
      else dst[c] = o[q];
    }
  }
}
__global__ __launch_bounds__(256) void colreduce4_kernel(const float* __restrict__ src, float* __restrict__ dst, long R,
                                                         long n, long ld, float* __restrict__ dst2, long n1) {
  colreduce4_block(src, dst, R, n, ld, dst2, n1, blockIdx.x, 0);
}
static inline unsigned colreduce4_blocks(long n) { return (unsigned)((n + 4 * CR4_CQ - 1) / (4 * CR4_CQ)); }

// Sum R rows of a [R, ld] fp32 slab into dst[n].  Two passes when R is large; tmp needs
// colreduce_tmp_floats(R, n) floats (may be null when that is 0).  Deterministic.
size_t colreduce_tmp_floats(long R, long n) {
  if (R <= 256) return 0;
  const long chunks = (R + 255) / 256;
  return (size_t)(chunks < 64 ? chunks : 64) * n;
}

template <typename T>
static void colreduce_t(const T* src, T* dst, long R, long n, long ld, T* tmp, hipStream_t s, T* dst2, long n1) {
  const unsigned gx = (unsigned)((n + 63) / 64);
  if (!dst2) n1 = n;
  if constexpr (sizeof(T) == 4) {
    if (R > 64 && R <= 2048 && (n & 3) == 0 && (ld & 3) == 0 && (reinterpret_cast<uintptr_t>(src) & 15) == 0) {
      colreduce4_kernel<<<colreduce4_blocks(n), 256, 0, s>>>(src, dst, R, n, ld, dst2, n1);
      return;
    }
  }
  if (R <= 256) {
    colreduce_kernel<T><<<dim3(gx, 1), 256, 0, s>>>(src, dst, R, n, ld, R, dst2, n1);
    return;
  }
  long chunks = (R + 255) / 256;
  if (chunks > 64) chunks = 64;
  const long per = (R + chunks - 1) / chunks;
  chunks = (R + per - 1) / per;
  colreduce_kernel<T><<<dim3(gx, (unsigned)chunks), 256, 0, s>>>(src, tmp, R, n, ld, per, nullptr, n);
  colreduce_kernel<T><<<dim3(gx, 1), 256, 0, s>>>(tmp, dst, chunks, n, n, chunks, dst2, n1);
}
void colreduce(const float* src, float* dst, long R, long n, long ld, float* tmp, hipStream_t s, float* dst2,
               long n1) {
  colreduce_t<float>(src, dst, R, n, ld, tmp, s, dst2, n1);
}
void colreduce(const double* src, double* dst, long R, long n, long ld, double* tmp, hipStream_t s) {
  colreduce_t<double>(src, dst, R, n, ld, tmp, s, nullptr, n);
}

// ------------------------------------------------------------------ deferred, batched reductions
// Parameter-gradient column sums recorded while deferral is on, then run as one launch: block b
// works on descriptor j (start[j] <= b < start[j + 1]) exactly as a colreduce4 block does.
struct RedDesc {
  const float* src;
  float *dst, *dst2;
  long R, n, ld, n1;
  long tapC;   // > 0: column tap*tapC + c stored at dst[c*9 + tap] (depthwise weight gradient)
};
constexpr int RED_BATCH = 48;   // descriptors per launch (kernel arguments < 4 KB)
struct RedBatch {
  RedDesc d[RED_BATCH];
  int start[RED_BATCH + 1];
  int count;
};

__global__ __launch_bounds__(256) void colreduce_batch_kernel(RedBatch b) {
  // descriptor of this block: the number of start offsets <= blockIdx.x, counted with one ballot
  // (a dynamically indexed walk over the kernel-argument table made every step a dependent load)
  __shared__ int jd;
  if (threadIdx.x < 64) {
    const int lane = threadIdx.x;
    const bool le = lane >= 1 && lane < b.count && b.start[lane] <= (int)blockIdx.x;
    const unsigned long long m = __ballot(le);
    if (lane == 0) jd = __popcll(m);
  }
  __syncthreads();
  const int j = __builtin_amdgcn_readfirstlane(jd);
  const RedDesc d = b.d[j];
  colreduce4_block(d.src, d.dst, d.R, d.n, d.ld, d.dst2, d.n1, (long)blockIdx.x - b.start[j], d.tapC);
}

static bool g_defer = false;
static std::vector<RedDesc> g_pending;

void colreduce_param(const float* src, float* dst, long R, long n, long ld, float* tmp, hipStream_t s, float* dst2,
                     long n1) {
  const bool fits = (n & 3) == 0 && (ld & 3) == 0 && (reinterpret_cast<uintptr_t>(src) & 15) == 0 && R > 0 &&
                    (n + 63) / 64 < (1L << 20);
  if (g_defer && fits) {
    g_pending.push_back(RedDesc{src, dst, dst2, R, n, ld, dst2 ? n1 : n, 0});
    return;
  }
  colreduce(src, dst, R, n, ld, tmp, s, dst2, n1);
}

bool colreduce_param_tap(const float* src, float* dst, long R, long C, long ld) {
  const long n = 9 * C;
  const bool fits = (n & 3) == 0 && (ld & 3) == 0 && (reinterpret_cast<uintptr_t>(src) & 15) == 0 && R > 0 &&
                    (n + 63) / 64 < (1L << 20);
  if (!g_defer || !fits) return false;
  g_pending.push_back(RedDesc{src, dst, nullptr, R, n, ld, n, C});
  return true;
}

}  // namespace ogv

using namespace ogv;

extern "C" int ogv_reduce_defer(int on) {
  g_defer = on != 0;
  return (int)g_pending.size();
}

extern "C" int ogv_reduce_flush(void* stream) {
  hipStream_t s = as_stream(stream);
  size_t i = 0;
  while (i < g_pending.size()) {
    RedBatch b{};
    int blocks = 0;
    for (; b.count < RED_BATCH && i < g_pending.size(); ++i) {
      const RedDesc& d = g_pending[i];
      b.d[b.count] = d;
      b.start[b.count] = blocks;
      blocks += (int)colreduce4_blocks(d.n);
      ++b.count;
    }
    b.start[b.count] = blocks;
    colreduce_batch_kernel<<<blocks, 256, 0, s>>>(b);
  }
  g_pending.clear();
  return check_launch("ogv_reduce_flush");
}

namespace ogv {

// ------------------------------------------------------------------ depthwise conv kernels
struct DwGeom {
  int B, H, W, C, Ho, Wo, stride;
};

// wt[tap*C + c] = w[c*9 + tap]
__global__ void dw_weight_t_kernel(const float* __restrict__ w, float* __restrict__ wt, int C) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= 9 * C) return;
  const int tap = i / C, c = i - tap * C;
  wt[i] = w[c * 9 + tap];
}

template <typename T, int V>
__global__ __launch_bounds__(256) void dw_fwd_kernel(const T* __restrict__ in, const float* __restrict__ wt,
                                                     const float* __restrict__ bias, T* __restrict__ out, DwGeom g) {
  const int nch = g.C / V;
  const long total = (long)g.B * g.Ho * g.Wo * nch;
  const long tid = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (tid >= total) return;
  const int c0 = (int)(tid % nch) * V;
  const long p = tid / nch;
  const int ox = (int)(p % g.Wo);
  const long t = p / g.Wo;
  const int oy = (int)(t % g.Ho);
  const long b = t / g.Ho;
  float acc[V];
#pragma unroll
  for (int i = 0; i < V; ++i) acc[i] = bias ? bias[c0 + i] : 0.f;
#pragma unroll
  for (int ki = 0; ki < 3; ++ki) {
    const int y = oy * g.stride + ki - 1;
    if (y < 0 || y >= g.H) continue;
#pragma unroll
    for (int kj = 0; kj < 3; ++kj) {
      const int x = ox * g.stride + kj - 1;
      if (x < 0 || x >= g.W) continue;
      float v[V], w[V];
      load_vec<T, V>(in + ((b * g.H + y) * g.W + x) * g.C + c0, v);
      load_vec<float, V>(wt + (ki * 3 + kj) * g.C + c0, w);
#pragma unroll
      for (int i = 0; i < V; ++i) acc[i] = fmaf(w[i], v[i], acc[i]);
    }
  }
  store_vec<T, V>(out + p * g.C + c0, acc);
}

template <typename T, int V>
__global__ __launch_bounds__(256) void dw_dgrad_kernel(const T* __restrict__ dout, const float* __restrict__ wt,
                                                       T* __restrict__ din, DwGeom g) {
  const int nch = g.C / V;
  const long total = (long)g.B * g.H * g.W * nch;
  const long tid = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (tid >= total) return;
  const int c0 = (int)(tid % nch) * V;
  const long p = tid / nch;
  const int x = (int)(p % g.W);
  const long t = p / g.W;
  const int y = (int)(t % g.H);
  const long b = t / g.H;
  float acc[V];
#pragma unroll
  for (int i = 0; i < V; ++i) acc[i] = 0.f;
#pragma unroll
  for (int ki = 0; ki < 3; ++ki) {
    const int ny = y + 1 - ki;
    if (ny < 0 || ny % g.stride) continue;
    const int oy = ny / g.stride;
    if (oy >= g.Ho) continue;
#pragma unroll
    for (int kj = 0; kj < 3; ++kj) {
      const int nx = x + 1 - kj;
      if (nx < 0 || nx % g.stride) continue;
      const int ox = nx / g.stride;
      if (ox >= g.Wo) continue;
      float d[V], w[V];
      load_vec<T, V>(dout + ((b * g.Ho + oy) * g.Wo + ox) * g.C + c0, d);
      load_vec<float, V>(wt + (ki * 3 + kj) * g.C + c0, w);
#pragma unroll
      for (int i = 0; i < V; ++i) acc[i] = fmaf(w[i], d[i], acc[i]);
    }
  }
  store_vec<T, V>(din + p * g.C + c0, acc);
}

// Block: 256 threads = LANES pixel lanes x NCHB channel chunks (V channels each) of one channel
// tile; grid = (channel tiles, S pixel slices).  part[s][tap*C + c] (+ part[s][9C + c] = dbias).
template <typename T, int V>
__global__ __launch_bounds__(256) void dw_wgrad_kernel(const T* __restrict__ dout, const T* __restrict__ in,
                                                       float* __restrict__ part, DwGeom g, int nchb,
                                                       long pix_per_slice, int with_bias) {
  __shared__ float red[256 * (V <= 4 ? 10 : 5)];
  const int lanes = 256 / nchb;
  const int cl = threadIdx.x % nchb, pl = threadIdx.x / nchb;
  const int c0 = (blockIdx.x * nchb + cl) * V;
  const bool active = pl < lanes && c0 < g.C;
  const long P = (long)g.B * g.Ho * g.Wo;
  const long p0 = (long)blockIdx.y * pix_per_slice;
  const long p1 = p0 + pix_per_slice < P ? p0 + pix_per_slice : P;
  float acc[10][V];
#pragma unroll
  for (int k = 0; k < 10; ++k)
#pragma unroll
    for (int i = 0; i < V; ++i) acc[k][i] = 0.f;
  if (active) {
    for (long p = p0 + pl; p < p1; p += lanes) {
      const int ox = (int)(p % g.Wo);
      const long t = p / g.Wo;
      const int oy = (int)(t % g.Ho);
      const long b = t / g.Ho;
      float d[V];
      load_vec<T, V>(dout + p * g.C + c0, d);
#pragma unroll
      for (int i = 0; i < V; ++i) acc[9][i] += d[i];
#pragma unroll
      for (int ki = 0; ki < 3; ++ki) {
        const int y = oy * g.stride + ki - 1;
        if (y < 0 || y >= g.H) continue;
#pragma unroll
        for (int kj = 0; kj < 3; ++kj) {
          const int x = ox * g.stride + kj - 1;
          if (x < 0 || x >= g.W) continue;
          float v[V];
          load_vec<T, V>(in + ((b * g.H + y) * g.W + x) * g.C + c0, v);
#pragma unroll
          for (int i = 0; i < V; ++i) acc[ki * 3 + kj][i] = fmaf(d[i], v[i], acc[ki * 3 + kj][i]);
        }
      }
    }
  }
  // reduce across the pixel lanes of each channel chunk: 10 taps (9 + bias) in LDS passes
  constexpr int TPP = V <= 4 ? 10 : 5;  // taps per pass
  float* out = part + (long)blockIdx.y * 10 * g.C;
#pragma unroll
  for (int k0 = 0; k0 < 10; k0 += TPP) {
#pragma unroll
    for (int i = 0; i < V; ++i) {
#pragma unroll
      for (int k = 0; k < TPP; ++k) red[k * 256 + threadIdx.x] = acc[k0 + k][i];
      __syncthreads();
      for (int idx = threadIdx.x; idx < nchb * TPP; idx += 256) {   // nchb*TPP can exceed 256
        const int k = idx / nchb, ch = idx % nchb;
        const int c = (blockIdx.x * nchb + ch) * V + i;
        float s = 0.f;
        for (int l = 0; l < lanes; ++l) s += red[k * 256 + l * nchb + ch];
        const int tap = k0 + k;
        if (c < g.C && (tap < 9 || with_bias)) out[(long)tap * g.C + c] = s;
      }
      __syncthreads();
    }
  }
}

// dw[c*9 + tap] = sum9[tap*C + c]
__global__ void dw_weight_untranspose_kernel(const float* __restrict__ s, float* __restrict__ dw, int C) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= 9 * C) return;
  const int c = i / 9, tap = i - c * 9;
  dw[i] = s[tap * C + c];
}

static int dw_vec(int C) { return C % 8 == 0 ? 8 : (C % 4 == 0 ? 4 : 1); }

static int dw_check(int B, int H, int W, int C, int stride, ogv_dtype dt, DwGeom& g, const char* who) {
  OGV_REQUIRE(B > 0 && H > 0 && W > 0 && C > 0, "%s: bad shape", who);
  OGV_REQUIRE(stride == 1 || stride == 2, "%s: stride %d unsupported", who, stride);
  OGV_REQUIRE(dt == OGV_F32 || dt == OGV_BF16, "%s: bad dtype", who);
  g.B = B; g.H = H; g.W = W; g.C = C; g.stride = stride;
  g.Ho = (H - 1) / stride + 1;
  g.Wo = (W - 1) / stride + 1;
  return OGV_OK;
}

struct DwWgradPlan {
  int nchb, ctiles, S;
  long per;
};
static DwWgradPlan dw_wgrad_plan(const DwGeom& g, int V) {
  DwWgradPlan p;
  const int nch = g.C / V;
  p.nchb = nch < 64 ? nch : 64;
  p.ctiles = (nch + p.nchb - 1) / p.nchb;
  const long P = (long)g.B * g.Ho * g.Wo;
  long S = (2048 + p.ctiles - 1) / p.ctiles;
  const long lanes = 256 / p.nchb;
  const long maxS = (P + lanes * 16 - 1) / (lanes * 16);  // >= 16 pixels per lane
  if (S > maxS) S = maxS;
  if (S < 1) S = 1;
  p.per = (P + S - 1) / S;
  p.S = (int)((P + p.per - 1) / p.per);
  return p;
}

}  // namespace ogv

using namespace ogv;

#define OGV_DW_DISPATCH(FN, ...)                                            \
  do {                                                                      \
    const int vv = dw_vec(C);                                               \
    if (dt == OGV_BF16) {                                                   \
      if (vv == 8) FN<bf16, 8>(__VA_ARGS__);                                \
      else if (vv == 4) FN<bf16, 4>(__VA_ARGS__);                           \
      else FN<bf16, 1>(__VA_ARGS__);                                        \
    } else {                                                                \
      if (vv == 8) FN<float, 8>(__VA_ARGS__);                               \
      else if (vv == 4) FN<float, 4>(__VA_ARGS__);                          \
      else FN<float, 1>(__VA_ARGS__);                                       \
    }                                                                       \
  } while (0)

template <typename T, int V>
static void dw_fwd_launch(const void* in, const float* wt, const float* bias, void* out, const DwGeom& g,
                          hipStream_t s) {
  const long total = (long)g.B * g.Ho * g.Wo * (g.C / V);
  dw_fwd_kernel<T, V><<<cdiv(total, 256), 256, 0, s>>>((const T*)in, wt, bias, (T*)out, g);
}
template <typename T, int V>
static void dw_dgrad_launch(const void* dout, const float* wt, void* din, const DwGeom& g, hipStream_t s) {
  const long total = (long)g.B * g.H * g.W * (g.C / V);
  dw_dgrad_kernel<T, V><<<cdiv(total, 256), 256, 0, s>>>((const T*)dout, wt, (T*)din, g);
}
template <typename T, int V>
static void dw_wgrad_launch(const void* dout, const void* in, float* part, const DwGeom& g, int with_bias,
                            hipStream_t s) {
  DwWgradPlan p = dw_wgrad_plan(g, V);
  dw_wgrad_kernel<T, V><<<dim3(p.ctiles, p.S), 256, 0, s>>>((const T*)dout, (const T*)in, part, g, p.nchb, p.per,
                                                             with_bias);
}

extern "C" size_t ogv_dwconv_fwd_ws_bytes(int C) { return (size_t)9 * C * sizeof(float); }

extern "C" int ogv_dwconv3x3_fwd(const void* x, const float* w, const float* bias, void* y, int B, int H, int W, int C,
                                 int stride, void* ws, ogv_dtype dt, void* stream) {
  OGV_REQUIRE(x && w && y && ws, "ogv_dwconv3x3_fwd: null pointer");
  DwGeom g;
  int rc = dw_check(B, H, W, C, stride, dt, g, "ogv_dwconv3x3_fwd");
  if (rc) return rc;
  hipStream_t s = as_stream(stream);
  float* wt = (float*)ws;
  dw_weight_t_kernel<<<cdiv(9 * C, 256), 256, 0, s>>>(w, wt, C);
  OGV_DW_DISPATCH(dw_fwd_launch, x, wt, bias, y, g, s);
  return check_launch("ogv_dwconv3x3_fwd");
}

extern "C" size_t ogv_dwconv_bwd_ws_bytes(int B, int H, int W, int C, int stride) {
  DwGeom g;
  if (dw_check(B, H, W, C, stride, OGV_F32, g, "ws") != OGV_OK) return 0;
  DwWgradPlan p = dw_wgrad_plan(g, dw_vec(C));
  const size_t part = (size_t)p.S * 10 * C;
  return (9 * (size_t)C + part + colreduce_tmp_floats(p.S, 10L * C) + 10 * (size_t)C) * sizeof(float);
}

extern "C" int ogv_dwconv3x3_bwd(const void* dy, const void* x, const float* w, void* dx, float* dw, float* dbias,
                                 int B, int H, int W, int C, int stride, void* ws, ogv_dtype dt, void* stream) {
  OGV_REQUIRE(dy && x && w && ws, "ogv_dwconv3x3_bwd: null pointer");
  DwGeom g;
  int rc = dw_check(B, H, W, C, stride, dt, g, "ogv_dwconv3x3_bwd");
  if (rc) return rc;
  hipStream_t s = as_stream(stream);
  DwWgradPlan p = dw_wgrad_plan(g, dw_vec(C));
  float* wt = (float*)ws;
  float* part = wt + 9 * (size_t)C;
  float* tmp = part + (size_t)p.S * 10 * C;
  float* sum10 = tmp + colreduce_tmp_floats(p.S, 10L * C);
  if (dx) {
    dw_weight_t_kernel<<<cdiv(9 * C, 256), 256, 0, s>>>(w, wt, C);
    OGV_DW_DISPATCH(dw_dgrad_launch, dy, wt, dx, g, s);
  }
  if (dw || dbias) {
    OGV_DW_DISPATCH(dw_wgrad_launch, dy, x, part, g, dbias ? 1 : 0, s);
    // tap sums -> sum10[0, 9C) (then untransposed into dw), bias sums straight into dbias
    colreduce(part, sum10, p.S, dbias ? 10L * C : 9L * C, 10L * C, tmp, s, dbias, 9L * C);
    if (dw) dw_weight_untranspose_kernel<<<cdiv(9 * C, 256), 256, 0, s>>>(sum10, dw, C);
  }
  return check_launch("ogv_dwconv3x3_bwd");
}
