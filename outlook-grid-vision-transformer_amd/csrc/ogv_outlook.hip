// Outlook aggregation on NHWC rows: per (pixel, head) softmax over the k*k logits, then a
// weighted gather of the zero-padded k*k neighbourhood of v.
//
// Reference semantics (src/model/outlook_attention.py:100-120, stride 1):
//   a   = softmax over j of logits[b, head*kk + j, y, x]          (no scaling, :106-107)
//   y[b, c, y, x] = sum_j a[b, y, x, head(c), j] * v_pad[b, c, y + ki - p, x + kj - p]
//   with j = ki*k + kj, p = k//2, out-of-image neighbours = 0 but still counted in the softmax.
// Forward never materialises the 9x unfolded tensor.  Backward is gather-form (no atomics):
//   dP[p,h,j]  = <dy[p, h-slice], v[p + off_j, h-slice]>
//   dlogit     = P * (dP - sum_j P*dP)
//   dv[q, c]   = sum_j P[q - off_j, h, j] * dy[q - off_j, c]      (the col2im fold, as a gather)
#include <initializer_list>

#include "ogv_common.h"
#include "ogv_gemm.h"

namespace ogv {

template <typename T, int V, int KS>
__global__ __launch_bounds__(256) void outlook_fwd_kernel(const T* __restrict__ v, const T* __restrict__ logits,
                                                          T* __restrict__ y, int B, int H, int W, int C,
                                                          int heads, int ldl, int ldv) {
  constexpr int KK = KS * KS;
  constexpr int PAD = KS / 2;
  const int nch = C / V;
  const int hd = C / heads;
  const long total = (long)B * H * W * nch;
  const long tid = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (tid >= total) return;
  const int chunk = (int)(tid % nch);
  const long p = tid / nch;
  const int c0 = chunk * V;
  const int head = c0 / hd;
  const int x = (int)(p % W);
  const long t = p / W;
  const int yy = (int)(t % H);
  const long rowbase = (t / H) * H;  // b * H

  const T* lg = logits + p * ldl + head * KK;
  if constexpr (sizeof(T) == 2 && V == 8 && KS == 3) {
    // bf16 x 8 channels: every neighbour row is fetched up front (clamped addresses, so the loads
    // are unconditional and independent of the softmax), then the logits — one memory round trip
    // per thread instead of logits -> softmax -> neighbours.  Out-of-image neighbours keep their
    // softmax mass and contribute zero (the reference's zero padding); same summation order.
    uint4 raw[KK];
    bool inb[KK];
#pragma unroll
    for (int ki = 0; ki < KS; ++ki) {
      const int y2 = yy + ki - PAD;
      const int y2c = min(max(y2, 0), H - 1);
#pragma unroll
      for (int kj = 0; kj < KS; ++kj) {
        const int x2 = x + kj - PAD;
        const int x2c = min(max(x2, 0), W - 1);
        inb[ki * KS + kj] = y2 >= 0 && y2 < H && x2 >= 0 && x2 < W;
        raw[ki * KS + kj] = *reinterpret_cast<const uint4*>(v + ((rowbase + y2c) * W + x2c) * ldv + c0);
      }
    }
    float a[KK];
    float mx = -INFINITY;
#pragma unroll
    for (int j = 0; j < KK; ++j) {
      a[j] = to_f(lg[j]);
      mx = fmaxf(mx, a[j]);
    }
    float s = 0.f;
#pragma unroll
    for (int j = 0; j < KK; ++j) {
      a[j] = __expf(a[j] - mx);
      s += a[j];
    }
    const float inv = 1.0f / s;
    float acc[V];
#pragma unroll
    for (int i = 0; i < V; ++i) acc[i] = 0.f;
#pragma unroll
    for (int j = 0; j < KK; ++j) {
      if (!inb[j]) continue;
      const bf16* e = reinterpret_cast<const bf16*>(&raw[j]);
#pragma unroll
      for (int i = 0; i < V; ++i) acc[i] = fmaf(a[j], (float)e[i], acc[i]);
    }
#pragma unroll
    for (int i = 0; i < V; ++i) acc[i] *= inv;
    store_vec<T, V>(y + p * C + c0, acc);
    return;
  }
  float a[KK];
  float mx = -INFINITY;
#pragma unroll
  for (int j = 0; j < KK; ++j) {
    a[j] = to_f(lg[j]);
    mx = fmaxf(mx, a[j]);
  }
  float s = 0.f;
#pragma unroll
  for (int j = 0; j < KK; ++j) {
    a[j] = __expf(a[j] - mx);
    s += a[j];
  }
  const float inv = 1.0f / s;

  float acc[V];
#pragma unroll
  for (int i = 0; i < V; ++i) acc[i] = 0.f;
#pragma unroll
  for (int ki = 0; ki < KS; ++ki) {
    const int y2 = yy + ki - PAD;
    if (y2 < 0 || y2 >= H) continue;
#pragma unroll
    for (int kj = 0; kj < KS; ++kj) {
      const int x2 = x + kj - PAD;
      if (x2 < 0 || x2 >= W) continue;
      float tmp[V];
      load_vec<T, V>(v + ((rowbase + y2) * W + x2) * ldv + c0, tmp);
      const float w = a[ki * KS + kj];
#pragma unroll
      for (int i = 0; i < V; ++i) acc[i] = fmaf(w, tmp[i], acc[i]);
    }
  }
#pragma unroll
  for (int i = 0; i < V; ++i) acc[i] *= inv;
  store_vec<T, V>(y + p * C + c0, acc);
}

// One thread per (pixel, head): recompute P, form dP by dotting dy with each neighbour's v,
// write dlogits and P (fp32 scratch for the dv gather).
template <typename T, int V, int KS>
__global__ __launch_bounds__(256) void outlook_bwd_logits_kernel(const T* __restrict__ dy, const T* __restrict__ v,
                                                                 const T* __restrict__ logits, T* __restrict__ dlogits,
                                                                 float* __restrict__ probs, int B, int H, int W,
                                                                 int C, int heads, int ldl, int ldv, int lddl,
                                                                 int dl_cols) {
  constexpr int KK = KS * KS;
  constexpr int PAD = KS / 2;
  const int hd = C / heads;
  const long total = (long)B * H * W * heads;
  const long tid = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (tid >= total) return;
  const int head = (int)(tid % heads);
  const long p = tid / heads;
  const int x = (int)(p % W);
  const long t = p / W;
  const int yy = (int)(t % H);
  const long rowbase = (t / H) * H;

  const T* lg = logits + p * ldl + head * KK;
  float a[KK];
  float mx = -INFINITY;
#pragma unroll
  for (int j = 0; j < KK; ++j) {
    a[j] = to_f(lg[j]);
    mx = fmaxf(mx, a[j]);
  }
  float s = 0.f;
#pragma unroll
  for (int j = 0; j < KK; ++j) {
    a[j] = __expf(a[j] - mx);
    s += a[j];
  }
  const float inv = 1.0f / s;
#pragma unroll
  for (int j = 0; j < KK; ++j) a[j] *= inv;

  float dp[KK];
#pragma unroll
  for (int j = 0; j < KK; ++j) dp[j] = 0.f;
  const int cb = head * hd;
  if constexpr (sizeof(T) == 2 && V == 8 && KS == 3) {
    // per 8-channel slice: dy and all neighbour v rows issued together (clamped, unconditional)
    bool inb[KK];
    long nb[KK];
#pragma unroll
    for (int ki = 0; ki < KS; ++ki)
#pragma unroll
      for (int kj = 0; kj < KS; ++kj) {
        const int y2 = yy + ki - PAD, x2 = x + kj - PAD;
        inb[ki * KS + kj] = y2 >= 0 && y2 < H && x2 >= 0 && x2 < W;
        nb[ki * KS + kj] = ((rowbase + min(max(y2, 0), H - 1)) * W + min(max(x2, 0), W - 1)) * ldv + cb;
      }
    for (int d = 0; d < hd; d += V) {
      const uint4 graw = *reinterpret_cast<const uint4*>(dy + p * C + cb + d);
      uint4 raw[KK];
#pragma unroll
      for (int j = 0; j < KK; ++j) raw[j] = *reinterpret_cast<const uint4*>(v + nb[j] + d);
      const bf16* ge = reinterpret_cast<const bf16*>(&graw);
#pragma unroll
      for (int j = 0; j < KK; ++j) {
        if (!inb[j]) continue;
        const bf16* e = reinterpret_cast<const bf16*>(&raw[j]);
        float acc = dp[j];
#pragma unroll
        for (int i = 0; i < V; ++i) acc = fmaf((float)ge[i], (float)e[i], acc);
        dp[j] = acc;
      }
    }
  } else
  for (int d = 0; d < hd; d += V) {
    float g[V];
    load_vec<T, V>(dy + p * C + cb + d, g);
#pragma unroll
    for (int ki = 0; ki < KS; ++ki) {
      const int y2 = yy + ki - PAD;
      if (y2 < 0 || y2 >= H) continue;
#pragma unroll
      for (int kj = 0; kj < KS; ++kj) {
        const int x2 = x + kj - PAD;
        if (x2 < 0 || x2 >= W) continue;
        float tmp[V];
        load_vec<T, V>(v + ((rowbase + y2) * W + x2) * ldv + cb + d, tmp);
        float acc = dp[ki * KS + kj];
#pragma unroll
        for (int i = 0; i < V; ++i) acc = fmaf(g[i], tmp[i], acc);
        dp[ki * KS + kj] = acc;
      }
    }
  }
  float sdp = 0.f;
#pragma unroll
  for (int j = 0; j < KK; ++j) sdp = fmaf(a[j], dp[j], sdp);
  T* dl = dlogits + p * lddl + head * KK;
  float* pr = probs + (p * heads + head) * KK;
#pragma unroll
  for (int j = 0; j < KK; ++j) {
    dl[j] = from_f<T>(a[j] * (dp[j] - sdp));
    pr[j] = a[j];
  }
  if (head == heads - 1)   // padding columns of a concatenated gradient
    for (int c = heads * KK; c < dl_cols; ++c) dlogits[p * lddl + c] = from_f<T>(0.f);
}

// One thread per (pixel q, V-channel chunk): dv[q] = sum_j P[q - off_j, head, j] * dy[q - off_j].
template <typename T, int V, int KS>
__global__ __launch_bounds__(256) void outlook_bwd_v_kernel(const T* __restrict__ dy, const float* __restrict__ probs,
                                                            T* __restrict__ dv, int B, int H, int W, int C,
                                                            int heads, int lddv) {
  constexpr int KK = KS * KS;
  constexpr int PAD = KS / 2;
  const int nch = C / V;
  const int hd = C / heads;
  const long total = (long)B * H * W * nch;
  const long tid = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (tid >= total) return;
  const int chunk = (int)(tid % nch);
  const long q = tid / nch;
  const int c0 = chunk * V;
  const int head = c0 / hd;
  const int x = (int)(q % W);
  const long t = q / W;
  const int yy = (int)(t % H);
  const long rowbase = (t / H) * H;

  float acc[V];
#pragma unroll
  for (int i = 0; i < V; ++i) acc[i] = 0.f;
  if constexpr (sizeof(T) == 2 && V == 8 && KS == 3) {
    // every neighbour's dy row and probability fetched up front (clamped, unconditional), then
    // accumulated in the same order with out-of-image neighbours skipped
    uint4 raw[KK];
    float wv[KK];
    bool inb[KK];
#pragma unroll
    for (int ki = 0; ki < KS; ++ki) {
      const int y2 = yy - (ki - PAD);
      const int y2c = min(max(y2, 0), H - 1);
#pragma unroll
      for (int kj = 0; kj < KS; ++kj) {
        const int x2 = x - (kj - PAD);
        const int x2c = min(max(x2, 0), W - 1);
        const long pp = (rowbase + y2c) * W + x2c;
        inb[ki * KS + kj] = y2 >= 0 && y2 < H && x2 >= 0 && x2 < W;
        wv[ki * KS + kj] = probs[(pp * heads + head) * KK + ki * KS + kj];
        raw[ki * KS + kj] = *reinterpret_cast<const uint4*>(dy + pp * C + c0);
      }
    }
#pragma unroll
    for (int j = 0; j < KK; ++j) {
      if (!inb[j]) continue;
      const bf16* e = reinterpret_cast<const bf16*>(&raw[j]);
#pragma unroll
      for (int i = 0; i < V; ++i) acc[i] = fmaf(wv[j], (float)e[i], acc[i]);
    }
    store_vec<T, V>(dv + q * lddv + c0, acc);
    return;
  }
#pragma unroll
  for (int ki = 0; ki < KS; ++ki) {
    const int y2 = yy - (ki - PAD);
    if (y2 < 0 || y2 >= H) continue;
#pragma unroll
    for (int kj = 0; kj < KS; ++kj) {
      const int x2 = x - (kj - PAD);
      if (x2 < 0 || x2 >= W) continue;
      const long pp = (rowbase + y2) * W + x2;
      const float w = probs[(pp * heads + head) * KK + ki * KS + kj];
      float g[V];
      load_vec<T, V>(dy + pp * C + c0, g);
#pragma unroll
      for (int i = 0; i < V; ++i) acc[i] = fmaf(w, g[i], acc[i]);
    }
  }
  store_vec<T, V>(dv + q * lddv + c0, acc);
}

// ------------------------------------------------------------------------------------------------
// LDS-tiled kernels (bf16, k = 3, head_dim % 8 == 0, head_dim <= 64): the hot configurations.
// A block owns G spatial tiles of TH x TW pixels for a group of HB heads (all heads whenever the
// tiles fit in LDS, so every staged pixel is one contiguous run of its row).  The tiles' v (and
// dy) channels of the group, plus the one-pixel halo, are staged into LDS once with coalesced
// 16-B loads (zeros outside the image = the reference's zero padding), the softmax of every
// staged pixel is computed once into LDS (fp32), and the 3x3 gathers read their 9 neighbours
// from LDS instead of re-fetching them from L2 (the thread-per-chunk kernels above issue 9 global
// loads per output vector).
//   fwd: y[p]      = sum_j P[p, j] v[p + off_j]
//   bwd: dP[p, j]  = <dy[p], v[p + off_j]>,  dlogit = P (dP - sum_j P dP)     (2 threads / pixel)
//        dv[q]     = sum_j P[q - off_j, j] dy[q - off_j]                      (col2im as a gather)
// ------------------------------------------------------------------------------------------------
// a / d for 0 <= a < 2^22 by a float reciprocal and one correction (the index math of the tile
// kernels divides by runtime tile / channel counts; integer division would dominate their VALU)
struct FDiv {
  int d;
  float r;
};
static inline FDiv fdiv_make(int d) { return FDiv{d, 1.0f / (float)d}; }
__device__ __forceinline__ int fdiv(int a, const FDiv& f) {
  int q = (int)((float)a * f.r);
  const int rem = a - q * f.d;
  q += (rem >= f.d) - (rem < 0);
  return q;
}

struct OTile {
  int TH, TW, G;          // tile shape, tiles per block
  int HB;                 // heads per block
  int ntx, nty;           // tiles per image row / column
  long ntiles;            // B * nty * ntx
  FDiv per_img, fntx, fTW, fHP, fHW2, fCB8, fHBCH, fPT, fHB, fCH;
};

__device__ __forceinline__ void otile_origin(const OTile& t, long tile, int& b, int& y0, int& x0) {
  b = fdiv((int)tile, t.per_img);
  const int r = (int)tile - b * t.per_img.d;
  const int ty = fdiv(r, t.fntx);
  y0 = ty * t.TH;
  x0 = (r - ty * t.ntx) * t.TW;
}

// stage [G][(TH+2)(TW+2)][CB] of src (row stride ld, first column col) into LDS; zeros outside.
// Loads are issued in batches of OT_WB per thread before any is stored, so staging costs a couple
// of memory round trips instead of one per loop trip.
constexpr int OT_WB = 8;
__device__ __forceinline__ void otile_stage(const bf16* __restrict__ src, int ld, int col, int CB, bf16* lds,
                                            const OTile& t, long tile0, int H, int W) {
  const int CH = CB / 8;
  const int HW2 = t.TW + 2, HP = (t.TH + 2) * HW2;
  const int total = t.G * HP * CH;
  for (int base = threadIdx.x; base < total; base += OT_WB * blockDim.x) {
    uint4 val[OT_WB];
#pragma unroll
    for (int u = 0; u < OT_WB; ++u) {
      const int idx = base + u * blockDim.x;
      val[u] = uint4{0u, 0u, 0u, 0u};
      if (idx < total) {
        const int s = fdiv(idx, t.fCB8), c8 = idx - s * CH;
        const int g = t.G > 1 ? fdiv(s, t.fHP) : 0, hp = s - g * HP;
        const long tile = tile0 + g;
        if (tile < t.ntiles) {
          int b, y0, x0;
          otile_origin(t, tile, b, y0, x0);
          const int hy = fdiv(hp, t.fHW2);
          const int yy = y0 - 1 + hy, xx = x0 - 1 + hp - hy * HW2;
          if (yy >= 0 && yy < H && xx >= 0 && xx < W)
            val[u] = *reinterpret_cast<const uint4*>(src + ((long)(b * H + yy) * W + xx) * ld + col + c8 * 8);
        }
      }
    }
#pragma unroll
    for (int u = 0; u < OT_WB; ++u) {
      const int idx = base + u * blockDim.x;
      if (idx < total) *reinterpret_cast<uint4*>(lds + (long)idx * 8) = val[u];
    }
  }
}

// P[(s*HB + hb)*9 + j]: softmax over the 9 logits of staged pixel s, head hb of the group, for every
// staged pixel in the image (halo) or the tile interiors only; 0 elsewhere
__device__ __forceinline__ void otile_probs(const bf16* __restrict__ lg, int ldl, int col, float* P, const OTile& t,
                                            long tile0, int H, int W, bool halo) {
  const int HW2 = t.TW + 2, HP = (t.TH + 2) * HW2, PT = t.TH * t.TW;
  const int per = halo ? HP : PT;
  for (int idx = threadIdx.x; idx < t.G * per * t.HB; idx += blockDim.x) {
    const int q = fdiv(idx, t.fHB), hb = idx - q * t.HB;
    const int g = t.G > 1 ? fdiv(q, halo ? t.fHP : t.fPT) : 0, r = q - g * per;
    int hp = r;
    if (!halo) {
      const int ry = fdiv(r, t.fTW);
      hp = (ry + 1) * HW2 + (r - ry * t.TW) + 1;
    }
    float a[9];
    bool ok = false;
    const long tile = tile0 + g;
    if (tile < t.ntiles) {
      int b, y0, x0;
      otile_origin(t, tile, b, y0, x0);
      const int hy = fdiv(hp, t.fHW2);
      const int yy = y0 - 1 + hy, xx = x0 - 1 + hp - hy * HW2;
      if (yy >= 0 && yy < H && xx >= 0 && xx < W) {
        ok = true;
        const bf16* l = lg + ((long)(b * H + yy) * W + xx) * ldl + col + hb * 9;
        float mx = -INFINITY;
#pragma unroll
        for (int j = 0; j < 9; ++j) {
          a[j] = (float)l[j];
          mx = fmaxf(mx, a[j]);
        }
        float sm = 0.f;
#pragma unroll
        for (int j = 0; j < 9; ++j) {
          a[j] = __expf(a[j] - mx);
          sm += a[j];
        }
        const float inv = 1.0f / sm;
#pragma unroll
        for (int j = 0; j < 9; ++j) a[j] *= inv;
      }
    }
    float* dst = P + ((long)(g * HP + hp) * t.HB + hb) * 9;
#pragma unroll
    for (int j = 0; j < 9; ++j) dst[j] = ok ? a[j] : 0.f;
  }
}

// The backward's two staged tensors (v, dy) in one batched pass: both sources' loads of a batch
// are issued before any LDS store (one memory round trip per batch instead of one per tensor).
__device__ __forceinline__ void otile_stage2(const bf16* __restrict__ s1, int ld1, const bf16* __restrict__ s2, int ld2,
                                             int col, int CB, bf16* l1, bf16* l2, const OTile& t, long tile0, int H,
                                             int W) {
  const int CH = CB / 8;
  const int HW2 = t.TW + 2, HP = (t.TH + 2) * HW2;
  const int total = t.G * HP * CH;
  for (int base = threadIdx.x; base < total; base += OT_WB * blockDim.x) {
    uint4 a[OT_WB], b[OT_WB];
#pragma unroll
    for (int u = 0; u < OT_WB; ++u) {
      const int idx = base + u * blockDim.x;
      a[u] = b[u] = uint4{0u, 0u, 0u, 0u};
      if (idx < total) {
        const int sidx = fdiv(idx, t.fCB8), c8 = idx - sidx * CH;
        const int g = t.G > 1 ? fdiv(sidx, t.fHP) : 0, hp = sidx - g * HP;
        const long tile = tile0 + g;
        if (tile < t.ntiles) {
          int bi, y0, x0;
          otile_origin(t, tile, bi, y0, x0);
          const int hy = fdiv(hp, t.fHW2);
          const int yy = y0 - 1 + hy, xx = x0 - 1 + hp - hy * HW2;
          if (yy >= 0 && yy < H && xx >= 0 && xx < W) {
            const long px = (long)(bi * H + yy) * W + xx;
            a[u] = *reinterpret_cast<const uint4*>(s1 + px * ld1 + col + c8 * 8);
            b[u] = *reinterpret_cast<const uint4*>(s2 + px * ld2 + col + c8 * 8);
          }
        }
      }
    }
#pragma unroll
    for (int u = 0; u < OT_WB; ++u) {
      const int idx = base + u * blockDim.x;
      if (idx < total) {
        *reinterpret_cast<uint4*>(l1 + (long)idx * 8) = a[u];
        *reinterpret_cast<uint4*>(l2 + (long)idx * 8) = b[u];
      }
    }
  }
}

// Softmax item idx of otile_probs split in two: the logits loads (into registers, so they can be
// issued ahead of the staging loads) and the softmax + LDS store.
template <typename LT>
__device__ __forceinline__ void otile_logits_load(const LT* __restrict__ lg, int ldl, int col, const OTile& t,
                                                  long tile0, int H, int W, bool halo, int idx, float (&a)[9],
                                                  int& dst, bool& ok) {
  const int HW2 = t.TW + 2, HP = (t.TH + 2) * HW2, PT = t.TH * t.TW;
  const int per = halo ? HP : PT;
  ok = false;
  dst = -1;
  if (idx >= t.G * per * t.HB) return;
  const int q = fdiv(idx, t.fHB), hb = idx - q * t.HB;
  const int g = t.G > 1 ? fdiv(q, halo ? t.fHP : t.fPT) : 0, r = q - g * per;
  int hp = r;
  if (!halo) {
    const int ry = fdiv(r, t.fTW);
    hp = (ry + 1) * HW2 + (r - ry * t.TW) + 1;
  }
  dst = (g * HP + hp) * t.HB + hb;
  const long tile = tile0 + g;
  if (tile < t.ntiles) {
    int b, y0, x0;
    otile_origin(t, tile, b, y0, x0);
    const int hy = fdiv(hp, t.fHW2);
    const int yy = y0 - 1 + hy, xx = x0 - 1 + hp - hy * HW2;
    if (yy >= 0 && yy < H && xx >= 0 && xx < W) {
      ok = true;
      const LT* l = lg + ((long)(b * H + yy) * W + xx) * ldl + col + hb * 9;
#pragma unroll
      for (int j = 0; j < 9; ++j) a[j] = (float)l[j];
    }
  }
}
__device__ __forceinline__ void otile_probs_store(float (&a)[9], int dst, bool ok, float* P) {
  if (dst < 0) return;
  if (ok) {
    float mx = -INFINITY;
#pragma unroll
    for (int j = 0; j < 9; ++j) mx = fmaxf(mx, a[j]);
    float sm = 0.f;
#pragma unroll
    for (int j = 0; j < 9; ++j) {
      a[j] = __expf(a[j] - mx);
      sm += a[j];
    }
    const float inv = 1.0f / sm;
#pragma unroll
    for (int j = 0; j < 9; ++j) a[j] *= inv;
  }
  float* d = P + (long)dst * 9;
#pragma unroll
  for (int j = 0; j < 9; ++j) d[j] = ok ? a[j] : 0.f;
}

template <int HD>
__global__ __launch_bounds__(256) void outlook_fwd_tile_kernel(const bf16* __restrict__ v, int ldv,
                                                               const bf16* __restrict__ lg, int ldl,
                                                               bf16* __restrict__ y, int ldy, int H, int W, int heads,
                                                               OTile t) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int CH = HD / 8;
  const int ngrp = heads / t.HB, CB = t.HB * HD;
  long id;
  if (!xcd_block((t.ntiles + t.G - 1) / t.G * ngrp, id)) return;
  const int hg = (int)(id % ngrp);
  const long tile0 = (id / ngrp) * t.G;
  const int HW2 = t.TW + 2, HP = (t.TH + 2) * HW2, PT = t.TH * t.TW;
  bf16* vs = reinterpret_cast<bf16*>(smem);
  float* P = reinterpret_cast<float*>(smem + (size_t)t.G * HP * CB * 2);
  {  // logits of this thread's first two softmax items loaded ahead of the v staging loads
    float la[2][9];
    int dst[2];
    bool lok[2];
    otile_logits_load(lg, ldl, hg * t.HB * 9, t, tile0, H, W, false, threadIdx.x, la[0], dst[0], lok[0]);
    otile_logits_load(lg, ldl, hg * t.HB * 9, t, tile0, H, W, false, threadIdx.x + blockDim.x, la[1], dst[1], lok[1]);
    otile_stage(v, ldv, hg * CB, CB, vs, t, tile0, H, W);
    otile_probs_store(la[0], dst[0], lok[0], P);
    otile_probs_store(la[1], dst[1], lok[1], P);
    const int np = t.G * PT * t.HB;
    for (int idx = threadIdx.x + 2 * blockDim.x; idx < np; idx += blockDim.x) {
      float a[9];
      int d;
      bool ok;
      otile_logits_load(lg, ldl, hg * t.HB * 9, t, tile0, H, W, false, idx, a, d, ok);
      otile_probs_store(a, d, ok, P);
    }
  }
  __syncthreads();
  // register blocking along x: a thread produces RX = 4 consecutive pixels of one tile row for one
  // 8-channel chunk from a 3 x (RX+2) window of staged vectors (18 LDS reads for 4 outputs
  // instead of 36 -- the 9-fold neighbour re-read is LDS-bandwidth-bound otherwise)
  constexpr int RX = 4;
  const int TWq = (t.TW + RX - 1) / RX;
  const int items = t.G * t.TH * TWq * t.HB * CH;
  for (int idx = threadIdx.x; idx < items; idx += blockDim.x) {
    const int q = fdiv(idx, t.fHBCH), cc = idx - q * t.HB * CH;   // cc: 8-channel chunk within the group
    const int hb = cc / CH;
    const int rowq = q / TWq, xq = q - rowq * TWq;                  // (tile g, row ty), x-quad
    const int g = rowq / t.TH, ty = rowq - g * t.TH;
    const long tile = tile0 + g;
    if (tile >= t.ntiles) continue;
    int b, y0, x0;
    otile_origin(t, tile, b, y0, x0);
    if (y0 + ty >= H) continue;
    const int tx0 = xq * RX;
    const int s0 = g * HP + (ty + 1) * HW2 + tx0 + 1;   // staged index of the first output pixel
    float acc[RX][8];
#pragma unroll
    for (int r = 0; r < RX; ++r)
#pragma unroll
      for (int i = 0; i < 8; ++i) acc[r][i] = 0.f;
    float pw[RX][9];
#pragma unroll
    for (int r = 0; r < RX; ++r) {
      const float* pp = P + ((long)(s0 + r) * t.HB + hb) * 9;
#pragma unroll
      for (int j = 0; j < 9; ++j) pw[r][j] = (tx0 + r < t.TW) ? pp[j] : 0.f;
    }
#pragma unroll
    for (int ki = 0; ki < 3; ++ki)
#pragma unroll
      for (int c = 0; c < RX + 2; ++c) {   // window column c - 1 relative to the first output
        const uint4 raw = *reinterpret_cast<const uint4*>(vs + (long)(s0 + (ki - 1) * HW2 + c - 1) * CB + cc * 8);
        const bf16* e = reinterpret_cast<const bf16*>(&raw);
        float f[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) f[i] = (float)e[i];
#pragma unroll
        for (int r = 0; r < RX; ++r) {
          const int kj = c - r;             // output r sees this column as tap kj
          if (kj < 0 || kj > 2) continue;
          const float w = pw[r][ki * 3 + kj];
#pragma unroll
          for (int i = 0; i < 8; ++i) acc[r][i] = fmaf(w, f[i], acc[r][i]);
        }
      }
#pragma unroll
    for (int r = 0; r < RX; ++r)
      if (tx0 + r < t.TW && x0 + tx0 + r < W)
        store_vec<bf16, 8>(y + ((long)(b * H + y0 + ty) * W + x0 + tx0 + r) * ldy + hg * CB + cc * 8, acc[r]);
  }
}

template <int HD, typename LT = bf16>   // LT: the logits' storage type (float: the fp32-logits forward's lg)
__global__ __launch_bounds__(256) void outlook_bwd_tile_kernel(const bf16* __restrict__ dy, int lddy,
                                                               const bf16* __restrict__ v, int ldv,
                                                               const LT* __restrict__ lg, int ldl,
                                                               bf16* __restrict__ dv, int lddv, bf16* __restrict__ dl,
                                                               int lddl, int dl_cols, int H, int W, int heads,
                                                               OTile t) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int CH = HD / 8;
  const int ngrp = heads / t.HB, CB = t.HB * HD;
  long id;
  if (!xcd_block((t.ntiles + t.G - 1) / t.G * ngrp, id)) return;
  const int hg = (int)(id % ngrp);
  const long tile0 = (id / ngrp) * t.G;
  const int HW2 = t.TW + 2, HP = (t.TH + 2) * HW2, PT = t.TH * t.TW;
  bf16* vs = reinterpret_cast<bf16*>(smem);
  bf16* gs = vs + (size_t)t.G * HP * CB;
  float* P = reinterpret_cast<float*>(gs + (size_t)t.G * HP * CB);
  // prologue in one memory round trip (for up to 2 softmax items per thread): the logits of this
  // thread's first two softmax items, then v and dy, are all loaded before anything is stored
  {
    float la[2][9];
    int dst[2];
    bool lok[2];
    otile_logits_load(lg, ldl, hg * t.HB * 9, t, tile0, H, W, true, threadIdx.x, la[0], dst[0], lok[0]);
    otile_logits_load(lg, ldl, hg * t.HB * 9, t, tile0, H, W, true, threadIdx.x + blockDim.x, la[1], dst[1], lok[1]);
    otile_stage2(v, ldv, dy, lddy, hg * CB, CB, vs, gs, t, tile0, H, W);
    otile_probs_store(la[0], dst[0], lok[0], P);
    otile_probs_store(la[1], dst[1], lok[1], P);
    const int np = t.G * HP * t.HB;
    for (int idx = threadIdx.x + 2 * blockDim.x; idx < np; idx += blockDim.x) {
      float a[9];
      int d;
      bool ok;
      otile_logits_load(lg, ldl, hg * t.HB * 9, t, tile0, H, W, true, idx, a, d, ok);
      otile_probs_store(a, d, ok, P);
    }
  }
  __syncthreads();
  // dlogits: two threads per (pixel, head), each over half of the head's channels
  const int nl = t.G * PT * t.HB * 2;
  for (int idx = threadIdx.x; idx < nl; idx += blockDim.x) {
    const int half = idx & 1, r = idx >> 1;
    const int q = fdiv(r, t.fHB), hb = r - q * t.HB;
    const int g = t.G > 1 ? fdiv(q, t.fPT) : 0, pt = q - g * PT;
    const long tile = tile0 + g;
    bool ok = tile < t.ntiles;
    int b = 0, y0 = 0, x0 = 0;
    if (ok) otile_origin(t, tile, b, y0, x0);
    const int ty = fdiv(pt, t.fTW), tx = pt - ty * t.TW;
    ok = ok && y0 + ty < H && x0 + tx < W;
    const int s = g * HP + (ty + 1) * HW2 + tx + 1;
    float dp[9];
#pragma unroll
    for (int j = 0; j < 9; ++j) dp[j] = 0.f;
    for (int c8 = half; c8 < CH; c8 += 2) {
      const int c = hb * HD + c8 * 8;
      const uint4 graw = *reinterpret_cast<const uint4*>(gs + (long)s * CB + c);
      const bf16* ge = reinterpret_cast<const bf16*>(&graw);
#pragma unroll
      for (int ki = 0; ki < 3; ++ki)
#pragma unroll
        for (int kj = 0; kj < 3; ++kj) {
          const uint4 raw = *reinterpret_cast<const uint4*>(vs + (long)(s + (ki - 1) * HW2 + (kj - 1)) * CB + c);
          const bf16* e = reinterpret_cast<const bf16*>(&raw);
          float a = dp[ki * 3 + kj];
#pragma unroll
          for (int i = 0; i < 8; ++i) a = fmaf((float)ge[i], (float)e[i], a);
          dp[ki * 3 + kj] = a;
        }
    }
#pragma unroll
    for (int j = 0; j < 9; ++j) dp[j] += __shfl_xor(dp[j], 1, 64);
    if (!ok) continue;
    const float* pp = P + ((long)s * t.HB + hb) * 9;
    float sdp = 0.f;
#pragma unroll
    for (int j = 0; j < 9; ++j) sdp = fmaf(pp[j], dp[j], sdp);
    bf16* out = dl + ((long)(b * H + y0 + ty) * W + x0 + tx) * lddl;
    const int head = hg * t.HB + hb;
    if (half == 0) {
#pragma unroll
      for (int j = 0; j < 9; ++j) out[head * 9 + j] = (bf16)(pp[j] * (dp[j] - sdp));
    } else if (head == heads - 1) {
      for (int c = heads * 9; c < dl_cols; ++c) out[c] = (bf16)0.f;   // padding columns of a concatenated gradient
    }
  }
  // dv: thread per (pixel, 8-channel chunk), pulling from the 9 pixels whose window covers it
  const int nv = t.G * PT * t.HB * CH;
  for (int idx = threadIdx.x; idx < nv; idx += blockDim.x) {
    const int q = fdiv(idx, t.fHBCH), cc = idx - q * t.HB * CH;
    const int hb = cc / CH;
    const int g = t.G > 1 ? fdiv(q, t.fPT) : 0, pt = q - g * PT;
    const long tile = tile0 + g;
    if (tile >= t.ntiles) continue;
    int b, y0, x0;
    otile_origin(t, tile, b, y0, x0);
    const int ty = fdiv(pt, t.fTW), tx = pt - ty * t.TW;
    if (y0 + ty >= H || x0 + tx >= W) continue;
    const int s = g * HP + (ty + 1) * HW2 + tx + 1;
    float acc[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) acc[i] = 0.f;
#pragma unroll
    for (int ki = 0; ki < 3; ++ki)
#pragma unroll
      for (int kj = 0; kj < 3; ++kj) {
        const int src = s - (ki - 1) * HW2 - (kj - 1);   // pixel q - off_j
        const uint4 raw = *reinterpret_cast<const uint4*>(gs + (long)src * CB + cc * 8);
        const bf16* e = reinterpret_cast<const bf16*>(&raw);
        const float w = P[((long)src * t.HB + hb) * 9 + ki * 3 + kj];
#pragma unroll
        for (int i = 0; i < 8; ++i) acc[i] = fmaf(w, (float)e[i], acc[i]);
      }
    store_vec<bf16, 8>(dv + ((long)(b * H + y0 + ty) * W + x0 + tx) * lddv + hg * CB + cc * 8, acc);
  }
}

static size_t otile_lds(const OTile& t, int hd, bool bwd) {
  const size_t hp = (size_t)(t.TH + 2) * (t.TW + 2) * t.G;
  return hp * t.HB * hd * 2 * (bwd ? 2 : 1) + hp * t.HB * 9 * 4;
}

static constexpr size_t OTILE_LDS_CAP = 60 * 1024;   // within the default dynamic LDS grant

// Tile 8 x 16 (clipped to the image); all heads in one block if that fits the LDS cap, else 4-row
// tiles, else fewer heads per block; small images: several whole images per block (<= 128 px).
static OTile otile_plan(int B, int H, int W, int heads, int hd, bool bwd) {
  OTile t{};
  t.TW = W < 16 ? W : 16;
  t.G = 1;
  bool found = false;
  for (int hb = heads; hb >= 1 && !found; --hb) {
    if (heads % hb) continue;
    for (int th : {8, 4}) {
      t.TH = H < th ? H : th;
      t.HB = hb;
      if (otile_lds(t, hd, bwd) <= OTILE_LDS_CAP) {
        found = true;
        break;
      }
    }
  }
  if (!found) { t.TH = 1; t.HB = 1; }
  t.ntx = (W + t.TW - 1) / t.TW;
  t.nty = (H + t.TH - 1) / t.TH;
  t.ntiles = (long)B * t.nty * t.ntx;
  const int pt = t.TH * t.TW;
  if (t.TH == H && t.TW == W) {   // whole images: pack several per block
    t.G = pt >= 128 ? 1 : 128 / pt;
    while (t.G > 1 && otile_lds(t, hd, bwd) > OTILE_LDS_CAP) --t.G;
  }
  t.per_img = fdiv_make(t.nty * t.ntx);
  t.fntx = fdiv_make(t.ntx);
  t.fTW = fdiv_make(t.TW);
  t.fHP = fdiv_make((t.TH + 2) * (t.TW + 2));
  t.fHW2 = fdiv_make(t.TW + 2);
  t.fCB8 = fdiv_make(t.HB * hd / 8);
  t.fHBCH = fdiv_make(t.HB * hd / 8);
  t.fPT = fdiv_make(pt);
  t.fHB = fdiv_make(t.HB);
  t.fCH = fdiv_make(hd / 8);
  return t;
}

template <int HD>
static void otile_fwd_run(const bf16* v, int ldv, const bf16* lg, int ldl, bf16* y, int ldy, int H, int W, int heads,
                          const OTile& t, hipStream_t s) {
  const long nb = (t.ntiles + t.G - 1) / t.G * (heads / t.HB);
  outlook_fwd_tile_kernel<HD><<<xcd_grid(nb), 256, otile_lds(t, HD, false), s>>>(v, ldv, lg, ldl, y, ldy, H, W, heads, t);
}

template <int HD, typename LT>
static void otile_bwd_run(const bf16* dy, int lddy, const bf16* v, int ldv, const LT* lg, int ldl, bf16* dv,
                          int lddv, bf16* dl, int lddl, int dl_cols, int H, int W, int heads, const OTile& t,
                          hipStream_t s) {
  const long nb = (t.ntiles + t.G - 1) / t.G * (heads / t.HB);
  outlook_bwd_tile_kernel<HD, LT><<<xcd_grid(nb), 256, otile_lds(t, HD, true), s>>>(dy, lddy, v, ldv, lg, ldl, dv, lddv,
                                                                                    dl, lddl, dl_cols, H, W, heads, t);
}

#define OGV_OTILE_HD(FN, hd, ...)                  \
  switch (hd) {                                    \
    case 8: FN<8>(__VA_ARGS__); break;             \
    case 16: FN<16>(__VA_ARGS__); break;           \
    case 24: FN<24>(__VA_ARGS__); break;           \
    case 32: FN<32>(__VA_ARGS__); break;           \
    case 40: FN<40>(__VA_ARGS__); break;           \
    case 48: FN<48>(__VA_ARGS__); break;           \
    case 56: FN<56>(__VA_ARGS__); break;           \
    default: FN<64>(__VA_ARGS__); break;           \
  }

static bool al16p(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }
// knob "outlook_tile" (bit mask): 1 = LDS-tiled forward, 2 = LDS-tiled backward.  Default 2,
// measured (tools/bench_outlook.py, cold L2, MI355X): the tiled backward beats the two
// thread-per-chunk kernels at every Model-A shape (7M stage 0: 106 vs 144 us, 224^2 stage 0:
// 1.48 vs 2.90 ms), the tiled forward loses to the single-round-trip thread kernel (63 vs 48 us).
static int g_outlook_tile = 2;
void set_outlook_tile(int v) { g_outlook_tile = v & 3; }

static int pick_vec(int hd, int C) {
  if (hd % 8 == 0 && C % 8 == 0) return 8;
  if (hd % 4 == 0 && C % 4 == 0) return 4;
  if (hd % 2 == 0 && C % 2 == 0) return 2;
  return 1;
}

template <typename T, int V, int KS>
static void launch_fwd(const void* v, const void* lg, void* y, int B, int H, int W, int C, int heads, int ldl,
                       int ldv, hipStream_t s) {
  const long total = (long)B * H * W * (C / V);
  outlook_fwd_kernel<T, V, KS><<<cdiv(total, 256), 256, 0, s>>>((const T*)v, (const T*)lg, (T*)y, B, H, W, C, heads,
                                                                 ldl, ldv);
}

template <typename T, int V, int KS>
static void launch_bwd(const void* dy, const void* v, const void* lg, void* dv, void* dl, float* probs, int B, int H,
                       int W, int C, int heads, int ldl, int ldv, int lddv, int lddl, int dl_cols, hipStream_t s) {
  const long t1 = (long)B * H * W * heads;
  outlook_bwd_logits_kernel<T, V, KS><<<cdiv(t1, 256), 256, 0, s>>>((const T*)dy, (const T*)v, (const T*)lg, (T*)dl,
                                                                     probs, B, H, W, C, heads, ldl, ldv, lddl,
                                                                     dl_cols);
  const long t2 = (long)B * H * W * (C / V);
  outlook_bwd_v_kernel<T, V, KS><<<cdiv(t2, 256), 256, 0, s>>>((const T*)dy, probs, (T*)dv, B, H, W, C, heads, lddv);
}

#define OGV_OUTLOOK_DISPATCH_V(T, KS, FN, ...)        \
  switch (vec) {                                      \
    case 8: FN<T, 8, KS>(__VA_ARGS__); break;         \
    case 4: FN<T, 4, KS>(__VA_ARGS__); break;         \
    case 2: FN<T, 2, KS>(__VA_ARGS__); break;         \
    default: FN<T, 1, KS>(__VA_ARGS__); break;        \
  }

#define OGV_OUTLOOK_DISPATCH(FN, ...)                                     \
  do {                                                                    \
    if (dt == OGV_BF16) {                                                 \
      if (k == 3) { OGV_OUTLOOK_DISPATCH_V(bf16, 3, FN, __VA_ARGS__) }    \
      else if (k == 5) { OGV_OUTLOOK_DISPATCH_V(bf16, 5, FN, __VA_ARGS__) } \
      else if (k == 1) { OGV_OUTLOOK_DISPATCH_V(bf16, 1, FN, __VA_ARGS__) } \
      else { OGV_OUTLOOK_DISPATCH_V(bf16, 7, FN, __VA_ARGS__) }           \
    } else {                                                              \
      if (k == 3) { OGV_OUTLOOK_DISPATCH_V(float, 3, FN, __VA_ARGS__) }   \
      else if (k == 5) { OGV_OUTLOOK_DISPATCH_V(float, 5, FN, __VA_ARGS__) } \
      else if (k == 1) { OGV_OUTLOOK_DISPATCH_V(float, 1, FN, __VA_ARGS__) } \
      else { OGV_OUTLOOK_DISPATCH_V(float, 7, FN, __VA_ARGS__) }          \
    }                                                                     \
  } while (0)

static int check_args(int B, int H, int W, int C, int heads, int k, int ldl, int ldv, ogv_dtype dt, const char* who) {
  OGV_REQUIRE(B > 0 && H > 0 && W > 0 && C > 0 && heads > 0, "%s: non-positive shape", who);
  OGV_REQUIRE(C % heads == 0, "%s: dim %d not divisible by heads %d", who, C, heads);
  OGV_REQUIRE(k == 1 || k == 3 || k == 5 || k == 7, "%s: kernel_size %d unsupported (1,3,5,7)", who, k);
  OGV_REQUIRE(ldl >= heads * k * k, "%s: ld_logits %d < heads*k*k", who, ldl);
  OGV_REQUIRE(ldv >= C, "%s: ld_v %d < dim %d", who, ldv, C);
  OGV_REQUIRE(dt == OGV_F32 || dt == OGV_BF16, "%s: bad dtype", who);
  return OGV_OK;
}

// widest vector that divides the head dim and every row stride
static int pick_vec_ld(int hd, int C, int ld1, int ld2) {
  for (int v = 8; v > 1; v >>= 1)
    if (hd % v == 0 && C % v == 0 && ld1 % v == 0 && ld2 % v == 0) return v;
  return 1;
}

// the LDS-tiled path: bf16, k = 3, 8 | head_dim <= 64, 16-B aligned rows
static bool use_tile(int bit, ogv_dtype dt, int k, int hd, std::initializer_list<const void*> ptrs,
                     std::initializer_list<int> lds) {
  if (!(g_outlook_tile & bit) || dt != OGV_BF16 || k != 3 || hd % 8 != 0 || hd > 64) return false;
  for (const void* p : ptrs)
    if (!al16p(p)) return false;
  for (int l : lds)
    if (l % 8 != 0) return false;
  return true;
}

// ------------------------------------------------------------------------------------------------
// Outlooker forward fused with its v / attn projections (north star: "unfold -> per-window softmax
// -> weighted fold, fused with the v-projection"; reference src/model/outlook_attention.py:100-120).
// Input: the LayerNorm2d output x [M, C] (bf16 rows) and the concatenated projection weight
// Wc = [W_v; W_attn; 0] fp32 [ldc, C] + bias [ldc].  A workgroup owns a TH x TW pixel tile of one
// image and its one-pixel halo:
//   1. x of the (TH+2)(TW+2) halo pixels -> LDS (16-B coalesced loads, zeros outside the image);
//   2. [v | logits] = x . Wc^T + b for every halo pixel on MFMA (v_mfma_f32_16x16x32_bf16, the
//      weight as bf16 hi + lo halves like every forward GEMM of the build, staged in LDS once per
//      persistent workgroup), rounded to bf16 in place over the x tile -- the same rounding point
//      as the unfused GEMM's output; out-of-image halo pixels get v = 0 (zero padding);
//   3. interior rows of [v | logits | 0] -> cat (the tensor the backward reads: written once,
//      never read back by the forward), softmax over the 9 logits per (pixel, head) into LDS;
//   4. y = the 3x3 gather of v weighted by the softmax, entirely from LDS.
// So the forward reads x once and writes cat and y: the v / logits round trip through HBM of the
// unfused path (GEMM writes cat, aggregation re-reads it with its halo) and one launch are gone.
// The halo's projections are recomputed by the neighbouring tiles ((TH+2)(TW+2) / (TH TW) = 1.4x
// MFMA work, which is not the bound).
// ------------------------------------------------------------------------------------------------
struct VTile {
  int TH, TW, ntx, nty;
  long ntiles;
  int HP, HPr;         // halo pixels, rounded up to 16
  int XP, RP, WP;      // LDS pitches (elements): x tile, result tile, weight slab
  int ncol;            // computed output columns (16 * NJ >= C + heads * 9)
  int l32;             // the logits kept in fp32 (result-tile slots C + 2 (n - C)): the fp32-logits forward
  FDiv per_img, fntx, fHW2, fTW, fHB, fCH, fQ;
};
// bf16 slots of a result-tile row whose logit columns are fp32: C + 2 * (9 heads rounded up to 4)
static inline int vtile_l32_slots(int C, int heads) { return C + 2 * ((heads * 9 + 3) / 4 * 4); }

// waves per workgroup: 4 with two workgroups per CU (16 | C <= 64), 8 with one (C > 64: the split
// weight slab alone is 47-53 KB); 16-B x chunks per thread and tile, prefetched into registers
constexpr int VP_RX = 2;   // gather: consecutive output pixels per thread
template <int NW>
__host__ __device__ constexpr int vp_pf() { return NW == 8 ? 5 : 9; }

// LDS: [x tile | interior softmax P (aliases x once the GEMM is done)] [result tile] [W hi | lo] [bias]
// (the x tile holds HP rows: the MFMA's reads of rows HP .. HPr-1 land in the result tile and only
// feed discarded outputs; the result tile holds HP + 2 rows: the gather window's overshoot)
static size_t vtile_x_bytes(const VTile& t, int heads) {
  const size_t xb = (size_t)t.HP * t.XP * 2, pb = (size_t)t.TH * t.TW * heads * 9 * 4;
  return ((xb > pb ? xb : pb) + 15) / 16 * 16;
}
static size_t vtile_lds(const VTile& t, int heads, bool sw) {
  return vtile_x_bytes(t, heads) + (size_t)(t.HP + 2) * t.RP * 2 + (size_t)(sw ? 2 : 1) * t.ncol * t.WP * 2 +
         (size_t)t.ncol * 4;
}

// L32 (the fp32-logits form): the logit columns stay fp32 in the result tile (slots C + 2 (n - C)), the softmax
// reads them unrounded, and training writes v to `cat` ([M, ldc] bf16 rows, v only) and the logits to
// lg ([M, ldl] fp32) -- the bf16 rounding of the logits (O(1-10) values whose rounding moves the softmax)
// is gone from both the forward and the backward (which recomputes the softmax from lg)
template <int NJ, int NK, bool SW, int NW, bool L32>
__global__ __launch_bounds__(NW * 64, 8 / NW) void outlook_vproj_fwd_kernel(
    const bf16* __restrict__ x, int ldx, const float* __restrict__ Wc, int wrows, const float* __restrict__ bias,
    bf16* __restrict__ cat, int ldc, bf16* __restrict__ y, int H, int W, int C, int heads, VTile t, int xbytes,
    int dbg, float* __restrict__ lg, int ldl) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int KP = NK * 32, NCOL = NJ * 16, NT = NW * 64, VP_PF = vp_pf<NW>();
  const int XP = t.XP, RP = t.RP, WP = t.WP, HW2 = t.TW + 2, HP = t.HP;
  bf16* xs = reinterpret_cast<bf16*>(smem);                          // [HP][XP]
  float* P = reinterpret_cast<float*>(smem);                         // [TH*TW][heads][9] (after the GEMM)
  bf16* rs = reinterpret_cast<bf16*>(smem + xbytes);                 // [HP + 2][RP]: [v | logits | 0]
  bf16* ws = rs + (size_t)(t.HP + 2) * RP;                           // [hi | lo][NCOL][WP]
  float* bs = reinterpret_cast<float*>(ws + (size_t)(SW ? 2 : 1) * NCOL * WP);   // [NCOL]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int fr = lane & 15, fg = lane >> 4;
  const int hd = C / heads, CH8 = C / 8;

  // weight slab (once per persistent workgroup): rows n < wrows of Wc, columns k < C, zeros elsewhere
  for (int idx = tid; idx < NCOL * (KP / 4); idx += NT) {
    const int n = idx / (KP / 4), k = (idx - n * (KP / 4)) * 4;
    float4 w4 = float4{0.f, 0.f, 0.f, 0.f};
    if (n < wrows && k < C) w4 = *reinterpret_cast<const float4*>(Wc + (long)n * C + k);
    const bf16x4 h = {(bf16)w4.x, (bf16)w4.y, (bf16)w4.z, (bf16)w4.w};
    *reinterpret_cast<bf16x4*>(ws + n * WP + k) = h;
    if constexpr (SW) {
      const bf16x4 l = {(bf16)(w4.x - (float)h[0]), (bf16)(w4.y - (float)h[1]), (bf16)(w4.z - (float)h[2]),
                        (bf16)(w4.w - (float)h[3])};
      *reinterpret_cast<bf16x4*>(ws + (NCOL + n) * WP + k) = l;
    }
  }
  for (int n = tid; n < NCOL; n += NT) bs[n] = (bias && n < wrows) ? bias[n] : 0.f;

  const int G = gridDim.x;
  const int vid = (blockIdx.x & 7) * (G / 8) + (blockIdx.x >> 3);   // XCD-contiguous logical id
  const int NI = t.HPr / 16, PT = t.TH * t.TW;
  constexpr int KC = KP / 8;
  const int total = HP * KC;   // 16-B chunks of the x halo tile (<= VP_PF * NT, checked by the plan)
  // x halo tile of `tile` -> registers (zeros outside the image and in columns [C, KP)): issued one
  // tile ahead, so the next tile's loads are in flight during this tile's MFMA / softmax / gather
  uint4 pf[VP_PF];
  auto load_x = [&](long tile) {
    if (dbg & 16) return;
    const int b = fdiv((int)tile, t.per_img);
    const int r0 = (int)tile - b * t.per_img.d;
    const int ty0 = fdiv(r0, t.fntx);
    const int y0 = ty0 * t.TH, x0 = (r0 - ty0 * t.ntx) * t.TW;
#pragma unroll
    for (int u = 0; u < VP_PF; ++u) {
      const int idx = tid + u * NT;
      pf[u] = uint4{0u, 0u, 0u, 0u};
      if (idx < total) {
        const int hp = idx / KC, c8 = idx - hp * KC;
        const int hy = fdiv(hp, t.fHW2);
        const int yy = y0 - 1 + hy, xx = x0 - 1 + hp - hy * HW2;
        if (c8 < CH8 && yy >= 0 && yy < H && xx >= 0 && xx < W)
          pf[u] = *reinterpret_cast<const uint4*>(x + ((long)(b * H + yy) * W + xx) * ldx + c8 * 8);
      }
    }
  };
  if (vid < t.ntiles) load_x(vid);
  for (long tile = vid; tile < t.ntiles; tile += G) {
    const int b = fdiv((int)tile, t.per_img);
    const int r0 = (int)tile - b * t.per_img.d;
    const int ty0 = fdiv(r0, t.fntx);
    const int y0 = ty0 * t.TH, x0 = (r0 - ty0 * t.ntx) * t.TW;
    __syncthreads();   // the previous tile's readers of P / the result tile are done (weights staged)
    // 1. x halo tile (registers) -> xs
#pragma unroll
    for (int u = 0; u < VP_PF; ++u) {
      const int idx = tid + u * NT;
      if (idx < total) {
        const int hp = idx / KC, c8 = idx - hp * KC;
        *reinterpret_cast<uint4*>(xs + hp * XP + c8 * 8) = pf[u];
      }
    }
    __syncthreads();
    if (tile + G < t.ntiles) load_x(tile + G);
    // 2. D[n][m] = Wc[n] . x[m] (+ bias) on MFMA, fragment by fragment into the result tile;
    // out-of-image halo pixels -> 0 (the reference's zero padding of v)
    // each wave owns row blocks i = wave, wave + NW, ...: its x fragments stay in registers while
    // the NJ column blocks run as independent MFMA chains (j unrolled at compile time)
    // each wave owns row blocks i = i0 + r * NW (r < RB): their x fragments stay in registers while
    // every weight fragment is read from LDS ONCE per wave and fed to all RB row blocks
    constexpr int RB = NW == 8 ? 2 : 3;
    for (int i0 = wave; i0 < ((dbg & 1) ? 0 : NI); i0 += NW * RB) {
      bf16x8 xf[RB][NK];
#pragma unroll
      for (int r = 0; r < RB; ++r) {
        const int i = i0 + r * NW;
#pragma unroll
        for (int kt = 0; kt < NK; ++kt)
          xf[r][kt] = i < NI ? *reinterpret_cast<const bf16x8*>(xs + (i * 16 + fr) * XP + kt * 32 + fg * 8) : bf16x8{};
      }
      f32x4 acc[RB][NJ];
#pragma unroll
      for (int r = 0; r < RB; ++r)
#pragma unroll
        for (int j = 0; j < NJ; ++j) acc[r][j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
#pragma unroll
        for (int kt = 0; kt < NK; ++kt) {
          const bf16x8 wh = *reinterpret_cast<const bf16x8*>(ws + (j * 16 + fr) * WP + kt * 32 + fg * 8);
#pragma unroll
          for (int r = 0; r < RB; ++r) acc[r][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wh, xf[r][kt], acc[r][j], 0, 0, 0);
          if constexpr (SW) {
            const bf16x8 wl = *reinterpret_cast<const bf16x8*>(ws + (NCOL + j * 16 + fr) * WP + kt * 32 + fg * 8);
#pragma unroll
            for (int r = 0; r < RB; ++r)
              acc[r][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wl, xf[r][kt], acc[r][j], 0, 0, 0);
          }
        }
      }
#pragma unroll
      for (int r = 0; r < RB; ++r) {
        const int m = (i0 + r * NW) * 16 + fr;   // lane: row m, columns 16 j + 4 fg .. + 3
        if (i0 + r * NW >= NI || m >= HP) continue;
        const int hy = fdiv(m, t.fHW2);
        const int yy = y0 - 1 + hy, xx = x0 - 1 + m - hy * HW2;
        const bool inb = yy >= 0 && yy < H && xx >= 0 && xx < W;
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
          const int n = j * 16 + 4 * fg;
          const float4 b4 = *reinterpret_cast<const float4*>(bs + n);
          if (L32 && n >= C) {   // logit columns: fp32 at slots C + 2 (n - C) (pad-only groups dropped)
            if (n < C + (heads * 9 + 3) / 4 * 4)
              *reinterpret_cast<float4*>(rs + m * RP + C + 2 * (n - C)) =
                  float4{inb ? acc[r][j][0] + b4.x : 0.f, inb ? acc[r][j][1] + b4.y : 0.f,
                         inb ? acc[r][j][2] + b4.z : 0.f, inb ? acc[r][j][3] + b4.w : 0.f};
            continue;
          }
          bf16x4 o;
          o[0] = (bf16)(inb ? acc[r][j][0] + b4.x : 0.f);
          o[1] = (bf16)(inb ? acc[r][j][1] + b4.y : 0.f);
          o[2] = (bf16)(inb ? acc[r][j][2] + b4.z : 0.f);
          o[3] = (bf16)(inb ? acc[r][j][3] + b4.w : 0.f);
          *reinterpret_cast<bf16x4*>(rs + m * RP + n) = o;
        }
      }
    }
    __syncthreads();   // the result tile is complete; xs is free (P aliases it)
    // 3a. interior rows of [v | logits | 0] -> cat (the backward's input); L32: v -> cat, fp32 logits -> lg
    if (L32 && cat && !(dbg & 8)) {
      const int VC = C / 8, LQ = (heads * 9 + 3) / 4, NQ = VC + LQ;
      for (int idx = tid; idx < PT * NQ; idx += NT) {
        const int pt = idx / NQ, q = idx - pt * NQ;
        const int ty = fdiv(pt, t.fTW), tx = pt - ty * t.TW;
        if (y0 + ty >= H || x0 + tx >= W) continue;
        const int s = (ty + 1) * HW2 + tx + 1;
        const long g = (long)(b * H + y0 + ty) * W + x0 + tx;
        if (q < VC)
          *reinterpret_cast<uint4*>(cat + g * ldc + q * 8) = *reinterpret_cast<const uint4*>(rs + s * RP + q * 8);
        else
          *reinterpret_cast<uint4*>(lg + g * ldl + (q - VC) * 4) =
              *reinterpret_cast<const uint4*>(rs + s * RP + C + (q - VC) * 8);
      }
    } else if (cat && !(dbg & 8)) {
      const int LC = ldc / 8;
      for (int idx = tid; idx < PT * LC; idx += NT) {
        const int pt = idx / LC, c8 = idx - pt * LC;
        const int ty = fdiv(pt, t.fTW), tx = pt - ty * t.TW;
        if (y0 + ty >= H || x0 + tx >= W) continue;
        const int s = (ty + 1) * HW2 + tx + 1;
        *reinterpret_cast<uint4*>(cat + ((long)(b * H + y0 + ty) * W + x0 + tx) * ldc + c8 * 8) =
            *reinterpret_cast<const uint4*>(rs + s * RP + c8 * 8);
      }
    }
    // 3b. softmax of the interior pixels' logits (bf16-rounded, as the unfused path reads them)
    for (int idx = tid; idx < ((dbg & 4) ? 0 : PT * heads); idx += NT) {
      const int pt = fdiv(idx, t.fHB), hb = idx - pt * heads;
      const int ty = fdiv(pt, t.fTW), tx = pt - ty * t.TW;
      const bf16* l = rs + ((ty + 1) * HW2 + tx + 1) * RP + C + hb * 9;
      const float* l32 = reinterpret_cast<const float*>(rs + ((ty + 1) * HW2 + tx + 1) * RP + C) + hb * 9;
      float a[9], mx = -INFINITY;
#pragma unroll
      for (int jj = 0; jj < 9; ++jj) {
        a[jj] = L32 ? l32[jj] : (float)l[jj];
        mx = fmaxf(mx, a[jj]);
      }
      float sm = 0.f;
#pragma unroll
      for (int jj = 0; jj < 9; ++jj) {
        a[jj] = __expf(a[jj] - mx);
        sm += a[jj];
      }
      const float inv = 1.0f / sm;
      float* d = P + (long)idx * 9;   // idx = pt * heads + hb
#pragma unroll
      for (int jj = 0; jj < 9; ++jj) d[jj] = a[jj] * inv;
    }
    __syncthreads();
    // 4. gather: VP_RX consecutive pixels of one tile row per thread and 8-channel chunk, from a
    // 3 x (VP_RX + 2) window of result-tile vectors
    const int TWq = (t.TW + VP_RX - 1) / VP_RX;
    const int items = (dbg & 2) ? 0 : t.TH * TWq * CH8;
    for (int idx = tid; idx < items; idx += NT) {
      const int q = fdiv(idx, t.fCH), cc = idx - q * CH8;
      const int ty = fdiv(q, t.fQ), xq = q - ty * TWq;
      if (y0 + ty >= H) continue;
      const int hb = (cc * 8) / hd;
      const int tx0 = xq * VP_RX;
      const int s0 = (ty + 1) * HW2 + tx0 + 1;
      float accy[VP_RX][8];
      float pw[VP_RX][9];
#pragma unroll
      for (int r = 0; r < VP_RX; ++r) {
#pragma unroll
        for (int i = 0; i < 8; ++i) accy[r][i] = 0.f;
        const bool ok = tx0 + r < t.TW;
        const float* pp = P + ((long)(ty * t.TW + (ok ? tx0 + r : 0)) * heads + hb) * 9;
#pragma unroll
        for (int jj = 0; jj < 9; ++jj) pw[r][jj] = ok ? pp[jj] : 0.f;
      }
#pragma unroll
      for (int ki = 0; ki < 3; ++ki)
#pragma unroll
        for (int c = 0; c < VP_RX + 2; ++c) {
          const uint4 raw = *reinterpret_cast<const uint4*>(rs + (s0 + (ki - 1) * HW2 + c - 1) * RP + cc * 8);
          const bf16* e = reinterpret_cast<const bf16*>(&raw);
          float fv[8];
#pragma unroll
          for (int i = 0; i < 8; ++i) fv[i] = (float)e[i];
#pragma unroll
          for (int r = 0; r < VP_RX; ++r) {
            const int kj = c - r;
            if (kj < 0 || kj > 2) continue;
            const float w = pw[r][ki * 3 + kj];
#pragma unroll
            for (int i = 0; i < 8; ++i) accy[r][i] = fmaf(w, fv[i], accy[r][i]);
          }
        }
#pragma unroll
      for (int r = 0; r < VP_RX; ++r)
        if (tx0 + r < t.TW && x0 + tx0 + r < W)
          store_vec<bf16, 8>(y + ((long)(b * H + y0 + ty) * W + x0 + tx0 + r) * C + cc * 8, accy[r]);
    }
  }
}

// ------------------------------------------------------------------------------------------------
// The fused Outlooker forward for WIDE stages (C > 96: 7M stages 2-3, every 14M / 22M stage after
// the first; C = 128 / 192 / 256 / 384).  The [ncol x C] split weight slab no longer fits in LDS
// next to the tile (190 KB at C = 192), so the projection phase streams it:
//   * each wave's halo rows of x go straight from HBM into registers (16-B loads, zeros outside the
//     image), held across the whole projection -- no x tile in LDS;
//   * the weight [W_v; W_attn; 0] streams through LDS in chunks of CJ 16-column blocks (fp32 ->
//     bf16 hi + lo from registers, double-buffered, ONE barrier per chunk), the chunk sequence
//     running on across tiles (the weight is the same for every tile), so the next chunk's global
//     loads are always in flight during the current chunk's MFMAs;
//   * each chunk's outputs (+ bias, v = 0 outside the image) go straight into the LDS result tile,
//     rounded to bf16 exactly where the unfused GEMM rounds its output;
//   * then, as in the narrow kernel: interior rows -> cat (training), softmax per (pixel, head) into
//     its own LDS region, the 3 x 3 gather from LDS -> y.
// One workgroup of 8 waves per CU; 8 x 8 pixel tiles (a whole 8 x 8 / 4 x 4 image at 7M stages 2-3).
// ------------------------------------------------------------------------------------------------
static size_t vbig_lds(const VTile& t, int C, int heads, int CJ, bool sw) {
  const size_t rs = ((size_t)(t.HP + 2) * t.RP * 2 + 15) / 16 * 16;
  const size_t P = ((size_t)t.TH * t.TW * heads * 9 * 4 + 15) / 16 * 16;
  const size_t wbuf = (size_t)(sw ? 2 : 1) * CJ * 16 * t.WP * 2;
  return rs + P + 2 * wbuf + (size_t)t.ncol * 4;
}

constexpr int VB_NW = 8;

template <int NK, int CJ, bool SW>
__global__ __launch_bounds__(VB_NW * 64, 1) void outlook_vproj_big_fwd_kernel(
    const bf16* __restrict__ x, int ldx, const float* __restrict__ Wc, int wrows, const float* __restrict__ bias,
    bf16* __restrict__ cat, int ldc, bf16* __restrict__ y, int H, int W, int C, int heads, VTile t, int dbg) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int NT = VB_NW * 64, KP = NK * 32;
  constexpr int WCH = CJ * 16 * (KP / 4);              // float4 of one weight chunk
  constexpr int WPT = (WCH + NT - 1) / NT;             // ... per thread
  const int RP = t.RP, WP = t.WP, HW2 = t.TW + 2, HP = t.HP;
  const int NJ = t.ncol / 16, NCH = (NJ + CJ - 1) / CJ;
  bf16* rs = reinterpret_cast<bf16*>(smem);                                          // [HP + 2][RP]
  const size_t rs_b = ((size_t)(HP + 2) * RP * 2 + 15) / 16 * 16;
  float* P = reinterpret_cast<float*>(smem + rs_b);                                  // [TH*TW][heads][9]
  const size_t p_b = ((size_t)t.TH * t.TW * heads * 9 * 4 + 15) / 16 * 16;
  bf16* wbuf = reinterpret_cast<bf16*>(smem + rs_b + p_b);                           // [2][hi | lo][CJ*16][WP]
  constexpr int WSL = CJ * 16;                                                       // rows per half
  float* bs = reinterpret_cast<float*>(wbuf + (size_t)2 * (SW ? 2 : 1) * WSL * WP);  // [ncol]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int fr = lane & 15, fg = lane >> 4;
  const int hd = C / heads, CH8 = C / 8;
  for (int n = tid; n < t.ncol; n += NT) bs[n] = (bias && n < wrows) ? bias[n] : 0.f;

  const int G = gridDim.x;
  const int vid = (blockIdx.x & 7) * (G / 8) + (blockIdx.x >> 3);   // XCD-contiguous logical id
  const int NI = t.HPr / 16, PT = t.TH * t.TW;

  // ---- weight chunk ch: registers <- Wc rows [16 CJ ch, 16 CJ (ch + 1)), columns < C
  float4 wr[WPT];
  auto load_w = [&](int ch) {
#pragma unroll
    for (int u = 0; u < WPT; ++u) {
      const int idx = tid + u * NT;
      const int r = idx / (KP / 4), k = (idx - r * (KP / 4)) * 4, n = ch * WSL + r;
      wr[u] = float4{0.f, 0.f, 0.f, 0.f};
      if (idx < WCH && n < wrows && k < C) wr[u] = *reinterpret_cast<const float4*>(Wc + (long)n * C + k);
    }
  };
  auto store_w = [&](int buf) {
    bf16* hi = wbuf + (size_t)buf * (SW ? 2 : 1) * WSL * WP;
#pragma unroll
    for (int u = 0; u < WPT; ++u) {
      const int idx = tid + u * NT;
      if (idx >= WCH) continue;
      const int r = idx / (KP / 4), k = (idx - r * (KP / 4)) * 4;
      const bf16x4 h = {(bf16)wr[u].x, (bf16)wr[u].y, (bf16)wr[u].z, (bf16)wr[u].w};
      *reinterpret_cast<bf16x4*>(hi + r * WP + k) = h;
      if constexpr (SW) {
        const bf16x4 l = {(bf16)(wr[u].x - (float)h[0]), (bf16)(wr[u].y - (float)h[1]), (bf16)(wr[u].z - (float)h[2]),
                          (bf16)(wr[u].w - (float)h[3])};
        *reinterpret_cast<bf16x4*>(hi + WSL * WP + r * WP + k) = l;
      }
    }
  };
  // ---- this wave's x fragments of tile `tile` (row block i = wave): pixel (i*16 + fr), k = 32 kt + 8 fg
  bf16x8 xf[NK];
  auto load_x = [&](long tile) {
    const int b = fdiv((int)tile, t.per_img);
    const int r0 = (int)tile - b * t.per_img.d;
    const int ty0 = fdiv(r0, t.fntx);
    const int y0 = ty0 * t.TH, x0 = (r0 - ty0 * t.ntx) * t.TW;
    const int m = wave * 16 + fr;
    const int hy = fdiv(m, t.fHW2);
    const int yy = y0 - 1 + hy, xx = x0 - 1 + m - hy * HW2;
    const bool ok = wave < NI && m < HP && yy >= 0 && yy < H && xx >= 0 && xx < W && !(dbg & 16);
    const bf16* src = x + ((long)(b * H + (ok ? yy : 0)) * W + (ok ? xx : 0)) * ldx;
#pragma unroll
    for (int kt = 0; kt < NK; ++kt) {
      const int k = kt * 32 + fg * 8;
      xf[kt] = (ok && k < C) ? *reinterpret_cast<const bf16x8*>(src + k) : bf16x8{};
    }
  };

  if (vid >= t.ntiles) return;
  load_w(0);
  load_x(vid);
  store_w(0);
  int gch = 0;   // global chunk counter (buffer parity), runs on across tiles
  for (long tile = vid; tile < t.ntiles; tile += G) {
    const int b = fdiv((int)tile, t.per_img);
    const int r0 = (int)tile - b * t.per_img.d;
    const int ty0 = fdiv(r0, t.fntx);
    const int y0 = ty0 * t.TH, x0 = (r0 - ty0 * t.ntx) * t.TW;
    const bool more = tile + G < t.ntiles;
    // this wave's row block: in-image mask of its pixel
    const int m = wave * 16 + fr;
    const int hy = fdiv(m, t.fHW2);
    const int yy = y0 - 1 + hy, xx = x0 - 1 + m - hy * HW2;
    const bool inb = m < HP && yy >= 0 && yy < H && xx >= 0 && xx < W;
    for (int ch = 0; ch < NCH; ++ch, ++gch) {
      __syncthreads();   // chunk ch staged by everyone; the other buffer's readers (chunk ch - 1) are done
      const bool last = ch + 1 == NCH;
      if (!last) load_w(ch + 1);
      else if (more) load_w(0);   // the next tile's first chunk
      const bf16* hi = wbuf + (size_t)(gch & 1) * (SW ? 2 : 1) * WSL * WP;
      if (wave < NI && !(dbg & 1)) {
#pragma unroll
        for (int jj = 0; jj < CJ; ++jj) {
          const int j = ch * CJ + jj;
          if (j >= NJ) break;
          f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
          for (int kt = 0; kt < NK; ++kt) {
            const bf16x8 wh = *reinterpret_cast<const bf16x8*>(hi + (jj * 16 + fr) * WP + kt * 32 + fg * 8);
            acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wh, xf[kt], acc, 0, 0, 0);
            if constexpr (SW) {
              const bf16x8 wl = *reinterpret_cast<const bf16x8*>(hi + WSL * WP + (jj * 16 + fr) * WP + kt * 32 + fg * 8);
              acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wl, xf[kt], acc, 0, 0, 0);
            }
          }
          // lane: pixel m, columns 16 j + 4 fg .. + 3
          if (m < HP) {
            const int n = j * 16 + 4 * fg;
            const float4 b4 = *reinterpret_cast<const float4*>(bs + n);
            bf16x4 o;
            o[0] = (bf16)(inb ? acc[0] + b4.x : 0.f);
            o[1] = (bf16)(inb ? acc[1] + b4.y : 0.f);
            o[2] = (bf16)(inb ? acc[2] + b4.z : 0.f);
            o[3] = (bf16)(inb ? acc[3] + b4.w : 0.f);
            *reinterpret_cast<bf16x4*>(rs + m * RP + n) = o;
          }
        }
      }
      if (last && more) load_x(tile + G);   // xf is dead: the next tile's rows fly during cat / softmax / gather
      if (!last || more) store_w((gch + 1) & 1);
    }
    __syncthreads();   // the result tile is complete
    // interior rows of [v | logits | 0] -> cat (the backward's input)
    if (cat && !(dbg & 8)) {
      const int LC = ldc / 8;
      for (int idx = tid; idx < PT * LC; idx += NT) {
        const int pt = idx / LC, c8 = idx - pt * LC;
        const int ty = fdiv(pt, t.fTW), tx = pt - ty * t.TW;
        if (y0 + ty >= H || x0 + tx >= W) continue;
        const int s = (ty + 1) * HW2 + tx + 1;
        *reinterpret_cast<uint4*>(cat + ((long)(b * H + y0 + ty) * W + x0 + tx) * ldc + c8 * 8) =
            *reinterpret_cast<const uint4*>(rs + s * RP + c8 * 8);
      }
    }
    // softmax of the interior pixels' logits (bf16-rounded, as the unfused path reads them)
    for (int idx = tid; idx < ((dbg & 4) ? 0 : PT * heads); idx += NT) {
      const int pt = fdiv(idx, t.fHB), hb = idx - pt * heads;
      const int ty = fdiv(pt, t.fTW), tx = pt - ty * t.TW;
      const bf16* l = rs + ((ty + 1) * HW2 + tx + 1) * RP + C + hb * 9;
      float a[9], mx = -INFINITY;
#pragma unroll
      for (int jj = 0; jj < 9; ++jj) {
        a[jj] = (float)l[jj];
        mx = fmaxf(mx, a[jj]);
      }
      float sm = 0.f;
#pragma unroll
      for (int jj = 0; jj < 9; ++jj) {
        a[jj] = __expf(a[jj] - mx);
        sm += a[jj];
      }
      const float inv = 1.0f / sm;
      float* d = P + (long)idx * 9;
#pragma unroll
      for (int jj = 0; jj < 9; ++jj) d[jj] = a[jj] * inv;
    }
    __syncthreads();
    // gather: VP_RX consecutive pixels of one tile row per thread and 8-channel chunk
    const int TWq = (t.TW + VP_RX - 1) / VP_RX;
    const int items = (dbg & 2) ? 0 : t.TH * TWq * CH8;
    for (int idx = tid; idx < items; idx += NT) {
      const int q = fdiv(idx, t.fCH), cc = idx - q * CH8;
      const int ty = fdiv(q, t.fQ), xq = q - ty * TWq;
      if (y0 + ty >= H) continue;
      const int hb = (cc * 8) / hd;
      const int tx0 = xq * VP_RX;
      const int s0 = (ty + 1) * HW2 + tx0 + 1;
      float accy[VP_RX][8];
      float pw[VP_RX][9];
#pragma unroll
      for (int r = 0; r < VP_RX; ++r) {
#pragma unroll
        for (int i = 0; i < 8; ++i) accy[r][i] = 0.f;
        const bool ok = tx0 + r < t.TW;
        const float* pp = P + ((long)(ty * t.TW + (ok ? tx0 + r : 0)) * heads + hb) * 9;
#pragma unroll
        for (int jj = 0; jj < 9; ++jj) pw[r][jj] = ok ? pp[jj] : 0.f;
      }
#pragma unroll
      for (int ki = 0; ki < 3; ++ki)
#pragma unroll
        for (int c = 0; c < VP_RX + 2; ++c) {
          const uint4 raw = *reinterpret_cast<const uint4*>(rs + (s0 + (ki - 1) * HW2 + c - 1) * RP + cc * 8);
          const bf16* e = reinterpret_cast<const bf16*>(&raw);
          float fv[8];
#pragma unroll
          for (int i = 0; i < 8; ++i) fv[i] = (float)e[i];
#pragma unroll
          for (int r = 0; r < VP_RX; ++r) {
            const int kj = c - r;
            if (kj < 0 || kj > 2) continue;
            const float w = pw[r][ki * 3 + kj];
#pragma unroll
            for (int i = 0; i < 8; ++i) accy[r][i] = fmaf(w, fv[i], accy[r][i]);
          }
        }
#pragma unroll
      for (int r = 0; r < VP_RX; ++r)
        if (tx0 + r < t.TW && x0 + tx0 + r < W)
          store_vec<bf16, 8>(y + ((long)(b * H + y0 + ty) * W + x0 + tx0 + r) * C + cc * 8, accy[r]);
    }
  }
}

// ------------------------------------------------------------------------------------------------
// Outlooker backward fused with the RECOMPUTE of its v / attn projections -- the training half of
// the fused Outlooker (the forward above then writes only y: [v | logits] never reaches HBM).
// Per TH x TW tile, as the forward: x of the halo pixels -> LDS, [v | logits] = x . Wc^T + b on
// MFMA with the forward's fragments, weights and rounding point (bit-identical v / logits to what
// the forward aggregated), then the softmax of EVERY in-image halo pixel into LDS and, from LDS,
//   dP[p,h,j]      = dy[p, h, :] . v[p + off_j, h, :]
//   dlogits[p,h,j] = P[p,h,j] (dP[p,h,j] - sum_j' P[p,h,j'] dP[p,h,j'])
//   dv[q, h, :]    = sum_j P[q - off_j, h, j] dy[q - off_j, h, :]   (the col2im fold as a gather)
// (the autograd of src/model/outlook_attention.py:100-120), written as ONE gradient
// dcat = [dv | dlogits | 0] [M, ld] that the concatenated projection's dgrad and wgrad consume.
// dlogits go into the result tile's (then dead) logit columns and leave with 16-B stores.
// HBM: x and dy read (with the halo), dcat written -- the unfused pair's cat write (forward GEMM),
// cat re-read (aggregation) and cat re-read (backward) are gone.
// LDS: [x tile | P over the halo (aliases x after the MFMA)] [result tile] [dy halo tile, pitch C]
//      [W hi | lo] [bias]
// ------------------------------------------------------------------------------------------------
static size_t vtile_bwd_x_bytes(const VTile& t, int heads) {
  const size_t xb = (size_t)t.HP * t.XP * 2, pb = (size_t)t.HP * heads * 9 * 4;
  return ((xb > pb ? xb : pb) + 15) / 16 * 16;
}
static size_t vtile_bwd_lds(const VTile& t, int C, int heads, bool sw) {
  return vtile_bwd_x_bytes(t, heads) + (size_t)(t.HP + 2) * t.RP * 2 + (size_t)t.HP * C * 2 +
         (size_t)(sw ? 2 : 1) * t.ncol * t.WP * 2 + (size_t)t.ncol * 4;
}

// 16-B chunks per thread and tile of each prefetched halo tile (x, dy): 6 at 4 waves covers 8 x 16
// tiles at K <= 64 and 8 x 8 tiles at K <= 80; 5 at 8 waves covers 8 x 16 tiles at K <= 96
template <int NW>
__host__ __device__ constexpr int vp_bwd_pf() { return NW == 8 ? 5 : 6; }

template <int NJ, int NK, bool SW, int NW>
__global__ __launch_bounds__(NW * 64, 8 / NW) void outlook_vproj_bwd_kernel(
    const bf16* __restrict__ x, int ldx, const float* __restrict__ Wc, int wrows, const float* __restrict__ bias,
    const bf16* __restrict__ dy, int lddy, bf16* __restrict__ dcat, int ldc, int H, int W, int C, int heads, VTile t,
    int xbytes, int dbg) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int KP = NK * 32, NCOL = NJ * 16, NT = NW * 64, VP_PF = vp_bwd_pf<NW>();
  const int XP = t.XP, RP = t.RP, WP = t.WP, HW2 = t.TW + 2, HP = t.HP;
  bf16* xs = reinterpret_cast<bf16*>(smem);                          // [HP][XP]
  float* P = reinterpret_cast<float*>(smem);                         // [HP][heads][9] (after the GEMM)
  bf16* rs = reinterpret_cast<bf16*>(smem + xbytes);                 // [HP + 2][RP]: [v | logits | 0]
  bf16* gs = rs + (size_t)(HP + 2) * RP;                             // [HP][C]: dy with the halo
  bf16* ws = gs + (size_t)HP * C;                                    // [hi | lo][NCOL][WP]
  float* bs = reinterpret_cast<float*>(ws + (size_t)(SW ? 2 : 1) * NCOL * WP);   // [NCOL]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int fr = lane & 15, fg = lane >> 4;
  const int hd = C / heads, CH8 = C / 8, HC8 = hd / 8;

  for (int idx = tid; idx < NCOL * (KP / 4); idx += NT) {
    const int n = idx / (KP / 4), k = (idx - n * (KP / 4)) * 4;
    float4 w4 = float4{0.f, 0.f, 0.f, 0.f};
    if (n < wrows && k < C) w4 = *reinterpret_cast<const float4*>(Wc + (long)n * C + k);
    const bf16x4 h = {(bf16)w4.x, (bf16)w4.y, (bf16)w4.z, (bf16)w4.w};
    *reinterpret_cast<bf16x4*>(ws + n * WP + k) = h;
    if constexpr (SW) {
      const bf16x4 l = {(bf16)(w4.x - (float)h[0]), (bf16)(w4.y - (float)h[1]), (bf16)(w4.z - (float)h[2]),
                        (bf16)(w4.w - (float)h[3])};
      *reinterpret_cast<bf16x4*>(ws + (NCOL + n) * WP + k) = l;
    }
  }
  for (int n = tid; n < NCOL; n += NT) bs[n] = (bias && n < wrows) ? bias[n] : 0.f;

  const int G = gridDim.x;
  const int vid = (blockIdx.x & 7) * (G / 8) + (blockIdx.x >> 3);   // XCD-contiguous logical id
  const int NI = t.HPr / 16, PT = t.TH * t.TW;
  constexpr int KC = KP / 8;
  const int total = HP * KC;      // 16-B chunks of the x halo tile (<= VP_PF * NT, checked by the plan)
  const int gtotal = HP * CH8;    // ... of the dy halo tile (<= total)
  // x and dy halo tiles of `tile` -> registers, issued one tile ahead
  uint4 pf[VP_PF], pg[VP_PF];
  auto load_tile = [&](long tile) {
    if (dbg & 16) return;
    const int b = fdiv((int)tile, t.per_img);
    const int r0 = (int)tile - b * t.per_img.d;
    const int ty0 = fdiv(r0, t.fntx);
    const int y0 = ty0 * t.TH, x0 = (r0 - ty0 * t.ntx) * t.TW;
#pragma unroll
    for (int u = 0; u < VP_PF; ++u) {
      const int idx = tid + u * NT;
      pf[u] = pg[u] = uint4{0u, 0u, 0u, 0u};
      if (idx < total) {
        const int hp = idx / KC, c8 = idx - hp * KC;
        const int hy = fdiv(hp, t.fHW2);
        const int yy = y0 - 1 + hy, xx = x0 - 1 + hp - hy * HW2;
        if (c8 < CH8 && yy >= 0 && yy < H && xx >= 0 && xx < W)
          pf[u] = *reinterpret_cast<const uint4*>(x + ((long)(b * H + yy) * W + xx) * ldx + c8 * 8);
      }
      if (idx < gtotal) {
        const int hp = fdiv(idx, t.fCH), c8 = idx - hp * CH8;
        const int hy = fdiv(hp, t.fHW2);
        const int yy = y0 - 1 + hy, xx = x0 - 1 + hp - hy * HW2;
        if (yy >= 0 && yy < H && xx >= 0 && xx < W)
          pg[u] = *reinterpret_cast<const uint4*>(dy + ((long)(b * H + yy) * W + xx) * lddy + c8 * 8);
      }
    }
  };
  if (vid < t.ntiles) load_tile(vid);
  for (long tile = vid; tile < t.ntiles; tile += G) {
    const int b = fdiv((int)tile, t.per_img);
    const int r0 = (int)tile - b * t.per_img.d;
    const int ty0 = fdiv(r0, t.fntx);
    const int y0 = ty0 * t.TH, x0 = (r0 - ty0 * t.ntx) * t.TW;
    __syncthreads();   // the previous tile's readers of P / gs / the result tile are done (weights staged)
    // 1. x and dy halo tiles (registers) -> LDS
#pragma unroll
    for (int u = 0; u < VP_PF; ++u) {
      const int idx = tid + u * NT;
      if (idx < total) {
        const int hp = idx / KC, c8 = idx - hp * KC;
        *reinterpret_cast<uint4*>(xs + hp * XP + c8 * 8) = pf[u];
      }
      if (idx < gtotal) *reinterpret_cast<uint4*>(gs + (long)idx * 8) = pg[u];   // [hp][C]: idx = hp * CH8 + c8
    }
    __syncthreads();
    if (tile + G < t.ntiles) load_tile(tile + G);
    // 2. [v | logits] of every halo pixel on MFMA (the forward kernel's phase 2, same order; two row
    // blocks per weight-fragment read: the x / dy prefetch registers are live across this phase)
    constexpr int RB = 2;
    for (int i0 = wave; i0 < ((dbg & 1) ? 0 : NI); i0 += NW * RB) {
      bf16x8 xf[RB][NK];
#pragma unroll
      for (int r = 0; r < RB; ++r) {
        const int i = i0 + r * NW;
#pragma unroll
        for (int kt = 0; kt < NK; ++kt)
          xf[r][kt] = i < NI ? *reinterpret_cast<const bf16x8*>(xs + (i * 16 + fr) * XP + kt * 32 + fg * 8) : bf16x8{};
      }
      f32x4 acc[RB][NJ];
#pragma unroll
      for (int r = 0; r < RB; ++r)
#pragma unroll
        for (int j = 0; j < NJ; ++j) acc[r][j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
#pragma unroll
        for (int kt = 0; kt < NK; ++kt) {
          const bf16x8 wh = *reinterpret_cast<const bf16x8*>(ws + (j * 16 + fr) * WP + kt * 32 + fg * 8);
#pragma unroll
          for (int r = 0; r < RB; ++r) acc[r][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wh, xf[r][kt], acc[r][j], 0, 0, 0);
          if constexpr (SW) {
            const bf16x8 wl = *reinterpret_cast<const bf16x8*>(ws + (NCOL + j * 16 + fr) * WP + kt * 32 + fg * 8);
#pragma unroll
            for (int r = 0; r < RB; ++r)
              acc[r][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wl, xf[r][kt], acc[r][j], 0, 0, 0);
          }
        }
      }
#pragma unroll
      for (int r = 0; r < RB; ++r) {
        const int m = (i0 + r * NW) * 16 + fr;
        if (i0 + r * NW >= NI || m >= HP) continue;
        const int hy = fdiv(m, t.fHW2);
        const int yy = y0 - 1 + hy, xx = x0 - 1 + m - hy * HW2;
        const bool inb = yy >= 0 && yy < H && xx >= 0 && xx < W;
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
          const int n = j * 16 + 4 * fg;
          const float4 b4 = *reinterpret_cast<const float4*>(bs + n);
          bf16x4 o;
          o[0] = (bf16)(inb ? acc[r][j][0] + b4.x : 0.f);
          o[1] = (bf16)(inb ? acc[r][j][1] + b4.y : 0.f);
          o[2] = (bf16)(inb ? acc[r][j][2] + b4.z : 0.f);
          o[3] = (bf16)(inb ? acc[r][j][3] + b4.w : 0.f);
          *reinterpret_cast<bf16x4*>(rs + m * RP + n) = o;
        }
      }
    }
    __syncthreads();   // the result tile is complete; xs is free (P aliases it)
    // 3. softmax of every halo pixel's logits (0 outside the image: those pixels take no part)
    for (int idx = tid; idx < ((dbg & 4) ? 0 : HP * heads); idx += NT) {
      const int hp = fdiv(idx, t.fHB), hb = idx - hp * heads;
      const int hy = fdiv(hp, t.fHW2);
      const int yy = y0 - 1 + hy, xx = x0 - 1 + hp - hy * HW2;
      float* d = P + (long)idx * 9;   // idx = hp * heads + hb
      if (yy < 0 || yy >= H || xx < 0 || xx >= W) {
#pragma unroll
        for (int jj = 0; jj < 9; ++jj) d[jj] = 0.f;
        continue;
      }
      const bf16* l = rs + hp * RP + C + hb * 9;
      float a[9], mx = -INFINITY;
#pragma unroll
      for (int jj = 0; jj < 9; ++jj) {
        a[jj] = (float)l[jj];
        mx = fmaxf(mx, a[jj]);
      }
      float sm = 0.f;
#pragma unroll
      for (int jj = 0; jj < 9; ++jj) {
        a[jj] = __expf(a[jj] - mx);
        sm += a[jj];
      }
      const float inv = 1.0f / sm;
#pragma unroll
      for (int jj = 0; jj < 9; ++jj) d[jj] = a[jj] * inv;
    }
    __syncthreads();
    // 4a. dlogits of the interior pixels: two threads per (pixel, head), each over half of the
    // head's 8-channel chunks; the result replaces the pixel's logits in the result tile (the
    // logit columns are dead after step 3; step 4 reads only the v columns of rs)
    for (int idx = tid; idx < ((dbg & 2) ? 0 : PT * heads * 2); idx += NT) {
      const int half = idx & 1, r = idx >> 1;
      const int pt = fdiv(r, t.fHB), hb = r - pt * heads;
      const int ty = fdiv(pt, t.fTW), tx = pt - ty * t.TW;
      const bool ok = y0 + ty < H && x0 + tx < W;
      const int s = (ty + 1) * HW2 + tx + 1;
      float dp[9];
#pragma unroll
      for (int j = 0; j < 9; ++j) dp[j] = 0.f;
      for (int c8 = half; c8 < HC8; c8 += 2) {
        const int c = hb * hd + c8 * 8;
        const uint4 graw = *reinterpret_cast<const uint4*>(gs + (long)s * C + c);
        const bf16* ge = reinterpret_cast<const bf16*>(&graw);
        float g8[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) g8[i] = (float)ge[i];
#pragma unroll
        for (int ki = 0; ki < 3; ++ki)
#pragma unroll
          for (int kj = 0; kj < 3; ++kj) {
            const uint4 raw = *reinterpret_cast<const uint4*>(rs + (long)(s + (ki - 1) * HW2 + (kj - 1)) * RP + c);
            const bf16* e = reinterpret_cast<const bf16*>(&raw);
            float a = dp[ki * 3 + kj];
#pragma unroll
            for (int i = 0; i < 8; ++i) a = fmaf(g8[i], (float)e[i], a);
            dp[ki * 3 + kj] = a;
          }
      }
#pragma unroll
      for (int j = 0; j < 9; ++j) dp[j] += __shfl_xor(dp[j], 1, 64);
      if (!ok || half) continue;
      const float* pp = P + ((long)s * heads + hb) * 9;
      float sdp = 0.f;
#pragma unroll
      for (int j = 0; j < 9; ++j) sdp = fmaf(pp[j], dp[j], sdp);
      bf16* o = rs + (long)s * RP + C + hb * 9;
#pragma unroll
      for (int j = 0; j < 9; ++j) o[j] = (bf16)(pp[j] * (dp[j] - sdp));
    }
    // 4b. dv of the interior pixels: thread per (pixel, 8-channel chunk), pulling from the 9 pixels
    // whose window covers it
    for (int idx = tid; idx < ((dbg & 2) ? 0 : PT * CH8); idx += NT) {
      const int pt = fdiv(idx, t.fCH), cc = idx - pt * CH8;
      const int hb = cc / HC8;
      const int ty = fdiv(pt, t.fTW), tx = pt - ty * t.TW;
      if (y0 + ty >= H || x0 + tx >= W) continue;
      const int s = (ty + 1) * HW2 + tx + 1;
      float acc[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) acc[i] = 0.f;
#pragma unroll
      for (int ki = 0; ki < 3; ++ki)
#pragma unroll
        for (int kj = 0; kj < 3; ++kj) {
          const int src = s - (ki - 1) * HW2 - (kj - 1);   // pixel q - off_j
          const uint4 raw = *reinterpret_cast<const uint4*>(gs + (long)src * C + cc * 8);
          const bf16* e = reinterpret_cast<const bf16*>(&raw);
          const float w = P[((long)src * heads + hb) * 9 + ki * 3 + kj];
#pragma unroll
          for (int i = 0; i < 8; ++i) acc[i] = fmaf(w, (float)e[i], acc[i]);
        }
      if (!(dbg & 8)) store_vec<bf16, 8>(dcat + ((long)(b * H + y0 + ty) * W + x0 + tx) * ldc + cc * 8, acc);
    }
    __syncthreads();
    // 5. [dlogits | 0] columns of the interior rows -> dcat (16-B stores; the padding columns of the
    // result tile are exact zeros: zero weight rows and bias)
    const int LC = (ldc - C) / 8;
    for (int idx = tid; idx < ((dbg & 8) ? 0 : PT * LC); idx += NT) {
      const int pt = idx / LC, c8 = idx - pt * LC;
      const int ty = fdiv(pt, t.fTW), tx = pt - ty * t.TW;
      if (y0 + ty >= H || x0 + tx >= W) continue;
      const int s = (ty + 1) * HW2 + tx + 1;
      *reinterpret_cast<uint4*>(dcat + ((long)(b * H + y0 + ty) * W + x0 + tx) * ldc + C + c8 * 8) =
          *reinterpret_cast<const uint4*>(rs + (long)s * RP + C + c8 * 8);
    }
  }
}

// ---- LDS bank model (MI355X_MICROARCH.md, LDS table) used to pick the result tile's row pitch: a
// 16-B read (ds_read_b128) is serviced in four lane groups of 16 over 64 banks, an 8-B write
// (ds_write_b64) in four groups of 16 contiguous lanes over 32 banks; each extra distinct dword on a
// busy bank costs one cycle.  (Measured on the fused kernel before this model: 46% of its LDS
// cycles were conflict cycles, SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE.)
static int lds_group_cycles(const long* addr, int kind) {   // kind 0: ds_read_b128, 1: ds_write_b64
  static const int g128[4][16] = {{0, 1, 2, 3, 12, 13, 14, 15, 20, 21, 22, 23, 24, 25, 26, 27},
                                  {4, 5, 6, 7, 8, 9, 10, 11, 16, 17, 18, 19, 28, 29, 30, 31},
                                  {32, 33, 34, 35, 44, 45, 46, 47, 52, 53, 54, 55, 56, 57, 58, 59},
                                  {36, 37, 38, 39, 40, 41, 42, 43, 48, 49, 50, 51, 60, 61, 62, 63}};
  const int nb = kind == 0 ? 64 : 32, width = kind == 0 ? 4 : 2;
  int total = 0;
  for (int g = 0; g < 4; ++g) {
    long seen[64][8];
    int cnt[64] = {0};
    int worst = 0;
    for (int u = 0; u < 16; ++u) {
      const int lane = kind == 0 ? g128[g][u] : g * 16 + u;
      if (addr[lane] < 0) continue;
      for (int w = 0; w < width; ++w) {
        const long d = addr[lane] / 4 + w;
        const int b = (int)(d % nb);
        bool dup = false;
        for (int q = 0; q < cnt[b]; ++q) dup |= seen[b][q] == d;
        if (!dup && cnt[b] < 8) seen[b][cnt[b]++] = d;
        worst = cnt[b] > worst ? cnt[b] : worst;
      }
    }
    total += worst;
  }
  return total;
}

// LDS cycles per tile of the result-tile accesses at row pitch RP (elements): the MFMA epilogue's
// 8-B writes, the cat copy's and the gather's 16-B reads
static long vtile_rs_cycles(const VTile& t, int C, int heads, int ldc, int RP) {
  long addr[64], tot = 0;
  const int HW2 = t.TW + 2, NI = t.HPr / 16, PT = t.TH * t.TW;
  for (int i = 0; i < NI; ++i)
    for (int j = 0; j < t.ncol / 16; ++j) {
      for (int l = 0; l < 64; ++l) addr[l] = 2L * ((i * 16 + (l & 15)) * RP + j * 16 + 4 * (l >> 4));
      tot += lds_group_cycles(addr, 1);
    }
  const int LC = ldc / 8;
  for (int base = 0; base < PT * LC; base += 64) {
    for (int l = 0; l < 64; ++l) {
      const int idx = base + l;
      if (idx >= PT * LC) { addr[l] = -1; continue; }
      const int pt = idx / LC, c8 = idx % LC, ty = pt / t.TW, tx = pt % t.TW;
      addr[l] = 2L * (((ty + 1) * HW2 + tx + 1) * RP + c8 * 8);
    }
    tot += lds_group_cycles(addr, 0);
  }
  const int CH8 = C / 8, TWq = (t.TW + VP_RX - 1) / VP_RX, items = t.TH * TWq * CH8;
  for (int base = 0; base < items; base += 64)
    for (int ki = 0; ki < 3; ++ki)
      for (int c = 0; c < VP_RX + 2; ++c) {
        for (int l = 0; l < 64; ++l) {
          const int idx = base + l;
          if (idx >= items) { addr[l] = -1; continue; }
          const int q = idx / CH8, cc = idx % CH8, ty = q / TWq, tx0 = (q % TWq) * VP_RX;
          addr[l] = 2L * (((ty + 1) * HW2 + tx0 + 1 + (ki - 1) * HW2 + c - 1) * RP + cc * 8);
        }
        tot += lds_group_cycles(addr, 0);
      }
  (void)heads;
  return tot;
}

// the least-conflicted result-tile pitch (the model above), memoised per tile geometry: the search
// costs ~1 ms of host time, so it must not run on every launch
static int vtile_best_rp(const VTile& t, int C, int heads, int ldc) {
  struct Entry { int C, heads, ldc, TH, TW, l32, rp; };
  static Entry cache[64];
  static int n = 0;
  for (int i = 0; i < n; ++i)
    if (cache[i].C == C && cache[i].heads == heads && cache[i].ldc == ldc && cache[i].TH == t.TH && cache[i].TW == t.TW &&
        cache[i].l32 == t.l32)
      return cache[i].rp;
  const int rp0 = t.l32 ? std::max(t.ncol, (vtile_l32_slots(C, heads) + 7) / 8 * 8) : t.ncol;
  int rp_best = rp0;
  long best = -1;
  for (int rp = rp0; rp <= rp0 + 72; rp += 8) {
    const long c = vtile_rs_cycles(t, C, heads, ldc, rp);
    if (best < 0 || c < best) { best = c; rp_best = rp; }
  }
  if (n < 64) cache[n++] = Entry{C, heads, ldc, t.TH, t.TW, t.l32, rp_best};
  return rp_best;
}

// knob "outlook_vproj": 0 = never, 1 = inference only, 2 = also in training with the forward writing
// cat for the LDS-tiled aggregation backward (default), 3 = training with the recompute backward
// (ogv_outlook_vproj_bwd; the forward writes only y).  Measured (tools/bench_vproj.py, cold L2,
// profiles/r03_vproj_tile.log, fwd + bwd per Outlooker): 7M stage 0 unfused 91.6 + 95.7 us, fused
// with cat 89.8 + 95.7, fused + recompute 78.5 + 121.5; 7M stage 1 52.6 / 43.4 (+ 51.8 either way);
// 14M stage 0 200 / 176 (+ 230) / 155 + 265; 22M stage 0 1102 / 987 (+ 1269) / 892 + 1557 -- the
// fused forward with cat wins at every shape, the recompute backward does not yet.
static int g_outlook_vproj = 2;
void set_outlook_vproj(int v) { g_outlook_vproj = v < 0 ? 0 : (v > 3 ? 3 : v); }
// knob "vp_dbg" (timing experiments only, wrong results): skip phases of the fused kernels --
// 1 the projection MFMAs, 2 the gather (backward: dlogits + dv), 4 the softmax, 8 the cat write
// (backward: the dcat stores), 16 the x (backward: x and dy) loads
static int g_vp_dbg = 0;
void set_vp_dbg(int v) { g_vp_dbg = v; }

// shapes the fused kernels take: bf16, k = 3, 16 | C <= 96, 8 | head_dim, ldc = C + 9 heads rounded
// up to 8, 16-B aligned rows, and an LDS footprint within one CU's 160 KB.
// Tile candidates: (1) 8 x 16 pixels at two workgroups of 4 waves per CU (<= 80 KB of LDS each),
// (2) 8 x 8 at two of 4 waves, (3) 8 x 16 at one workgroup of 8 waves (<= 160 KB), (4) 8 x 8 at one
// of 8 waves; tried in the order 1, 3, 2, 4 -- measured (tools/bench_vproj.py with the knob
// "vp_tile" = n forcing candidate n, profiles/r03_vproj_tile.log): 8 x 16 at 8 waves beats 8 x 8 at
// 4 waves on every Model-A shape, forward (14M stage 0 with cat 215 -> 176 us, 22M 1262 -> 987 us)
// and backward (7M stage 0 140 -> 122 us), and 8 x 8 at 8 waves loses to both.
static int g_vp_tile = 0;
void set_vp_tile(int v) { g_vp_tile = v < 0 ? 0 : (v > 4 ? 4 : v); }

static bool vtile_plan(int B, int H, int W, int C, int heads, int k, int ldc, ogv_dtype dt, bool bwd, VTile& t,
                       int& nw, bool l32 = false) {
  if (dt != OGV_BF16 || k != 3 || B <= 0 || H <= 0 || W <= 0 || heads <= 0) return false;
  if (C % 16 != 0 || C > 96 || C % heads != 0 || (C / heads) % 8 != 0) return false;
  const int NL = heads * 9;
  if (ldc != (C + NL + 7) / 8 * 8) return false;
  const int KP = (C + 31) / 32 * 32;
  const int tws[4] = {16, 8, 16, 8};
  const size_t caps[4] = {80 * 1024, 80 * 1024, 160 * 1024, 160 * 1024};
  const int order[4] = {0, 2, 1, 3};
  bool ok = false;
  for (int i = 0; i < (g_vp_tile ? 1 : 4) && !ok; ++i) {
    const int pass = g_vp_tile ? g_vp_tile - 1 : order[i];
    t = VTile{};
    t.l32 = l32 && !bwd;
    t.TH = H < 8 ? H : 8;
    t.TW = W < tws[pass] ? W : tws[pass];
    t.ntx = (W + t.TW - 1) / t.TW;
    t.nty = (H + t.TH - 1) / t.TH;
    t.ntiles = (long)B * t.nty * t.ntx;
    t.HP = (t.TH + 2) * (t.TW + 2);
    t.HPr = (t.HP + 15) / 16 * 16;
    t.ncol = (C + NL + 15) / 16 * 16;
    // 16 B per row over 16 rows: a pitch of KP + 16 elements puts the 16 fragment rows of one lane
    // group on 16 distinct bank quads (KP = 32, 64, 96: conflict-free by the bank model)
    // (the conflict-free pitches first; if they push the tile over the LDS budget, the previous
    // pad-8 pitches -- 2-way conflicts on the fragment reads -- rather than a smaller tile)
    for (int pad = 16; pad >= 8 && !ok; pad -= 8) {
      t.XP = KP + pad;
      t.WP = KP + pad;
      t.RP = pad == 16 ? vtile_best_rp(t, C, heads, ldc)
                       : (t.l32 ? std::max(t.ncol, (vtile_l32_slots(C, heads) + 7) / 8 * 8) : t.ncol);
      nw = pass < 2 ? 4 : 8;
      const size_t lds = bwd ? vtile_bwd_lds(t, C, heads, true) : vtile_lds(t, heads, true);
      const int pf = bwd ? (nw == 8 ? vp_bwd_pf<8>() : vp_bwd_pf<4>()) : (nw == 8 ? vp_pf<8>() : vp_pf<4>());
      ok = lds <= caps[pass] && t.HP * (KP / 8) <= pf * nw * 64;
    }
  }
  if (!ok || t.ntiles >= (1L << 22) || t.ncol > 128) return false;
  t.per_img = fdiv_make(t.nty * t.ntx);
  t.fntx = fdiv_make(t.ntx);
  t.fHW2 = fdiv_make(t.TW + 2);
  t.fTW = fdiv_make(t.TW);
  t.fHB = fdiv_make(heads);
  t.fCH = fdiv_make(C / 8);
  t.fQ = fdiv_make((t.TW + VP_RX - 1) / VP_RX);
  return true;
}

static bool vproj_plan(int B, int H, int W, int C, int heads, int k, int ldc, ogv_dtype dt, VTile& t, int& nw,
                       bool l32 = false) {
  return g_outlook_vproj && vtile_plan(B, H, W, C, heads, k, ldc, dt, false, t, nw, l32);
}

template <int NJ, int NK, int NW>
static int vproj_run(const bf16* x, int ldx, const float* Wc, int wrows, const float* bias, bf16* cat, int ldc, bf16* y,
                      int H, int W, int C, int heads, const VTile& t, bool sw, hipStream_t s, float* lg = nullptr,
                      int ldl = 0) {
  const size_t lds = vtile_lds(t, heads, sw);
  const long per_cu = NW == 4 ? 2 : 1;
  const long nb = std::min<long>(t.ntiles, 256 * per_cu);
  const unsigned grid = (unsigned)((nb + 7) / 8 * 8);
  auto kern = t.l32 ? (sw ? outlook_vproj_fwd_kernel<NJ, NK, true, NW, true> : outlook_vproj_fwd_kernel<NJ, NK, false, NW, true>)
                    : (sw ? outlook_vproj_fwd_kernel<NJ, NK, true, NW, false> : outlook_vproj_fwd_kernel<NJ, NK, false, NW, false>);
  if (!lds_grant(reinterpret_cast<const void*>(kern), lds)) {
    set_error("%s: dynamic LDS grant of %zu bytes refused", "ogv_outlook_vproj_fwd", lds);
    return OGV_ERR_LAUNCH;
  }
  kern<<<grid, NW * 64, lds, s>>>(x, ldx, Wc, wrows, bias, cat, ldc, y, H, W, C, heads, t,
                                    (int)vtile_x_bytes(t, heads), g_vp_dbg, lg, ldl);
  return OGV_OK;
}

// wide stages (C > 96): the weight-streaming kernel, 8 x 8 tiles, CJ 16-column blocks per weight chunk
// (the largest that fits 160 KB with split weights: C = 128 -> 6, 192 -> 3, 256 -> 2, 384 -> 1).
// Knob "vp_big" (default 0 = the wide stages keep the unfused GEMM + aggregation; 1 = this kernel).
// Measured slower than the unfused pair at every wide Model-A shape (tools/bench_vproj.py, cold L2,
// profiles/r04_vproj_wide.log; fused with cat vs unfused, us): 7M s2 43.8 vs 34.2, 7M s3 48.2 vs 20.5,
// 14M s1 164 vs 135, s2 116 vs 80, s3 54 vs 46, 22M s1 875 vs 843, s2 641 vs 436, s3 354 vs 186 --
// every tile re-streams the whole [ncol x C] split weight through LDS (344 KB per 8 x 8 tile at C = 256:
// 2.2 GB of L2 traffic at 22M stage 2) with the chunk loads' latency exposed, while the GEMM reads it
// once per 128-row panel; so it stays opt-in.
static int g_vp_big = 0;
void set_vp_big(int v) { g_vp_big = v ? 1 : 0; }
static int vbig_cj(int nk) { return nk == 4 ? 6 : nk == 6 ? 3 : nk == 8 ? 2 : nk == 12 ? 1 : 0; }

static bool vbig_plan(int B, int H, int W, int C, int heads, int k, int ldc, ogv_dtype dt, VTile& t) {
  if (!g_outlook_vproj || !g_vp_big) return false;
  if (dt != OGV_BF16 || k != 3 || B <= 0 || H <= 0 || W <= 0 || heads <= 0) return false;
  if (C <= 96 || C % 32 != 0 || C % heads != 0 || (C / heads) % 8 != 0 || C / heads > 64) return false;
  const int cj = vbig_cj(C / 32);
  if (!cj) return false;
  const int NL = heads * 9;
  if (ldc != (C + NL + 7) / 8 * 8) return false;
  t = VTile{};
  t.TH = H < 8 ? H : 8;
  t.TW = W < 8 ? W : 8;
  t.ntx = (W + t.TW - 1) / t.TW;
  t.nty = (H + t.TH - 1) / t.TH;
  t.ntiles = (long)B * t.nty * t.ntx;
  t.HP = (t.TH + 2) * (t.TW + 2);
  t.HPr = (t.HP + 15) / 16 * 16;
  t.ncol = (C + NL + 15) / 16 * 16;
  t.RP = t.ncol + 8;
  t.WP = C + 8;   // (C + 8) / 2 dwords: an odd multiple of 4 mod 64 -> conflict-free 16-B fragment rows
  t.XP = 0;
  if (t.HPr / 16 > VB_NW || t.ntiles >= (1L << 22) || vbig_lds(t, C, heads, cj, true) > 160 * 1024) return false;
  t.per_img = fdiv_make(t.nty * t.ntx);
  t.fntx = fdiv_make(t.ntx);
  t.fHW2 = fdiv_make(t.TW + 2);
  t.fTW = fdiv_make(t.TW);
  t.fHB = fdiv_make(heads);
  t.fCH = fdiv_make(C / 8);
  t.fQ = fdiv_make((t.TW + VP_RX - 1) / VP_RX);
  return true;
}

template <int NK>
static int vbig_run(const bf16* x, int ldx, const float* Wc, int wrows, const float* bias, bf16* cat, int ldc, bf16* y,
                     int H, int W, int C, int heads, const VTile& t, bool sw, hipStream_t s) {
  constexpr int CJ = NK == 4 ? 6 : NK == 6 ? 3 : NK == 8 ? 2 : 1;
  const size_t lds = vbig_lds(t, C, heads, CJ, sw);
  const long nb = std::min<long>(t.ntiles, 256);
  const unsigned grid = (unsigned)((nb + 7) / 8 * 8);
  auto kern = sw ? outlook_vproj_big_fwd_kernel<NK, CJ, true> : outlook_vproj_big_fwd_kernel<NK, CJ, false>;
  if (!lds_grant(reinterpret_cast<const void*>(kern), lds)) {
    set_error("%s: dynamic LDS grant of %zu bytes refused", "ogv_outlook_vproj_fwd", lds);
    return OGV_ERR_LAUNCH;
  }
  kern<<<grid, VB_NW * 64, lds, s>>>(x, ldx, Wc, wrows, bias, cat, ldc, y, H, W, C, heads, t, g_vp_dbg);
  return OGV_OK;
}

// ------------------------------------------------------------------------------------------------
// The fused Outlooker forward for WIDE stages on SMALL images (7M stages 2-3: 8 x 8 / 4 x 4 pixels,
// C = 192 / 256; 14M stage 3, 22M stage 3), decomposed by HEAD instead of by pixel tile:
//   * a panel is IPP WHOLE images (RI = H*W rounded up to 16 rows each, R = IPP * RI <= 128 rows), so
//     every 3 x 3 neighbour of a panel pixel is in the panel or outside its image (zero padding):
//     no halo, no recomputed projection;
//   * a workgroup owns ONE head and a strided set of panels: its weight slice -- the head's hd rows of
//     W_v and 9 rows of W_attn (+ bias), 16 (hd + 16) x C as bf16 hi + lo -- is staged in LDS once,
//     so the weight is read from L2 once per workgroup instead of once per tile (the streaming kernel
//     above re-reads all of [W_v; W_attn] per 8 x 8 tile, which is what made it lose);
//   * per panel: the wave's x rows go straight from HBM into MFMA operand registers (16-B loads,
//     the NEXT panel's issued right after this panel's MFMAs), [v_h | logits_h] = x . W_h^T + b on
//     v_mfma_f32_16x16x32_bf16 (transposed product, weight = A operand), rounded to bf16 into an LDS
//     result tile exactly where the unfused GEMM rounds its output; the head's columns of cat (the
//     backward's input, training) are written from it, softmax over the 9 logits per pixel, and the
//     3 x 3 gather y[:, head] from LDS.
// grid = RG row groups x heads, block b -> head (b / 8) % heads, row group (b % 8) + 8 (b / 8 heads):
// all heads of a row group run on ONE XCD (b % 8), so a panel's x rows are fetched from HBM once
// into that XCD's L2 and its cat rows (whose columns the heads write piecewise) are assembled there.
// ------------------------------------------------------------------------------------------------
struct VHead {
  int RI, IPP, R, npanels, RG;
  int WP, RP;
  FDiv fRI, fW;
  int S, units;                      // units per head (head_dim / 32) and heads * S: a unit = 32 v columns of a head
  int halo, TH, TW, HWD, TX, TPI, NOUT;   // halo mode: TH x TW output tiles, (TH + 2) x HWD halo rows, HWD = TW + 2
  FDiv fHWD, fTX, fTPI, fTW;
};

// rows of the panel's LDS result tile, its softmax table and the weight slab (bf16 hi [+ lo]) + bias
static size_t vhead_lds(const VHead& t, bool sw) {
  constexpr int NCOL = 48;
  return (size_t)(sw ? 2 : 1) * NCOL * t.WP * 2 + (size_t)NCOL * 4 + ((size_t)t.R * t.RP * 2 + 15) / 16 * 16 +
         (size_t)(t.halo ? t.NOUT : t.R) * 9 * 4;
}

// A unit of work = 32 v columns of one head plus that head's 9 logit columns: NCOL = 48 slab rows
// (head_dim 64 -- 14M / 22M stage 3 -- is two units that both compute the head's logits, so the weight
// slice stays 48 x C and two workgroups fit a CU).  Two panel forms:
//   HALO = false: a panel is IPP whole images (<= 128 rows), no halo;
//   HALO = true (images of > 128 pixels: 14M stages 1-2, 22M stages 1-3): a panel is a TH x TW pixel tile
//     of one image plus its 1-pixel halo, (TH + 2) x (TW + 2) rows whose projection is computed (the halo
//     rows' again by the neighbouring tiles: ~1.3-1.5x the MFMA work, x re-read from L2) so the gather never
//     leaves the LDS tile; out-of-image halo rows are skipped by the gather (the reference's zero padding).
// L32: the fp32-logits form (as outlook_vproj_fwd_kernel's): the 9 logits stay fp32 in result-tile slots
// 32 .. 49, the softmax reads them unrounded, training writes v_u to cat ([M, ldc] bf16, v only) and the head's
// logits to lg ([M, ldl] fp32)
template <int NK, int NF, bool SW, bool HALO, int NW, bool L32>
__global__ __launch_bounds__(NW * 64, 8 / NW) void outlook_vproj_head_fwd_kernel(
    const bf16* __restrict__ x, int ldx, const float* __restrict__ Wc, const float* __restrict__ bias,
    bf16* __restrict__ cat, int ldc, bf16* __restrict__ y, int B, int H, int W, int C, int heads, VHead t, int dbg,
    float* __restrict__ lg, int ldl) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int NJ = 3, NCOL = 48, KP = NK * 32, UD = 32, UD8 = 4, NT = NW * 64;
  const int WP = t.WP, RP = t.RP, R = t.R, HW = H * W;
  bf16* ws = reinterpret_cast<bf16*>(smem);                                  // [hi | lo][NCOL][WP]
  float* bs = reinterpret_cast<float*>(ws + (size_t)(SW ? 2 : 1) * NCOL * WP);   // [NCOL]
  bf16* rs = reinterpret_cast<bf16*>(bs + NCOL);                             // [R][RP]: [v_u | logits_h | 0]
  float* P = reinterpret_cast<float*>(reinterpret_cast<char*>(rs) + ((size_t)R * RP * 2 + 15) / 16 * 16);  // [.][9]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int fr = lane & 15, fg = lane >> 4;
  const int u = (blockIdx.x >> 3) % t.units;
  const int rg = (blockIdx.x & 7) + 8 * (int)(blockIdx.x / (8 * t.units));
  const int head = t.S == 1 ? u : (u >> 1), sub = u - head * t.S;
  const int vc0 = head * (C / heads) + sub * UD;   // this unit's first v column (W_v row, cat / y column)
  // panel p -> (image, top-left pixel of its halo tile); panel-local row r -> global row (or -1)
  struct Pos { long img; int y0, x0; };
  auto pos_of = [&](int p) -> Pos {
    if constexpr (HALO) {
      const int img = fdiv(p, t.fTPI), tt = p - img * t.TPI;
      const int ty = fdiv(tt, t.fTX), tx = tt - ty * t.TX;
      return Pos{img, ty * t.TH - 1, tx * t.TW - 1};
    } else {
      return Pos{(long)p * t.IPP, 0, 0};
    }
  };
  auto grow_of = [&](const Pos& q, int r) -> long {
    if constexpr (HALO) {
      const int ly = fdiv(r, t.fHWD), lx = r - ly * t.HWD;
      const int gy = q.y0 + ly, gx = q.x0 + lx;
      return (ly < t.TH + 2 && gy >= 0 && gy < H && gx >= 0 && gx < W) ? q.img * HW + gy * W + gx : -1L;
    } else {
      const int i = fdiv(r, t.fRI), pix = r - i * t.RI;
      const long img = q.img + i;
      return (pix < HW && img < B) ? img * HW + pix : -1L;
    }
  };
  const int NFR = R / 16;   // row fragments per panel; wave w owns fragments w, w + NW, ...
  bf16x8 xf[NF][NK];
  auto load_x = [&](int p) {
    if (dbg & 16) return;
    const Pos q = pos_of(p);
#pragma unroll
    for (int i = 0; i < NF; ++i) {
      const int f = wave + NW * i;
      const long g = f < NFR ? grow_of(q, f * 16 + fr) : -1L;
      const bf16* src = x + (g < 0 ? 0L : g) * ldx + fg * 8;   // clamped: always a valid address
#pragma unroll
      for (int kt = 0; kt < NK; ++kt) {
        const bf16x8 v = (kt * 32 + fg * 8 < C) ? *reinterpret_cast<const bf16x8*>(src + kt * 32) : bf16x8{};
        xf[i][kt] = g < 0 ? bf16x8{} : v;
      }
    }
  };
  if (rg < t.npanels) load_x(rg);   // the first panel's x in flight while the weights are staged
  // weight slice of this unit: slab row n < 32 <- Wc[vc0 + n] (v), 32 <= n < 41 <- Wc[C + 9 head + n - 32]
  // (logits), zero rows above; columns >= C zero (every load issued before the first conversion)
  constexpr int WPT = (NCOL * (KP / 4) + NT - 1) / NT;
  auto wrow = [&](int n) { return n < UD ? vc0 + n : (n < UD + 9 ? C + 9 * head + n - UD : -1); };
  float4 wv[WPT];
#pragma unroll
  for (int k4 = 0; k4 < WPT; ++k4) {
    const int idx = tid + k4 * NT;
    const int n = idx / (KP / 4), k = (idx - n * (KP / 4)) * 4;
    const int row = wrow(n);
    const bool ok = idx < NCOL * (KP / 4) && row >= 0 && k < C;
    const float4 w4 = *reinterpret_cast<const float4*>(Wc + (ok ? (long)row * C + k : 0L));   // clamped address
    wv[k4] = ok ? w4 : float4{0.f, 0.f, 0.f, 0.f};
  }
#pragma unroll
  for (int k4 = 0; k4 < WPT; ++k4) {
    const int idx = tid + k4 * NT;
    if (idx >= NCOL * (KP / 4)) break;
    const int n = idx / (KP / 4), k = (idx - n * (KP / 4)) * 4;
    const float4 w4 = wv[k4];
    const bf16x4 h = {(bf16)w4.x, (bf16)w4.y, (bf16)w4.z, (bf16)w4.w};
    *reinterpret_cast<bf16x4*>(ws + n * WP + k) = h;
    if constexpr (SW) {
      const bf16x4 l = {(bf16)(w4.x - (float)h[0]), (bf16)(w4.y - (float)h[1]), (bf16)(w4.z - (float)h[2]),
                        (bf16)(w4.w - (float)h[3])};
      *reinterpret_cast<bf16x4*>(ws + (NCOL + n) * WP + k) = l;
    }
  }
  for (int n = tid; n < NCOL; n += NT) {
    const int row = wrow(n);
    bs[n] = (bias && row >= 0) ? bias[row] : 0.f;
  }
  // interior output o of a halo panel -> its halo-tile row and global row (or -1: past a ragged edge)
  auto out_of = [&](const Pos& q, int o, int& r) -> long {
    const int oy = fdiv(o, t.fTW), ox = o - oy * t.TW;
    r = (oy + 1) * t.HWD + ox + 1;
    const int gy = q.y0 + 1 + oy, gx = q.x0 + 1 + ox;
    return (gy < H && gx < W) ? q.img * HW + gy * W + gx : -1L;
  };
  const int NOUT = HALO ? t.NOUT : R;   // rows that produce output (halo: the tile's interior)
  for (int p = rg; p < t.npanels; p += t.RG) {
    const Pos q = pos_of(p);
    // 1. [v_u | logits_h] of the panel's rows on MFMA
    f32x4 acc[NF][NJ];
#pragma unroll
    for (int i = 0; i < NF; ++i)
#pragma unroll
      for (int j = 0; j < NJ; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    __syncthreads();   // weights staged (first panel) / the previous panel's gather is done with rs and P
#pragma unroll
    for (int kt = 0; kt < ((dbg & 8) ? 0 : NK); ++kt)
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        const bf16x8 wh = *reinterpret_cast<const bf16x8*>(ws + (j * 16 + fr) * WP + kt * 32 + fg * 8);
#pragma unroll
        for (int i = 0; i < NF; ++i) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wh, xf[i][kt], acc[i][j], 0, 0, 0);
        if constexpr (SW) {
          const bf16x8 wl = *reinterpret_cast<const bf16x8*>(ws + (NCOL + j * 16 + fr) * WP + kt * 32 + fg * 8);
#pragma unroll
          for (int i = 0; i < NF; ++i) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wl, xf[i][kt], acc[i][j], 0, 0, 0);
        }
      }
    if (p + t.RG < t.npanels) load_x(p + t.RG);   // in flight during the epilogue, softmax and gather
    // lane: row f * 16 + fr, columns 16 j + 4 fg .. + 3 (+ bias, rounded to bf16 as the GEMM output)
#pragma unroll
    for (int i = 0; i < NF; ++i) {
      const int f = wave + NW * i;
      if (f >= NFR) continue;
      const int m = f * 16 + fr;
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        const int n = j * 16 + 4 * fg;
        const float4 b4 = *reinterpret_cast<const float4*>(bs + n);
        if (L32 && j == NJ - 1) {   // the logit columns 32 .. 40: fp32 at slots 32 + 2 (n - 32) (44 .. 47: pad, dropped)
          if (fg < 3)
            *reinterpret_cast<float4*>(rs + m * RP + UD + 8 * fg) =
                float4{acc[i][j][0] + b4.x, acc[i][j][1] + b4.y, acc[i][j][2] + b4.z, acc[i][j][3] + b4.w};
          continue;
        }
        const bf16x4 o = {(bf16)(acc[i][j][0] + b4.x), (bf16)(acc[i][j][1] + b4.y), (bf16)(acc[i][j][2] + b4.z),
                          (bf16)(acc[i][j][3] + b4.w)};
        *reinterpret_cast<bf16x4*>(rs + m * RP + n) = o;
      }
    }
    __syncthreads();
    // 2a. the unit's columns of cat (training): v_u as 16-B rows, the head's 9 logits (first unit) as bf16 elements
    if (cat) {
      for (int idx = tid; idx < ((dbg & 2) ? 0 : NOUT * UD8); idx += NT) {
        const int o = idx >> 2, c8 = idx & 3;
        int r = o;
        const long g = HALO ? out_of(q, o, r) : grow_of(q, o);
        if (g >= 0)
          *reinterpret_cast<uint4*>(cat + g * ldc + vc0 + c8 * 8) = *reinterpret_cast<const uint4*>(rs + r * RP + c8 * 8);
      }
      if (sub == 0)
        for (int idx = tid; idx < ((dbg & 1) ? 0 : NOUT * 9); idx += NT) {
          const int o = idx / 9, jj = idx - o * 9;
          int r = o;
          const long g = HALO ? out_of(q, o, r) : grow_of(q, o);
          if (g < 0) continue;
          if constexpr (L32) lg[g * ldl + 9 * head + jj] = reinterpret_cast<const float*>(rs + r * RP + UD)[jj];
          else cat[g * ldc + C + 9 * head + jj] = rs[r * RP + UD + jj];
        }
      const int pad = ldc - C - 9 * heads;   // the zero columns of [v | logits | 0] (the last unit's)
      if (!L32 && u == t.units - 1)
        for (int idx = tid; idx < NOUT * pad; idx += NT) {
          const int o = idx / pad, jj = idx - o * pad;
          int r = o;
          const long g = HALO ? out_of(q, o, r) : grow_of(q, o);
          if (g >= 0) cat[g * ldc + C + 9 * heads + jj] = (bf16)0.f;
        }
    }
    // 2b. softmax over the 9 (bf16-rounded) logits of every output pixel of the panel
    for (int o = tid; o < NOUT; o += NT) {
      int r = o;
      if constexpr (HALO) out_of(q, o, r);
      const bf16* l = rs + r * RP + UD;
      float a[9], mx = -INFINITY;
#pragma unroll
      for (int jj = 0; jj < 9; ++jj) {
        a[jj] = L32 ? reinterpret_cast<const float*>(l)[jj] : (float)l[jj];
        mx = fmaxf(mx, a[jj]);
      }
      float sm = 0.f;
#pragma unroll
      for (int jj = 0; jj < 9; ++jj) {
        a[jj] = __expf(a[jj] - mx);
        sm += a[jj];
      }
      const float inv = 1.0f / sm;
#pragma unroll
      for (int jj = 0; jj < 9; ++jj) P[o * 9 + jj] = a[jj] * inv;
    }
    __syncthreads();
    // 3. y[:, unit] = 3 x 3 gather of v_u weighted by the softmax (out-of-image neighbours: v = 0)
    for (int idx = tid; idx < ((dbg & 4) ? 0 : NOUT * UD8); idx += NT) {
      const int o = idx >> 2, cc = idx & 3;
      int r = o;
      const long g = HALO ? out_of(q, o, r) : grow_of(q, o);
      if (g < 0) continue;
      int yy, xx, rbase, rstride;   // global pixel; the halo-tile row of the (-1, -1) neighbour and the row stride
      if constexpr (HALO) {
        const int oy = fdiv(o, t.fTW), ox = o - oy * t.TW;
        yy = q.y0 + 1 + oy;
        xx = q.x0 + 1 + ox;
        rbase = oy * t.HWD + ox;
        rstride = t.HWD;
      } else {
        const int i = fdiv(o, t.fRI), pix = o - i * t.RI;
        yy = fdiv(pix, t.fW);
        xx = pix - yy * W;
        rbase = i * t.RI + (yy - 1) * W + (xx - 1);
        rstride = W;
      }
      float accy[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) accy[e] = 0.f;
#pragma unroll
      for (int ki = 0; ki < 3; ++ki)
#pragma unroll
        for (int kj = 0; kj < 3; ++kj) {
          const int ny = yy + ki - 1, nx = xx + kj - 1;
          if (ny < 0 || ny >= H || nx < 0 || nx >= W) continue;
          const float w = P[o * 9 + ki * 3 + kj];
          const uint4 raw = *reinterpret_cast<const uint4*>(rs + (rbase + ki * rstride + kj) * RP + cc * 8);
          const bf16* e8 = reinterpret_cast<const bf16*>(&raw);
#pragma unroll
          for (int e = 0; e < 8; ++e) accy[e] = fmaf(w, (float)e8[e], accy[e]);
        }
      store_vec<bf16, 8>(y + g * C + vc0 + cc * 8, accy);
    }
  }
}

// knob "vp_head" (default 1): the per-head kernel above for the wide stages it plans (whole-image panels for
// images of <= 128 pixels, halo tiles above); 2: also head_dim 64 (two 32-column units per head; the round-5
// form with one 80-row slab per head measured slower than the unfused pair, 86 vs 48 us at 14M stage 3,
// profiles/r05b_vph.log); 0: off.  "vph_rows": target rows per whole-image panel (<= 128)
static int g_vp_head = 1;
void set_vp_head(int v) { g_vp_head = v < 0 ? 0 : (v > 3 ? 3 : v); }
// (0 = auto: 128 for images of <= 32 pixels, 64 otherwise -- measured, tools/bench_vproj.py cold L2,
// profiles/r05c_vph.log: 7M stage 3 (4 x 4) 21.2 -> 19.4 us at 128 rows, stage 2 (8 x 8) 34.6 vs 41.9 us at 64)
static int g_vph_rows = 0;
void set_vph_rows(int v) { g_vph_rows = v <= 0 ? 0 : (v < 16 ? 16 : (v > 128 ? 128 : v)); }
// "vph_wgs": workgroups per CU the grid is sized for (default 3, as many as the LDS allows below that); "vph_dbg" (timing only, wrong results):
// skip 1 the cat logit stores, 2 the cat v stores, 4 the gather, 8 the MFMAs, 16 the x loads
static int g_vph_wgs = 3;
void set_vph_wgs(int v) { g_vph_wgs = v < 1 ? 1 : (v > 8 ? 8 : v); }
static int g_vph_dbg = 0;
void set_vph_dbg(int v) { g_vph_dbg = v; }
// "vph_halo": the halo-tile form -- 0 (default) off (images > 128 pixels keep the unfused pair); 1 where a pixel's
// x is re-read by at most 4 units (C = 128: 14M / 22M stage 1); 2 every wide shape; 3 every wide shape with 8-wave
// workgroups (tiles of <= 384 computed rows instead of 192).  Measured (tools/bench_vproj.py, cold L2,
// profiles/r06b_vproj_halo.log, fused_train vs the unfused GEMM + aggregation): 4 units 137.5 vs 139.6 us (14M
// stage 1), 786 vs 840 us (22M stage 1); 8 units 111 vs 87 us (14M stage 2), 631 vs 444 us (22M stage 2); 12 units
// (head_dim 64 as two units) 92 vs 48 us, 608 (438 with 8 waves) vs 188 us.  Phase what-ifs at 22M stage 2
// (vph_dbg, r06c): no x loads and no MFMAs 296 us -- the per-panel phases (cat / y stores, softmax, gather, three
// barriers) alone take 2/3 of the unfused pair's time once every pixel is visited by 8 workgroups.
// "vph_tile" (TH * 100 + TW, 0 = auto): force a halo tile
// Default 0: at the step level the 4-unit form measured no gain (14M 43.31 / 43.46 ms off vs 43.60 / 43.55 on,
// 22M 340.5 / 338.8 vs 339.5 / 339.5 ms, profiles/r06d_halo_step.log), so it stays opt-in.
static int g_vph_halo = 0;
void set_vph_halo(int v) { g_vph_halo = v < 0 ? 0 : (v > 3 ? 3 : v); }
static int g_vph_tile = 0;
void set_vph_tile(int v) { g_vph_tile = v < 0 ? 0 : v; }

// the halo tile with the fewest computed rows per output pixel (ragged edge tiles counted whole), R <= rmax
static bool vhead_halo_tile(int H, int W, int rmax, int& TH, int& TW) {
  if (g_vph_tile) {
    TH = g_vph_tile / 100;
    TW = g_vph_tile % 100;
    return TH >= 1 && TW >= 1 && ((TH + 2) * (TW + 2) + 15) / 16 * 16 <= rmax;
  }
  double best = 1e30;
  TH = TW = 0;
  for (int tw = 4; tw <= 62 && tw <= W + 2; tw += 2)
    for (int th = 1; th <= 32; ++th) {
      const int rr = ((th + 2) * (tw + 2) + 15) / 16 * 16;
      if (rr > rmax) break;
      const double tiles = (double)((H + th - 1) / th) * ((W + tw - 1) / tw);
      const double cost = tiles * rr / ((double)H * W) + 1e-3 * tiles;   // rows computed per pixel, then fewer tiles
      if (cost < best) { best = cost; TH = th; TW = tw; }
    }
  return TH > 0;
}

static bool vhead_plan(int B, int H, int W, int C, int heads, int k, int ldc, ogv_dtype dt, VHead& t, int& nw) {
  if (!g_outlook_vproj || !g_vp_head) return false;
  if (dt != OGV_BF16 || k != 3 || B <= 0 || H <= 0 || W <= 0 || heads <= 0) return false;
  if (C % 32 != 0 || !vbig_cj(C / 32) || C % heads != 0) return false;   // C in {128, 192, 256, 384}
  const int hd = C / heads;
  if (hd != 32 && !(hd == 64 && g_vp_head >= 2)) return false;
  if (ldc != (C + heads * 9 + 7) / 8 * 8) return false;
  const int HW = H * W;
  t = VHead{};
  t.S = hd / 32;
  t.units = heads * t.S;
  t.RI = (HW + 15) / 16 * 16;
  nw = 4;
  if (t.RI <= 128) {
    const int rows = g_vph_rows ? g_vph_rows : (t.RI <= 32 ? 128 : 64);
    t.IPP = rows / t.RI < 1 ? 1 : rows / t.RI;
    t.R = t.IPP * t.RI;
    t.npanels = (B + t.IPP - 1) / t.IPP;
  } else {
    if (!g_vph_halo || (g_vph_halo == 1 && t.units > 4)) return false;
    nw = g_vph_halo == 3 ? 8 : 4;
    int TH, TW;
    if (!vhead_halo_tile(H, W, 48 * nw, TH, TW)) return false;
    t.halo = 1;
    t.TH = TH;
    t.TW = TW;
    t.HWD = TW + 2;
    t.TX = (W + TW - 1) / TW;
    t.TPI = t.TX * ((H + TH - 1) / TH);
    t.NOUT = TH * TW;
    t.R = ((TH + 2) * t.HWD + 15) / 16 * 16;
    if ((long)B * t.TPI >= (1L << 22)) return false;
    t.npanels = B * t.TPI;
    t.fHWD = fdiv_make(t.HWD);
    t.fTX = fdiv_make(t.TX);
    t.fTPI = fdiv_make(t.TPI);
    t.fTW = fdiv_make(TW);
  }
  t.WP = C + 8;      // (C + 8) / 2 dwords per row: 16 fragment rows on distinct bank quads
  t.RP = 48 + 8;
  const size_t lds = vhead_lds(t, true);
  if (lds > 160 * 1024) return false;
  const int fit = (int)((160 * 1024) / lds);
  const int want = nw == 8 ? (g_vph_wgs + 1) / 2 : g_vph_wgs;
  const int per_cu = want < fit ? want : fit;
  int rg = (256 * per_cu / t.units) / 8 * 8;
  const int np8 = (t.npanels + 7) / 8 * 8;
  t.RG = rg < 8 ? 8 : (rg > np8 ? np8 : rg);
  if ((long)t.RG * t.units >= (1L << 24)) return false;
  t.fRI = fdiv_make(t.RI);
  t.fW = fdiv_make(W);
  return true;
}

template <int NK, int NF, bool HALO, int NW>
static int vhead_run(const bf16* x, int ldx, const float* Wc, const float* bias, bf16* cat, int ldc, bf16* y, int B,
                      int H, int W, int C, int heads, const VHead& t, bool sw, hipStream_t s, float* lg, int ldl,
                      bool l32) {
  const size_t lds = vhead_lds(t, sw);
  auto kern = l32 ? (sw ? outlook_vproj_head_fwd_kernel<NK, NF, true, HALO, NW, true>
                        : outlook_vproj_head_fwd_kernel<NK, NF, false, HALO, NW, true>)
                  : (sw ? outlook_vproj_head_fwd_kernel<NK, NF, true, HALO, NW, false>
                        : outlook_vproj_head_fwd_kernel<NK, NF, false, HALO, NW, false>);
  if (!lds_grant(reinterpret_cast<const void*>(kern), lds)) {
    set_error("%s: dynamic LDS grant of %zu bytes refused", "ogv_outlook_vproj_fwd", lds);
    return OGV_ERR_LAUNCH;
  }
  kern<<<(unsigned)(t.RG * t.units), NW * 64, lds, s>>>(x, ldx, Wc, bias, cat, ldc, y, B, H, W, C, heads, t, g_vph_dbg,
                                                          lg, ldl);
  return OGV_OK;
}

template <int NK>
static int vhead_dispatch(const bf16* x, int ldx, const float* Wc, const float* bias, bf16* cat, int ldc, bf16* y,
                          int B, int H, int W, int C, int heads, const VHead& t, int nw, bool sw, hipStream_t s,
                          float* lg, int ldl, bool l32) {
  if (t.halo)
    return nw == 8 ? vhead_run<NK, 3, true, 8>(x, ldx, Wc, bias, cat, ldc, y, B, H, W, C, heads, t, sw, s, lg, ldl, l32)
                   : vhead_run<NK, 3, true, 4>(x, ldx, Wc, bias, cat, ldc, y, B, H, W, C, heads, t, sw, s, lg, ldl, l32);
  return t.R > 64 ? vhead_run<NK, 2, false, 4>(x, ldx, Wc, bias, cat, ldc, y, B, H, W, C, heads, t, sw, s, lg, ldl, l32)
                  : vhead_run<NK, 1, false, 4>(x, ldx, Wc, bias, cat, ldc, y, B, H, W, C, heads, t, sw, s, lg, ldl, l32);
}

static bool vproj_bwd_plan(int B, int H, int W, int C, int heads, int k, int ldc, ogv_dtype dt, VTile& t, int& nw) {
  return vtile_plan(B, H, W, C, heads, k, ldc, dt, true, t, nw);
}

template <int NJ, int NK, int NW>
static int vproj_bwd_run(const bf16* x, int ldx, const float* Wc, int wrows, const float* bias, const bf16* dy,
                          bf16* dcat, int ldc, int H, int W, int C, int heads, const VTile& t, bool sw, hipStream_t s) {
  const size_t lds = vtile_bwd_lds(t, C, heads, sw);
  const long per_cu = NW == 4 ? 2 : 1;
  const long nb = std::min<long>(t.ntiles, 256 * per_cu);
  const unsigned grid = (unsigned)((nb + 7) / 8 * 8);
  auto kern = sw ? outlook_vproj_bwd_kernel<NJ, NK, true, NW> : outlook_vproj_bwd_kernel<NJ, NK, false, NW>;
  if (!lds_grant(reinterpret_cast<const void*>(kern), lds)) {
    set_error("%s: dynamic LDS grant of %zu bytes refused", "ogv_outlook_vproj_bwd", lds);
    return OGV_ERR_LAUNCH;
  }
  kern<<<grid, NW * 64, lds, s>>>(x, ldx, Wc, wrows, bias, dy, C, dcat, ldc, H, W, C, heads, t,
                                    (int)vtile_bwd_x_bytes(t, heads), g_vp_dbg);
  return OGV_OK;
}

}  // namespace ogv

using namespace ogv;

extern "C" int ogv_outlook_vproj_supported(int B, int H, int W, int C, int heads, int k, int ldc, int train,
                                           ogv_dtype dt) {
  VTile t;
  if (g_outlook_vproj < (train ? 2 : 1) || !lds_160k()) return 0;   // every fused variant may need > 64 KB
  int nw = 0;
  VHead th;
  int thw = 4;
  if (vhead_plan(B, H, W, C, heads, k, ldc, dt, th, thw)) return 1;   // wide stages: the per-head kernel
  if (vbig_plan(B, H, W, C, heads, k, ldc, dt, t)) return 1;   // wide stages: forward with cat, tiled backward
  if (!vproj_plan(B, H, W, C, heads, k, ldc, dt, t, nw)) return 0;
  if (!train || g_outlook_vproj < 3) return 1;
  return vproj_bwd_plan(B, H, W, C, heads, k, ldc, dt, t, nw) ? 2 : 1;
}

extern "C" int ogv_outlook_vproj_bwd_supported(int B, int H, int W, int C, int heads, int k, int ldc, ogv_dtype dt) {
  VTile t;
  int nw = 0;
  return lds_160k() && vproj_bwd_plan(B, H, W, C, heads, k, ldc, dt, t, nw) ? 1 : 0;
}

extern "C" int ogv_outlook_vproj_bwd(const void* x, int ldx, const float* w, const float* bias, const void* dy,
                                     void* dcat, int ldc, int B, int H, int W, int C, int heads, int k, ogv_dtype dt,
                                     void* stream) {
  if (skip_mask() & 64) return OGV_OK;
  OGV_REQUIRE(x && w && dy && dcat, "ogv_outlook_vproj_bwd: null pointer");
  int rc = check_args(B, H, W, C, heads, k, heads * k * k, C, dt, "ogv_outlook_vproj_bwd");
  if (rc) return rc;
  VTile t;
  int nw = 0;
  OGV_REQUIRE(vproj_bwd_plan(B, H, W, C, heads, k, ldc, dt, t, nw),
              "ogv_outlook_vproj_bwd: unsupported shape (needs bf16, k=3, 16 | C <= 96, 8 | head_dim, "
              "ldc = C + 9*heads rounded up to 8; see ogv_outlook_vproj_supported)");
  OGV_REQUIRE(ldx >= C && ldx % 8 == 0 && al16p(x) && al16p(dy) && al16p(dcat) && al16p(w),
              "ogv_outlook_vproj_bwd: rows must be 16-B aligned (ldx %d)", ldx);
  const int NJ = t.ncol / 16, NK = (C + 31) / 32;
  const bool sw = (split_w() & 1) != 0;   // the forward's weights (bit-identical v / logits)
  hipStream_t s = as_stream(stream);
  const bf16* xb = (const bf16*)x;
  const bf16* gb = (const bf16*)dy;
  bf16* db = (bf16*)dcat;
#define OGV_VPROJ_BWD(nj, nk)                                                                          \
  if (NJ == nj && NK == nk) {                                                                          \
    const int e = nw == 4 ? vproj_bwd_run<nj, nk, 4>(xb, ldx, w, ldc, bias, gb, db, ldc, H, W, C, heads, t, sw, s) \
                          : vproj_bwd_run<nj, nk, 8>(xb, ldx, w, ldc, bias, gb, db, ldc, H, W, C, heads, t, sw, s); \
    return e ? e : check_launch("ogv_outlook_vproj_bwd");                                              \
  }
  // (NJ, NK) pairs the plan admits: 16 | C <= 96, 8 | head_dim, ncol = C + 9 heads rounded to 16 <= 128
  OGV_VPROJ_BWD(2, 1) OGV_VPROJ_BWD(3, 1) OGV_VPROJ_BWD(4, 1) OGV_VPROJ_BWD(5, 1)
  OGV_VPROJ_BWD(4, 2) OGV_VPROJ_BWD(5, 2) OGV_VPROJ_BWD(6, 2) OGV_VPROJ_BWD(7, 2)
  OGV_VPROJ_BWD(6, 3) OGV_VPROJ_BWD(7, 3) OGV_VPROJ_BWD(8, 3)
#undef OGV_VPROJ_BWD
  OGV_REQUIRE(false, "ogv_outlook_vproj_bwd: no instantiation for %d column / %d k blocks", NJ, NK);
  return OGV_ERR_ARG;
}

// l32: the fp32-logits form -- `cat` receives v only ([M, ldc] bf16 rows), `lg` the logits ([M, ldl] fp32);
// the weight has wrows = C + 9 heads rounded up to 8 rows either way
static int vproj_fwd_impl(const void* x, int ldx, const float* w, const float* bias, void* cat, int ldc, float* lg,
                          int ldl, bool l32, void* y, int B, int H, int W, int C, int heads, int k, ogv_dtype dt,
                          void* stream) {
  OGV_REQUIRE(x && w && y, "ogv_outlook_vproj_fwd: null pointer");
  int rc = check_args(B, H, W, C, heads, k, heads * k * k, C, dt, "ogv_outlook_vproj_fwd");
  if (rc) return rc;
  const int wrows = (C + heads * k * k + 7) / 8 * 8;
  if (l32) {
    OGV_REQUIRE(!cat == !lg, "ogv_outlook_vproj_fwd_l32: v and logits are written together (both or neither)");
    OGV_REQUIRE(!cat || (ldc >= C && ldc % 8 == 0 && ldl >= (heads * 9 + 3) / 4 * 4 && ldl % 4 == 0 && al16p(lg)),
                "ogv_outlook_vproj_fwd_l32: ld_v %d (>= C, 8 | ld_v) / ld_logits %d (>= 9 heads rounded to 4, 16-B rows)",
                ldc, ldl);
  }
  VTile t;
  int nw = 0;
  VHead th;
  int thw = 4;
  if (vhead_plan(B, H, W, C, heads, k, wrows, dt, th, thw)) {
    OGV_REQUIRE(ldx >= C && ldx % 8 == 0 && al16p(x) && al16p(y) && (!cat || al16p(cat)) && al16p(w),
                "ogv_outlook_vproj_fwd: rows must be 16-B aligned (ldx %d)", ldx);
    const bool sw = (split_w() & 1) != 0;
    hipStream_t s = as_stream(stream);
    const bf16* xb = (const bf16*)x;
    bf16 *cb = (bf16*)cat, *yb = (bf16*)y;
    int e;
    switch (C / 32) {
      case 4: e = vhead_dispatch<4>(xb, ldx, w, bias, cb, ldc, yb, B, H, W, C, heads, th, thw, sw, s, lg, ldl, l32); break;
      case 6: e = vhead_dispatch<6>(xb, ldx, w, bias, cb, ldc, yb, B, H, W, C, heads, th, thw, sw, s, lg, ldl, l32); break;
      case 8: e = vhead_dispatch<8>(xb, ldx, w, bias, cb, ldc, yb, B, H, W, C, heads, th, thw, sw, s, lg, ldl, l32); break;
      default: e = vhead_dispatch<12>(xb, ldx, w, bias, cb, ldc, yb, B, H, W, C, heads, th, thw, sw, s, lg, ldl, l32); break;
    }
    return e ? e : check_launch("ogv_outlook_vproj_fwd");
  }
  const bool big = !l32 && vbig_plan(B, H, W, C, heads, k, wrows, dt, t);
  OGV_REQUIRE(big || vproj_plan(B, H, W, C, heads, k, wrows, dt, t, nw, l32),
              "ogv_outlook_vproj_fwd: unsupported shape (needs bf16, k=3, 8 | head_dim, 16 | C <= 96 or "
              "C in {128, 192, 256, 384} with head_dim <= 64, ldc = C + 9*heads rounded up to 8; see "
              "ogv_outlook_vproj_supported)");
  OGV_REQUIRE(ldx >= C && ldx % 8 == 0 && al16p(x) && al16p(y) && (!cat || al16p(cat)) && al16p(w),
              "ogv_outlook_vproj_fwd: rows must be 16-B aligned (ldx %d)", ldx);
  if (big) {
    const bool sw = (split_w() & 1) != 0;
    hipStream_t s = as_stream(stream);
    const bf16* xb = (const bf16*)x;
    bf16 *cb = (bf16*)cat, *yb = (bf16*)y;
    int e;
    switch (C / 32) {
      case 4: e = vbig_run<4>(xb, ldx, w, wrows, bias, cb, ldc, yb, H, W, C, heads, t, sw, s); break;
      case 6: e = vbig_run<6>(xb, ldx, w, wrows, bias, cb, ldc, yb, H, W, C, heads, t, sw, s); break;
      case 8: e = vbig_run<8>(xb, ldx, w, wrows, bias, cb, ldc, yb, H, W, C, heads, t, sw, s); break;
      default: e = vbig_run<12>(xb, ldx, w, wrows, bias, cb, ldc, yb, H, W, C, heads, t, sw, s); break;
    }
    return e ? e : check_launch("ogv_outlook_vproj_fwd");
  }
  const int NJ = t.ncol / 16, NK = (C + 31) / 32;
  const bool sw = (split_w() & 1) != 0;
  hipStream_t s = as_stream(stream);
  const bf16* xb = (const bf16*)x;
  bf16 *cb = (bf16*)cat, *yb = (bf16*)y;
#define OGV_VPROJ(nj, nk)                                                                      \
  if (NJ == nj && NK == nk) {                                                                  \
    const int e = nw == 4 ? vproj_run<nj, nk, 4>(xb, ldx, w, wrows, bias, cb, ldc, yb, H, W, C, heads, t, sw, s, lg, ldl) \
                          : vproj_run<nj, nk, 8>(xb, ldx, w, wrows, bias, cb, ldc, yb, H, W, C, heads, t, sw, s, lg, ldl); \
    return e ? e : check_launch("ogv_outlook_vproj_fwd");                                      \
  }
  // (NJ, NK) pairs the plan admits: 16 | C <= 96, 8 | head_dim, ncol = C + 9 heads rounded to 16 <= 128
  OGV_VPROJ(2, 1) OGV_VPROJ(3, 1) OGV_VPROJ(4, 1) OGV_VPROJ(5, 1)
  OGV_VPROJ(4, 2) OGV_VPROJ(5, 2) OGV_VPROJ(6, 2) OGV_VPROJ(7, 2)
  OGV_VPROJ(6, 3) OGV_VPROJ(7, 3) OGV_VPROJ(8, 3)
#undef OGV_VPROJ
  OGV_REQUIRE(false, "ogv_outlook_vproj_fwd: no instantiation for %d column / %d k blocks", NJ, NK);
  return OGV_ERR_ARG;
}

extern "C" int ogv_outlook_vproj_fwd(const void* x, int ldx, const float* w, const float* bias, void* cat, int ldc,
                                     void* y, int B, int H, int W, int C, int heads, int k, ogv_dtype dt,
                                     void* stream) {
  if (k > 0 && heads > 0)
    OGV_REQUIRE(ldc == (C + heads * k * k + 7) / 8 * 8, "ogv_outlook_vproj_fwd: unsupported shape (ldc %d must be C + heads*k*k rounded up to 8)",
                ldc);
  return vproj_fwd_impl(x, ldx, w, bias, cat, ldc, nullptr, 0, false, y, B, H, W, C, heads, k, dt, stream);
}

// knob "vp_l32" (default 1): the fused Outlooker keeps the logits in fp32 (ogv_outlook_vproj_fwd_l32 +
// ogv_outlook_agg_bwd_l32) wherever its per-head or tile kernel runs; 0: the round-5 bf16 cat
static int g_vp_l32 = 1;
namespace ogv {
void set_vp_l32(int v) { g_vp_l32 = v ? 1 : 0; }
}  // namespace ogv

extern "C" int ogv_outlook_vproj_l32_supported(int B, int H, int W, int C, int heads, int k, int train, ogv_dtype dt) {
  if (!g_vp_l32 || g_outlook_vproj < (train ? 2 : 1) || !lds_160k() || heads <= 0 || k != 3) return 0;
  const int wrows = (C + heads * k * k + 7) / 8 * 8;
  VTile t;
  VHead th;
  int nw = 0;
  if (vhead_plan(B, H, W, C, heads, k, wrows, dt, th, nw)) return 1;
  if (g_vp_big && vbig_plan(B, H, W, C, heads, k, wrows, dt, t)) return 0;   // the streaming kernel: bf16 cat only
  return vproj_plan(B, H, W, C, heads, k, wrows, dt, t, nw, true) ? 1 : 0;
}

extern "C" int ogv_outlook_vproj_fwd_l32(const void* x, int ldx, const float* w, const float* bias, void* v, int ldv,
                                         float* logits, int ldl, void* y, int B, int H, int W, int C, int heads, int k,
                                         ogv_dtype dt, void* stream) {
  return vproj_fwd_impl(x, ldx, w, bias, v, ldv, logits, ldl, true, y, B, H, W, C, heads, k, dt, stream);
}

extern "C" int ogv_outlook_agg_fwd(const void* v, const void* logits, void* y, int B, int H, int W, int C, int heads,
                                   int k, int ldl, int ldv, ogv_dtype dt, void* stream) {
  if (skip_mask() & 64) return OGV_OK;
  OGV_REQUIRE(v && logits && y, "ogv_outlook_agg_fwd: null pointer");
  int rc = check_args(B, H, W, C, heads, k, ldl, ldv, dt, "ogv_outlook_agg_fwd");
  if (rc) return rc;
  const int hd = C / heads;
  if (use_tile(1, dt, k, hd, {v, y}, {ldv, C})) {
    const OTile t = otile_plan(B, H, W, heads, hd, false);
    OGV_REQUIRE(t.ntiles < (1L << 22), "ogv_outlook_agg: %ld tiles exceed the tile kernels' index range", t.ntiles);
    OGV_OTILE_HD(otile_fwd_run, hd, (const bf16*)v, ldv, (const bf16*)logits, ldl, (bf16*)y, C, H, W, heads, t,
                 as_stream(stream));
    return check_launch("ogv_outlook_agg_fwd");
  }
  const int vec = pick_vec_ld(hd, C, ldv, C);
  OGV_OUTLOOK_DISPATCH(launch_fwd, v, logits, y, B, H, W, C, heads, ldl, ldv, as_stream(stream));
  return check_launch("ogv_outlook_agg_fwd");
}

extern "C" size_t ogv_outlook_bwd_ws_bytes(int B, int H, int W, int C, int heads, int k, ogv_dtype dt) {
  if (dt == OGV_BF16 && (g_outlook_tile & 2) && k == 3 && heads > 0 && C % heads == 0 && (C / heads) % 8 == 0 &&
      C / heads <= 64)
    return 0;   // the tiled kernel keeps the probabilities in LDS
  return (size_t)B * H * W * heads * k * k * sizeof(float);
}

extern "C" int ogv_outlook_agg_bwd(const void* dy, const void* v, const void* logits, void* dv, void* dlogits,
                                   float* probs_ws, int B, int H, int W, int C, int heads, int k, int ldl, int ldv,
                                   int lddv, int lddl, int dl_cols, ogv_dtype dt, void* stream) {
  if (skip_mask() & 64) return OGV_OK;
  OGV_REQUIRE(dy && v && logits && dv && dlogits, "ogv_outlook_agg_bwd: null pointer");
  int rc = check_args(B, H, W, C, heads, k, ldl, ldv, dt, "ogv_outlook_agg_bwd");
  if (rc) return rc;
  OGV_REQUIRE(lddv >= C && lddl >= heads * k * k && dl_cols >= heads * k * k && dl_cols <= lddl,
              "ogv_outlook_agg_bwd: ld_dv %d / ld_dlogits %d / dl_cols %d too small", lddv, lddl, dl_cols);
  const int hd = C / heads;
  if (use_tile(2, dt, k, hd, {dy, v, dv}, {ldv, lddv, C})) {
    const OTile t = otile_plan(B, H, W, heads, hd, true);
    OGV_REQUIRE(t.ntiles < (1L << 22), "ogv_outlook_agg: %ld tiles exceed the tile kernels' index range", t.ntiles);
    OGV_OTILE_HD(otile_bwd_run, hd, (const bf16*)dy, C, (const bf16*)v, ldv, (const bf16*)logits, ldl, (bf16*)dv, lddv,
                 (bf16*)dlogits, lddl, dl_cols, H, W, heads, t, as_stream(stream));
    return check_launch("ogv_outlook_agg_bwd");
  }
  OGV_REQUIRE(probs_ws, "ogv_outlook_agg_bwd: probs_ws is required (ogv_outlook_bwd_ws_bytes > 0)");
  const int vec = pick_vec_ld(hd, C, ldv, lddv);
  OGV_OUTLOOK_DISPATCH(launch_bwd, dy, v, logits, dv, dlogits, probs_ws, B, H, W, C, heads, ldl, ldv, lddv, lddl,
                       dl_cols, as_stream(stream));
  return check_launch("ogv_outlook_agg_bwd");
}

extern "C" int ogv_outlook_agg_bwd_l32(const void* dy, const void* v, const float* logits, void* dv, void* dlogits,
                                       int B, int H, int W, int C, int heads, int k, int ldl, int ldv, int lddv,
                                       int lddl, int dl_cols, ogv_dtype dt, void* stream) {
  if (skip_mask() & 64) return OGV_OK;
  OGV_REQUIRE(dy && v && logits && dv && dlogits, "ogv_outlook_agg_bwd_l32: null pointer");
  int rc = check_args(B, H, W, C, heads, k, ldl, ldv, dt, "ogv_outlook_agg_bwd_l32");
  if (rc) return rc;
  OGV_REQUIRE(lddv >= C && lddl >= heads * k * k && dl_cols >= heads * k * k && dl_cols <= lddl,
              "ogv_outlook_agg_bwd_l32: ld_dv %d / ld_dlogits %d / dl_cols %d too small", lddv, lddl, dl_cols);
  const int hd = C / heads;
  OGV_REQUIRE(use_tile(2, dt, k, hd, {dy, v, dv}, {ldv, lddv, C}),
              "ogv_outlook_agg_bwd_l32: needs the LDS-tiled backward (bf16, k = 3, 8 | head_dim <= 64, 16-B rows, "
              "knob outlook_tile bit 2)");
  const OTile t = otile_plan(B, H, W, heads, hd, true);
  OGV_REQUIRE(t.ntiles < (1L << 22), "ogv_outlook_agg: %ld tiles exceed the tile kernels' index range", t.ntiles);
  OGV_OTILE_HD(otile_bwd_run, hd, (const bf16*)dy, C, (const bf16*)v, ldv, logits, ldl, (bf16*)dv, lddv,
               (bf16*)dlogits, lddl, dl_cols, H, W, heads, t, as_stream(stream));
  return check_launch("ogv_outlook_agg_bwd_l32");
}
