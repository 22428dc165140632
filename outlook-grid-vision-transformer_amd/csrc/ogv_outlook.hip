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
__device__ __forceinline__ void otile_logits_load(const bf16* __restrict__ lg, int ldl, int col, const OTile& t,
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
      const bf16* l = lg + ((long)(b * H + yy) * W + xx) * ldl + col + hb * 9;
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

template <int HD>
__global__ __launch_bounds__(256) void outlook_bwd_tile_kernel(const bf16* __restrict__ dy, int lddy,
                                                               const bf16* __restrict__ v, int ldv,
                                                               const bf16* __restrict__ lg, int ldl,
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

template <int HD>
static void otile_bwd_run(const bf16* dy, int lddy, const bf16* v, int ldv, const bf16* lg, int ldl, bf16* dv,
                          int lddv, bf16* dl, int lddl, int dl_cols, int H, int W, int heads, const OTile& t,
                          hipStream_t s) {
  const long nb = (t.ntiles + t.G - 1) / t.G * (heads / t.HB);
  outlook_bwd_tile_kernel<HD><<<xcd_grid(nb), 256, otile_lds(t, HD, true), s>>>(dy, lddy, v, ldv, lg, ldl, dv, lddv,
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

}  // namespace ogv

using namespace ogv;

extern "C" int ogv_outlook_agg_fwd(const void* v, const void* logits, void* y, int B, int H, int W, int C, int heads,
                                   int k, int ldl, int ldv, ogv_dtype dt, void* stream) {
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
