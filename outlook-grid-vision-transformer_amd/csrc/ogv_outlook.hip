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
#include "ogv_common.h"

namespace ogv {

template <typename T, int V, int KS>
__global__ __launch_bounds__(256) void outlook_fwd_kernel(const T* __restrict__ v, const T* __restrict__ logits,
                                                          T* __restrict__ y, int B, int H, int W, int C,
                                                          int heads, int ldl) {
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
        raw[ki * KS + kj] = *reinterpret_cast<const uint4*>(v + ((rowbase + y2c) * W + x2c) * C + c0);
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
      load_vec<T, V>(v + ((rowbase + y2) * W + x2) * C + c0, tmp);
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
                                                                 int C, int heads, int ldl) {
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
        nb[ki * KS + kj] = ((rowbase + min(max(y2, 0), H - 1)) * W + min(max(x2, 0), W - 1)) * C + cb;
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
        load_vec<T, V>(v + ((rowbase + y2) * W + x2) * C + cb + d, tmp);
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
  T* dl = dlogits + p * ldl + head * KK;
  float* pr = probs + (p * heads + head) * KK;
#pragma unroll
  for (int j = 0; j < KK; ++j) {
    dl[j] = from_f<T>(a[j] * (dp[j] - sdp));
    pr[j] = a[j];
  }
}

// One thread per (pixel q, V-channel chunk): dv[q] = sum_j P[q - off_j, head, j] * dy[q - off_j].
template <typename T, int V, int KS>
__global__ __launch_bounds__(256) void outlook_bwd_v_kernel(const T* __restrict__ dy, const float* __restrict__ probs,
                                                            T* __restrict__ dv, int B, int H, int W, int C,
                                                            int heads) {
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
    store_vec<T, V>(dv + q * C + c0, acc);
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
  store_vec<T, V>(dv + q * C + c0, acc);
}

static int pick_vec(int hd, int C) {
  if (hd % 8 == 0 && C % 8 == 0) return 8;
  if (hd % 4 == 0 && C % 4 == 0) return 4;
  if (hd % 2 == 0 && C % 2 == 0) return 2;
  return 1;
}

template <typename T, int V, int KS>
static void launch_fwd(const void* v, const void* lg, void* y, int B, int H, int W, int C, int heads, int ldl,
                       hipStream_t s) {
  const long total = (long)B * H * W * (C / V);
  outlook_fwd_kernel<T, V, KS><<<cdiv(total, 256), 256, 0, s>>>((const T*)v, (const T*)lg, (T*)y, B, H, W, C, heads,
                                                                 ldl);
}

template <typename T, int V, int KS>
static void launch_bwd(const void* dy, const void* v, const void* lg, void* dv, void* dl, float* probs, int B, int H,
                       int W, int C, int heads, int ldl, hipStream_t s) {
  const long t1 = (long)B * H * W * heads;
  outlook_bwd_logits_kernel<T, V, KS><<<cdiv(t1, 256), 256, 0, s>>>((const T*)dy, (const T*)v, (const T*)lg, (T*)dl,
                                                                     probs, B, H, W, C, heads, ldl);
  const long t2 = (long)B * H * W * (C / V);
  outlook_bwd_v_kernel<T, V, KS><<<cdiv(t2, 256), 256, 0, s>>>((const T*)dy, probs, (T*)dv, B, H, W, C, heads);
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

static int check_args(int B, int H, int W, int C, int heads, int k, int ldl, ogv_dtype dt, const char* who) {
  OGV_REQUIRE(B > 0 && H > 0 && W > 0 && C > 0 && heads > 0, "%s: non-positive shape", who);
  OGV_REQUIRE(C % heads == 0, "%s: dim %d not divisible by heads %d", who, C, heads);
  OGV_REQUIRE(k == 1 || k == 3 || k == 5 || k == 7, "%s: kernel_size %d unsupported (1,3,5,7)", who, k);
  OGV_REQUIRE(ldl >= heads * k * k, "%s: ld_logits %d < heads*k*k", who, ldl);
  OGV_REQUIRE(dt == OGV_F32 || dt == OGV_BF16, "%s: bad dtype", who);
  return OGV_OK;
}

}  // namespace ogv

using namespace ogv;

extern "C" int ogv_outlook_agg_fwd(const void* v, const void* logits, void* y, int B, int H, int W, int C, int heads,
                                   int k, int ldl, ogv_dtype dt, void* stream) {
  OGV_REQUIRE(v && logits && y, "ogv_outlook_agg_fwd: null pointer");
  int rc = check_args(B, H, W, C, heads, k, ldl, dt, "ogv_outlook_agg_fwd");
  if (rc) return rc;
  const int vec = pick_vec(C / heads, C);
  OGV_OUTLOOK_DISPATCH(launch_fwd, v, logits, y, B, H, W, C, heads, ldl, as_stream(stream));
  return check_launch("ogv_outlook_agg_fwd");
}

extern "C" int ogv_outlook_agg_bwd(const void* dy, const void* v, const void* logits, void* dv, void* dlogits,
                                   float* probs_ws, int B, int H, int W, int C, int heads, int k, int ldl,
                                   ogv_dtype dt, void* stream) {
  OGV_REQUIRE(dy && v && logits && dv && dlogits && probs_ws, "ogv_outlook_agg_bwd: null pointer");
  int rc = check_args(B, H, W, C, heads, k, ldl, dt, "ogv_outlook_agg_bwd");
  if (rc) return rc;
  const int vec = pick_vec(C / heads, C);
  OGV_OUTLOOK_DISPATCH(launch_bwd, dy, v, logits, dv, dlogits, probs_ws, B, H, W, C, heads, ldl, as_stream(stream));
  return check_launch("ogv_outlook_agg_bwd");
}
