// Grid multi-head self-attention on NHWC rows with the strided grid partition folded into the
// addressing (no partition/unpartition copies, no qkv split copies).
//
// Reference (src/model/grid_partition.py:13-15, src/model/grid_attention.py:70-86):
//   grids = x.view(B, H/g, g, W/g, g, C).permute(0,2,4,1,3,5)  -> group (b, gi, gj) holds
//           pixels (ty*g + gi, tx*g + gj), token n = ty*(W/g) + tx
//   qkv channel = s*C + head*hd + d;  S = (q @ k^T) * hd^-0.5;  P = softmax(S);  O = P @ V
//   out channel = head*hd + d (transpose(1,2).reshape(B,N,C)), written back at the pixel.
// bf16 with N >= 16 and head_dim <= 64 runs on the MFMA flash-style kernels of ogv_grid_mfma.hip.
// The rest (N = 4 groups of Model-A-7M stages 1-3, fp32 parity mode, the probability-capturing
// analysis path): one thread per (query, head) walks the group's keys with an online softmax;
// keys/values of a group are shared through L1/L2 by the N*heads threads of the group, which are
// adjacent in the launch.
#include "ogv_common.h"

namespace ogv {

struct GridGeom {
  int B, H, W, C, heads, g, Hg, Wg, N, hd;
  __device__ __forceinline__ long pixel(long grp, int tok) const {
    const int gj = (int)(grp % g);
    const long r = grp / g;
    const int gi = (int)(r % g);
    const long b = r / g;
    const int ty = tok / Wg, tx = tok - ty * Wg;
    return (b * H + (long)ty * g + gi) * W + (long)tx * g + gj;
  }
};

template <typename T, int V>
__device__ __forceinline__ float dot_row(const T* __restrict__ p, const float* q, int hd) {
  float s = 0.f;
  for (int d = 0; d < hd; d += V) {
    float t[V];
    load_vec<T, V>(p + d, t);
#pragma unroll
    for (int i = 0; i < V; ++i) s = fmaf(q[d + i], t[i], s);
  }
  return s;
}

// NOTE: q[] etc. are HDMAX-sized register arrays; every index below is a compile-time-unrollable
// loop over HDMAX with a runtime `d < hd` guard so nothing spills to scratch.
template <typename T, int HDMAX, int V>
__global__ __launch_bounds__(256) void grid_fwd_kernel(const T* __restrict__ qkv, T* __restrict__ out,
                                                       float* __restrict__ lse, float* __restrict__ probs,
                                                       GridGeom G, float scale) {
  const long total = (long)G.B * G.g * G.g * G.N * G.heads;
  const long tid = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (tid >= total) return;
  const int h = (int)(tid % G.heads);
  const long r = tid / G.heads;
  const int t = (int)(r % G.N);
  const long grp = r / G.N;
  const int hd = G.hd;
  const long C3 = 3L * G.C;
  const long pq = G.pixel(grp, t);

  float q[HDMAX], o[HDMAX];
  {
    // every chunk loaded at a clamped (valid) offset, then zeroed past hd: one round trip, where a
    // guarded load_vec per chunk made the compiler wait for each chunk in turn
    RawVec<T, V> rq[HDMAX / V];
#pragma unroll
    for (int d0 = 0; d0 < HDMAX; d0 += V) rq[d0 / V].load(qkv + pq * C3 + h * hd + min(d0, hd - V));
#pragma unroll
    for (int d0 = 0; d0 < HDMAX; d0 += V) {
      rq[d0 / V].unpack(q + d0);
      if (d0 >= hd) {
#pragma unroll
        for (int i = 0; i < V; ++i) q[d0 + i] = 0.f;
      }
    }
  }
#pragma unroll
  for (int d = 0; d < HDMAX; ++d) { q[d] *= scale; o[d] = 0.f; }

  float m = -INFINITY, l = 0.f;
  for (int u = 0; u < G.N; ++u) {
    const long pk = G.pixel(grp, u);
    const T* kp = qkv + pk * C3 + G.C + h * hd;
    float s = 0.f;
    if constexpr (sizeof(T) == 2 && V == 8) {
      // bf16: this key's k AND v rows are issued together (v does not depend on the score), so a
      // key costs one memory round trip instead of two; same arithmetic order as below
      // (clamped, always-valid chunk offsets: the chunks past hd reload the last one and are skipped
      // below -- a per-chunk guard made the compiler wait for each load in turn)
      uint4 rk[HDMAX / 8], rv[HDMAX / 8];
#pragma unroll
      for (int c = 0; c < HDMAX / 8; ++c) {
        const int cc = min(c * 8, hd - 8);
        rk[c] = *reinterpret_cast<const uint4*>(kp + cc);
        rv[c] = *reinterpret_cast<const uint4*>(kp + G.C + cc);
      }
#pragma unroll
      for (int c = 0; c < HDMAX / 8; ++c) {
        if (c * 8 < hd) {
          const bf16* e = reinterpret_cast<const bf16*>(&rk[c]);
#pragma unroll
          for (int i = 0; i < 8; ++i) s = fmaf(q[c * 8 + i], (float)e[i], s);
        }
      }
      float pw;
      if (s > m) {
        const float corr = __expf(m - s);
        l *= corr;
#pragma unroll
        for (int d = 0; d < HDMAX; ++d) o[d] *= corr;
        m = s;
        pw = 1.f;
      } else {
        pw = __expf(s - m);
      }
      l += pw;
#pragma unroll
      for (int c = 0; c < HDMAX / 8; ++c) {
        if (c * 8 < hd) {
          const bf16* e = reinterpret_cast<const bf16*>(&rv[c]);
#pragma unroll
          for (int i = 0; i < 8; ++i) o[c * 8 + i] = fmaf(pw, (float)e[i], o[c * 8 + i]);
        }
      }
      continue;
    }
#pragma unroll
    for (int d0 = 0; d0 < HDMAX; d0 += V) {
      if (d0 < hd) {
        float tk[V];
        load_vec<T, V>(kp + d0, tk);
#pragma unroll
        for (int i = 0; i < V; ++i) s = fmaf(q[d0 + i], tk[i], s);
      }
    }
    float pw;
    if (s > m) {
      const float corr = __expf(m - s);  // m = -inf on the first key -> 0
      l *= corr;
#pragma unroll
      for (int d = 0; d < HDMAX; ++d) o[d] *= corr;
      m = s;
      pw = 1.f;
    } else {
      pw = __expf(s - m);
    }
    l += pw;
    const T* vp = kp + G.C;
#pragma unroll
    for (int d0 = 0; d0 < HDMAX; d0 += V) {
      if (d0 < hd) {
        float tv[V];
        load_vec<T, V>(vp + d0, tv);
#pragma unroll
        for (int i = 0; i < V; ++i) o[d0 + i] = fmaf(pw, tv[i], o[d0 + i]);
      }
    }
  }
  const float inv = 1.f / l;
#pragma unroll
  for (int d0 = 0; d0 < HDMAX; d0 += V) {
    if (d0 < hd) {
      float tmp[V];
#pragma unroll
      for (int i = 0; i < V; ++i) tmp[i] = o[d0 + i] * inv;
      store_vec<T, V>(out + pq * G.C + h * hd + d0, tmp);
    }
  }
  const float lse_v = m + __logf(l);
  lse[pq * G.heads + h] = lse_v;
  if (probs) {
    float* pr = probs + ((grp * G.heads + h) * G.N + t) * (long)G.N;
    for (int u = 0; u < G.N; ++u) {
      const long pk = G.pixel(grp, u);
      const T* kp = qkv + pk * C3 + G.C + h * hd;
      float s = 0.f;
#pragma unroll
      for (int d0 = 0; d0 < HDMAX; d0 += V) {
        if (d0 < hd) {
          float tk[V];
          load_vec<T, V>(kp + d0, tk);
#pragma unroll
          for (int i = 0; i < V; ++i) s = fmaf(q[d0 + i], tk[i], s);
        }
      }
      pr[u] = __expf(s - lse_v);
    }
  }
}

// delta[p, h] = <dO[p, h-slice], O[p, h-slice]>  (= sum_j P_ij dP_ij)
template <typename T, int V>
__global__ __launch_bounds__(256) void grid_bwd_delta_kernel(const T* __restrict__ dout, const T* __restrict__ out,
                                                             float* __restrict__ delta, long M, int C, int heads) {
  const long tid = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (tid >= M * heads) return;
  const int h = (int)(tid % heads);
  const long p = tid / heads;
  const int hd = C / heads;
  float s = 0.f;
  for (int d = 0; d < hd; d += V) {
    float a[V], b[V];
    load_vec<T, V>(dout + p * C + h * hd + d, a);
    load_vec<T, V>(out + p * C + h * hd + d, b);
#pragma unroll
    for (int i = 0; i < V; ++i) s = fmaf(a[i], b[i], s);
  }
  delta[tid] = s;
}

// dQ_i = scale * sum_j P_ij (dP_ij - delta_i) K_j        (thread per (query, head)).
// delta_i = <dO_i, O_i> is formed here from the query's own rows (grid_bwd_delta_kernel's arithmetic, same
// order) and written for the dK / dV kernel that follows: no separate delta launch
template <typename T, int HDMAX, int V>
__global__ __launch_bounds__(256) void grid_bwd_dq_kernel(const T* __restrict__ dout, const T* __restrict__ qkv,
                                                          const T* __restrict__ out, const float* __restrict__ lse,
                                                          float* __restrict__ delta, T* __restrict__ dqkv,
                                                          GridGeom G, float scale) {
  const long total = (long)G.B * G.g * G.g * G.N * G.heads;
  const long tid = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (tid >= total) return;
  const int h = (int)(tid % G.heads);
  const long r = tid / G.heads;
  const int t = (int)(r % G.N);
  const long grp = r / G.N;
  const int hd = G.hd;
  const long C3 = 3L * G.C;
  const long pq = G.pixel(grp, t);

  float q[HDMAX], go[HDMAX], dq[HDMAX], ov[HDMAX];
#pragma unroll
  for (int d0 = 0; d0 < HDMAX; d0 += V) {
    if (d0 < hd) {
      load_vec<T, V>(qkv + pq * C3 + h * hd + d0, q + d0);
      load_vec<T, V>(dout + pq * G.C + h * hd + d0, go + d0);
      load_vec<T, V>(out + pq * G.C + h * hd + d0, ov + d0);
    } else {
#pragma unroll
      for (int i = 0; i < V; ++i) { q[d0 + i] = 0.f; go[d0 + i] = 0.f; ov[d0 + i] = 0.f; }
    }
  }
  float dl = 0.f;
#pragma unroll
  for (int d0 = 0; d0 < HDMAX; d0 += V)
    if (d0 < hd) {
#pragma unroll
      for (int i = 0; i < V; ++i) dl = fmaf(go[d0 + i], ov[d0 + i], dl);
    }
  delta[pq * G.heads + h] = dl;
#pragma unroll
  for (int d = 0; d < HDMAX; ++d) { q[d] *= scale; dq[d] = 0.f; }
  const float lq = lse[pq * G.heads + h];
  for (int u = 0; u < G.N; ++u) {
    const long pk = G.pixel(grp, u);
    const T* kp = qkv + pk * C3 + G.C + h * hd;
    const T* vp = kp + G.C;
    float kr[HDMAX];
    float s = 0.f, dp = 0.f;
#pragma unroll
    for (int d0 = 0; d0 < HDMAX; d0 += V) {
      if (d0 < hd) {
        float tv[V];
        load_vec<T, V>(kp + d0, kr + d0);
        load_vec<T, V>(vp + d0, tv);
#pragma unroll
        for (int i = 0; i < V; ++i) {
          s = fmaf(q[d0 + i], kr[d0 + i], s);
          dp = fmaf(go[d0 + i], tv[i], dp);
        }
      } else {
#pragma unroll
        for (int i = 0; i < V; ++i) kr[d0 + i] = 0.f;
      }
    }
    const float pw = __expf(s - lq);
    const float ds = pw * (dp - dl);
#pragma unroll
    for (int d = 0; d < HDMAX; ++d) dq[d] = fmaf(ds, kr[d], dq[d]);
  }
#pragma unroll
  for (int d0 = 0; d0 < HDMAX; d0 += V) {
    if (d0 < hd) {
      float tmp[V];
#pragma unroll
      for (int i = 0; i < V; ++i) tmp[i] = dq[d0 + i] * scale;
      store_vec<T, V>(dqkv + pq * C3 + h * hd + d0, tmp);
    }
  }
}

// dK_j = scale * sum_i dS_ij Q_i ; dV_j = sum_i P_ij dO_i   (thread per (key, head))
template <typename T, int HDMAX, int V>
__global__ __launch_bounds__(256) void grid_bwd_dkv_kernel(const T* __restrict__ dout, const T* __restrict__ qkv,
                                                           const float* __restrict__ lse,
                                                           const float* __restrict__ delta, T* __restrict__ dqkv,
                                                           GridGeom G, float scale) {
  const long total = (long)G.B * G.g * G.g * G.N * G.heads;
  const long tid = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (tid >= total) return;
  const int h = (int)(tid % G.heads);
  const long r = tid / G.heads;
  const int u = (int)(r % G.N);
  const long grp = r / G.N;
  const int hd = G.hd;
  const long C3 = 3L * G.C;
  const long pk = G.pixel(grp, u);

  float kk[HDMAX], vv[HDMAX], dk[HDMAX], dv[HDMAX];
#pragma unroll
  for (int d0 = 0; d0 < HDMAX; d0 += V) {
    if (d0 < hd) {
      load_vec<T, V>(qkv + pk * C3 + G.C + h * hd + d0, kk + d0);
      load_vec<T, V>(qkv + pk * C3 + 2 * G.C + h * hd + d0, vv + d0);
    } else {
#pragma unroll
      for (int i = 0; i < V; ++i) { kk[d0 + i] = 0.f; vv[d0 + i] = 0.f; }
    }
  }
#pragma unroll
  for (int d = 0; d < HDMAX; ++d) { kk[d] *= scale; dk[d] = 0.f; dv[d] = 0.f; }
  for (int t = 0; t < G.N; ++t) {
    const long pq = G.pixel(grp, t);
    const T* qp = qkv + pq * C3 + h * hd;
    const T* gp = dout + pq * G.C + h * hd;
    float qr[HDMAX], gr[HDMAX];
    float s = 0.f, dp = 0.f;
#pragma unroll
    for (int d0 = 0; d0 < HDMAX; d0 += V) {
      if (d0 < hd) {
        load_vec<T, V>(qp + d0, qr + d0);
        load_vec<T, V>(gp + d0, gr + d0);
#pragma unroll
        for (int i = 0; i < V; ++i) {
          s = fmaf(qr[d0 + i], kk[d0 + i], s);
          dp = fmaf(gr[d0 + i], vv[d0 + i], dp);
        }
      } else {
#pragma unroll
        for (int i = 0; i < V; ++i) { qr[d0 + i] = 0.f; gr[d0 + i] = 0.f; }
      }
    }
    const float pw = __expf(s - lse[pq * G.heads + h]);
    const float ds = pw * (dp - delta[pq * G.heads + h]);
#pragma unroll
    for (int d = 0; d < HDMAX; ++d) {
      dk[d] = fmaf(ds, qr[d], dk[d]);
      dv[d] = fmaf(pw, gr[d], dv[d]);
    }
  }
#pragma unroll
  for (int d0 = 0; d0 < HDMAX; d0 += V) {
    if (d0 < hd) {
      float a[V], b[V];
#pragma unroll
      for (int i = 0; i < V; ++i) { a[i] = dk[d0 + i] * scale; b[i] = dv[d0 + i]; }
      store_vec<T, V>(dqkv + pk * C3 + G.C + h * hd + d0, a);
      store_vec<T, V>(dqkv + pk * C3 + 2 * G.C + h * hd + d0, b);
    }
  }
}

static int pick_vec(int hd) {
  if (hd % 8 == 0) return 8;
  if (hd % 4 == 0) return 4;
  if (hd % 2 == 0) return 2;
  return 1;
}

template <typename T, int HDMAX, int V>
static void fwd_launch(const void* qkv, void* out, float* lse, float* probs, const GridGeom& G, float scale,
                       hipStream_t s) {
  const long total = (long)G.B * G.g * G.g * G.N * G.heads;
  grid_fwd_kernel<T, HDMAX, V><<<cdiv(total, 256), 256, 0, s>>>((const T*)qkv, (T*)out, lse, probs, G, scale);
}

template <typename T, int HDMAX, int V>
static void bwd_launch(const void* dout, const void* qkv, const void* out, const float* lse, void* dqkv,
                       float* delta, const GridGeom& G, float scale, hipStream_t s) {
  const long total = (long)G.B * G.g * G.g * G.N * G.heads;   // (the dQ kernel writes delta for dK / dV)
  grid_bwd_dq_kernel<T, HDMAX, V><<<cdiv(total, 256), 256, 0, s>>>((const T*)dout, (const T*)qkv, (const T*)out, lse,
                                                                   delta, (T*)dqkv, G, scale);
  grid_bwd_dkv_kernel<T, HDMAX, V><<<cdiv(total, 256), 256, 0, s>>>((const T*)dout, (const T*)qkv, lse, delta,
                                                                    (T*)dqkv, G, scale);
}

#define OGV_GRID_DISPATCH_V(T, HDM, FN, ...)         \
  switch (vec) {                                     \
    case 8: FN<T, HDM, 8>(__VA_ARGS__); break;       \
    case 4: FN<T, HDM, 4>(__VA_ARGS__); break;       \
    case 2: FN<T, HDM, 2>(__VA_ARGS__); break;       \
    default: FN<T, HDM, 1>(__VA_ARGS__); break;      \
  }
#define OGV_GRID_DISPATCH_H(T, FN, ...)                                   \
  if (G.hd <= 32) { OGV_GRID_DISPATCH_V(T, 32, FN, __VA_ARGS__) }         \
  else if (G.hd <= 64) { OGV_GRID_DISPATCH_V(T, 64, FN, __VA_ARGS__) }    \
  else { OGV_GRID_DISPATCH_V(T, 128, FN, __VA_ARGS__) }
#define OGV_GRID_DISPATCH(FN, ...)                                        \
  do {                                                                    \
    if (dt == OGV_BF16) { OGV_GRID_DISPATCH_H(bf16, FN, __VA_ARGS__) }    \
    else { OGV_GRID_DISPATCH_H(float, FN, __VA_ARGS__) }                  \
  } while (0)

static int make_geom(GridGeom& G, int B, int H, int W, int C, int heads, int g, ogv_dtype dt, const char* who) {
  OGV_REQUIRE(B > 0 && H > 0 && W > 0 && C > 0 && heads > 0 && g > 0, "%s: non-positive shape", who);
  OGV_REQUIRE(H % g == 0 && W % g == 0, "%s: H=%d, W=%d not divisible by grid_size %d", who, H, W, g);
  OGV_REQUIRE(C % heads == 0, "%s: dim %d not divisible by heads %d", who, C, heads);
  OGV_REQUIRE(C / heads <= 128, "%s: head_dim %d > 128 unsupported", who, C / heads);
  OGV_REQUIRE(dt == OGV_F32 || dt == OGV_BF16, "%s: bad dtype", who);
  G.B = B; G.H = H; G.W = W; G.C = C; G.heads = heads; G.g = g;
  G.Hg = H / g; G.Wg = W / g; G.N = G.Hg * G.Wg; G.hd = C / heads;
  return OGV_OK;
}

// MFMA flash-style kernels for N >= 16 (ogv_grid_mfma.hip); false = shape not covered
bool grid_mfma_fwd(const void* qkv, void* out, float* lse, int B, int H, int W, int C, int heads, int g, float scale,
                   hipStream_t s);
bool grid_mfma_bwd(const void* dout, const void* qkv, const float* lse, const float* delta, void* dqkv, int B, int H,
                   int W, int C, int heads, int g, float scale, hipStream_t s);

template <typename T>
static void delta_launch(const void* dout, const void* out, float* delta, const GridGeom& G, int vec, hipStream_t s) {
  const long M = (long)G.B * G.H * G.W;
  const unsigned grid = cdiv(M * G.heads, 256);
  switch (vec) {
    case 8: grid_bwd_delta_kernel<T, 8><<<grid, 256, 0, s>>>((const T*)dout, (const T*)out, delta, M, G.C, G.heads); break;
    case 4: grid_bwd_delta_kernel<T, 4><<<grid, 256, 0, s>>>((const T*)dout, (const T*)out, delta, M, G.C, G.heads); break;
    case 2: grid_bwd_delta_kernel<T, 2><<<grid, 256, 0, s>>>((const T*)dout, (const T*)out, delta, M, G.C, G.heads); break;
    default: grid_bwd_delta_kernel<T, 1><<<grid, 256, 0, s>>>((const T*)dout, (const T*)out, delta, M, G.C, G.heads);
  }
}

static int g_grid_mfma = 1;  // tuning knob "grid_mfma"
void set_grid_mfma(int v) { g_grid_mfma = v; }

}  // namespace ogv

using namespace ogv;

extern "C" int ogv_grid_attn_fwd(const void* qkv, void* out, float* lse, float* probs, int B, int H, int W, int C,
                                 int heads, int g, float scale, ogv_dtype dt, void* stream) {
  if (skip_mask() & 32) return OGV_OK;
  OGV_REQUIRE(qkv && out && lse, "ogv_grid_attn_fwd: null pointer");
  GridGeom G;
  int rc = make_geom(G, B, H, W, C, heads, g, dt, "ogv_grid_attn_fwd");
  if (rc) return rc;
  const int vec = pick_vec(G.hd);
  if (dt == OGV_BF16 && !probs && g_grid_mfma &&
      grid_mfma_fwd(qkv, out, lse, B, H, W, C, heads, g, scale, as_stream(stream)))
    return check_launch("ogv_grid_attn_fwd");
  OGV_GRID_DISPATCH(fwd_launch, qkv, out, lse, probs, G, scale, as_stream(stream));
  return check_launch("ogv_grid_attn_fwd");
}

extern "C" int ogv_grid_attn_bwd(const void* dout, const void* qkv, const void* out, const float* lse, void* dqkv,
                                 float* delta_ws, int B, int H, int W, int C, int heads, int g, float scale,
                                 ogv_dtype dt, void* stream) {
  if (skip_mask() & 32) return OGV_OK;
  OGV_REQUIRE(dout && qkv && out && lse && dqkv && delta_ws, "ogv_grid_attn_bwd: null pointer");
  GridGeom G;
  int rc = make_geom(G, B, H, W, C, heads, g, dt, "ogv_grid_attn_bwd");
  if (rc) return rc;
  const int vec = pick_vec(G.hd);
  if (dt == OGV_BF16 && g_grid_mfma && G.N >= 16 && G.hd % 8 == 0 && G.hd <= 64) {
    delta_launch<bf16>(dout, out, delta_ws, G, vec, as_stream(stream));
    if (grid_mfma_bwd(dout, qkv, lse, delta_ws, dqkv, B, H, W, C, heads, g, scale, as_stream(stream)))
      return check_launch("ogv_grid_attn_bwd");
  }
  OGV_GRID_DISPATCH(bwd_launch, dout, qkv, out, lse, dqkv, delta_ws, G, scale, as_stream(stream));
  return check_launch("ogv_grid_attn_bwd");
}
