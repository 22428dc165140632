// Batch mixing for the training loop: MixUp / CutMix images and their soft targets
// (src/training/cutmix_mixup_aug.py:17-64, called by one_epoch_train.py:77-82).
//
// The reference clones the batch, gathers images[perm] and pastes a box (CutMix), or forms
// images*lam + images[perm]*(1-lam) (MixUp), then one-hots both label vectors and blends them —
// five to seven ATen launches and two full copies of the batch.  Here one launch writes the mixed
// batch (reads x and x[perm] once, writes out once) and one launch writes the [B, K] soft targets.
// HBM-bound elementwise work: 16-B vector accesses, one image row-slab per block so the perm
// lookup is a single scalar load.  Arithmetic follows ATen's rounding points exactly
// (separate products, then the sum; no fused multiply-add), so fp32 results are bit-identical;
// for bf16 images the blend is computed in fp32 and rounded once (ATen rounds each bf16 op).
#include "ogv_common.h"

// hipcc contracts a*b + c*d into an FMA by default; ATen's CPU MixUp rounds each product.
// (The pragma must cover the expression itself: __fmul_rn/__fadd_rn are header inlines compiled
// with contraction on.)
#pragma clang fp contract(off)

namespace ogv {

__device__ __forceinline__ float blend(float a, float la, float b, float lb) {
  const float pa = a * la;
  const float pb = b * lb;
  return pa + pb;
}

// out[b, e] for e in one image (n = C*H*W elements).  mode 0: MixUp, 1: CutMix.
// CutMix: an element (c, y, x) comes from image perm[b] when y1 <= y < y2 and x1 <= x < x2.
template <typename T, bool CL>
__global__ void __launch_bounds__(256) mix_images_kernel(const T* __restrict__ x, T* __restrict__ out,
                                                         const int64_t* __restrict__ perm, long n, int C, int H,
                                                         int W, int mode, float lam_a, float lam_b, int y1, int y2,
                                                         int x1, int x2) {
  const int b = blockIdx.y;
  const long pb = perm[b];
  const T* __restrict__ xa = x + (long)b * n;
  const T* __restrict__ xb = x + pb * n;
  T* __restrict__ o = out + (long)b * n;
  constexpr int V = 16 / sizeof(T);
  const long nv = n / V;
  for (long v = (long)blockIdx.x * blockDim.x + threadIdx.x; v < nv; v += (long)gridDim.x * blockDim.x) {
    const long e0 = v * V;
    float a[V], r[V];
    if (mode == 0) {
      load_vec<T, V>(xa + e0, a);
      load_vec<T, V>(xb + e0, r);
#pragma unroll
      for (int i = 0; i < V; ++i) r[i] = blend(a[i], lam_a, r[i], lam_b);
      store_vec<T, V>(o + e0, r);
    } else {
      bool in[V];
      int cnt = 0;
#pragma unroll
      for (int i = 0; i < V; ++i) {
        const long e = e0 + i;
        int yy, xx;
        if (CL) { const long p = e / C; yy = (int)(p / W); xx = (int)(p % W); }
        else    { const long p = e % ((long)H * W); yy = (int)(p / W); xx = (int)(p % W); }
        in[i] = yy >= y1 && yy < y2 && xx >= x1 && xx < x2;
        cnt += in[i];
      }
      if (cnt == 0) {
        load_vec<T, V>(xa + e0, r);
      } else if (cnt == V) {
        load_vec<T, V>(xb + e0, r);
      } else {
        load_vec<T, V>(xa + e0, a);
        load_vec<T, V>(xb + e0, r);
#pragma unroll
        for (int i = 0; i < V; ++i) r[i] = in[i] ? r[i] : a[i];
      }
      store_vec<T, V>(o + e0, r);
    }
  }
}

// Tail / unaligned path: one element per thread.
template <typename T, bool CL>
__global__ void __launch_bounds__(256) mix_images_scalar_kernel(const T* __restrict__ x, T* __restrict__ out,
                                                                const int64_t* __restrict__ perm, long n, long e_beg,
                                                                int C, int H, int W, int mode, float lam_a,
                                                                float lam_b, int y1, int y2, int x1, int x2) {
  const int b = blockIdx.y;
  const long pb = perm[b];
  for (long e = e_beg + (long)blockIdx.x * blockDim.x + threadIdx.x; e < n; e += (long)gridDim.x * blockDim.x) {
    const float a = to_f(x[(long)b * n + e]);
    const float r = to_f(x[pb * n + e]);
    float v;
    if (mode == 0) {
      v = blend(a, lam_a, r, lam_b);
    } else {
      int yy, xx;
      if (CL) { const long p = e / C; yy = (int)(p / W); xx = (int)(p % W); }
      else    { const long p = e % ((long)H * W); yy = (int)(p / W); xx = (int)(p % W); }
      v = (yy >= y1 && yy < y2 && xx >= x1 && xx < x2) ? r : a;
    }
    out[(long)b * n + e] = from_f<T>(v);
  }
}

// soft[b, k] = onehot(t[b])[k] * lam_a + onehot(t[perm[b]])[k] * lam_b; perm == nullptr: one-hot.
__global__ void __launch_bounds__(256) mix_targets_kernel(const int64_t* __restrict__ t,
                                                          const int64_t* __restrict__ perm, float* __restrict__ out,
                                                          int B, int K, float lam_a, float lam_b) {
  const long total = (long)B * K;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int b = (int)(i / K), k = (int)(i % K);
    // a label outside [0, K) (F.one_hot raises on it) makes its row NaN: the loss turns
    // non-finite and the training step's device guard skips the update and counts it
    const int64_t ta = t[b];
    const int64_t tb = perm ? t[perm[b]] : 0;
    if (ta < 0 || ta >= K || tb < 0 || tb >= K) { out[i] = __builtin_nanf(""); continue; }
    const float y1 = ta == k ? 1.f : 0.f;
    if (perm == nullptr) { out[i] = y1; continue; }
    const float y2 = tb == k ? 1.f : 0.f;
    out[i] = blend(y1, lam_a, y2, lam_b);
  }
}

template <typename T, bool CL>
static void mix_images_run(const void* x, void* out, const int64_t* perm, int B, int C, int H, int W, int mode,
                           float lam_a, float lam_b, int y1, int y2, int x1, int x2, hipStream_t s) {
  const long n = (long)C * H * W;
  constexpr int V = 16 / sizeof(T);
  const bool aligned = ((uintptr_t)x % 16 == 0) && ((uintptr_t)out % 16 == 0) && (n % V == 0);
  const long nv = aligned ? n / V : 0;
  if (nv > 0) {
    dim3 grid(cdiv(nv, 256) < 64 ? cdiv(nv, 256) : 64, B);
    mix_images_kernel<T, CL><<<grid, 256, 0, s>>>((const T*)x, (T*)out, perm, n, C, H, W, mode, lam_a, lam_b, y1, y2,
                                                   x1, x2);
  }
  const long beg = nv * V;
  if (beg < n) {
    dim3 grid(cdiv(n - beg, 256) < 64 ? cdiv(n - beg, 256) : 64, B);
    mix_images_scalar_kernel<T, CL><<<grid, 256, 0, s>>>((const T*)x, (T*)out, perm, n, beg, C, H, W, mode, lam_a,
                                                          lam_b, y1, y2, x1, x2);
  }
}

}  // namespace ogv

using namespace ogv;

extern "C" int ogv_mix_images(const void* x, void* out, const int64_t* perm, int B, int C, int H, int W,
                              int channels_last, int mode, float lam_a, float lam_b, int y1, int y2, int x1, int x2,
                              ogv_dtype dt, void* stream) {
  OGV_REQUIRE(B >= 0 && C > 0 && H > 0 && W > 0, "ogv_mix_images: bad shape B=%d C=%d H=%d W=%d", B, C, H, W);
  OGV_REQUIRE(mode == 0 || mode == 1, "ogv_mix_images: mode must be 0 (mixup) or 1 (cutmix), got %d", mode);
  OGV_REQUIRE(dt == OGV_F32 || dt == OGV_BF16, "ogv_mix_images: bad dtype %d", (int)dt);
  OGV_REQUIRE(B <= 65535, "ogv_mix_images: B=%d exceeds the grid's y extent", B);
  if (B == 0) return OGV_OK;
  OGV_REQUIRE(x && out && perm, "ogv_mix_images: null pointer");
  OGV_REQUIRE(x != out, "ogv_mix_images: in-place mixing is not supported (rows are read through perm)");
  OGV_REQUIRE(mode == 0 || (0 <= y1 && y1 <= y2 && y2 <= H && 0 <= x1 && x1 <= x2 && x2 <= W),
              "ogv_mix_images: box [%d,%d)x[%d,%d) outside %dx%d", y1, y2, x1, x2, H, W);
  hipStream_t s = as_stream(stream);
  if (dt == OGV_F32) {
    if (channels_last) mix_images_run<float, true>(x, out, perm, B, C, H, W, mode, lam_a, lam_b, y1, y2, x1, x2, s);
    else mix_images_run<float, false>(x, out, perm, B, C, H, W, mode, lam_a, lam_b, y1, y2, x1, x2, s);
  } else {
    if (channels_last) mix_images_run<bf16, true>(x, out, perm, B, C, H, W, mode, lam_a, lam_b, y1, y2, x1, x2, s);
    else mix_images_run<bf16, false>(x, out, perm, B, C, H, W, mode, lam_a, lam_b, y1, y2, x1, x2, s);
  }
  return check_launch("ogv_mix_images");
}

extern "C" int ogv_mix_targets(const int64_t* targets, const int64_t* perm, float* out, int B, int K, float lam_a,
                               float lam_b, void* stream) {
  OGV_REQUIRE(B >= 0 && K > 0, "ogv_mix_targets: bad shape B=%d K=%d", B, K);
  if (B == 0) return OGV_OK;
  OGV_REQUIRE(targets && out, "ogv_mix_targets: null pointer");
  const long total = (long)B * K;
  const unsigned grid = cdiv(total, 256) < 1024 ? cdiv(total, 256) : 1024;
  mix_targets_kernel<<<grid, 256, 0, as_stream(stream)>>>(targets, perm, out, B, K, lam_a, lam_b);
  return check_launch("ogv_mix_targets");
}
