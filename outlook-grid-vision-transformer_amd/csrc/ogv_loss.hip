// The training loss of the benchmarked step: F.cross_entropy(logits.float(), targets,
// label_smoothing=ls) with mean reduction (src/training/one_epoch_train.py:96), forward in two
// native launches and backward in one, instead of ATen's log_softmax / nll / smoothing-sum / mean
// chain (~12 launches per step, each a few us of a 200 KB problem).
//
// torch's definition (label smoothing, mean, no class weights, ignore_index -100):
//   loss = (1 - ls) * sum_i nll_i / n + (ls / K) * sum_i smooth_i / n,    n = #rows with y != -100
//   nll_i = lse_i - z[i, y_i],   smooth_i = -sum_k logp_ik = K * lse_i - sum_k z[i, k]
//   dz[i, k] = g / n * (softmax_ik - (1 - ls) [k == y_i] - ls / K)   (0 for ignored rows)
// A label outside [0, K) (torch raises, which needs a device sync) makes the loss NaN, so the step's
// found_inf guard skips the update; the forward ALSO adds the number of such rows to a separate
// device counter (bad_labels, when given), which the Trainer reads to raise as torch would -- a
// bad label is a data error, not a non-finite step.  The forward also writes that guard
// (found = !isfinite(loss)) when asked, so the step needs no separate flag launch.
#include "ogv_common.h"

#include <cmath>

namespace ogv {

// Forward in two launches: ce_rows_kernel (a wave per row, B / 4 workgroups) writes each row's
// logsumexp and its two loss terms; ce_final_kernel (one workgroup) sums them in a fixed order.
// ws = [lse (B) | nll (B) | smooth (B) | valid (B) | n_valid | bad (B)]
__device__ __forceinline__ float wave_max_f(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

__global__ __launch_bounds__(256) void ce_rows_kernel(const float* __restrict__ z, const int64_t* __restrict__ y,
                                                      int B, int K, float* __restrict__ ws) {
  const int lane = threadIdx.x & 63;
  const int i = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (i >= B) return;
  const float* zr = z + (long)i * K;
  float mx = -INFINITY;
  for (int k = lane; k < K; k += 64) mx = fmaxf(mx, zr[k]);
  mx = wave_max_f(mx);
  float s = 0.f, sz = 0.f;
  for (int k = lane; k < K; k += 64) {
    const float v = zr[k];
    s += expf(v - mx);
    sz += v;
  }
  s = wave_sum(s);
  sz = wave_sum(sz);
  if (lane == 0) {
    const float lse = mx + logf(s);
    const long t = y[i];
    const bool valid = t != -100;
    const long tc = t < 0 ? 0 : (t >= K ? K - 1 : t);
    const float nll = (t >= 0 && t < K) ? lse - zr[tc] : NAN;
    ws[i] = lse;
    ws[B + i] = valid ? nll : 0.f;
    ws[2 * B + i] = valid ? (float)K * lse - sz : 0.f;
    ws[3 * B + i] = valid ? 1.f : 0.f;
    ws[4 * B + 1 + i] = (valid && (t < 0 || t >= K)) ? 1.f : 0.f;
  }
}

__global__ __launch_bounds__(256) void ce_final_kernel(float* __restrict__ ws, int B, int K, float ls,
                                                       float* __restrict__ loss, float* __restrict__ found,
                                                       float* __restrict__ bad_labels) {
  __shared__ double part[4][256];
  double a = 0.0, b = 0.0, n = 0.0, nb = 0.0;
  for (int i = threadIdx.x; i < B; i += 256) {
    a += (double)ws[B + i];
    b += (double)ws[2 * B + i];
    n += (double)ws[3 * B + i];
    nb += (double)ws[4 * B + 1 + i];
  }
  part[0][threadIdx.x] = a;
  part[1][threadIdx.x] = b;
  part[2][threadIdx.x] = n;
  part[3][threadIdx.x] = nb;
  __syncthreads();
  for (int h = 128; h > 0; h >>= 1) {
    if ((int)threadIdx.x < h) {
      part[0][threadIdx.x] += part[0][threadIdx.x + h];
      part[1][threadIdx.x] += part[1][threadIdx.x + h];
      part[2][threadIdx.x] += part[2][threadIdx.x + h];
      part[3][threadIdx.x] += part[3][threadIdx.x + h];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    const double nv = part[2][0];
    const float l = (float)((1.0 - (double)ls) * (part[0][0] / nv) + ((double)ls / K) * (part[1][0] / nv));
    *loss = l;
    ws[4 * B] = (float)nv;
    if (found) *found = __builtin_isfinite(l) ? 0.f : 1.f;
    if (bad_labels) *bad_labels += (float)part[3][0];    // accumulates over steps until the host reads it
  }
}

// dz[i, k] = g / n * (exp(z - lse_i) - (1 - ls) [k == y_i] - ls / K), a thread per 4 logits
__global__ __launch_bounds__(256) void ce_ls_bwd_kernel(const float* __restrict__ z, const int64_t* __restrict__ y,
                                                        const float* __restrict__ ws, const float* __restrict__ gout,
                                                        int B, int K, float ls, float* __restrict__ dz) {
  const long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const long e0 = idx * 4;
  if (e0 >= (long)B * K) return;
  const float g = *gout / ws[4 * B];
  const float off = ls / (float)K, hot = 1.f - ls;
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const long e = e0 + u;
    if (e >= (long)B * K) break;
    const long i = e / K;
    const int k = (int)(e - i * K);
    const long t = y[i];
    float d = 0.f;
    if (t != -100) {
      d = expf(z[e] - ws[i]) - off - (k == t ? hot : 0.f);
      if (t < 0 || t >= K) d = NAN;
      d *= g;
    }
    dz[e] = d;
  }
}

}  // namespace ogv

using namespace ogv;

extern "C" size_t ogv_ce_ls_ws_bytes(int B) { return (size_t)(B > 0 ? 5 * B + 1 : 1) * sizeof(float); }

extern "C" int ogv_ce_ls_fwd(const float* logits, const int64_t* target, int B, int K, float label_smoothing,
                             float* loss, float* ws, float* found, float* bad_labels, void* stream) {
  OGV_REQUIRE(logits && target && loss && ws, "ogv_ce_ls_fwd: null pointer");
  OGV_REQUIRE(B > 0 && K > 0, "ogv_ce_ls_fwd: bad shape B=%d K=%d", B, K);
  OGV_REQUIRE(label_smoothing >= 0.f && label_smoothing <= 1.f, "ogv_ce_ls_fwd: label_smoothing %g not in [0, 1]",
              (double)label_smoothing);
  ce_rows_kernel<<<cdiv(B, 4), 256, 0, as_stream(stream)>>>(logits, target, B, K, ws);
  ce_final_kernel<<<1, 256, 0, as_stream(stream)>>>(ws, B, K, label_smoothing, loss, found, bad_labels);
  return check_launch("ogv_ce_ls_fwd");
}

extern "C" int ogv_ce_ls_bwd(const float* logits, const int64_t* target, const float* ws, const float* grad_loss,
                             int B, int K, float label_smoothing, float* dlogits, void* stream) {
  OGV_REQUIRE(logits && target && ws && grad_loss && dlogits, "ogv_ce_ls_bwd: null pointer");
  OGV_REQUIRE(B > 0 && K > 0, "ogv_ce_ls_bwd: bad shape B=%d K=%d", B, K);
  const long n4 = ((long)B * K + 3) / 4;
  ce_ls_bwd_kernel<<<(unsigned)((n4 + 255) / 256), 256, 0, as_stream(stream)>>>(logits, target, ws, grad_loss, B, K,
                                                                                label_smoothing, dlogits);
  return check_launch("ogv_ce_ls_bwd");
}
