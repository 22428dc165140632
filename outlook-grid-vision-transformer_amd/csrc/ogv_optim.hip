// Clip-by-global-norm + AdamW over the parameter tensors of a training step, as two kinds of native
// launches: what the reference's training loop does with
//   torch.nn.utils.clip_grad_norm_(model.parameters(), max_norm)   src/training/one_epoch_train.py:121
//   torch.optim.AdamW(...).step()                                  src/training/train_full_model.py
// and what ogv/train.py did with torch's foreach norm / mul launches and its fused AdamW (9 + ~17
// launches, 0.36 ms per Model-A-7M step for ~35 us of HBM traffic).
//
// The tensor table travels in kernel arguments (64 tensors per launch, AdamWBatch below), so a
// hipGraph captured over a step bakes the parameter / gradient / moment pointers into its nodes
// and no host->device table copy is needed.  Work unit = one chunk of up to opt_chunk elements of
// one tensor (one workgroup).
//   pass 1 (adamw_norm_kernel): per-chunk sum of grad^2 -> norm_ws[chunk]; the first workgroup of
//          each launch advances its tensors' step counters unless found_inf is set;
//   pass 2 (adamw_update_kernel): every workgroup reduces the whole norm_ws in the same order (the
//          same clip coefficient everywhere, deterministic), returns at once when found_inf is
//          set, else g = grad * coef (written back: clip_grad_norm_ scales .grad in place) and the
//          AdamW update of torch's fused kernel (decoupled weight decay, bias corrections from the
//          tensor's step counter, fp32 math).
#include "ogv_common.h"

#include <cstring>
#include <vector>

namespace ogv {

constexpr int OPT_MAXT = 64;
// knob "opt_chunk": elements per workgroup (a power of two, 1024-16384; default 2048: more workgroups per launch)
static int g_opt_chunk = 2048;   // 7M step, 30 steps: 8192 14.831 / 14.825, 4096 14.814, 2048 14.810 / 14.815, 1024 14.831 ms (profiles/r05t_opt_chunk.log)
void set_opt_chunk(int v) {
  int c = 1024;
  while (c < v && c < 16384) c <<= 1;
  g_opt_chunk = c;
}

struct AdamWBatch {
  float* p[OPT_MAXT];
  float* g[OPT_MAXT];
  float* m[OPT_MAXT];
  float* v[OPT_MAXT];
  float* step[OPT_MAXT];
  int numel[OPT_MAXT];
  int chunk_end[OPT_MAXT];       // exclusive prefix of chunks within this launch
  unsigned char group[OPT_MAXT];
  int n;                         // tensors in this launch
  int chunk_base;                // global index of this launch's first chunk in norm_ws
  int csz;                       // elements per chunk
};

struct AdamWGroups {
  const float* lr[4];
  float wd[4], beta1[4], beta2[4], eps[4], omb1[4], omb2[4];
};

__device__ __forceinline__ int opt_find(const AdamWBatch& b, int chunk) {
  int t = 0;
  while (t + 1 < b.n && b.chunk_end[t] <= chunk) ++t;
  return t;
}

__device__ __forceinline__ float opt_block_sum(float x, float* red) {
  for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o, 64);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  if (lane == 0) red[wave] = x;
  __syncthreads();
  float s = 0.f;
  if (threadIdx.x == 0) {
    for (int w = 0; w < (int)(blockDim.x >> 6); ++w) s += red[w];
    red[0] = s;
  }
  __syncthreads();
  s = red[0];
  __syncthreads();
  return s;
}

__global__ __launch_bounds__(256) void adamw_norm_kernel(AdamWBatch b, const float* __restrict__ found,
                                                         float* __restrict__ norm_ws) {
  __shared__ float red[4];
  const int chunk = blockIdx.x;
  const int t = opt_find(b, chunk);
  const int c0 = t ? b.chunk_end[t - 1] : 0;
  const long e0 = (long)(chunk - c0) * b.csz;
  const int n = min((long)b.csz, (long)b.numel[t] - e0);
  const float* __restrict__ g = b.g[t] + e0;
  float s = 0.f;
  if ((reinterpret_cast<uintptr_t>(g) & 15) == 0) {
    const int n4 = n >> 2;
    for (int i = threadIdx.x; i < n4; i += blockDim.x) {
      const float4 x = reinterpret_cast<const float4*>(g)[i];
      s += x.x * x.x + x.y * x.y + x.z * x.z + x.w * x.w;
    }
    for (int i = (n4 << 2) + threadIdx.x; i < n; i += blockDim.x) s += g[i] * g[i];
  } else {
    for (int i = threadIdx.x; i < n; i += blockDim.x) s += g[i] * g[i];
  }
  s = opt_block_sum(s, red);
  if (threadIdx.x == 0) norm_ws[b.chunk_base + chunk] = s;
  if (blockIdx.x == 0 && threadIdx.x < b.n && !(found && *found != 0.f)) b.step[threadIdx.x][0] += 1.f;
}

__global__ __launch_bounds__(256) void adamw_update_kernel(AdamWBatch b, AdamWGroups G, const float* __restrict__ found,
                                                           const float* __restrict__ norm_ws, int nchunks,
                                                           float max_norm) {
  __shared__ float red[4];
  if (found && *found != 0.f) return;   // uniform over the grid: skipped step
  float coef = 1.f;
  if (max_norm >= 0.f) {   // < 0: no clipping (grad_clip_norm=None)
    float s = 0.f;
    for (int i = threadIdx.x; i < nchunks; i += blockDim.x) s += norm_ws[i];
    s = opt_block_sum(s, red);
    // torch: clip_coef = max_norm / (total_norm + 1e-6), clamped to <= 1 (NaN propagates)
    coef = max_norm / (sqrtf(s) + 1e-6f);
    if (coef > 1.f) coef = 1.f;
  }
  const int chunk = blockIdx.x;
  const int t = opt_find(b, chunk);
  const int c0 = t ? b.chunk_end[t - 1] : 0;
  const long e0 = (long)(chunk - c0) * b.csz;
  const int n = min((long)b.csz, (long)b.numel[t] - e0);
  const int gi = b.group[t];
  const float lr = *G.lr[gi], wd = G.wd[gi], b1 = G.beta1[gi], b2 = G.beta2[gi], eps = G.eps[gi];
  const float omb1 = G.omb1[gi], omb2 = G.omb2[gi];
  const float stp = *b.step[t];
  const float bc1 = 1.f - powf(b1, stp), bc2 = 1.f - powf(b2, stp);
  const float step_size = lr / bc1, bc2_sqrt = sqrtf(bc2);
  float* __restrict__ P = b.p[t] + e0;
  float* __restrict__ Gp = b.g[t] + e0;
  float* __restrict__ M = b.m[t] + e0;
  float* __restrict__ V = b.v[t] + e0;
  auto upd = [&](float& p, float& g, float& m, float& v) {
    g *= coef;
    p -= lr * wd * p;
    m = b1 * m + omb1 * g;
    v = b2 * v + omb2 * g * g;
    const float denom = sqrtf(v) / bc2_sqrt + eps;
    p -= step_size * m / denom;
  };
  const bool vec = ((reinterpret_cast<uintptr_t>(P) | reinterpret_cast<uintptr_t>(Gp) | reinterpret_cast<uintptr_t>(M) |
                     reinterpret_cast<uintptr_t>(V)) & 15) == 0;
  int done = 0;
  if (vec) {
    const int n4 = n >> 2;
    for (int i = threadIdx.x; i < n4; i += blockDim.x) {
      float4 p = reinterpret_cast<float4*>(P)[i], g = reinterpret_cast<float4*>(Gp)[i];
      float4 m = reinterpret_cast<float4*>(M)[i], v = reinterpret_cast<float4*>(V)[i];
      upd(p.x, g.x, m.x, v.x);
      upd(p.y, g.y, m.y, v.y);
      upd(p.z, g.z, m.z, v.z);
      upd(p.w, g.w, m.w, v.w);
      reinterpret_cast<float4*>(P)[i] = p;
      reinterpret_cast<float4*>(Gp)[i] = g;
      reinterpret_cast<float4*>(M)[i] = m;
      reinterpret_cast<float4*>(V)[i] = v;
    }
    done = n4 << 2;
  }
  for (int i = done + threadIdx.x; i < n; i += blockDim.x) {
    float p = P[i], g = Gp[i], m = M[i], v = V[i];
    upd(p, g, m, v);
    P[i] = p;
    Gp[i] = g;
    M[i] = m;
    V[i] = v;
  }
}

static int opt_chunks(long long numel) { return (int)((numel + g_opt_chunk - 1) / g_opt_chunk); }

}  // namespace ogv

using namespace ogv;

extern "C" size_t ogv_clip_adamw_ws_bytes(const ogv_adamw_tensor* tensors, int n) {
  long long c = 0;
  for (int i = 0; i < n; ++i) c += opt_chunks(tensors[i].numel);
  return (size_t)(c > 0 ? c : 1) * sizeof(float);
}

extern "C" int ogv_clip_adamw(const ogv_adamw_tensor* tensors, int n, const ogv_adamw_group* groups, int ngroups,
                              const float* found_inf, float max_norm, float* norm_ws, void* stream) {
  OGV_REQUIRE(n >= 0 && (n == 0 || tensors), "ogv_clip_adamw: tensor table");
  OGV_REQUIRE(ngroups >= 1 && ngroups <= 4 && groups, "ogv_clip_adamw: 1-4 parameter groups");
  OGV_REQUIRE(norm_ws, "ogv_clip_adamw: norm workspace");
  if (n == 0) return OGV_OK;
  AdamWGroups G{};
  for (int i = 0; i < ngroups; ++i) {
    OGV_REQUIRE(groups[i].lr, "ogv_clip_adamw: group lr tensor");
    G.lr[i] = groups[i].lr;
    G.wd[i] = groups[i].weight_decay;
    G.beta1[i] = groups[i].beta1;
    G.beta2[i] = groups[i].beta2;
    G.eps[i] = groups[i].eps;
    G.omb1[i] = groups[i].one_minus_beta1;
    G.omb2[i] = groups[i].one_minus_beta2;
  }
  std::vector<AdamWBatch> batches;
  int total = 0;
  for (int i = 0; i < n; ++i) {
    const ogv_adamw_tensor& T = tensors[i];
    OGV_REQUIRE(T.param && T.grad && T.exp_avg && T.exp_avg_sq && T.step, "ogv_clip_adamw: null tensor pointer");
    OGV_REQUIRE(T.numel > 0 && T.numel < (1LL << 31), "ogv_clip_adamw: numel");
    OGV_REQUIRE(T.group >= 0 && T.group < ngroups, "ogv_clip_adamw: group index");
    if (batches.empty() || batches.back().n == OPT_MAXT) {
      batches.emplace_back();
      std::memset(&batches.back(), 0, sizeof(AdamWBatch));
      batches.back().chunk_base = total;
      batches.back().csz = g_opt_chunk;
    }
    AdamWBatch& b = batches.back();
    const int k = b.n++;
    b.p[k] = T.param;
    b.g[k] = T.grad;
    b.m[k] = T.exp_avg;
    b.v[k] = T.exp_avg_sq;
    b.step[k] = T.step;
    b.numel[k] = (int)T.numel;
    b.group[k] = (unsigned char)T.group;
    const int c = opt_chunks(T.numel);
    b.chunk_end[k] = (k ? b.chunk_end[k - 1] : 0) + c;
    total += c;
  }
  hipStream_t s = as_stream(stream);
  for (const AdamWBatch& b : batches)
    adamw_norm_kernel<<<(unsigned)b.chunk_end[b.n - 1], 256, 0, s>>>(b, found_inf, norm_ws);
  for (const AdamWBatch& b : batches)
    adamw_update_kernel<<<(unsigned)b.chunk_end[b.n - 1], 256, 0, s>>>(b, G, found_inf, norm_ws, total, max_norm);
  return check_launch("ogv_clip_adamw");
}
