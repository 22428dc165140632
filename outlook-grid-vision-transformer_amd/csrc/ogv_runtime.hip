// Library runtime: version, thread-local last error, launch checking, dtype casts.
#include "ogv_common.h"
#include "ogv_gemm.h"

#include <cstring>
#include <mutex>
#include <vector>

namespace ogv {

void set_bn_red_rg(int v);   // ogv_mbconv.hip
void set_opt_chunk(int v);   // ogv_optim.hip
void set_mb_a3(int v);       // ogv_mbconv.hip

static thread_local char g_err[512] = "";

void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}

static thread_local const char* g_refused = nullptr;   // a launch skipped because its LDS grant was refused

int check_launch(const char* what) {
  if (g_refused) {
    set_error("%s: %s not launched: dynamic LDS grant refused", what, g_refused);
    g_refused = nullptr;
    return OGV_ERR_LAUNCH;
  }
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    set_error("%s: launch failed: %s", what, hipGetErrorString(e));
    return OGV_ERR_LAUNCH;
  }
  return OGV_OK;
}

bool lds_160k() {
  int dev = 0, n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n == 0) {   // no device: a pure shape query (nothing can launch)
    (void)hipGetLastError();
    return true;
  }
  if (hipGetDevice(&dev) != hipSuccess) return false;
  static std::mutex mu;
  static std::vector<std::pair<int, bool>> seen;
  std::lock_guard<std::mutex> lock(mu);
  for (const auto& d : seen)
    if (d.first == dev) return d.second;
  int optin = 0;
  const bool ok = hipDeviceGetAttribute(&optin, hipDeviceAttributeSharedMemPerBlockOptin, dev) == hipSuccess &&
                  optin >= 160 * 1024;
  if (!ok) (void)hipGetLastError();
  seen.emplace_back(dev, ok);
  return ok;
}

bool lds_grant(const void* kern, size_t bytes) {
  if (bytes <= 64 * 1024) return true;   // the default grant
  if (bytes > 160 * 1024 || !lds_160k()) return false;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return false;
  struct Grant { const void* kern; int dev; bool ok; };
  static std::mutex mu;
  static std::vector<Grant> done;
  std::lock_guard<std::mutex> lock(mu);
  for (const Grant& g : done)
    if (g.kern == kern && g.dev == dev) return g.ok;
  const bool ok = hipFuncSetAttribute(kern, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024) == hipSuccess;
  if (!ok) (void)hipGetLastError();
  done.push_back(Grant{kern, dev, ok});
  return ok;
}

bool lds_ok(const void* kern, size_t bytes, const char* kname) {
  if (lds_grant(kern, bytes)) return true;
  g_refused = kname;
  return false;
}

template <typename S, typename D>
__global__ void cast_kernel(const S* __restrict__ src, D* __restrict__ dst, size_t n) {
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  for (; i < n; i += stride) dst[i] = from_f<D>(to_f(src[i]));
}

__global__ void step_flag_kernel(const float* __restrict__ x, int mode, float* __restrict__ found) {
  const float v = *x;
  *found = (mode == 0 ? !__builtin_isfinite(v) : v > 0.f) ? 1.f : 0.f;
}

struct LrGroups {
  float* lr[OGV_MAX_LR_GROUPS];
  float base[OGV_MAX_LR_GROUPS];
};

// warmup.py:38-52 in fp64 (the host formula), one thread
__global__ void schedule_step_kernel(const float* __restrict__ found, float* counter, float* nonfinite, LrGroups g,
                                     int n, int warmup, int total, float min_lr) {
  const float f = *found;
  *nonfinite += f;
  const float t = *counter + (1.f - f);
  *counter = t;
  const double td = (double)t;
  for (int i = 0; i < n; ++i) {
    const double base = g.base[i];
    double lr;
    if (warmup > 0 && td <= (double)warmup) {
      lr = base * (td / (double)warmup);
    } else {
      const double tt = td < (double)total ? td : (double)total;
      const double prog = (tt - (double)warmup) / (double)(total - warmup > 1 ? total - warmup : 1);
      lr = (double)min_lr + (base - (double)min_lr) * 0.5 * (1.0 + cos(3.14159265358979323846 * prog));
    }
    *g.lr[i] = (float)lr;
  }
}

}  // namespace ogv

using namespace ogv;

extern "C" int ogv_step_flag(const float* x, int mode, float* found, void* stream) {
  OGV_REQUIRE(x && found, "ogv_step_flag: null pointer");
  OGV_REQUIRE(mode == 0 || mode == 1, "ogv_step_flag: mode %d (0 = non-finite, 1 = positive)", mode);
  step_flag_kernel<<<1, 1, 0, as_stream(stream)>>>(x, mode, found);
  return check_launch("ogv_step_flag");
}

extern "C" int ogv_schedule_step(const float* found, float* counter, float* nonfinite, float* const* lr,
                                 const float* base_lr, int n_groups, int warmup_steps, int total_steps, float min_lr,
                                 void* stream) {
  OGV_REQUIRE(found && counter && nonfinite && lr && base_lr, "ogv_schedule_step: null pointer");
  OGV_REQUIRE(n_groups >= 0 && n_groups <= OGV_MAX_LR_GROUPS, "ogv_schedule_step: %d groups (max %d)", n_groups,
              OGV_MAX_LR_GROUPS);
  LrGroups g;
  for (int i = 0; i < OGV_MAX_LR_GROUPS; ++i) {
    g.lr[i] = i < n_groups ? lr[i] : nullptr;
    g.base[i] = i < n_groups ? base_lr[i] : 0.f;
  }
  for (int i = 0; i < n_groups; ++i) OGV_REQUIRE(g.lr[i], "ogv_schedule_step: null lr pointer %d", i);
  schedule_step_kernel<<<1, 1, 0, as_stream(stream)>>>(found, counter, nonfinite, g, n_groups, warmup_steps,
                                                      total_steps, min_lr);
  return check_launch("ogv_schedule_step");
}

extern "C" const char* ogv_version(void) { return "ogv-hip 0.1.0 (gfx950)"; }
extern "C" const char* ogv_last_error(void) { return g_err; }

extern "C" int ogv_set_option(const char* name, int value) {
  OGV_REQUIRE(name, "ogv_set_option: null name");
  if (!strcmp(name, "sgemm")) {
    set_sgemm_mode(value ? 1 : 0);
    return OGV_OK;
  }
  if (!strcmp(name, "grid_big")) {
    set_grid_big(value);
    return OGV_OK;
  }
  if (!strcmp(name, "grid_lds")) {
    set_grid_lds(value ? 1 : 0);
    return OGV_OK;
  }
  if (!strcmp(name, "gemm_bn64")) {
    set_gemm_bn64(value ? 1 : 0);
    return OGV_OK;
  }
  if (!strcmp(name, "ln_bwd_blocks")) {
    set_ln_bwd_blocks(value);
    return OGV_OK;
  }
  if (!strcmp(name, "mb_side")) {
    set_mb_side(value ? 1 : 0);
    return OGV_OK;
  }
  if (!strcmp(name, "ln_rpi")) {
    set_ln_rpi(value);
    return OGV_OK;
  }
  if (!strcmp(name, "dw_tw")) {
    set_dw_tw(value);
    return OGV_OK;
  }
  if (!strcmp(name, "dw_blocks")) {
    set_dw_blocks(value);
    return OGV_OK;
  }
  if (!strcmp(name, "grid_mfma")) {
    set_grid_mfma(value ? 1 : 0);
    return OGV_OK;
  }
  if (!strcmp(name, "bm64_max_m")) {
    set_bm64_max_m(value);
    return OGV_OK;
  }
  if (!strcmp(name, "bk64_max_m")) {
    set_bk64_max_m(value);
    return OGV_OK;
  }
  if (!strcmp(name, "splitk_max")) {
    set_splitk_max(value);
    return OGV_OK;
  }
  if (!strcmp(name, "sg_prefetch")) {
    set_sg_prefetch(value);
    return OGV_OK;
  }
  if (!strcmp(name, "sg_per_cu")) {
    set_sg_per_cu(value);
    return OGV_OK;
  }
  if (!strcmp(name, "outlook_tile")) {
    set_outlook_tile(value);
    return OGV_OK;
  }
  if (!strcmp(name, "outlook_vproj")) {
    set_outlook_vproj(value);
    return OGV_OK;
  }
  if (!strcmp(name, "swg_min_m")) {
    set_swg_min_m(value);
    return OGV_OK;
  }
  if (!strcmp(name, "wg2")) {
    set_wg2(value);
    return OGV_OK;
  }
  if (!strcmp(name, "wg2_blocks")) {
    set_wg2_blocks(value);
    return OGV_OK;
  }
  if (!strcmp(name, "wg2_pbeta")) {
    set_wg2_pbeta(value);
    return OGV_OK;
  }
  if (!strcmp(name, "wg2_tile")) {
    set_wg2_tile(value);
    return OGV_OK;
  }
  if (!strcmp(name, "skip")) {
    set_skip(value);
    return OGV_OK;
  }
  if (!strcmp(name, "dw_fuse")) {
    set_dw_fuse(value);
    return OGV_OK;
  }
  if (!strcmp(name, "stem_wgs")) {
    set_stem_wgs(value);
    return OGV_OK;
  }
  if (!strcmp(name, "stem")) {
    set_stem(value);
    return OGV_OK;
  }
  if (!strcmp(name, "dw_bwd_r")) {
    set_dw_bwd_r(value);
    return OGV_OK;
  }
  if (!strcmp(name, "opt_chunk")) {
    set_opt_chunk(value);
    return OGV_OK;
  }
  if (!strcmp(name, "bn_red_rg")) {
    set_bn_red_rg(value);
    return OGV_OK;
  }
  if (!strcmp(name, "mb_a3")) {
    set_mb_a3(value);
    return OGV_OK;
  }
  if (!strcmp(name, "pg_conv_rs1")) {
    set_pg_conv_rs1(value);
    return OGV_OK;
  }
  if (!strcmp(name, "bn_slices")) {
    set_bn_slices(value);
    return OGV_OK;
  }
  if (!strcmp(name, "dw_fwd_r")) {
    set_dw_fwd_r(value);
    return OGV_OK;
  }
  if (!strcmp(name, "dw_bn2")) {
    set_dw_bn2(value);
    return OGV_OK;
  }
  if (!strcmp(name, "se_gemv")) {
    set_se_gemv(value);
    return OGV_OK;
  }
  if (!strcmp(name, "vp_dbg")) {
    set_vp_dbg(value);
    return OGV_OK;
  }
  if (!strcmp(name, "wg2_fuse")) {
    set_wg2_fuse(value);
    return OGV_OK;
  }
  if (!strcmp(name, "wg2_conv")) {
    set_wg2_conv(value);
    return OGV_OK;
  }
  if (!strcmp(name, "vp_big")) {
    set_vp_big(value);
    return OGV_OK;
  }
  if (!strcmp(name, "vp_head")) {
    set_vp_head(value);
    return OGV_OK;
  }
  if (!strcmp(name, "vph_wgs")) {
    set_vph_wgs(value);
    return OGV_OK;
  }
  if (!strcmp(name, "ln_epi")) {
    set_ln_epi(value);
    return OGV_OK;
  }
  if (!strcmp(name, "pg_tconv1")) {
    set_pg_tconv1(value);
    return OGV_OK;
  }
  if (!strcmp(name, "vp_l32")) {
    set_vp_l32(value);
    return OGV_OK;
  }
  if (!strcmp(name, "vph_halo")) {
    set_vph_halo(value);
    return OGV_OK;
  }
  if (!strcmp(name, "vph_tile")) {
    set_vph_tile(value);
    return OGV_OK;
  }
  if (!strcmp(name, "vph_dbg")) {
    set_vph_dbg(value);
    return OGV_OK;
  }
  if (!strcmp(name, "vph_rows")) {
    set_vph_rows(value);
    return OGV_OK;
  }
  if (!strcmp(name, "vp_tile")) {
    set_vp_tile(value);
    return OGV_OK;
  }
  if (!strcmp(name, "pg_split")) {
    set_pg_split(value);
    return OGV_OK;
  }
  if (!strcmp(name, "split_w")) {
    set_split_w(value);
    return OGV_OK;
  }
  if (!strcmp(name, "pgemm")) {
    set_pgemm(value ? 1 : 0);
    return OGV_OK;
  }
  if (!strcmp(name, "sg_wgs")) {
    set_sg_wgs(value);
    return OGV_OK;
  }
  if (!strcmp(name, "wg_blocks")) {
    set_wg_blocks(value);
    return OGV_OK;
  }
  if (!strcmp(name, "wg_tile")) {
    set_wg_tile(value);
    return OGV_OK;
  }
  if (!strcmp(name, "pg_lds_kb")) {
    set_pg_lds_kb(value);
    return OGV_OK;
  }
  if (!strcmp(name, "pg_dbg")) {
    set_pg_dbg(value);
    return OGV_OK;
  }
  if (!strcmp(name, "pg_per_cu")) {
    set_pg_per_cu(value);
    return OGV_OK;
  }
  if (!strcmp(name, "pg_rs")) {
    set_pg_rs(value == 1 || value == 2 ? value : 0);
    return OGV_OK;
  }
  if (!strcmp(name, "pg_pa_wide")) {
    set_pg_pa_wide(value);
    return OGV_OK;
  }
  if (!strcmp(name, "pg_tn4_max_m")) {
    set_pg_tn4_max_m(value);
    return OGV_OK;
  }
  if (!strcmp(name, "pg_tn")) {
    set_pg_tn(value == 4 || value == 8 || value == 12 ? value : 0);
    return OGV_OK;
  }
  if (!strcmp(name, "sgemm_min_m")) {
    set_sgemm_min_m(value);
    return OGV_OK;
  }
  set_error("ogv_set_option: unknown option '%s'", name);
  return OGV_ERR_ARG;
}

extern "C" int ogv_cast(const void* src, ogv_dtype sdt, void* dst, ogv_dtype ddt, size_t n, void* stream) {
  OGV_REQUIRE(src && dst, "ogv_cast: null pointer");
  if (n == 0) return OGV_OK;
  const unsigned grid = (unsigned)((n + 255) / 256 < 4096 ? (n + 255) / 256 : 4096);
  hipStream_t s = as_stream(stream);
  if (sdt == OGV_F32 && ddt == OGV_BF16)
    cast_kernel<float, bf16><<<grid, 256, 0, s>>>((const float*)src, (bf16*)dst, n);
  else if (sdt == OGV_BF16 && ddt == OGV_F32)
    cast_kernel<bf16, float><<<grid, 256, 0, s>>>((const bf16*)src, (float*)dst, n);
  else if (sdt == OGV_F32 && ddt == OGV_F32)
    cast_kernel<float, float><<<grid, 256, 0, s>>>((const float*)src, (float*)dst, n);
  else
    cast_kernel<bf16, bf16><<<grid, 256, 0, s>>>((const bf16*)src, (bf16*)dst, n);
  return check_launch("ogv_cast");
}

// ---------------------------------------------------------------- batched segment copies
// The data-parallel gradient exchange packs every parameter gradient (and the BatchNorm buffers)
// into one flat bucket and unpacks it after the all_reduce.  torch.cat / _foreach_copy_ do that as
// one hipMemcpyAsync per tensor (~290 copy dispatches per step for Model-A-7M, 1.1 ms of a 16.3 ms
// step at world size 1, profiles/r04_dp_*); here a launch takes 64 segments in its kernel arguments
// (graph-capturable, no table upload) and one workgroup copies one 8192-element chunk.
namespace ogv {

constexpr int CPY_CHUNK = 8192;
constexpr int CPY_MAXS = 64;

struct CopyBatch {
  const float* src[CPY_MAXS];
  float* dst[CPY_MAXS];
  int numel[CPY_MAXS];
  int chunk_end[CPY_MAXS];   // exclusive prefix of chunks within this launch
  int n;
};

__global__ __launch_bounds__(256) void copy_batch_kernel(CopyBatch b, float scale) {
  const int chunk = blockIdx.x;
  int t = 0;
  while (t + 1 < b.n && b.chunk_end[t] <= chunk) ++t;
  const long e0 = (long)(chunk - (t ? b.chunk_end[t - 1] : 0)) * CPY_CHUNK;
  const int n = (int)min((long)CPY_CHUNK, (long)b.numel[t] - e0);
  const float* __restrict__ s = b.src[t] ? b.src[t] + e0 : nullptr;
  float* __restrict__ d = b.dst[t] + e0;
  if (!s) {   // zero fill (a parameter that received no gradient)
    for (int i = threadIdx.x; i < n; i += blockDim.x) d[i] = 0.f;
    return;
  }
  int done = 0;
  if (((reinterpret_cast<uintptr_t>(s) | reinterpret_cast<uintptr_t>(d)) & 15) == 0) {
    const int n4 = n >> 2;
    for (int i = threadIdx.x; i < n4; i += blockDim.x) {
      float4 v = reinterpret_cast<const float4*>(s)[i];
      if (scale != 1.f) v = make_float4(v.x * scale, v.y * scale, v.z * scale, v.w * scale);
      reinterpret_cast<float4*>(d)[i] = v;
    }
    done = n4 << 2;
  }
  for (int i = done + threadIdx.x; i < n; i += blockDim.x) d[i] = scale != 1.f ? s[i] * scale : s[i];
}

}  // namespace ogv

extern "C" int ogv_copy_batch_f32(const ogv_copy_seg* segs, int n, float scale, void* stream) {
  OGV_REQUIRE(n >= 0 && (n == 0 || segs), "ogv_copy_batch_f32: segment table");
  hipStream_t s = as_stream(stream);
  CopyBatch b;
  std::memset(&b, 0, sizeof(b));
  auto flush = [&]() {
    if (b.n) copy_batch_kernel<<<(unsigned)b.chunk_end[b.n - 1], 256, 0, s>>>(b, scale);
    std::memset(&b, 0, sizeof(b));
  };
  for (int i = 0; i < n; ++i) {
    const ogv_copy_seg& g = segs[i];
    OGV_REQUIRE(g.dst, "ogv_copy_batch_f32: null destination (segment %d)", i);
    OGV_REQUIRE(g.numel >= 0 && g.numel < (1LL << 31), "ogv_copy_batch_f32: numel (segment %d)", i);
    if (g.numel == 0) continue;
    if (b.n == CPY_MAXS) flush();
    const int k = b.n++;
    b.src[k] = g.src;
    b.dst[k] = g.dst;
    b.numel[k] = (int)g.numel;
    b.chunk_end[k] = (k ? b.chunk_end[k - 1] : 0) + (int)((g.numel + CPY_CHUNK - 1) / CPY_CHUNK);
  }
  flush();
  return check_launch("ogv_copy_batch_f32");
}
