// Library runtime: version, thread-local last error, launch checking, dtype casts.
#include "ogv_common.h"
#include "ogv_gemm.h"

namespace ogv {

static thread_local char g_err[512] = "";

void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}

int check_launch(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    set_error("%s: launch failed: %s", what, hipGetErrorString(e));
    return OGV_ERR_LAUNCH;
  }
  return OGV_OK;
}

template <typename S, typename D>
__global__ void cast_kernel(const S* __restrict__ src, D* __restrict__ dst, size_t n) {
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  for (; i < n; i += stride) dst[i] = from_f<D>(to_f(src[i]));
}

}  // namespace ogv

using namespace ogv;

extern "C" const char* ogv_version(void) { return "ogv-hip 0.1.0 (gfx950)"; }
extern "C" const char* ogv_last_error(void) { return g_err; }

extern "C" int ogv_set_option(const char* name, int value) {
  OGV_REQUIRE(name, "ogv_set_option: null name");
  if (!strcmp(name, "sgemm")) {
    set_sgemm_mode(value ? 1 : 0);
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
  if (!strcmp(name, "dw_blocks")) {
    set_dw_blocks(value);
    return OGV_OK;
  }
  if (!strcmp(name, "grid_mfma")) {
    set_grid_mfma(value ? 1 : 0);
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
