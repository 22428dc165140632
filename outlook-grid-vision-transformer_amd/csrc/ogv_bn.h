// BatchNorm building blocks shared by the fused MBConv and the conv/BN/act ops.
#pragma once
#include "ogv_common.h"

namespace ogv {

// Sum q[NQ][V] over the 64 slots of each of the 4 channel chunks (chunk = tid & 3,
// slot = tid >> 2): xor-shuffles over lane bits 2..5 inside each wave, then the 4 waves through
// LDS (4*NQ*4*V floats; the LDS may be reused).  out[k*qstride + c], c = cbase + chunk*V + i < C.
template <int NQ, int V, typename A = float>
__device__ __forceinline__ void chunk_reduce_store(A (&q)[NQ][V], A* lds, A* out, long qstride, int C, int cbase,
                                                   const float* gate = nullptr, float* dz = nullptr) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
  for (int k = 0; k < NQ; ++k)
#pragma unroll
    for (int i = 0; i < V; ++i) {
      A v = q[k][i];
      v += __shfl_xor(v, 4, 64);
      v += __shfl_xor(v, 8, 64);
      v += __shfl_xor(v, 16, 64);
      v += __shfl_xor(v, 32, 64);
      q[k][i] = v;
    }
  __syncthreads();
  if (lane < 4) {
#pragma unroll
    for (int k = 0; k < NQ; ++k)
#pragma unroll
      for (int i = 0; i < V; ++i) lds[((wave * NQ + k) * 4 + lane) * V + i] = q[k][i];
  }
  __syncthreads();
  for (int idx = threadIdx.x; idx < NQ * 4 * V; idx += 256) {
    const int k = idx / (4 * V), r = idx - k * 4 * V;
    const int ch = r / V, i = r - ch * V;
    A sum = 0;
#pragma unroll
    for (int w = 0; w < 4; ++w) sum += lds[((w * NQ + k) * 4 + ch) * V + i];
    const int c = cbase + ch * V + i;
    if (c < C) {
      out[(long)k * qstride + c] = sum;
      // SE: quantity 0 is dgate; dz2 = dgate * g * (1 - g) (the sigmoid backward, fused)
      if (dz && k == 0) dz[c] = (float)sum * gate[c] * (1.f - gate[c]);
    }
  }
}

// Train: batch mean/var from fp64 sums [sum(x - rm), sum((x - rm)^2)] (shift = running mean
// before its update; fp64 so the variance does not cancel when the batch mean is far from the
// shift), running-stat update (momentum, unbiased var); eval: running stats.
// Writes mean, invstd and the apply coefficients sc = gamma*invstd, sh = beta - mean*sc.
void bn_finalize_launch(const double* sums, int K, double n, const float* gamma, const float* beta, float eps,
                        float momentum, float* rm, float* rv, float* mean, float* invstd, float* sc, float* sh, int train,
                        hipStream_t s);
// From S = [sum dz, sum dz*xhat]: dgamma, dbeta and coef = [gamma*invstd, S0/n, S1/n] (train) or
// [gamma*invstd, 0, 0] (eval);  dx = coef0 * (dz - coef1 - xhat*coef2).
void bn_coeffs_launch(const float* S, int K, float n, const float* gamma, const float* invstd, float* dgamma,
                      float* dbeta, float* coef, int train, hipStream_t s);
// The column reduction of R partial rows ([R][ld]: columns c and K + c) fused with the train-mode
// finalize / the coefficients: one launch instead of colreduce (1-2 launches) + finalize / coeffs
// (ogv_mbconv.hip; fixed-order, deterministic).
void bn_reduce_finalize_launch(const double* part, long R, long ld, int K, double n, const float* gamma,
                               const float* beta, float eps, float momentum, float* rm, float* rv, float* mean,
                               float* invstd, float* sc, float* sh, hipStream_t s);
void bn_reduce_coeffs_launch(const float* part, long R, long ld, int K, float n, const float* gamma,
                             const float* invstd, float* dgamma, float* dbeta, float* coef, int train, hipStream_t s);

}  // namespace ogv
