// Internal (C++) GEMM launchers shared by the C-ABI wrappers and the fused MBConv.
#pragma once
#include "ogv_common.h"

namespace ogv {

// A-operand prologue, applied while staging A (fwd) or X (wgrad) tiles:
//   a' = act(a * sc[k] + sh[k]) * gate[(m / rps) * gld + k]      (each factor optional)
// Elements outside [0, M) x [0, Ka) stay exactly zero.
struct Pro {
  int act = OGV_ACT_NONE;
  const float* sc = nullptr;
  const float* sh = nullptr;
  const float* gate = nullptr;
  int rps = 1, gld = 0;
  bool any() const { return act != OGV_ACT_NONE || sc || sh || gate; }
};

// Epilogue: out = res + rs[m/rps] * (acc + bias[n]);  out *= act'(Z[m,n]) (zact);
// optional per-column batch statistics of the stored (rounded) output:
//   stat[mt][0][n] = sum_rows (out - shift[n]),  stat[mt][1][n] = sum_rows (out - shift[n])^2
// for each 128-row panel mt (deterministic partials; reduce with colreduce).
struct Epi {
  const float* bias = nullptr;
  const void* res = nullptr;
  const float* rs = nullptr;
  int rps = 1;
  const void* Z = nullptr;
  int ldz = 0, zact = 0;
  float* stat = nullptr;
  const float* stat_shift = nullptr;
};

constexpr int GEMM_BM = 128;
inline int gemm_stat_rows(int M) { return (M + GEMM_BM - 1) / GEMM_BM; }

// out[M,N] = epi( pro(A)[M,K] . W[N,K]^T );  Ka / Kb = valid reduction columns of A / W.
void gemm_fwd_launch(ogv_dtype dt, const void* A, int lda, const Pro& pro, const float* W, int ldw, void* out,
                     int ldo, int M, int N, int K, int Ka, int Kb, const Epi& epi, hipStream_t s);

// dA[M,K] = act'(Z) * rs * (dOut[M,N] . W[N,K]);  ws >= dgrad_ws_bytes(N, K); res added if given
size_t dgrad_ws_bytes(int N, int K);
void gemm_dgrad_launch(ogv_dtype dt, const void* dout, int ldd, const float* W, const void* Z, int ldz, int zact,
                       const float* rs, int rps, const void* res, void* dA, int lda, int M, int N, int K, void* ws,
                       hipStream_t s);

// dW[N,K] = sum_m rs*G[m,n] * pro(X)[m,k];  dbias[n] = sum_m rs*G[m,n]
size_t wgrad_ws_bytes(int M, int N, int K);
void gemm_wgrad_launch(ogv_dtype dt, const void* G, int ldg, const void* X, int ldx, const Pro& pro, const float* rs,
                       int rps, float* dW, float* dbias, int M, int N, int K, void* ws, hipStream_t s);

}  // namespace ogv
