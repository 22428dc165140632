// Squeeze-Excite MLP on B pooled rows (MBConv, src/model/mbc_conv.py:9-27): the four small fp32
// products of the SE gate, one launch each, no split-K partials and no reduce launch.
//
//   forward   z1   = pooled . W1^T + b1            [B, se]    (RM = false)
//             z2   = act(z1) . W2^T + b2, gate = sigmoid(z2)  [B, mid]  (RM = false)
//   backward  dz1  = act'(z1) * (dz2 . W2)        [B, se]    (RM = true: W2 read reduction-major)
//             dpool = dz1 . W1                    [B, mid]   (RM = true)
//
// These are GEMVs over a batch of B = 512 rows with weights of 0.01-2.4 MB: latency chains, not
// flops.  The split-K tiled GEMM + reduce they replace cost 23-30 us per product plus the reduce
// launch (profiles/r02_head_step_breakdown.txt); here a block stages RB input rows in LDS (the
// prologue activation applied once, on the way in) and streams the weight straight from L2:
//   RM = false: 16 lanes per output column walk the contiguous weight row with 16-B loads, a
//               4-step xor reduction per row;
//   RM = true : lanes own consecutive output columns (coalesced weight rows), the 4 waves split the
//               reduction and combine through LDS in a fixed order (deterministic).
#include "ogv_gemm.h"

namespace ogv {

constexpr int SE_RB = 8;     // batch rows per block
static int g_se_gemv = 1;
bool se_gemv_on() { return g_se_gemv != 0; }
void set_se_gemv(int v) { g_se_gemv = v; }
constexpr int SE_NT = 256;   // threads per block

template <bool RM>
__global__ __launch_bounds__(SE_NT) void se_gemv_kernel(const float* __restrict__ in, int ldi, int pro_act,
                                                        const float* __restrict__ W, int ldw,
                                                        const float* __restrict__ bias, const float* __restrict__ Z,
                                                        int ldz, int zact, float* __restrict__ out, int ldo,
                                                        float* __restrict__ sig_out, int B, int N, int K) {
  extern __shared__ __attribute__((aligned(16))) float xs[];   // [SE_RB][Kp] (+ RM: [4][SE_RB][64])
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int b0 = blockIdx.x * SE_RB;
  const int Kp = (K + 3) / 4 * 4, K4 = Kp / 4, tot4 = SE_RB * K4;
  // staging: up to SU independent 16-B loads per thread in flight before any is stored (one L2
  // round trip per batch, not per element)
  constexpr int SU = 8;
  const bool av = (ldi & 3) == 0 && (reinterpret_cast<uintptr_t>(in) & 15) == 0;
  for (int base = tid; base < tot4; base += SE_NT * SU) {
    float4 v[SU];
#pragma unroll
    for (int u = 0; u < SU; ++u) {
      const int idx = base + u * SE_NT, r = idx / K4, k = (idx - r * K4) * 4;
      v[u] = float4{0.f, 0.f, 0.f, 0.f};
      if (idx < tot4 && b0 + r < B) {
        const float* src = in + (long)(b0 + r) * ldi + k;
        if (av && k + 4 <= K) v[u] = *reinterpret_cast<const float4*>(src);
        else {
          v[u].x = k < K ? src[0] : 0.f;
          v[u].y = k + 1 < K ? src[1] : 0.f;
          v[u].z = k + 2 < K ? src[2] : 0.f;
          v[u].w = k + 3 < K ? src[3] : 0.f;
        }
      }
    }
#pragma unroll
    for (int u = 0; u < SU; ++u) {
      const int idx = base + u * SE_NT, r = idx / K4, k = (idx - r * K4) * 4;
      if (idx >= tot4) continue;
      const bool live = b0 + r < B;
      float4 a;
      a.x = live && k < K ? act_fwd(pro_act, v[u].x) : 0.f;
      a.y = live && k + 1 < K ? act_fwd(pro_act, v[u].y) : 0.f;
      a.z = live && k + 2 < K ? act_fwd(pro_act, v[u].z) : 0.f;
      a.w = live && k + 3 < K ? act_fwd(pro_act, v[u].w) : 0.f;
      *reinterpret_cast<float4*>(xs + r * Kp + k) = a;
    }
  }
  __syncthreads();
  auto finish = [&](int r, int n, float v) {
    if (bias) v += bias[n];
    if (zact) v *= act_grad(zact, Z[(long)(b0 + r) * ldz + n]);
    out[(long)(b0 + r) * ldo + n] = v;
    if (sig_out) sig_out[(long)(b0 + r) * ldo + n] = fast_sigmoid(v);
  };
  if constexpr (!RM) {
    // column n = blockIdx.y * 32 + 8 * wave + 4 * pass + (lane >> 4); lane & 15 walks k in 16-B steps
    const int kl = lane & 15;
    const bool wv = (ldw & 3) == 0 && (reinterpret_cast<uintptr_t>(W) & 15) == 0 && (K & 3) == 0;
#pragma unroll
    for (int pass = 0; pass < 2; ++pass) {
      const int n = blockIdx.y * 32 + 8 * wave + 4 * pass + (lane >> 4);
      float acc[SE_RB];
#pragma unroll
      for (int r = 0; r < SE_RB; ++r) acc[r] = 0.f;
      if (n < N) {
        const float* wr = W + (long)n * ldw;
#pragma unroll 4
        for (int k = 4 * kl; k < K; k += 64) {
          float w4[4];
          if (wv) {
            const float4 t = *reinterpret_cast<const float4*>(wr + k);
            w4[0] = t.x; w4[1] = t.y; w4[2] = t.z; w4[3] = t.w;
          } else {
#pragma unroll
            for (int e = 0; e < 4; ++e) w4[e] = k + e < K ? wr[k + e] : 0.f;
          }
#pragma unroll
          for (int r = 0; r < SE_RB; ++r) {
            const float4 x = *reinterpret_cast<const float4*>(xs + r * Kp + k);
            acc[r] = fmaf(x.x, w4[0], fmaf(x.y, w4[1], fmaf(x.z, w4[2], fmaf(x.w, w4[3], acc[r]))));
          }
        }
      }
#pragma unroll
      for (int r = 0; r < SE_RB; ++r) acc[r] = group_sum<16>(acc[r]);
      if (n < N && kl < SE_RB && b0 + kl < B) {
        float v = acc[0];
#pragma unroll
        for (int r = 1; r < SE_RB; ++r) v = kl == r ? acc[r] : v;
        finish(kl, n, v);
      }
    }
  } else {
    // column n = blockIdx.y * 64 + lane; wave w reduces the contiguous k range [k0, k1) in steps of 4
    // (four coalesced weight rows, one 16-B broadcast read of each staged input row), then the four
    // waves combine in a fixed order
    float* red = xs + SE_RB * Kp;   // [4][SE_RB][64]
    const int n = blockIdx.y * 64 + lane;
    const int kq = (Kp / 4 + 3) / 4 * 4;   // k per wave, a multiple of 4
    const int k0 = wave * kq, k1 = min(Kp, k0 + kq);
    float acc[SE_RB];
#pragma unroll
    for (int r = 0; r < SE_RB; ++r) acc[r] = 0.f;
    if (n < N) {
#pragma unroll 2
      for (int k = k0; k < k1; k += 4) {
        float w4[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) w4[e] = k + e < K ? W[(long)(k + e) * ldw + n] : 0.f;
#pragma unroll
        for (int r = 0; r < SE_RB; ++r) {
          const float4 x = *reinterpret_cast<const float4*>(xs + r * Kp + k);
          acc[r] = fmaf(x.x, w4[0], fmaf(x.y, w4[1], fmaf(x.z, w4[2], fmaf(x.w, w4[3], acc[r]))));
        }
      }
    }
#pragma unroll
    for (int r = 0; r < SE_RB; ++r) red[(wave * SE_RB + r) * 64 + lane] = acc[r];
    __syncthreads();
    for (int i = tid; i < SE_RB * 64; i += SE_NT) {
      const int r = i / 64, c = i - r * 64, nn = blockIdx.y * 64 + c;
      if (nn >= N || b0 + r >= B) continue;
      const float v = (red[(0 * SE_RB + r) * 64 + c] + red[(1 * SE_RB + r) * 64 + c]) +
                      (red[(2 * SE_RB + r) * 64 + c] + red[(3 * SE_RB + r) * 64 + c]);
      finish(r, nn, v);
    }
  }
}

// out[B, N] = epi(act(in[B, K]) . W^T): W [N][ldw] (rm = false) or W [K][ldw] read reduction-major
// (rm = true).  Epilogue: + bias[n]; * act'(Z) (zact); gate = sigmoid (sig_out).
void se_gemv_launch(const float* in, int ldi, int pro_act, const float* W, int ldw, const float* bias,
                    const float* Z, int ldz, int zact, float* out, int ldo, float* sig_out, int B, int N, int K,
                    bool rm, hipStream_t s) {
  if (B <= 0 || N <= 0) return;
  const int Kp = (K + 3) / 4 * 4;
  const size_t lds = ((size_t)SE_RB * Kp + (rm ? 4 * SE_RB * 64 : 0)) * sizeof(float);
  if (!lds_ok(reinterpret_cast<const void*>(rm ? se_gemv_kernel<true> : se_gemv_kernel<false>), lds, "se_gemv_kernel"))
    return;
  dim3 grid((unsigned)cdiv(B, SE_RB), (unsigned)cdiv(N, rm ? 64 : 32));
  if (rm)
    se_gemv_kernel<true><<<grid, SE_NT, lds, s>>>(in, ldi, pro_act, W, ldw, bias, Z, ldz, zact, out, ldo, sig_out, B,
                                                  N, K);
  else
    se_gemv_kernel<false><<<grid, SE_NT, lds, s>>>(in, ldi, pro_act, W, ldw, bias, Z, ldz, zact, out, ldo, sig_out, B,
                                                   N, K);
}

}  // namespace ogv
