// Persistent streaming GEMM for the tall-skinny projections (gfx950).
//
// The 1x1 projections of the OutGridBlock are out[M,N] = A[M,K] . B[N,K]^T with M = B*H*W in the
// hundreds of thousands and N*K <= 384*96 at the large-M stages: an HBM stream of A and out with a
// weight tile small enough to live in LDS.  So, unlike a classic tiled GEMM:
//   * each workgroup converts its weight tile to bf16 into LDS ONCE (one barrier in the kernel),
//   * every wave then walks its own sequence of 16*RS-row panels with no block barriers: the A
//     fragments are loaded straight from HBM into registers in MFMA layout (16 B per lane; lane l
//     reads row l&15, k = 8*(l>>4) of a 32-wide k step), the NEXT panel's fragments are in flight
//     while the current one is multiplied, and the B fragments come from the LDS tile,
//   * the epilogue stages each 16 x 64 accumulator block through a wave-private LDS slab and
//     re-reads it as 8-column runs: 16-B residual / Z loads and 16-B stores of out,
//   * BatchNorm column statistics (fp64, shifted) accumulate in wave-private LDS across panels and
//     leave the kernel as ONE partial row per workgroup (gridDim.x rows instead of M/128).
// B[n][k] = W[n*ldw + k] (forward: W is [N][K]) or W[k*ldw + n] (BT, data gradient: the forward
// weight [Nf][Kf] read as [reduction][output], transposed while it is staged).
// A / out rows whose index is >= M are neither read nor written; k >= K is zero in both operands.
#include "ogv_gemm.h"

namespace ogv {

constexpr int SG_CW = 64;  // output columns per accumulator chunk (4 MFMA n-subtiles)
constexpr int SG_NW = 8;   // waves per workgroup (they share one weight tile)
constexpr int SG_WB = 8;   // weight-staging loads in flight per thread

template <int KT>
__host__ __device__ constexpr int sg_kp() { return KT * 32 + 8; }  // W tile pitch: 16(4KT+1) B, conflict-free

// PA: -1 = no A prologue, else the prologue's activation (OGV_ACT_*; sc / sh / gate applied when
// non-null).  ZA: activation whose derivative at Z scales the output (0 = none).  All operand
// rows are 16-B aligned runs (checked by the host): N, K, lda, ldo, ldz multiples of 8.
//
// The product is computed transposed, D[n][m] = W-tile . A^T (v_mfma_f32_16x16x32_bf16 with the
// weight fragment as the A operand), so each lane's accumulator holds 4 CONSECUTIVE output
// columns of one row: bias / residual / Z are read and out is written as 8-byte runs straight
// from registers (the four lanes of a row group cover 32 contiguous bytes per instruction, the
// four n-subtiles of a chunk the whole 128-byte line), with no LDS staging and no wave barrier.
//
// SW: the weight is staged as two bf16 tiles (hi = bf16(w), lo = bf16(w - hi)) and every A
// fragment meets both, as in the tiled kernel (ogv_gemm.hip, knob "split_w").
template <int KT, int RS, int PA, int ZA, bool STATS, bool BT, bool SW>
__global__ __launch_bounds__(SG_NW * 64) void sgemm_bf16_kernel(const bf16* __restrict__ A, int lda, Pro pro,
                                                                const float* __restrict__ W, int ldw, Epi epi,
                                                                bf16* __restrict__ out, int ldo, int M, int N, int K,
                                                                int NB, int pf) {
  constexpr int KP = sg_kp<KT>();
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int n0 = blockIdx.y * NB;
  const int nb = min(NB, N - n0);  // multiple of 8
  const int nbp = (nb + SG_CW - 1) / SG_CW * SG_CW;
  bf16* Ws = reinterpret_cast<bf16*>(smem);
  bf16* Wl = Ws + (size_t)nbp * KP;  // SW: lo tile
  double* sacc = reinterpret_cast<double*>(smem + (size_t)nbp * KP * 2 * (SW ? 2 : 1));
  float* cvec = reinterpret_cast<float*>(sacc + (STATS ? SG_NW * 2 * nbp : 0));  // [bias | stat shift]
  // prologue variants: [sc | sh] (K each) and one gate row per wave (the SE gate of the image the
  // wave's current panel belongs to), so the prologue reads no global memory of its own
  constexpr int KK = KT * 32;
  float* pvec = cvec + 2 * nbp;                 // PA >= 0: [sc | sh]
  float* gsl = pvec + 2 * KK + wave * KK;       // PA >= 0: this wave's gate row

  // ---- weight tile -> LDS (bf16), zero outside [0,nb) x [0,K).  Batches of SG_WB independent
  // 16-B loads per thread are issued before any is consumed, so staging costs a few L2 round trips
  // rather than one per loop trip.
  constexpr int NT = SG_NW * 64;
  if constexpr (!BT) {
    constexpr int QPR = KT * 32 / 4;  // float4 quads per tile row
    const bool wv = ((ldw & 3) == 0) && ((reinterpret_cast<uintptr_t>(W) & 15) == 0);
    const int total = nbp * QPR;
    for (int base = tid; base < total; base += SG_WB * NT) {
      float4 v[SG_WB];
#pragma unroll
      for (int b = 0; b < SG_WB; ++b) {
        const int idx = base + b * NT;
        const int r = idx / QPR, k = (idx - r * QPR) * 4;
        v[b] = float4{0.f, 0.f, 0.f, 0.f};
        if (idx < total && r < nb) {
          const float* src = W + (long)(n0 + r) * ldw + k;
          if (wv && k + 4 <= K) v[b] = *reinterpret_cast<const float4*>(src);
          else if (k < K) {
            v[b].x = src[0];
            v[b].y = k + 1 < K ? src[1] : 0.f;
            v[b].z = k + 2 < K ? src[2] : 0.f;
            v[b].w = k + 3 < K ? src[3] : 0.f;
          }
        }
      }
#pragma unroll
      for (int b = 0; b < SG_WB; ++b) {
        const int idx = base + b * NT;
        if (idx < total) {
          const int r = idx / QPR, k = (idx - r * QPR) * 4;
          bf16x4 w4 = {(bf16)v[b].x, (bf16)v[b].y, (bf16)v[b].z, (bf16)v[b].w};
          *reinterpret_cast<bf16x4*>(Ws + r * KP + k) = w4;
          if constexpr (SW) {
            bf16x4 l4 = {(bf16)(v[b].x - (float)w4[0]), (bf16)(v[b].y - (float)w4[1]), (bf16)(v[b].z - (float)w4[2]),
                         (bf16)(v[b].w - (float)w4[3])};
            *reinterpret_cast<bf16x4*>(Wl + r * KP + k) = l4;
          }
        }
      }
    }
  } else {  // W is [reduction][output]: 4 consecutive output columns per 16-B load
    const bool wv = ((ldw & 3) == 0) && ((reinterpret_cast<uintptr_t>(W) & 15) == 0) && ((n0 & 3) == 0);
    const int q4 = nbp / 4;
    const int total = q4 * KT * 32;
    for (int base = tid; base < total; base += SG_WB * NT) {
      float4 v[SG_WB];
#pragma unroll
      for (int b = 0; b < SG_WB; ++b) {
        const int idx = base + b * NT;
        const int k = idx / q4, r = (idx - k * q4) * 4;
        v[b] = float4{0.f, 0.f, 0.f, 0.f};
        if (idx < total && k < K && r < nb) {
          const float* src = W + (long)k * ldw + n0 + r;
          if (wv && r + 4 <= nb) v[b] = *reinterpret_cast<const float4*>(src);
          else {
            v[b].x = src[0];
            v[b].y = r + 1 < nb ? src[1] : 0.f;
            v[b].z = r + 2 < nb ? src[2] : 0.f;
            v[b].w = r + 3 < nb ? src[3] : 0.f;
          }
        }
      }
#pragma unroll
      for (int b = 0; b < SG_WB; ++b) {
        const int idx = base + b * NT;
        if (idx < total) {
          const int k = idx / q4, r = (idx - k * q4) * 4;
          const float vv[4] = {v[b].x, v[b].y, v[b].z, v[b].w};
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const bf16 h = (bf16)vv[e];
            Ws[(r + e) * KP + k] = h;
            if constexpr (SW) Wl[(r + e) * KP + k] = (bf16)(vv[e] - (float)h);
          }
        }
      }
    }
  }
  if constexpr (STATS) {
    for (int i = lane; i < 2 * nbp; i += 64) sacc[wave * 2 * nbp + i] = 0.0;
  }
  if constexpr (PA >= 0) {
    for (int k = tid; k < KK; k += SG_NW * 64) {
      pvec[k] = (pro.sc && k < K) ? pro.sc[k] : 1.f;
      pvec[KK + k] = (pro.sh && k < K) ? pro.sh[k] : 0.f;
    }
  }
  for (int c = tid; c < nbp; c += SG_NW * 64) {
    cvec[c] = (epi.bias && c < nb) ? epi.bias[n0 + c] : 0.f;
    if (STATS) cvec[nbp + c] = (epi.stat_shift && c < nb) ? bn_shift(epi.stat_shift[n0 + c]) : 0.f;
  }
  __syncthreads();

  const int fr = lane & 15, fg = lane >> 4;
  const long P = ((long)M + 16 * RS - 1) / (16 * RS);
  const long GW = (long)gridDim.x * SG_NW;
  const bf16* res = static_cast<const bf16*>(epi.res);
  const bf16* Z = static_cast<const bf16*>(epi.Z);

  // gate row of panel pp (pipelined prologue: every row of a panel belongs to one image), raw:
  // lane holds gate[img][lane + 64 u]
  constexpr int GPL = (KK + 63) / 64;
  auto fetch_gate = [&](long pp, float (&g)[GPL]) {
    if constexpr (PA >= 0) {
      const long mi = pp * 16 * RS;
      const float* gp = pro.gate + (mi < M ? mi / pro.rps : 0) * pro.gld;
#pragma unroll
      for (int u = 0; u < GPL; ++u) g[u] = (lane + 64 * u < K) ? gp[lane + 64 * u] : 1.f;
    }
  };
  // A fragments (+ row scales) of panel pp, raw
  auto fetch = [&](long pp, bf16x8 (&dst)[RS][KT], float (&rs)[RS]) {
#pragma unroll
    for (int i = 0; i < RS; ++i) {
      const long mi = pp * 16 * RS + i * 16 + fr;
#pragma unroll
      for (int kt = 0; kt < KT; ++kt) {
        const int k = kt * 32 + fg * 8;
        bf16x8 v = {};
        if (mi < M && k < K) v = *reinterpret_cast<const bf16x8*>(A + mi * lda + k);
        dst[i][kt] = v;
      }
      rs[i] = epi.rs ? epi.rs[(mi < M ? mi : M - 1) / epi.rps] : 1.f;
    }
  };
  // Without an A prologue the next panel's fragments are fetched right after the current ones are
  // taken, so a wave keeps two panels of loads in flight across its MFMAs and stores (knob
  // "sg_prefetch").  With a prologue its sc / sh / gate loads would wait on that prefetch
  // (in-order vmcnt), so those variants fetch each panel when they reach it.
  // With a prologue the pipeline stays on when its operands come from LDS: sc / sh (staged above)
  // and a gate that is constant over a panel (16 RS | rows per image): the gate row is prefetched
  // with the panel and parked in a wave-private LDS row.
  const bool gate_rows = PA >= 0 && pro.gate != nullptr;
  const bool pipe = (pf & 1) && (PA < 0 || ((pf & 2) && (!gate_rows || pro.rps % (16 * RS) == 0)));
  bf16x8 an[RS][KT];
  float rsn[RS];
  float gn[GPL];
  if (pipe && (long)blockIdx.x * SG_NW + wave < P) {
    fetch((long)blockIdx.x * SG_NW + wave, an, rsn);
    if (gate_rows) fetch_gate((long)blockIdx.x * SG_NW + wave, gn);
  }

  for (long p = (long)blockIdx.x * SG_NW + wave; p < P; p += GW) {
    const long mp = p * 16 * RS;
    bf16x8 a[RS][KT];
    long m[RS];
    float rsc[RS];
#pragma unroll
    for (int i = 0; i < RS; ++i) m[i] = mp + i * 16 + fr;
    if (pipe) {
#pragma unroll
      for (int i = 0; i < RS; ++i) {
        rsc[i] = rsn[i];
#pragma unroll
        for (int kt = 0; kt < KT; ++kt) a[i][kt] = an[i][kt];
      }
      if (gate_rows) {   // park this panel's gate row before its registers are reused
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
#pragma unroll
        for (int u = 0; u < GPL; ++u)
          if (lane + 64 * u < KK) gsl[lane + 64 * u] = gn[u];
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      }
      if (p + GW < P) {
        fetch(p + GW, an, rsn);
        if (gate_rows) fetch_gate(p + GW, gn);
      }
    } else {
      fetch(p, a, rsc);
    }
    if constexpr (PA >= 0) {
      if (pipe) {   // sc / sh / gate from LDS (broadcast reads: the 16 lanes of a column group agree)
#pragma unroll
        for (int i = 0; i < RS; ++i) {
#pragma unroll
          for (int kt = 0; kt < KT; ++kt) {
            const int k = kt * 32 + fg * 8;
            if (m[i] < M && k < K) {
              float f[8], sc[8], sh[8], g8[8];
              load_vec<float, 8>(pvec + k, sc);
              load_vec<float, 8>(pvec + KK + k, sh);
              if (gate_rows) load_vec<float, 8>(gsl + k, g8);
#pragma unroll
              for (int q = 0; q < 8; ++q) {
                f[q] = act_fwd(PA, fmaf((float)a[i][kt][q], sc[q], sh[q]));
                if (gate_rows) f[q] *= g8[q];
                a[i][kt][q] = (bf16)f[q];
              }
            }
          }
        }
      }
    }
    if constexpr (PA >= 0) if (!pipe) {
#pragma unroll
      for (int i = 0; i < RS; ++i) {
#pragma unroll
        for (int kt = 0; kt < KT; ++kt) {
          const int k = kt * 32 + fg * 8;
          if (m[i] < M && k < K) {
            float f[8];
#pragma unroll
            for (int q = 0; q < 8; ++q) f[q] = (float)a[i][kt][q];
            if (pro.sc) {
              float t[8];
              load_vec<float, 8>(pro.sc + k, t);
#pragma unroll
              for (int q = 0; q < 8; ++q) f[q] *= t[q];
            }
            if (pro.sh) {
              float t[8];
              load_vec<float, 8>(pro.sh + k, t);
#pragma unroll
              for (int q = 0; q < 8; ++q) f[q] += t[q];
            }
#pragma unroll
            for (int q = 0; q < 8; ++q) f[q] = act_fwd(PA, f[q]);
            if (pro.gate) {
              float t[8];
              load_vec<float, 8>(pro.gate + (m[i] / pro.rps) * pro.gld + k, t);
#pragma unroll
              for (int q = 0; q < 8; ++q) f[q] *= t[q];
            }
#pragma unroll
            for (int q = 0; q < 8; ++q) a[i][kt][q] = (bf16)f[q];
          }
        }
      }
    }
    for (int c0 = 0; c0 < nb; c0 += SG_CW) {
      // residual / Z runs of this chunk first (their latency overlaps the MFMAs)
      // (clamped, always-valid addresses under a uniform branch: per-lane guards made the compiler
      // wait after each of these loads -- one round trip per 8-B load)
      uint2 rv[RS][4], zv[RS][4];
#pragma unroll
      for (int i = 0; i < RS; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) rv[i][j] = zv[i][j] = uint2{0u, 0u};
      if (res) {
#pragma unroll
        for (int i = 0; i < RS; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const long mc = m[i] < M ? m[i] : M - 1;
            const int cc = min(c0 + j * 16 + 4 * fg, nb - 4);
            rv[i][j] = *reinterpret_cast<const uint2*>(res + mc * ldo + n0 + cc);
          }
      }
      if constexpr (ZA != 0) {
#pragma unroll
        for (int i = 0; i < RS; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const long mc = m[i] < M ? m[i] : M - 1;
            const int cc = min(c0 + j * 16 + 4 * fg, nb - 4);
            zv[i][j] = *reinterpret_cast<const uint2*>(Z + mc * epi.ldz + n0 + cc);
          }
      }
      f32x4 acc[RS][4];
#pragma unroll
      for (int i = 0; i < RS; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kt = 0; kt < KT; ++kt) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const bf16x8 w = *reinterpret_cast<const bf16x8*>(Ws + (c0 + j * 16 + fr) * KP + kt * 32 + fg * 8);
#pragma unroll
          for (int i = 0; i < RS; ++i) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w, a[i][kt], acc[i][j], 0, 0, 0);
          if constexpr (SW) {
            const bf16x8 wl = *reinterpret_cast<const bf16x8*>(Wl + (c0 + j * 16 + fr) * KP + kt * 32 + fg * 8);
#pragma unroll
            for (int i = 0; i < RS; ++i)
              acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wl, a[i][kt], acc[i][j], 0, 0, 0);
          }
        }
      }
      // ---- epilogue: lane holds out[m = mp + i*16 + fr][n0 + c0 + j*16 + 4*fg + r], r = 0..3
      float s1[4][4], s2[4][4];
      if constexpr (STATS) {
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
          for (int r = 0; r < 4; ++r) { s1[j][r] = 0.f; s2[j][r] = 0.f; }
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int cc = c0 + j * 16 + 4 * fg;
        const float4 bs = *reinterpret_cast<const float4*>(cvec + cc);
        const float bias[4] = {bs.x, bs.y, bs.z, bs.w};
        float shift[4] = {0.f, 0.f, 0.f, 0.f};
        if constexpr (STATS) {
          const float4 h = *reinterpret_cast<const float4*>(cvec + nbp + cc);
          shift[0] = h.x; shift[1] = h.y; shift[2] = h.z; shift[3] = h.w;
        }
#pragma unroll
        for (int i = 0; i < RS; ++i) {
          if (!(m[i] < M && cc < nb)) continue;
          const bf16* rb = reinterpret_cast<const bf16*>(&rv[i][j]);
          const bf16* zb = reinterpret_cast<const bf16*>(&zv[i][j]);
          uint2 ov;
          bf16* ob = reinterpret_cast<bf16*>(&ov);
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            float x = (acc[i][j][r] + bias[r]) * rsc[i] + (float)rb[r];  // rb = 0 without a residual
            if constexpr (ZA != 0) x *= act_grad(ZA, (float)zb[r]);
            ob[r] = (bf16)x;
            if constexpr (STATS) {
              const float d = (float)ob[r] - shift[r];
              s1[j][r] += d;
              s2[j][r] = fmaf(d, d, s2[j][r]);
            }
          }
          *reinterpret_cast<uint2*>(out + m[i] * ldo + n0 + cc) = ov;
          if (epi.aout) {
            uint2 av;
            bf16* ab = reinterpret_cast<bf16*>(&av);
#pragma unroll
            for (int r = 0; r < 4; ++r) ab[r] = (bf16)act_fwd(epi.aact, (float)ob[r]);
            *reinterpret_cast<uint2*>(static_cast<bf16*>(epi.aout) + (long)m[i] * epi.ldao + n0 + cc) = av;
          }
        }
      }
      if constexpr (STATS) {
        // rows are spread over the 16 lanes fr of a group: reduce (DPP butterfly), fp32 over <= 32 rows,
        // then fp64 across panels in the wave's LDS accumulator
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            s1[j][r] = group_sum<16>(s1[j][r]);
            s2[j][r] = group_sum<16>(s2[j][r]);
          }
        if (fr == 0) {
          double* sa = sacc + wave * 2 * nbp;
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const int cc = c0 + j * 16 + 4 * fg;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              sa[cc + r] += (double)s1[j][r];
              sa[nbp + cc + r] += (double)s2[j][r];
            }
          }
        }
      }
    }
  }

  if constexpr (STATS) {  // one partial row per workgroup: stat[blockIdx.x][q][n]
    __syncthreads();
    for (int c = tid; c < nb; c += SG_NW * 64) {
      double t1 = 0.0, t2 = 0.0;
#pragma unroll
      for (int w = 0; w < SG_NW; ++w) {
        t1 += sacc[w * 2 * nbp + c];
        t2 += sacc[w * 2 * nbp + nbp + c];
      }
      epi.stat[((long)blockIdx.x * 2 + 0) * N + n0 + c] = t1;
      epi.stat[((long)blockIdx.x * 2 + 1) * N + n0 + c] = t2;
    }
  }
}

// ------------------------------------------------------------------------------------------------
// plan + dispatch
// ------------------------------------------------------------------------------------------------
static int g_sgemm_mode = -1;  // -1: unset (read OGV_SGEMM once), 0 off, 1 on
int sgemm_mode() {
  if (g_sgemm_mode < 0) {
    const char* e = getenv("OGV_SGEMM");
    g_sgemm_mode = e ? atoi(e) : 1;
  }
  return g_sgemm_mode;
}
void set_sgemm_mode(int v) { g_sgemm_mode = v; }
static int g_sg_per_cu = 2;     // workgroups per CU the planner asks for (tuning knob "sg_per_cu"),
                                // clamped at launch to the kernel's real occupancy
void set_sg_per_cu(int v) { g_sg_per_cu = v < 1 ? 1 : (v > 4 ? 4 : v); }
// knob "sg_prefetch": bit 1 next-panel register prefetch, bit 2 also for the prologue variants
// (sc / sh / gate then come from LDS); default 3
static int g_sg_prefetch = 3;
void set_sg_prefetch(int v) { g_sg_prefetch = v & 3; }
static int g_sg_wgs = 0;
void set_sg_wgs(int v) { g_sg_wgs = v < 0 ? 0 : v; }
// smallest M routed to the streaming kernels (tuning knob "sgemm_min_m"): 262144 since round 4 -- with
// the panel kernel's 64-column tiles, 7M stage 1 (M = 131072) runs faster there (paired 40-step runs:
// 15.56-15.66 -> 15.48-15.53 ms; 14M 45.46 -> 45.30 ms, profiles/r04_sgemm_min_m.log)
static int g_sg_min_m = 262144;
void set_sgemm_min_m(int v) { g_sg_min_m = v; }
int sgemm_min_m() { return g_sg_min_m; }

static int device_cus() {
  static int cus = 0;
  if (!cus) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
      cus = 256;
  }
  return cus;
}

struct SgPlan {
  int ok = 0, KT = 0, RS = 1, NB = 0, ntiles = 1, grid = 0, sw = 0;
  size_t lds = 0;
};

static constexpr size_t SG_LDS_CAP = 80 * 1024;  // per workgroup: 2 eight-wave workgroups per CU (the VGPR limit)

static bool al16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

// Routing (measured, tools/bench_sgemm.py, cold caches, MI355X): the streaming kernel wins for
// reductions up to 192 everywhere; at 256-384 only when the A prologue (GELU) makes the tiled
// kernel VALU-bound; a data-gradient whose output needs two weight tiles loses to the tiled kernel.
// split weights (knob "split_w") double the weight tile; a shape whose split tiles do not fit
// runs unsplit on this kernel rather than moving to the tiled one
static SgPlan sgemm_plan_w(int M, int N, int K, bool stats, bool prologue, bool dgrad, int wtiles);
static SgPlan sgemm_plan(int M, int N, int K, bool stats, bool prologue, bool dgrad) {
  if (split_w() & (dgrad ? 2 : 1)) {
    SgPlan p = sgemm_plan_w(M, N, K, stats, prologue, dgrad, 2);
    if (p.ok) return p;
  }
  return sgemm_plan_w(M, N, K, stats, prologue, dgrad, 1);
}

static SgPlan sgemm_plan_w(int M, int N, int K, bool stats, bool prologue, bool dgrad, int wtiles) {
  SgPlan p;
  p.sw = wtiles == 2;
  if (M < g_sg_min_m || (K & 7) != 0 || (N & 7) != 0) return p;  // small M: the tiled kernel fills the chip better
  int KT;
  if (K <= 64) KT = 2;
  else if (K <= 96) KT = 3;
  else if (K <= 128) KT = 4;
  else if (K <= 192) KT = 6;
  else if (K <= 256) KT = 8;
  else if (K <= 384) KT = 12;
  else return p;
  if (KT > 6 && !prologue) return p;
  const int KP = KT * 32 + 8;
  p.KT = KT;
  p.RS = KT <= 2 ? 2 : 1;
  auto lds_of = [&](int nb) {  // nb padded to the chunk (+ the prologue's [sc | sh] and per-wave gate rows)
    return (size_t)nb * KP * 2 * wtiles + (stats ? (size_t)SG_NW * 2 * nb * 8 : 0) + (size_t)nb * 8 +
           (prologue ? (size_t)(2 + SG_NW) * KT * 32 * 4 : 0);
  };
  // widest tile (multiple of the 64-column chunk) whose bf16 copy fits next to the staging slabs
  int NB = (N + SG_CW - 1) / SG_CW * SG_CW;
  while (NB > SG_CW && lds_of(NB) > SG_LDS_CAP) NB -= SG_CW;
  if (lds_of(NB) > SG_LDS_CAP) return p;
  p.ntiles = (N + NB - 1) / NB;
  if (dgrad && p.ntiles > 1) return p;
  NB = (N + p.ntiles - 1) / p.ntiles;  // balance the tiles
  NB = (NB + 15) / 16 * 16;
  p.ntiles = (N + NB - 1) / NB;
  p.NB = NB;
  p.lds = lds_of((NB + SG_CW - 1) / SG_CW * SG_CW);
  const int per_cu = (int)std::max<size_t>(1, std::min<size_t>((size_t)g_sg_per_cu, (160 * 1024) / p.lds));
  const long panels = ((long)M + 16 * p.RS - 1) / (16 * p.RS);
  const long want = (panels + SG_NW - 1) / SG_NW;
  p.grid = (int)std::min<long>(want, (long)device_cus() * per_cu);
  if (g_sg_wgs > 0)  // knob "sg_wgs": total workgroups over all N-tiles (persistent at small M)
    p.grid = (int)std::max<long>(8, std::min<long>(want, (long)g_sg_wgs / p.ntiles));
  p.grid = (p.grid + 7) / 8 * 8;  // the N-tiles of one row range share an XCD: x % 8 fixes the XCD
  if (stats) p.grid = std::min(p.grid, std::max(8, ((M + GEMM_BM - 1) / GEMM_BM) / 8 * 8));  // <= gemm_stat_rows
  p.ok = 1;
  return p;
}

// Returns the workgroup count launched along x (= BatchNorm partial rows with STATS).  Panels are
// dealt to waves statically, so every workgroup must be resident at once: above 2 per CU the
// planner's grid is clamped to the occupancy the runtime reports for this instantiation
// (VGPRs / LDS), never raised above the plan (the partial-row buffer is sized for the plan).
template <int KT, int RS, int PA, int ZA, bool STATS, bool BT>
static int sg_launch(const SgPlan& p, const bf16* A, int lda, const Pro& pro, const float* W, int ldw,
                     const Epi& epi, bf16* out, int ldo, int M, int N, int K, hipStream_t s) {
  if (skip_mask() & 2) return p.grid;
  const int sw = p.sw;
  auto kern = sw ? sgemm_bf16_kernel<KT, RS, PA, ZA, STATS, BT, true> : sgemm_bf16_kernel<KT, RS, PA, ZA, STATS, BT, false>;
  if (!lds_ok(reinterpret_cast<const void*>(kern), p.lds, "sgemm_bf16_kernel")) return p.grid;
  int gx = p.grid;
  if (g_sg_per_cu > 2) {
    int occ = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, reinterpret_cast<const void*>(kern), SG_NW * 64,
                                                     p.lds) != hipSuccess || occ < 1)
      occ = 2;
    // (the API reads one block per CU high for SGPR counts 81-112 on ROCm 7.2 — MI355X_MICROARCH.md;
    // harmless here: a non-resident workgroup only delays the tail, nothing waits on it)
    const long cap = (long)device_cus() * std::min(occ, g_sg_per_cu);
    if (gx > cap) gx = (int)std::max(8L, cap / 8 * 8);
  }
  dim3 grid((unsigned)gx, (unsigned)p.ntiles);
  kern<<<grid, SG_NW * 64, p.lds, s>>>(A, lda, pro, W, ldw, epi, out, ldo, M, N, K, p.NB, g_sg_prefetch);
  return gx;
}

template <int PA, int ZA, bool STATS, bool BT>
static int sg_dispatch(const SgPlan& p, const bf16* A, int lda, const Pro& pro, const float* W, int ldw,
                        const Epi& epi, bf16* out, int ldo, int M, int N, int K, hipStream_t s) {
  switch (p.KT) {
    case 2: return sg_launch<2, 2, PA, ZA, STATS, BT>(p, A, lda, pro, W, ldw, epi, out, ldo, M, N, K, s);
    case 3: return sg_launch<3, 1, PA, ZA, STATS, BT>(p, A, lda, pro, W, ldw, epi, out, ldo, M, N, K, s);
    case 4: return sg_launch<4, 1, PA, ZA, STATS, BT>(p, A, lda, pro, W, ldw, epi, out, ldo, M, N, K, s);
    case 6: return sg_launch<6, 1, PA, ZA, STATS, BT>(p, A, lda, pro, W, ldw, epi, out, ldo, M, N, K, s);
    case 8: return sg_launch<8, 1, PA, ZA, STATS, BT>(p, A, lda, pro, W, ldw, epi, out, ldo, M, N, K, s);
    default: return sg_launch<12, 1, PA, ZA, STATS, BT>(p, A, lda, pro, W, ldw, epi, out, ldo, M, N, K, s);
  }
}

static bool epi_ok(const void* out, int ldo, const Epi& e) {
  return al16(out) && (ldo & 7) == 0 && (!e.res || al16(e.res)) &&
         (!e.zact || (e.Z && al16(e.Z) && (e.ldz & 7) == 0));
}

// Returns the number of BatchNorm partial rows written (>= 1) when it handled the call, 0 if the
// shape / operand combination is not one it covers (the caller falls back to the tiled kernel).
int sgemm_fwd_try(const void* A, int lda, const Pro& pro, const float* W, int ldw, void* out, int ldo, int M,
                  int N, int K, const Epi& epi, hipStream_t s) {
  if (!sgemm_mode() || epi.zact || !al16(A) || (lda & 7) || !epi_ok(out, ldo, epi)) return 0;
  if (pro.any() && pro.act != OGV_ACT_NONE && pro.act != OGV_ACT_GELU && pro.act != OGV_ACT_SILU) return 0;
  if (pro.gate && (pro.gld & 3)) return 0;
  const bool st = epi.stat != nullptr;
  const SgPlan p = sgemm_plan(M, N, K, st, pro.any(), false);
  if (!p.ok) return 0;
  const bf16* a = static_cast<const bf16*>(A);
  bf16* o = static_cast<bf16*>(out);
  int gx = p.grid;
#define OGV_SG_FWD(PA_)                                                                       \
  do {                                                                                        \
    if (st) gx = sg_dispatch<PA_, 0, true, false>(p, a, lda, pro, W, ldw, epi, o, ldo, M, N, K, s); \
    else gx = sg_dispatch<PA_, 0, false, false>(p, a, lda, pro, W, ldw, epi, o, ldo, M, N, K, s);   \
  } while (0)
  if (!pro.any()) OGV_SG_FWD(-1);
  else if (pro.act == OGV_ACT_GELU) OGV_SG_FWD(OGV_ACT_GELU);
  else if (pro.act == OGV_ACT_SILU) OGV_SG_FWD(OGV_ACT_SILU);
  else OGV_SG_FWD(OGV_ACT_NONE);
#undef OGV_SG_FWD
  return st ? gx : 1;
}

// dA[M, Kf] = epi(dOut[M, Nf] . W[Nf, Kf]):  reduction Nf, output columns Kf.
bool sgemm_dgrad_try(const void* dout, int ldd, const float* W, void* dA, int lda, int M, int Nf, int Kf,
                     const Epi& epi, hipStream_t s) {
  if (!sgemm_mode() || epi.stat || !al16(dout) || (ldd & 7) || !epi_ok(dA, lda, epi)) return false;
  if (epi.zact != OGV_ACT_NONE && epi.zact != OGV_ACT_GELU && epi.zact != OGV_ACT_SILU) return false;
  const SgPlan p = sgemm_plan(M, Kf, Nf, false, false, true);
  if (!p.ok) return false;
  const bf16* a = static_cast<const bf16*>(dout);
  bf16* o = static_cast<bf16*>(dA);
  if (epi.zact == OGV_ACT_GELU) sg_dispatch<-1, OGV_ACT_GELU, false, true>(p, a, ldd, Pro(), W, Kf, epi, o, lda, M, Kf, Nf, s);
  else if (epi.zact == OGV_ACT_SILU) sg_dispatch<-1, OGV_ACT_SILU, false, true>(p, a, ldd, Pro(), W, Kf, epi, o, lda, M, Kf, Nf, s);
  else sg_dispatch<-1, 0, false, true>(p, a, ldd, Pro(), W, Kf, epi, o, lda, M, Kf, Nf, s);
  return true;
}

// Spin on the device wall clock (100 MHz class counter) for ~us microseconds: queued in front of a
// timed launch it keeps the GPU behind the host, so HIP events around the launch time the kernel
// and not the host's launch latency (bench.py's roofline probe).  Reads the clock only.
__global__ void gpu_sleep_kernel(unsigned long long ticks) {
  const unsigned long long t0 = wall_clock64();
  while (wall_clock64() - t0 < ticks) __builtin_amdgcn_s_sleep(8);
}

int sgemm_route(int kind, int M, int N, int K, int act) {
  if (sgemm_mode()) {
    if (kind == 0 && sgemm_plan(M, N, K, false, act != OGV_ACT_NONE, false).ok) return 1;
    if (kind != 0 && sgemm_plan(M, K, N, false, false, true).ok) return 1;  // dgrad: output K, reduction N
  }
  return pgemm_route(kind, M, N, K, act) ? 2 : 0;
}

}  // namespace ogv

using namespace ogv;

extern "C" int ogv_gemm_stream_route(int kind, int M, int N, int K, ogv_act act_in) {
  return sgemm_route(kind, M, N, K, act_in);
}

extern "C" int ogv_gpu_sleep(int microseconds, void* stream) {
  static int khz = 0;
  if (!khz) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev) != hipSuccess ||
        khz <= 0)
      khz = 100000;
  }
  const unsigned long long ticks = (unsigned long long)(microseconds > 0 ? microseconds : 0) * (unsigned long long)khz / 1000ull;
  gpu_sleep_kernel<<<1, 64, 0, as_stream(stream)>>>(ticks);
  return check_launch("ogv_gpu_sleep");
}
