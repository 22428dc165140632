/*
 * ogv.h — C-ABI of libogv_hip.so, the MI355X (gfx950) kernels behind the OutGridBlock hot path.
 *
 * The reference (pablo-reyes8/outlook-grid-vision-transformer) has no FFI: its hot path is a
 * set of nn.Modules whose arithmetic runs in ATen.  Each entry point below replaces the ATen op
 * chain named in its comment (reference file:line); the Python drop-in modules under
 * outlook-grid-vision-transformer_amd/src/model bind these through ctypes.
 *
 * Conventions
 *   - Activations are row-major [M, C] matrices with M = B*H*W in NHWC order (a channels_last
 *     NCHW tensor is exactly this layout), element type `ogv_dtype` (fp32 or bf16), fp32 math.
 *   - Weights/bias/affine parameters are fp32 (the AMP master copy); bf16 kernels round them
 *     to bf16 when staging.  Weight gradients are produced in fp32.
 *   - The library never allocates memory, frees or synchronises.  Scratch is passed in by the caller
 *     (sizes from the *_ws_bytes queries).  Every call enqueues on `stream` (a hipStream_t); the fused
 *     MBConv backward also forks independent weight-gradient work onto a library-owned side stream
 *     (created once per device) and joins it back into `stream` before returning (graph-capturable).
 *   - Return 0 on success; otherwise a non-zero code and ogv_last_error() (thread-local) says why.
 *     Shapes are validated on the host before any launch.
 */
#ifndef OGV_H
#define OGV_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef enum { OGV_F32 = 0, OGV_BF16 = 1 } ogv_dtype;
typedef enum { OGV_ACT_NONE = 0, OGV_ACT_GELU = 1, OGV_ACT_SILU = 2, OGV_ACT_RELU = 3 } ogv_act;

enum {
  OGV_OK = 0,
  OGV_ERR_ARG = 1,       /* bad shape / pointer / enum */
  OGV_ERR_UNSUPPORTED = 2,
  OGV_ERR_LAUNCH = 3     /* hipGetLastError after the launch */
};

const char* ogv_version(void);
const char* ogv_last_error(void);
/* Tuning switch (no reference counterpart; process-wide, set before capture):
 *   "sgemm" 1 (default) / 0: persistent streaming kernels (projection fwd/dgrad and weight gradient)
 *   for tall-skinny bf16 shapes on/off;  "sgemm_min_m" (default 65536): smallest M routed to them;
 *   "bk64_max_m": largest M using 64-wide k-steps in the tiled GEMM; "grid_mfma" 1/0: MFMA grid
 *   attention for bf16; "dw_blocks" (default 0 = ~32 rows per block): target block count of the
 *   depthwise kernels; "mb_side" 1/0: weight gradients of the fused MBConv backward on a side stream;
 *   "ln_bwd_blocks" (default 1024): grid cap of the LayerNorm backward; "sg_prefetch" (bit mask, default 3):
 *   bit 1 next-panel register prefetch in the streaming GEMM, bit 2 also for its prologue variants;
 *   "sg_per_cu" (default 2): streaming-GEMM workgroups per CU; "splitk_max" (default 32): K-slab
 *   cap of the fp32 split-K GEMM; "se_gemv" 1 (default) / 0: the Squeeze-Excite MLP on the GEMV
 *   kernels of ogv_se.hip instead of split-K GEMM + reduce; "outlook_vproj" 0/1/2/3: fused Outlooker
 *   projection + aggregation never / inference only / also training with the forward writing cat for
 *   the tiled backward (default) / training with the recompute backward ogv_outlook_vproj_bwd;
 *   "vp_tile" 0 (default) / 1-4: force a tile candidate of the fused Outlooker kernels; "wg2_fuse" 0
 *   (default) / 1: in-kernel last-workgroup reduction of the split-M weight gradient instead of the
 *   column-reduce launch (measured slower); "grid_big" 0/1/2 (default 2): one-(group, head)-pair-per-block
 *   LDS-resident grid attention for groups too large for the multi-pair kernels off / first generation /
 *   second generation (exp2 + lazy rescale + paired 16x16x32 MFMAs); "vp_dbg", "pg_dbg": phase-skipping timing experiments
 *   (wrong results); "bn_slices" (default 1024): cap on the row slices of the conv+BN statistics / backward
 *   reductions; "bn_red_rg" 16 / 64 (default): row groups per block of the fused BatchNorm finalize /
 *   coefficient reductions; "opt_chunk" (default 2048): elements per workgroup of ogv_clip_adamw (also
 *   sizes ogv_clip_adamw_ws_bytes); "pg_conv_rs1" 0 / 1 (default): 64-row statistics panels for small
 *   implicit-conv forwards; "mb_a3" 0 / 1 / 2 / 3 (default): how the fused MBConv keeps the project GEMM's input
 *   A3 = act(BN2(d)) * gate -- 0 recomputed in the GEMM prologues, 1 materialised in the forward workspace,
 *   2 materialised AND saved for the backward (ogv_mbconv_saved_bytes grows by [M, mid]), 3 = 2 where A3 is
 *   at most 512 MB else 1 (resolved per shape by ogv_mbconv_a3_mode; a desc with a3 >= 0 ignores the knob);
 *   "vp_head" 0 / 1 (default) / 2: the per-head fused Outlooker forward for the wide stages off / on / also
 *   head_dim 64 (two 32-column units per head); "vph_halo" 0 (default) / 1 / 2 / 3: its halo-tile form for images of
 *   more than 128 pixels off / where <= 4 units share a pixel (C = 128) / every wide shape / with 8-wave workgroups; "vph_tile" (TH * 100 + TW, 0 = auto): force its tile; "ln_epi" 0 / 1 (default) / 2: ogv_gemm_fwd_ln never / below
 *   sgemm_min_m rows / at every M; "pg_tconv1" 1 (default) / 0: a stride-2 transposed conv's four parity classes as one launch / four; "vp_l32" 1 (default) / 0: the fused Outlooker's fp32-logits form
 *   (ogv_outlook_vproj_l32_supported answers 0 with 0); "vph_rows" (0 = auto): target rows per panel of that kernel; "vph_wgs" (default 3):
 *   workgroups per CU its grid is sized for; "vph_dbg": phase-skipping timing experiments (wrong results);
 *   "dw_tw" 8 / 16 / 32 (default): column strip width of the depthwise kernels; "ln_rpi" 2 (default) / 4:
 *   rows per iteration of the LayerNorm kernels; "wg2_pbeta" (percent, 0 = off): cap the split-M weight gradient's slab
 *   count so its fp32 partials stay below that fraction of the launch's operand bytes (at least one workgroup per CU).
 * Options pick kernel plans, and every *_ws_bytes query sizes the workspace for the plans in force
 * when it is called: set options first, then size workspaces (a workspace sized under other option
 * values can be too small -- e.g. wg_blocks / wg_tile / swg_min_m change the split-M partial count).
 * Returns OGV_ERR_ARG for an unknown name. */
int ogv_set_option(const char* name, int value);
/* Diagnostics (no reference counterpart): which kernel ogv_gemm_fwd (kind 0) / ogv_gemm_dgrad
 * (kind 1) of this bf16 shape runs on (contiguous 16-B aligned operands): 1 = the persistent
 * streaming kernel (large M), 2 = the pipelined panel kernel (small M), 0 = the LDS-tiled kernel;
 * ogv_gpu_sleep queues a ~microseconds device-side spin on the stream (timing harnesses). */
int ogv_gemm_stream_route(int kind, int M, int N, int K, ogv_act act_in);
/* Deferred parameter-gradient reductions (no reference counterpart; a training-step scheduling
 * aid).  While ogv_reduce_defer(1) is in force, the final column reductions that turn slab partials
 * into PARAMETER gradients -- ogv_gemm_wgrad's dW / dbias, ogv_layernorm_bwd's dgamma / dbeta and the
 * expand / project / SE weight gradients of ogv_mbconv_bwd --
 * are recorded instead of launched (their workspaces must stay allocated, and the gradients unread,
 * until the flush); ogv_reduce_flush(stream) runs every recorded reduction as one batched launch
 * (48 per launch) on `stream`, which must be ordered after all the producing launches.  Returns: defer
 * -> the number of reductions pending; flush -> 0 or an error code. */
int ogv_reduce_defer(int on);
int ogv_reduce_flush(void* stream);
int ogv_gpu_sleep(int microseconds, void* stream);

/* ---------------------------------------------------------------------------------------------
 * Outlook aggregation.  Replaces, for stride 1:
 *   softmax over the k*k logits per (pixel, head)   src/model/outlook_attention.py:106-107
 *   F.unfold(v, k, padding=k//2) + mul + sum(-1)    src/model/outlook_attention.py:111-120
 * logits: [M, heads*k*k] (channel = head*k*k + ki*k + kj, unscaled), v: [M, C], y/dy: [M, C]
 * contiguous, M = B*H*W.  Zero-padded neighbours keep their softmax mass (reference semantics).
 * Row strides in elements: ld_logits (>= heads*k*k) for logits, ld_v (>= C) for v, ld_dv for dv,
 * ld_dlogits for dlogits -- so v and the logits may be the two column ranges of ONE [M, ld]
 * projection output (the fused v / attn 1x1 GEMM, OutlookAttention2d with no hooks on .attn/.v),
 * and dv / dlogits the matching column ranges of one gradient buffer.
 * bwd writes dv [M, C] and dlogits [M, heads*k*k]; columns [heads*k*k, dl_cols) of every dlogits
 * row are written with zeros (the padding columns of a concatenated gradient).  probs_ws is fp32
 * scratch of ogv_outlook_bwd_ws_bytes(...) bytes (0 = may be NULL: the LDS-tiled bf16 kernels,
 * k = 3 and head_dim % 8 == 0, <= 64, keep the probabilities in LDS).
 * ------------------------------------------------------------------------------------------- */
int ogv_outlook_agg_fwd(const void* v, const void* logits, void* y, int B, int H, int W, int C,
                        int heads, int k, int ld_logits, int ld_v, ogv_dtype dt, void* stream);
size_t ogv_outlook_bwd_ws_bytes(int B, int H, int W, int C, int heads, int k, ogv_dtype dt);

/* Outlooker forward FUSED with its v / attn projections (bf16, k = 3).  Replaces
 *   v = self.v(x); a = self.attn(x)                  src/model/outlook_attention.py:100,111
 *   softmax + F.unfold + mul + sum                   src/model/outlook_attention.py:106-120
 * x: [M, C] rows (row stride ldx, the LayerNorm2d output); w: fp32 [ldc, C] = [W_v; W_attn; 0]
 * (rows C .. C+heads*9-1 are attn.weight, the rest zero), bias: fp32 [ldc] or NULL.
 * Writes y [M, C] and, when cat != NULL, cat [M, ldc] = [v | logits | 0] rounded to bf16 (what
 * ogv_outlook_agg_bwd reads in training).  ldc must be C + heads*9 rounded up to 8.
 * ogv_outlook_vproj_supported() says whether a shape takes this kernel (16 | C <= 96, or the
 * weight-streaming variant for the wide stages C in {128, 192, 256, 384} with head_dim <= 64; 8 | head_dim)
 * for inference (train = 0) or training (train = 1) under knob "outlook_vproj":
 * 0 never; 1 inference only; 2 (default) training too, returning 1 = the forward writes cat for
 * ogv_outlook_agg_bwd; 3 returning 2 = the forward writes only y and ogv_outlook_vproj_bwd
 * recomputes [v | logits] (1 when that backward does not take the shape).
 * ogv_outlook_vproj_fwd itself runs any shape the kernel supports and returns OGV_ERR_ARG for the
 * others.
 * ogv_outlook_vproj_bwd: the backward of the same fused op with the projections RECOMPUTED from x
 * (the forward's weights and rounding, so v / logits are those the forward used): reads x, dy
 * ([M, C] contiguous) and writes dcat [M, ldc] = [dv | dlogits | 0], the gradient of the
 * concatenated projection output, for one dgrad + one wgrad of w.  Replaces the autograd of
 * src/model/outlook_attention.py:100-120 (unfold / softmax / fold).  16 | C <= 96 only:
 * ogv_outlook_vproj_bwd_supported() says whether it takes a shape (the wide stages save cat). */
int ogv_outlook_vproj_bwd_supported(int B, int H, int W, int C, int heads, int k, int ldc, ogv_dtype dt);
int ogv_outlook_vproj_supported(int B, int H, int W, int C, int heads, int k, int ldc, int train,
                                ogv_dtype dt);
int ogv_outlook_vproj_fwd(const void* x, int ldx, const float* w, const float* bias, void* cat, int ldc,
                          void* y, int B, int H, int W, int C, int heads, int k, ogv_dtype dt, void* stream);
/* The fp32-logits form of the fused Outlooker (training and inference; no reference counterpart -- a
 * precision choice): the same projections, softmax and gather as ogv_outlook_vproj_fwd, but the logits stay
 * fp32 -- the softmax reads them unrounded and training writes them to `logits` ([M, ld_logits] fp32,
 * ld_logits >= 9*heads rounded up to 4, 16-B rows) while `v` ([M, ld_v] bf16, ld_v >= C, 8 | ld_v) receives
 * only the v columns; both NULL = inference.  w is [C + 9*heads rounded up to 8, C] as above.  The
 * reference's own bf16 path rounds the attn conv's output (the logits) to bf16 (autocast); keeping them fp32
 * moves the bf16 gradients closer to the fp32 reference.
 * ogv_outlook_vproj_l32_supported: 1 when this form takes the shape (the per-head kernel where it plans,
 * else the tile kernel; not the weight-streaming kernel), knob "vp_l32" on.
 * ogv_outlook_agg_bwd_l32: ogv_outlook_agg_bwd reading those fp32 logits (the LDS-tiled backward only:
 * bf16, k = 3, 8 | head_dim <= 64). */
int ogv_outlook_vproj_l32_supported(int B, int H, int W, int C, int heads, int k, int train, ogv_dtype dt);
int ogv_outlook_vproj_fwd_l32(const void* x, int ldx, const float* w, const float* bias, void* v, int ld_v,
                              float* logits, int ld_logits, void* y, int B, int H, int W, int C, int heads, int k,
                              ogv_dtype dt, void* stream);
int ogv_outlook_agg_bwd_l32(const void* dy, const void* v, const float* logits, void* dv, void* dlogits,
                            int B, int H, int W, int C, int heads, int k, int ld_logits, int ld_v, int ld_dv,
                            int ld_dlogits, int dl_cols, ogv_dtype dt, void* stream);
int ogv_outlook_vproj_bwd(const void* x, int ldx, const float* w, const float* bias, const void* dy,
                          void* dcat, int ldc, int B, int H, int W, int C, int heads, int k, ogv_dtype dt,
                          void* stream);
int ogv_outlook_agg_bwd(const void* dy, const void* v, const void* logits, void* dv, void* dlogits,
                        float* probs_ws, int B, int H, int W, int C, int heads, int k, int ld_logits,
                        int ld_v, int ld_dv, int ld_dlogits, int dl_cols, ogv_dtype dt, void* stream);

/* ---------------------------------------------------------------------------------------------
 * Grid multi-head self-attention core.  Replaces
 *   grid_partition (strided regroup)                 src/model/grid_partition.py:3-17
 *   qkv reshape/permute, (q@k^T)*scale, softmax, @v  src/model/grid_attention.py:70-86
 *   grid_unpartition                                  src/model/grid_partition.py:20-32
 * The partition is folded into the addressing: group (b, gi, gj) holds the N = (H/g)*(W/g)
 * pixels (ty*g+gi, tx*g+gj), token index ty*(W/g)+tx.
 * qkv: [M, 3C] (channel = s*C + head*hd + d, s in {q,k,v}); out: [M, C]; lse: fp32 [M, heads]
 * (log-sum-exp of the scaled scores, saved for bwd).  probs (nullable) receives the
 * post-softmax matrix fp32 [B*g*g, heads, N, N] for the capture_attn hook (:77-83).
 * bwd: dqkv [M, 3C]; delta_ws fp32 [M, heads] scratch.
 * ------------------------------------------------------------------------------------------- */
int ogv_grid_attn_fwd(const void* qkv, void* out, float* lse, float* probs, int B, int H, int W, int C,
                      int heads, int g, float scale, ogv_dtype dt, void* stream);
int ogv_grid_attn_bwd(const void* dout, const void* qkv, const void* out, const float* lse, void* dqkv,
                      float* delta_ws, int B, int H, int W, int C, int heads, int g, float scale,
                      ogv_dtype dt, void* stream);

/* ---------------------------------------------------------------------------------------------
 * LayerNorm over the contiguous channel dim of [M, C] rows.  Replaces nn.LayerNorm inside
 * LayerNorm2d (src/model/outlook_attention.py:26-31, eps 1e-6) and OutGridBlock.norm2/norm3
 * (src/model/Out_Grid_Block.py:69,84, eps 1e-5).  mean/rstd: fp32 [M] (saved for bwd).
 * bwd: dx [M, C] (+ dres [M, C] when non-null: the gradient of a residual branch that reused x,
 * summed in the same pass); dgamma/dbeta fp32 [C] (overwritten); ws >= ogv_layernorm_bwd_ws_bytes(M, C).
 * ------------------------------------------------------------------------------------------- */
int ogv_layernorm_fwd(const void* x, const float* gamma, const float* beta, void* y, float* mean,
                      float* rstd, int M, int C, float eps, ogv_dtype dt, void* stream);
size_t ogv_layernorm_bwd_ws_bytes(int M, int C);
int ogv_layernorm_bwd(const void* dy, const void* x, const float* gamma, const float* mean,
                      const float* rstd, const void* dres, void* dx, float* dgamma, float* dbeta, void* ws,
                      int M, int C, ogv_dtype dt, void* stream);

/* ---------------------------------------------------------------------------------------------
 * Dense projection GEMMs on MFMA (1x1 Conv2d / nn.Linear of the hot path:
 * outlook_attention.py:83-88,37-40; grid_attention.py:57-59; Out_Grid_Block.py:18-21).
 *
 * fwd:   out[m,n] = res[m,n] + rs[m/rps] * ( sum_k act_in(A[m,k]) * W[n,k] + bias[n] )
 *        A: [M, K] (row stride lda), W: fp32 [N, K], out/res: [M, N] (row stride ldo).
 *        act_in is applied to A on load (the producer stored the pre-activation).
 *        res / rs / bias nullable; rps = rows per sample (H*W) for the per-sample DropPath scale.
 * dgrad: dA[m,k] = act_in'(Z[m,k]) * sum_n (rs[m/rps]*dOut[m,n]) * W[n,k]
 *        (Z = the pre-activation input of fwd, nullable when act_in = NONE).
 * wgrad: dW[n,k] = sum_m rs*dOut[m,n] * act_in(A[m,k]);  dbias[n] = sum_m rs*dOut[m,n]
 *        (dbias nullable).  dW/dbias are fp32 and overwritten; ws >= ogv_gemm_wgrad_ws_bytes.
 * ------------------------------------------------------------------------------------------- */
int ogv_gemm_fwd(const void* A, int lda, const float* W, const float* bias, const void* res,
                 const float* rs, int rps, void* out, int ldo, int M, int N, int K, ogv_act act_in,
                 ogv_dtype dt, void* stream);
/* Forward with a second output (no reference counterpart; fuses the activation module between two
 * Linear layers, src/model/Out_Grid_Block.py MLP fc1 -> act -> fc2): out = A . W^T + bias and
 * aout = act_out(out) of the stored bf16 values, both [M, N] bf16.  bf16 only. */
/* fwd fused with the residual stream's next LayerNorm (no reference counterpart: the producing Linear of a
 * pre-norm block -- Outlook_Block.py:58-60, Out_Grid_Block.py:100-102 -- hands LN its rows in registers):
 * out as ogv_gemm_fwd with act_in = NONE, and ln_out[m, :] = (out[m, :] - mean[m]) * rstd[m] * gamma + beta
 * (row stride ldo; mean / rstd fp32 [M], rstd = 1 / sqrt(var + eps), the biased variance of the stored bf16
 * row) -- what ogv_layernorm_fwd would compute from out.  bf16, N <= 192 (one column tile holds whole rows),
 * knob "ln_epi"; returns OGV_ERR_UNSUPPORTED with nothing launched otherwise (the caller runs ogv_gemm_fwd +
 * ogv_layernorm_fwd). */
int ogv_gemm_fwd_ln(const void* A, int lda, const float* W, const float* bias, const void* res, const float* rs,
                    int rps, void* out, int ldo, void* ln_out, const float* gamma, const float* beta, float eps,
                    float* mean, float* rstd, int M, int N, int K, ogv_dtype dt, void* stream);
int ogv_gemm_fwd_act(const void* A, int lda, const float* W, const float* bias, void* out, int ldo,
                     void* aout, int ldao, int M, int N, int K, ogv_act act_out, ogv_dtype dt, void* stream);
size_t ogv_gemm_dgrad_ws_bytes(int N, int K);
int ogv_gemm_dgrad(const void* dout, int ldd, const float* W, const void* Z, int ldz, const float* rs,
                   int rps, void* dA, int lda, int M, int N, int K, ogv_act act_in, void* ws,
                   ogv_dtype dt, void* stream);
size_t ogv_gemm_wgrad_ws_bytes(int M, int N, int K);
int ogv_gemm_wgrad(const void* dout, int ldd, const void* A, int lda, const float* rs, int rps,
                   float* dW, float* dbias, int M, int N, int K, ogv_act act_in, void* ws,
                   ogv_dtype dt, void* stream);

/* ---------------------------------------------------------------------------------------------
 * Depthwise 3x3 convolution, padding 1, stride 1|2, on NHWC rows.  Replaces MBConv.depthwise's
 * Conv2d(mid, mid, 3, stride, padding=1, groups=mid) (src/model/mbc_conv.py:75-79).
 * w: fp32 [C, 1, 3, 3]; bias nullable.  x: [B*H*W, C] -> y: [B*Ho*Wo, C].
 * bwd: dx (nullable) [B*H*W, C]; dw fp32 [C,1,3,3] and dbias fp32 [C] (nullable, overwritten).
 * ------------------------------------------------------------------------------------------- */
size_t ogv_dwconv_fwd_ws_bytes(int C);
int ogv_dwconv3x3_fwd(const void* x, const float* w, const float* bias, void* y, int B, int H, int W, int C,
                      int stride, void* ws, ogv_dtype dt, void* stream);
size_t ogv_dwconv_bwd_ws_bytes(int B, int H, int W, int C, int stride);
int ogv_dwconv3x3_bwd(const void* dy, const void* x, const float* w, void* dx, float* dw, float* dbias, int B,
                      int H, int W, int C, int stride, void* ws, ogv_dtype dt, void* stream);

/* ---------------------------------------------------------------------------------------------
 * Fused MBConv, stride 1, use_bn=True, expand_ratio != 1, se_ratio > 0 (the OutGridBlock
 * configuration).  Replaces MBConv.forward (src/model/mbc_conv.py:90-98) incl. SqueezeExcite
 * (:22-27) and the three BatchNorm2d (train: batch statistics + running-stat update, momentum;
 * eval: running statistics):
 *   e = x.We^T -> a1 = act(BN1(e)) -> d = dw3x3(a1) -> a2 = act(BN2(d)) -> g = SE(a2)
 *   -> p = (a2*g).Wp^T -> out = x + BN3(p)
 * x/out: [B*H*W, C] rows.  `saved` (>= ogv_mbconv_saved_bytes) is written by fwd and read by
 * bwd; `ws` (>= ogv_mbconv_ws_bytes) is scratch for either; bwd also takes `param_ws`
 * (>= ogv_mbconv_param_ws_bytes): the slab partials of its weight gradients (expand, project,
 * SE fc1 / fc2, depthwise), whose column reductions are deferred under ogv_reduce_defer -- keep it allocated
 * until ogv_reduce_flush.  bwd writes dx (= the residual
 * gradient + the branch gradient) and every parameter gradient (fp32, overwritten).
 * num_batches_tracked is left to the caller.
 * ------------------------------------------------------------------------------------------- */
typedef struct {
  int B, H, W, C;   /* input/output [B, C, H, W] (NHWC rows) */
  int mid, se;      /* expanded channels (int(round(C*expand_ratio))), squeeze channels */
  int train;        /* 1: BatchNorm batch statistics; 0: running statistics */
  float bn_eps, bn_momentum;
  int act;          /* ogv_act of MBConvConfig.act (silu in all reference configs) */
  int a3;           /* the saved-data variant: how the project GEMM's input A3 = act(BN2(d)) * gate is kept
                       (0 prologue, 1 forward workspace, 2 saved for the backward -- ogv_mbconv_saved_bytes
                       grows by [M, mid]); -1 = resolve knob "mb_a3" at each call.  Pin it with
                       ogv_mbconv_a3_mode() before the forward and pass the SAME desc to the backward: the
                       saved buffer's contents depend on it. */
} ogv_mbconv_desc;

typedef struct {
  const float* w_expand;                                  /* [mid, C, 1, 1] */
  const float *bn1_w, *bn1_b; float *bn1_rm, *bn1_rv;     /* [mid] */
  const float* w_dw;                                      /* [mid, 1, 3, 3] */
  const float *bn2_w, *bn2_b; float *bn2_rm, *bn2_rv;     /* [mid] */
  const float *se_w1, *se_b1;                             /* [se, mid, 1, 1], [se] */
  const float *se_w2, *se_b2;                             /* [mid, se, 1, 1], [mid] */
  const float* w_proj;                                    /* [C, mid, 1, 1] */
  const float *bn3_w, *bn3_b; float *bn3_rm, *bn3_rv;     /* [C] */
} ogv_mbconv_params;

typedef struct {
  float *w_expand, *bn1_w, *bn1_b, *w_dw, *bn2_w, *bn2_b, *se_w1, *se_b1, *se_w2, *se_b2, *w_proj, *bn3_w, *bn3_b;
} ogv_mbconv_grads;

/* the A3 mode knob "mb_a3" selects for this shape now (0, 1 or 2; -1 for a NULL desc) */
int ogv_mbconv_a3_mode(const ogv_mbconv_desc* desc, ogv_dtype dt);
size_t ogv_mbconv_saved_bytes(const ogv_mbconv_desc* desc, ogv_dtype dt);
size_t ogv_mbconv_ws_bytes(const ogv_mbconv_desc* desc, ogv_dtype dt);
size_t ogv_mbconv_param_ws_bytes(const ogv_mbconv_desc* desc);
int ogv_mbconv_fwd(const void* x, void* out, void* saved, void* ws, const ogv_mbconv_desc* desc,
                   const ogv_mbconv_params* params, ogv_dtype dt, void* stream);
int ogv_mbconv_bwd(const void* dout, const void* x, const void* saved, void* dx, const ogv_mbconv_grads* grads,
                   void* ws, void* param_ws, const ogv_mbconv_desc* desc, const ogv_mbconv_params* params,
                   ogv_dtype dt, void* stream);

/* ---------------------------------------------------------------------------------------------
 * MaxOutNet around the blocks: 3x3 convolution (padding 1, stride 1|2) -> BatchNorm2d -> act on
 * NHWC rows.  Replaces the stem  Conv2d(in, stem, 3, 1, 1) + BN + SiLU  (src/model/stem_head.py:
 * 23-32) and Downsample(kind="conv")  Conv2d(C, C', 3, 2, 1) + BN + SiLU  (src/model/
 * downsampling.py:28-65).  The convolution is an implicit GEMM on MFMA (tap-major K = 9*Cin);
 * BatchNorm follows nn.BatchNorm2d (train: biased batch variance for the normalisation, running
 * statistics updated with momentum and the unbiased variance; eval: running statistics).
 * x: [B*H*W, Cin] rows -> out: [B*Ho*Wo, Cout], Ho = (H-1)/stride + 1.  w: fp32 [Cout, Cin, 3, 3],
 * bias nullable (present when use_bn=False).  has_bn=0 skips the BatchNorm (bn_* ignored).
 * bwd: dx nullable (the stem's input needs no gradient); dw fp32 [Cout, Cin, 3, 3], dbias,
 * dbn_w, dbn_b fp32 [Cout] nullable, all overwritten.  num_batches_tracked is left to the caller.
 * ------------------------------------------------------------------------------------------- */
typedef struct {
  int B, H, W, Cin, Cout, stride;
  int has_bn, train;
  float bn_eps, bn_momentum;
  int act;
  int w_layout;   /* 0: w / dw stored [Cout, Cin, 3, 3]; 1: stored [Cout, 3, 3, Cin] (a channels_last
                     weight tensor, which is the tap-major matrix the kernels multiply by: no weight
                     transpose launches, dw written in place) */
} ogv_convbn_desc;

typedef struct {
  const float* w;                                   /* [Cout, Cin, 3, 3] (w_layout 0) or [Cout, 3, 3, Cin] */
  const float* bias;                                /* [Cout] or NULL */
  const float *bn_w, *bn_b; float *bn_rm, *bn_rv;   /* [Cout] */
} ogv_convbn_params;

size_t ogv_convbn_saved_bytes(const ogv_convbn_desc* desc, ogv_dtype dt);
size_t ogv_convbn_ws_bytes(const ogv_convbn_desc* desc, ogv_dtype dt);
int ogv_convbn_fwd(const void* x, void* out, void* saved, void* ws, const ogv_convbn_desc* desc,
                   const ogv_convbn_params* params, ogv_dtype dt, void* stream);
int ogv_convbn_bwd(const void* dout, const void* x, const void* saved, void* dx, float* dw, float* dbias,
                   float* dbn_w, float* dbn_b, void* ws, const ogv_convbn_desc* desc,
                   const ogv_convbn_params* params, ogv_dtype dt, void* stream);

/* ---------------------------------------------------------------------------------------------
 * BatchNorm2d (+ act) alone on [M, C] NHWC rows: MaxOutNet.head_norm (src/Model_A_OutGridNet.py:
 * 52,66; act NONE).  saved (>= ogv_bn_act_saved_bytes(C)) keeps mean/invstd/scale/shift for bwd.
 * ------------------------------------------------------------------------------------------- */
size_t ogv_bn_act_saved_bytes(int C);
size_t ogv_bn_act_ws_bytes(int M, int C);
int ogv_bn_act_fwd(const void* x, void* out, float* saved, void* ws, const float* bn_w, const float* bn_b,
                   float* running_mean, float* running_var, int M, int C, int train, float eps,
                   float momentum, int act, ogv_dtype dt, void* stream);
int ogv_bn_act_bwd(const void* dout, const void* x, const float* saved, void* dx, float* dbn_w, float* dbn_b,
                   void* ws, const float* bn_w, int M, int C, int train, int act, ogv_dtype dt,
                   void* stream);

/* ---------------------------------------------------------------------------------------------
 * The classifier head's BatchNorm2d + global average pool as ONE op (src/Model_A_OutGridNet.py:64-66,
 * src/Model_B_OutGridNet.py head): BatchNorm is a per-channel affine map, so mean_p(BN(x)) = BN(mean_p(x));
 * pooled[b, c] = sc[c] * (sum_p x[b, p, c] / HW) + sh[c] with the batch statistics (train, running-stat
 * update, shift = running mean as ogv_bn_act_fwd) or the running ones (eval), from ONE read of x [B*HW, C]
 * (image-major NHWC rows).  pooled_raw (fp32 [B, C], the plain means) and saved (>= ogv_bn_act_saved_bytes(C))
 * are kept for the backward, which writes dx from one read of x:
 *   dx[b, p, c] = gamma*invstd * (dpooled[b, c]/HW - sum_b dpooled/N - xhat[b, p, c] * sum_b dpooled*xhat_b/N)
 * (eval: gamma*invstd * dpooled/HW), xhat_b = (pooled_raw - mean)*invstd, N = B*HW; dgamma = sum_b dpooled*xhat_b,
 * dbeta = sum_b dpooled.  Replaces ogv_bn_act_fwd/bwd + the pool and its broadcast gradient (7 launches -> 6,
 * 10 passes over [B*HW, C] -> 2).
 * ------------------------------------------------------------------------------------------- */
size_t ogv_head_bn_pool_ws_bytes(int B, int C);
int ogv_head_bn_pool_fwd(const void* x, float* pooled_raw, float* pooled, float* saved, void* ws, const float* bn_w,
                         const float* bn_b, float* running_mean, float* running_var, int B, int HW, int C, int train,
                         float eps, float momentum, ogv_dtype dt, void* stream);
int ogv_head_bn_pool_bwd(const float* dpooled, const void* x, const float* pooled_raw, const float* saved, void* dx,
                         float* dbn_w, float* dbn_b, void* ws, const float* bn_w, int B, int HW, int C, int train,
                         ogv_dtype dt, void* stream);

/* ---------------------------------------------------------------------------------------------
 * Batch mixing (training-loop input side).  Replaces apply_mixup_cutmix's tensor work
 * (src/training/cutmix_mixup_aug.py:17-64: clone + images[perm] box paste, or
 * images*lam + images[perm]*(1-lam), and the one_hot(targets)*lam + one_hot(targets[perm])*(1-lam)
 * blend, :6-7 and :64); the host draws perm / lam / box exactly as the reference does.
 *   x, out  [B, C, H, W] contiguous NCHW (channels_last = 0) or NHWC (channels_last = 1), dtype dt;
 *           out must not alias x.  perm [B] int64 device indices in [0, B).
 *   mode    0 = MixUp: out = x*lam_a + x[perm]*lam_b (fp32 math, ATen's rounding points)
 *           1 = CutMix: out = x with rows y1..y2-1, columns x1..x2-1 taken from x[perm].
 * ogv_mix_targets: out [B, K] fp32 = onehot(t)*lam_a + onehot(t[perm])*lam_b; perm == NULL writes
 * onehot(t) (the no-mix branch, :30-34).  A label outside [0, K) (F.one_hot raises on it; raising
 * needs a device sync) gives a NaN row, so the loss is non-finite and the training step's device
 * guard (ogv_step_flag) skips the update and counts it. */
int ogv_mix_images(const void* x, void* out, const int64_t* perm, int B, int C, int H, int W, int channels_last,
                   int mode, float lam_a, float lam_b, int y1, int y2, int x1, int x2, ogv_dtype dt, void* stream);
int ogv_mix_targets(const int64_t* targets, const int64_t* perm, float* out, int B, int K, float lam_a, float lam_b,
                    void* stream);

/* Elementwise helpers used by the autograd glue. */
int ogv_cast(const void* src, ogv_dtype src_dt, void* dst, ogv_dtype dst_dt, size_t n, void* stream);

/* Batched fp32 segment copies (the data-parallel gradient bucket: the pack before the all_reduce and
 * the unpack after it replace torch.cat / _foreach_copy_, which issue one hipMemcpyAsync per tensor):
 * for every segment dst[0:numel] = src[0:numel] * scale, or = 0 when src is NULL.  `segs` is a HOST
 * array; 64 segments travel in each launch's kernel arguments (graph-capturable).  Segments must not
 * overlap.  Replaces nothing in the reference (it has no data parallelism: SURVEY §8e). */
typedef struct {
  const float* src;     /* NULL: zero fill */
  float* dst;
  long long numel;      /* < 2^31 */
} ogv_copy_seg;
int ogv_copy_batch_f32(const ogv_copy_seg* segs, int n, float scale, void* stream);

/* Gradient clipping + AdamW of one training step (src/training/one_epoch_train.py:121/141
 * clip_grad_norm_(model.parameters(), grad_clip_norm); src/training/train_full_model.py:57
 * torch.optim.AdamW(param_groups, betas=(0.9, 0.999), eps=1e-8)), as torch's
 * clip_grad_norm_(foreach) + AdamW(fused, capturable).step() compute them, on the optimizer's own
 * state tensors (a torch AdamW state_dict stays valid): total = sqrt(sum of every grad^2);
 * coef = min(max_norm / (total + 1e-6), 1) for max_norm >= 0 (NaN propagates; max_norm = 0 zeroes the
 * gradients as torch's clip_grad_norm_(max_norm=0) does); max_norm < 0: no clipping (grad_clip_norm=None); unless
 * *found_inf != 0 (then nothing changes): step += 1, grad *= coef (in place, as clip_grad_norm_),
 * param -= lr*wd*param, exp_avg = b1*exp_avg + (1-b1)*grad, exp_avg_sq = b2*exp_avg_sq + (1-b2)*grad^2 ((1-b) given),
 * param -= lr/(1-b1^step) * exp_avg / (sqrt(exp_avg_sq)/sqrt(1-b2^step) + eps).  All fp32, device
 * pointers; `tensors` / `groups` are HOST arrays (their pointers travel in kernel arguments: 64
 * tensors per launch, 2 launches per 64; graph-capturable).  lr is a device scalar per group (the
 * schedule writes it).  norm_ws: fp32 workspace of ogv_clip_adamw_ws_bytes(tensors, n). */
typedef struct {
  float* param;
  float* grad;
  float* exp_avg;
  float* exp_avg_sq;
  float* step;          /* device fp32 scalar (torch's capturable state['step']) */
  long long numel;      /* < 2^31 */
  int group;            /* index into groups[], < ngroups <= 4 */
} ogv_adamw_tensor;
typedef struct {
  const float* lr;      /* device fp32 scalar */
  float weight_decay, beta1, beta2, eps;
  float one_minus_beta1, one_minus_beta2;   /* rounded from double on the host, as torch forms them */
} ogv_adamw_group;
size_t ogv_clip_adamw_ws_bytes(const ogv_adamw_tensor* tensors, int n);
int ogv_clip_adamw(const ogv_adamw_tensor* tensors, int n, const ogv_adamw_group* groups, int ngroups,
                   const float* found_inf, float max_norm, float* norm_ws, void* stream);

/* Training loss: F.cross_entropy(logits, target, label_smoothing=ls), mean reduction, ignore_index
 * -100, over fp32 logits [B, K] row-major (src/training/one_epoch_train.py:96; torch's
 * cross_entropy_loss_label_smoothing).  Forward: a row pass (a wave per row) + a one-workgroup
 * fixed-order sum; backward: one launch.
 * ogv_ce_ls_fwd: *loss = (1-ls) * mean nll + (ls/K) * mean(-sum_k log_softmax); ws (ogv_ce_ls_ws_bytes)
 *   receives the per-row logsumexp and the count of non-ignored rows for the backward; found != NULL:
 *   *found = !isfinite(loss) (ogv_step_flag mode 0, fused).  A label outside [0, K) other than -100
 *   (torch raises; a raise needs a device sync) makes the loss NaN, so the guarded step is skipped, and
 *   bad_labels != NULL: *bad_labels += the number of such rows (a device counter the host reads to raise
 *   as torch does: a bad label is a data error, not a non-finite step).
 * ogv_ce_ls_bwd: dlogits = (*grad_loss / n) * (softmax - (1-ls) onehot - ls/K), 0 on ignored rows. */
size_t ogv_ce_ls_ws_bytes(int B);
int ogv_ce_ls_fwd(const float* logits, const int64_t* target, int B, int K, float label_smoothing, float* loss,
                  float* ws, float* found, float* bad_labels, void* stream);
int ogv_ce_ls_bwd(const float* logits, const int64_t* target, const float* ws, const float* grad_loss, int B, int K,
                  float label_smoothing, float* dlogits, void* stream);

/* Training-step guard and schedule (src/training/one_epoch_train.py:98-108, :152-153;
 * src/training/warmup.py:38-52), one single-thread launch each, capturable, no host sync:
 * ogv_step_flag: *found = 1.0f when the fp32 scalar *x is not finite (mode 0: x = the loss) or
 *   when *x > 0 (mode 1: x = the all-reduced count of ranks with a non-finite loss), else 0.0f.
 *   *found is the found_inf the fused AdamW reads (1 = the whole update is skipped).
 * ogv_schedule_step: after the optimizer: *nonfinite += *found; *counter += 1 - *found (the
 *   reference does not step its scheduler on a skipped step); then every group's lr tensor
 *   lr[g][0] = warmup-cosine(counter, base_lr[g]) computed in fp64 as warmup.py does.
 *   n_groups <= OGV_MAX_LR_GROUPS. */
#define OGV_MAX_LR_GROUPS 8
int ogv_step_flag(const float* x, int mode, float* found, void* stream);
int ogv_schedule_step(const float* found, float* counter, float* nonfinite, float* const* lr, const float* base_lr,
                      int n_groups, int warmup_steps, int total_steps, float min_lr, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* OGV_H */
