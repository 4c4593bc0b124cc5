/*
 * dsvt.h -- C-ABI of the MI355X (gfx950) DINO-SVT forward/loss hot path.
 *
 * The reference (Luke-537/Dino-Video-Summarization-Transformer) has no FFI: its hot path
 * is the PyTorch module API.  These entry points are what that API's implicit device
 * kernels become (SURVEY.md §2.2 K1-K14, §8(b) "What the C-ABI replacement must export").
 * Each entry point names the reference code it replaces.
 *
 * Conventions (all entry points):
 *   - plain device pointers + sizes, no framework types; `stream` is a hipStream_t;
 *   - dtype selects the activation/weight STORAGE type: DSVT_BF16 (perf mode: bf16 MFMA,
 *     fp32 accumulate) or DSVT_F32 (parity mode: fp32 MFMA / fp32 VALU). The residual
 *     token stream X, LayerNorm statistics, softmax statistics and losses are always fp32;
 *   - return 0 on success, non-zero on error; dsvt_last_error() gives the text
 *     (thread-local).  Nothing aborts, nothing allocates device memory: scratch space is
 *     a caller-provided workspace sized by dsvt_workspace_bytes();
 *   - all kernels are asynchronous on `stream` and safe to capture into a hipGraph.
 *
 * Token layout of X (models/timesformer.py:312, :322): X[b][i][c], i = 0 is CLS,
 * i = 1 + n*T + t is patch n of frame t ('b (n t) m').  Row maps: an operation that
 * reads or writes X through a row map uses  row(m) = (m / rpg) * gstride + goff + m % rpg.
 */
#ifndef DSVT_H
#define DSVT_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* 2 (r05): dsvt_bn_bwd takes param_sums (SyncBatchNorm's local dgamma / dbeta); dsvt_window_scatter_add
 * takes (row_scale, group) BEFORE stream -- a version-1 caller would pass its stream as row_scale;
 * DSVT_EPI_GELU_SAVE's aux holds GELU'(pre) (r04; was pre); the r03 grouped / stream-K / add-LN /
 * row-LN GEMM entry points are gone and the variant knobs moved to dsvt_debug.h (r04).  Added in 2:
 * dsvt_layernorm_bwd_params / _cast, the Swin training entries.  tests/test_capi_symbols.py freezes
 * every entry point's parameter count per ABI version: a signature change without a version bump
 * fails it. */
#define DSVT_ABI_VERSION 2

#define DSVT_BF16 0
#define DSVT_F32 1

/* GEMM epilogues (out = A[M,K] . W[N,K]^T, i.e. nn.Linear with weight [out,in]) */
#define DSVT_EPI_BIAS 0       /* out[row(m)] = acc + bias                  (Linear)          */
#define DSVT_EPI_BIAS_GELU 1  /* out[row(m)] = GELU_erf(acc + bias)        (Mlp.fc1 + act)   */
#define DSVT_EPI_BIAS_RESID 2 /* X[row(m)]  += acc + bias   (fp32 X)       (residual adds)   */
#define DSVT_EPI_GELU_SAVE 4  /* out = GELU_erf(acc + bias), aux = GELU_erf'(acc + bias) (fc1) */
#define DSVT_EPI_DGELU 5      /* out = acc * aux                          (fc1 backward)    */
/* OR-ed into the epilogue argument of dsvt_gemm_fwd / dsvt_ln_gemm_fwd: a few-row GEMM (the
 * CLS-only last block's rows, timesformer.py:181-184 on the CLS tokens, and the DINOHead MLP,
 * vision_transformer.py:271-281) -- the K-split skinny kernel where eligible, whatever M is, so a
 * batch split over streams stays bitwise equal to the whole batch.  A per-call flag: no state. */
#define DSVT_GEMM_FEW_ROWS 0x100

/* token orders for patch embedding */
#define DSVT_TOKENS_NT 0      /* divided / joint: X[b][1 + n*T + t]   (timesformer.py:312-323)  */
#define DSVT_TOKENS_FRAME 1   /* space_only / 2-D ViT: X[b*T + t][1 + n] (timesformer.py:288-306) */

/* probe families (bit mask) */
#define DSVT_PROBE_GEMM 1
#define DSVT_PROBE_ATTN_SPATIAL 2
#define DSVT_PROBE_ATTN_TEMPORAL 4
#define DSVT_PROBE_NORM 8
#define DSVT_PROBE_LOSS 16

/* workspace ops */
#define DSVT_WS_LN_GEMM 1
#define DSVT_WS_PATCH_EMBED 2
#define DSVT_WS_ATTN_SPATIAL 3
#define DSVT_WS_DINO_LOSS 4
#define DSVT_WS_PAIR_LOSS 5
#define DSVT_WS_LN_BWD 6
#define DSVT_WS_COLSUM 7
#define DSVT_WS_ATTN_BWD 8
#define DSVT_WS_EMBED_BWD 9
#define DSVT_WS_SELECT 10      /* M = number of scores, N = frames of the unsampled video */
#define DSVT_WS_AUGMENT 11     /* M = output frames T, N = output size S */
#define DSVT_WS_WGRAD 12       /* M = rows, N, K: the weight gradient is [N, K] */
#define DSVT_WS_ATTN_CLS 14    /* M = B*T sequences, N = heads, K = keys per sequence 1 + (L-1)/T */
#define DSVT_WS_ATTN_CLS_BWD 15 /* M = B*T sequences, N = heads */
#define DSVT_WS_ATTN_WIN_BWD 16 /* M = windows, N = heads, K = tokens per window */

int dsvt_version(void);
const char *dsvt_last_error(void);

/* Scratch bytes needed by an op (M,N,K meaning per op: LN_GEMM: rows, -, K;
 * PATCH_EMBED: patch rows, -, Cin*p*p; ATTN_SPATIAL: B*T, C, -; DINO_LOSS: pairs, rows, -;
 * PAIR_LOSS: rows, -, -). */
int64_t dsvt_workspace_bytes(int op, int dtype, int64_t M, int64_t N, int64_t K);

/* K4/K7/K9/K12: MFMA GEMM with fused epilogue.
 * Replaces nn.Linear in Attention.qkv/proj (models/timesformer.py:63-64, 71, 83),
 * temporal_fc (:108, :133), Mlp.fc1/act/fc2 (:41-52) and DINOHead.mlp / last_layer
 * (vision_transformer.py:255-281).  Requires K % 32 == 0 (bf16 calls with K % 64 != 0 -- Video
 * Swin's C = 96 -- run on the persistent kernel; r06, was K % 64), N % 4 == 0.  A rows are contiguous with stride lda (elements of dtype); W [N,K]
 * contiguous with stride ldw; out stride ldo (elements). out_f32 selects fp32 output for
 * EPI_BIAS / EPI_BIAS_GELU (otherwise dtype). */
int dsvt_gemm_fwd(int dtype, int epilogue, int out_f32, const void *A, int64_t lda, const void *W,
                  int64_t ldw, const float *bias, void *out, int64_t ldo, int64_t M, int64_t N,
                  int64_t K, int64_t rpg, int64_t gstride, int64_t goff, void *stream);
/* Out-of-place residual GEMM (training forward): x_out[row(m)] = x_in[row(m)] + A[m] . W^T +
 * bias, fp32 x_in / x_out with the same row map and row stride ldx, rows of x_out outside the
 * map untouched.  The reference's `x = x + drop_path(sublayer(norm(x)))`
 * (models/timesformer.py:133-135, 181, 184) with the pre-sublayer x kept intact for the
 * LayerNorm backward instead of copied. */
int dsvt_gemm_resid_fwd(int dtype, const void *A, int64_t lda, const void *W, int64_t ldw, const float *bias,
                        const float *x_in, float *x_out, int64_t ldx, int64_t M, int64_t N, int64_t K,
                        int64_t rpg, int64_t gstride, int64_t goff, void *stream);

/* Training-mode DropPath form of dsvt_gemm_resid_fwd (identity row map):
 *   x_out[m] = x_in[m] + A[m] . W^T + bias_row_scale[m] * bias
 * A already carries the per-sample DropPath scale (models/vit_utils.py:152-167: drop_path of
 * attn / mlp, timesformer.py:181, 184 -- the scaled branch is linear in A), so only the bias
 * term takes the row scale; replaces a GEMM without bias + a separate scaled-bias pass. */
int dsvt_gemm_resid_scaled_fwd(int dtype, const void *A, int64_t lda, const void *W, int64_t ldw, const float *bias,
                               const float *bias_row_scale, const float *x_in, float *x_out, int64_t ldx, int64_t M,
                               int64_t N, int64_t K, void *stream);

/* ------------------------------------------------------------------------------------------
 * LayerNorm folded into the GEMM that reads it (bf16, C = 768): norm1 -> attn.qkv, temporal_norm1
 * -> temporal_attn.qkv, norm2 -> mlp.fc1 (models/timesformer.py:127/131, :159, :184).  With
 * W' = W * gamma and mu / rstd the row's statistics,
 *   LayerNorm(x) . W^T + b = rstd * (x . W'^T - mu * sum_k W'[n, k]) + (b + W . beta),
 * so the GEMM reads the bf16 copy of the fp32 token row directly and applies the affine in its
 * epilogue; the row statistics come as LN_PARTS = 12 float2 (sum x, sum x^2) partials per row
 * (one per 64-column slab), written by the residual GEMM that produced the row
 * (dsvt_gemm_resid_stats_fwd: attn.proj / temporal_fc / mlp.fc2 + residual, :133-135, 181, 184)
 * or, for the rows a forward starts with, by dsvt_ln_stats_fwd.  No LayerNorm pass and no
 * normalized copy of the rows in HBM.
 * ------------------------------------------------------------------------------------------ */
#define DSVT_LN_FOLD_C 768
#define DSVT_LN_PARTS 12
/* Wf [N, K] bf16 = W * gamma (per column k), wsum[N] = row sums of Wf, bias_f[N] = bias + W . beta
 * (bias nullable).  W [N, K] fp32 (nn.Linear weight), gamma / beta [K] (the nn.LayerNorm before it). */
int dsvt_ln_fold_weights(const float *W, const float *gamma, const float *beta, const float *bias, void *Wf,
                         float *wsum, float *bias_f, int64_t N, int64_t K, void *stream);
/* xb [rows, 768] bf16 = x, stats [rows, 12] float2 = the partials of x [rows, 768] fp32. */
int dsvt_ln_stats_fwd(const float *x, void *xb, float *stats, int64_t rows, int64_t C, void *stream);
/* The residual GEMM X[row(m)] += A[m] . W^T + bias (as dsvt_gemm_fwd, DSVT_EPI_BIAS_RESID, bf16,
 * N = ldx = 768) that also writes, for every row it updates, xb[row] = bf16(X[row]) and
 * stats[row][12] (the partials dsvt_gemm_lnx_fwd reads). */
int dsvt_gemm_resid_stats_fwd(const void *A, int64_t lda, const void *W, int64_t ldw, const float *bias, float *X,
                              void *xb, float *stats, int64_t ldx, int64_t M, int64_t N, int64_t K, int64_t rpg,
                              int64_t gstride, int64_t goff, void *stream);
/* out[row(m)] = epilogue(LayerNorm(x[a_row(m)]) . W^T + b) with xb = bf16(x) rows (ldxb) read
 * through the A row map a_row(m) = (m / a_rpg) * a_gstride + a_goff + m % a_rpg (a_rpg <= 0:
 * identity), stats[a_row(m)] their partials, Wf / wsum / bias_f from dsvt_ln_fold_weights;
 * epilogue DSVT_EPI_BIAS or DSVT_EPI_BIAS_GELU, bf16 out, K = 768, N % 256 == 0.  Replaces
 * dsvt_ln_gemm_fwd on the bf16 hot path (same results up to the bf16 rounding of x and W*gamma). */
int dsvt_gemm_lnx_fwd(int epilogue, const void *xb, int64_t ldxb, int64_t a_rpg, int64_t a_gstride, int64_t a_goff,
                      const float *stats, float eps, const void *Wf, const float *wsum, const float *bias_f, void *out,
                      int64_t ldo, int64_t M, int64_t N, int64_t K, int64_t rpg, int64_t gstride, int64_t goff,
                      void *stream);
/* The temporal branch's LayerNorm -> qkv -> T = 8 attention in ONE kernel (temporal_norm1 ->
 * temporal_attn, models/timesformer.py:127-131 with Attention.forward :55-87 over the
 * 'b (h w t) m -> (b h w) t m' sequences): out[m][h*64 + d] (bf16, compact patch rows m, ldo) =
 * the attention output of head h for token m -- what dsvt_gemm_lnx_fwd into a [M, 3C] qkv
 * followed by dsvt_attn_temporal_fwd gives, without the qkv tensor in HBM.  The patch rows m are
 * read through the A row map like dsvt_gemm_lnx_fwd; consecutive groups of T rows are the
 * sequences (M a multiple of T); T == 8, heads * 64 == 768; scale = head_dim ** -0.5.
 * Wf / wsum / bias_f: the qkv weight folded with the LayerNorm in the head-interleaved row order of
 * dsvt_ln_fold_qkv_heads. */
int dsvt_qkv_temporal_attn_fwd(const void *xb, int64_t ldxb, int64_t a_rpg, int64_t a_gstride, int64_t a_goff,
                               const float *stats, float eps, const void *Wf, const float *wsum, const float *bias_f,
                               void *out, int64_t ldo, int64_t M, int64_t heads, int64_t T, float scale, void *stream);
/* dsvt_ln_fold_weights for an attention qkv weight W [3 * heads * 64, K] with its rows written in
 * the head-interleaved order dsvt_qkv_temporal_attn_fwd reads: row part*C + h*64 + d (part = q, k,
 * v; C = heads * 64) goes to row h*192 + (d / 32)*96 + part*32 + d % 32 of Wf / wsum / bias_f. */
int dsvt_ln_fold_qkv_heads(const float *W, const float *gamma, const float *beta, const float *bias, void *Wf,
                           float *wsum, float *bias_f, int64_t heads, int64_t K, void *stream);

/* ------------------------------------------------------------------------------------------
 * DINOHead(use_bn=True) (vision_transformer.py:255-262, --use_bn_in_head; train_ssl.py:319-321
 * makes them SyncBatchNorm): Linear -> BatchNorm1d -> GELU per hidden layer.  x [R, D] fp32 is the
 * Linear's output; sums [2D] fp64 = (column sums, column sums of squares) -- for SyncBatchNorm the
 * caller all-reduces sums and the row count over the group between dsvt_bn_stats_fwd and
 * dsvt_bn_finalize.  training = 1: batch statistics (biased variance normalises) and the running
 * estimates updated in place (unbiased variance, momentum); 0: the running statistics.
 * dsvt_bn_gelu_fwd: y = GELU_erf((x - mean) * rstd * gamma + beta) in dtype, optionally GELU'(.)
 * (dtype) and xhat (fp32) for the backward.  Backward from dz = dL/d(BatchNorm output):
 * dsvt_bn_bwd_sums (sum dz, sum dz * xhat; all-reduced for SyncBatchNorm), then dsvt_bn_bwd:
 * dx = gamma * rstd * (dz - sum dz / count - xhat * sum(dz xhat) / count) (fp32) from `sums`,
 * dgamma = sum dz xhat, dbeta = sum dz (nullable, accumulate into them when accumulate != 0) from
 * `param_sums` -- for SyncBatchNorm the LOCAL (un-reduced) sums, as torch's SyncBatchNorm returns
 * local weight / bias gradients that DDP then averages; NULL = `sums`.
 * ------------------------------------------------------------------------------------------ */
int dsvt_bn_stats_fwd(const float *x, int64_t R, int64_t D, double *sums, void *stream);
int dsvt_bn_finalize(const double *sums, double count, int64_t D, float eps, float momentum, int training,
                     float *running_mean, float *running_var, float *mean, float *rstd, void *stream);
int dsvt_bn_gelu_fwd(int dtype, const float *x, const float *mean, const float *rstd, const float *gamma,
                     const float *beta, void *y, void *gelu_grad, float *xhat, int64_t R, int64_t D, void *stream);
int dsvt_bn_bwd_sums(int dtype, const void *dz, const float *xhat, int64_t R, int64_t D, double *sums, void *stream);
int dsvt_bn_bwd(int dtype, const void *dz, const float *xhat, const double *sums, const double *param_sums,
                double count, const float *gamma,
                const float *rstd, float *dx, float *dgamma, float *dbeta, int accumulate, int64_t R, int64_t D,
                void *stream);

/* K3: LayerNorm(eps) over rows of fp32 X read through a row map, written compact
 * (rows x C) in dtype (or fp32 when out_f32 bit 0); with out_f32 bit 1 the output rows follow
 * the same row map as the input.  nn.LayerNorm(eps=1e-6) at
 * models/timesformer.py:99,105,112,131,159,184,245,342. */
int dsvt_layernorm_fwd(int dtype, int out_f32, const float *x, void *y, const float *gamma,
                       const float *beta, int64_t rows, int64_t C, int64_t rpg, int64_t gstride,
                       int64_t goff, float eps, void *stream);

/* K3+K4 / K3+K9: LayerNorm prologue + GEMM (norm1->qkv, temporal_norm1->temporal qkv,
 * norm2->fc1: models/timesformer.py:131, :159, :184).  x rows read through (in_rpg,
 * in_gstride, in_goff); the normalized rows go through `workspace`. */
int dsvt_ln_gemm_fwd(int dtype, int epilogue, int out_f32, const float *x, int64_t in_rpg,
                     int64_t in_gstride, int64_t in_goff, const float *gamma, const float *beta,
                     float eps, const void *W, const float *bias, void *out, int64_t ldo,
                     int64_t M, int64_t N, int64_t K, int64_t rpg, int64_t gstride, int64_t goff,
                     void *workspace, int64_t workspace_bytes, void *stream);

/* K1+K2: PatchEmbed (Conv2d k=s=16 as im2col GEMM, models/timesformer.py:203-209) fused
 * with the CLS concat, pos-embed add (nearest-resized via pos_index, :288-306) and
 * time-embed add (nearest-resized via time_index, :309-323).  x is [B,Cin,T,H,W] fp32.
 * w is the conv weight [C, Cin*16*16] in dtype; pos_embed [1+P*P, C] fp32 with
 * pos_index[Np] indexing the P*P grid; time_embed [T0, C] (NULL for space_only) with
 * time_index[T].  Writes X fp32: tokens_order DSVT_TOKENS_NT -> [B, 1+Np*T, C],
 * DSVT_TOKENS_FRAME -> [B*T, 1+Np, C].  frame_index (nullable): x is then a frame bank
 * [F, Cin, H, W] and frame t of clip b is x[frame_index[b*T + t]] (-1 = zero frame) -- the
 * per-frame local/global views of datasets_custom/dino_loss_loader.py:126-171 without
 * materializing them. */
int dsvt_patch_embed_fwd(int dtype, int tokens_order, const float *x, int64_t B, int64_t Cin,
                         int64_t T, int64_t H, int64_t W, int64_t patch, const void *w,
                         const float *bias, const float *cls_token, const float *pos_embed,
                         const int32_t *pos_index, const float *time_embed,
                         const int32_t *time_index, int64_t C, float *X,
                         const int32_t *frame_index, void *workspace, int64_t workspace_bytes,
                         void *stream);

/* vision_transformer.py:174-194 interpolate_pos_encoding: bicubic (A=-0.75,
 * align_corners=False, scale_factor semantics of ATen upsample_bicubic2d) resize of the
 * s x s patch grid of pos_embed [1+s*s, C] to out [1+OH*OW, C] (row 0 = CLS pos copied). */
int dsvt_pos_bicubic_fwd(const float *pos_embed, float *out, int64_t s, int64_t OH, int64_t OW,
                         int64_t C, double scale_h, double scale_w, void *stream);
/* Its backward (2-D ViT training): dpos [1+s*s, C] (+)= the transpose of that linear map applied
 * to dout [1+OH*OW, C] (fp32; a gather per source cell, no atomics). */
int dsvt_pos_bicubic_bwd(const float *dout, float *dpos, int64_t s, int64_t OH, int64_t OW, int64_t C,
                         double scale_h, double scale_w, int accumulate, void *stream);

/* K5: temporal attention of the divided block (models/timesformer.py:127-131 via
 * Attention.forward :68-87).  qkv compact [(nseq*T), 3C] (sequence = (b,n), T rows each),
 * out [(nseq*T), C].  head_dim must be 64, T <= 64. */
int dsvt_attn_temporal_fwd(int dtype, const void *qkv, void *out, int64_t nseq, int64_t T,
                           int64_t heads, int64_t head_dim, float scale, void *stream);

/* K6+K8: spatial attention of the divided block with the CLS replicate / mean over
 * frames (models/timesformer.py:139-175).  qkv rows follow X's token layout
 * ([B*L, 3C]); sequence (b,t) = {CLS row b*L} U {row b*L + 1 + n*T + t}.  Patch outputs go
 * to out at the same rows; the CLS output is the mean over t, written to row b*L.
 * workspace: >= dsvt_workspace_bytes(DSVT_WS_ATTN_SPATIAL, ., B*T, C, 0). */
int dsvt_attn_spatial_fwd(int dtype, const void *qkv, void *out, int64_t B, int64_t T, int64_t L,
                          int64_t heads, int64_t head_dim, float scale, void *workspace,
                          int64_t workspace_bytes, void *stream);
/* The CLS output ONLY of dsvt_attn_spatial_fwd: for every frame sequence (b,t) the attention of
 * the CLS query (row b*L) over CLS + the N patch rows of frame t, averaged over t, written to
 * out[b*ld_out + c] (c < C; compact rows).  Replaces the last block's attention when
 * VisionTransformer.forward_features returns the CLS token only (models/timesformer.py:139-167,
 * 341-345): that block's patch-row outputs never reach the result.  T = 1 is the joint /
 * space-only case: sequence b = the L contiguous rows b*L ... (models/timesformer.py:120-123).
 * Keys are split in chunks of 256 (one wave each) and merged; workspace >=
 * dsvt_workspace_bytes(DSVT_WS_ATTN_CLS, ., B*T, heads, 1 + (L-1)/T). */
int dsvt_attn_spatial_cls_fwd(int dtype, const void *qkv, void *out, int64_t ld_out, int64_t B, int64_t T,
                              int64_t L, int64_t heads, int64_t head_dim, float scale, void *workspace,
                              int64_t workspace_bytes, void *stream);
/* dsvt_attn_spatial_cls_fwd with frame t's output scaled by seq_scale[b*T + t] before the mean over
 * frames: the training CLS-only last block under DropPath (timesformer.py:159 drop_path over the
 * [(B*T), 1+N, C] batch, then the CLS mean :160-163). */
int dsvt_attn_spatial_cls_scaled_fwd(int dtype, const void *qkv, void *out, int64_t ld_out, const float *seq_scale,
                                     int64_t B, int64_t T, int64_t L, int64_t heads, int64_t head_dim, float scale,
                                     void *workspace, int64_t workspace_bytes, void *stream);
/* Backward of dsvt_attn_spatial_cls_fwd / _scaled_fwd (the training CLS-only last block: the
 * patch rows' queries do not exist there): dqkv [B*L, 3C] (storage dtype, every row written) from
 * qkv and dout [B, C] (the gradient of the frame-mean CLS output, storage dtype, compact rows).
 * Patch rows get the dk / dv of their frame's CLS query and dq = 0; the CLS row the sums over t
 * of its dq, dk, dv (fixed order).  seq_scale nullable.  Keys per sequence <= 512.
 * workspace >= dsvt_workspace_bytes(DSVT_WS_ATTN_CLS_BWD, ., B*T, heads, 0). */
int dsvt_attn_spatial_cls_bwd(int dtype, const void *qkv, const void *dout, void *dqkv, const float *seq_scale,
                              int64_t B, int64_t T, int64_t L, int64_t heads, int64_t head_dim, float scale,
                              void *workspace, int64_t workspace_bytes, void *stream);
/* dsvt_attn_spatial_fwd with the output of sequence (b,t) scaled by seq_scale[b*T + t] before the
 * CLS mean: training-mode DropPath of the spatial branch, whose mask is per (b,t) sequence
 * (timesformer.py:159 drop_path over the [(B*T), 1+N, C] batch). */
int dsvt_attn_spatial_scaled_fwd(int dtype, const void *qkv, void *out, const float *seq_scale, int64_t B,
                                 int64_t T, int64_t L, int64_t heads, int64_t head_dim, float scale,
                                 void *workspace, int64_t workspace_bytes, void *stream);
/* Same as dsvt_attn_spatial_fwd, and also writes the softmax probabilities of every frame
 * sequence (CLS + N patches) to probs [B*T][heads][1+N][1+N] fp32 -- the last-block
 * attention map of VisionTransformer.forward_features(get_attn=True), models/timesformer.py:
 * 77-78, 155-157, 325-331.  bf16 mode: 1+N <= 256. */
int dsvt_attn_spatial_probs_fwd(int dtype, const void *qkv, void *out, float *probs, int64_t B, int64_t T,
                                int64_t L, int64_t heads, int64_t head_dim, float scale, void *workspace,
                                int64_t workspace_bytes, void *stream);

/* K10: plain (joint space-time / space-only / 2-D ViT) attention over each of nb
 * contiguous sequences of L rows (models/timesformer.py:120-123, vision_transformer.py:80-92). */
int dsvt_attn_joint_fwd(int dtype, const void *qkv, void *out, int64_t nb, int64_t L,
                        int64_t heads, int64_t head_dim, float scale, void *stream);

/* CLS mean over frames for space_only (models/timesformer.py:338-340) and dtype casts. */
int dsvt_frame_mean_fwd(const float *x, float *y, int64_t B, int64_t T, int64_t rowlen,
                        void *stream);
int dsvt_cast_fwd(int dtype, const float *x, void *y, int64_t n, void *stream);

/* K12 pieces: F.normalize(x, dim=-1, p=2, eps) (vision_transformer.py:280) and the
 * weight-norm of DINOHead.last_layer (w = g * v / ||v||_row, :267-269). */
int dsvt_dino_head_norm_fwd(int dtype, const float *x, void *y, int64_t rows, int64_t D,
                            float eps, void *stream);
int dsvt_weight_norm_fwd(int dtype, const float *v, const float *g, void *w, int64_t rows,
                         int64_t D, void *stream);

/* K13+K14: DINOLoss.forward (train_ssl.py:633-671, two_token=False).  student
 * [ncrops*B, D], teacher [global_crops*B, D], center [D], all fp32.  Writes the scalar
 * loss to loss_out[0] (device) and the teacher column sum (pre all-reduce,
 * train_ssl.py:686) to teacher_colsum[D].  No host sync. */
int dsvt_dino_loss_fwd(const float *student, const float *teacher, const float *center,
                       int64_t B, int64_t ncrops, int64_t global_crops, int64_t D,
                       float student_temp, float teacher_temp, float *loss_out,
                       float *teacher_colsum, void *workspace, int64_t workspace_bytes,
                       void *stream);

/* dino_similarity.DINOLoss (dino_similarity.py:129-135), one loss per row pair -- the
 * per-frame importance score (dino_similarity.py:87-88). */
int dsvt_dino_pair_loss_fwd(const float *student, const float *teacher, const float *center,
                            int64_t rows, int64_t D, float student_temp, float teacher_temp,
                            float *out, void *workspace, int64_t workspace_bytes, void *stream);

/* K14: center = center*momentum + colsum*(1-momentum)*inv_count (train_ssl.py:687-691,
 * after the caller's all-reduce of colsum). */
int dsvt_center_ema(float *center, const float *colsum, int64_t D, float momentum,
                    float inv_count, void *stream);

/* ------------------------------------------------------------------------------------------
 * Backward / training step (loss.backward() at train_ssl.py:538/545).
 * Gradients are fp32 and ACCUMULATED where `accumulate` != 0 (param.grad semantics).  The
 * weight-gradient GEMMs dW = dY^T . X are plain library GEMMs on the host side; these entry
 * points are the rest of the backward.
 * ------------------------------------------------------------------------------------------ */

/* dsvt_gemm_fwd with a second storage-dtype operand aux [M, ld_aux] (rows through the output
 * row map): DSVT_EPI_GELU_SAVE (Mlp.fc1 + nn.GELU saving GELU'(pre-activation), timesformer.py:
 * 46-47) or DSVT_EPI_DGELU (dX of fc1 through GELU: out = (dY . W2) * aux, aux = GELU'(pre)). */
int dsvt_gemm_aux_fwd(int dtype, int epilogue, int out_f32, const void *A, int64_t lda, const void *W,
                      int64_t ldw, const float *bias, void *out, int64_t ldo, void *aux, int64_t ld_aux,
                      int64_t M, int64_t N, int64_t K, int64_t rpg, int64_t gstride, int64_t goff,
                      void *stream);
/* dsvt_gemm_fwd (DSVT_EPI_BIAS, storage-dtype out) / dsvt_gemm_aux_fwd (DSVT_EPI_GELU_SAVE) with
 * output row m scaled by row_scale[m / rs_group] after the bias / GELU -- the training
 * DropPath of the sample that row belongs to (models/vit_utils.py:152-167; timesformer.py:
 * 133 temporal branch before temporal_fc, :184 MLP branch); the saved pre-activation aux is
 * not scaled.  No row map (rows are the GEMM's own). */
int dsvt_gemm_rowscale_fwd(int dtype, int epilogue, const void *A, int64_t lda, const void *W, int64_t ldw,
                           const float *bias, void *out, int64_t ldo, void *aux, int64_t ld_aux, int64_t M,
                           int64_t N, int64_t K, const float *row_scale, int64_t rs_group, void *stream);
/* nn.LayerNorm backward: dx[row(m)] += dLN(x[row(m)], dy[m]) (dx has x's layout: the residual
 * gradient of the pre-LN sub-layer), dgamma/dbeta (+)= column sums.  dy_dtype: storage dtype of
 * dy (DSVT_BF16 or DSVT_F32).  workspace >= dsvt_workspace_bytes(DSVT_WS_LN_BWD, ., rows, 0, C). */
int dsvt_layernorm_bwd(int dy_dtype, const float *x, const void *dy, const float *gamma, float *dx,
                       int64_t rows, int64_t C, int64_t rpg, int64_t gstride, int64_t goff, float eps,
                       float *dgamma, float *dbeta, int accumulate, void *workspace,
                       int64_t workspace_bytes, void *stream);
/* dgamma = dbeta = NULL in dsvt_layernorm_bwd: the affine-parameter partial sums stay in its workspace
 * and this finishes them (fixed order, (+)= into dgamma / dbeta) -- on another stream if the caller
 * likes (the training backward runs them beside the dX chain), after the dsvt_layernorm_bwd. */
int dsvt_layernorm_bwd_params(int64_t rows, int64_t C, const void *workspace, int64_t workspace_bytes, float *dgamma,
                              float *dbeta, int accumulate, void *stream);
/* dsvt_layernorm_bwd for C = 768 that also stores each updated dx row as bf16 into dxb [*, 768]
 * (the copy the next GEMMs of the dX chain read): token row r goes to dxb row
 * (r / og) * (og - osk) + r % og - osk when r % og >= osk (og = rows, osk = 0: the same rows;
 * og = L, osk = 1: the patch rows of [B, L] token rows, compact), replacing a cast pass over dx. */
int dsvt_layernorm_bwd_cast(int dy_dtype, const float *x, const void *dy, const float *gamma, float *dx, int64_t rows,
                            int64_t C, int64_t rpg, int64_t gstride, int64_t goff, float eps, float *dgamma,
                            float *dbeta, int accumulate, void *dxb, int64_t og, int64_t osk, void *workspace,
                            int64_t workspace_bytes, void *stream);
/* bias gradient: out[c] (+)= sum_m row_scale[m] * y[row(m)][c]  (y in dtype, row stride ld;
 * row_scale nullable = 1). */
int dsvt_colsum_bwd(int dtype, const void *y, int64_t rows, int64_t C, int64_t ld, int64_t rpg,
                    int64_t gstride, int64_t goff, const float *row_scale, float *out, int accumulate,
                    void *workspace, int64_t workspace_bytes, void *stream);
/* Attention backward: dqkv [rows, 3C] (same layout as qkv) from qkv and dout [rows, C].
 * temporal: as dsvt_attn_temporal_fwd; spatial: as dsvt_attn_spatial_fwd (the CLS row's dout is
 * the gradient of the frame MEAN, its dq/dk/dv are summed over frames); joint: contiguous
 * sequences.  seq_scale (nullable): the forward's per-(b,t) DropPath scale, applied to dout.
 * workspace >= dsvt_workspace_bytes(DSVT_WS_ATTN_BWD, ., B*T (or nb), C, seqlen). */
int dsvt_attn_temporal_bwd(int dtype, const void *qkv, const void *dout, void *dqkv, int64_t nseq,
                           int64_t T, int64_t heads, int64_t head_dim, float scale, void *stream);
int dsvt_attn_spatial_bwd(int dtype, const void *qkv, const void *dout, void *dqkv, const float *seq_scale,
                          int64_t B, int64_t T, int64_t L, int64_t heads, int64_t head_dim, float scale,
                          void *workspace, int64_t workspace_bytes, void *stream);
int dsvt_attn_joint_bwd(int dtype, const void *qkv, const void *dout, void *dqkv, int64_t nb, int64_t L,
                        int64_t heads, int64_t head_dim, float scale, void *workspace,
                        int64_t workspace_bytes, void *stream);
/* DINOLoss backward (train_ssl.py:653-669): dstudent = dloss[0] * d loss / d student_output
 * (the teacher branch is detached).  Same workspace as dsvt_dino_loss_fwd. */
int dsvt_dino_loss_bwd(const float *student, const float *teacher, const float *center, int64_t B,
                       int64_t ncrops, int64_t global_crops, int64_t D, float student_temp,
                       float teacher_temp, const float *dloss, float *dstudent, void *workspace,
                       int64_t workspace_bytes, void *stream);
/* F.normalize backward (vision_transformer.py:280) and weight-norm backward (dv, dg). */
int dsvt_dino_head_norm_bwd(const float *x, const float *dz, float *dx, int64_t rows, int64_t D,
                            float eps, void *stream);
int dsvt_weight_norm_bwd(const float *v, const float *g, const float *dw, float *dv, float *dg,
                         int64_t rows, int64_t D, int accumulate, void *stream);
/* y[m] = cast(x[row(m)] * row_scale[m / group]) (compact gather of row-mapped fp32 rows,
 * row_scale nullable); y = cast(x)^T for x [R, C]. */
int dsvt_cast_rows(int dtype, const float *x, void *y, int64_t rows, int64_t C, int64_t rpg,
                   int64_t gstride, int64_t goff, const float *row_scale, int64_t group, void *stream);
/* Training DropPath (models/vit_utils.py:152-167) on a residual branch: y[m] *= row_scale[m/group]
 * in place (ld = row stride), and X[m] += row_scale[m] * bias (a branch bias under DropPath). */
int dsvt_row_scale(int dtype, void *y, int64_t rows, int64_t C, int64_t ld, const float *row_scale,
                   int64_t group, void *stream);
int dsvt_rowscale_bias_add(float *X, int64_t rows, int64_t C, const float *row_scale, const float *bias,
                           void *stream);
int dsvt_cast_transpose(int dtype, const float *x, void *y, int64_t R, int64_t C, void *stream);
/* Token-embedding gradients from dX [B, 1 + Np*T, C] (NT order): dpos[1 + pos_index[n]] +=,
 * dtime[time_index[t]] += (time_index may be NULL with dtime NULL), dcls += and dpos[0] +=
 * the CLS rows (timesformer.py:288-323). */
int dsvt_embed_bwd(const float *dX, int64_t B, int64_t Np, int64_t T, int64_t C, const int32_t *pos_index,
                   const int32_t *time_index, float *dpos, float *dtime, float *dcls, void *workspace,
                   int64_t workspace_bytes, void *stream);
/* Multi-tensor ops over fp32 tensor lists (device arrays of pointers / sizes, work split in
 * 4096-element chunks: chunk i covers tensor chunk_tensor[i] from chunk_start[i]).
 * EMA: teacher = m*teacher + (1-m)*student (train_ssl.py:555-558).  clip: per-tensor L2 norms
 * (norms[ntensors]), grads *= clip/(norm+1e-6) where that is < 1 (utils/utils.py:102-111;
 * clip <= 0: norms only); first_chunk[ntensors+1] = chunk ranges; workspace >= nchunks*4 B. */
/* bf16 copies of a list of fp32 tensors in one launch (the weight cache's refresh after an
 * optimizer / EMA step): dst[i][j] = bf16(src[i][j]); chunk tables as dsvt_ema. */
int dsvt_cast_multi(const float *const *src, void *const *dst, const int64_t *sizes,
                    const int32_t *chunk_tensor, const int64_t *chunk_start, int64_t nchunks, void *stream);
/* bf16 transposed copies W^T [cols, rows] of fp32 matrices [rows, cols] in one launch (the B
 * operands of the backward's dX = dY . W GEMMs): one 64 x 64 tile per entry of
 * (tile_tensor[t], tile_rc[t] = row_tile << 16 | col_tile). */
int dsvt_cast_transpose_multi(const float *const *src, void *const *dst, const int64_t *rows,
                              const int64_t *cols, const int32_t *tile_tensor, const int32_t *tile_rc,
                              int64_t ntiles, void *stream);
int dsvt_ema(float *const *teacher, const float *const *student, const int64_t *sizes,
             const int32_t *chunk_tensor, const int64_t *chunk_start, int64_t nchunks, float momentum,
             void *stream);
int dsvt_clip_grads(float *const *grads, const int64_t *sizes, const int32_t *chunk_tensor,
                    const int64_t *chunk_start, const int32_t *first_chunk, int64_t nchunks,
                    int64_t ntensors, float clip, float *norms, void *workspace, int64_t workspace_bytes,
                    void *stream);
/* Weight (and bias) gradient of an nn.Linear in the backward of loss.backward()
 * (train_ssl.py:538): G[n, k] (+)= sum_m dY[m, n] * X[m, k] over m < M, i.e. dW = dY^T . X
 * with dY [M, N] (ldy) and X [M, K] (ldx) in bf16 and G [N, K] fp32 (row stride K); db
 * (optional, fp32 [N]) (+)= sum_m dY[m, n], the bias gradient, fused; accumulate != 0 adds
 * to G and db.  Deterministic (M slices reduced in a fixed order through the workspace,
 * DSVT_WS_WGRAD).  N, K multiples of 8. */
int dsvt_wgrad_bwd(int dtype, const void *dy, int64_t ldy, const void *x, int64_t ldx, float *G,
                   float *db, int64_t M, int64_t N, int64_t K, int accumulate, void *workspace,
                   int64_t workspace_bytes, void *stream);
/* AdamW step over one tensor list that shares lr / weight decay / step count (replaces
 * torch.optim.AdamW(params_groups).step(), train_ssl.py:384 / :551): per element
 * p *= 1 - lr*wd; m += (1-beta1)(g-m); v = beta2 v + (1-beta2) g^2;
 * p += -lr/(1-beta1^step) * m / (sqrt(v)/sqrt(1-beta2^step) + eps).  step >= 1. */
int dsvt_adamw(float *const *params, const float *const *grads, float *const *exp_avg,
               float *const *exp_avg_sq, const int64_t *sizes, const int32_t *chunk_tensor,
               const int64_t *chunk_start, int64_t nchunks, float lr, float weight_decay, float beta1,
               float beta2, float eps, int64_t step, void *stream);

/* ------------------------------------------------------------------------------------------
 * Video Swin Transformer backbone (models/swin_transformer.py, config 5).  Tokens: fp32
 * X [B, D, H, W, C] channels-last.  Linear layers run on dsvt_gemm_fwd with K zero-padded to
 * the MFMA tile (ldk: C = 96 -> 128 in bf16); window rows are gathered / scattered through
 * int32 index maps that encode the cyclic shift and the padding (-1 = zero row).
 * ------------------------------------------------------------------------------------------ */
/* PatchEmbed3D (:419-460): Conv3d(k = s = (pd, ph, pw)) with zero padding, as im2col + GEMM;
 * w [C, ldk] storage dtype (Conv3d weight flattened, zero-padded); X [B*Do*Ho*Wo, C] fp32. */
int dsvt_swin_patch_embed_fwd(int dtype, const float *x, int64_t B, int64_t Cin, int64_t D, int64_t H,
                              int64_t W, int64_t pd, int64_t ph, int64_t pw, const void *w, int64_t ldk,
                              const float *bias, int64_t C, float *X, void *workspace,
                              int64_t workspace_bytes, void *stream);
/* out[m] = LayerNorm(x[idx[m]]) (idx NULL = identity; idx[m] < 0 = zero row), columns C..ldo-1
 * zero: norm1 + pad + roll + window_partition (:221-237) and norm2 (:254). */
int dsvt_swin_ln_rows_fwd(int dtype, const float *x, const int32_t *idx, const float *gamma,
                          const float *beta, void *out, int64_t rows, int64_t C, int64_t ldo, float eps,
                          void *stream);
/* PatchMerging (:293-315): 2x2 gather (x0, x1, x2, x3 order, zero pad) + LayerNorm(4C). */
int dsvt_swin_merge_ln_fwd(int dtype, const float *x, const float *gamma, const float *beta, void *out,
                           int64_t B, int64_t D, int64_t H, int64_t W, int64_t C, float eps, void *stream);
/* X[idx[m]] += s[m / group] * y[m] (idx[m] >= 0): window_reverse + reverse roll + crop + residual
 * (:241-251); row_scale (nullable = 1): the training DropPath scale of the row's sample (:263, x =
 * shortcut + drop_path(x)), window rows of one sample in runs of `group`.  Also the reverse of any
 * row gather (the PatchMerging 2x2 gather's gradient). */
int dsvt_window_scatter_add(float *X, const float *y, const int32_t *idx, int64_t rows, int64_t C,
                            const float *row_scale, int64_t group, void *stream);
/* attn.proj with the window_reverse + residual add in its epilogue (bf16; swin_transformer.py:170-171
 * then :241-251, :269): X[idx[m]] += A[m] . W^T + bias for m < M -- dsvt_gemm_fwd into an fp32 [M, N]
 * buffer followed by dsvt_window_scatter_add, without the buffer.  Every idx[m] must be >= 0 and
 * distinct (a window map without padding rows; with padding use the two-call form). */
int dsvt_gemm_resid_rows_fwd(const void *A, int64_t lda, const void *W, int64_t ldw, const float *bias, float *X,
                             int64_t ldx, const int32_t *idx, int64_t M, int64_t N, int64_t K, void *stream);
/* ---- Video Swin training (swin_bwd.hip; the --arch swin student, train_ssl.py:237-239) ----------
 * out[m] = dtype(s[m / group] * x[idx[m]]) for c < C, zero for idx[m] < 0 and columns C..ldo-1 (idx
 * NULL = identity, row_scale NULL = 1): window_partition of a token gradient (the window-row gradient
 * of the attention branch), row-scaled / K-padded casts, the PatchMerging 2x2 gather (:300-310). */
int dsvt_swin_gather_rows(int dtype, const float *x, const int32_t *idx, const float *row_scale, int64_t group,
                          void *out, int64_t rows, int64_t C, int64_t ldo, void *stream);
/* WindowAttention3D backward (:139-171): dqkv [nwin*N, 3C] (qkv's layout) from the forward's qkv,
 * its output o [nwin*N, ldo] and dout [nwin*N, lddo] (the gradient of o); P recomputed with the
 * relative-position bias and the shift mask (-100 across regions); dqkv rows ld_dqkv apart (>= 3C:
 * room for the zero K padding the next GEMM needs).  dbias [heads][N][N] fp32 = the
 * gradient of the bias added to the scores, summed over the windows in a fixed order (written, not
 * accumulated).  workspace >= dsvt_workspace_bytes(DSVT_WS_ATTN_WIN_BWD, ., nwin, heads, N). */
int dsvt_attn_window_bwd(int dtype, const void *qkv, const void *o, int64_t ldo, const void *dout, int64_t lddo,
                         const float *bias, const int32_t *region, int64_t nwin, int64_t nwc, int64_t N, int64_t heads,
                         int64_t head_dim, float scale, void *dqkv, int64_t ld_dqkv, float *dbias, void *workspace,
                         int64_t workspace_bytes, void *stream);
/* relative_position_bias_table gradient (:152-156 backward): dtable[e][h] (+)= sum over i, j < N with
 * index[i*nmax + j] == e of dbias[h][i][j]; entries = rows of the table.  Deterministic (no atomics). */
int dsvt_relpos_bias_bwd(const float *dbias, const int64_t *index, int64_t nmax, int64_t N, int64_t heads,
                         int64_t entries, float *dtable, int accumulate, void *stream);
/* out[h][i][j] = table[index[i*nmax + j]][h], i, j < N (:152-156, the [:N, :N] slice). */
int dsvt_relpos_bias_fwd(const float *table, const int64_t *index, int64_t nmax, int64_t N,
                         int64_t heads, float *out, void *stream);
/* WindowAttention3D (:139-171): qkv [nwin*N, 3C] window-ordered, out [nwin*N, ldo]; scores
 * q.k*scale + bias[h] + (-100 where region[w % nwc][i] != region[w % nwc][j]); head_dim 32,
 * N <= 128.  region all-zero = no shift mask. */
int dsvt_attn_window_fwd(int dtype, const void *qkv, void *out, int64_t ldo, const float *bias,
                         const int32_t *region, int64_t nwin, int64_t nwc, int64_t N, int64_t heads,
                         int64_t head_dim, float scale, void *stream);
/* The bf16 form with the bias in MFMA-fragment order: frag (dsvt_attn_window_bias_frag_floats(N,
 * heads) floats, 16-byte aligned) = dsvt_attn_window_bias_frag(bias [heads][N][N]), built once per
 * bias table; out columns heads*32..ldo-1 are zeroed.  Bitwise the same out as dsvt_attn_window_fwd. */
int64_t dsvt_attn_window_bias_frag_floats(int64_t N, int64_t heads);
int dsvt_attn_window_bias_frag(const float *bias, int64_t N, int64_t heads, float *frag, void *stream);
int dsvt_attn_window_frag_fwd(const void *qkv, void *out, int64_t ldo, const float *frag, const int32_t *region,
                              int64_t nwin, int64_t nwc, int64_t N, int64_t heads, float scale, void *stream);
/* y [N, ldk] = x [N, K] cast to the storage dtype with zero columns K..ldk-1. */
int dsvt_cast_pad_fwd(int dtype, const float *x, void *y, int64_t N, int64_t K, int64_t ldk, void *stream);

/* Score -> frame-index selection, the "adaptive" method of
 * datasets_custom/frame_selection_loader.py:115-166 (replaces that inline numpy loop), bit-exact
 * in float64: pdf = loss / np.sum(loss) (numpy pairwise summation), cdf = np.cumsum(pdf),
 * idx_i = argmin |cdf - i/N| (first minimum), then the reference's collision walk over multiples
 * of `rate` (pre_sampling_rate) below n_unsampled (frames_unsampled.size(0)).
 * loss [n_loss] float64 device; only the first min(n_loss, n_frames) values are used (the
 * reference truncates to frames.size(0) = n_frames).  Outputs (device): indices [N] int64 (the
 * reference's `indices` list, in unsampled-video frame numbers) and frame_pos [N] int32 (which
 * pre-sampled frame the reference stacks for slot i: idx_i, or n_frames - 1 for frames[-1]);
 * cdf_out [n] float64 optional (NULL: kept in the workspace).
 * workspace >= dsvt_workspace_bytes(DSVT_WS_SELECT, ., n, n_unsampled, 0), n = min(n_loss,
 * n_frames).  Errors: a size < 1, N > 65535, or (n - 1) * rate >= n_unsampled (the pre-sampled
 * frames are frames_unsampled[::rate], so every score indexes the unsampled video). */
int dsvt_select_frames(const double *loss, int64_t n_loss, int64_t n_frames, int64_t n_unsampled, int64_t rate,
                       int64_t N, int64_t *indices, int32_t *frame_pos, double *cdf_out, void *workspace,
                       size_t workspace_bytes, void *stream);
/* Video DINO augmentation of one crop, VideoDataAugmentationDINO (datasets_custom/transform.py:
 * 661-749): replaces random_resized_crop (:134-173, bicubic F.interpolate), horizontal_flip
 * (:176-203), color_jitter (:371-461: brightness / contrast / saturation in the drawn order),
 * grayscale (:349-368) and color_normalization (:494-516) applied to one clip.  The random draws
 * stay on the host (dsvt/augment.py makes the reference's own RNG calls); the parameters below
 * are their results. */
#define DSVT_AUG_BRIGHTNESS 1
#define DSVT_AUG_CONTRAST 2
#define DSVT_AUG_SATURATION 3
typedef struct dsvt_aug_params {
  int32_t y0, x0, h, w; /* crop window of the input frame, already clipped to it (the reference slices) */
  int32_t size;         /* output S x S (bicubic, align_corners=False) */
  int32_t flip;         /* horizontal flip of the resized crop */
  int32_t n_ops;        /* colour-jitter ops applied, in order (0 = jitter not drawn) */
  int32_t op[3];        /* DSVT_AUG_* */
  float alpha[3];       /* blend weight as the float tensor op sees it: (float)alpha */
  float beta[3];        /* (float)(1 - alpha) */
  int32_t gray;         /* grayscale after the jitter */
  float mean[3], std[3];
} dsvt_aug_params;
/* frames: T_in frames, 3 channels, H x W, uint8 (frames_u8 = 1, scaled by 1/255 as
 * `x.float() / 255.0`) or fp32, addressed by element strides (sT, sC, sH, sW) -- the decoder's
 * [T, H, W, C] and the reference's [T, C, H, W] both work.  frame_index [T] int32 device
 * (nullable = identity; values clamped to [0, T_in)) picks the input frame of each output frame
 * (the loader's temporal index_select, which commutes with the per-frame augmentation).
 * out fp32: out_layout 0 = [T, 3, S, S] (the reference crop), 1 = [3, T, S, S] (the model input
 * after the loader's `t c h w -> c t h w`).  workspace >= dsvt_workspace_bytes(DSVT_WS_AUGMENT,
 * ., T, S, 0) (the per-frame contrast-mean partial sums). */
int dsvt_video_augment(const void *frames, int frames_u8, int64_t T_in, int64_t T, const int32_t *frame_index,
                       int64_t H, int64_t W, int64_t sT, int64_t sC, int64_t sH, int64_t sW,
                       const dsvt_aug_params *params, float *out, int out_layout, void *workspace,
                       size_t workspace_bytes, void *stream);

/* dst[r] = src[idx[r]], rows of row_bytes bytes (the `torch.stack(selected_frames)` of
 * frame_selection_loader.py:166 / any frame gather); rows <= 65535. */
int dsvt_gather_rows(const void *src, int64_t row_bytes, const int32_t *idx, int64_t rows, void *dst, void *stream);

/* Kernel-choice overrides for tools and tests: include/dsvt_debug.h (not part of this interface). */

/* Measurement probe: when enabled, every launch of a family in `mask` is bracketed by a
 * pair of hipEvents on its own stream (diagnostic; not thread-safe). */
int dsvt_probe_enable(int mask, int capacity);
int dsvt_probe_disable(void);
/* Synchronizes the recorded events; fills per-launch ms, algorithmic work (FLOP for
 * GEMM/attention, bytes for norm/loss), algorithmic HBM bytes of GEMM launches (operands and
 * output once; 0 where not recorded), family and tag (GEMM: kernel instantiation id =
 * variant*32 + dtype*16 + epilogue*2 + fp32_out; variant 0 = fp32 128x128, 1 = bf16 128x128,
 * 10 = bf16 persistent 256x128; epilogue 3 = patch embed).  Any output pointer may be NULL.
 * Returns the number of launches (negative on error). */
int dsvt_probe_read(float *ms, double *work, double *bytes, int32_t *family, int32_t *tag, int capacity);

#ifdef __cplusplus
}
#endif
#endif /* DSVT_H */
