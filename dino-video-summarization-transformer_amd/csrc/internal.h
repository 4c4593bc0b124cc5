// Internal launcher interface between the C-ABI layer (capi.hip) and the kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/dsvt.h"

namespace dsvt {

struct GemmParams {
  const void* A; int64_t lda;
  const void* W; int64_t ldw;
  const float* bias;
  void* out; int64_t ldo;
  int64_t M, N, K;
  int64_t rpg, gstride, goff;  // output row map
  // patch-embed epilogue (X = acc + bias + pos[1 + pidx[n]] + temb[tidx[t]])
  const float* pos; const int32_t* pidx; const float* temb; const int32_t* tidx;
  int64_t T;  // frames per patch group (1 for the frame-major order)
  // backward / training epilogues: second operand in the storage dtype, row-major, ld_aux
  void* aux; int64_t ld_aux;
  // persistent 256x256 kernel: tile order, GM m-tile rows per group walked n-column-major (0 = row-major)
  int tile_group;
  // EPI_RESID: the residual read (same row map and ldo as out); nullptr = out itself (in place)
  const float* resid = nullptr;
  // EPI_BIAS / EPI_GELU_SAVE: output row m scaled by row_scale[m / rs_group] after the bias /
  // GELU (DropPath's per-sample scale, models/vit_utils.py:152-167); the saved pre-activation
  // is not scaled.  Only the 128x128 and persistent kernels take it (gemm_variant_for).
  const float* row_scale = nullptr;
  int64_t rs_group = 1;
  // K-split skinny kernel for this call (DSVT_GEMM_FEW_ROWS: the few-row GEMMs of the CLS-only
  // tail and the DINO head, chosen by call site)
  bool few_rows = false;
  // LayerNorm folded into the GEMM (dsvt_gemm_lnx_fwd, 256x256 kernel): A = the bf16 copy of the
  // fp32 token rows, read through the A row map a_row(m) = (m / a_rpg) * a_gstride + a_goff +
  // m % a_rpg; W = W * gamma (bf16); the epilogue forms
  //   out = rstd(r) * (acc - mu(r) * ln_wsum[n]) + bias[n]      (bias = b + W . beta)
  // with mu / rstd of A row r from ln_stats[r][LN_PARTS] (float2 partial sums of x and x^2 over
  // 64-column slabs, written by the residual epilogue that produced the row) and ln_eps.
  const float* ln_stats = nullptr;
  const float* ln_wsum = nullptr;
  float ln_eps = 0.f, ln_invk = 0.f;   // ln_invk = 1 / K
  int64_t a_rpg = INT64_MAX, a_gstride = 0, a_goff = 0;
  // residual epilogue that also writes the next LayerNorm's inputs (dsvt_gemm_resid_stats_fwd):
  // the bf16 copy of every updated X row (xb_out, row stride ldo) and its LN_PARTS partials
  // (stats_out, rows of the output row map)
  void* xb_out = nullptr;
  float* stats_out = nullptr;
  // temporal attention epilogue (launch_gemm_tattn): softmax scale
  float attn_scale = 0.f;
  // EPI_RESID output rows through an index instead of the affine map: row(m) = row_idx[m] (every
  // entry >= 0, no two equal; dsvt_gemm_resid_rows_fwd: Video Swin's window_reverse + residual add).
  // The persistent kernels only (variants 10-15).
  const int32_t* row_idx = nullptr;
};

// float2 (sum, sum of squares) partials per token row: one per 64-column slab of C = 768
constexpr int LN_PARTS = 12;

// the DropPath scale of GEMM row m (1 when none)
__device__ __forceinline__ float row_scale_of(const GemmParams& p, int64_t m) {
  if (!p.row_scale || m >= p.M) return 1.0f;
  return p.row_scale[(uint32_t)m / (uint32_t)p.rs_group];
}

// EPI_RESID residual source: out-of-place (training keeps the pre-sublayer X as its saved
// activation) or the output rows themselves
__host__ __device__ inline const float* resid_src(const GemmParams& p) {
  return p.resid ? p.resid : (const float*)p.out;
}

// EPI_GELU_SAVE: out = GELU(acc + bias), aux = GELU'(acc + bias) (what the backward multiplies by)
// EPI_DGELU:     out = acc * aux          (Mlp.fc1 backward through nn.GELU, bias ignored)
enum { EPI_BIAS = 0, EPI_GELU = 1, EPI_RESID = 2, EPI_PATCH = 3, EPI_GELU_SAVE = 4, EPI_DGELU = 5 };

hipError_t launch_gemm(const GemmParams& p, int dtype, int epi, int out_f32, hipStream_t s);
int gemm_variant_for(const GemmParams& p, int dtype, int epi, int out_f32);  // the kernel launch_gemm dispatches
hipError_t launch_gemm_big(const GemmParams& p, int variant, int epi, int out_f32, hipStream_t s);
hipError_t launch_gemm_8ph(const GemmParams& p, int epi, int out_f32, hipStream_t s, int abl = 0);  // variant 20
bool gemm_8ph_ok(const GemmParams& p, int epi);
hipError_t launch_gemm_4w(const GemmParams& p, int epi, int out_f32, hipStream_t s, int abl = 0);   // variant 40
bool gemm_4w_ok(const GemmParams& p, int epi, int out_f32);
hipError_t launch_gemm_192(const GemmParams& p, int epi, int out_f32, hipStream_t s);    // variant 30
bool gemm_192_ok(const GemmParams& p, int epi);
// the LayerNorm-folded temporal qkv GEMM with the T = 8 attention in its epilogue (gemm_192.hip)
bool gemm_tattn_ok(const GemmParams& p);
hipError_t launch_gemm_tattn(const GemmParams& p, hipStream_t s);
// K split over the 8 waves of a workgroup, 64-row blocks (variant 50, gemm_big.hip)
bool gemm_skinny_ok(const GemmParams& p, int epi);
hipError_t launch_gemm_skinny(const GemmParams& p, int epi, int out_f32, hipStream_t s);
void set_gemm_variant(int v);

// multi-tensor bf16 weight copies (backward.hip)
hipError_t launch_cast_multi(const float* const* src, void* const* dst, const int64_t* sizes, const int32_t* ctensor,
                             const int64_t* cstart, int64_t nchunks, hipStream_t s);
hipError_t launch_cast_transpose_multi(const float* const* src, void* const* dst, const int64_t* rows,
                                       const int64_t* cols, const int32_t* tile_tensor, const int32_t* tile_rc,
                                       int64_t ntiles, hipStream_t s);

// Weight gradients (wgrad.hip): G[n, k] (+)= sum_m dY[m, n] X[m, k] and optionally
// db[n] (+)= sum_m dY[m, n], bf16 in, fp32 out
int64_t wgrad_slices(int64_t M, int64_t N, int64_t K);
int64_t wgrad_workspace_floats(int64_t M, int64_t N, int64_t K);
hipError_t launch_wgrad(const unsigned short* dy, int64_t ldy, const unsigned short* x, int64_t ldx, float* G,
                        float* db, int64_t M, int64_t N, int64_t K, int accumulate, float* partial, hipStream_t s);

// bf16 copy + LN_PARTS row-statistics partials of fp32 rows [rows, 768] (dsvt_ln_stats_fwd)
hipError_t launch_ln_stats(const float* x, void* xb, float* stats, int64_t rows, hipStream_t s);
// LayerNorm-folded GEMM weights: Wf = bf16(W * gamma), wsum = row sums of Wf, bf = b + W . beta
hipError_t launch_ln_fold(const float* W, const float* gamma, const float* beta, const float* b, void* Wf, float* wsum,
                          float* bf, int64_t N, int64_t K, hipStream_t s, int heads = 0);
hipError_t launch_layernorm(int dtype, int out_f32, const float* x, void* y, const float* g,
                            const float* b, int64_t rows, int64_t C, int64_t rpg, int64_t gstride,
                            int64_t goff, float eps, hipStream_t s);
hipError_t launch_im2col(int dtype, int order_nt, const float* x, void* a, int64_t B, int64_t Cin,
                         int64_t T, int64_t H, int64_t W, int64_t Hp, int64_t Wp, const int32_t* fidx,
                         hipStream_t s);
hipError_t launch_pos_bicubic(const float* pos, float* out, int64_t sgrid, int64_t OH, int64_t OW, int64_t C,
                              float inv_scale_h, float inv_scale_w, hipStream_t s);
hipError_t launch_pos_bicubic_bwd(const float* dout, float* dpos, int64_t sgrid, int64_t OH, int64_t OW, int64_t C,
                                  float inv_h, float inv_w, int accumulate, hipStream_t s);
hipError_t launch_cls_init(float* X, const float* cls, const float* pos0, int64_t rows,
                           int64_t row_stride_elems, int64_t C, hipStream_t s);
hipError_t launch_cls_mean(int dtype, const float* aux, void* out, int64_t B, int64_t T, int64_t L,
                           int64_t C, hipStream_t s);
hipError_t launch_frame_mean(const float* x, float* y, int64_t B, int64_t T, int64_t rowlen,
                             hipStream_t s);
hipError_t launch_cast(int dtype, const float* x, void* y, int64_t n, hipStream_t s);
hipError_t launch_l2norm(int dtype, const float* x, void* y, int64_t rows, int64_t D, float eps,
                         hipStream_t s);
hipError_t launch_weight_norm(int dtype, const float* v, const float* g, void* w, int64_t rows,
                              int64_t D, hipStream_t s);

// Attention.  Token row of position i in sequence (b, t):
//   b*L + (i == 0 ? 0 : 1 + (i-1)*tok_stride + t)
struct AttnParams {
  const void* qkv; int64_t ld_qkv;
  void* out; int64_t ld_out;
  float* cls_aux;          // when non-null, position 0's output goes to cls_aux[(b*tin+t)*C + ...]
  int64_t nb, tin, L, tok_stride, seqlen, heads, C;
  float scale;
  float* probs;            // optional: softmax probabilities [nb*tin][heads][seqlen][seqlen] (get_attn)
  const float* seq_scale;  // optional: per-sequence output scale (training DropPath over (b, t), timesformer.py:159)
};
hipError_t launch_attn_seq(int dtype, const AttnParams& p, hipStream_t s);
// flash attention over contiguous sequences (attn_flash.hip): joint space-time / space-only
bool attn_flash_ok(int dtype, const AttnParams& p);
hipError_t launch_attn_flash(const AttnParams& p, hipStream_t s, int cfg = 0);   // cfg: workgroup shape 1-5, 0 = auto
void set_attn_variant(int v);
// CLS query only of every spatial sequence, mean over frames -> out[b * ld_out + c] (attention.hip)
int64_t attn_cls_ws_bytes(int64_t nseq, int64_t heads, int64_t seqlen);   // nseq = B*T
hipError_t launch_attn_cls(int dtype, const void* qkv, void* out, int64_t ld_out, int64_t B, int64_t T, int64_t L,
                           int64_t heads, float scale, float* ws, hipStream_t s, const float* seq_scale = nullptr);
// its backward (training CLS-only last block): dqkv [B*L, 3C] from do_cls [B, C]; ws [B*T, 3C] fp32
int64_t attn_cls_bwd_ws_bytes(int64_t nseq, int64_t heads);
hipError_t launch_attn_cls_bwd(int dtype, const void* qkv, const void* dout, void* dqkv, float* ws,
                               const float* seq_scale, int64_t B, int64_t T, int64_t L, int64_t heads, float scale,
                               hipStream_t s);
hipError_t launch_attn_temporal(int dtype, const void* qkv, void* out, int64_t nseq, int64_t T,
                                int64_t heads, int64_t C, float scale, hipStream_t s);

// Backward (backward.hip).  Attention backward: sequence layout as AttnParams; the
// dO of position 0 is scaled by cls_scale and its dq/dk/dv go to cls_aux [nb*tin, 3C] fp32
// (then summed over t into the CLS row) when cls_aux is non-null; stats = [nb*tin*heads*seqlen][2].
struct AttnBwdParams {
  const void* qkv; int64_t ld_qkv;
  const void* dout; int64_t ld_dout;
  void* dqkv; int64_t ld_dqkv;
  float* cls_aux;
  float* stats;
  int64_t nb, tin, L, tok_stride, seqlen, heads, C;
  float scale, cls_scale;
  const float* seq_scale;  // optional: dO of sequence seq scaled (the forward's DropPath scale)
};
int ln_bwd_blocks(int64_t rows);
int64_t colsum_parts(int64_t rows);
hipError_t launch_ln_bwd(int dy_dtype, const float* x, const void* dy, const float* gamma, float* dx, int64_t rows,
                         int64_t C, int64_t rpg, int64_t gstride, int64_t goff, float eps, float* partial,
                         hipStream_t s);
hipError_t launch_reduce_partials(const float* partial, int64_t nparts, int64_t width, int64_t stride, float* out,
                                  int accumulate, hipStream_t s);
// the LayerNorm backward's partial rows [nparts][dgamma C | dbeta C] -> dgamma, dbeta in one pass (per column the
// order of launch_reduce_partials)
hipError_t launch_ln_params_reduce(const float* partial, int64_t nparts, int64_t C, float* dgamma, float* dbeta,
                                   int accumulate, hipStream_t s);
hipError_t launch_ln_bwd_cast(int dy_dtype, const float* x, const void* dy, const float* gamma, float* dx,
                              int64_t rows, int64_t rpg, int64_t gstride, int64_t goff, float eps, float* partial,
                              void* dxb, int64_t og, int64_t osk, hipStream_t s);
hipError_t launch_colsum_rows(int dtype, const void* y, int64_t rows, int64_t C, int64_t ld, int64_t rpg,
                              int64_t gstride, int64_t goff, const float* row_scale, float* partial, float* out,
                              int accumulate, hipStream_t s);
hipError_t launch_attn_temporal_bwd(int dtype, const void* qkv, const void* dout, void* dqkv, int64_t nseq, int64_t T,
                                    int64_t heads, int64_t C, float scale, hipStream_t s);
hipError_t launch_attn_bwd_generic(int dtype, const AttnBwdParams& p, hipStream_t s);
void set_attn_bwd_variant(int v);
hipError_t launch_dino_loss_bwd(const float* student, const float* teacher, const float* center, int64_t B,
                                int64_t ncrops, int64_t gc, int64_t D, float inv_ts, float inv_tt, const float* t_m,
                                const float* t_z, const float* s_m, const float* s_z, const float* dloss, float coef,
                                float* grad, hipStream_t s);
hipError_t launch_l2norm_bwd(const float* x, const float* dz, float* dx, int64_t rows, int64_t D, float eps,
                             hipStream_t s);
hipError_t launch_weightnorm_bwd(const float* v, const float* g, const float* dw, float* dv, float* dg, int64_t rows,
                                 int64_t D, int accumulate, hipStream_t s);
hipError_t launch_cast_rows(int dtype, const float* x, void* y, int64_t rows, int64_t C, int64_t rpg, int64_t gstride,
                            int64_t goff, const float* row_scale, int64_t group, hipStream_t s);
hipError_t launch_row_scale(int dtype, void* y, int64_t rows, int64_t C, int64_t ld, const float* row_scale,
                            int64_t group, hipStream_t s);
hipError_t launch_rowscale_bias_add(float* X, int64_t rows, int64_t C, const float* row_scale, const float* bias,
                                    hipStream_t s);
hipError_t launch_cast_transpose(int dtype, const float* x, void* y, int64_t R, int64_t C, hipStream_t s);
hipError_t launch_embed_grads(const float* dX, int64_t B, int64_t Np, int64_t T, int64_t C, float* gn, float* gt,
                              float* gcls, float* S, hipStream_t s);
hipError_t launch_index_accum(const float* src, const int32_t* dst, int64_t n, int64_t C, int64_t dst_off, float* out,
                              hipStream_t s);
hipError_t launch_ema(float* const* teacher, const float* const* student, const int64_t* sizes, const int32_t* ctensor,
                      const int64_t* cstart, int64_t nchunks, float m, hipStream_t s);
hipError_t launch_clip_grads(float* const* grads, const int64_t* sizes, const int32_t* ctensor, const int64_t* cstart,
                             const int32_t* first_chunk, int64_t nchunks, int64_t ntensors, float clip, float* partial,
                             float* norms, hipStream_t s);
struct AdamWArgs {
  float lr, wd, beta1, beta2, eps, bc2_sqrt, step_size;
};
hipError_t launch_adamw(float* const* param, const float* const* grad, float* const* exp_avg, float* const* exp_avg_sq,
                        const int64_t* sizes, const int32_t* ctensor, const int64_t* cstart, int64_t nchunks,
                        const AdamWArgs& a, hipStream_t s);

// Video Swin (swin.hip)
hipError_t launch_im2col3d(int dtype, const float* x, void* a, int64_t B, int64_t Cin, int64_t D, int64_t H,
                           int64_t W, int pd, int ph, int pw, int64_t ldk, hipStream_t s);
hipError_t launch_swin_ln_rows(int dtype, const float* x, const int32_t* idx, const float* gamma, const float* beta,
                               void* out, int64_t rows, int64_t C, int64_t ldo, float eps, hipStream_t s);
hipError_t launch_swin_merge_ln(int dtype, const float* x, const float* gamma, const float* beta, void* out, int64_t B,
                                int64_t D, int64_t H, int64_t W, int64_t C, float eps, hipStream_t s);
hipError_t launch_window_scatter_add(float* X, const float* y, const int32_t* idx, int64_t rows, int64_t C,
                                     const float* row_scale, int64_t group, hipStream_t s);
// Video Swin training (swin_bwd.hip)
int64_t attn_window_bwd_groups(int64_t nwin, int64_t heads);
hipError_t launch_swin_gather_rows(int dtype, const float* x, const int32_t* idx, const float* row_scale,
                                   int64_t group, void* out, int64_t rows, int64_t C, int64_t ldo, hipStream_t s);
hipError_t launch_attn_window_bwd(int dtype, const void* qkv, const void* o, int64_t ldo, const void* dout,
                                  int64_t lddo, const float* bias, const int32_t* region, int64_t nwin, int64_t nwc,
                                  int64_t N, int64_t heads, int64_t C, float scale, void* dqkv, int64_t lddq,
                                  float* dbias, float* workspace, hipStream_t s);
hipError_t launch_relpos_bias_bwd(const float* dbias, const int64_t* index, int64_t nmax, int64_t N, int64_t heads,
                                  int64_t entries, float* dtable, int accumulate, hipStream_t s);
hipError_t launch_relpos_bias(const float* table, const int64_t* index, int64_t nmax, int64_t N, int64_t heads,
                              float* out, hipStream_t s);
hipError_t launch_attn_window(int dtype, const void* qkv, void* out, int64_t ldo, const float* bias,
                              const int32_t* region, int64_t nwin, int64_t nwc, int64_t N, int64_t heads, int64_t C,
                              float scale, hipStream_t s);
hipError_t launch_cast_pad(int dtype, const float* x, void* y, int64_t N, int64_t K, int64_t ldk, hipStream_t s);
// bf16 window attention with the bias in MFMA-fragment order (attn_window_bias_frag: [heads][ceil(N/16)][8][64]
// float4) and the out columns C..ldo-1 zeroed
int64_t attn_window_frag_floats(int64_t N, int64_t heads);
hipError_t launch_attn_window_bias_frag(const float* bias, int64_t N, int64_t heads, float* frag, hipStream_t s);
hipError_t launch_attn_window_frag(const void* qkv, void* out, int64_t ldo, const float* frag, const int32_t* region,
                                   int64_t nwin, int64_t nwc, int64_t N, int64_t heads, int64_t C, float scale,
                                   hipStream_t s);

// frame selection (select.hip)
int64_t select_frames_ws_bytes(int64_t n, int64_t n_unsampled);
hipError_t launch_select_frames(const double* loss, int64_t n, int64_t n_frames, int64_t n_unsampled, int64_t rate,
                                int64_t N, int64_t* indices, int32_t* frame_pos, double* cdf_out, void* ws,
                                hipStream_t s);
hipError_t launch_gather_rows(const void* src, int64_t row_bytes, const int32_t* idx, int64_t rows, void* dst,
                              hipStream_t s);

// video augmentation (augment.hip)
int64_t augment_ws_bytes(int64_t T, int64_t size);
hipError_t launch_video_augment(const void* frames, int u8, int64_t T_in, int64_t T, const int32_t* fidx, int64_t H,
                                int64_t W, int64_t sT, int64_t sC, int64_t sH, int64_t sW, const ::dsvt_aug_params& p,
                                float* out, int layout, void* ws, hipStream_t s);

// BatchNorm1d + GELU of DINOHead(use_bn=True) (head_bn.hip); sums are fp64 [2D]
hipError_t launch_bn_colsum2(const float* x, int64_t R, int64_t D, double* sums, hipStream_t s);
hipError_t launch_bn_finalize(const double* sums, double count, int64_t D, float eps, float momentum, int training,
                              float* run_mean, float* run_var, float* mean, float* rstd, hipStream_t s);
hipError_t launch_bn_gelu(int dtype, const float* x, const float* mean, const float* rstd, const float* gamma,
                          const float* beta, void* y, void* gelu_grad, float* xhat, int64_t R, int64_t D, hipStream_t s);
hipError_t launch_bn_bwd_sums(int dtype, const void* dz, const float* xhat, int64_t R, int64_t D, double* sums,
                              hipStream_t s);
hipError_t launch_bn_bwd_dx(int dtype, const void* dz, const float* xhat, const double* sums,
                            const double* param_sums, double count,
                            const float* gamma, const float* rstd, float* dx, float* dgamma, float* dbeta,
                            int accumulate, int64_t R, int64_t D, hipStream_t s);

hipError_t launch_softmax_stats(const float* x, const float* center, float inv_temp, int64_t rows,
                                int64_t D, float* m_out, float* z_out, hipStream_t s);
hipError_t launch_pair_ce(const float* student, const float* teacher, const float* center,
                          const int32_t* pair_rows /*unused if null*/, int64_t npairs,
                          int64_t B, int64_t ncrops, int64_t global_crops, int64_t D,
                          float inv_ts, float inv_tt, const float* t_m, const float* t_z,
                          const float* s_m, const float* s_z, float* ce, hipStream_t s);
hipError_t launch_loss_reduce(const float* ce, int64_t npairs, float scale, float* out,
                              hipStream_t s);
hipError_t launch_colsum(const float* x, int64_t rows, int64_t D, float* out, hipStream_t s);
hipError_t launch_center_ema(float* center, const float* colsum, int64_t D, float momentum,
                             float inv_count, hipStream_t s);

}  // namespace dsvt
