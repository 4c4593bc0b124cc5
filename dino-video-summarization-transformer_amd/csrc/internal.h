// Internal launcher interface between the C-ABI layer (capi.hip) and the kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

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
};

enum { EPI_BIAS = 0, EPI_GELU = 1, EPI_RESID = 2, EPI_PATCH = 3 };

hipError_t launch_gemm(const GemmParams& p, int dtype, int epi, int out_f32, hipStream_t s);
int gemm_variant_for(const GemmParams& p, int dtype, int epi, int out_f32);  // the kernel launch_gemm dispatches
hipError_t launch_gemm_big(const GemmParams& p, int variant, int epi, int out_f32, hipStream_t s);
void set_gemm_variant(int v);

hipError_t launch_layernorm(int dtype, int out_f32, const float* x, void* y, const float* g,
                            const float* b, int64_t rows, int64_t C, int64_t rpg, int64_t gstride,
                            int64_t goff, float eps, hipStream_t s);
hipError_t launch_im2col(int dtype, int order_nt, const float* x, void* a, int64_t B, int64_t Cin,
                         int64_t T, int64_t H, int64_t W, int64_t Hp, int64_t Wp, const int32_t* fidx,
                         hipStream_t s);
hipError_t launch_pos_bicubic(const float* pos, float* out, int64_t sgrid, int64_t OH, int64_t OW, int64_t C,
                              float inv_scale_h, float inv_scale_w, hipStream_t s);
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
};
hipError_t launch_attn_seq(int dtype, const AttnParams& p, hipStream_t s);
void set_attn_variant(int v);
hipError_t launch_attn_temporal(int dtype, const void* qkv, void* out, int64_t nseq, int64_t T,
                                int64_t heads, int64_t C, float scale, hipStream_t s);

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
