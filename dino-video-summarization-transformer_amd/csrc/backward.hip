// Backward kernels of the DINO-SVT student: what autograd
// runs for loss.backward() at train_ssl.py:538/545 through the divided block
// (models/timesformer.py:116-185), the DINO head (vision_transformer.py:278-282) and the
// DINO loss (train_ssl.py:653-669).  The weight-gradient GEMMs (dW = dY^T . X) are plain
// library GEMMs (hipBLASLt via torch); everything else of the backward is here or in the
// dsvt GEMM with its backward epilogues (gemm.hip / gemm_big.hip: DGELU).
//
//   ln_bwd_kernel          LayerNorm input gradient, ADDED into the fp32 residual gradient dX
//                          through a row map (the residual branch of every pre-LN sub-layer),
//                          plus per-block dgamma / dbeta partial sums (deterministic: no atomics)
//   colsum_partial_kernel  bias gradients (column sums) through a row map, per-block partials
//   reduce_partials_kernel fixed-order sum of the partials (optionally accumulated into .grad)
//   attn_temporal_bwd      per (patch, head) sequence of T frames, LDS-resident, VALU
//   attn_rows_bwd /        generic (spatial-with-CLS / joint) attention backward, two passes:
//   attn_cols_bwd            per query (lse, D = sum P dP, dQ), then per key (dK, dV); VALU,
//                            K/V/Q/dO read through L2 -- parity mode and the fallback
//   cls_sum_kernel         the CLS row is shared by the T frame sequences: its dq/dk/dv are the
//                          sum over frames (timesformer.py:140-146 repeat -> gradient sum)
//   dino_loss_bwd_kernel   d loss / d student logits
//   l2norm_bwd / weightnorm_bwd   F.normalize and the weight-normed last layer
//   cast_rows / cast_transpose    layout helpers (row-mapped gather-cast, W^T in storage dtype)
//   embed_grad kernels     dpos / dtime / dcls sums of the token gradient
//   ema / sumsq / scale    multi-tensor teacher EMA (train_ssl.py:555-558) and per-tensor
//                          gradient norm clipping (utils/utils.py:102-111)
#include <math.h>
#include <stdlib.h>

#include "common.h"

namespace dsvt {

// ================================================================ LayerNorm backward
// x: fp32 rows through the row map (the saved residual stream), dy: compact rows [rows, C]
// (storage dtype or fp32), dx: fp32 with x's layout (the residual gradient) -- dx[row] += dLN.
// One wave per row (grid-stride).  VEC (C % 256 == 0): lane owns columns i*256 + 4*lane + e
// (16-B x / dx accesses); else columns i*64 + lane.  dgamma / dbeta are accumulated in
// registers, reduced over the 4 waves in LDS and written per block.
template <typename DyT, bool VEC, int NI = 4, bool FAST = false>
__global__ __launch_bounds__(256) void ln_bwd_kernel(const float* __restrict__ x, const DyT* __restrict__ dy,
                                                     const float* __restrict__ gamma, float* __restrict__ dx,
                                                     int64_t rows, int C, int64_t rpg, int64_t gstride, int64_t goff,
                                                     float eps, float* __restrict__ partial) {
  __shared__ float red[4][2][1024];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int n = VEC ? 4 * NI : (C >> 6);                        // slots in use (<= 16; VEC: C = 256 NI)
  auto col = [&](int k) { return VEC ? (k >> 2) * 256 + lane * 4 + (k & 3) : k * 64 + lane; };
  float dg[16], db[16], g[16];
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    dg[k] = 0.f; db[k] = 0.f;
    g[k] = k < n ? gamma[col(k)] : 0.f;
  }
  if constexpr (VEC) {
    // one row per wave per iteration, software-pipelined: the next row's x, dy AND the dx it
    // read-modify-writes are loaded before this row's reductions (one HBM round trip per row
    // in flight behind the compute instead of two in series)
    const int64_t stride = (int64_t)gridDim.x * 4;
    constexpr int NK = 4 * NI;
    float cx[NK], cd[NK], co[NK], nx[NK], nd[NK], no[NK];
    auto load_row = [&](int64_t r, float (&vx)[NK], float (&vd)[NK], float (&vo)[NK]) {
      const int64_t xr = map_row(r, rpg, gstride, goff) * C;
#pragma unroll
      for (int i = 0; i < NI; ++i) {
          load4(x + xr + i * 256 + lane * 4, vx + 4 * i);
          load4(dy + r * C + i * 256 + lane * 4, vd + 4 * i);
          load4(dx + xr + i * 256 + lane * 4, vo + 4 * i);
        }
    };
    int64_t r = (int64_t)blockIdx.x * 4 + wave;
    if (r < rows) load_row(r, cx, cd, co);
    for (; r < rows; r += stride) {
      if (r + stride < rows) load_row(r + stride, nx, nd, no);
      const int64_t xr = map_row(r, rpg, gstride, goff) * C;
      float s = 0.f;
#pragma unroll
      for (int k = 0; k < NK; ++k)
        s += cx[k];
      const float inv_c = 1.0f / (float)C;
      const float mean = FAST ? wave_sum_dpp(s) * inv_c : wave_sum(s) / C;
      float q = 0.f;
#pragma unroll
      for (int k = 0; k < NK; ++k)
        { cx[k] -= mean; q += cx[k] * cx[k]; }
      const float rstd = FAST ? __builtin_amdgcn_rsqf(wave_sum_dpp(q) * inv_c + eps) : 1.0f / sqrtf(wave_sum(q) / C + eps);
      float s1 = 0.f, s2 = 0.f;
#pragma unroll
      for (int k = 0; k < NK; ++k)
        {
          const float xh = cx[k] * rstd, gd = g[k] * cd[k];
          cx[k] = xh;
          s1 += gd;
          s2 += gd * xh;
          dg[k] += cd[k] * xh;
          db[k] += cd[k];
        }
      if (FAST) {
        s1 = wave_sum_dpp(s1) * inv_c;
        s2 = wave_sum_dpp(s2) * inv_c;
      } else {
        s1 = wave_sum(s1) / C;
        s2 = wave_sum(s2) / C;
      }
#pragma unroll
      for (int i = 0; i < NI; ++i) {
          float4 o;
          o.x = co[4 * i] + rstd * (g[4 * i] * cd[4 * i] - s1 - cx[4 * i] * s2);
          o.y = co[4 * i + 1] + rstd * (g[4 * i + 1] * cd[4 * i + 1] - s1 - cx[4 * i + 1] * s2);
          o.z = co[4 * i + 2] + rstd * (g[4 * i + 2] * cd[4 * i + 2] - s1 - cx[4 * i + 2] * s2);
          o.w = co[4 * i + 3] + rstd * (g[4 * i + 3] * cd[4 * i + 3] - s1 - cx[4 * i + 3] * s2);
          *reinterpret_cast<float4*>(dx + xr + i * 256 + lane * 4) = o;
        }
#pragma unroll
      for (int k = 0; k < NK; ++k) { cx[k] = nx[k]; cd[k] = nd[k]; co[k] = no[k]; }
    }
  } else {
  for (int64_t r = (int64_t)blockIdx.x * 4 + wave; r < rows; r += (int64_t)gridDim.x * 4) {
      const int64_t xr = map_row(r, rpg, gstride, goff) * C;
      float v[16], d[16];
      float s = 0.f;
      if constexpr (VEC) {
#pragma unroll
        for (int i = 0; i < 4; ++i)
          if (4 * i < n) {
            load4(x + xr + i * 256 + lane * 4, v + 4 * i);
            load4(dy + r * C + i * 256 + lane * 4, d + 4 * i);
            s += (v[4 * i] + v[4 * i + 1]) + (v[4 * i + 2] + v[4 * i + 3]);
          }
      } else {
#pragma unroll
        for (int k = 0; k < 16; ++k)
          if (k < n) {
            v[k] = x[xr + col(k)];
            d[k] = Elem<DyT>::to_f(dy[r * C + col(k)]);
            s += v[k];
          }
      }
      const float mean = wave_sum(s) / C;
      float q = 0.f;
#pragma unroll
      for (int k = 0; k < 16; ++k)
        if (k < n) { v[k] -= mean; q += v[k] * v[k]; }
      const float rstd = 1.0f / sqrtf(wave_sum(q) / C + eps);
      float s1 = 0.f, s2 = 0.f;
#pragma unroll
      for (int k = 0; k < 16; ++k)
        if (k < n) {
          const float xh = v[k] * rstd, gd = g[k] * d[k];
          v[k] = xh;
          s1 += gd;
          s2 += gd * xh;
          dg[k] += d[k] * xh;
          db[k] += d[k];
        }
      s1 = wave_sum(s1) / C;
      s2 = wave_sum(s2) / C;
      if constexpr (VEC) {
#pragma unroll
        for (int i = 0; i < 4; ++i)
          if (4 * i < n) {
            float4* p = reinterpret_cast<float4*>(dx + xr + i * 256 + lane * 4);
            float4 o = *p;
            o.x += rstd * (g[4 * i] * d[4 * i] - s1 - v[4 * i] * s2);
            o.y += rstd * (g[4 * i + 1] * d[4 * i + 1] - s1 - v[4 * i + 1] * s2);
            o.z += rstd * (g[4 * i + 2] * d[4 * i + 2] - s1 - v[4 * i + 2] * s2);
            o.w += rstd * (g[4 * i + 3] * d[4 * i + 3] - s1 - v[4 * i + 3] * s2);
            *p = o;
          }
      } else {
#pragma unroll
        for (int k = 0; k < 16; ++k)
          if (k < n) dx[xr + col(k)] += rstd * (g[k] * d[k] - s1 - v[k] * s2);
      }
    }
  }
#pragma unroll
  for (int k = 0; k < 16; ++k)
    if (k < n) { red[wave][0][col(k)] = dg[k]; red[wave][1][col(k)] = db[k]; }
  __syncthreads();
  for (int c = threadIdx.x; c < C; c += 256) {
    partial[(int64_t)blockIdx.x * 2 * C + c] = (red[0][0][c] + red[1][0][c]) + (red[2][0][c] + red[3][0][c]);
    partial[(int64_t)blockIdx.x * 2 * C + C + c] = (red[0][1][c] + red[1][1][c]) + (red[2][1][c] + red[3][1][c]);
  }
}

// The narrow Video Swin widths (C = 96 / 192 / 384): LPR lanes per row, 64 / LPR rows per wave,
// lane `sub` owns the VPL = C / LPR contiguous columns sub*VPL.. (8-byte loads, gamma held in
// registers), the row sums over the LPR-lane group by xor shuffles, dgamma / dbeta partials in
// registers per lane and combined over (wave, row group) in a fixed order through LDS.  One wave
// per row (ln_bwd_wide_kernel at C = 96) left a third of the lanes idle and ran the four
// reductions of each row one after another: ~270 us per call at Swin stage 1.
template <typename DyT, int C, int LPR>
__global__ __launch_bounds__(256) void ln_bwd_small_kernel(const float* __restrict__ x, const DyT* __restrict__ dy,
                                                           const float* __restrict__ gamma, float* __restrict__ dx,
                                                           int64_t rows, int64_t rpg, int64_t gstride, int64_t goff,
                                                           float eps, float* __restrict__ partial) {
  constexpr int VPL = C / LPR, RPW = 64 / LPR;
  static_assert(C % LPR == 0 && VPL % 2 == 0 && 64 % LPR == 0, "row split");
  __shared__ float red[4][RPW][2][C];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, sub = lane % LPR, rsub = lane / LPR;
  const int c0 = sub * VPL;
  float gm[VPL], dg[VPL], db[VPL];
#pragma unroll
  for (int i = 0; i < VPL; ++i) { gm[i] = gamma[c0 + i]; dg[i] = 0.f; db[i] = 0.f; }
  const int64_t step = (int64_t)gridDim.x * 4 * RPW;
  for (int64_t rb = ((int64_t)blockIdx.x * 4 + wave) * RPW; rb < rows; rb += step) {
    const int64_t r = rb + rsub;
    const bool live = r < rows;                         // uniform over the lane's LPR group
    const int64_t xr = live ? map_row(r, rpg, gstride, goff) * C : 0;
    float v[VPL], d[VPL];
    float s = 0.f;
    if (live) {
      const float2* xp = reinterpret_cast<const float2*>(x + xr + c0);
#pragma unroll
      for (int i = 0; i < VPL / 2; ++i) {
        const float2 t = xp[i];
        v[2 * i] = t.x; v[2 * i + 1] = t.y;
        s += t.x + t.y;
      }
      if constexpr (sizeof(DyT) == 2) {
        const unsigned* dp = reinterpret_cast<const unsigned*>(dy + r * C + c0);
#pragma unroll
        for (int i = 0; i < VPL / 2; ++i) {
          const unsigned w = dp[i];
          d[2 * i] = __uint_as_float(w << 16);
          d[2 * i + 1] = __uint_as_float(w & 0xffff0000u);
        }
      } else {
        const float2* dp = reinterpret_cast<const float2*>(dy + r * C + c0);
#pragma unroll
        for (int i = 0; i < VPL / 2; ++i) {
          const float2 t = dp[i];
          d[2 * i] = t.x; d[2 * i + 1] = t.y;
        }
      }
    } else {
#pragma unroll
      for (int i = 0; i < VPL; ++i) { v[i] = 0.f; d[i] = 0.f; }
    }
#pragma unroll
    for (int o = 1; o < LPR; o <<= 1) s += __shfl_xor(s, o);
    const float mean = s / C;
    float q = 0.f;
#pragma unroll
    for (int i = 0; i < VPL; ++i) { v[i] -= mean; q += v[i] * v[i]; }
#pragma unroll
    for (int o = 1; o < LPR; o <<= 1) q += __shfl_xor(q, o);
    const float rstd = 1.0f / sqrtf(q / C + eps);
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int i = 0; i < VPL; ++i) {
      const float xh = v[i] * rstd, gd = gm[i] * d[i];
      v[i] = xh;
      s1 += gd;
      s2 += gd * xh;
      dg[i] += d[i] * xh;
      db[i] += d[i];
    }
#pragma unroll
    for (int o = 1; o < LPR; o <<= 1) { s1 += __shfl_xor(s1, o); s2 += __shfl_xor(s2, o); }
    s1 /= C;
    s2 /= C;
    if (live) {
      float2* op = reinterpret_cast<float2*>(dx + xr + c0);
#pragma unroll
      for (int i = 0; i < VPL / 2; ++i) {
        float2 t = op[i];
        t.x += rstd * (gm[2 * i] * d[2 * i] - s1 - v[2 * i] * s2);
        t.y += rstd * (gm[2 * i + 1] * d[2 * i + 1] - s1 - v[2 * i + 1] * s2);
        op[i] = t;
      }
    }
  }
#pragma unroll
  for (int i = 0; i < VPL; ++i) { red[wave][rsub][0][c0 + i] = dg[i]; red[wave][rsub][1][c0 + i] = db[i]; }
  __syncthreads();
  for (int c = threadIdx.x; c < C; c += 256) {
    float a = 0.f, b = 0.f;
#pragma unroll
    for (int w = 0; w < 4; ++w)
#pragma unroll
      for (int k = 0; k < RPW; ++k) { a += red[w][k][0][c]; b += red[w][k][1][c]; }
    partial[(int64_t)blockIdx.x * 2 * C + c] = a;
    partial[(int64_t)blockIdx.x * 2 * C + C + c] = b;
  }
}

// Any C % 32 == 0 up to 2048 (the Video Swin widths: 96 / 192 / 384 / 768, 128 ... 1024, and the
// PatchMerging norms over 4C up to 2048): one wave per row, lane owns columns k*64 + lane.
template <typename DyT>
__global__ __launch_bounds__(256) void ln_bwd_wide_kernel(const float* __restrict__ x, const DyT* __restrict__ dy,
                                                          const float* __restrict__ gamma, float* __restrict__ dx,
                                                          int64_t rows, int C, int64_t rpg, int64_t gstride,
                                                          int64_t goff, float eps, float* __restrict__ partial) {
  __shared__ float red[4][2][2048];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int n = (C + 63) >> 6;                                  // slots (<= 32)
  float dg[32], db[32];
#pragma unroll
  for (int k = 0; k < 32; ++k) { dg[k] = 0.f; db[k] = 0.f; }
  for (int64_t r = (int64_t)blockIdx.x * 4 + wave; r < rows; r += (int64_t)gridDim.x * 4) {
    const int64_t xr = map_row(r, rpg, gstride, goff) * C;
    float v[32], d[32];
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < 32; ++k) {
      const int c = k * 64 + lane;
      const bool in = k < n && c < C;
      v[k] = in ? x[xr + c] : 0.f;
      d[k] = in ? Elem<DyT>::to_f(dy[r * C + c]) : 0.f;
      s += v[k];
    }
    const float mean = wave_sum(s) / C;
    float q = 0.f;
#pragma unroll
    for (int k = 0; k < 32; ++k)
      if (k < n && k * 64 + lane < C) { v[k] -= mean; q += v[k] * v[k]; }
    const float rstd = 1.0f / sqrtf(wave_sum(q) / C + eps);
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int k = 0; k < 32; ++k) {
      const int c = k * 64 + lane;
      if (k < n && c < C) {
        const float xh = v[k] * rstd, gd = gamma[c] * d[k];
        v[k] = xh;
        s1 += gd;
        s2 += gd * xh;
        dg[k] += d[k] * xh;
        db[k] += d[k];
      }
    }
    s1 = wave_sum(s1) / C;
    s2 = wave_sum(s2) / C;
#pragma unroll
    for (int k = 0; k < 32; ++k) {
      const int c = k * 64 + lane;
      if (k < n && c < C) dx[xr + c] += rstd * (gamma[c] * d[k] - s1 - v[k] * s2);
    }
  }
#pragma unroll
  for (int k = 0; k < 32; ++k) {
    const int c = k * 64 + lane;
    if (k < n && c < C) { red[wave][0][c] = dg[k]; red[wave][1][c] = db[k]; }
  }
  __syncthreads();
  for (int c = threadIdx.x; c < C; c += 256) {
    partial[(int64_t)blockIdx.x * 2 * C + c] = (red[0][0][c] + red[1][0][c]) + (red[2][0][c] + red[3][0][c]);
    partial[(int64_t)blockIdx.x * 2 * C + C + c] = (red[0][1][c] + red[1][1][c]) + (red[2][1][c] + red[3][1][c]);
  }
}

// C = 768 (ViT-B), the training step's LayerNorm backward (the default, DSVT_LNB_VARIANT=2): the
// same arithmetic as ln_bwd_kernel<DyT, true, 3, true>, with TWO rows in flight ahead of the one
// being reduced instead of one (x, dy, dx of three rows live, dy kept as packed bf16 until used;
// 224 VGPRs: 2 blocks per CU, 512 blocks).  Alone 59.1 -> 56.0 us at 25 104 rows (4.6 -> 4.8
// TB/s), train step +0.3-0.7 % (tools/gpu_s17.sh, gpu_s19.sh).
// dxb (optional): the updated dx rows also stored as bf16 -- the copy the next GEMMs of the dX chain
// read -- at row (r / og) * (og - osk) + r % og - osk of dxb for the rows with r % og >= osk (og
// = rows, osk = 0: the same rows; og = L, osk = 1: the patch rows of [B, L] token rows, compact),
// instead of a cast_rows pass re-reading dx.
template <typename DyT>
__global__ __launch_bounds__(256, 2) void ln_bwd768_kernel(const float* __restrict__ x, const DyT* __restrict__ dy,
                                                        const float* __restrict__ gamma, float* __restrict__ dx,
                                                        int64_t rows, int64_t rpg, int64_t gstride, int64_t goff,
                                                        float eps, float* __restrict__ partial,
                                                        bf16_t* __restrict__ dxb = nullptr, int64_t og = 1,
                                                        int64_t osk = 0) {
  constexpr int C = 768, NK = 12;
  constexpr bool BF = std::is_same<DyT, bf16_t>::value;
  constexpr int ND = BF ? 6 : 12;                 // dy registers per row (packed bf16 pairs / fp32)
  __shared__ float red[4][2][C];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  float dg[NK], db[NK], g[NK];
#pragma unroll
  for (int k = 0; k < NK; ++k) {
    dg[k] = 0.f;
    db[k] = 0.f;
    g[k] = gamma[(k >> 2) * 256 + lane * 4 + (k & 3)];
  }
  struct RowRegs {
    float x[NK], o[NK];
    unsigned d[ND];
  };
  auto load_row = [&](int64_t r, RowRegs& R) {
    const int64_t xr = map_row(r, rpg, gstride, goff) * C;
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      load4(x + xr + i * 256 + lane * 4, R.x + 4 * i);
      if constexpr (BF) {
        const uint2 u = *reinterpret_cast<const uint2*>(dy + r * C + i * 256 + lane * 4);
        R.d[2 * i] = u.x;
        R.d[2 * i + 1] = u.y;
      } else {
        const float4 u = *reinterpret_cast<const float4*>(dy + r * C + i * 256 + lane * 4);
        R.d[4 * i] = __float_as_uint(u.x); R.d[4 * i + 1] = __float_as_uint(u.y);
        R.d[4 * i + 2] = __float_as_uint(u.z); R.d[4 * i + 3] = __float_as_uint(u.w);
      }
      load4(dx + xr + i * 256 + lane * 4, R.o + 4 * i);
    }
  };
  auto dy_of = [&](const RowRegs& R, int k) -> float {
    if constexpr (BF) return (k & 1) ? bf16_hi(R.d[k >> 1]) : bf16_lo(R.d[k >> 1]);
    else return __uint_as_float(R.d[k]);
  };
  auto reduce_row = [&](int64_t r, RowRegs& R) {
    const int64_t xr = map_row(r, rpg, gstride, goff) * C;
    float cd[NK];
#pragma unroll
    for (int k = 0; k < NK; ++k) cd[k] = dy_of(R, k);
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < NK; ++k) s += R.x[k];
    const float inv_c = 1.0f / (float)C;
    const float mean = wave_sum_dpp(s) * inv_c;
    float q = 0.f;
#pragma unroll
    for (int k = 0; k < NK; ++k) { R.x[k] -= mean; q += R.x[k] * R.x[k]; }
    const float rstd = __builtin_amdgcn_rsqf(wave_sum_dpp(q) * inv_c + eps);
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int k = 0; k < NK; ++k) {
      const float xh = R.x[k] * rstd, gd = g[k] * cd[k];
      R.x[k] = xh;
      s1 += gd;
      s2 += gd * xh;
      dg[k] += cd[k] * xh;
      db[k] += cd[k];
    }
    s1 = wave_sum_dpp(s1) * inv_c;
    s2 = wave_sum_dpp(s2) * inv_c;
    const int64_t rr = r % og;
    const bool cp = dxb != nullptr && rr >= osk;                 // wave-uniform
    bf16_t* const ob = dxb + ((r / og) * (og - osk) + rr - osk) * C;
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      float4 o;
      o.x = R.o[4 * i] + rstd * (g[4 * i] * cd[4 * i] - s1 - R.x[4 * i] * s2);
      o.y = R.o[4 * i + 1] + rstd * (g[4 * i + 1] * cd[4 * i + 1] - s1 - R.x[4 * i + 1] * s2);
      o.z = R.o[4 * i + 2] + rstd * (g[4 * i + 2] * cd[4 * i + 2] - s1 - R.x[4 * i + 2] * s2);
      o.w = R.o[4 * i + 3] + rstd * (g[4 * i + 3] * cd[4 * i + 3] - s1 - R.x[4 * i + 3] * s2);
      *reinterpret_cast<float4*>(dx + xr + i * 256 + lane * 4) = o;
      if (cp)
        *reinterpret_cast<uint2*>(ob + i * 256 + lane * 4) = make_uint2(cvt_pk_bf16(o.x, o.y), cvt_pk_bf16(o.z, o.w));
    }
  };
  const int64_t S = (int64_t)gridDim.x * 4;
  int64_t r = (int64_t)blockIdx.x * 4 + wave;
  RowRegs A, B, D;
  if (r < rows) load_row(r, A);
  if (r + S < rows) load_row(r + S, B);
  while (r < rows) {                     // three rows per trip: A, B, D rotate without moves
    if (r + 2 * S < rows) load_row(r + 2 * S, D);
    reduce_row(r, A);
    r += S;
    if (r >= rows) break;
    if (r + 2 * S < rows) load_row(r + 2 * S, A);
    reduce_row(r, B);
    r += S;
    if (r >= rows) break;
    if (r + 2 * S < rows) load_row(r + 2 * S, B);
    reduce_row(r, D);
    r += S;
  }
#pragma unroll
  for (int k = 0; k < NK; ++k) {
    const int c = (k >> 2) * 256 + lane * 4 + (k & 3);
    red[wave][0][c] = dg[k];
    red[wave][1][c] = db[k];
  }
  __syncthreads();
  for (int c = threadIdx.x; c < C; c += 256) {
    partial[(int64_t)blockIdx.x * 2 * C + c] = (red[0][0][c] + red[1][0][c]) + (red[2][0][c] + red[3][0][c]);
    partial[(int64_t)blockIdx.x * 2 * C + C + c] = (red[0][1][c] + red[1][1][c]) + (red[2][1][c] + red[3][1][c]);
  }
}

// >= 4 rows per wave; at most 768 blocks = 3 per CU, what the C = 768 kernel's 163 VGPRs keep
// resident (a 1024-block grid left a second, partial round on a third of the CUs)
static int lnb_variant() {
  static const int v = getenv("DSVT_LNB_VARIANT") ? atoi(getenv("DSVT_LNB_VARIANT")) : 2;   // tuning only
  return v;
}

int ln_bwd_blocks(int64_t rows) {
  const int64_t cap = lnb_variant() == 2 ? 512 : 768;      // ln_bwd768_kernel: 2 blocks per CU
  int64_t b = (rows + 15) / 16;
  return (int)(b < 1 ? 1 : (b > cap ? cap : b));
}

hipError_t launch_ln_bwd_cast(int dy_dtype, const float* x, const void* dy, const float* gamma, float* dx,
                              int64_t rows, int64_t rpg, int64_t gstride, int64_t goff, float eps, float* partial,
                              void* dxb, int64_t og, int64_t osk, hipStream_t s) {
  const int nb = ln_bwd_blocks(rows);
  if (dy_dtype == 0)
    ln_bwd768_kernel<bf16_t><<<nb, 256, 0, s>>>(x, (const bf16_t*)dy, gamma, dx, rows, rpg, gstride, goff, eps, partial,
                                                (bf16_t*)dxb, og, osk);
  else
    ln_bwd768_kernel<float><<<nb, 256, 0, s>>>(x, (const float*)dy, gamma, dx, rows, rpg, gstride, goff, eps, partial,
                                               (bf16_t*)dxb, og, osk);
  return hipGetLastError();
}

hipError_t launch_ln_bwd(int dy_dtype, const float* x, const void* dy, const float* gamma, float* dx, int64_t rows,
                         int64_t C, int64_t rpg, int64_t gstride, int64_t goff, float eps, float* partial,
                         hipStream_t s) {
  const int nb = ln_bwd_blocks(rows);
#define DSVT_LNB(T, V) ln_bwd_kernel<T, V><<<nb, 256, 0, s>>>(x, (const T*)dy, gamma, dx, rows, (int)C, rpg, gstride, \
                                                             goff, eps, partial)
#define DSVT_LNB3(T) ln_bwd_kernel<T, true, 3><<<nb, 256, 0, s>>>(x, (const T*)dy, gamma, dx, rows, (int)C, rpg, \
                                                                  gstride, goff, eps, partial)
  const int lnb_v = lnb_variant();
#define DSVT_LNBS(CC, LPR)                                                                                       \
  {                                                                                                               \
    if (dy_dtype == 0)                                                                                            \
      ln_bwd_small_kernel<bf16_t, CC, LPR><<<nb, 256, 0, s>>>(x, (const bf16_t*)dy, gamma, dx, rows, rpg, gstride,  \
                                                              goff, eps, partial);                                \
    else                                                                                                          \
      ln_bwd_small_kernel<float, CC, LPR><<<nb, 256, 0, s>>>(x, (const float*)dy, gamma, dx, rows, rpg, gstride,    \
                                                             goff, eps, partial);                                 \
    return hipGetLastError();                                                                                     \
  }
  // the narrow Video Swin widths (8-byte aligned rows)
  if (((uintptr_t)x & 7) == 0 && ((uintptr_t)dx & 7) == 0 && ((uintptr_t)dy & 7) == 0) {
    if (C == 96) DSVT_LNBS(96, 16)
    if (C == 192) DSVT_LNBS(192, 16)
    if (C == 384) DSVT_LNBS(384, 32)
  }
#undef DSVT_LNBS
  if (C == 768 && lnb_v == 2) {        // two rows of look-ahead: 2 blocks per CU (224 VGPRs)
    if (dy_dtype == 0)
      ln_bwd768_kernel<bf16_t><<<nb, 256, 0, s>>>(x, (const bf16_t*)dy, gamma, dx, rows, rpg, gstride, goff, eps, partial);
    else
      ln_bwd768_kernel<float><<<nb, 256, 0, s>>>(x, (const float*)dy, gamma, dx, rows, rpg, gstride, goff, eps, partial);
  } else if (C == 768 && lnb_v == 1) {        // DPP reductions, reciprocal multiplies
    if (dy_dtype == 0)
      ln_bwd_kernel<bf16_t, true, 3, true><<<nb, 256, 0, s>>>(x, (const bf16_t*)dy, gamma, dx, rows, (int)C, rpg,
                                                              gstride, goff, eps, partial);
    else
      ln_bwd_kernel<float, true, 3, true><<<nb, 256, 0, s>>>(x, (const float*)dy, gamma, dx, rows, (int)C, rpg,
                                                             gstride, goff, eps, partial);
  } else if (C == 768) {               // ViT-B: 3 float4 chunks per lane, a tighter register file
    if (dy_dtype == 0) DSVT_LNB3(bf16_t); else DSVT_LNB3(float);
  } else if (C % 256 == 0 && C <= 1024) {   // VEC: NI = C / 256 float4 chunks per lane
#define DSVT_LNBN(T, NI_) ln_bwd_kernel<T, true, NI_><<<nb, 256, 0, s>>>(x, (const T*)dy, gamma, dx, rows, (int)C, rpg, \
                                                                        gstride, goff, eps, partial)
    switch (C / 256) {
      case 1: if (dy_dtype == 0) DSVT_LNBN(bf16_t, 1); else DSVT_LNBN(float, 1); break;
      case 2: if (dy_dtype == 0) DSVT_LNBN(bf16_t, 2); else DSVT_LNBN(float, 2); break;
      default: if (dy_dtype == 0) DSVT_LNBN(bf16_t, 4); else DSVT_LNBN(float, 4); break;   // C = 1024
    }
#undef DSVT_LNBN
  } else if (C % 64 != 0 || C > 1024) {
    if (dy_dtype == 0)
      ln_bwd_wide_kernel<bf16_t><<<nb, 256, 0, s>>>(x, (const bf16_t*)dy, gamma, dx, rows, (int)C, rpg, gstride, goff,
                                                    eps, partial);
    else
      ln_bwd_wide_kernel<float><<<nb, 256, 0, s>>>(x, (const float*)dy, gamma, dx, rows, (int)C, rpg, gstride, goff,
                                                   eps, partial);
  } else {
    if (dy_dtype == 0) DSVT_LNB(bf16_t, false); else DSVT_LNB(float, false);
  }
#undef DSVT_LNB
#undef DSVT_LNB3
  return hipGetLastError();
}

// ================================================================ column sums (bias grads)
// Block = 64 column groups of 4 (256 columns, 8-/16-B loads) x 4 row lanes; grid.y = row chunks.
// Each thread sums its 4 columns over the chunk's rows r = lane_row (mod 4); the 4 row lanes are
// combined in LDS and the block writes one partial row.  C % 4 == 0.
template <typename T>
__global__ __launch_bounds__(256) void colsum_partial_kernel(const T* __restrict__ y, int64_t rows, int64_t C,
                                                             int64_t ld, int64_t rpg, int64_t gstride, int64_t goff,
                                                             const float* __restrict__ row_scale, int64_t chunk,
                                                             float* __restrict__ partial) {
  __shared__ float4 red[4][64];
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  const int64_t r0 = (int64_t)blockIdx.y * chunk;
  const int64_t r1 = r0 + chunk < rows ? r0 + chunk : rows;
  const int64_t c = ((int64_t)blockIdx.x * 64 + tx) * 4;
  float a[4] = {0.f, 0.f, 0.f, 0.f};
  if (c < C) {
    for (int64_t r = r0 + ty; r < r1; r += 4) {
      float v[4];
      load4(y + map_row(r, rpg, gstride, goff) * ld + c, v);
      const float sc = row_scale ? row_scale[r] : 1.0f;
#pragma unroll
      for (int e = 0; e < 4; ++e) a[e] = fmaf(v[e], sc, a[e]);
    }
  }
  red[ty][tx] = make_float4(a[0], a[1], a[2], a[3]);
  __syncthreads();
  if (ty == 0 && c < C) {
    const float4 p0 = red[0][tx], p1 = red[1][tx], p2 = red[2][tx], p3 = red[3][tx];
    *reinterpret_cast<float4*>(partial + (int64_t)blockIdx.y * C + c) =
        make_float4((p0.x + p1.x) + (p2.x + p3.x), (p0.y + p1.y) + (p2.y + p3.y), (p0.z + p1.z) + (p2.z + p3.z),
                    (p0.w + p1.w) + (p2.w + p3.w));
  }
}

// out[c] (+)= sum_p partial[p*stride + c]: block = 32 columns x 8 part lanes, LDS combine
// (fixed order -> deterministic)
// (out2: columns >= split go to out2[c - split] -- the LayerNorm backward's [dgamma | dbeta]
// partial rows reduced in one pass, each column in the same order as alone)
__global__ __launch_bounds__(256) void reduce_partials_kernel(const float* __restrict__ partial, int64_t nparts,
                                                              int64_t width, int64_t stride, float* __restrict__ out,
                                                              int accumulate, float* __restrict__ out2 = nullptr,
                                                              int64_t split = INT64_MAX) {
  __shared__ float red[8][33];
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;
  const int64_t c = (int64_t)blockIdx.x * 32 + tx;
  float a = 0.f;
  if (c < width)
    for (int64_t p = ty; p < nparts; p += 8) a += partial[p * stride + c];
  red[ty][tx] = a;
  __syncthreads();
  if (ty == 0 && c < width) {
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < 8; ++k) s += red[k][tx];
    float* o = c < split ? out + c : out2 + (c - split);
    *o = accumulate ? *o + s : s;
  }
}

// Level 1 of the two-level partial reduction: slice s of the parts (chunk rows) summed per
// column, in order, into the slice's own first row (the partials are workspace: consumed).
__global__ __launch_bounds__(256) void reduce_slices_kernel(float* __restrict__ partial, int64_t nparts, int64_t width,
                                                            int64_t stride, int64_t chunk) {
  const int64_t c = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t p0 = (int64_t)blockIdx.y * chunk, p1 = p0 + chunk < nparts ? p0 + chunk : nparts;
  if (c >= width || p0 >= nparts) return;
  float a = 0.f;
  for (int64_t q = p0; q < p1; ++q) a += partial[q * stride + c];
  partial[p0 * stride + c] = a;
}

// fixed-order sum of nparts partial rows: one kernel for few parts; otherwise 64 slices summed
// in parallel first (the single-kernel form ran on width/32 = 24 workgroups: ~12 us per call)
static hipError_t reduce_parts(const float* partial, int64_t nparts, int64_t width, int64_t stride, float* out,
                               int accumulate, hipStream_t s, float* out2 = nullptr, int64_t split = INT64_MAX) {
  if (nparts > 128) {
    const int64_t slices = 64, chunk = (nparts + slices - 1) / slices;
    const int64_t used = (nparts + chunk - 1) / chunk;
    dim3 g1((unsigned)((width + 255) / 256), (unsigned)used);
    reduce_slices_kernel<<<g1, 256, 0, s>>>(const_cast<float*>(partial), nparts, width, stride, chunk);
    if (hipError_t e = hipGetLastError()) return e;
    reduce_partials_kernel<<<(unsigned)((width + 31) / 32), 256, 0, s>>>(partial, used, width, chunk * stride, out,
                                                                         accumulate, out2, split);
    return hipGetLastError();
  }
  reduce_partials_kernel<<<(unsigned)((width + 31) / 32), 256, 0, s>>>(partial, nparts, width, stride, out,
                                                                       accumulate, out2, split);
  return hipGetLastError();
}

// row chunks of the bias-gradient column sums: up to 512 (x C/256 workgroups) so that the
// 25k-row calls fill the chip; the partials then take the two-level reduction
int64_t colsum_parts(int64_t rows) {
  int64_t p = (rows + 31) / 32;
  return p < 1 ? 1 : (p > 512 ? 512 : p);
}

hipError_t launch_colsum_rows(int dtype, const void* y, int64_t rows, int64_t C, int64_t ld, int64_t rpg,
                              int64_t gstride, int64_t goff, const float* row_scale, float* partial, float* out,
                              int accumulate, hipStream_t s) {
  const int64_t parts = colsum_parts(rows), chunk = (rows + parts - 1) / parts;
  dim3 grid((unsigned)((C + 255) / 256), (unsigned)parts);
  if (dtype == 0)
    colsum_partial_kernel<bf16_t><<<grid, 256, 0, s>>>((const bf16_t*)y, rows, C, ld, rpg, gstride, goff, row_scale,
                                                       chunk, partial);
  else
    colsum_partial_kernel<float><<<grid, 256, 0, s>>>((const float*)y, rows, C, ld, rpg, gstride, goff, row_scale,
                                                      chunk, partial);
  if (hipError_t e = hipGetLastError()) return e;
  return reduce_parts(partial, parts, C, C, out, accumulate, s);
}

hipError_t launch_reduce_partials(const float* partial, int64_t nparts, int64_t width, int64_t stride, float* out,
                                  int accumulate, hipStream_t s) {
  return reduce_parts(partial, nparts, width, stride, out, accumulate, s);
}

hipError_t launch_ln_params_reduce(const float* partial, int64_t nparts, int64_t C, float* dgamma, float* dbeta,
                                   int accumulate, hipStream_t s) {
  return reduce_parts(partial, nparts, 2 * C, 2 * C, dgamma, accumulate, s, dbeta, C);
}

// ================================================================ temporal attention backward
// grid (nseq, ceil(heads/G)); LDS per head: q, k, v, dO [T][64] fp32 and P, dS [T][T].
// Phase 1, item (head hh, query i), 16 lanes x 4 dims: scores, softmax, dP = dO_i.v_j,
// D_i = sum_j P dP, dS = P (dP - D), dq_i = scale sum_j dS_ij k_j.  Phase 2, item (hh, key j):
// dk_j = scale sum_i dS_ij q_i, dv_j = sum_i P_ij dO_i.
__device__ __forceinline__ float sum16(float v) {
  v += __shfl_xor(v, 1, 64);
  v += __shfl_xor(v, 2, 64);
  v += __shfl_xor(v, 4, 64);
  v += __shfl_xor(v, 8, 64);
  return v;
}

template <typename T>
__global__ __launch_bounds__(256) void attn_temporal_bwd_kernel(const T* __restrict__ qkv, const T* __restrict__ dout,
                                                                T* __restrict__ dqkv, int Tf, int heads, int G,
                                                                int64_t C, float scale) {
  extern __shared__ __attribute__((aligned(16))) char dyn_smem[];
  float* sm = reinterpret_cast<float*>(dyn_smem);
  const int tid = threadIdx.x;
  const int64_t sq = blockIdx.x;
  const int h0 = blockIdx.y * G;
  const int gh = (heads - h0) < G ? (heads - h0) : G;
  const int per_head = 4 * Tf * 64 + 2 * Tf * Tf;
  // stage q, k, v, dO of the group's heads as fp32, one 16-byte piece (8 bf16 / 4 fp32) per load
  constexpr int PE = 16 / (int)sizeof(T);                   // elements per piece
  for (int e = tid; e < gh * Tf * 4 * (64 / PE); e += 256) {
    const int d = (e % (64 / PE)) * PE, rest = e / (64 / PE);
    const int which = rest % 4, tt = (rest / 4) % Tf, hh = rest / (4 * Tf);
    const int64_t row = sq * Tf + tt;
    const int64_t col = (int64_t)(h0 + hh) * 64 + d;
    const T* src = which < 3 ? qkv + row * 3 * C + which * C + col : dout + row * C + col;
    const uint4 u = *reinterpret_cast<const uint4*>(src);
    float* dst = sm + hh * per_head + (which * Tf + tt) * 64 + d;
    if constexpr (sizeof(T) == 2) {
      const unsigned w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
      for (int k = 0; k < 4; ++k) { dst[2 * k] = bf16_lo(w[k]); dst[2 * k + 1] = bf16_hi(w[k]); }
    } else {
      dst[0] = __uint_as_float(u.x); dst[1] = __uint_as_float(u.y);
      dst[2] = __uint_as_float(u.z); dst[3] = __uint_as_float(u.w);
    }
  }
  __syncthreads();
  const int sub = tid & 15, d0 = sub * 4;
  for (int it = tid >> 4; it < gh * Tf; it += 16) {
    const int hh = it % gh, i = it / gh;
    float* H = sm + hh * per_head;
    const float* q = H + i * 64 + d0;
    const float* dO = H + (3 * Tf + i) * 64 + d0;
    float* P = H + 4 * Tf * 64;
    float* dS = P + Tf * Tf;
    float m = -INFINITY;
    for (int j = 0; j < Tf; ++j) {
      const float* k = H + (Tf + j) * 64 + d0;
      const float s = sum16(q[0] * k[0] + q[1] * k[1] + q[2] * k[2] + q[3] * k[3]) * scale;
      if (sub == 0) P[i * Tf + j] = s;
      m = fmaxf(m, s);
    }
    __builtin_amdgcn_wave_barrier();
    // probabilities once per (i, j): exp2 of the log2e-scaled logits, written back over them
    float l = 0.f;
    for (int j = 0; j < Tf; ++j) l += exp2f((P[i * Tf + j] - m) * 1.4426950408889634f);
    const float inv = 1.0f / l;
    __builtin_amdgcn_wave_barrier();
    if (sub == 0)
      for (int j = 0; j < Tf; ++j) P[i * Tf + j] = exp2f((P[i * Tf + j] - m) * 1.4426950408889634f) * inv;
    __builtin_amdgcn_wave_barrier();
    float D = 0.f;
    for (int j = 0; j < Tf; ++j) {
      const float* v = H + (2 * Tf + j) * 64 + d0;
      const float dp = sum16(dO[0] * v[0] + dO[1] * v[1] + dO[2] * v[2] + dO[3] * v[3]);
      D += P[i * Tf + j] * dp;
      if (sub == 0) dS[i * Tf + j] = dp;
    }
    __builtin_amdgcn_wave_barrier();
    float dq[4] = {0.f, 0.f, 0.f, 0.f};
    for (int j = 0; j < Tf; ++j) {
      const float ds = P[i * Tf + j] * (dS[i * Tf + j] - D);
      const float* k = H + (Tf + j) * 64 + d0;
#pragma unroll
      for (int e = 0; e < 4; ++e) dq[e] = fmaf(ds, k[e], dq[e]);
    }
    __builtin_amdgcn_wave_barrier();
    if (sub == 0)
      for (int j = 0; j < Tf; ++j) dS[i * Tf + j] = P[i * Tf + j] * (dS[i * Tf + j] - D);
    store4(dqkv + (sq * Tf + i) * 3 * C + (int64_t)(h0 + hh) * 64 + d0, dq[0] * scale, dq[1] * scale, dq[2] * scale,
           dq[3] * scale);
  }
  __syncthreads();
  for (int it = tid >> 4; it < gh * Tf; it += 16) {
    const int hh = it % gh, j = it / gh;
    const float* H = sm + hh * per_head;
    const float* P = H + 4 * Tf * 64;
    const float* dS = P + Tf * Tf;
    float dk[4] = {0.f, 0.f, 0.f, 0.f}, dv[4] = {0.f, 0.f, 0.f, 0.f};
    for (int i = 0; i < Tf; ++i) {
      const float* q = H + i * 64 + d0;
      const float* dO = H + (3 * Tf + i) * 64 + d0;
      const float ds = dS[i * Tf + j], p = P[i * Tf + j];
#pragma unroll
      for (int e = 0; e < 4; ++e) { dk[e] = fmaf(ds, q[e], dk[e]); dv[e] = fmaf(p, dO[e], dv[e]); }
    }
    T* o = dqkv + (sq * Tf + j) * 3 * C + (int64_t)(h0 + hh) * 64 + d0;
    store4(o + C, dk[0] * scale, dk[1] * scale, dk[2] * scale, dk[3] * scale);
    store4(o + 2 * C, dv[0], dv[1], dv[2], dv[3]);
  }
}

static thread_local int g_attn_bwd_variant = 0;  // 0 = auto, 1 = force the generic VALU kernels (tests / tools)

// 16-lane butterflies of the register temporal kernels: reduce-scatter (after the stage with
// mask m the lane keeps the half selected by sub & m) and the reverse all-gather of the lane's
// VPL entries (natural index order)
template <int NV, int S>
__device__ __forceinline__ void tb_rs_stage(float (&vals)[NV], int sub) {
  constexpr int mask = 8 >> S, half = NV >> (S + 1);   // compile-time trip counts: fully unrolled
  const bool hi = (sub & mask) != 0;
#pragma unroll
  for (int k = 0; k < half; ++k) {
    const float mine = hi ? vals[half + k] : vals[k];
    const float oth = hi ? vals[k] : vals[half + k];
    vals[k] = mine + __shfl_xor(oth, mask, 64);
  }
}

template <int NV>
__device__ __forceinline__ void tb_reduce_scatter(float (&vals)[NV], int sub) {
  tb_rs_stage<NV, 0>(vals, sub);
  tb_rs_stage<NV, 1>(vals, sub);
  tb_rs_stage<NV, 2>(vals, sub);
  tb_rs_stage<NV, 3>(vals, sub);
}

template <int NV, int VPL, int S>
__device__ __forceinline__ void tb_ag_stage(float (&vals)[NV], int sub) {
  constexpr int mask = 1 << S, n = VPL << S;
  const bool hi = (sub & mask) != 0;
#pragma unroll
  for (int k = 0; k < n; ++k) {
    const float recv = __shfl_xor(vals[k], mask, 64);
    const float mine = vals[k];
    vals[k] = hi ? recv : mine;
    vals[n + k] = hi ? mine : recv;
  }
}

template <int NV, int VPL>
__device__ __forceinline__ void tb_all_gather(float (&vals)[NV], int sub) {
  tb_ag_stage<NV, VPL, 0>(vals, sub);
  tb_ag_stage<NV, VPL, 1>(vals, sub);
  tb_ag_stage<NV, VPL, 2>(vals, sub);
  tb_ag_stage<NV, VPL, 3>(vals, sub);
}

// bf16, T <= TP (4 or 8): the register-resident form of the kernel above, laid out like the
// forward attn_temporal_reg (attention.hip): 16 lanes per (sequence, head), 4 of the 64 dims
// per lane, q / k / v / dO of the T rows held as packed bf16.  S = Q.K^T and dP = dO.V^T are
// lane-partial dots reduce-scattered over the 16 lanes (butterfly 8,4,2,1), so lane `sub` owns
// the VPL = TP*TP/16 entries idx = sub*VPL + k (row i = sub / LPR) of both: softmax, the row
// sums D_i = sum_j P dP (LPR lanes) and dS = P (dP - D) stay in-lane; the reverse butterfly
// all-gathers dS (for dq = scale dS.K and dk = scale dS^T.Q) and then P (for dv = P^T.dO).  Rows
// and keys past T are masked by P = 0.  Reads qkv + dO and writes dqkv once: HBM-bound.
template <int TP>
__global__ __launch_bounds__(256) void attn_temporal_bwd_reg(const bf16_t* __restrict__ qkv,
                                                             const bf16_t* __restrict__ dout,
                                                             bf16_t* __restrict__ dqkv, int64_t groups, int Tf,
                                                             int heads, int64_t C, float scale) {
  constexpr int NV = TP * TP, VPL = NV / 16, LPR = TP / VPL;
  static_assert(NV >= 16 && NV % 16 == 0, "TP must be 4 or 8");
  const int64_t grp = ((int64_t)blockIdx.x * 256 + threadIdx.x) >> 4;
  const int sub = threadIdx.x & 15;
  if (grp >= groups) return;  // the whole 16-lane group leaves together
  const int64_t sq = grp / heads;
  const int h = (int)(grp % heads);
  const bf16_t* base = qkv + sq * Tf * 3 * C + (int64_t)h * 64 + sub * 4;
  const bf16_t* dbase = dout + sq * Tf * C + (int64_t)h * 64 + sub * 4;
  uint2 rq[TP], rk[TP], rv[TP], rd[TP];
#pragma unroll
  for (int t = 0; t < TP; ++t) {
    const int tt = t < Tf ? t : Tf - 1;
    const bf16_t* r = base + (int64_t)tt * 3 * C;
    rq[t] = *reinterpret_cast<const uint2*>(r);
    rk[t] = *reinterpret_cast<const uint2*>(r + C);
    rv[t] = *reinterpret_cast<const uint2*>(r + 2 * C);
    rd[t] = *reinterpret_cast<const uint2*>(dbase + (int64_t)tt * C);
  }
  // 4-dim partial dot straight from the packed operands (v_dot2c_f32_bf16: no unpacking, so
  // the 64 partials of S or dP fit beside the four packed row sets)
  typedef __bf16 bf2_t __attribute__((ext_vector_type(2)));
  auto dot4 = [](uint2 a, uint2 b) {
    const float lo = __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(bf2_t, a.x), __builtin_bit_cast(bf2_t, b.x),
                                                     0.f, false);
    return __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(bf2_t, a.y), __builtin_bit_cast(bf2_t, b.y), lo, false);
  };
  const int i0 = sub / LPR, j0 = (sub % LPR) * VPL;   // the lane's row and first key
  // ---- P (recomputed exactly as the forward), lane entries only
  float vals[NV];
#pragma unroll
  for (int i = 0; i < TP; ++i)
#pragma unroll
    for (int j = 0; j < TP; ++j) vals[i * TP + j] = dot4(rq[i], rk[j]);
  tb_reduce_scatter<NV>(vals, sub);
  const float sl2 = scale * 1.4426950408889634f;
  float p[VPL];
  float mx = -INFINITY;
#pragma unroll
  for (int k = 0; k < VPL; ++k) {
    p[k] = (j0 + k < Tf) ? vals[k] * sl2 : -INFINITY;
    mx = fmaxf(mx, p[k]);
  }
#pragma unroll
  for (int m = 1; m < LPR; m <<= 1) mx = fmaxf(mx, __shfl_xor(mx, m, 64));
  float sum = 0.f;
#pragma unroll
  for (int k = 0; k < VPL; ++k) {
    p[k] = exp2f(p[k] - mx);
    sum += p[k];
  }
#pragma unroll
  for (int m = 1; m < LPR; m <<= 1) sum += __shfl_xor(sum, m, 64);
  const float inv = i0 < Tf ? 1.0f / sum : 0.f;      // padded query rows: P = 0 (no dk / dv share)
#pragma unroll
  for (int k = 0; k < VPL; ++k) p[k] *= inv;
  // ---- dP = dO.V^T on the same entries; D_i; dS = P (dP - D)
#pragma unroll
  for (int i = 0; i < TP; ++i)
#pragma unroll
    for (int j = 0; j < TP; ++j) vals[i * TP + j] = dot4(rd[i], rv[j]);
  tb_reduce_scatter<NV>(vals, sub);
  float D = 0.f;
#pragma unroll
  for (int k = 0; k < VPL; ++k) D += p[k] * vals[k];
#pragma unroll
  for (int m = 1; m < LPR; m <<= 1) D += __shfl_xor(D, m, 64);
#pragma unroll
  for (int k = 0; k < VPL; ++k) vals[k] = p[k] * (vals[k] - D);
  tb_all_gather<NV, VPL>(vals, sub);                 // vals = dS (full, row-major)
  bf16_t* obase = dqkv + sq * Tf * 3 * C + (int64_t)h * 64 + sub * 4;
  auto store_bf16x4 = [](bf16_t* dst, float a, float b, float c, float d) {
    uint2 w;
    w.x = pack_bf16x2(a, b);
    w.y = pack_bf16x2(c, d);
    *reinterpret_cast<uint2*>(dst) = w;
  };
  // dq_i = scale sum_j dS_ij k_j ; dk_j = scale sum_i dS_ij q_i
#pragma unroll
  for (int i = 0; i < TP; ++i) {
    float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
#pragma unroll
    for (int j = 0; j < TP; ++j) {
      const float ds = vals[i * TP + j];
      a0 = fmaf(ds, bf16_lo(rk[j].x), a0); a1 = fmaf(ds, bf16_hi(rk[j].x), a1);
      a2 = fmaf(ds, bf16_lo(rk[j].y), a2); a3 = fmaf(ds, bf16_hi(rk[j].y), a3);
    }
    if (i < Tf) store_bf16x4(obase + (int64_t)i * 3 * C, a0 * scale, a1 * scale, a2 * scale, a3 * scale);
  }
#pragma unroll
  for (int j = 0; j < TP; ++j) {
    float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
#pragma unroll
    for (int i = 0; i < TP; ++i) {
      const float ds = vals[i * TP + j];
      a0 = fmaf(ds, bf16_lo(rq[i].x), a0); a1 = fmaf(ds, bf16_hi(rq[i].x), a1);
      a2 = fmaf(ds, bf16_lo(rq[i].y), a2); a3 = fmaf(ds, bf16_hi(rq[i].y), a3);
    }
    if (j < Tf) store_bf16x4(obase + (int64_t)j * 3 * C + C, a0 * scale, a1 * scale, a2 * scale, a3 * scale);
  }
  // dv_j = sum_i P_ij dO_i
#pragma unroll
  for (int k = 0; k < VPL; ++k) vals[k] = p[k];
  tb_all_gather<NV, VPL>(vals, sub);                 // vals = P (full)
#pragma unroll
  for (int j = 0; j < TP; ++j) {
    float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
#pragma unroll
    for (int i = 0; i < TP; ++i) {
      const float pp = vals[i * TP + j];
      a0 = fmaf(pp, bf16_lo(rd[i].x), a0); a1 = fmaf(pp, bf16_hi(rd[i].x), a1);
      a2 = fmaf(pp, bf16_lo(rd[i].y), a2); a3 = fmaf(pp, bf16_hi(rd[i].y), a3);
    }
    if (j < Tf) store_bf16x4(obase + (int64_t)j * 3 * C + 2 * C, a0, a1, a2, a3);
  }
}

hipError_t launch_attn_temporal_bwd(int dtype, const void* qkv, const void* dout, void* dqkv, int64_t nseq, int64_t T,
                                    int64_t heads, int64_t C, float scale, hipStream_t s) {
  if (dtype == 0 && T <= 8 && (g_attn_bwd_variant == 0 || g_attn_bwd_variant == 2)) {
    const int64_t groups = nseq * heads;
    const unsigned blocks = (unsigned)((groups * 16 + 255) / 256);
    if (T <= 4)
      attn_temporal_bwd_reg<4><<<blocks, 256, 0, s>>>((const bf16_t*)qkv, (const bf16_t*)dout, (bf16_t*)dqkv, groups,
                                                      (int)T, (int)heads, C, scale);
    else
      attn_temporal_bwd_reg<8><<<blocks, 256, 0, s>>>((const bf16_t*)qkv, (const bf16_t*)dout, (bf16_t*)dqkv, groups,
                                                      (int)T, (int)heads, C, scale);
    return hipGetLastError();
  }
  const int64_t per_head = (4 * T * 64 + 2 * T * T) * 4;
  int64_t G = (48 * 1024) / per_head;
  if (G < 1) G = 1;
  if (G > heads) G = heads;
  dim3 grid((unsigned)nseq, (unsigned)((heads + G - 1) / G));
  const size_t smem = (size_t)(per_head * G);
  if (dtype == 0)
    attn_temporal_bwd_kernel<bf16_t><<<grid, 256, smem, s>>>((const bf16_t*)qkv, (const bf16_t*)dout, (bf16_t*)dqkv,
                                                            (int)T, (int)heads, (int)G, C, scale);
  else
    attn_temporal_bwd_kernel<float><<<grid, 256, smem, s>>>((const float*)qkv, (const float*)dout, (float*)dqkv,
                                                           (int)T, (int)heads, (int)G, C, scale);
  return hipGetLastError();
}

// ================================================================ generic attention backward
// Sequence (b, t) position i -> token row b*L + (i == 0 ? 0 : 1 + (i-1)*tok_stride + t)
// (spatial: CLS + every T-th patch row; joint / 2-D: tok_stride = 1, tin = 1, contiguous).
__device__ __forceinline__ int64_t brow(const AttnBwdParams& p, int64_t b, int64_t t, int64_t i) {
  return b * p.L + (i == 0 ? 0 : 1 + (i - 1) * p.tok_stride + t);
}

template <typename T>
__device__ __forceinline__ void ld4(const T* p, float* v) { load4(p, v); }

// pass 1: 16 lanes per (seq, head, query): lse, D = sum_j P_ij dP_ij, dq
template <typename T>
__global__ __launch_bounds__(256) void attn_rows_bwd(AttnBwdParams p) {
  const int64_t item = ((int64_t)blockIdx.x * 256 + threadIdx.x) >> 4;
  const int sub = threadIdx.x & 15, d0 = sub * 4;
  const int64_t total = p.nb * p.tin * p.heads * p.seqlen;
  if (item >= total) return;
  const int64_t i = item % p.seqlen;
  const int h = (int)((item / p.seqlen) % p.heads);
  const int64_t seq = item / (p.seqlen * p.heads), b = seq / p.tin, t = seq % p.tin;
  const T* qkv = (const T*)p.qkv;
  const T* dout = (const T*)p.dout;
  const int64_t C = p.C;
  float q[4], dO[4];
  ld4(qkv + brow(p, b, t, i) * p.ld_qkv + h * 64 + d0, q);
  ld4(dout + brow(p, b, t, i) * p.ld_dout + h * 64 + d0, dO);
  {
    const float sc = (i == 0 && p.cls_aux ? p.cls_scale : 1.0f) * (p.seq_scale ? p.seq_scale[seq] : 1.0f);
#pragma unroll
    for (int e = 0; e < 4; ++e) dO[e] *= sc;
  }
  float m = -INFINITY, l = 0.f;
  for (int64_t j = 0; j < p.seqlen; ++j) {
    float k[4];
    ld4(qkv + brow(p, b, t, j) * p.ld_qkv + C + h * 64 + d0, k);
    const float s = sum16(q[0] * k[0] + q[1] * k[1] + q[2] * k[2] + q[3] * k[3]) * p.scale;
    const float mn = fmaxf(m, s);
    l = l * expf(m - mn) + expf(s - mn);
    m = mn;
  }
  const float lse = m + logf(l);
  float D = 0.f;
  for (int64_t j = 0; j < p.seqlen; ++j) {
    float k[4], v[4];
    const T* r = qkv + brow(p, b, t, j) * p.ld_qkv + h * 64 + d0;
    ld4(r + C, k);
    ld4(r + 2 * C, v);
    const float s = sum16(q[0] * k[0] + q[1] * k[1] + q[2] * k[2] + q[3] * k[3]) * p.scale;
    const float dp = sum16(dO[0] * v[0] + dO[1] * v[1] + dO[2] * v[2] + dO[3] * v[3]);
    D += expf(s - lse) * dp;
  }
  float dq[4] = {0.f, 0.f, 0.f, 0.f};
  for (int64_t j = 0; j < p.seqlen; ++j) {
    float k[4], v[4];
    const T* r = qkv + brow(p, b, t, j) * p.ld_qkv + h * 64 + d0;
    ld4(r + C, k);
    ld4(r + 2 * C, v);
    const float s = sum16(q[0] * k[0] + q[1] * k[1] + q[2] * k[2] + q[3] * k[3]) * p.scale;
    const float dp = sum16(dO[0] * v[0] + dO[1] * v[1] + dO[2] * v[2] + dO[3] * v[3]);
    const float ds = expf(s - lse) * (dp - D);
#pragma unroll
    for (int e = 0; e < 4; ++e) dq[e] = fmaf(ds, k[e], dq[e]);
  }
  if (sub == 0) {
    p.stats[2 * item] = lse;
    p.stats[2 * item + 1] = D;
  }
#pragma unroll
  for (int e = 0; e < 4; ++e) dq[e] *= p.scale;
  if (i == 0 && p.cls_aux)
    store4(p.cls_aux + seq * 3 * C + h * 64 + d0, dq[0], dq[1], dq[2], dq[3]);
  else
    store4((T*)p.dqkv + brow(p, b, t, i) * p.ld_dqkv + h * 64 + d0, dq[0], dq[1], dq[2], dq[3]);
}

// pass 2: 16 lanes per (seq, head, key): dk, dv
template <typename T>
__global__ __launch_bounds__(256) void attn_cols_bwd(AttnBwdParams p) {
  const int64_t item = ((int64_t)blockIdx.x * 256 + threadIdx.x) >> 4;
  const int sub = threadIdx.x & 15, d0 = sub * 4;
  const int64_t total = p.nb * p.tin * p.heads * p.seqlen;
  if (item >= total) return;
  const int64_t j = item % p.seqlen;
  const int h = (int)((item / p.seqlen) % p.heads);
  const int64_t seq = item / (p.seqlen * p.heads), b = seq / p.tin, t = seq % p.tin;
  const T* qkv = (const T*)p.qkv;
  const T* dout = (const T*)p.dout;
  const int64_t C = p.C;
  float k[4], v[4];
  const T* kr = qkv + brow(p, b, t, j) * p.ld_qkv + h * 64 + d0;
  ld4(kr + C, k);
  ld4(kr + 2 * C, v);
  const float* st = p.stats + 2 * (seq * p.heads + h) * p.seqlen;
  float dk[4] = {0.f, 0.f, 0.f, 0.f}, dv[4] = {0.f, 0.f, 0.f, 0.f};
  const float ssc = p.seq_scale ? p.seq_scale[seq] : 1.0f;
  for (int64_t i = 0; i < p.seqlen; ++i) {
    float q[4], dO[4];
    ld4(qkv + brow(p, b, t, i) * p.ld_qkv + h * 64 + d0, q);
    ld4(dout + brow(p, b, t, i) * p.ld_dout + h * 64 + d0, dO);
    {
      const float sc = (i == 0 && p.cls_aux ? p.cls_scale : 1.0f) * ssc;
#pragma unroll
      for (int e = 0; e < 4; ++e) dO[e] *= sc;
    }
    const float s = sum16(q[0] * k[0] + q[1] * k[1] + q[2] * k[2] + q[3] * k[3]) * p.scale;
    const float dp = sum16(dO[0] * v[0] + dO[1] * v[1] + dO[2] * v[2] + dO[3] * v[3]);
    const float P = expf(s - st[2 * i]);
    const float ds = P * (dp - st[2 * i + 1]);
#pragma unroll
    for (int e = 0; e < 4; ++e) { dk[e] = fmaf(ds, q[e], dk[e]); dv[e] = fmaf(P, dO[e], dv[e]); }
  }
#pragma unroll
  for (int e = 0; e < 4; ++e) dk[e] *= p.scale;
  if (j == 0 && p.cls_aux) {
    float* o = p.cls_aux + seq * 3 * C + h * 64 + d0;
    store4(o + C, dk[0], dk[1], dk[2], dk[3]);
    store4(o + 2 * C, dv[0], dv[1], dv[2], dv[3]);
  } else {
    T* o = (T*)p.dqkv + brow(p, b, t, j) * p.ld_dqkv + h * 64 + d0;
    store4(o + C, dk[0], dk[1], dk[2], dk[3]);
    store4(o + 2 * C, dv[0], dv[1], dv[2], dv[3]);
  }
}

// dqkv[b*L][:] = sum_t cls_aux[b*tin + t][:]   (3C wide)
template <typename T>
__global__ __launch_bounds__(256) void cls_sum_kernel(const float* __restrict__ aux, T* __restrict__ dqkv, int tin,
                                                      int64_t L, int64_t width, int64_t ld) {
  const int64_t b = blockIdx.y;
  const int64_t c = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (c >= width) return;
  float a = 0.f;
  for (int t = 0; t < tin; ++t) a += aux[(b * tin + t) * width + c];
  dqkv[b * L * ld + c] = Elem<T>::from_f(a);
}

// ---------------------------------------------------------------- bf16 MFMA, whole sequence in LDS
// One workgroup per (sequence, head) with Q, K, V and dO of the whole sequence (<= 16*NKT rows)
// staged in LDS (bf16, 72-element rows; rows past the sequence are zero).  Same MFMA
// decomposition as the forward attn_short_bf16 (attention.hip): 16x16x32 bf16 tiles,
// ds_read_b64_tr_b16 for the transposed operands, the k-slot permutation for P-like B operands.
//   phase 1 (wave per 16-query tile): S^T = K.Q^T and dP^T = V.dO^T (lane = query, 4 keys per
//     tile), P = softmax, D = sum_k P dP, dS = P (dP - D), dQ^T = K^T.dS^T; the row statistic
//     M2 = max*c + log2(sum) and D go to LDS;
//   phase 2 (wave per 16-key tile): S = Q.K^T and dP = dO.V^T (lane = key, 4 queries per tile),
//     P = exp2(S c - M2[q]), dS = P (dP - D[q]); dV^T += dO^T.P and dK^T += Q^T.dS over 32-query
//     steps.
// Every tile loop is straight-line code (see attn_short_bf16 on MFMA result hazards under
// branches); per-lane stores are fenced.
constexpr int BKV = 72;   // bf16 per LDS row

template <int NKT, int NW>
__global__ __launch_bounds__(64 * NW, 1) void attn_bwd_short_bf16(AttnBwdParams p) {
  constexpr int NKP = (NKT + 1) / 2, SN = 2 * NKP, LP = NKP * 32;
  constexpr int NT = 64 * NW, PCS = (LP * 8 + NT - 1) / NT;
  __shared__ __attribute__((aligned(16))) bf16_t sm[4][LP * BKV];   // Q, K, V, dO
  __shared__ float m2s[LP], dds[LP];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int r16 = lane & 15, g = lane >> 4;
  const int h = blockIdx.x;
  const int64_t seq = blockIdx.y, b = seq / p.tin, t = seq % p.tin;
  const int L = (int)p.seqlen;
  const bf16_t* qkv = (const bf16_t*)p.qkv;
  const bf16_t* dout = (const bf16_t*)p.dout;
  const int64_t C = p.C;
  const float ssc = p.seq_scale ? p.seq_scale[seq] : 1.0f;
  const float sl2 = p.scale * 1.4426950408889634f;

  // ---- stage Q, K, V, dO (dO scaled by the DropPath scale and, for the CLS row, 1/T)
#pragma unroll
  for (int i = 0; i < PCS; ++i) {
    const int pc = tid + NT * i, r = pc >> 3, ch = pc & 7;
    if (r < LP) {
      uint4 vq = make_uint4(0, 0, 0, 0), vk = vq, vv = vq, vd = vq;
      if (r < L) {
        const int64_t row = brow(p, b, t, r);
        const bf16_t* src = qkv + row * p.ld_qkv + h * 64 + ch * 8;
        vq = *reinterpret_cast<const uint4*>(src);
        vk = *reinterpret_cast<const uint4*>(src + C);
        vv = *reinterpret_cast<const uint4*>(src + 2 * C);
        vd = *reinterpret_cast<const uint4*>(dout + row * p.ld_dout + h * 64 + ch * 8);
        const float sc = ssc * ((r == 0 && p.cls_aux) ? p.cls_scale : 1.0f);
        if (sc != 1.0f) {
          unsigned* u = reinterpret_cast<unsigned*>(&vd);
#pragma unroll
          for (int e = 0; e < 4; ++e) u[e] = pack_bf16x2(bf16_lo(u[e]) * sc, bf16_hi(u[e]) * sc);
        }
      }
      *reinterpret_cast<uint4*>(&sm[0][r * BKV + ch * 8]) = vq;
      *reinterpret_cast<uint4*>(&sm[1][r * BKV + ch * 8]) = vk;
      *reinterpret_cast<uint4*>(&sm[2][r * BKV + ch * 8]) = vv;
      *reinterpret_cast<uint4*>(&sm[3][r * BKV + ch * 8]) = vd;
    }
  }
  __syncthreads();
  const bf16_t* Qs = sm[0];
  const bf16_t* Ks = sm[1];
  const bf16_t* Vs = sm[2];
  const bf16_t* Ds = sm[3];
  const int nkt = (L + 15) >> 4;
  typedef __attribute__((address_space(3))) sv4* LDS4;

  // ================= phase 1: dQ, row statistics
  for (int qt = wave; qt < nkt; qt += NW) {
    const bf16_t* qr = Qs + (qt * 16 + r16) * BKV + g * 8;
    const bf16_t* dr = Ds + (qt * 16 + r16) * BKV + g * 8;
    const sv8 qf0 = *reinterpret_cast<const sv8*>(qr), qf1 = *reinterpret_cast<const sv8*>(qr + 32);
    const sv8 df0 = *reinterpret_cast<const sv8*>(dr), df1 = *reinterpret_cast<const sv8*>(dr + 32);
    fv4 s[SN], dp[SN];
#pragma unroll
    for (int kt = 0; kt < SN; ++kt) {
      const bf16_t* kr = Ks + (kt * 16 + r16) * BKV + g * 8;
      const bf16_t* vr = Vs + (kt * 16 + r16) * BKV + g * 8;
      fv4 z = fv4{0.f, 0.f, 0.f, 0.f};
      z = __builtin_amdgcn_mfma_f32_16x16x32_bf16(*reinterpret_cast<const sv8*>(kr), qf0, z, 0, 0, 0);
      s[kt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(*reinterpret_cast<const sv8*>(kr + 32), qf1, z, 0, 0, 0);
      fv4 y = fv4{0.f, 0.f, 0.f, 0.f};
      y = __builtin_amdgcn_mfma_f32_16x16x32_bf16(*reinterpret_cast<const sv8*>(vr), df0, y, 0, 0, 0);
      dp[kt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(*reinterpret_cast<const sv8*>(vr + 32), df1, y, 0, 0, 0);
    }
    float mx = -INFINITY;
#pragma unroll
    for (int kt = 0; kt < SN; ++kt) {
#pragma unroll
      for (int j = 0; j < 4; ++j) s[kt][j] = (kt * 16 + 4 * g + j < L) ? s[kt][j] : -INFINITY;
      mx = fmaxf(mx, fmaxf(fmaxf(s[kt][0], s[kt][1]), fmaxf(s[kt][2], s[kt][3])));
    }
    mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
    mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
    const float mxs = mx * sl2;
    float rs = 0.f;
#pragma unroll
    for (int kt = 0; kt < SN; ++kt)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        s[kt][j] = __builtin_amdgcn_exp2f(fmaf(s[kt][j], sl2, -mxs));
        rs += s[kt][j];
      }
    rs += __shfl_xor(rs, 16, 64);
    rs += __shfl_xor(rs, 32, 64);
    const float inv = 1.0f / rs;
    float D = 0.f;
#pragma unroll
    for (int kt = 0; kt < SN; ++kt)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        s[kt][j] *= inv;                    // P
        D = fmaf(s[kt][j], dp[kt][j], D);
      }
    D += __shfl_xor(D, 16, 64);
    D += __shfl_xor(D, 32, 64);
    // dQ^T = K^T . dS^T (K^T fragments by transposed LDS reads; dS in the P.V k-slot order)
    fv4 dq[4];
#pragma unroll
    for (int d = 0; d < 4; ++d) dq[d] = fv4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kp = 0; kp < NKP; ++kp) {
      sv8 pb;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        pb[j] = (short)f2bf(s[2 * kp][j] * (dp[2 * kp][j] - D));
        pb[4 + j] = (short)f2bf(s[2 * kp + 1][j] * (dp[2 * kp + 1][j] - D));
      }
      const int kr0 = kp * 32 + 4 * g + (r16 >> 2), kr1 = kr0 + 16;
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) {
        const int col = dt * 16 + 4 * (r16 & 3);
        const sv4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS4)(Ks + kr0 * BKV + col));
        const sv4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS4)(Ks + kr1 * BKV + col));
        dq[dt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7),
                                                         pb, dq[dt], 0, 0, 0);
      }
    }
    mfma_result_fence();
    const int qo = qt * 16 + r16;
    if (g == 0) {
      m2s[qo] = qo < L ? mxs + __log2f(rs) : INFINITY;
      dds[qo] = qo < L ? D : 0.f;
    }
    if (qo < L) {
      if (qo == 0 && p.cls_aux) {
        float* dst = p.cls_aux + seq * 3 * C + h * 64 + 4 * g;
#pragma unroll
        for (int dt = 0; dt < 4; ++dt)
          store4(dst + dt * 16, dq[dt][0] * p.scale, dq[dt][1] * p.scale, dq[dt][2] * p.scale, dq[dt][3] * p.scale);
      } else {
        bf16_t* dst = (bf16_t*)p.dqkv + brow(p, b, t, qo) * p.ld_dqkv + h * 64 + 4 * g;
#pragma unroll
        for (int dt = 0; dt < 4; ++dt)
          store4(dst + dt * 16, dq[dt][0] * p.scale, dq[dt][1] * p.scale, dq[dt][2] * p.scale, dq[dt][3] * p.scale);
      }
    }
  }
  // query rows of tiles past the sequence (whole 32-row PV steps): P = 0
  for (int q = nkt * 16 + tid; q < LP; q += NT) { m2s[q] = INFINITY; dds[q] = 0.f; }
  __syncthreads();

  // ================= phase 2: dK, dV
  for (int kt = wave; kt < nkt; kt += NW) {
    const bf16_t* kr = Ks + (kt * 16 + r16) * BKV + g * 8;
    const bf16_t* vr = Vs + (kt * 16 + r16) * BKV + g * 8;
    const sv8 kf0 = *reinterpret_cast<const sv8*>(kr), kf1 = *reinterpret_cast<const sv8*>(kr + 32);
    const sv8 vf0 = *reinterpret_cast<const sv8*>(vr), vf1 = *reinterpret_cast<const sv8*>(vr + 32);
    fv4 dk[4], dv[4];
#pragma unroll
    for (int d = 0; d < 4; ++d) { dk[d] = fv4{0.f, 0.f, 0.f, 0.f}; dv[d] = dk[d]; }
#pragma unroll
    for (int qp = 0; qp < NKP; ++qp) {
      fv4 P[2], dS[2];
#pragma unroll
      for (int hq = 0; hq < 2; ++hq) {
        const int q0 = (2 * qp + hq) * 16;
        const bf16_t* qr = Qs + (q0 + r16) * BKV + g * 8;
        const bf16_t* dr = Ds + (q0 + r16) * BKV + g * 8;
        fv4 z = fv4{0.f, 0.f, 0.f, 0.f};
        z = __builtin_amdgcn_mfma_f32_16x16x32_bf16(*reinterpret_cast<const sv8*>(qr), kf0, z, 0, 0, 0);
        const fv4 sc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(*reinterpret_cast<const sv8*>(qr + 32), kf1, z, 0, 0, 0);
        fv4 y = fv4{0.f, 0.f, 0.f, 0.f};
        y = __builtin_amdgcn_mfma_f32_16x16x32_bf16(*reinterpret_cast<const sv8*>(dr), vf0, y, 0, 0, 0);
        const fv4 dpv = __builtin_amdgcn_mfma_f32_16x16x32_bf16(*reinterpret_cast<const sv8*>(dr + 32), vf1, y, 0, 0, 0);
        // lane (key r16) holds queries q0 + 4g + j
        const float4 m2 = *reinterpret_cast<const float4*>(&m2s[q0 + 4 * g]);
        const float4 dd = *reinterpret_cast<const float4*>(&dds[q0 + 4 * g]);
        const float mm[4] = {m2.x, m2.y, m2.z, m2.w}, D4[4] = {dd.x, dd.y, dd.z, dd.w};
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          P[hq][j] = __builtin_amdgcn_exp2f(fmaf(sc[j], sl2, -mm[j]));
          dS[hq][j] = P[hq][j] * (dpv[j] - D4[j]);
        }
      }
      sv8 pb, sb;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        pb[j] = (short)f2bf(P[0][j]);
        pb[4 + j] = (short)f2bf(P[1][j]);
        sb[j] = (short)f2bf(dS[0][j]);
        sb[4 + j] = (short)f2bf(dS[1][j]);
      }
      const int qr0 = qp * 32 + 4 * g + (r16 >> 2), qr1 = qr0 + 16;
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) {
        const int col = dt * 16 + 4 * (r16 & 3);
        const sv4 dlo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS4)(Ds + qr0 * BKV + col));
        const sv4 dhi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS4)(Ds + qr1 * BKV + col));
        dv[dt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_shufflevector(dlo, dhi, 0, 1, 2, 3, 4, 5, 6, 7),
                                                         pb, dv[dt], 0, 0, 0);
        const sv4 qlo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS4)(Qs + qr0 * BKV + col));
        const sv4 qhi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS4)(Qs + qr1 * BKV + col));
        dk[dt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_shufflevector(qlo, qhi, 0, 1, 2, 3, 4, 5, 6, 7),
                                                         sb, dk[dt], 0, 0, 0);
      }
    }
    mfma_result_fence();
    const int ko = kt * 16 + r16;
    if (ko < L) {
      if (ko == 0 && p.cls_aux) {
        float* dst = p.cls_aux + seq * 3 * C + h * 64 + 4 * g;
#pragma unroll
        for (int dt = 0; dt < 4; ++dt) {
          store4(dst + C + dt * 16, dk[dt][0] * p.scale, dk[dt][1] * p.scale, dk[dt][2] * p.scale, dk[dt][3] * p.scale);
          store4(dst + 2 * C + dt * 16, dv[dt][0], dv[dt][1], dv[dt][2], dv[dt][3]);
        }
      } else {
        bf16_t* dst = (bf16_t*)p.dqkv + brow(p, b, t, ko) * p.ld_dqkv + h * 64 + 4 * g;
#pragma unroll
        for (int dt = 0; dt < 4; ++dt) {
          store4(dst + C + dt * 16, dk[dt][0] * p.scale, dk[dt][1] * p.scale, dk[dt][2] * p.scale, dk[dt][3] * p.scale);
          store4(dst + 2 * C + dt * 16, dv[dt][0], dv[dt][1], dv[dt][2], dv[dt][3]);
        }
      }
    }
  }
}

// The same math with HALF the LDS (variant 2): phase 1 keeps only K and V of the whole sequence in
// LDS (each wave's Q / dO tile comes straight from global memory in MFMA fragment layout), phase 2
// only Q and dO (K / V tiles from global), restaged in between -- 66 KB instead of 130, so two
// 4-wave workgroups share a CU and one's staging runs under the other's MFMAs.  Alone 152.5 vs
// 158.0 us at the train step's global shape (tools/attn_bwd_bench.py); in the step 141.2 / 141.1
// vs 142.2 / 141.8 clips/s (DSVT_ATTN_BWD_SPLIT=1): selectable (variant 2), off by default.
template <int NKT, int NW>
__global__ __launch_bounds__(64 * NW, 2) void attn_bwd_split_bf16(AttnBwdParams p) {
  constexpr int NKP = (NKT + 1) / 2, SN = 2 * NKP, LP = NKP * 32;
  constexpr int NT = 64 * NW, PCS = (LP * 8 + NT - 1) / NT;
  __shared__ __attribute__((aligned(16))) bf16_t sm[2][LP * BKV];   // phase 1: K, V; phase 2: Q, dO
  __shared__ float m2s[LP], dds[LP];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int r16 = lane & 15, g = lane >> 4;
  const int h = blockIdx.x;
  const int64_t seq = blockIdx.y, b = seq / p.tin, t = seq % p.tin;
  const int L = (int)p.seqlen;
  const bf16_t* qkv = (const bf16_t*)p.qkv;
  const bf16_t* dout = (const bf16_t*)p.dout;
  const int64_t C = p.C;
  const float ssc = p.seq_scale ? p.seq_scale[seq] : 1.0f;
  const float sl2 = p.scale * 1.4426950408889634f;
  auto dscale = [&](int r) { return ssc * ((r == 0 && p.cls_aux) ? p.cls_scale : 1.0f); };
  auto scale8 = [&](uint4& v, float sc) {
    unsigned* u = reinterpret_cast<unsigned*>(&v);
#pragma unroll
    for (int e = 0; e < 4; ++e) u[e] = pack_bf16x2(bf16_lo(u[e]) * sc, bf16_hi(u[e]) * sc);
  };
  // two tensors of the whole sequence into sm[0] / sm[1]: K, V (qd = false) or Q, scaled dO
  auto stage2 = [&](bool qd) {
#pragma unroll
    for (int i = 0; i < PCS; ++i) {
      const int pc = tid + NT * i, r = pc >> 3, ch = pc & 7;
      if (r < LP) {
        uint4 va = make_uint4(0, 0, 0, 0), vb = va;
        if (r < L) {
          const int64_t row = brow(p, b, t, r);
          const bf16_t* src = qkv + row * p.ld_qkv + h * 64 + ch * 8;
          if (qd) {
            va = *reinterpret_cast<const uint4*>(src);
            vb = *reinterpret_cast<const uint4*>(dout + row * p.ld_dout + h * 64 + ch * 8);
            const float sc = dscale(r);
            if (sc != 1.0f) scale8(vb, sc);
          } else {
            va = *reinterpret_cast<const uint4*>(src + C);
            vb = *reinterpret_cast<const uint4*>(src + 2 * C);
          }
        }
        *reinterpret_cast<uint4*>(&sm[0][r * BKV + ch * 8]) = va;
        *reinterpret_cast<uint4*>(&sm[1][r * BKV + ch * 8]) = vb;
      }
    }
  };
  // one 16-row tile's MFMA fragments (row r16 of the tile, columns 8g.. and 32 + 8g..) from global
  auto frag_g = [&](const bf16_t* base, int64_t ld, int64_t off, int row, bool sc_d, sv8& f0, sv8& f1) {
    uint4 a = make_uint4(0, 0, 0, 0), c = a;
    if (row < L) {
      const bf16_t* src = base + brow(p, b, t, row) * ld + off + g * 8;
      a = *reinterpret_cast<const uint4*>(src);
      c = *reinterpret_cast<const uint4*>(src + 32);
      if (sc_d) {
        const float sc = dscale(row);
        if (sc != 1.0f) { scale8(a, sc); scale8(c, sc); }
      }
    }
    f0 = __builtin_bit_cast(sv8, a);
    f1 = __builtin_bit_cast(sv8, c);
  };
  const int nkt = (L + 15) >> 4;
  typedef __attribute__((address_space(3))) sv4* LDS4;

  stage2(false);
  __syncthreads();
  {
    const bf16_t* Ks = sm[0];
    const bf16_t* Vs = sm[1];
    // ================= phase 1: dQ, row statistics
    for (int qt = wave; qt < nkt; qt += NW) {
      sv8 qf0, qf1, df0, df1;
      frag_g(qkv, p.ld_qkv, h * 64, qt * 16 + r16, false, qf0, qf1);
      frag_g(dout, p.ld_dout, h * 64, qt * 16 + r16, true, df0, df1);
      fv4 s[SN], dp[SN];
#pragma unroll
      for (int kt = 0; kt < SN; ++kt) {
        const bf16_t* kr = Ks + (kt * 16 + r16) * BKV + g * 8;
        const bf16_t* vr = Vs + (kt * 16 + r16) * BKV + g * 8;
        fv4 z = fv4{0.f, 0.f, 0.f, 0.f};
        z = __builtin_amdgcn_mfma_f32_16x16x32_bf16(*reinterpret_cast<const sv8*>(kr), qf0, z, 0, 0, 0);
        s[kt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(*reinterpret_cast<const sv8*>(kr + 32), qf1, z, 0, 0, 0);
        fv4 y = fv4{0.f, 0.f, 0.f, 0.f};
        y = __builtin_amdgcn_mfma_f32_16x16x32_bf16(*reinterpret_cast<const sv8*>(vr), df0, y, 0, 0, 0);
        dp[kt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(*reinterpret_cast<const sv8*>(vr + 32), df1, y, 0, 0, 0);
      }
      float mx = -INFINITY;
#pragma unroll
      for (int kt = 0; kt < SN; ++kt) {
#pragma unroll
        for (int j = 0; j < 4; ++j) s[kt][j] = (kt * 16 + 4 * g + j < L) ? s[kt][j] : -INFINITY;
        mx = fmaxf(mx, fmaxf(fmaxf(s[kt][0], s[kt][1]), fmaxf(s[kt][2], s[kt][3])));
      }
      mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
      mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
      const float mxs = mx * sl2;
      float rs = 0.f;
#pragma unroll
      for (int kt = 0; kt < SN; ++kt)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          s[kt][j] = __builtin_amdgcn_exp2f(fmaf(s[kt][j], sl2, -mxs));
          rs += s[kt][j];
        }
      rs += __shfl_xor(rs, 16, 64);
      rs += __shfl_xor(rs, 32, 64);
      const float inv = 1.0f / rs;
      float D = 0.f;
#pragma unroll
      for (int kt = 0; kt < SN; ++kt)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          s[kt][j] *= inv;
          D = fmaf(s[kt][j], dp[kt][j], D);
        }
      D += __shfl_xor(D, 16, 64);
      D += __shfl_xor(D, 32, 64);
      fv4 dq[4];
#pragma unroll
      for (int d = 0; d < 4; ++d) dq[d] = fv4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kp = 0; kp < NKP; ++kp) {
        sv8 pb;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          pb[j] = (short)f2bf(s[2 * kp][j] * (dp[2 * kp][j] - D));
          pb[4 + j] = (short)f2bf(s[2 * kp + 1][j] * (dp[2 * kp + 1][j] - D));
        }
        const int kr0 = kp * 32 + 4 * g + (r16 >> 2), kr1 = kr0 + 16;
#pragma unroll
        for (int dt = 0; dt < 4; ++dt) {
          const int col = dt * 16 + 4 * (r16 & 3);
          const sv4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS4)(Ks + kr0 * BKV + col));
          const sv4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS4)(Ks + kr1 * BKV + col));
          dq[dt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7),
                                                           pb, dq[dt], 0, 0, 0);
        }
      }
      mfma_result_fence();
      const int qo = qt * 16 + r16;
      if (g == 0) {
        m2s[qo] = qo < L ? mxs + __log2f(rs) : INFINITY;
        dds[qo] = qo < L ? D : 0.f;
      }
      if (qo < L) {
        if (qo == 0 && p.cls_aux) {
          float* dst = p.cls_aux + seq * 3 * C + h * 64 + 4 * g;
#pragma unroll
          for (int dt = 0; dt < 4; ++dt)
            store4(dst + dt * 16, dq[dt][0] * p.scale, dq[dt][1] * p.scale, dq[dt][2] * p.scale, dq[dt][3] * p.scale);
        } else {
          bf16_t* dst = (bf16_t*)p.dqkv + brow(p, b, t, qo) * p.ld_dqkv + h * 64 + 4 * g;
#pragma unroll
          for (int dt = 0; dt < 4; ++dt)
            store4(dst + dt * 16, dq[dt][0] * p.scale, dq[dt][1] * p.scale, dq[dt][2] * p.scale, dq[dt][3] * p.scale);
        }
      }
    }
  }
  for (int q = nkt * 16 + tid; q < LP; q += NT) { m2s[q] = INFINITY; dds[q] = 0.f; }
  __syncthreads();                       // every phase-1 read of K, V done; statistics visible
  stage2(true);
  __syncthreads();
  const bf16_t* Qs = sm[0];
  const bf16_t* Ds = sm[1];
  // ================= phase 2: dK, dV
  for (int kt = wave; kt < nkt; kt += NW) {
    sv8 kf0, kf1, vf0, vf1;
    frag_g(qkv, p.ld_qkv, C + h * 64, kt * 16 + r16, false, kf0, kf1);
    frag_g(qkv, p.ld_qkv, 2 * C + h * 64, kt * 16 + r16, false, vf0, vf1);
    fv4 dk[4], dv[4];
#pragma unroll
    for (int d = 0; d < 4; ++d) { dk[d] = fv4{0.f, 0.f, 0.f, 0.f}; dv[d] = dk[d]; }
#pragma unroll
    for (int qp = 0; qp < NKP; ++qp) {
      fv4 P[2], dS[2];
#pragma unroll
      for (int hq = 0; hq < 2; ++hq) {
        const int q0 = (2 * qp + hq) * 16;
        const bf16_t* qr = Qs + (q0 + r16) * BKV + g * 8;
        const bf16_t* dr = Ds + (q0 + r16) * BKV + g * 8;
        fv4 z = fv4{0.f, 0.f, 0.f, 0.f};
        z = __builtin_amdgcn_mfma_f32_16x16x32_bf16(*reinterpret_cast<const sv8*>(qr), kf0, z, 0, 0, 0);
        const fv4 sc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(*reinterpret_cast<const sv8*>(qr + 32), kf1, z, 0, 0, 0);
        fv4 y = fv4{0.f, 0.f, 0.f, 0.f};
        y = __builtin_amdgcn_mfma_f32_16x16x32_bf16(*reinterpret_cast<const sv8*>(dr), vf0, y, 0, 0, 0);
        const fv4 dpv = __builtin_amdgcn_mfma_f32_16x16x32_bf16(*reinterpret_cast<const sv8*>(dr + 32), vf1, y, 0, 0, 0);
        const float4 m2 = *reinterpret_cast<const float4*>(&m2s[q0 + 4 * g]);
        const float4 dd = *reinterpret_cast<const float4*>(&dds[q0 + 4 * g]);
        const float mm[4] = {m2.x, m2.y, m2.z, m2.w}, D4[4] = {dd.x, dd.y, dd.z, dd.w};
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          P[hq][j] = __builtin_amdgcn_exp2f(fmaf(sc[j], sl2, -mm[j]));
          dS[hq][j] = P[hq][j] * (dpv[j] - D4[j]);
        }
      }
      sv8 pb, sb;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        pb[j] = (short)f2bf(P[0][j]);
        pb[4 + j] = (short)f2bf(P[1][j]);
        sb[j] = (short)f2bf(dS[0][j]);
        sb[4 + j] = (short)f2bf(dS[1][j]);
      }
      const int qr0 = qp * 32 + 4 * g + (r16 >> 2), qr1 = qr0 + 16;
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) {
        const int col = dt * 16 + 4 * (r16 & 3);
        const sv4 dlo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS4)(Ds + qr0 * BKV + col));
        const sv4 dhi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS4)(Ds + qr1 * BKV + col));
        dv[dt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_shufflevector(dlo, dhi, 0, 1, 2, 3, 4, 5, 6, 7),
                                                         pb, dv[dt], 0, 0, 0);
        const sv4 qlo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS4)(Qs + qr0 * BKV + col));
        const sv4 qhi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS4)(Qs + qr1 * BKV + col));
        dk[dt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_shufflevector(qlo, qhi, 0, 1, 2, 3, 4, 5, 6, 7),
                                                         sb, dk[dt], 0, 0, 0);
      }
    }
    mfma_result_fence();
    const int ko = kt * 16 + r16;
    if (ko < L) {
      if (ko == 0 && p.cls_aux) {
        float* dst = p.cls_aux + seq * 3 * C + h * 64 + 4 * g;
#pragma unroll
        for (int dt = 0; dt < 4; ++dt) {
          store4(dst + C + dt * 16, dk[dt][0] * p.scale, dk[dt][1] * p.scale, dk[dt][2] * p.scale, dk[dt][3] * p.scale);
          store4(dst + 2 * C + dt * 16, dv[dt][0], dv[dt][1], dv[dt][2], dv[dt][3]);
        }
      } else {
        bf16_t* dst = (bf16_t*)p.dqkv + brow(p, b, t, ko) * p.ld_dqkv + h * 64 + 4 * g;
#pragma unroll
        for (int dt = 0; dt < 4; ++dt) {
          store4(dst + C + dt * 16, dk[dt][0] * p.scale, dk[dt][1] * p.scale, dk[dt][2] * p.scale, dk[dt][3] * p.scale);
          store4(dst + 2 * C + dt * 16, dv[dt][0], dv[dt][1], dv[dt][2], dv[dt][3]);
        }
      }
    }
  }
}

void set_attn_bwd_variant(int v) { g_attn_bwd_variant = v; }

hipError_t launch_attn_bwd_generic(int dtype, const AttnBwdParams& p, hipStream_t s) {
  const int64_t items = p.nb * p.tin * p.heads * p.seqlen;
  const unsigned blocks = (unsigned)((items * 16 + 255) / 256);
  static const int split_env = getenv("DSVT_ATTN_BWD_SPLIT") ? atoi(getenv("DSVT_ATTN_BWD_SPLIT")) : 0;
  const bool split = g_attn_bwd_variant == 2 || (g_attn_bwd_variant == 0 && split_env);
  if (dtype == 0 && p.seqlen > 64 && p.seqlen <= 208 && split) {
    dim3 grid((unsigned)p.heads, (unsigned)(p.nb * p.tin));
    attn_bwd_split_bf16<13, 4><<<grid, 256, 0, s>>>(p);
  } else if (dtype == 0 && p.seqlen <= 256 && (g_attn_bwd_variant == 0 || g_attn_bwd_variant == 2)) {
    dim3 grid((unsigned)p.heads, (unsigned)(p.nb * p.tin));
    if (p.seqlen <= 64) attn_bwd_short_bf16<4, 4><<<grid, 256, 0, s>>>(p);
    else if (p.seqlen <= 208) attn_bwd_short_bf16<13, 8><<<grid, 512, 0, s>>>(p);
    else attn_bwd_short_bf16<16, 8><<<grid, 512, 0, s>>>(p);
  } else if (dtype == 0) {
    attn_rows_bwd<bf16_t><<<blocks, 256, 0, s>>>(p);
    attn_cols_bwd<bf16_t><<<blocks, 256, 0, s>>>(p);
  } else {
    attn_rows_bwd<float><<<blocks, 256, 0, s>>>(p);
    attn_cols_bwd<float><<<blocks, 256, 0, s>>>(p);
  }
  if (hipError_t e = hipGetLastError()) return e;
  if (p.cls_aux) {
    dim3 grid((unsigned)((3 * p.C + 255) / 256), (unsigned)p.nb);
    if (dtype == 0)
      cls_sum_kernel<bf16_t><<<grid, 256, 0, s>>>(p.cls_aux, (bf16_t*)p.dqkv, (int)p.tin, p.L, 3 * p.C, p.ld_dqkv);
    else
      cls_sum_kernel<float><<<grid, 256, 0, s>>>(p.cls_aux, (float*)p.dqkv, (int)p.tin, p.L, 3 * p.C, p.ld_dqkv);
  }
  return hipGetLastError();
}

// ================================================================ DINO loss backward
// d loss / d s[v*B + b][j] = coef * (n_v * softmax(s/ts)[j] - sum_{iq != v, iq < gc} q_iq[b][j])
// with q = softmax((t - center)/tt) (teacher, detached), coef = dloss / (npairs * B * ts),
// n_v = #global crops other than v (train_ssl.py:653-669).  One block per student row; the row
// statistics (max, sum of exp) are passed in (softmax_stats_kernel of the forward).
__global__ __launch_bounds__(256) void dino_loss_bwd_kernel(const float* __restrict__ student,
                                                            const float* __restrict__ teacher,
                                                            const float* __restrict__ center, int64_t B, int64_t gc,
                                                            int64_t D, float inv_ts, float inv_tt,
                                                            const float* __restrict__ t_m, const float* __restrict__ t_z,
                                                            const float* __restrict__ s_m, const float* __restrict__ s_z,
                                                            const float* __restrict__ dloss, float coef,
                                                            float* __restrict__ grad) {
  const int64_t row = blockIdx.x;           // student row v*B + b
  const int64_t v = row / B, b = row % B;
  const float g = coef * dloss[0];
  const float sm = s_m[row], sz = 1.0f / s_z[row];
  int nv = 0;
  for (int64_t iq = 0; iq < gc; ++iq) nv += (iq != v);
  for (int64_t j = (int64_t)threadIdx.x * 4; j < D; j += 1024) {
    const float4 sv = *reinterpret_cast<const float4*>(student + row * D + j);
    const float4 cv = center ? *reinterpret_cast<const float4*>(center + j) : make_float4(0.f, 0.f, 0.f, 0.f);
    float a[4] = {nv * expf(sv.x * inv_ts - sm) * sz, nv * expf(sv.y * inv_ts - sm) * sz,
                  nv * expf(sv.z * inv_ts - sm) * sz, nv * expf(sv.w * inv_ts - sm) * sz};
    for (int64_t iq = 0; iq < gc; ++iq) {
      if (iq == v) continue;
      const int64_t tr = iq * B + b;
      const float4 tv = *reinterpret_cast<const float4*>(teacher + tr * D + j);
      const float tm = t_m[tr], tz = 1.0f / t_z[tr];
      a[0] -= expf((tv.x - cv.x) * inv_tt - tm) * tz;
      a[1] -= expf((tv.y - cv.y) * inv_tt - tm) * tz;
      a[2] -= expf((tv.z - cv.z) * inv_tt - tm) * tz;
      a[3] -= expf((tv.w - cv.w) * inv_tt - tm) * tz;
    }
    *reinterpret_cast<float4*>(grad + row * D + j) = make_float4(g * a[0], g * a[1], g * a[2], g * a[3]);
  }
}

hipError_t launch_dino_loss_bwd(const float* student, const float* teacher, const float* center, int64_t B,
                                int64_t ncrops, int64_t gc, int64_t D, float inv_ts, float inv_tt, const float* t_m,
                                const float* t_z, const float* s_m, const float* s_z, const float* dloss, float coef,
                                float* grad, hipStream_t s) {
  dino_loss_bwd_kernel<<<(unsigned)(ncrops * B), 256, 0, s>>>(student, teacher, center, B, gc, D, inv_ts, inv_tt, t_m,
                                                              t_z, s_m, s_z, dloss, coef, grad);
  return hipGetLastError();
}

// ================================================================ F.normalize / weight-norm backward
// z = x / max(||x||, eps):  dx = (dz - z (z.dz)) / ||x||   (||x|| > eps),  dz / eps otherwise
__global__ __launch_bounds__(256) void l2norm_bwd_kernel(const float* __restrict__ x, const float* __restrict__ dz,
                                                         float* __restrict__ dx, int64_t rows, int D, float eps) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int64_t r = (int64_t)blockIdx.x * 4 + wave;
  if (r >= rows) return;
  const float* xr = x + r * D;
  const float* gr = dz + r * D;
  float ss = 0.f, xd = 0.f;
  for (int c = lane; c < D; c += 64) { ss += xr[c] * xr[c]; xd += xr[c] * gr[c]; }
  ss = wave_sum(ss);
  xd = wave_sum(xd);
  const float nrm = sqrtf(ss);
  if (nrm > eps) {
    const float inv = 1.0f / nrm, k = xd * inv * inv * inv;
    for (int c = lane; c < D; c += 64) dx[r * D + c] = gr[c] * inv - xr[c] * k;
  } else {
    for (int c = lane; c < D; c += 64) dx[r * D + c] = gr[c] / eps;
  }
}

// w = g v / ||v|| per row: dv = (g/||v||)(dW - w_hat (w_hat.dW)), dg = w_hat.dW (accumulated)
__global__ __launch_bounds__(256) void weightnorm_bwd_kernel(const float* __restrict__ v, const float* __restrict__ g,
                                                             const float* __restrict__ dw, float* __restrict__ dv,
                                                             float* __restrict__ dg, int64_t rows, int D,
                                                             int accumulate) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int64_t r = (int64_t)blockIdx.x * 4 + wave;
  if (r >= rows) return;
  const float* vr = v + r * D;
  const float* gr = dw + r * D;
  float ss = 0.f, vd = 0.f;
  for (int c = lane; c < D; c += 64) { ss += vr[c] * vr[c]; vd += vr[c] * gr[c]; }
  ss = wave_sum(ss);
  vd = wave_sum(vd);
  const float nrm = sqrtf(ss), inv = 1.0f / nrm;
  const float gg = g[r], dot = vd * inv;   // w_hat . dW
  for (int c = lane; c < D; c += 64) {
    const float val = gg * inv * (gr[c] - vr[c] * inv * dot);
    dv[r * D + c] = accumulate ? dv[r * D + c] + val : val;
  }
  if (dg && lane == 0) dg[r] = accumulate ? dg[r] + dot : dot;
}

hipError_t launch_l2norm_bwd(const float* x, const float* dz, float* dx, int64_t rows, int64_t D, float eps,
                             hipStream_t s) {
  l2norm_bwd_kernel<<<(unsigned)((rows + 3) / 4), 256, 0, s>>>(x, dz, dx, rows, (int)D, eps);
  return hipGetLastError();
}

hipError_t launch_weightnorm_bwd(const float* v, const float* g, const float* dw, float* dv, float* dg, int64_t rows,
                                 int64_t D, int accumulate, hipStream_t s) {
  weightnorm_bwd_kernel<<<(unsigned)((rows + 3) / 4), 256, 0, s>>>(v, g, dw, dv, dg, rows, (int)D, accumulate);
  return hipGetLastError();
}

// ================================================================ layout helpers
// y[m] = cast(x[row(m)]) for compact rows m < rows (C % 4 == 0)
// y[m] = cast(x[row(m)] * row_scale[m / group]) (row_scale nullable)
template <typename OutT>
__global__ __launch_bounds__(256) void cast_rows_kernel(const float* __restrict__ x, OutT* __restrict__ y,
                                                        int64_t rows, int64_t C, int64_t rpg, int64_t gstride,
                                                        int64_t goff, const float* __restrict__ row_scale,
                                                        int64_t group) {
  const int64_t c4 = C / 4, total = rows * c4;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < total; i += (int64_t)gridDim.x * 256) {
    const int64_t m = i / c4, c = (i % c4) * 4;
    const float4 f = *reinterpret_cast<const float4*>(x + map_row(m, rpg, gstride, goff) * C + c);
    const float sc = row_scale ? row_scale[m / group] : 1.0f;
    store4(y + m * C + c, f.x * sc, f.y * sc, f.z * sc, f.w * sc);
  }
}

static unsigned grid_for(int64_t work) {
  int64_t blocks = (work + 255) / 256;
  if (blocks > 16384) blocks = 16384;
  return (unsigned)(blocks < 1 ? 1 : blocks);
}

hipError_t launch_cast_rows(int dtype, const float* x, void* y, int64_t rows, int64_t C, int64_t rpg, int64_t gstride,
                            int64_t goff, const float* row_scale, int64_t group, hipStream_t s) {
  const unsigned blocks = grid_for(rows * C / 4);
  if (dtype == 0)
    cast_rows_kernel<bf16_t><<<blocks, 256, 0, s>>>(x, (bf16_t*)y, rows, C, rpg, gstride, goff, row_scale, group);
  else
    cast_rows_kernel<float><<<blocks, 256, 0, s>>>(x, (float*)y, rows, C, rpg, gstride, goff, row_scale, group);
  return hipGetLastError();
}

// in place: y[m][c] *= row_scale[m / group]  (DropPath of a compact branch activation)
template <typename T>
__global__ __launch_bounds__(256) void row_scale_kernel(T* __restrict__ y, int64_t rows, int64_t C, int64_t ld,
                                                        const float* __restrict__ row_scale, int64_t group) {
  const int64_t c4 = C / 4, total = rows * c4;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < total; i += (int64_t)gridDim.x * 256) {
    const int64_t m = i / c4, c = (i % c4) * 4;
    float v[4];
    load4(y + m * ld + c, v);
    const float sc = row_scale[m / group];
    store4(y + m * ld + c, v[0] * sc, v[1] * sc, v[2] * sc, v[3] * sc);
  }
}

hipError_t launch_row_scale(int dtype, void* y, int64_t rows, int64_t C, int64_t ld, const float* row_scale,
                            int64_t group, hipStream_t s) {
  const unsigned blocks = grid_for(rows * C / 4);
  if (dtype == 0) row_scale_kernel<bf16_t><<<blocks, 256, 0, s>>>((bf16_t*)y, rows, C, ld, row_scale, group);
  else row_scale_kernel<float><<<blocks, 256, 0, s>>>((float*)y, rows, C, ld, row_scale, group);
  return hipGetLastError();
}

// X[m][c] += row_scale[m] * bias[c]  (the DropPath-scaled bias of a residual branch)
__global__ __launch_bounds__(256) void rowscale_bias_kernel(float* __restrict__ X, int64_t rows, int64_t C,
                                                            const float* __restrict__ row_scale,
                                                            const float* __restrict__ bias) {
  const int64_t c4 = C / 4, total = rows * c4;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < total; i += (int64_t)gridDim.x * 256) {
    const int64_t m = i / c4, c = (i % c4) * 4;
    const float sc = row_scale[m];
    float4 x = *reinterpret_cast<float4*>(X + m * C + c);
    const float4 b = *reinterpret_cast<const float4*>(bias + c);
    x.x += sc * b.x; x.y += sc * b.y; x.z += sc * b.z; x.w += sc * b.w;
    *reinterpret_cast<float4*>(X + m * C + c) = x;
  }
}

hipError_t launch_rowscale_bias_add(float* X, int64_t rows, int64_t C, const float* row_scale, const float* bias,
                                    hipStream_t s) {
  rowscale_bias_kernel<<<grid_for(rows * C / 4), 256, 0, s>>>(X, rows, C, row_scale, bias);
  return hipGetLastError();
}

// y[c][r] = cast(x[r][c]), x [R, C] fp32: 64x64 tiles through LDS (coalesced both ways)
template <typename OutT>
__global__ __launch_bounds__(256) void cast_transpose_kernel(const float* __restrict__ x, OutT* __restrict__ y,
                                                             int64_t R, int64_t C) {
  __shared__ float tile[64][65];
  const int64_t r0 = (int64_t)blockIdx.y * 64, c0 = (int64_t)blockIdx.x * 64;
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  for (int i = ty; i < 64; i += 4) {
    const int64_t r = r0 + i, c = c0 + tx;
    tile[i][tx] = (r < R && c < C) ? x[r * C + c] : 0.f;
  }
  __syncthreads();
  for (int i = ty; i < 64; i += 4) {
    const int64_t c = c0 + i, r = r0 + tx;
    if (c < C && r < R) y[c * R + r] = Elem<OutT>::from_f(tile[tx][i]);
  }
}

hipError_t launch_cast_transpose(int dtype, const float* x, void* y, int64_t R, int64_t C, hipStream_t s) {
  dim3 grid((unsigned)((C + 63) / 64), (unsigned)((R + 63) / 64));
  if (dtype == 0) cast_transpose_kernel<bf16_t><<<grid, 256, 0, s>>>(x, (bf16_t*)y, R, C);
  else cast_transpose_kernel<float><<<grid, 256, 0, s>>>(x, (float*)y, R, C);
  return hipGetLastError();
}

// ================================================================ multi-tensor streaming helpers
__device__ __forceinline__ bool aligned16(const void* p) { return ((uintptr_t)p & 15) == 0; }

// Each workgroup loops over chunks (blockIdx.x, += gridDim.x): 8 resident workgroups per CU
// instead of one short-lived workgroup per chunk (27k of them for the ViT-B + head lists).
static inline unsigned tail_grid(int64_t nchunks) {
  static const int64_t cap = getenv("DSVT_TAIL_GRID") ? atoll(getenv("DSVT_TAIL_GRID")) : 2048;   // tuning only
  return (unsigned)(cap > 0 && nchunks > cap ? cap : nchunks);
}

// ================================================================ multi-tensor weight casts
// The bf16 copies of a whole model's weights in ONE launch each (after every optimizer / EMA
// step the weight cache refreshes them all): tensor i = src[i] (fp32, sizes[i] elements) ->
// dst[i]; work items are (tensor, 4096-element chunk) pairs like the EMA's.
__global__ __launch_bounds__(256) void cast_multi_kernel(const float* const* __restrict__ src,
                                                         bf16_t* const* __restrict__ dst,
                                                         const int64_t* __restrict__ sizes,
                                                         const int32_t* __restrict__ ctensor,
                                                         const int64_t* __restrict__ cstart, int64_t nchunks) {
  for (int64_t chunk = blockIdx.x; chunk < nchunks; chunk += gridDim.x) {
    const int ti = ctensor[chunk];
    const int64_t s0 = cstart[chunk], n = sizes[ti];
    const float* x = src[ti];
    bf16_t* y = dst[ti];
    const int64_t end = s0 + 4096 < n ? s0 + 4096 : n;
    int64_t i = s0;
    if (aligned16(x) && ((uintptr_t)y & 7) == 0) {
      const int64_t vend = s0 + ((end - s0) & ~(int64_t)3);
      float4 xv[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int64_t j = s0 + 4 * (threadIdx.x + 256 * k);
        if (j < vend) xv[k] = *(const float4*)(x + j);
      }
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int64_t j = s0 + 4 * (threadIdx.x + 256 * k);
        if (j < vend) {
          const uint32_t lo = (uint32_t)f2bf(xv[k].x) | ((uint32_t)f2bf(xv[k].y) << 16);
          const uint32_t hi = (uint32_t)f2bf(xv[k].z) | ((uint32_t)f2bf(xv[k].w) << 16);
          *(uint2*)(y + j) = make_uint2(lo, hi);
        }
      }
      i = vend;
    }
    for (i += threadIdx.x; i < end; i += 256) y[i] = f2bf(x[i]);
  }
}

// W^T copies ([R, C] fp32 -> [C, R] bf16) of a tensor list: one 64 x 64 tile per workgroup,
// tile table entries (tensor, row tile << 16 | column tile)
__global__ __launch_bounds__(256) void cast_transpose_multi_kernel(const float* const* __restrict__ src,
                                                                   bf16_t* const* __restrict__ dst,
                                                                   const int64_t* __restrict__ rows,
                                                                   const int64_t* __restrict__ cols,
                                                                   const int32_t* __restrict__ tile_tensor,
                                                                   const int32_t* __restrict__ tile_rc) {
  __shared__ float tile[64][65];
  const int ti = tile_tensor[blockIdx.x], rc = tile_rc[blockIdx.x];
  const int64_t R = rows[ti], C = cols[ti], r0 = (int64_t)(rc >> 16) * 64, c0 = (int64_t)(rc & 0xffff) * 64;
  const float* x = src[ti];
  bf16_t* y = dst[ti];
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  for (int i = ty; i < 64; i += 4) {
    const int64_t r = r0 + i, c = c0 + tx;
    tile[i][tx] = (r < R && c < C) ? x[r * C + c] : 0.f;
  }
  __syncthreads();
  for (int i = ty; i < 64; i += 4) {
    const int64_t c = c0 + i, r = r0 + tx;
    if (c < C && r < R) y[c * R + r] = f2bf(tile[tx][i]);
  }
}

hipError_t launch_cast_multi(const float* const* src, void* const* dst, const int64_t* sizes, const int32_t* ctensor,
                             const int64_t* cstart, int64_t nchunks, hipStream_t s) {
  cast_multi_kernel<<<tail_grid(nchunks), 256, 0, s>>>(src, (bf16_t* const*)dst, sizes, ctensor, cstart, nchunks);
  return hipGetLastError();
}

hipError_t launch_cast_transpose_multi(const float* const* src, void* const* dst, const int64_t* rows,
                                       const int64_t* cols, const int32_t* tile_tensor, const int32_t* tile_rc,
                                       int64_t ntiles, hipStream_t s) {
  cast_transpose_multi_kernel<<<(unsigned)ntiles, 256, 0, s>>>(src, (bf16_t* const*)dst, rows, cols, tile_tensor,
                                                               tile_rc);
  return hipGetLastError();
}

// ================================================================ token-embedding gradients
// Token gradient dX [B, L = 1 + Np*T, C] (NT order).  gn[n][c] = sum_{b,t} dX[b][1 + n*T + t][c],
// gt[t][c] = sum_{b,n} dX[b][1 + n*T + t][c], gc[c] = sum_b dX[b][0][c].
// stage 1: S[i][c] = sum_b dX[b][i][c] for every token position i in [0, L) (clip-sum)
__global__ __launch_bounds__(256) void embed_bsum_kernel(const float* __restrict__ dX, int64_t B, int64_t L, int64_t C,
                                                         float* __restrict__ S) {
  const int64_t i = blockIdx.y;
  const int64_t c = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (c >= C) return;
  float a = 0.f;
  for (int64_t b = 0; b < B; ++b) a += dX[(b * L + i) * C + c];
  S[i * C + c] = a;
}

// stage 2: gn[n] = sum_t S[1 + n*T + t], gt[t] = sum_n S[1 + n*T + t], gcls = S[0]
__global__ __launch_bounds__(256) void embed_sums_kernel(const float* __restrict__ S, int64_t Np, int64_t T, int64_t C,
                                                         float* __restrict__ gn, float* __restrict__ gt,
                                                         float* __restrict__ gcls) {
  const int64_t c = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (c >= C) return;
  const int64_t which = blockIdx.y;      // 0..Np-1 -> gn, Np..Np+T-1 -> gt, Np+T -> cls
  float a = 0.f;
  if (which < Np) {
    for (int64_t t = 0; t < T; ++t) a += S[(1 + which * T + t) * C + c];
    gn[which * C + c] = a;
  } else if (which < Np + T) {
    const int64_t t = which - Np;
    for (int64_t n = 0; n < Np; ++n) a += S[(1 + n * T + t) * C + c];
    gt[t * C + c] = a;
  } else {
    gcls[c] = S[c];
  }
}

// out[dst[i]][c] += src[i][c] for i < n (sequential over i: duplicates in dst are summed
// deterministically) -- the nearest-resize index maps of pos_embed / time_embed
__global__ __launch_bounds__(256) void index_accum_kernel(const float* __restrict__ src, const int32_t* __restrict__ dst,
                                                          int64_t n, int64_t C, int64_t dst_off,
                                                          float* __restrict__ out) {
  const int64_t c = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (c >= C) return;
  for (int64_t i = 0; i < n; ++i) out[((int64_t)dst[i] + dst_off) * C + c] += src[i * C + c];
}

hipError_t launch_embed_grads(const float* dX, int64_t B, int64_t Np, int64_t T, int64_t C, float* gn, float* gt,
                              float* gcls, float* S, hipStream_t s) {
  const int64_t L = 1 + Np * T;
  embed_bsum_kernel<<<dim3((unsigned)((C + 255) / 256), (unsigned)L), 256, 0, s>>>(dX, B, L, C, S);
  embed_sums_kernel<<<dim3((unsigned)((C + 255) / 256), (unsigned)(Np + T + 1)), 256, 0, s>>>(S, Np, T, C, gn, gt,
                                                                                            gcls);
  return hipGetLastError();
}

hipError_t launch_index_accum(const float* src, const int32_t* dst, int64_t n, int64_t C, int64_t dst_off, float* out,
                              hipStream_t s) {
  index_accum_kernel<<<(unsigned)((C + 255) / 256), 256, 0, s>>>(src, dst, n, C, dst_off, out);
  return hipGetLastError();
}

// ================================================================ multi-tensor EMA / grad clipping
// Tensor list: ptrs[i] (fp32), sizes[i]; work items are (tensor, 4096-element chunk) pairs
// listed in chunk_tensor / chunk_start (built once on the host per parameter list).
// The optimizer-tail kernels stream a 4096-element chunk per loop trip: 1024 float4 slots,
// four per thread, all loads issued before the first store.  A tensor whose pointers are not
// all 16-B aligned, and the last (size % 4) elements of a tensor, take the scalar path.
// Measured in the train step (r05, ~144M parameters): AdamW 28 B/param in 2 x 0.35 ms and EMA
// 12 B/param in 0.32 ms were already ~5.5 TB/s as scalar loops and did not move; the grad
// sum of squares (4 B/param) went 0.167 -> 0.105 ms.  DSVT_TAIL_GRID 0/1024/2048/4096 equal.

__global__ __launch_bounds__(256) void ema_kernel(float* const* __restrict__ teacher, const float* const* __restrict__ student,
                                                  const int64_t* __restrict__ sizes, const int32_t* __restrict__ ctensor,
                                                  const int64_t* __restrict__ cstart, float m, int64_t nchunks) {
  for (int64_t chunk = blockIdx.x; chunk < nchunks; chunk += gridDim.x) {
    const int ti = ctensor[chunk];
    const int64_t s0 = cstart[chunk], n = sizes[ti];
    float* t = teacher[ti];
    const float* q = student[ti];
    const int64_t end = s0 + 4096 < n ? s0 + 4096 : n;
    int64_t i = s0;
    if (aligned16(t) && aligned16(q)) {
      const int64_t vend = s0 + ((end - s0) & ~(int64_t)3);
      float4 tv[4], qv[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int64_t j = s0 + 4 * (threadIdx.x + 256 * k);
        if (j < vend) {
          tv[k] = *(const float4*)(t + j);
          qv[k] = *(const float4*)(q + j);
        }
      }
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int64_t j = s0 + 4 * (threadIdx.x + 256 * k);
        if (j < vend) {
          float4 r;
          r.x = tv[k].x * m + (1.0f - m) * qv[k].x;
          r.y = tv[k].y * m + (1.0f - m) * qv[k].y;
          r.z = tv[k].z * m + (1.0f - m) * qv[k].z;
          r.w = tv[k].w * m + (1.0f - m) * qv[k].w;
          *(float4*)(t + j) = r;
        }
      }
      i = vend;
    }
    for (i += threadIdx.x; i < end; i += 256) t[i] = t[i] * m + (1.0f - m) * q[i];
  }
}

// per-chunk sum of squares of grads -> partial[chunk]
__global__ __launch_bounds__(256) void sumsq_kernel(const float* const* __restrict__ x, const int64_t* __restrict__ sizes,
                                                    const int32_t* __restrict__ ctensor, const int64_t* __restrict__ cstart,
                                                    float* __restrict__ partial, int64_t nchunks) {
  __shared__ float red[4];
  for (int64_t chunk = blockIdx.x; chunk < nchunks; chunk += gridDim.x) {
    const int ti = ctensor[chunk];
    const int64_t s0 = cstart[chunk], n = sizes[ti];
    const float* p = x[ti];
    const int64_t end = s0 + 4096 < n ? s0 + 4096 : n;
    float a = 0.f;
    int64_t i = s0;
    if (aligned16(p)) {
      const int64_t vend = s0 + ((end - s0) & ~(int64_t)3);
      float4 pv[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int64_t j = s0 + 4 * (threadIdx.x + 256 * k);
        pv[k] = j < vend ? *(const float4*)(p + j) : make_float4(0.f, 0.f, 0.f, 0.f);
      }
#pragma unroll
      for (int k = 0; k < 4; ++k) a += (pv[k].x * pv[k].x + pv[k].y * pv[k].y) + (pv[k].z * pv[k].z + pv[k].w * pv[k].w);
      i = vend;
    }
    for (i += threadIdx.x; i < end; i += 256) a += p[i] * p[i];
    a = wave_sum(a);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = a;
    __syncthreads();
    if (threadIdx.x == 0) partial[chunk] = (red[0] + red[1]) + (red[2] + red[3]);
    __syncthreads();  // red[] is rewritten by the next chunk
  }
}

// norms[i] = sqrt(sum of the tensor's chunk partials) (chunks of one tensor are contiguous):
// one workgroup per tensor, lane-strided partial sums then a fixed-order tree (deterministic;
// the head's 65536 x 256 last layer alone has 4096 chunks, a serial loop took 0.36 ms)
__global__ __launch_bounds__(256) void chunk_norms_kernel(const float* __restrict__ partial,
                                                          const int32_t* __restrict__ first_chunk, int ntensors,
                                                          float* __restrict__ norms) {
  __shared__ float red[4];
  const int i = blockIdx.x;
  float a = 0.f;
  for (int c = first_chunk[i] + (int)threadIdx.x; c < first_chunk[i + 1]; c += 256) a += partial[c];
  a = wave_sum(a);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = a;
  __syncthreads();
  if (threadIdx.x == 0) norms[i] = sqrtf((red[0] + red[1]) + (red[2] + red[3]));
}

// utils/utils.py:102-111: clip_coef = clip / (norm + 1e-6); grad *= clip_coef if < 1
__global__ __launch_bounds__(256) void clip_scale_kernel(float* const* __restrict__ x, const int64_t* __restrict__ sizes,
                                                         const int32_t* __restrict__ ctensor,
                                                         const int64_t* __restrict__ cstart,
                                                         const float* __restrict__ norms, float clip, int64_t nchunks) {
  for (int64_t chunk = blockIdx.x; chunk < nchunks; chunk += gridDim.x) {
    const int ti = ctensor[chunk];
    const float coef = clip / (norms[ti] + 1e-6f);
    if (coef >= 1.0f) continue;
    const int64_t s0 = cstart[chunk], n = sizes[ti];
    float* p = x[ti];
    const int64_t end = s0 + 4096 < n ? s0 + 4096 : n;
    int64_t i = s0;
    if (aligned16(p)) {
      const int64_t vend = s0 + ((end - s0) & ~(int64_t)3);
      float4 pv[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int64_t j = s0 + 4 * (threadIdx.x + 256 * k);
        if (j < vend) pv[k] = *(const float4*)(p + j);
      }
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int64_t j = s0 + 4 * (threadIdx.x + 256 * k);
        if (j < vend) {
          pv[k].x *= coef;
          pv[k].y *= coef;
          pv[k].z *= coef;
          pv[k].w *= coef;
          *(float4*)(p + j) = pv[k];
        }
      }
      i = vend;
    }
    for (i += threadIdx.x; i < end; i += 256) p[i] *= coef;
  }
}

// AdamW (decoupled weight decay), the update torch.optim.AdamW applies for the reference's
// `torch.optim.AdamW(params_groups)` (train_ssl.py:384, step at :551), per element:
//   p *= 1 - lr*wd;  m = m + (1-b1)(g - m);  v = b2 v + (1-b2) g^2;
//   p += step_size * m / (sqrt(v) / sqrt(1 - b2^t) + eps),  step_size = -lr / (1 - b1^t)
// One launch per (param group, step count) tensor list; one workgroup per 4096-element chunk.
__global__ __launch_bounds__(256) void adamw_kernel(float* const* __restrict__ param, const float* const* __restrict__ grad,
                                                    float* const* __restrict__ exp_avg,
                                                    float* const* __restrict__ exp_avg_sq,
                                                    const int64_t* __restrict__ sizes, const int32_t* __restrict__ ctensor,
                                                    const int64_t* __restrict__ cstart, AdamWArgs a, int64_t nchunks) {
  for (int64_t chunk = blockIdx.x; chunk < nchunks; chunk += gridDim.x) {
    const int ti = ctensor[chunk];
    const int64_t s0 = cstart[chunk], n = sizes[ti];
    float* p = param[ti];
    const float* g = grad[ti];
    float* m = exp_avg[ti];
    float* v = exp_avg_sq[ti];
    const float decay = 1.0f - a.lr * a.wd, w1 = 1.0f - a.beta1, w2 = 1.0f - a.beta2;
    const int64_t end = s0 + 4096 < n ? s0 + 4096 : n;
    int64_t i = s0;
    if (aligned16(p) && aligned16(g) && aligned16(m) && aligned16(v)) {
      const int64_t vend = s0 + ((end - s0) & ~(int64_t)3);
      float4 pv[4], gv[4], mv[4], vv[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int64_t j = s0 + 4 * (threadIdx.x + 256 * k);
        if (j < vend) {
          gv[k] = *(const float4*)(g + j);
          mv[k] = *(const float4*)(m + j);
          vv[k] = *(const float4*)(v + j);
          pv[k] = *(const float4*)(p + j);
        }
      }
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int64_t j = s0 + 4 * (threadIdx.x + 256 * k);
        if (j < vend) {
          float* pe = &pv[k].x;
          float* ge = &gv[k].x;
          float* me = &mv[k].x;
          float* ve = &vv[k].x;
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const float gi = ge[e];
            const float mi = me[e] + w1 * (gi - me[e]);
            const float vi = ve[e] * a.beta2 + w2 * gi * gi;
            const float denom = sqrtf(vi) / a.bc2_sqrt + a.eps;
            me[e] = mi;
            ve[e] = vi;
            pe[e] = pe[e] * decay + a.step_size * (mi / denom);
          }
          *(float4*)(m + j) = mv[k];
          *(float4*)(v + j) = vv[k];
          *(float4*)(p + j) = pv[k];
        }
      }
      i = vend;
    }
    for (i += threadIdx.x; i < end; i += 256) {
      const float gi = g[i];
      const float mi = m[i] + w1 * (gi - m[i]);
      const float vi = v[i] * a.beta2 + w2 * gi * gi;
      const float denom = sqrtf(vi) / a.bc2_sqrt + a.eps;
      m[i] = mi;
      v[i] = vi;
      p[i] = p[i] * decay + a.step_size * (mi / denom);
    }
  }
}

hipError_t launch_adamw(float* const* param, const float* const* grad, float* const* exp_avg, float* const* exp_avg_sq,
                        const int64_t* sizes, const int32_t* ctensor, const int64_t* cstart, int64_t nchunks,
                        const AdamWArgs& a, hipStream_t s) {
  adamw_kernel<<<tail_grid(nchunks), 256, 0, s>>>(param, grad, exp_avg, exp_avg_sq, sizes, ctensor, cstart, a, nchunks);
  return hipGetLastError();
}

hipError_t launch_ema(float* const* teacher, const float* const* student, const int64_t* sizes, const int32_t* ctensor,
                      const int64_t* cstart, int64_t nchunks, float m, hipStream_t s) {
  ema_kernel<<<tail_grid(nchunks), 256, 0, s>>>(teacher, student, sizes, ctensor, cstart, m, nchunks);
  return hipGetLastError();
}

hipError_t launch_clip_grads(float* const* grads, const int64_t* sizes, const int32_t* ctensor, const int64_t* cstart,
                             const int32_t* first_chunk, int64_t nchunks, int64_t ntensors, float clip, float* partial,
                             float* norms, hipStream_t s) {
  sumsq_kernel<<<tail_grid(nchunks), 256, 0, s>>>(grads, sizes, ctensor, cstart, partial, nchunks);
  chunk_norms_kernel<<<(unsigned)ntensors, 256, 0, s>>>(partial, first_chunk, (int)ntensors, norms);
  if (clip > 0.f)
    clip_scale_kernel<<<tail_grid(nchunks), 256, 0, s>>>(grads, sizes, ctensor, cstart, norms, clip, nchunks);
  return hipGetLastError();
}

}  // namespace dsvt
