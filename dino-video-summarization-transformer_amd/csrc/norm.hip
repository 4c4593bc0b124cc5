// Row-wise normalizations and the small layout kernels of the hot path.
//   LayerNorm (K3), F.normalize + weight-norm (K12), im2col for PatchEmbed (K1),
//   CLS token init (K2), CLS mean over frames (K8), dtype cast.
// All are HBM-bound: one wave per row, 16-B vector loads where the row length allows.
#include <stdlib.h>

#include "common.h"

namespace dsvt {

// ---------------------------------------------------------------- LayerNorm
// One wave per row; VEC: C % 256 == 0 (float4 per lane per 256 cols), else C % 64 == 0.
template <typename OutT, bool VEC, bool MAPOUT = false>
__global__ __launch_bounds__(256) void layernorm_kernel(const float* __restrict__ x, OutT* __restrict__ y,
                                                        const float* __restrict__ gamma,
                                                        const float* __restrict__ beta, int64_t rows,
                                                        int C, int64_t rpg, int64_t gstride,
                                                        int64_t goff, float eps) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int64_t r = (int64_t)blockIdx.x * 4 + wave;
  if (r >= rows) return;
  const int64_t xrow = map_row(r, rpg, gstride, goff);
  const float* xr = x + xrow * C;
  OutT* yr = y + (MAPOUT ? xrow : r) * C;
  float v[16];
  float s = 0.f;
  if constexpr (VEC) {
    const int n4 = C >> 8;
#pragma unroll
    for (int i = 0; i < 4; ++i)
      if (i < n4) {
        float4 f = *reinterpret_cast<const float4*>(xr + i * 256 + lane * 4);
        v[4 * i] = f.x; v[4 * i + 1] = f.y; v[4 * i + 2] = f.z; v[4 * i + 3] = f.w;
        s += (f.x + f.y) + (f.z + f.w);
      }
    const float mean = wave_sum(s) / C;
    float q = 0.f;
#pragma unroll
    for (int i = 0; i < 16; ++i)
      if (i < 4 * n4) { v[i] -= mean; q += v[i] * v[i]; }
    const float rstd = 1.0f / sqrtf(wave_sum(q) / C + eps);
#pragma unroll
    for (int i = 0; i < 4; ++i)
      if (i < n4) {
        const int c = i * 256 + lane * 4;
        const float4 gg = *reinterpret_cast<const float4*>(gamma + c);
        const float4 bb = *reinterpret_cast<const float4*>(beta + c);
        store4(yr + c, v[4 * i] * rstd * gg.x + bb.x, v[4 * i + 1] * rstd * gg.y + bb.y,
               v[4 * i + 2] * rstd * gg.z + bb.z, v[4 * i + 3] * rstd * gg.w + bb.w);
      }
  } else {
    const int n = C >> 6;
#pragma unroll
    for (int i = 0; i < 16; ++i)
      if (i < n) { v[i] = xr[i * 64 + lane]; s += v[i]; }
    const float mean = wave_sum(s) / C;
    float q = 0.f;
#pragma unroll
    for (int i = 0; i < 16; ++i)
      if (i < n) { v[i] -= mean; q += v[i] * v[i]; }
    const float rstd = 1.0f / sqrtf(wave_sum(q) / C + eps);
#pragma unroll
    for (int i = 0; i < 16; ++i)
      if (i < n) {
        const int c = i * 64 + lane;
        yr[c] = Elem<OutT>::from_f(v[i] * rstd * gamma[c] + beta[c]);
      }
  }
}

// C = 768 (ViT-B): a wave walks rows with a grid stride and issues the NEXT row's three 16-B
// loads before the current row's two reductions, so each wave keeps a row of loads in flight
// under its own arithmetic (the one-row-per-wave kernel above waits out a full HBM round trip
// per row).  gamma / beta stay in registers.  Same formula and summation order as
// layernorm_kernel<., true>; a row's result does not depend on the grid size.
// Measured (tools/ln_bench.py, fp32 -> bf16): 25104 rows 21.0 -> 18.9 us, 13872 rows 13.6 -> 10.7 us.
template <typename OutT, bool MAPOUT = false>
__global__ __launch_bounds__(256) void layernorm768_kernel(const float* __restrict__ x, OutT* __restrict__ y,
                                                           const float* __restrict__ gamma,
                                                           const float* __restrict__ beta, int64_t rows,
                                                           int64_t rpg, int64_t gstride, int64_t goff, float eps) {
  constexpr int C = 768;
  const int lane = threadIdx.x & 63;
  const int64_t nw = (int64_t)gridDim.x * 4;
  int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= rows) return;
  float4 gg[3], bb[3], cur[3];
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    gg[i] = *reinterpret_cast<const float4*>(gamma + i * 256 + lane * 4);
    bb[i] = *reinterpret_cast<const float4*>(beta + i * 256 + lane * 4);
  }
  const float* xr = x + map_row(r, rpg, gstride, goff) * C;
#pragma unroll
  for (int i = 0; i < 3; ++i) cur[i] = *reinterpret_cast<const float4*>(xr + i * 256 + lane * 4);
  while (true) {
    const int64_t rn = r + nw;
    const float* xn = x + map_row(rn < rows ? rn : r, rpg, gstride, goff) * C;   // clamped: branch-free
    float4 nxt[3];
#pragma unroll
    for (int i = 0; i < 3; ++i) nxt[i] = *reinterpret_cast<const float4*>(xn + i * 256 + lane * 4);
    float v[12];
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      const float4 f = cur[i];
      v[4 * i] = f.x; v[4 * i + 1] = f.y; v[4 * i + 2] = f.z; v[4 * i + 3] = f.w;
      s += (f.x + f.y) + (f.z + f.w);
    }
    const float mean = wave_sum(s) / C;
    float q = 0.f;
#pragma unroll
    for (int i = 0; i < 12; ++i) { v[i] -= mean; q += v[i] * v[i]; }
    const float rstd = 1.0f / sqrtf(wave_sum(q) / C + eps);
    OutT* yr = y + (MAPOUT ? map_row(r, rpg, gstride, goff) : r) * C;
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      const float4 g4 = gg[i], b4 = bb[i];
      store4(yr + i * 256 + lane * 4, v[4 * i] * rstd * g4.x + b4.x, v[4 * i + 1] * rstd * g4.y + b4.y,
             v[4 * i + 2] * rstd * g4.z + b4.z, v[4 * i + 3] * rstd * g4.w + b4.w);
    }
    if (rn >= rows) break;
    r = rn;
#pragma unroll
    for (int i = 0; i < 3; ++i) cur[i] = nxt[i];
  }
}

// ---------------------------------------------------------------- LayerNorm inputs of a folded GEMM
// For dsvt_gemm_lnx_fwd (the LayerNorm folded into the GEMM that reads its output): the bf16 copy
// of every fp32 token row and its row-statistics partials, float2 (sum x, sum x^2) over each
// 64-column slab (LN_PARTS = 12 for C = 768) -- what the residual epilogue of
// dsvt_gemm_resid_stats_fwd writes for the rows it updates; this pass covers the rows a forward
// starts with (after the patch embedding).  One wave per row, grid-strided, C = 768.
__global__ __launch_bounds__(256) void ln_stats768_kernel(const float* __restrict__ x, bf16_t* __restrict__ xb,
                                                          float* __restrict__ stats, int64_t rows) {
  constexpr int C = 768;
  const int lane = threadIdx.x & 63;
  const int64_t nw = (int64_t)gridDim.x * 4;
  for (int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); r < rows; r += nw) {
    float4 v[3];
#pragma unroll
    for (int i = 0; i < 3; ++i) v[i] = *reinterpret_cast<const float4*>(x + r * C + i * 256 + lane * 4);
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      store4(xb + r * C + i * 256 + lane * 4, v[i].x, v[i].y, v[i].z, v[i].w);
      // lanes 16q .. 16q + 15 of chunk i hold slab 4i + q
      float s = (v[i].x + v[i].y) + (v[i].z + v[i].w);
      float q = sumsq4(v[i].x, v[i].y, v[i].z, v[i].w);
#pragma unroll
      for (int o = 1; o < 16; o <<= 1) {
        s += __shfl_xor(s, o);
        q += __shfl_xor(q, o);
      }
      if ((lane & 15) == 0)
        *reinterpret_cast<float2*>(stats + (r * LN_PARTS + i * 4 + (lane >> 4)) * 2) = make_float2(s, q);
    }
  }
}

hipError_t launch_ln_stats(const float* x, void* xb, float* stats, int64_t rows, hipStream_t s) {
  const int64_t wg = (rows + 3) / 4;
  ln_stats768_kernel<<<dim3((unsigned)(wg < 1024 ? wg : 1024)), dim3(256), 0, s>>>(x, (bf16_t*)xb, stats, rows);
  return hipGetLastError();
}

// The weights of a LayerNorm-folded GEMM (dsvt_ln_fold_weights): for W [N, K] fp32 following
// LayerNorm(gamma, beta):  Wf = bf16(W * gamma) [N, K],  wsum[n] = sum_k Wf[n, k] (of the bf16
// values the MFMA multiplies),  bf[n] = b[n] + sum_k W[n, k] * beta[k].  One wave per row.
// heads > 0 (an attention qkv weight, N = 3 * heads * 64): output row o(n) head-interleaved for the
// temporal-attention GEMM (gemm_192.hip) -- row n = part*C + h*64 + d (part q / k / v) goes to
// o = h*192 + (d / 32)*96 + part*32 + d % 32.
__global__ __launch_bounds__(256) void ln_fold_kernel(const float* __restrict__ W, const float* __restrict__ gamma,
                                                      const float* __restrict__ beta, const float* __restrict__ b,
                                                      bf16_t* __restrict__ Wf, float* __restrict__ wsum,
                                                      float* __restrict__ bf, int64_t N, int64_t K, int heads) {
  const int lane = threadIdx.x & 63;
  const int64_t n = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (n >= N) return;
  int64_t o = n;
  if (heads > 0) {
    const int64_t C = N / 3, part = n / C, h = (n % C) / 64, d = n % 64;
    o = h * 192 + (d / 32) * 96 + part * 32 + d % 32;
  }
  float s = 0.f, t = 0.f;
  for (int64_t k = lane * 4; k < K; k += 256) {
    const float4 w = *reinterpret_cast<const float4*>(W + n * K + k);
    const float4 gg = *reinterpret_cast<const float4*>(gamma + k);
    const float4 bb = *reinterpret_cast<const float4*>(beta + k);
    const unsigned lo = cvt_pk_bf16(w.x * gg.x, w.y * gg.y), hi = cvt_pk_bf16(w.z * gg.z, w.w * gg.w);
    *reinterpret_cast<uint2*>(Wf + o * K + k) = make_uint2(lo, hi);
    s += (__uint_as_float(lo << 16) + __uint_as_float(lo & 0xffff0000u)) +
         (__uint_as_float(hi << 16) + __uint_as_float(hi & 0xffff0000u));
    t += (w.x * bb.x + w.y * bb.y) + (w.z * bb.z + w.w * bb.w);
  }
  s = wave_sum(s);
  t = wave_sum(t);
  if (lane == 0) {
    wsum[o] = s;
    bf[o] = (b ? b[n] : 0.f) + t;
  }
}

hipError_t launch_ln_fold(const float* W, const float* gamma, const float* beta, const float* b, void* Wf, float* wsum,
                          float* bf, int64_t N, int64_t K, hipStream_t s, int heads) {
  ln_fold_kernel<<<dim3((unsigned)((N + 3) / 4)), dim3(256), 0, s>>>(W, gamma, beta, b, (bf16_t*)Wf, wsum, bf, N, K,
                                                                    heads);
  return hipGetLastError();
}

template <typename OutT, bool MAPOUT>
static hipError_t ln_t(const float* x, OutT* y, const float* g, const float* b, int64_t rows, int64_t C,
                       int64_t rpg, int64_t gstride, int64_t goff, float eps, hipStream_t s) {
  dim3 grid((unsigned)((rows + 3) / 4)), block(256);
  const int cap = 1024;                 // workgroups of the C = 768 kernel
  if (C == 768) {
    if (grid.x > (unsigned)cap) grid.x = (unsigned)cap;
    layernorm768_kernel<OutT, MAPOUT><<<grid, block, 0, s>>>(x, y, g, b, rows, rpg, gstride, goff, eps);
  } else if (C % 256 == 0)
    layernorm_kernel<OutT, true, MAPOUT><<<grid, block, 0, s>>>(x, y, g, b, rows, (int)C, rpg, gstride, goff, eps);
  else
    layernorm_kernel<OutT, false, MAPOUT><<<grid, block, 0, s>>>(x, y, g, b, rows, (int)C, rpg, gstride, goff, eps);
  return hipGetLastError();
}

// out_f32 bit 0: fp32 output; bit 1: output row = input row (the row map applies to both)
hipError_t launch_layernorm(int dtype, int out_f32, const float* x, void* y, const float* g,
                            const float* b, int64_t rows, int64_t C, int64_t rpg, int64_t gstride,
                            int64_t goff, float eps, hipStream_t s) {
  const bool f32 = dtype == 1 || (out_f32 & 1), mapout = (out_f32 & 2) != 0;
  if (f32 && mapout) return ln_t<float, true>(x, (float*)y, g, b, rows, C, rpg, gstride, goff, eps, s);
  if (f32) return ln_t<float, false>(x, (float*)y, g, b, rows, C, rpg, gstride, goff, eps, s);
  if (mapout) return ln_t<bf16_t, true>(x, (bf16_t*)y, g, b, rows, C, rpg, gstride, goff, eps, s);
  return ln_t<bf16_t, false>(x, (bf16_t*)y, g, b, rows, C, rpg, gstride, goff, eps, s);
}

// ---------------------------------------------------------------- L2 row norms
// MODE 0: F.normalize  y = x / max(||x||, eps)          (vision_transformer.py:280)
// MODE 1: weight_norm  y = x * (g[r] / ||x||)           (torch._weight_norm, dim=0)
template <typename OutT, int MODE>
__global__ __launch_bounds__(256) void rownorm_kernel(const float* __restrict__ x, const float* __restrict__ g,
                                                      OutT* __restrict__ y, int64_t rows, int D, float eps) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int64_t r = (int64_t)blockIdx.x * 4 + wave;
  if (r >= rows) return;
  const float* xr = x + r * D;
  OutT* yr = y + r * D;
  float s = 0.f;
  for (int c = lane * 4; c < D; c += 256) {
    const float4 f = *reinterpret_cast<const float4*>(xr + c);
    s += f.x * f.x + f.y * f.y + f.z * f.z + f.w * f.w;
  }
  const float nrm = sqrtf(wave_sum_dpp(s));
  const float sc = MODE == 0 ? 1.0f / fmaxf(nrm, eps) : g[r] / nrm;
  for (int c = lane * 4; c < D; c += 256) {
    const float4 f = *reinterpret_cast<const float4*>(xr + c);
    store4(yr + c, f.x * sc, f.y * sc, f.z * sc, f.w * sc);
  }
}

// D == 256, many rows (the DINO head's last-layer weight rows): one float4 per lane per row, 4 rows per
// wave with their loads issued together (one row per wave left 65536 single-load waves at
// 2.9 TB/s on the last layer's weight norm).
template <typename OutT, int MODE>
__global__ __launch_bounds__(256) void rownorm256_kernel(const float* __restrict__ x, const float* __restrict__ g,
                                                         OutT* __restrict__ y, int64_t rows, float eps) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int64_t r0 = ((int64_t)blockIdx.x * 4 + wave) * 4;
  float4 f[4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
    f[i] = r0 + i < rows ? *reinterpret_cast<const float4*>(x + (r0 + i) * 256 + lane * 4) : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    if (r0 + i >= rows) break;
    const float nrm = sqrtf(wave_sum_dpp(f[i].x * f[i].x + f[i].y * f[i].y + f[i].z * f[i].z + f[i].w * f[i].w));
    const float sc = MODE == 0 ? 1.0f / fmaxf(nrm, eps) : g[r0 + i] / nrm;
    store4(y + (r0 + i) * 256 + lane * 4, f[i].x * sc, f[i].y * sc, f[i].z * sc, f[i].w * sc);
  }
}

hipError_t launch_l2norm(int dtype, const float* x, void* y, int64_t rows, int64_t D, float eps, hipStream_t s) {
  if (D == 256 && rows >= 4096) {          // few rows (the head's 16-64 crop rows): one row per wave
    dim3 grid((unsigned)((rows + 15) / 16)), block(256);
    if (dtype == 0) rownorm256_kernel<bf16_t, 0><<<grid, block, 0, s>>>(x, nullptr, (bf16_t*)y, rows, eps);
    else rownorm256_kernel<float, 0><<<grid, block, 0, s>>>(x, nullptr, (float*)y, rows, eps);
    return hipGetLastError();
  }
  dim3 grid((unsigned)((rows + 3) / 4)), block(256);
  if (dtype == 0) rownorm_kernel<bf16_t, 0><<<grid, block, 0, s>>>(x, nullptr, (bf16_t*)y, rows, (int)D, eps);
  else rownorm_kernel<float, 0><<<grid, block, 0, s>>>(x, nullptr, (float*)y, rows, (int)D, eps);
  return hipGetLastError();
}

hipError_t launch_weight_norm(int dtype, const float* v, const float* g, void* w, int64_t rows, int64_t D,
                              hipStream_t s) {
  if (D == 256 && rows >= 4096) {
    dim3 grid((unsigned)((rows + 15) / 16)), block(256);
    if (dtype == 0) rownorm256_kernel<bf16_t, 1><<<grid, block, 0, s>>>(v, g, (bf16_t*)w, rows, 0.f);
    else rownorm256_kernel<float, 1><<<grid, block, 0, s>>>(v, g, (float*)w, rows, 0.f);
    return hipGetLastError();
  }
  dim3 grid((unsigned)((rows + 3) / 4)), block(256);
  if (dtype == 0) rownorm_kernel<bf16_t, 1><<<grid, block, 0, s>>>(v, g, (bf16_t*)w, rows, (int)D, 0.f);
  else rownorm_kernel<float, 1><<<grid, block, 0, s>>>(v, g, (float*)w, rows, (int)D, 0.f);
  return hipGetLastError();
}

// ---------------------------------------------------------------- cast fp32 -> T
template <typename OutT>
__global__ void cast_kernel(const float* __restrict__ x, OutT* __restrict__ y, int64_t n4) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += (int64_t)gridDim.x * blockDim.x) {
    const float4 f = reinterpret_cast<const float4*>(x)[i];
    store4(y + 4 * i, f.x, f.y, f.z, f.w);
  }
}

hipError_t launch_cast(int dtype, const float* x, void* y, int64_t n, hipStream_t s) {
  const int64_t n4 = n / 4;
  unsigned blocks = (unsigned)((n4 + 255) / 256);
  if (blocks > 4096) blocks = 4096;
  if (blocks == 0) return hipSuccess;
  if (dtype == 0) cast_kernel<bf16_t><<<blocks, 256, 0, s>>>(x, (bf16_t*)y, n4);
  else cast_kernel<float><<<blocks, 256, 0, s>>>(x, (float*)y, n4);
  return hipGetLastError();
}

// ---------------------------------------------------------------- im2col (PatchEmbed)
// A[m][k], k = c*256 + kh*16 + kw; order_nt: m = (b*Np + np)*T + t, else m = (b*T + t)*Np + np.
// One thread per 4 consecutive kw (one float4 of the input row).
// fidx (nullable): x is a frame bank [F][Cin][H][W]; frame t of clip b = fidx[b*Tf + t], -1 = zeros.
template <typename T>
__global__ void im2col_kernel(const float* __restrict__ x, T* __restrict__ a, int64_t total, int Cin, int Tf,
                              int H, int W, int Hp, int Wp, int order_nt, const int32_t* __restrict__ fidx) {
  const int K = Cin * 256, kq = K / 4, Np = Hp * Wp;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t m = i / kq;
    const int k = (int)(i % kq) * 4;
    const int c = k >> 8, kh = (k >> 4) & 15, kw = k & 15;
    int64_t b; int t, np;
    if (order_nt) { t = (int)(m % Tf); np = (int)((m / Tf) % Np); b = m / ((int64_t)Tf * Np); }
    else { np = (int)(m % Np); t = (int)((m / Np) % Tf); b = m / ((int64_t)Tf * Np); }
    const int ph = np / Wp, pw = np % Wp;
    float4 f = make_float4(0.f, 0.f, 0.f, 0.f);
    if (fidx) {
      const int fi = fidx[b * Tf + t];
      if (fi >= 0) f = *reinterpret_cast<const float4*>(x + ((((int64_t)fi * Cin + c) * H + ph * 16 + kh) * (int64_t)W + pw * 16 + kw));
    } else {
      f = *reinterpret_cast<const float4*>(x + ((((b * Cin + c) * Tf + t) * H + ph * 16 + kh) * (int64_t)W + pw * 16 + kw));
    }
    store4(a + m * K + k, f.x, f.y, f.z, f.w);
  }
}

hipError_t launch_im2col(int dtype, int order_nt, const float* x, void* a, int64_t B, int64_t Cin, int64_t T,
                         int64_t H, int64_t W, int64_t Hp, int64_t Wp, const int32_t* fidx, hipStream_t s) {
  const int64_t total = B * T * Hp * Wp * Cin * 64;
  unsigned blocks = (unsigned)((total + 255) / 256);
  if (blocks > 16384) blocks = 16384;
  if (dtype == 0)
    im2col_kernel<bf16_t><<<blocks, 256, 0, s>>>(x, (bf16_t*)a, total, (int)Cin, (int)T, (int)H, (int)W, (int)Hp, (int)Wp, order_nt, fidx);
  else
    im2col_kernel<float><<<blocks, 256, 0, s>>>(x, (float*)a, total, (int)Cin, (int)T, (int)H, (int)W, (int)Hp, (int)Wp, order_nt, fidx);
  return hipGetLastError();
}

// ---------------------------------------------------------------- bicubic pos-embed resize
// ATen upsample_bicubic2d (align_corners=False, scale given): real = inv_scale*(dst+0.5)-0.5,
// idx = min(floor(real), size-1), t = clamp(real-idx, 0, 1), taps idx-1..idx+2 clamped,
// A = -0.75; interpolate along x for 4 rows, then along y (same op order as ATen's CPU loop).
__device__ __forceinline__ void cubic_coeffs(float t, float* c) {
  const float A = -0.75f;
  float x1 = t;
  c[0] = ((A * (x1 + 1.f) - 5.f * A) * (x1 + 1.f) + 8.f * A) * (x1 + 1.f) - 4.f * A;
  c[1] = ((A + 2.f) * x1 - (A + 3.f)) * x1 * x1 + 1.f;
  float x2 = 1.f - t;
  c[2] = ((A + 2.f) * x2 - (A + 3.f)) * x2 * x2 + 1.f;
  c[3] = ((A * (x2 + 1.f) - 5.f * A) * (x2 + 1.f) + 8.f * A) * (x2 + 1.f) - 4.f * A;
}

__global__ void pos_bicubic_kernel(const float* __restrict__ pos, float* __restrict__ out, int sg, int OH, int OW,
                                   int C, float inv_h, float inv_w) {
  const int o = blockIdx.x;  // 0 = CLS row
  for (int c = threadIdx.x; c < C; c += blockDim.x) {
    if (o == 0) { out[c] = pos[c]; continue; }
    const int oy = (o - 1) / OW, ox = (o - 1) % OW;
    const float ry = inv_h * ((float)oy + 0.5f) - 0.5f, rx = inv_w * ((float)ox + 0.5f) - 0.5f;
    int iy = (int)floorf(ry); iy = iy < sg - 1 ? iy : sg - 1;
    int ix = (int)floorf(rx); ix = ix < sg - 1 ? ix : sg - 1;
    const float ty = fminf(fmaxf(ry - iy, 0.f), 1.f), tx = fminf(fmaxf(rx - ix, 0.f), 1.f);
    float cy[4], cx[4], rows[4];
    cubic_coeffs(ty, cy);
    cubic_coeffs(tx, cx);
    for (int i = 0; i < 4; ++i) {
      int yy = iy - 1 + i; yy = yy < 0 ? 0 : (yy > sg - 1 ? sg - 1 : yy);
      float v[4];
      for (int j = 0; j < 4; ++j) {
        int xx = ix - 1 + j; xx = xx < 0 ? 0 : (xx > sg - 1 ? sg - 1 : xx);
        v[j] = pos[(int64_t)(1 + yy * sg + xx) * C + c];
      }
      rows[i] = v[0] * cx[0] + v[1] * cx[1] + v[2] * cx[2] + v[3] * cx[3];
    }
    out[(int64_t)o * C + c] = rows[0] * cy[0] + rows[1] * cy[1] + rows[2] * cy[2] + rows[3] * cy[3];
  }
}

hipError_t launch_pos_bicubic(const float* pos, float* out, int64_t sgrid, int64_t OH, int64_t OW, int64_t C,
                              float inv_h, float inv_w, hipStream_t s) {
  pos_bicubic_kernel<<<(unsigned)(1 + OH * OW), 256, 0, s>>>(pos, out, (int)sgrid, (int)OH, (int)OW, (int)C, inv_h, inv_w);
  return hipGetLastError();
}

// Backward of pos_bicubic (the 2-D ViT's interpolate_pos_encoding in training): dpos[1 + n][c]
// (+)= sum over output cells o of w(o, n) * dout[o][c], w(o, n) = the sum of the forward's
// stencil weights cy[i] * cx[j] whose (clamped) tap is source cell n; dpos[0] (+)= dout[0].
// One workgroup per source row, a gather over every output cell: no atomics, one summation order.
__global__ void pos_bicubic_bwd_kernel(const float* __restrict__ dout, float* __restrict__ dpos, int sg, int OH,
                                       int OW, int C, float inv_h, float inv_w, int accumulate) {
  const int n = blockIdx.x;  // 0 = CLS row
  for (int c = threadIdx.x; c < C; c += blockDim.x) {
    float acc = 0.f;
    if (n == 0) {
      acc = dout[c];
    } else {
      const int sy = (n - 1) / sg, sx = (n - 1) % sg;
      for (int o = 1; o <= OH * OW; ++o) {
        const int oy = (o - 1) / OW, ox = (o - 1) % OW;
        const float ry = inv_h * ((float)oy + 0.5f) - 0.5f, rx = inv_w * ((float)ox + 0.5f) - 0.5f;
        int iy = (int)floorf(ry); iy = iy < sg - 1 ? iy : sg - 1;
        int ix = (int)floorf(rx); ix = ix < sg - 1 ? ix : sg - 1;
        const float ty = fminf(fmaxf(ry - iy, 0.f), 1.f), tx = fminf(fmaxf(rx - ix, 0.f), 1.f);
        float cy[4], cx[4];
        cubic_coeffs(ty, cy);
        cubic_coeffs(tx, cx);
        float wy = 0.f, wx = 0.f;
        for (int i = 0; i < 4; ++i) {
          int yy = iy - 1 + i; yy = yy < 0 ? 0 : (yy > sg - 1 ? sg - 1 : yy);
          if (yy == sy) wy += cy[i];
          int xx = ix - 1 + i; xx = xx < 0 ? 0 : (xx > sg - 1 ? sg - 1 : xx);
          if (xx == sx) wx += cx[i];
        }
        if (wy != 0.f && wx != 0.f) acc += (wy * wx) * dout[(int64_t)o * C + c];
      }
    }
    float* d = dpos + (int64_t)n * C + c;
    *d = accumulate ? *d + acc : acc;
  }
}

hipError_t launch_pos_bicubic_bwd(const float* dout, float* dpos, int64_t sgrid, int64_t OH, int64_t OW, int64_t C,
                                  float inv_h, float inv_w, int accumulate, hipStream_t s) {
  pos_bicubic_bwd_kernel<<<(unsigned)(1 + sgrid * sgrid), 256, 0, s>>>(dout, dpos, (int)sgrid, (int)OH, (int)OW,
                                                                      (int)C, inv_h, inv_w, accumulate);
  return hipGetLastError();
}

// ---------------------------------------------------------------- CLS rows
// X[r*stride + c] = cls[c] + pos0[c]   (timesformer.py:288-305: cat(cls) then + pos_embed[0])
__global__ void cls_init_kernel(float* __restrict__ X, const float* __restrict__ cls, const float* __restrict__ pos0,
                                int64_t rows, int64_t stride, int C) {
  const int64_t r = blockIdx.x;
  for (int c = threadIdx.x; c < C; c += blockDim.x) X[r * stride + c] = cls[c] + pos0[c];
}

hipError_t launch_cls_init(float* X, const float* cls, const float* pos0, int64_t rows, int64_t stride, int64_t C,
                           hipStream_t s) {
  cls_init_kernel<<<(unsigned)rows, 256, 0, s>>>(X, cls, pos0, rows, stride, (int)C);
  return hipGetLastError();
}

// out[b*L][c] = mean_t aux[(b*T + t)][c]  (timesformer.py:162-164; proj is affine, so the
// mean is taken before it -- see DESIGN.md)
template <typename T>
__global__ void cls_mean_kernel(const float* __restrict__ aux, T* __restrict__ out, int Tf, int64_t L, int C) {
  const int64_t b = blockIdx.x;
  const float inv = 1.0f / Tf;
  for (int c = threadIdx.x; c < C; c += blockDim.x) {
    float s = 0.f;
    for (int t = 0; t < Tf; ++t) s += aux[(b * Tf + t) * C + c];
    out[b * L * C + c] = Elem<T>::from_f(s * inv);
  }
}

// T = 8 (the hot path): one thread per (clip, 4 channels), the 8 frame rows' float4 loads issued
// together and summed in the order of the generic kernel (t = 0..7) -- bit-identical to it; the
// generic kernel's 16 workgroups of a 16-clip call each walked 768 channels x 8 dependent loads.
template <typename T>
__global__ __launch_bounds__(64) void cls_mean8_kernel(const float* __restrict__ aux, T* __restrict__ out, int64_t B,
                                                       int64_t L, int C) {
  const int64_t i = (int64_t)blockIdx.x * 64 + threadIdx.x;      // (clip, channel quad)
  const int cq = C >> 2;
  if (i >= B * cq) return;
  const int64_t b = i / cq;
  const int c = (int)(i - b * cq) * 4;
  float4 v[8];
#pragma unroll
  for (int t = 0; t < 8; ++t) v[t] = *reinterpret_cast<const float4*>(aux + (b * 8 + t) * C + c);
  float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
  for (int t = 0; t < 8; ++t) { s.x += v[t].x; s.y += v[t].y; s.z += v[t].z; s.w += v[t].w; }
  const float inv = 1.0f / 8;
  store4(out + b * L * C + c, s.x * inv, s.y * inv, s.z * inv, s.w * inv);
}

hipError_t launch_cls_mean(int dtype, const float* aux, void* out, int64_t B, int64_t T, int64_t L, int64_t C,
                           hipStream_t s) {
  if (T == 8 && C % 4 == 0) {
    const unsigned grid = (unsigned)((B * (C / 4) + 63) / 64);
    if (dtype == 0) cls_mean8_kernel<bf16_t><<<grid, 64, 0, s>>>(aux, (bf16_t*)out, B, L, (int)C);
    else cls_mean8_kernel<float><<<grid, 64, 0, s>>>(aux, (float*)out, B, L, (int)C);
    return hipGetLastError();
  }
  if (dtype == 0) cls_mean_kernel<bf16_t><<<(unsigned)B, 256, 0, s>>>(aux, (bf16_t*)out, (int)T, L, (int)C);
  else cls_mean_kernel<float><<<(unsigned)B, 256, 0, s>>>(aux, (float*)out, (int)T, L, (int)C);
  return hipGetLastError();
}

// y[b][i] = mean_t x[(b*T + t)][i]   (space_only prediction average, timesformer.py:338-340)
__global__ void frame_mean_kernel(const float* __restrict__ x, float* __restrict__ y, int Tf, int64_t rowlen) {
  const int64_t b = blockIdx.y;
  const float inv = 1.0f / Tf;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < rowlen; i += (int64_t)gridDim.x * blockDim.x) {
    float s = 0.f;
    for (int t = 0; t < Tf; ++t) s += x[(b * Tf + t) * rowlen + i];
    y[b * rowlen + i] = s * inv;
  }
}

// Many rows per mean (Video Swin's AdaptiveAvgPool3d over D*H*W = 98 token rows per clip): one
// workgroup per (b, 64 columns), each of its 4 waves sums every 4th row, the 4 partials are added
// in wave order through LDS (one fixed summation order).  The kernel above walks all T rows in one
// thread: 24 us for config 5's [8 x 98, 768].
__global__ __launch_bounds__(256) void frame_mean_split_kernel(const float* __restrict__ x, float* __restrict__ y,
                                                               int Tf, int64_t rowlen) {
  __shared__ float part[4][64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int64_t b = blockIdx.y, i = (int64_t)blockIdx.x * 64 + lane;
  float s = 0.f;
  if (i < rowlen)
    for (int t = wave; t < Tf; t += 4) s += x[(b * Tf + t) * rowlen + i];
  part[wave][lane] = s;
  __syncthreads();
  if (wave == 0 && i < rowlen) y[b * rowlen + i] = (((part[0][lane] + part[1][lane]) + part[2][lane]) + part[3][lane]) / Tf;
}

hipError_t launch_frame_mean(const float* x, float* y, int64_t B, int64_t T, int64_t rowlen, hipStream_t s) {
  if (T > 16) {
    frame_mean_split_kernel<<<dim3((unsigned)((rowlen + 63) / 64), (unsigned)B), 256, 0, s>>>(x, y, (int)T, rowlen);
    return hipGetLastError();
  }
  unsigned bx = (unsigned)((rowlen + 255) / 256);
  if (bx > 1024) bx = 1024;
  frame_mean_kernel<<<dim3(bx, (unsigned)B), 256, 0, s>>>(x, y, (int)T, rowlen);
  return hipGetLastError();
}

}  // namespace dsvt
