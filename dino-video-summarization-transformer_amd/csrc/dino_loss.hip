// DINO loss (K13) and center update (K14).  All fp32, HBM-bound, deterministic (fixed
// reduction orders, no float atomics), no host synchronization.
//
// DINOLoss.forward (train_ssl.py:653-671):
//   q_iq = softmax((t_iq - center)/tt)           per teacher row
//   CE(q, s_v) = sum_j -q_j * log_softmax(s_v/ts)_j = sum_j q_j * (lse_v - s_vj/ts)
//   loss = 1/(n_terms*B) * sum_{iq} sum_{v != iq} sum_b CE(q_{iq,b}, s_{v,b})
// pairwise (dino_similarity.py:129-135): CE of row r against row r.
#include <math.h>

#include "common.h"

namespace dsvt {

// Block-wide reductions over NW waves (DPP inside each wave, one LDS exchange across waves).
template <int NW>
__device__ __forceinline__ float block_sum(float v, float* red) {
  v = wave_sum_dpp(v);
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  __syncthreads();
  if (lane == 0) red[wave] = v;
  __syncthreads();
  float t = 0.f;
#pragma unroll
  for (int w = 0; w < NW; ++w) t += red[w];
  return t;
}
template <int NW>
__device__ __forceinline__ float block_max(float v, float* red) {
  v = wave_max(v);
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  __syncthreads();
  if (lane == 0) red[wave] = v;
  __syncthreads();
  float t = -INFINITY;
#pragma unroll
  for (int w = 0; w < NW; ++w) t = fmaxf(t, red[w]);
  return t;
}

// One workgroup of 1024 threads per row; each thread's columns are read in batches of SB float4
// (all loads of a batch in flight together -- one load per iteration left these latency-bound,
// 47 us for a 65536-wide row); a row of <= 1024*4*SB columns stays in registers between the
// max and the exp-sum pass (one HBM read).
constexpr int SM_NW = 16, SB = 16;
constexpr int64_t SM_SPAN = 1024 * 4;      // columns per batch slot

__device__ __forceinline__ float4 centered(const float* xr, const float* center, int64_t j) {
  float4 v = *reinterpret_cast<const float4*>(xr + j);
  if (center) {
    const float4 c = *reinterpret_cast<const float4*>(center + j);
    v.x -= c.x; v.y -= c.y; v.z -= c.z; v.w -= c.w;
  }
  return v;
}

// Per row: m = max_j z_j, Z = sum_j exp(z_j - m), z = (x - center) * inv_temp.  D % 4 == 0.
__global__ __launch_bounds__(1024) void softmax_stats_kernel(const float* __restrict__ x, const float* __restrict__ center,
                                                             float inv_temp, int64_t D, float* m_out, float* z_out) {
  __shared__ float red[SM_NW];
  const int64_t r = blockIdx.x;
  const float* xr = x + r * D;
  const int64_t j0 = threadIdx.x * 4;
  float mx = -INFINITY;
  // (x-c)*inv_temp is monotone in (x-c) for inv_temp > 0: max commutes with the scale
  if (D <= SM_SPAN * SB) {
    float4 v[SB];
#pragma unroll
    for (int u = 0; u < SB; ++u) {
      const int64_t j = j0 + u * SM_SPAN;
      v[u] = j < D ? centered(xr, center, j) : make_float4(-INFINITY, -INFINITY, -INFINITY, -INFINITY);
    }
#pragma unroll
    for (int u = 0; u < SB; ++u) mx = fmaxf(mx, fmaxf(fmaxf(v[u].x, v[u].y), fmaxf(v[u].z, v[u].w)) * inv_temp);
    mx = block_max<SM_NW>(mx, red);
    float s = 0.f;
#pragma unroll
    for (int u = 0; u < SB; ++u)
      if (j0 + u * SM_SPAN < D)
        s += expf(v[u].x * inv_temp - mx) + expf(v[u].y * inv_temp - mx) + expf(v[u].z * inv_temp - mx) +
             expf(v[u].w * inv_temp - mx);
    s = block_sum<SM_NW>(s, red);
    if (threadIdx.x == 0) { m_out[r] = mx; z_out[r] = s; }
    return;
  }
  for (int64_t jb = j0; jb < D; jb += SM_SPAN * SB) {
    float4 v[SB];
#pragma unroll
    for (int u = 0; u < SB; ++u) {
      const int64_t j = jb + u * SM_SPAN;
      v[u] = j < D ? centered(xr, center, j) : make_float4(-INFINITY, -INFINITY, -INFINITY, -INFINITY);
    }
#pragma unroll
    for (int u = 0; u < SB; ++u) mx = fmaxf(mx, fmaxf(fmaxf(v[u].x, v[u].y), fmaxf(v[u].z, v[u].w)) * inv_temp);
  }
  mx = block_max<SM_NW>(mx, red);
  float s = 0.f;
  for (int64_t jb = j0; jb < D; jb += SM_SPAN * SB) {
    float4 v[SB];
#pragma unroll
    for (int u = 0; u < SB; ++u) {
      const int64_t j = jb + u * SM_SPAN;
      v[u] = j < D ? centered(xr, center, j) : make_float4(0.f, 0.f, 0.f, 0.f);
    }
#pragma unroll
    for (int u = 0; u < SB; ++u)
      if (jb + u * SM_SPAN < D)
        s += expf(v[u].x * inv_temp - mx) + expf(v[u].y * inv_temp - mx) + expf(v[u].z * inv_temp - mx) +
             expf(v[u].w * inv_temp - mx);
  }
  s = block_sum<SM_NW>(s, red);
  if (threadIdx.x == 0) { m_out[r] = mx; z_out[r] = s; }
}

hipError_t launch_softmax_stats(const float* x, const float* center, float inv_temp, int64_t rows, int64_t D,
                                float* m_out, float* z_out, hipStream_t s) {
  softmax_stats_kernel<<<(unsigned)rows, 1024, 0, s>>>(x, center, inv_temp, D, m_out, z_out);
  return hipGetLastError();
}

// One workgroup (1024 threads) per (teacher row, student row) pair.  global_crops == 0: pair p
// = rows (p, p) (frame scoring); else p = pair_idx*B + b over the (iq, v != iq) terms in the
// reference's loop order (train_ssl.py:661-669).  Columns in batches of SB float4 per operand.
__global__ __launch_bounds__(1024) void pair_ce_kernel(const float* __restrict__ student, const float* __restrict__ teacher,
                                                       const float* __restrict__ center, int64_t B, int64_t ncrops,
                                                       int64_t global_crops, int64_t D, float inv_ts, float inv_tt,
                                                       const float* t_m, const float* t_z, const float* s_m,
                                                       const float* s_z, float* ce) {
  __shared__ float red[SM_NW];
  const int64_t p = blockIdx.x;
  int64_t rt, rs;
  if (global_crops == 0) {
    rt = p; rs = p;
  } else {
    const int64_t pair = p / B, b = p % B;
    const int64_t iq = pair / (ncrops - 1), vv = pair % (ncrops - 1);
    const int64_t v = vv < iq ? vv : vv + 1;
    rt = iq * B + b; rs = v * B + b;
  }
  const float* tr = teacher + rt * D;
  const float* sr = student + rs * D;
  const float tm = t_m[rt], tz_inv = 1.0f / t_z[rt];
  const float lse = s_m[rs] + logf(s_z[rs]);
  constexpr int PB = SB / 2;                 // two operands per column: half the batch depth
  float acc = 0.f;
  for (int64_t jb = threadIdx.x * 4; jb < D; jb += SM_SPAN * PB) {
    float4 tv[PB], sv[PB];
#pragma unroll
    for (int u = 0; u < PB; ++u) {
      const int64_t j = jb + u * SM_SPAN;
      if (j < D) {
        tv[u] = centered(tr, center, j);
        sv[u] = *reinterpret_cast<const float4*>(sr + j);
      }
    }
#pragma unroll
    for (int u = 0; u < PB; ++u) {
      if (jb + u * SM_SPAN < D) {
        acc += expf(tv[u].x * inv_tt - tm) * tz_inv * (lse - sv[u].x * inv_ts);
        acc += expf(tv[u].y * inv_tt - tm) * tz_inv * (lse - sv[u].y * inv_ts);
        acc += expf(tv[u].z * inv_tt - tm) * tz_inv * (lse - sv[u].z * inv_ts);
        acc += expf(tv[u].w * inv_tt - tm) * tz_inv * (lse - sv[u].w * inv_ts);
      }
    }
  }
  acc = block_sum<SM_NW>(acc, red);
  if (threadIdx.x == 0) ce[p] = acc;
}

hipError_t launch_pair_ce(const float* student, const float* teacher, const float* center, const int32_t*,
                          int64_t npairs, int64_t B, int64_t ncrops, int64_t global_crops, int64_t D, float inv_ts,
                          float inv_tt, const float* t_m, const float* t_z, const float* s_m, const float* s_z,
                          float* ce, hipStream_t s) {
  pair_ce_kernel<<<(unsigned)npairs, 1024, 0, s>>>(student, teacher, center, B, ncrops, global_crops, D, inv_ts, inv_tt,
                                                   t_m, t_z, s_m, s_z, ce);
  return hipGetLastError();
}

// loss = scale * sum_p ce[p], summed in a fixed order (double) by one thread.
__global__ void loss_reduce_kernel(const float* ce, int64_t n, float scale, float* out) {
  if (threadIdx.x == 0 && blockIdx.x == 0) {
    double s = 0.0;
    for (int64_t i = 0; i < n; ++i) s += ce[i];
    out[0] = (float)(s * scale);
  }
}

hipError_t launch_loss_reduce(const float* ce, int64_t npairs, float scale, float* out, hipStream_t s) {
  loss_reduce_kernel<<<1, 64, 0, s>>>(ce, npairs, scale, out);
  return hipGetLastError();
}

// colsum[j] = sum_r x[r][j]  (train_ssl.py:686, before the all-reduce); row order fixed.
__global__ void colsum_kernel(const float* __restrict__ x, int64_t rows, int64_t D, float* __restrict__ out) {
  for (int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j < D; j += (int64_t)gridDim.x * blockDim.x) {
    float s = 0.f;
    for (int64_t r = 0; r < rows; ++r) s += x[r * D + j];
    out[j] = s;
  }
}

hipError_t launch_colsum(const float* x, int64_t rows, int64_t D, float* out, hipStream_t s) {
  unsigned blocks = (unsigned)((D + 255) / 256);
  if (blocks > 2048) blocks = 2048;
  colsum_kernel<<<blocks, 256, 0, s>>>(x, rows, D, out);
  return hipGetLastError();
}

// center = center*momentum + colsum*inv_count*(1-momentum)   (train_ssl.py:687-691)
__global__ void center_ema_kernel(float* __restrict__ center, const float* __restrict__ colsum, int64_t D,
                                  float momentum, float inv_count) {
  for (int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j < D; j += (int64_t)gridDim.x * blockDim.x)
    center[j] = center[j] * momentum + (colsum[j] * inv_count) * (1.0f - momentum);
}

hipError_t launch_center_ema(float* center, const float* colsum, int64_t D, float momentum, float inv_count,
                             hipStream_t s) {
  unsigned blocks = (unsigned)((D + 255) / 256);
  if (blocks > 2048) blocks = 2048;
  center_ema_kernel<<<blocks, 256, 0, s>>>(center, colsum, D, momentum, inv_count);
  return hipGetLastError();
}

}  // namespace dsvt
