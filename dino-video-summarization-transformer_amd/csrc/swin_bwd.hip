// Video Swin training (models/swin_transformer.py, the `--arch swin` student of train_ssl.py:
// 237-239): the backward pieces the Swin layers need beside the shared GEMM / wgrad / LayerNorm
// backward kernels.
//
//   swin_gather_rows_kernel   out[m] = cast(s[m / group] * x[idx[m]]), zero rows for idx < 0 and
//                             zero K-padding columns: the window-row gradient of the attention
//                             branch (window_partition of the token gradient, the DropPath scale
//                             of the sample), row-scaled / padded casts and the PatchMerging 2x2
//                             gather
//   attn_window_bwd_kernel    W-MSA / SW-MSA backward (:139-171): per (head, window group) the
//                             window's q, k, v, dO, O in LDS (fp32), P recomputed from the scores
//                             with the relative-position bias and the shift mask, dV = P^T dO,
//                             dS = P (dP - rowsum(dO O)), dQ = dS K * scale, dK = dS^T Q * scale;
//                             dS summed over the group's windows in registers (one fixed pair
//                             set per thread) and written as one partial per window group: the
//                             bias gradient, reduced in a fixed order (deterministic)
//   relpos_bias_bwd_kernel    d relative_position_bias_table: a gather over the (i, j) pairs of
//                             each table entry (the forward's index map :152-156), no atomics
#include <math.h>

#include "common.h"
#include "internal.h"

namespace dsvt {

namespace {

template <typename T>
__global__ __launch_bounds__(256) void swin_gather_rows_kernel(const float* __restrict__ x, const int32_t* __restrict__ idx,
                                                               const float* __restrict__ row_scale, int64_t group,
                                                               T* __restrict__ out, int64_t rows, int C, int ldo) {
  const int64_t total = rows * ldo;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < total; i += (int64_t)gridDim.x * 256) {
    const int64_t m = i / ldo;
    const int c = (int)(i % ldo);
    const int64_t src = idx ? (int64_t)idx[m] : m;
    float v = 0.f;
    if (c < C && src >= 0) {
      v = x[src * C + c];
      if (row_scale) v *= row_scale[m / group];
    }
    out[i] = Elem<T>::from_f(v);
  }
}

constexpr int WB_NMAX = 128;          // tokens per window (the forward kernel's limit)
constexpr int WB_LD = 33;             // fp32 LDS row of one head's 32 values (+1: bank spread)
constexpr int WB_PAIRS = WB_NMAX * WB_NMAX / 256;   // (i, j) pairs per thread at N = 128

struct WinBwdParams {
  const void* qkv; const void* o; int64_t ldo; const void* dout; int64_t lddo;
  const float* bias; const int32_t* region;
  void* dqkv; int64_t lddq; float* dbias_part;
  int64_t nwin, nwc, N, heads, C;
  float scale;
};

template <typename T>
__global__ __launch_bounds__(256) void attn_window_bwd_kernel(WinBwdParams p) {
  __shared__ float q_s[WB_NMAX * WB_LD], k_s[WB_NMAX * WB_LD], v_s[WB_NMAX * WB_LD], do_s[WB_NMAX * WB_LD];
  __shared__ float P[WB_NMAX * (WB_NMAX + 1)];
  __shared__ float dsum[WB_NMAX];
  const int tid = threadIdx.x;
  const int h = blockIdx.x;
  const int N = (int)p.N, NN = N * N, LDP = WB_NMAX + 1;
  const int64_t C = p.C;
  const float* bias = p.bias + (int64_t)h * NN;
  float dB[WB_PAIRS];
#pragma unroll
  for (int k = 0; k < WB_PAIRS; ++k) dB[k] = 0.f;
  for (int64_t win = blockIdx.y; win < p.nwin; win += gridDim.y) {
    const int64_t r0 = win * N;
    const T* qkv = (const T*)p.qkv + r0 * 3 * C + h * 32;
    // ---- stage q, k, v, dO (fp32) and D_i = dO_i . O_i
    for (int e = tid; e < N * 32; e += 256) {
      const int i = e >> 5, d = e & 31;
      const T* row = qkv + (int64_t)i * 3 * C;
      q_s[i * WB_LD + d] = Elem<T>::to_f(row[d]);
      k_s[i * WB_LD + d] = Elem<T>::to_f(row[C + d]);
      v_s[i * WB_LD + d] = Elem<T>::to_f(row[2 * C + d]);
      do_s[i * WB_LD + d] = Elem<T>::to_f(((const T*)p.dout)[(r0 + i) * p.lddo + h * 32 + d]);
    }
    __syncthreads();
    if (tid < N) {
      const T* orow = (const T*)p.o + (r0 + tid) * p.ldo + h * 32;
      float s = 0.f;
#pragma unroll
      for (int d = 0; d < 32; ++d) s = fmaf(do_s[tid * WB_LD + d], Elem<T>::to_f(orow[d]), s);
      dsum[tid] = s;
    }
    // ---- scores (the forward's: q.k * scale + bias + shift mask)
    const int32_t* reg = p.region + (win % p.nwc) * N;
    for (int e = tid; e < NN; e += 256) {
      const int i = e / N, j = e - i * N;
      float s = 0.f;
#pragma unroll
      for (int d = 0; d < 32; ++d) s = fmaf(q_s[i * WB_LD + d], k_s[j * WB_LD + d], s);
      P[i * LDP + j] = s * p.scale + bias[e] + ((reg[i] != reg[j]) ? -100.0f : 0.0f);
    }
    __syncthreads();
    // ---- softmax rows (one thread per row)
    if (tid < N) {
      float* pr = P + tid * LDP;
      float mx = -INFINITY;
      for (int j = 0; j < N; ++j) mx = fmaxf(mx, pr[j]);
      float l = 0.f;
      for (int j = 0; j < N; ++j) {
        const float e = expf(pr[j] - mx);
        pr[j] = e;
        l += e;
      }
      const float inv = 1.0f / l;
      for (int j = 0; j < N; ++j) pr[j] *= inv;
    }
    __syncthreads();
    T* dq = (T*)p.dqkv + r0 * p.lddq + h * 32;
    // ---- dV_j = sum_i P_ij dO_i
    for (int e = tid; e < N * 32; e += 256) {
      const int j = e >> 5, d = e & 31;
      float s = 0.f;
      for (int i = 0; i < N; ++i) s = fmaf(P[i * LDP + j], do_s[i * WB_LD + d], s);
      dq[(int64_t)j * p.lddq + 2 * C + d] = Elem<T>::from_f(s);
    }
    __syncthreads();
    // ---- dS_ij = P_ij (dO_i . v_j - D_i), in place; the bias gradient accumulates dS
#pragma unroll
    for (int k = 0; k < WB_PAIRS; ++k) {
      const int e = tid + 256 * k;
      if (e < NN) {
        const int i = e / N, j = e - i * N;
        float dp = 0.f;
#pragma unroll
        for (int d = 0; d < 32; ++d) dp = fmaf(do_s[i * WB_LD + d], v_s[j * WB_LD + d], dp);
        const float ds = P[i * LDP + j] * (dp - dsum[i]);
        P[i * LDP + j] = ds;
        dB[k] += ds;
      }
    }
    __syncthreads();
    // ---- dQ_i = scale * sum_j dS_ij k_j ;  dK_j = scale * sum_i dS_ij q_i
    for (int e = tid; e < N * 32; e += 256) {
      const int i = e >> 5, d = e & 31;
      float sq = 0.f, sk = 0.f;
      for (int j = 0; j < N; ++j) {
        sq = fmaf(P[i * LDP + j], k_s[j * WB_LD + d], sq);
        sk = fmaf(P[j * LDP + i], q_s[j * WB_LD + d], sk);
      }
      dq[(int64_t)i * p.lddq + d] = Elem<T>::from_f(sq * p.scale);
      dq[(int64_t)i * p.lddq + C + d] = Elem<T>::from_f(sk * p.scale);
    }
    __syncthreads();             // LDS reused by the next window
  }
  float* part = p.dbias_part + ((int64_t)blockIdx.y * p.heads + h) * NN;
#pragma unroll
  for (int k = 0; k < WB_PAIRS; ++k) {
    const int e = tid + 256 * k;
    if (e < NN) part[e] = dB[k];
  }
}

// dtable[e][h] (+)= sum over i, j < N with index[i][j] == e of dbias[h][i][j]
__global__ __launch_bounds__(256) void relpos_bias_bwd_kernel(const float* __restrict__ dbias,
                                                              const int64_t* __restrict__ index, int nmax, int N,
                                                              int heads, int64_t entries, float* __restrict__ dtable,
                                                              int accumulate) {
  const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (t >= entries * heads) return;
  const int64_t e = t / heads;
  const int h = (int)(t % heads);
  const float* db = dbias + (int64_t)h * N * N;
  float s = 0.f;
  for (int i = 0; i < N; ++i)
    for (int j = 0; j < N; ++j)
      if (index[(int64_t)i * nmax + j] == e) s += db[i * N + j];
  dtable[t] = accumulate ? dtable[t] + s : s;
}

// The same with the head's dbias [N][N] and the index slice staged in LDS once per workgroup
// (grid: entry chunks x heads; the index as int16, 6 bytes per pair: 56 KiB at N = 98): every
// thread's scan reads broadcast LDS words instead of an int64 index and an fp32 value through the
// cache per pair (9.6k pairs at N = 98).  Pairs in the same (i, j) order as above:
// bitwise-equal sums.
__global__ __launch_bounds__(256) void relpos_bias_bwd_lds_kernel(const float* __restrict__ dbias,
                                                                  const int64_t* __restrict__ index, int nmax, int N,
                                                                  int heads, int64_t entries,
                                                                  float* __restrict__ dtable, int accumulate) {
  extern __shared__ __attribute__((aligned(16))) char rb_smem[];
  const int nn = N * N;
  float* sd = reinterpret_cast<float*>(rb_smem);
  short* si = reinterpret_cast<short*>(rb_smem + (size_t)nn * 4);      // entries < 32768
  const int h = blockIdx.y;
  for (int p = threadIdx.x; p < nn; p += 256) {
    si[p] = (short)index[(int64_t)(p / N) * nmax + p % N];
    sd[p] = dbias[(int64_t)h * nn + p];
  }
  __syncthreads();
  const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (e >= entries) return;
  float s = 0.f;
  for (int p = 0; p < nn; ++p)
    if (si[p] == (int)e) s += sd[p];
  const int64_t t = e * heads + h;
  dtable[t] = accumulate ? dtable[t] + s : s;
}

}  // namespace

int64_t attn_window_bwd_groups(int64_t nwin, int64_t heads) {
  int64_t g = 512 / (heads < 1 ? 1 : heads);
  if (g < 1) g = 1;
  return g < nwin ? g : nwin;
}

hipError_t launch_swin_gather_rows(int dtype, const float* x, const int32_t* idx, const float* row_scale,
                                   int64_t group, void* out, int64_t rows, int64_t C, int64_t ldo, hipStream_t s) {
  int64_t blocks = (rows * ldo + 255) / 256;
  if (blocks > 16384) blocks = 16384;
  const unsigned nb = (unsigned)(blocks < 1 ? 1 : blocks);
  if (dtype == 0)
    swin_gather_rows_kernel<bf16_t><<<nb, 256, 0, s>>>(x, idx, row_scale, group, (bf16_t*)out, rows, (int)C, (int)ldo);
  else
    swin_gather_rows_kernel<float><<<nb, 256, 0, s>>>(x, idx, row_scale, group, (float*)out, rows, (int)C, (int)ldo);
  return hipGetLastError();
}

hipError_t launch_attn_window_bwd(int dtype, const void* qkv, const void* o, int64_t ldo, const void* dout,
                                  int64_t lddo, const float* bias, const int32_t* region, int64_t nwin, int64_t nwc,
                                  int64_t N, int64_t heads, int64_t C, float scale, void* dqkv, int64_t lddq,
                                  float* dbias, float* workspace, hipStream_t s) {
  const int64_t G = attn_window_bwd_groups(nwin, heads);
  WinBwdParams p{qkv, o, ldo, dout, lddo, bias, region, dqkv, lddq, workspace, nwin, nwc, N, heads, C, scale};
  const dim3 grid((unsigned)heads, (unsigned)G);
  if (dtype == 0) attn_window_bwd_kernel<bf16_t><<<grid, 256, 0, s>>>(p);
  else attn_window_bwd_kernel<float><<<grid, 256, 0, s>>>(p);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  // dbias[h][i][j] = sum over the window groups, in group order
  return launch_reduce_partials(workspace, G, heads * N * N, heads * N * N, dbias, 0, s);
}

hipError_t launch_relpos_bias_bwd(const float* dbias, const int64_t* index, int64_t nmax, int64_t N, int64_t heads,
                                  int64_t entries, float* dtable, int accumulate, hipStream_t s) {
  const int64_t lds = N * N * 6;
  if (lds <= 64 * 1024 && entries < 32768) {
    relpos_bias_bwd_lds_kernel<<<dim3((unsigned)((entries + 255) / 256), (unsigned)heads), 256, lds, s>>>(
        dbias, index, (int)nmax, (int)N, (int)heads, entries, dtable, accumulate);
    return hipGetLastError();
  }
  const int64_t n = entries * heads;
  relpos_bias_bwd_kernel<<<(unsigned)((n + 255) / 256), 256, 0, s>>>(dbias, index, (int)nmax, (int)N, (int)heads,
                                                                       entries, dtable, accumulate);
  return hipGetLastError();
}

}  // namespace dsvt
