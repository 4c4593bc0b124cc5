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

// bf16 MFMA form (N <= 112: Swin's 2x7x7 = 98-token windows), same grid, partials and outputs.
// Per window: q, k, v, dO rows (bf16, zero past N) in LDS; per 16-query tile (phase 1, one wave):
//   S = K.Q^T and dP = V.dO^T (one 16x16x32 MFMA per 16 keys each, head_dim 32), the forward's
//   score math (scale, bias, -100 shift mask, exp2) -> P; D = dO.O over the row; dS = P (dP - D);
//   dQ = scale dS.K (the forward's P.V form: dS packed as the B operand, K^T by ds_read_tr16_b64);
//   P and dS stored (bf16) to LDS, dS added to the lane's fixed bias-gradient pairs (fp32);
// per 16-key tile (phase 2, one wave): dV = P^T.dO and dK = scale dS^T.Q, both operands by
// transposed reads over 32-query steps.  The head's bias [N][N] is staged in LDS once per
// workgroup (float4 reads).  P / dS enter the MFMAs in bf16 (the VALU kernel above keeps fp32).
constexpr int WM_NP = 112, WM_SN = 7, WM_ROW = 40, WM_PROW = 120, WM_BROW = 116, WM_LPW = 128;
__global__ __launch_bounds__(256) void attn_window_bwd_mfma(WinBwdParams p) {
  __shared__ __attribute__((aligned(16))) bf16_t qs[WM_LPW * WM_ROW], ks[WM_LPW * WM_ROW], vs[WM_LPW * WM_ROW],
      dos[WM_LPW * WM_ROW];
  __shared__ __attribute__((aligned(16))) bf16_t ps[WM_LPW * WM_PROW], dss[WM_LPW * WM_PROW];
  __shared__ __attribute__((aligned(16))) float bs[WM_NP * WM_BROW];
  __shared__ __attribute__((aligned(16))) int rg[WM_NP];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int r16 = lane & 15, g = lane >> 4;
  const int h = blockIdx.x;
  const int N = (int)p.N, nqt = (N + 15) >> 4;
  const int64_t C = p.C;
  const float l2e = 1.4426950408889634f;
  {
    const float* bias = p.bias + (int64_t)h * N * N;
    for (int e = tid; e < WM_NP * WM_NP; e += 256) {
      const int i = e / WM_NP, j = e - i * WM_NP;
      bs[i * WM_BROW + j] = (i < N && j < N) ? bias[i * N + j] : 0.f;
    }
    // P / dS rows past the last query tile stay zero (phase 2 sums over all 128 rows)
    for (int e = tid; e < (WM_LPW - nqt * 16) * (WM_PROW / 4); e += 256) {
      const int r = nqt * 16 + e / (WM_PROW / 4), c = (e % (WM_PROW / 4)) * 4;
      *reinterpret_cast<uint2*>(&ps[r * WM_PROW + c]) = make_uint2(0, 0);
      *reinterpret_cast<uint2*>(&dss[r * WM_PROW + c]) = make_uint2(0, 0);
    }
  }
  float dB[2][WM_SN][4];
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int kt = 0; kt < WM_SN; ++kt)
#pragma unroll
      for (int j = 0; j < 4; ++j) dB[t][kt][j] = 0.f;
  for (int64_t win = blockIdx.y; win < p.nwin; win += gridDim.y) {
    const int64_t r0 = win * N;
    const bf16_t* qkv = (const bf16_t*)p.qkv + r0 * 3 * C + h * 32;
    for (int pc = tid; pc < WM_LPW * 4; pc += 256) {
      const int r = pc >> 2, ch = pc & 3;
      uint4 q4 = make_uint4(0, 0, 0, 0), k4 = q4, v4 = q4, d4 = q4;
      if (r < N) {
        const bf16_t* src = qkv + (int64_t)r * 3 * C + ch * 8;
        q4 = *reinterpret_cast<const uint4*>(src);
        k4 = *reinterpret_cast<const uint4*>(src + C);
        v4 = *reinterpret_cast<const uint4*>(src + 2 * C);
        d4 = *reinterpret_cast<const uint4*>((const bf16_t*)p.dout + (r0 + r) * p.lddo + h * 32 + ch * 8);
      }
      *reinterpret_cast<uint4*>(&qs[r * WM_ROW + ch * 8]) = q4;
      *reinterpret_cast<uint4*>(&ks[r * WM_ROW + ch * 8]) = k4;
      *reinterpret_cast<uint4*>(&vs[r * WM_ROW + ch * 8]) = v4;
      *reinterpret_cast<uint4*>(&dos[r * WM_ROW + ch * 8]) = d4;
    }
    const int32_t* reg = p.region + (win % p.nwc) * N;
    if (tid < WM_NP) rg[tid] = reg[tid < N ? tid : N - 1];
    __syncthreads();
    bf16_t* dq = (bf16_t*)p.dqkv + r0 * p.lddq + h * 32;
    // ---- phase 1: query tiles
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const int qt = wave + 4 * t;
      if (qt >= nqt) break;
      const int qi = qt * 16 + r16;
      const int qc = qi < N ? qi : N - 1;
      const sv8 qf = *reinterpret_cast<const sv8*>(&qs[qc * WM_ROW + g * 8]);
      const sv8 df = *reinterpret_cast<const sv8*>(&dos[qc * WM_ROW + g * 8]);
      // D = dO . O over the row (lane group g: dims 8g..8g+7)
      float dd;
      {
        const uint4 ou = *reinterpret_cast<const uint4*>((const bf16_t*)p.o + (r0 + qc) * p.ldo + h * 32 + g * 8);
        const unsigned ow[4] = {ou.x, ou.y, ou.z, ou.w};
        dd = 0.f;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          dd = fmaf(bf2f((bf16_t)df[2 * e]), __uint_as_float(ow[e] << 16), dd);
          dd = fmaf(bf2f((bf16_t)df[2 * e + 1]), __uint_as_float(ow[e] & 0xffff0000u), dd);
        }
        dd += __shfl_xor(dd, 16, 64);
        dd += __shfl_xor(dd, 32, 64);
      }
      fv4 s[WM_SN], dp[WM_SN];
#pragma unroll
      for (int kt = 0; kt < WM_SN; ++kt) {
        const sv8 kf = *reinterpret_cast<const sv8*>(&ks[(kt * 16 + r16) * WM_ROW + g * 8]);
        const sv8 vf = *reinterpret_cast<const sv8*>(&vs[(kt * 16 + r16) * WM_ROW + g * 8]);
        s[kt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kf, qf, fv4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
        dp[kt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(vf, df, fv4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
      }
      mfma_result_fence();
      const int rq = rg[qc];
      float mx = -INFINITY;
#pragma unroll
      for (int kt = 0; kt < WM_SN; ++kt) {
        const float4 bq = *reinterpret_cast<const float4*>(&bs[qc * WM_BROW + kt * 16 + 4 * g]);
        const int4 rk = *reinterpret_cast<const int4*>(&rg[kt * 16 + 4 * g]);
        const float bb[4] = {bq.x, bq.y, bq.z, bq.w};
        const int rr[4] = {rk.x, rk.y, rk.z, rk.w};
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int key = kt * 16 + 4 * g + j;
          float v = s[kt][j] * p.scale + bb[j] + ((rr[j] != rq) ? -100.0f : 0.0f);
          v = key < N ? v * l2e : -INFINITY;
          s[kt][j] = v;
          mx = fmaxf(mx, v);
        }
      }
      mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
      mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
      float rs = 0.f;
#pragma unroll
      for (int kt = 0; kt < WM_SN; ++kt)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          s[kt][j] = __builtin_amdgcn_exp2f(s[kt][j] - mx);
          rs += s[kt][j];
        }
      rs += __shfl_xor(rs, 16, 64);
      rs += __shfl_xor(rs, 32, 64);
      const float inv = 1.0f / rs;
      const bool qv = qi < N;
#pragma unroll
      for (int kt = 0; kt < WM_SN; ++kt) {
        float pv[4], sv[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          pv[j] = s[kt][j] * inv;                                   // P
          sv[j] = pv[j] * (dp[kt][j] - dd);                         // dS
          dB[t][kt][j] += sv[j];
          s[kt][j] = sv[j];                                         // s now holds dS
          if (!qv) { pv[j] = 0.f; sv[j] = 0.f; }
        }
        *reinterpret_cast<uint2*>(&ps[qi * WM_PROW + kt * 16 + 4 * g]) =
            make_uint2(pack_bf16x2(pv[0], pv[1]), pack_bf16x2(pv[2], pv[3]));
        *reinterpret_cast<uint2*>(&dss[qi * WM_PROW + kt * 16 + 4 * g]) =
            make_uint2(pack_bf16x2(sv[0], sv[1]), pack_bf16x2(sv[2], sv[3]));
      }
      // dQ = scale * dS . K
      fv4 o[2] = {fv4{0.f, 0.f, 0.f, 0.f}, fv4{0.f, 0.f, 0.f, 0.f}};
#pragma unroll
      for (int kp = 0; kp < 4; ++kp) {
        sv8 pb;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          pb[j] = (short)f2bf(s[2 * kp][j]);
          pb[4 + j] = (2 * kp + 1 < WM_SN) ? (short)f2bf(s[(2 * kp + 1) % WM_SN][j]) : (short)0;
        }
        const int vr0 = kp * 32 + 4 * g + (r16 >> 2), vr1 = vr0 + 16;
#pragma unroll
        for (int dt = 0; dt < 2; ++dt) {
          const int col = dt * 16 + 4 * (r16 & 3);
          const sv4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) sv4*)(&ks[vr0 * WM_ROW + col]));
          const sv4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) sv4*)(&ks[vr1 * WM_ROW + col]));
          o[dt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7), pb,
                                                          o[dt], 0, 0, 0);
        }
      }
      mfma_result_fence();
      if (qv) {
#pragma unroll
        for (int dt = 0; dt < 2; ++dt)
          store4(dq + (int64_t)qi * p.lddq + dt * 16 + 4 * g, o[dt][0] * p.scale, o[dt][1] * p.scale,
                 o[dt][2] * p.scale, o[dt][3] * p.scale);
      }
    }
    __syncthreads();
    // ---- phase 2: key tiles -- dV = P^T.dO, dK = scale * dS^T.Q
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const int kt2 = wave + 4 * t;
      if (kt2 >= nqt) break;
      fv4 dv[2] = {fv4{0.f, 0.f, 0.f, 0.f}, fv4{0.f, 0.f, 0.f, 0.f}};
      fv4 dk[2] = {fv4{0.f, 0.f, 0.f, 0.f}, fv4{0.f, 0.f, 0.f, 0.f}};
#pragma unroll
      for (int qp = 0; qp < 4; ++qp) {
        const int vr0 = qp * 32 + 4 * g + (r16 >> 2), vr1 = vr0 + 16;
        const int pc = kt2 * 16 + 4 * (r16 & 3);
        typedef __attribute__((address_space(3))) sv4* L4;
        const sv4 plo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((L4)(&ps[vr0 * WM_PROW + pc]));
        const sv4 phi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((L4)(&ps[vr1 * WM_PROW + pc]));
        const sv4 slo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((L4)(&dss[vr0 * WM_PROW + pc]));
        const sv4 shi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((L4)(&dss[vr1 * WM_PROW + pc]));
        const sv8 pT = __builtin_shufflevector(plo, phi, 0, 1, 2, 3, 4, 5, 6, 7);
        const sv8 sT = __builtin_shufflevector(slo, shi, 0, 1, 2, 3, 4, 5, 6, 7);
#pragma unroll
        for (int dt = 0; dt < 2; ++dt) {
          const int col = dt * 16 + 4 * (r16 & 3);
          const sv4 dlo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((L4)(&dos[vr0 * WM_ROW + col]));
          const sv4 dhi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((L4)(&dos[vr1 * WM_ROW + col]));
          const sv4 qlo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((L4)(&qs[vr0 * WM_ROW + col]));
          const sv4 qhi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((L4)(&qs[vr1 * WM_ROW + col]));
          dv[dt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_shufflevector(dlo, dhi, 0, 1, 2, 3, 4, 5, 6, 7), pT,
                                                           dv[dt], 0, 0, 0);
          dk[dt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_shufflevector(qlo, qhi, 0, 1, 2, 3, 4, 5, 6, 7), sT,
                                                           dk[dt], 0, 0, 0);
        }
      }
      mfma_result_fence();
      const int k = kt2 * 16 + r16;
      if (k < N) {
#pragma unroll
        for (int dt = 0; dt < 2; ++dt) {
          bf16_t* row = dq + (int64_t)k * p.lddq + dt * 16 + 4 * g;
          store4(row + 2 * C, dv[dt][0], dv[dt][1], dv[dt][2], dv[dt][3]);
          store4(row + C, dk[dt][0] * p.scale, dk[dt][1] * p.scale, dk[dt][2] * p.scale, dk[dt][3] * p.scale);
        }
      }
    }
    __syncthreads();             // LDS reused by the next window
  }
  float* part = p.dbias_part + ((int64_t)blockIdx.y * p.heads + h) * N * N;
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    const int qi = (wave + 4 * t) * 16 + r16;
    if (wave + 4 * t >= nqt || qi >= N) continue;
#pragma unroll
    for (int kt = 0; kt < WM_SN; ++kt)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int key = kt * 16 + 4 * g + j;
        if (key < N) part[qi * N + key] = dB[t][kt][j];
      }
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
// (grid: entry chunks x heads; the index as int16, 6 bytes per pair, padded to a multiple of 8
// pairs with index -1: 56 KiB at N = 98), the scan reading 8 pairs per step as one 16-byte index
// load and two 16-byte value loads (broadcast: every lane of the wave reads the same words), then
// adding the matches in pair order -- bitwise the sums of relpos_bias_bwd_kernel.  A one-pair-per-
// step LDS loop is latency bound (~450 us per call at N = 98, 24 heads).
__global__ __launch_bounds__(256) void relpos_bias_bwd_lds_kernel(const float* __restrict__ dbias,
                                                                  const int64_t* __restrict__ index, int nmax, int N,
                                                                  int heads, int64_t entries,
                                                                  float* __restrict__ dtable, int accumulate) {
  extern __shared__ __attribute__((aligned(16))) char rb_smem[];
  const int nn = N * N, nn8 = (nn + 7) & ~7;
  float* sd = reinterpret_cast<float*>(rb_smem);
  short* si = reinterpret_cast<short*>(rb_smem + (size_t)nn8 * 4);     // entries < 32768
  const int h = blockIdx.y;
  for (int p = threadIdx.x; p < nn8; p += 256) {
    const bool in = p < nn;
    si[p] = in ? (short)index[(int64_t)(p / N) * nmax + p % N] : (short)-1;
    sd[p] = in ? dbias[(int64_t)h * nn + p] : 0.f;
  }
  __syncthreads();
  const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (e >= entries) return;
  const short es = (short)e;
  float s = 0.f;
#pragma unroll 4
  for (int p = 0; p < nn8; p += 8) {               // (unrolled: four steps' LDS loads in flight)
    const uint4 iv = *reinterpret_cast<const uint4*>(si + p);
    const float4 va = *reinterpret_cast<const float4*>(sd + p);
    const float4 vb = *reinterpret_cast<const float4*>(sd + p + 4);
    const unsigned w[4] = {iv.x, iv.y, iv.z, iv.w};
    const float v[8] = {va.x, va.y, va.z, va.w, vb.x, vb.y, vb.z, vb.w};
#pragma unroll
    for (int u = 0; u < 8; ++u)
      if ((short)(w[u >> 1] >> (16 * (u & 1))) == es) s += v[u];
  }
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
#ifndef DSVT_WIN_BWD_MFMA
#define DSVT_WIN_BWD_MFMA 1
#endif
  if (dtype == 0 && DSVT_WIN_BWD_MFMA && N <= WM_NP && C % 8 == 0 && ldo % 8 == 0 && lddo % 8 == 0 && lddq % 4 == 0)
    attn_window_bwd_mfma<<<grid, 256, 0, s>>>(p);
  else if (dtype == 0) attn_window_bwd_kernel<bf16_t><<<grid, 256, 0, s>>>(p);
  else attn_window_bwd_kernel<float><<<grid, 256, 0, s>>>(p);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  // dbias[h][i][j] = sum over the window groups, in group order
  return launch_reduce_partials(workspace, G, heads * N * N, heads * N * N, dbias, 0, s);
}

hipError_t launch_relpos_bias_bwd(const float* dbias, const int64_t* index, int64_t nmax, int64_t N, int64_t heads,
                                  int64_t entries, float* dtable, int accumulate, hipStream_t s) {
  const int64_t lds = (N * N + 7) / 8 * 8 * 6;
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
