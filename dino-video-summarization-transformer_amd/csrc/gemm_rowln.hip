// Full-row residual GEMM with the following LayerNorm fused into its epilogue (bf16 perf mode,
// N = 768 = the ViT-B embed dim):
//
//   X[xrow(m)] += A[m] . W^T + bias                 fp32 residual stream (timesformer.py:133-135,
//                                                   181, 184: temporal_fc / attn.proj / mlp.fc2)
//   Y[yrow(m)]  = LN(X[xrow(m)]) * gamma + beta      bf16 A operand of the next QKV / fc1 GEMM
//                                                   (norm1 / norm2 / next block's temporal_norm1)
//
// Why full rows: the LayerNorm of a row needs all 768 updated values.  A 2-D tiled GEMM
// writes X and a separate LayerNorm kernel reads all of X back (77 MB per 25k-row call); here
// each workgroup owns whole rows, so the statistics are a cross-wave reduction in LDS and the
// normalized row leaves straight from registers.
//
// Geometry: one 512-thread workgroup per CU, rows dealt out in 16-row units, contiguous and
// balanced (25 104 rows = 1 569 units -> 6 or 7 per workgroup); a workgroup computes up to MU
// units x 768 columns in one pass over K (more units: several passes).  Wave w owns columns
// [96w, 96w + 96): acc[MU][6] 16x16 fragments (168 VGPRs at MU = 7), v_mfma_f32_16x16x32_bf16
// with the W fragment as the A operand (a lane ends with 4 consecutive columns of one row).
//
// K advances 32 per step.  LDS: W slab 768 rows x 64 B (48 KiB) double-buffered, A slab MU x
// 16 rows x 64 B in a 4-slot ring, every slot its own __shared__ array and the K loop unrolled
// by 4 so each slot is named statically: the compiler then sees which LDS-DMA writes a
// fragment read can alias (only its own slot's) and its inserted waits match the intended
// counts instead of draining every prefetch.  Every wave stages exactly the W rows it
// multiplies (its own 6 x 1 KiB pieces); unit u's A piece is staged by wave u, so one barrier
// per step makes the A slab visible.  Step k: wait for this wave's W(k) (its A(k+2) stays in
// flight), barrier, the MU + 6 fragment reads, W(k+1) and A(k+3) issued, the MU x 6 MFMAs.
// 64-byte LDS rows: the 16-byte chunk c of row r is stored at chunk (c + 2*((r >> 2) & 3)) & 3,
// which spreads every ds_read_b128 lane group over all 64 banks (the swizzle is applied to the
// DMA source address).
#include "common.h"

namespace dsvt {

namespace {

constexpr int RL_N = 768;                 // output columns
constexpr int RL_NW = 8;                  // waves per workgroup (two per SIMD: 256 registers each)
constexpr int RL_NJ = 6;                  // 16-column MFMA tiles per wave (8 waves x 96 columns)
constexpr int RL_ROWB = 64;               // bytes per staged row: 32 bf16 of K
constexpr int RL_WSLAB = RL_N * RL_ROWB;  // 48 KiB
constexpr int RL_MAXU = 7;                // units per pass (an A ring slot holds RL_MAXU KiB)

template <int N>
__device__ __forceinline__ void rl_vmwait() {
  static_assert(N >= 0 && N < 64, "vmcnt immediate");
  __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | 0x0F70);
}

__device__ __forceinline__ void rl_barrier() {
  __builtin_amdgcn_sched_barrier(0);
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
}

__device__ __forceinline__ int rl_phys(int r, int c) { return (c + 2 * ((r >> 2) & 3)) & 3; }
__device__ __forceinline__ int rl_logical(int r, int c) { return (c - 2 * ((r >> 2) & 3)) & 3; }

// Y row for X row xr: ROWLN_Y_X = xr (full layout), ROWLN_Y_COMPACT = index among the patch
// rows (CLS rows -- xr % L == 0 -- have none: -1).
__device__ __forceinline__ int64_t rl_yrow(const RowLnParams& p, int64_t xr) {
  if (p.ymode == ROWLN_Y_COMPACT) {
    const int64_t c = xr / p.L, t = xr - c * p.L;
    return t == 0 ? -1 : c * (p.L - 1) + t - 1;
  }
  return xr;
}

// the LDS buffers, each its own object (see the header comment)
__shared__ __attribute__((aligned(16))) char rl_w0[RL_WSLAB];
__shared__ __attribute__((aligned(16))) char rl_w1[RL_WSLAB];
__shared__ __attribute__((aligned(16))) char rl_a0[RL_MAXU * 1024];
__shared__ __attribute__((aligned(16))) char rl_a1[RL_MAXU * 1024];
__shared__ __attribute__((aligned(16))) char rl_a2[RL_MAXU * 1024];
__shared__ __attribute__((aligned(16))) char rl_a3[RL_MAXU * 1024];
__shared__ __attribute__((aligned(16))) float rl_vec[3 * RL_N];                 // bias, gamma, beta
__shared__ __attribute__((aligned(16))) float rl_red[RL_MAXU * 2 * 16 * RL_NW];  // row partials

}  // namespace

template <int MU>
__global__ __launch_bounds__(512, 1) void gemm_rowln_kernel(RowLnParams p) {
  static_assert(MU >= 1 && MU <= RL_MAXU && MU <= RL_NW, "units per pass");
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r16 = lane & 15, g = lane >> 4;
  const int64_t U = (p.M + 15) >> 4;
  const int64_t G = gridDim.x, b = blockIdx.x;
  const int64_t u_begin = b * U / G, u_end = (b + 1) * U / G;
  const int nk = (int)(p.K >> 5);                   // a multiple of 4 (host check)
  const int64_t lda_b = p.lda * 2, ldw_b = p.ldw * 2;   // byte extents below 2^32 (host check)
  const bool has_a = wave < MU;                     // wave u stages unit u's A piece

  // DMA lane role inside a 1 KiB piece: LDS row prow, physical chunk pch <- logical chunk lch.
  // Sources are a scalar base + a 32-bit lane offset (the saddr form of global_load_lds).
  const int prow = lane >> 2, pch = lane & 3;
  const int lch = rl_logical(prow, pch);
  const char* const Wg = (const char*)p.W;
  const char* const Ag = (const char*)p.A;
  const uint32_t wvoff = (uint32_t)((wave * RL_NJ * 16 + prow) * ldw_b + lch * 16);
  const uint32_t wq = (uint32_t)(16 * ldw_b);      // W source stride between pieces (uniform)
  const int frag = r16 * RL_ROWB + rl_phys(r16, g) * 16;   // fragment read offset in a piece
  const int col0 = wave * (RL_NJ * 16) + 4 * g;     // first output column of this lane

  for (int c = tid; c < RL_N; c += 64 * RL_NW) {   // visible after the first K-step barrier
    rl_vec[c] = p.bias ? p.bias[c] : 0.f;
    rl_vec[RL_N + c] = p.gamma ? p.gamma[c] : 0.f;
    rl_vec[2 * RL_N + c] = p.beta ? p.beta[c] : 0.f;
  }

  for (int64_t c0 = u_begin; c0 < u_end; c0 += MU) {
    const int64_t m0 = c0 * 16;
    int64_t ar = m0 + wave * 16 + prow;
    ar = ar < p.M ? ar : p.M - 1;                   // rows past M re-read the last row (masked)
    const uint32_t avoff = (uint32_t)(ar * lda_b + lch * 16);

    // stage K-step k (clamped: steps past the end re-load the last slab into a slot nobody
    // reads again, so every step issues the same loads and waits the same counts)
    auto stage_w = [&](char* wdst, int k) {
      const int kk = k < nk ? k : nk - 1;
#pragma unroll
      for (int q = 0; q < RL_NJ; ++q)
        __builtin_amdgcn_global_load_lds((const void*)(Wg + (wvoff + (uint32_t)(kk * 64) + (uint32_t)q * wq)),
                                         LDS_PTR(wdst + (wave * RL_NJ + q) * 1024), 16, 0, 0);
    };
    auto stage_a = [&](char* adst, int k) {
      const int kk = k < nk ? k : nk - 1;
      if (has_a)
        __builtin_amdgcn_global_load_lds((const void*)(Ag + (avoff + (uint32_t)(kk * 64))),
                                         LDS_PTR(adst + wave * 1024), 16, 0, 0);
    };

    // zero-initialised accumulators (a bias-initialised chain makes the compiler keep a second
    // copy of every accumulator); the bias is added in the epilogue
    fv4 acc[MU][RL_NJ];
#pragma unroll
    for (int i = 0; i < MU; ++i)
#pragma unroll
      for (int j = 0; j < RL_NJ; ++j) acc[i][j] = fv4{0.f, 0.f, 0.f, 0.f};

    // one K step: wcur / acur hold step k; W(k+1) -> wnxt, A(k+3) -> aiss (the slot step k-1 read)
    auto step = [&](const char* wcur, const char* acur, char* wnxt, char* aiss, int k) {
      if (has_a) rl_vmwait<1>();                    // this wave's W(k) landed, its A(k+2) in flight
      else rl_vmwait<0>();
      rl_barrier();                                 // every wave's A(k) piece landed; step k-1 reads done
      sv8 af[MU], wf[RL_NJ];
#pragma unroll
      for (int i = 0; i < MU; ++i) af[i] = *reinterpret_cast<const sv8*>(acur + i * 1024 + frag);
#pragma unroll
      for (int j = 0; j < RL_NJ; ++j) wf[j] = *reinterpret_cast<const sv8*>(wcur + (wave * RL_NJ + j) * 1024 + frag);
      stage_w(wnxt, k + 1);
      stage_a(aiss, k + 3);
#pragma unroll
      for (int i = 0; i < MU; ++i)
#pragma unroll
        for (int j = 0; j < RL_NJ; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[j], af[i], acc[i][j], 0, 0, 0);
    };

    // prologue in the steady-state issue order: A(0) A(1) W(0) A(2)
    stage_a(rl_a0, 0);
    stage_a(rl_a1, 1);
    stage_w(rl_w0, 0);
    stage_a(rl_a2, 2);
    for (int k = 0; k < nk; k += 4) {
      step(rl_w0, rl_a0, rl_w1, rl_a3, k);
      step(rl_w1, rl_a1, rl_w0, rl_a0, k + 1);
      step(rl_w0, rl_a2, rl_w1, rl_a1, k + 2);
      step(rl_w1, rl_a3, rl_w0, rl_a2, k + 3);
    }

    // ---- epilogue, one 16-row unit at a time (only that unit's 24 values are held beside the
    // accumulators): v = acc + bias + X -> X; row mean and variance by a two-level reduction
    // (4 lane groups, then the 8 waves through LDS); Y = (v - mean) * rstd * gamma + beta.
    rl_vmwait<0>();                                 // the clamped tail stages
    mfma_result_fence();
    const int nu = (int)((u_end - c0) < MU ? (u_end - c0) : MU);
    const bool ln = p.ymode != ROWLN_Y_NONE;
    const float* vb = rl_vec + col0;
#pragma unroll
    for (int i = 0; i < MU; ++i) {
      __builtin_amdgcn_sched_barrier(0);            // one unit at a time: short live ranges
      int64_t m = m0 + i * 16 + r16;
      const bool valid = i < nu && m < p.M;
      m = m < p.M ? m : p.M - 1;
      const int64_t xr = map_row(m, p.rpg, p.gstride, p.goff);
      float* xo = p.X + xr * RL_N + col0;
      fv4 v[RL_NJ];
      float s = 0.f;
#pragma unroll
      for (int j = 0; j < RL_NJ; ++j) {
        const float4 xx = *reinterpret_cast<const float4*>(xo + j * 16);
        const float4 bb = *reinterpret_cast<const float4*>(vb + j * 16);
        v[j] = fv4{acc[i][j][0] + bb.x + xx.x, acc[i][j][1] + bb.y + xx.y, acc[i][j][2] + bb.z + xx.z,
                   acc[i][j][3] + bb.w + xx.w};
        s += (v[j][0] + v[j][1]) + (v[j][2] + v[j][3]);
      }
      if (valid) {
#pragma unroll
        for (int j = 0; j < RL_NJ; ++j) *reinterpret_cast<fv4*>(xo + j * 16) = v[j];
      }
      if (!ln) continue;
      float* rs = rl_red + i * 2 * 16 * RL_NW;      // this unit's [16 rows][8 waves] sums, then squares
      s += __shfl_xor(s, 16, 64);
      s += __shfl_xor(s, 32, 64);
      if (g == 0) rs[r16 * RL_NW + wave] = s;
      __syncthreads();
      const float4 s0 = *reinterpret_cast<const float4*>(rs + r16 * RL_NW);
      const float4 s1 = *reinterpret_cast<const float4*>(rs + r16 * RL_NW + 4);
      const float mean = (((s0.x + s0.y) + (s0.z + s0.w)) + ((s1.x + s1.y) + (s1.z + s1.w))) * (1.0f / RL_N);
      float q = 0.f;
#pragma unroll
      for (int j = 0; j < RL_NJ; ++j)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float d = v[j][e] - mean;
          q += d * d;
        }
      q += __shfl_xor(q, 16, 64);
      q += __shfl_xor(q, 32, 64);
      if (g == 0) rs[16 * RL_NW + r16 * RL_NW + wave] = q;
      __syncthreads();
      const float4 q0 = *reinterpret_cast<const float4*>(rs + 16 * RL_NW + r16 * RL_NW);
      const float4 q1 = *reinterpret_cast<const float4*>(rs + 16 * RL_NW + r16 * RL_NW + 4);
      const float var = (((q0.x + q0.y) + (q0.z + q0.w)) + ((q1.x + q1.y) + (q1.z + q1.w))) * (1.0f / RL_N);
      const float rstd = 1.0f / sqrtf(var + p.eps);
      const int64_t yr = rl_yrow(p, xr);
      if (valid && yr >= 0) {
        bf16_t* yo = p.Y + yr * RL_N + col0;
#pragma unroll
        for (int j = 0; j < RL_NJ; ++j) {
          const float4 gm = *reinterpret_cast<const float4*>(vb + RL_N + j * 16);
          const float4 bt = *reinterpret_cast<const float4*>(vb + 2 * RL_N + j * 16);
          store4(yo + j * 16, (v[j][0] - mean) * rstd * gm.x + bt.x, (v[j][1] - mean) * rstd * gm.y + bt.y,
                 (v[j][2] - mean) * rstd * gm.z + bt.z, (v[j][3] - mean) * rstd * gm.w + bt.w);
        }
      }
    }
    rl_barrier();                                   // `rl_red` reads done before the next pass
  }
}

hipError_t launch_gemm_rowln(const RowLnParams& p, hipStream_t s) {
  const int64_t U = (p.M + 15) / 16;
  int64_t G = 256;                                  // one workgroup per CU
  if (U < G) G = U;
  const int64_t mu = (U + G - 1) / G;               // > 7: several passes of 7
  dim3 grid((unsigned)G), block(64 * RL_NW);
  if (mu <= 1) gemm_rowln_kernel<1><<<grid, block, 0, s>>>(p);
  else if (mu <= 2) gemm_rowln_kernel<2><<<grid, block, 0, s>>>(p);
  else if (mu <= 4) gemm_rowln_kernel<4><<<grid, block, 0, s>>>(p);
  else gemm_rowln_kernel<7><<<grid, block, 0, s>>>(p);
  return hipGetLastError();
}

}  // namespace dsvt
