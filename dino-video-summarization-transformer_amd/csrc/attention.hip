// Attention kernels of the divided space-time block (and the plain/joint variants).
//
// attn_seq_bf16 (K6/K10, perf mode): flash-style, one workgroup = 4 waves = 64 queries of
//   one (sequence, head); K/V streamed through a 2-stage LDS ring in 64-key chunks
//   (register-staged: the rows are GATHERED -- the spatial sequence (b,t) is the CLS row
//   plus every T-th token row of X -- so they cannot use lane-linear LDS-DMA), online
//   softmax in fp32.  S^T = K.Q^T is issued with K as the MFMA A operand so each lane
//   holds 16 scores of ONE query: the row max / sum are in-register + 2 cross-lane xors,
//   and the probabilities feed O^T = V^T.P^T directly as the B operand (k order permuted
//   to match); V^T fragments come from ds_read_b64_tr_b16 transposed LDS reads.
//   Used for sequences longer than 256 keys (joint space-time attention).
// attn_short_bf16 (L <= 256: spatial 1+N per frame, 2-D ViT): one workgroup per (sequence,
//   head) with the whole K/V sequence staged in LDS once, 16-query tiles per wave, 16-key
//   tiles, exact two-pass softmax in registers (1 + 196 keys: XOR-swizzled 52 KB, 3 WGs / CU).
// attn_seq_f32 (parity mode): same decomposition on the fp32 VALU, one query per lane.
// attn_temporal_reg (K5, bf16, T <= 8): register-only, 16 lanes per (patch, head), butterfly
//   reduce-scatter of Q.K^T; HBM-bound.  attn_temporal_kernel: LDS-staged general-T fallback.
#include <math.h>
#include <stdlib.h>

#include "common.h"

namespace dsvt {

__device__ __forceinline__ int64_t tok_row(const AttnParams& p, int64_t b, int64_t t, int64_t i) {
  return b * p.L + (i == 0 ? 0 : 1 + (i - 1) * p.tok_stride + t);
}

// ---------------------------------------------------------------- bf16 MFMA flash kernel
constexpr int KV_ROW = 72;  // bf16 per LDS row: 64 + 8 pad (144 B rows: conflict-light b128 + tr reads)

__global__ __launch_bounds__(256) void attn_seq_bf16(AttnParams p) {
  __shared__ __attribute__((aligned(16))) bf16_t kv[2][2][64 * KV_ROW];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int r16 = lane & 15, g = lane >> 4;
  const int64_t seq = blockIdx.z, b = seq / p.tin, t = seq % p.tin;
  const int h = blockIdx.y;
  const int64_t q0 = (int64_t)blockIdx.x * 64 + wave * 16;
  const bf16_t* qkv = (const bf16_t*)p.qkv;
  const int64_t C = p.C;

  int64_t qi = q0 + r16;
  if (qi > p.seqlen - 1) qi = p.seqlen - 1;
  const bf16_t* qrow = qkv + tok_row(p, b, t, qi) * p.ld_qkv + h * 64;
  const sv8 qf0 = *reinterpret_cast<const sv8*>(qrow + g * 8);
  const sv8 qf1 = *reinterpret_cast<const sv8*>(qrow + 32 + g * 8);

  const int nchunks = (int)((p.seqlen + 63) / 64);
  // K/V staging: thread owns 16-B pieces pc = tid and tid + 256 of the 64x128 B chunk
  const int row_a = tid >> 3, row_b = (tid + 256) >> 3, ch = tid & 7;
  uint4 ka, kb, va, vb;
#define DSVT_LOAD_CHUNK(c)                                                              \
  {                                                                                     \
    int64_t kia = (int64_t)(c) * 64 + row_a, kib = (int64_t)(c) * 64 + row_b;           \
    kia = kia < p.seqlen ? kia : p.seqlen - 1;                                          \
    kib = kib < p.seqlen ? kib : p.seqlen - 1;                                          \
    const bf16_t* pa = qkv + tok_row(p, b, t, kia) * p.ld_qkv + C + h * 64 + ch * 8;    \
    const bf16_t* pb_ = qkv + tok_row(p, b, t, kib) * p.ld_qkv + C + h * 64 + ch * 8;   \
    ka = *reinterpret_cast<const uint4*>(pa);                                           \
    va = *reinterpret_cast<const uint4*>(pa + C);                                       \
    kb = *reinterpret_cast<const uint4*>(pb_);                                          \
    vb = *reinterpret_cast<const uint4*>(pb_ + C);                                      \
  }
#define DSVT_STORE_CHUNK(st)                                                            \
  {                                                                                     \
    *reinterpret_cast<uint4*>(&kv[st][0][row_a * KV_ROW + ch * 8]) = ka;                \
    *reinterpret_cast<uint4*>(&kv[st][1][row_a * KV_ROW + ch * 8]) = va;                \
    *reinterpret_cast<uint4*>(&kv[st][0][row_b * KV_ROW + ch * 8]) = kb;                \
    *reinterpret_cast<uint4*>(&kv[st][1][row_b * KV_ROW + ch * 8]) = vb;                \
  }

  float m = -INFINITY, l = 0.f;
  fv4 o[4];
#pragma unroll
  for (int d = 0; d < 4; ++d) o[d] = fv4{0.f, 0.f, 0.f, 0.f};
  const float sl2 = p.scale * 1.4426950408889634f;

  DSVT_LOAD_CHUNK(0);
  DSVT_STORE_CHUNK(0);
  __syncthreads();
  for (int c = 0; c < nchunks; ++c) {
    const int st = c & 1;
    if (c + 1 < nchunks) DSVT_LOAD_CHUNK(c + 1);
    const bf16_t* Ks = kv[st][0];
    const bf16_t* Vs = kv[st][1];

    // S^T tiles: s[kt][j] = score(query q0 + r16, key c*64 + kt*16 + 4g + j)
    fv4 s[4];
#pragma unroll
    for (int kt = 0; kt < 4; ++kt) {
      const bf16_t* kr = Ks + (kt * 16 + r16) * KV_ROW + g * 8;
      const sv8 k0 = *reinterpret_cast<const sv8*>(kr);
      const sv8 k1 = *reinterpret_cast<const sv8*>(kr + 32);
      fv4 z = fv4{0.f, 0.f, 0.f, 0.f};
      z = __builtin_amdgcn_mfma_f32_16x16x32_bf16(k0, qf0, z, 0, 0, 0);
      s[kt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(k1, qf1, z, 0, 0, 0);
    }
    float mx = -INFINITY;
#pragma unroll
    for (int kt = 0; kt < 4; ++kt)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int64_t key = (int64_t)c * 64 + kt * 16 + 4 * g + j;
        const float v = key < p.seqlen ? s[kt][j] * sl2 : -INFINITY;
        s[kt][j] = v;
        mx = fmaxf(mx, v);
      }
    mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
    mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
    const float mn = fmaxf(m, mx);
    const float alpha = __builtin_amdgcn_exp2f(m - mn);          // args <= 0 (-inf -> 0)
    float rs = 0.f;
#pragma unroll
    for (int kt = 0; kt < 4; ++kt)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float e = __builtin_amdgcn_exp2f(s[kt][j] - mn);
        s[kt][j] = e;
        rs += e;
      }
    rs += __shfl_xor(rs, 16, 64);
    rs += __shfl_xor(rs, 32, 64);
    l = l * alpha + rs;
    m = mn;
#pragma unroll
    for (int d = 0; d < 4; ++d) o[d] *= alpha;

    // O^T += V^T . P^T over two 32-key steps; k-slot (g, jj): jj<4 -> key tile 2st2, jj>=4 -> 2st2+1
#pragma unroll
    for (int st2 = 0; st2 < 2; ++st2) {
      sv8 pb;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        pb[j] = (short)f2bf(s[2 * st2][j]);
        pb[4 + j] = (short)f2bf(s[2 * st2 + 1][j]);
      }
      const int vr0 = (2 * st2) * 16 + 4 * g + (r16 >> 2);
      const int vr1 = vr0 + 16;
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) {
        const int col = dt * 16 + 4 * (r16 & 3);
        const sv4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
            (__attribute__((address_space(3))) sv4*)(Vs + vr0 * KV_ROW + col));
        const sv4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
            (__attribute__((address_space(3))) sv4*)(Vs + vr1 * KV_ROW + col));
        const sv8 vf = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
        o[dt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(vf, pb, o[dt], 0, 0, 0);
      }
    }
    if (c + 1 < nchunks) DSVT_STORE_CHUNK(st ^ 1);
    __syncthreads();
  }

#undef DSVT_LOAD_CHUNK
#undef DSVT_STORE_CHUNK
  mfma_result_fence();   // accumulators read below, after the loop exit branch
  // lane holds O[query q0 + r16][d = dt*16 + 4g + 0..3]
  const int64_t qo = q0 + r16;
  if (qo < p.seqlen) {
    const float inv = (p.seq_scale ? p.seq_scale[seq] : 1.0f) / l;
    if (qo == 0 && p.cls_aux) {
      float* dst = p.cls_aux + seq * C + h * 64 + 4 * g;
#pragma unroll
      for (int dt = 0; dt < 4; ++dt)
        store4(dst + dt * 16, o[dt][0] * inv, o[dt][1] * inv, o[dt][2] * inv, o[dt][3] * inv);
    } else {
      bf16_t* dst = (bf16_t*)p.out + tok_row(p, b, t, qo) * p.ld_out + h * 64 + 4 * g;
#pragma unroll
      for (int dt = 0; dt < 4; ++dt)
        store4(dst + dt * 16, o[dt][0] * inv, o[dt][1] * inv, o[dt][2] * inv, o[dt][3] * inv);
    }
  }
}

// ---------------------------------------------------------------- fp32 VALU (parity mode)
__global__ __launch_bounds__(64) void attn_seq_f32(AttnParams p) {
  __shared__ float ks[64][65], vs[64][65];
  const int lane = threadIdx.x;
  const int64_t seq = blockIdx.z, b = seq / p.tin, t = seq % p.tin;
  const int h = blockIdx.y;
  const float* qkv = (const float*)p.qkv;
  const int64_t C = p.C;
  const int64_t qi = (int64_t)blockIdx.x * 64 + lane;
  const int64_t qc = qi < p.seqlen ? qi : p.seqlen - 1;
  float q[64], o[64];
  const float* qrow = qkv + tok_row(p, b, t, qc) * p.ld_qkv + h * 64;
#pragma unroll
  for (int d = 0; d < 64; ++d) { q[d] = qrow[d]; o[d] = 0.f; }
  float m = -INFINITY, l = 0.f;
  const int nchunks = (int)((p.seqlen + 63) / 64);
  for (int c = 0; c < nchunks; ++c) {
    __syncthreads();
    int64_t ki = (int64_t)c * 64 + lane;
    if (ki > p.seqlen - 1) ki = p.seqlen - 1;
    const float* base = qkv + tok_row(p, b, t, ki) * p.ld_qkv + h * 64;
    for (int d = 0; d < 64; ++d) { ks[lane][d] = base[C + d]; vs[lane][d] = base[2 * C + d]; }
    __syncthreads();
    const int64_t rem = p.seqlen - (int64_t)c * 64;
    const int nk = rem < 64 ? (int)rem : 64;
    for (int j = 0; j < nk; ++j) {
      float sdot = 0.f;
#pragma unroll
      for (int d = 0; d < 64; ++d) sdot = fmaf(q[d], ks[j][d], sdot);
      const float sc = sdot * p.scale;
      const float mn = fmaxf(m, sc);
      const float corr = expf(m - mn), pe = expf(sc - mn);
      l = l * corr + pe;
#pragma unroll
      for (int d = 0; d < 64; ++d) o[d] = fmaf(pe, vs[j][d], o[d] * corr);
      m = mn;
    }
  }
  if (p.probs) {                            // get_attn: exp(s - m) / l, second pass over the keys
    float* prow = p.probs + ((seq * p.heads + h) * p.seqlen + qc) * p.seqlen;
    for (int c = 0; c < nchunks; ++c) {
      __syncthreads();
      int64_t ki = (int64_t)c * 64 + lane;
      if (ki > p.seqlen - 1) ki = p.seqlen - 1;
      const float* base = qkv + tok_row(p, b, t, ki) * p.ld_qkv + h * 64;
      for (int d = 0; d < 64; ++d) ks[lane][d] = base[C + d];
      __syncthreads();
      const int64_t rem = p.seqlen - (int64_t)c * 64;
      const int nk = rem < 64 ? (int)rem : 64;
      for (int j = 0; j < nk; ++j) {
        float sdot = 0.f;
#pragma unroll
        for (int d = 0; d < 64; ++d) sdot = fmaf(q[d], ks[j][d], sdot);
        if (qi < p.seqlen) prow[(int64_t)c * 64 + j] = expf(sdot * p.scale - m) / l;
      }
    }
  }
  if (qi < p.seqlen) {
    const float inv = (p.seq_scale ? p.seq_scale[seq] : 1.0f) / l;
    float* dst = (qi == 0 && p.cls_aux) ? p.cls_aux + seq * C + h * 64
                                        : (float*)p.out + tok_row(p, b, t, qi) * p.ld_out + h * 64;
#pragma unroll
    for (int d = 0; d < 64; ++d) dst[d] = o[d] * inv;
  }
}

// ---------------------------------------------------------------- short sequences (L <= 16*NKT)
// One workgroup per (sequence, head): K and V of the WHOLE sequence are gathered into LDS once
// (rows past L zero-filled), then the 4 waves take the 16-query tiles round-robin.  Keys are
// handled in 16-key tiles (197 -> 13 tiles = 208 slots instead of 4 x 64 = 256), and with
// every score of a query row in registers the softmax is exact two-pass (no rescaling).  Same
// MFMA decomposition as attn_seq_bf16: S^T = K.Q^T (lane = one query, 4 keys per tile) and
// O^T = V^T.P^T with the k-slot permutation and ds_read_b64_tr_b16 V^T fragments.
// DBG (diagnostic builds only): 1 = drain lgkmcnt before every P.V MFMA, 2 = V^T fragments by
// scalar LDS reads instead of ds_read_b64_tr_b16, 3 = the loads, LDS staging and stores alone (no
// math), 4 = the grid as (sequence, head) instead of (head, sequence).
// SWZ: LDS rows of exactly 64 bf16 with the 16-B chunks XOR-swizzled by (row & 7) instead of the
// 72-element padded rows, and only the NKT staged key tiles (an odd last tile finishes with a
// 16x16x32 P.V step whose second 16-key half is zero in both operands -- one MFMA shape per
// accumulator chain): 2 x 208 x 128 B = 52 KB per workgroup at 1 + 196 keys, so
// 3 workgroups (12 waves) share a CU instead of 2.
// ds_read_b64_tr_b16 as inline asm: the compiler does not track it, so it adds no vmcnt wait
// for in-flight LDS-DMA of OTHER buffers before it (the caller waits lgkmcnt itself)
__device__ __forceinline__ sv4 ds_read_tr16_asm(const bf16_t* lds_ptr) {
  sv4 r;
  const unsigned a = (unsigned)(uintptr_t)(__attribute__((address_space(3))) const bf16_t*)lds_ptr;
  asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(r) : "v"(a));
  return r;
}

// One 16-query tile of a short sequence against its K / V staged in LDS (`lds` layout below):
// scores, exact two-pass softmax, P.V and the output stores.
template <int NKT, int DBG, bool SWZ>
__device__ __forceinline__ void short_tile(const AttnParams& p, const bf16_t* Ks, const bf16_t* Vs, const sv8 qf0,
                                           const sv8 qf1, const int qt, const int L, const int nkt, const int64_t seq,
                                           const int64_t b, const int64_t t, const int h, const float sl2, const int r16,
                                           const int g, const float oscale) {
  constexpr int NKP = SWZ ? NKT / 2 : (NKT + 1) / 2;   // full 32-key PV steps
  constexpr bool HALF = SWZ && (NKT & 1);              // + one 16-key step
  constexpr int SN = SWZ ? NKT : 2 * NKP;    // score tiles held (padded: the last of an odd NKT is 0)
  auto lds = [](int r, int c) { return SWZ ? r * 64 + ((c ^ (r & 7)) << 3) : r * KV_ROW + c * 8; };
  const int64_t C = p.C;
  // scores: s[kt][j] = raw score(query qt*16 + r16, key kt*16 + 4g + j); the row max is taken
  // on raw scores (scale > 0) and the scale folded into the exponent: exp2(s*c - max*c)
  // Every tile of the compile-time extent is computed (rows past the sequence are staged
  // zeros; their scores are masked by a select): the score -> max -> exp -> P.V chain is
  // straight-line code.  A runtime branch between an MFMA and the VALU reading its result
  // made the ROCm 7.2 hazard recognizer under-insert wait states on the taken path (stale
  // scores in the row max: ~1-ulp nondeterminism at 4 waves, NaN at 8).
  fv4 s[SN];
#pragma unroll
  for (int kt = 0; kt < SN; ++kt) {
    const int kr = kt * 16 + r16;
    const sv8 k0 = *reinterpret_cast<const sv8*>(Ks + lds(kr, g));
    const sv8 k1 = *reinterpret_cast<const sv8*>(Ks + lds(kr, g + 4));
    fv4 z = fv4{0.f, 0.f, 0.f, 0.f};
    z = __builtin_amdgcn_mfma_f32_16x16x32_bf16(k0, qf0, z, 0, 0, 0);
    s[kt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(k1, qf1, z, 0, 0, 0);
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
  for (int kt = 0; kt < SN; ++kt) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float e = __builtin_amdgcn_exp2f(fmaf(s[kt][j], sl2, -mxs));   // args <= 0; masked -> 0
      s[kt][j] = e;
      rs += e;
    }
  }
  rs += __shfl_xor(rs, 16, 64);
  rs += __shfl_xor(rs, 32, 64);
  // O^T += V^T . P^T over 32-key steps; k-slot (g, jj): jj<4 -> key tile 2kp, jj>=4 -> 2kp+1
  fv4 o[4];
#pragma unroll
  for (int d = 0; d < 4; ++d) o[d] = fv4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int kp = 0; kp < NKP; ++kp) {
    sv8 pb;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      pb[j] = (short)f2bf(s[2 * kp][j]);
      pb[4 + j] = (short)f2bf(s[2 * kp + 1][j]);
    }
    const int vr0 = kp * 32 + 4 * g + (r16 >> 2);
    const int vr1 = vr0 + 16;
    sv4 vlo[4], vhi[4];
    if constexpr (DBG == 5) {
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) {
        const int col = dt * 16 + 4 * (r16 & 3);
        vlo[dt] = ds_read_tr16_asm(Vs + lds(vr0, col >> 3) + (col & 7));
        vhi[dt] = ds_read_tr16_asm(Vs + lds(vr1, col >> 3) + (col & 7));
      }
      asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(vlo[0]), "+v"(vlo[1]), "+v"(vlo[2]), "+v"(vlo[3]), "+v"(vhi[0]),
                   "+v"(vhi[1]), "+v"(vhi[2]), "+v"(vhi[3]));
    }
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) {
      const int col = dt * 16 + 4 * (r16 & 3);
      sv8 vf;
      if constexpr (DBG == 5) {
        vf = __builtin_shufflevector(vlo[dt], vhi[dt], 0, 1, 2, 3, 4, 5, 6, 7);
      } else if constexpr (DBG == 2) {
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) {
          vf[jj] = (short)Vs[(kp * 32 + 4 * g + jj) * KV_ROW + dt * 16 + r16];
          vf[4 + jj] = (short)Vs[(kp * 32 + 16 + 4 * g + jj) * KV_ROW + dt * 16 + r16];
        }
      } else {
        const sv4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
            (__attribute__((address_space(3))) sv4*)(Vs + lds(vr0, col >> 3) + (col & 7)));
        const sv4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
            (__attribute__((address_space(3))) sv4*)(Vs + lds(vr1, col >> 3) + (col & 7)));
        vf = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
      }
      if constexpr (DBG == 1) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      o[dt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(vf, pb, o[dt], 0, 0, 0);
    }
  }
  if constexpr (HALF) {   // odd last key tile: the same 16x16x32 step with the second key tile's
    constexpr int kt = 2 * NKP;   // k-slots zero in both operands (one MFMA shape in the chain:
    sv8 pb;                       // mixing in 16x16x16 left a srcC hazard under 3-WG occupancy)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      pb[j] = (short)f2bf(s[kt][j]);
      pb[4 + j] = 0;
    }
    const int vr0 = kt * 16 + 4 * g + (r16 >> 2);
    sv4 vlo[4];
    if constexpr (DBG == 5) {
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) vlo[dt] = ds_read_tr16_asm(Vs + lds(vr0, (dt * 16 + 4 * (r16 & 3)) >> 3) + (4 * (r16 & 3) & 7));
      asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(vlo[0]), "+v"(vlo[1]), "+v"(vlo[2]), "+v"(vlo[3]));
    }
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) {
      const int col = dt * 16 + 4 * (r16 & 3);
      const sv4 lo = DBG == 5 ? vlo[dt] : __builtin_amdgcn_ds_read_tr16_b64_v4i16(
          (__attribute__((address_space(3))) sv4*)(Vs + lds(vr0, col >> 3) + (col & 7)));
      const sv8 vf = __builtin_shufflevector(lo, sv4{0, 0, 0, 0}, 0, 1, 2, 3, 4, 5, 6, 7);
      o[dt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(vf, pb, o[dt], 0, 0, 0);
    }
  }
  mfma_result_fence();     // the stores below are under per-lane branches
  // lane holds O[query qt*16 + r16][d = dt*16 + 4g + 0..3]
  const int qo = qt * 16 + r16;
  if (p.probs && qo < L) {                 // get_attn: normalized probabilities, fp32
    const float inv = 1.0f / rs;
    float* prow = p.probs + ((seq * p.heads + h) * (int64_t)L + qo) * L;
#pragma unroll
    for (int kt = 0; kt < SN; ++kt) {
      if (kt < nkt) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int key = kt * 16 + 4 * g + j;
          if (key < L) prow[key] = s[kt][j] * inv;
        }
      }
    }
  }
  // the row's 64 outputs as two 16-byte pieces per lane (fragment pairs packed across the lane
  // groups by v_permlane16_swap, every lane taking part before the per-lane store branch):
  // each store instruction writes 16 rows x 64 contiguous bytes instead of 16 rows x 32
  const float inv = oscale / rs;   // oscale: the sequence's DropPath scale or 1
#pragma unroll
  for (int dt = 0; dt < 4; ++dt) o[dt] *= inv;
  const uint4 pk0 = pack_pair_bf16(o[0], o[1]), pk1 = pack_pair_bf16(o[2], o[3]);
#ifndef DSVT_ATTN_PAIRSTORE
#define DSVT_ATTN_PAIRSTORE 1
#endif
  if (qo < L) {
    if ((qo == 0 && p.cls_aux) || !DSVT_ATTN_PAIRSTORE) {
      float* dst = p.cls_aux + seq * C + h * 64 + 4 * g;
      bf16_t* dsto = (bf16_t*)p.out + tok_row(p, b, t, qo) * p.ld_out + h * 64 + 4 * g;
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) {
        if (qo == 0 && p.cls_aux) store4(dst + dt * 16, o[dt][0], o[dt][1], o[dt][2], o[dt][3]);
        else store4(dsto + dt * 16, o[dt][0], o[dt][1], o[dt][2], o[dt][3]);
      }
    } else {
      bf16_t* dst = (bf16_t*)p.out + tok_row(p, b, t, qo) * p.ld_out + h * 64 + pair_off(g);
      *reinterpret_cast<uint4*>(dst) = pk0;
      *reinterpret_cast<uint4*>(dst + 32) = pk1;
    }
  }
}

template <int NKT, int NW, int DBG = 0, bool SWZ = false>
__global__ __launch_bounds__(64 * NW, SWZ ? 3 : 2) void attn_short_bf16(AttnParams p) {
  constexpr int NKP = SWZ ? NKT / 2 : (NKT + 1) / 2;   // full 32-key PV steps
  constexpr bool HALF = SWZ && (NKT & 1);              // + one 16-key step
  constexpr int SN = SWZ ? NKT : 2 * NKP;    // score tiles held (padded: the last of an odd NKT is 0)
  constexpr int LP = SWZ ? NKT * 16 : NKP * 32;        // LDS rows
  constexpr int ROW = SWZ ? 64 : KV_ROW;
  // element offset of (row r, 16-B chunk c) inside a K or V buffer
  auto lds = [](int r, int c) { return SWZ ? r * 64 + ((c ^ (r & 7)) << 3) : r * KV_ROW + c * 8; };
  __shared__ __attribute__((aligned(16))) bf16_t kv[2][LP * ROW];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int r16 = lane & 15, g = lane >> 4;
  const int h = DBG == 4 ? blockIdx.y : blockIdx.x;
  const int64_t seq = DBG == 4 ? blockIdx.x : blockIdx.y, b = seq / p.tin, t = seq % p.tin;
  const bf16_t* qkv = (const bf16_t*)p.qkv;
  const int64_t C = p.C;
  const int L = (int)p.seqlen;
  const int nkt = (L + 15) >> 4;
  const int nqt = nkt;

  // Issue EVERY global load up front (this wave's Q fragments for all its query tiles, and
  // the thread's <= 8 K/V pieces), then one wait, then the LDS writes: a load -> ds_write
  // loop would serialize one HBM round trip per iteration.
  constexpr int QT_W = (NKT + NW - 1) / NW;  // query tiles per wave
  sv8 qa[QT_W], qb[QT_W];
#pragma unroll
  for (int w = 0; w < QT_W; ++w) {
    int qi = (wave + NW * w) * 16 + r16;
    if (qi > L - 1) qi = L - 1;
    const bf16_t* qrow = qkv + tok_row(p, b, t, qi) * p.ld_qkv + h * 64;
    qa[w] = *reinterpret_cast<const sv8*>(qrow + g * 8);
    qb[w] = *reinterpret_cast<const sv8*>(qrow + 32 + g * 8);
  }
  constexpr int NT = 64 * NW;
  constexpr int PCS = (LP * 8 + NT - 1) / NT;  // K/V 16-B pieces per thread
  uint4 kq[PCS], vq[PCS];
#pragma unroll
  for (int i = 0; i < PCS; ++i) {
    const int pc = tid + NT * i, r = pc >> 3, ch = pc & 7;
    kq[i] = make_uint4(0, 0, 0, 0);
    vq[i] = kq[i];
    if (r < L) {
      const bf16_t* src = qkv + tok_row(p, b, t, r) * p.ld_qkv + C + h * 64 + ch * 8;
      kq[i] = *reinterpret_cast<const uint4*>(src);
      vq[i] = *reinterpret_cast<const uint4*>(src + C);
    }
  }
#pragma unroll
  for (int i = 0; i < PCS; ++i) {
    const int pc = tid + NT * i, r = pc >> 3, ch = pc & 7;
    if (r < LP) {
      *reinterpret_cast<uint4*>(&kv[0][lds(r, ch)]) = kq[i];
      *reinterpret_cast<uint4*>(&kv[1][lds(r, ch)]) = vq[i];
    }
  }
  __syncthreads();
  const bf16_t* Ks = kv[0];
  const bf16_t* Vs = kv[1];
  const float sl2 = p.scale * 1.4426950408889634f;
  if constexpr (DBG == 3) {   // the loads, the LDS staging and the output stores alone (no math)
#pragma unroll
    for (int w = 0; w < QT_W; ++w) {
      const int qt = wave + NW * w;
      if (qt >= nqt) break;
      const int qo = qt * 16 + r16;
      if (qo < L) {
        sv8 v = qa[w];
        const sv8 kx = *reinterpret_cast<const sv8*>(Ks + lds(qo, g));
        const sv8 vx = *reinterpret_cast<const sv8*>(Vs + lds(qo, g));
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] ^= kx[e] ^ vx[e] ^ qb[w][e];
        bf16_t* dst = (bf16_t*)p.out + tok_row(p, b, t, qo) * p.ld_out + h * 64 + g * 8;
        *reinterpret_cast<sv8*>(dst) = v;
        *reinterpret_cast<sv8*>(dst + 32) = v;
      }
    }
    return;
  }

#pragma unroll
  for (int w = 0; w < QT_W; ++w) {
    const int qt = wave + NW * w;
    if (qt >= nqt) break;
    short_tile<NKT, DBG, SWZ>(p, Ks, Vs, qa[w], qb[w], qt, L, nkt, seq, b, t, h, sl2, r16, g,
                              p.seq_scale ? p.seq_scale[seq] : 1.0f);
  }
}

// 0 = auto; otherwise forced (tools/attn_check.py, tests).  Per calling thread: a diagnostic
// override on one thread never changes the kernels another thread's launches pick.
static thread_local int g_attn_variant = 0;
void set_attn_variant(int v) { g_attn_variant = v; }

hipError_t launch_attn_seq(int dtype, const AttnParams& p, hipStream_t s) {
  const int v = g_attn_variant;
  if (dtype == 0 && p.seqlen <= 256 && v != 4) {
    dim3 grid((unsigned)p.heads, (unsigned)(p.nb * p.tin));
    // measured at 1 + 196 keys x 8 frames x 16 clips (tools/attn_bench.py): <13, 4> 60 us,
    // <16, 4> 63 us, <13, 8> 66 us, streaming flash kernel 77 us
    if (v == 1) attn_short_bf16<16, 4><<<grid, 256, 0, s>>>(p);
    else if (v == 2 && p.seqlen <= 208) attn_short_bf16<13, 8><<<grid, 512, 0, s>>>(p);
    else if (v == 5 && p.seqlen <= 208) attn_short_bf16<13, 4, 1><<<grid, 256, 0, s>>>(p);
    else if (v == 6 && p.seqlen <= 208) attn_short_bf16<13, 4, 2><<<grid, 256, 0, s>>>(p);
    else if (v == 7 && p.seqlen <= 48) attn_short_bf16<3, 4, 0, true><<<grid, 256, 0, s>>>(p);
    else if (p.seqlen <= 64 && v == 0) attn_short_bf16<4, 4><<<grid, 256, 0, s>>>(p);
    else if (v == 3 && p.seqlen <= 208) attn_short_bf16<13, 4><<<grid, 256, 0, s>>>(p);   // padded rows
    else if (v == 9 && p.seqlen <= 208) attn_short_bf16<13, 4, 3, true><<<grid, 256, 0, s>>>(p);   // diagnostic
    else if (v == 10 && p.seqlen <= 208)                                      // (sequence, head) grid
      attn_short_bf16<13, 4, 4, true><<<dim3(grid.y, grid.x), 256, 0, s>>>(p);
    // 1 + 196 patches: swizzled exact-tile LDS, 3 workgroups per CU -- 53.4 vs 62.2 us at the
    // bench's global call (16 clips x 8 frames x 12 heads); 25.3 vs 24.5 us at 1 + 36 (kept <4, 4>)
    else if (p.seqlen <= 208) attn_short_bf16<13, 4, 0, true><<<grid, 256, 0, s>>>(p);
    else attn_short_bf16<16, 4><<<grid, 256, 0, s>>>(p);
    return hipGetLastError();
  }
  // contiguous sequences (joint space-time, space-only): the LDS-DMA flash kernel
  // (attn_flash.hip); variant 8 keeps the register-staged kernel below (A/B, tests)
  // variants 11-15: the flash kernel's workgroup shape forced (attn_flash.hip kShapes 1-5: 4 waves
  // x 1 / 2 query tiles, 8 waves x 3 + 2 / 2 + 1 / 2 + 2)
  if (v != 8 && attn_flash_ok(dtype, p)) return launch_attn_flash(p, s, v >= 11 && v <= 15 ? v - 10 : 0);
  dim3 grid((unsigned)((p.seqlen + 63) / 64), (unsigned)p.heads, (unsigned)(p.nb * p.tin));
  if (dtype == 0) attn_seq_bf16<<<grid, 256, 0, s>>>(p);
  else attn_seq_f32<<<grid, 64, 0, s>>>(p);
  return hipGetLastError();
}

// ---------------------------------------------------------------- temporal attention
// grid (nseq, ceil(heads/G)); LDS holds [T][3][G][64] of the sequence's q/k/v for the
// workgroup's G heads.  Work item = (head hh, query i), 16 lanes each, 4 dims per lane.
template <typename T>
__global__ __launch_bounds__(256) void attn_temporal_kernel(const T* __restrict__ qkv, T* __restrict__ out,
                                                            int Tf, int heads, int G, int64_t C, float scale) {
  extern __shared__ __attribute__((aligned(16))) char dyn_smem[];
  T* sm = reinterpret_cast<T*>(dyn_smem);
  const int tid = threadIdx.x;
  const int64_t sq = blockIdx.x;
  const int h0 = blockIdx.y * G;
  const int gh = (heads - h0) < G ? (heads - h0) : G;
  constexpr int PER = Elem<T>::PER16;
  const int seg_pieces = 64 / PER;  // 16-B pieces per 64-elem head segment
  const int total = Tf * 3 * gh * seg_pieces;
  for (int pc = tid; pc < total; pc += 256) {
    const int piece = pc % seg_pieces;
    const int rest = pc / seg_pieces;
    const int hh = rest % gh, which = (rest / gh) % 3, tt = rest / (gh * 3);
    const T* src = qkv + (sq * Tf + tt) * 3 * C + which * C + (int64_t)(h0 + hh) * 64 + piece * PER;
    T* dst = sm + (((int64_t)tt * 3 + which) * G + hh) * 64 + piece * PER;
    *reinterpret_cast<uint4*>(dst) = *reinterpret_cast<const uint4*>(src);
  }
  __syncthreads();
  const int sub = tid & 15, d0 = sub * 4;
  const int items = gh * Tf;
  for (int it = tid >> 4; it < items; it += 16) {
    const int hh = it % gh, i = it / gh;
    float q[4], o[4] = {0.f, 0.f, 0.f, 0.f};
    load4(sm + (((int64_t)i * 3 + 0) * G + hh) * 64 + d0, q);
    float m = -INFINITY, l = 0.f;
    for (int j = 0; j < Tf; ++j) {
      float k[4], v[4];
      load4(sm + (((int64_t)j * 3 + 1) * G + hh) * 64 + d0, k);
      float part = q[0] * k[0] + q[1] * k[1] + q[2] * k[2] + q[3] * k[3];
      part += __shfl_xor(part, 1, 64);
      part += __shfl_xor(part, 2, 64);
      part += __shfl_xor(part, 4, 64);
      part += __shfl_xor(part, 8, 64);
      const float sc = part * scale;
      const float mn = fmaxf(m, sc);
      const float corr = expf(m - mn), pe = expf(sc - mn);
      load4(sm + (((int64_t)j * 3 + 2) * G + hh) * 64 + d0, v);
      l = l * corr + pe;
#pragma unroll
      for (int e = 0; e < 4; ++e) o[e] = fmaf(pe, v[e], o[e] * corr);
      m = mn;
    }
    const float inv = 1.0f / l;
    store4(out + (sq * Tf + i) * C + (int64_t)(h0 + hh) * 64 + d0, o[0] * inv, o[1] * inv, o[2] * inv, o[3] * inv);
  }
}

// ---------------------------------------------------------------- bf16 register kernel, T <= 8
// 16 lanes own one (sequence, head); lane `sub` holds dims 4*sub..4*sub+3 of q/k/v for all
// T tokens (8-B loads: a wave reads 4 heads x 128 B = 512 B contiguous per token and role,
// all 3*TP loads issued before any use -> deep memory-level parallelism, no LDS).
// S = Q K^T: each lane forms TP*TP partial dots over its 4 dims; a butterfly reduce-scatter
// over the 16 lanes (masks 8,4,2,1: NV/2+NV/4+.. shuffles instead of 4*NV) leaves lane sub with
// the VPL = TP*TP/16 fully-reduced scores idx = sub*VPL + k (row i = idx / TP).  Softmax runs
// in-lane plus a LPR-lane max/sum; the reverse butterfly all-gathers P for the P.V product.
template <int TP>
__global__ __launch_bounds__(256) void attn_temporal_reg(const bf16_t* __restrict__ qkv, bf16_t* __restrict__ out,
                                                         int64_t groups, int Tf, int heads, int64_t C, float sl2) {
  constexpr int NV = TP * TP, VPL = NV / 16, LPR = TP / VPL;
  static_assert(NV >= 16 && NV % 16 == 0, "TP must be 4 or 8");
  const int64_t grp = ((int64_t)blockIdx.x * 256 + threadIdx.x) >> 4;
  const int sub = threadIdx.x & 15;
  if (grp >= groups) return;  // the whole 16-lane group leaves together
  const int64_t sq = grp / heads;
  const int h = (int)(grp % heads);
  const bf16_t* base = qkv + sq * Tf * 3 * C + (int64_t)h * 64 + sub * 4;
  uint2 rq[TP], rk[TP], rv[TP];
#pragma unroll
  for (int t = 0; t < TP; ++t) {
    const int tt = t < Tf ? t : Tf - 1;
    const bf16_t* r = base + (int64_t)tt * 3 * C;
    rq[t] = *reinterpret_cast<const uint2*>(r);
    rk[t] = *reinterpret_cast<const uint2*>(r + C);
    rv[t] = *reinterpret_cast<const uint2*>(r + 2 * C);
  }
  float vals[NV];
#pragma unroll
  for (int i = 0; i < TP; ++i) {
    const float q0 = bf16_lo(rq[i].x), q1 = bf16_hi(rq[i].x), q2 = bf16_lo(rq[i].y), q3 = bf16_hi(rq[i].y);
#pragma unroll
    for (int j = 0; j < TP; ++j)
      vals[i * TP + j] = q0 * bf16_lo(rk[j].x) + q1 * bf16_hi(rk[j].x) + q2 * bf16_lo(rk[j].y) + q3 * bf16_hi(rk[j].y);
  }
  // reduce-scatter: after the stage with mask m the lane keeps the half selected by (sub & m)
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    const int mask = 8 >> s, half = NV >> (s + 1);
    const bool hi = (sub & mask) != 0;
#pragma unroll
    for (int k = 0; k < half; ++k) {
      const float mine = hi ? vals[half + k] : vals[k];
      const float oth = hi ? vals[k] : vals[half + k];
      vals[k] = mine + __shfl_xor(oth, mask, 64);
    }
  }
  // lane holds scores idx = sub*VPL + k: row i = sub / LPR, key j = (sub % LPR)*VPL + k
  const int j0 = (sub % LPR) * VPL;
  float mx = -INFINITY;
#pragma unroll
  for (int k = 0; k < VPL; ++k) {
    vals[k] = (j0 + k < Tf) ? vals[k] * sl2 : -INFINITY;
    mx = fmaxf(mx, vals[k]);
  }
#pragma unroll
  for (int m = 1; m < LPR; m <<= 1) mx = fmaxf(mx, __shfl_xor(mx, m, 64));
  float sum = 0.f;
#pragma unroll
  for (int k = 0; k < VPL; ++k) {
    vals[k] = exp2f(vals[k] - mx);
    sum += vals[k];
  }
#pragma unroll
  for (int m = 1; m < LPR; m <<= 1) sum += __shfl_xor(sum, m, 64);
  const float inv = 1.0f / sum;
#pragma unroll
  for (int k = 0; k < VPL; ++k) vals[k] *= inv;
  // all-gather P (reverse butterfly: blocks stay in natural index order)
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    const int mask = 1 << s, n = VPL << s;
    const bool hi = (sub & mask) != 0;
#pragma unroll
    for (int k = 0; k < n; ++k) {
      const float recv = __shfl_xor(vals[k], mask, 64);
      const float mine = vals[k];
      vals[k] = hi ? recv : mine;
      vals[n + k] = hi ? mine : recv;
    }
  }
  float vf[TP][4];
#pragma unroll
  for (int j = 0; j < TP; ++j) {
    vf[j][0] = bf16_lo(rv[j].x); vf[j][1] = bf16_hi(rv[j].x);
    vf[j][2] = bf16_lo(rv[j].y); vf[j][3] = bf16_hi(rv[j].y);
  }
  bf16_t* obase = out + sq * Tf * C + (int64_t)h * 64 + sub * 4;
#pragma unroll
  for (int i = 0; i < TP; ++i) {
    if (i >= Tf) break;
    float o0 = 0.f, o1 = 0.f, o2 = 0.f, o3 = 0.f;
#pragma unroll
    for (int j = 0; j < TP; ++j) {
      const float pj = vals[i * TP + j];
      o0 = fmaf(pj, vf[j][0], o0); o1 = fmaf(pj, vf[j][1], o1);
      o2 = fmaf(pj, vf[j][2], o2); o3 = fmaf(pj, vf[j][3], o3);
    }
    uint2 w;
    w.x = pack_bf16x2(o0, o1);
    w.y = pack_bf16x2(o2, o3);
    *reinterpret_cast<uint2*>(obase + (int64_t)i * C) = w;
  }
}

hipError_t launch_attn_temporal(int dtype, const void* qkv, void* out, int64_t nseq, int64_t T, int64_t heads,
                                int64_t C, float scale, hipStream_t s) {
  if (dtype == 0 && T <= 8) {
    const int64_t groups = nseq * heads;
    const unsigned blocks = (unsigned)((groups * 16 + 255) / 256);
    const float sl2 = scale * 1.4426950408889634f;
    if (T <= 4)
      attn_temporal_reg<4><<<blocks, 256, 0, s>>>((const bf16_t*)qkv, (bf16_t*)out, groups, (int)T, (int)heads, C, sl2);
    else
      attn_temporal_reg<8><<<blocks, 256, 0, s>>>((const bf16_t*)qkv, (bf16_t*)out, groups, (int)T, (int)heads, C, sl2);
    return hipGetLastError();
  }
  const int64_t esz = dtype == 0 ? 2 : 4;
  const int64_t per_head = T * 3 * 64 * esz;
  int64_t G = (48 * 1024) / per_head;
  if (G < 1) G = 1;
  if (G > heads) G = heads;
  const size_t smem = (size_t)(per_head * G);
  dim3 grid((unsigned)nseq, (unsigned)((heads + G - 1) / G));
  if (dtype == 0)
    attn_temporal_kernel<bf16_t><<<grid, 256, smem, s>>>((const bf16_t*)qkv, (bf16_t*)out, (int)T, (int)heads, (int)G, C, scale);
  else
    attn_temporal_kernel<float><<<grid, 256, smem, s>>>((const float*)qkv, (float*)out, (int)T, (int)heads, (int)G, C, scale);
  return hipGetLastError();
}


// ---------------------------------------------------------------- CLS-query attention
// The attention of the LAST block when forward_features returns the CLS token only
// (timesformer.py:139-167, 341-345): the patch rows' outputs of that block never reach the
// result, so only the CLS query is evaluated.
//   divided (T frames): sequence (b, t) = CLS row b*L + the N patch rows 1 + n*T + t of frame t;
//     the T outputs are averaged (the reference's cls_token mean over frames);
//   joint / space-only (T = 1): sequence b = the L contiguous rows of clip (or frame) b.
// Split-K over the keys ("flash decoding"), two launches:
//   attn_cls_part_kernel: one wave per (b, t, head, chunk of ATTN_CLS_CHUNK keys) -- 1536 waves
//     for the bench's 16 global clips, 312 for config 4's two joint clips -- leaves the chunk's
//     max m, sum l and unnormalized P.V row (66 floats) in the workspace;
//   attn_cls_merge_kernel: one thread per (b, channel): a frame's chunks merged with the
//     log-sum-exp rescale, the frames summed in order (deterministic), / T.
// Lane layout in a wave: 8 groups of 8 lanes; a group owns one key row per step, a lane 8 of its
// 64 dims (one 16-byte piece of bf16 / two of fp32), so one wave instruction reads 8 whole 128-B
// rows; the score loop is unrolled by 2 (16 keys, two rows' loads in flight per lane).
constexpr int ATTN_CLS_CHUNK = 256;

template <typename TI>
__device__ __forceinline__ void load8f(const TI* p, float (&v)[8]) {
  if constexpr (sizeof(TI) == 2) {
    const uint4 u = *reinterpret_cast<const uint4*>(p);
    v[0] = bf16_lo(u.x); v[1] = bf16_hi(u.x); v[2] = bf16_lo(u.y); v[3] = bf16_hi(u.y);
    v[4] = bf16_lo(u.z); v[5] = bf16_hi(u.z); v[6] = bf16_lo(u.w); v[7] = bf16_hi(u.w);
  } else {
    const float4 a = *reinterpret_cast<const float4*>(p), b = *reinterpret_cast<const float4*>(p + 4);
    v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
  }
}

template <typename TI>
__global__ __launch_bounds__(256) void attn_cls_part_kernel(const TI* __restrict__ qkv, float* __restrict__ part,
                                                            int64_t items, int64_t L, int T, int seqlen, int nchunk,
                                                            int heads, float scale) {
  __shared__ float sc[4][ATTN_CLS_CHUNK];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int64_t item = (int64_t)blockIdx.x * 4 + w;       // ((b * T + t) * heads + h) * nchunk + chunk
  if (item >= items) return;                               // wave-uniform; no block barrier below
  const int chunk = (int)(item % nchunk);
  const int64_t bth = item / nchunk;
  const int h = (int)(bth % heads);
  const int64_t bt = bth / heads;
  const int t = (int)(bt % T);
  const int64_t b = bt / T;
  const int grp = lane >> 3, c = lane & 7;
  const int64_t C = (int64_t)heads * 64, ld = 3 * C;
  const TI* base = qkv + b * L * ld;
  const int j0c = chunk * ATTN_CLS_CHUNK, nk = min(seqlen - j0c, ATTN_CLS_CHUNK);
  auto key_row = [&](int j) -> int64_t { return j == 0 ? 0 : 1 + (int64_t)(j - 1) * T + t; };
  float q[8];
  load8f(base + h * 64 + c * 8, q);
#pragma unroll
  for (int i = 0; i < 8; ++i) q[i] *= scale;
  float* s = sc[w];
  float mx = -INFINITY;
  for (int j0 = 0; j0 < nk; j0 += 16) {
    float part[2];
    int jj[2];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      jj[u] = j0 + 8 * u + grp;
      const int jl = jj[u] < nk ? jj[u] : nk - 1;          // clamped: loads stay in bounds
      float k[8];
      load8f(base + key_row(j0c + jl) * ld + C + h * 64 + c * 8, k);
      float a = 0.f;
#pragma unroll
      for (int i = 0; i < 8; ++i) a = fmaf(q[i], k[i], a);
      part[u] = a;
    }
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      part[u] += __shfl_xor(part[u], 1);
      part[u] += __shfl_xor(part[u], 2);
      part[u] += __shfl_xor(part[u], 4);
      if (jj[u] < nk) {
        if (c == 0) s[jj[u]] = part[u];
        mx = fmaxf(mx, part[u]);
      }
    }
  }
#pragma unroll
  for (int o = 8; o < 64; o <<= 1) mx = fmaxf(mx, __shfl_xor(mx, o));
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  float sum = 0.f;
  for (int j = lane; j < nk; j += 64) {
    const float e = __expf(s[j] - mx);
    s[j] = e;
    sum += e;
  }
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) sum += __shfl_xor(sum, o);
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  // P.V: group grp takes keys grp (mod 8) of the chunk, lane c dims c*8 .. c*8+7
  float acc[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) acc[i] = 0.f;
  for (int j = grp; j < nk; j += 16) {
    const int j2 = j + 8 < nk ? j + 8 : j;
    float v0[8], v1[8];
    load8f(base + key_row(j0c + j) * ld + 2 * C + h * 64 + c * 8, v0);
    load8f(base + key_row(j0c + j2) * ld + 2 * C + h * 64 + c * 8, v1);
    const float p0 = s[j], p1 = j + 8 < nk ? s[j2] : 0.f;
#pragma unroll
    for (int i = 0; i < 8; ++i) acc[i] = fmaf(p1, v1[i], fmaf(p0, v0[i], acc[i]));
  }
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    acc[i] += __shfl_xor(acc[i], 8);
    acc[i] += __shfl_xor(acc[i], 16);
    acc[i] += __shfl_xor(acc[i], 32);
  }
  float* dst = part + item * 66;
  if (grp == 0) {
#pragma unroll
    for (int i = 0; i < 8; ++i) dst[c * 8 + i] = acc[i];
  }
  if (lane == 0) {
    dst[64] = mx;
    dst[65] = sum;
  }
}

// seq_scale (nullable): frame t's output of clip b scaled by seq_scale[b * T + t] before the mean --
// training DropPath over the (b, t) sequences of the spatial branch (timesformer.py:159)
template <typename TI>
__global__ __launch_bounds__(256) void attn_cls_merge_kernel(const float* __restrict__ part, TI* __restrict__ out,
                                                             int64_t ld_out, int64_t B, int T, int nchunk, int heads,
                                                             const float* __restrict__ seq_scale) {
  const int64_t C = (int64_t)heads * 64;
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= B * C) return;
  const int64_t b = i / C;
  const int hc = (int)(i % C), h = hc >> 6, d = hc & 63;
  float m = 0.f;
  for (int t = 0; t < T; ++t) {
    const float* pp = part + (((b * T + t) * heads + h) * nchunk) * 66;
    float M = -INFINITY;
    for (int k = 0; k < nchunk; ++k) M = fmaxf(M, pp[k * 66 + 64]);
    float l = 0.f, o = 0.f;
    for (int k = 0; k < nchunk; ++k) {
      const float f = __expf(pp[k * 66 + 64] - M);
      l = fmaf(pp[k * 66 + 65], f, l);
      o = fmaf(pp[k * 66 + d], f, o);
    }
    m += seq_scale ? seq_scale[b * T + t] * (o / l) : o / l;
  }
  out[b * ld_out + hc] = Elem<TI>::from_f(m / (float)T);
}

int64_t attn_cls_ws_bytes(int64_t nseq, int64_t heads, int64_t seqlen) {
  return nseq * heads * ((seqlen + ATTN_CLS_CHUNK - 1) / ATTN_CLS_CHUNK) * 66 * 4;
}

hipError_t launch_attn_cls(int dtype, const void* qkv, void* out, int64_t ld_out, int64_t B, int64_t T, int64_t L,
                           int64_t heads, float scale, float* ws, hipStream_t s, const float* seq_scale) {
  const int64_t seqlen = 1 + (L - 1) / T;
  const int nchunk = (int)((seqlen + ATTN_CLS_CHUNK - 1) / ATTN_CLS_CHUNK);
  const int64_t items = B * T * heads * nchunk;
  const unsigned g1 = (unsigned)((items + 3) / 4), g2 = (unsigned)((B * heads * 64 + 255) / 256);
  if (dtype == 0) {
    attn_cls_part_kernel<bf16_t><<<g1, 256, 0, s>>>((const bf16_t*)qkv, ws, items, L, (int)T, (int)seqlen, nchunk,
                                                    (int)heads, scale);
    attn_cls_merge_kernel<bf16_t><<<g2, 256, 0, s>>>(ws, (bf16_t*)out, ld_out, B, (int)T, nchunk, (int)heads,
                                                     seq_scale);
  } else {
    attn_cls_part_kernel<float><<<g1, 256, 0, s>>>((const float*)qkv, ws, items, L, (int)T, (int)seqlen, nchunk,
                                                   (int)heads, scale);
    attn_cls_merge_kernel<float><<<g2, 256, 0, s>>>(ws, (float*)out, ld_out, B, (int)T, nchunk, (int)heads,
                                                    seq_scale);
  }
  return hipGetLastError();
}

// ---------------------------------------------------------------- CLS-query attention backward
// The training form of the CLS-only last block (dsvt.training, VisionTransformer.cls_tail): only
// the CLS query of every frame sequence (b, t) is evaluated, o_cls[b] = (1/T) sum_t s_bt O_bt
// (s = the DropPath scale of the sequence, 1 without), so the backward of that attention is one
// query per (b, t, head):
//   dO = s_bt / T * do_cls[b];  P = softmax(scale q.k_j);  dP_j = dO.v_j;  D = sum_j P_j dP_j;
//   dS_j = P_j (dP_j - D);  dq = scale sum_j dS_j k_j;  dk_j = scale dS_j q;  dv_j = P_j dO.
// One wave per (b, t, head) (lane layout of attn_cls_part_kernel: 8 groups of 8 lanes, a group one
// key row per step, a lane 8 of its 64 dims).  The patch rows of frame t belong to that sequence
// only: their dk / dv go straight to dqkv (bf16 / fp32 storage) and their dq is written ZERO (the
// patch rows' queries do not exist in the CLS-only block).  The CLS row is in all T sequences: its
// dq, dk, dv partials go to ws[(b*T + t)][3C] (fp32), summed over t in order by
// attn_cls_bwd_reduce_kernel into the CLS row of dqkv (deterministic).  Keys <= ATTN_CLS_BWD_MAX.
constexpr int ATTN_CLS_BWD_MAX = 512;

template <typename TI, typename TO>
__global__ __launch_bounds__(256) void attn_cls_bwd_kernel(const TI* __restrict__ qkv, const TO* __restrict__ dout,
                                                           TI* __restrict__ dqkv, float* __restrict__ ws,
                                                           const float* __restrict__ seq_scale, int64_t items,
                                                           int64_t L, int T, int seqlen, int heads, float scale) {
  __shared__ float sp[4][ATTN_CLS_BWD_MAX], sdp[4][ATTN_CLS_BWD_MAX];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int64_t item = (int64_t)blockIdx.x * 4 + w;        // (b * T + t) * heads + h
  if (item >= items) return;                                // wave-uniform; no block barrier below
  const int h = (int)(item % heads);
  const int64_t bt = item / heads;
  const int t = (int)(bt % T);
  const int64_t b = bt / T;
  const int grp = lane >> 3, c = lane & 7;
  const int64_t C = (int64_t)heads * 64, ld = 3 * C;
  const TI* base = qkv + b * L * ld;
  auto key_row = [&](int j) -> int64_t { return j == 0 ? 0 : 1 + (int64_t)(j - 1) * T + t; };
  float q[8], dO[8];
  load8f(base + h * 64 + c * 8, q);
  {
    float d[8];
    load8f(dout + b * C + h * 64 + c * 8, d);
    const float f = (seq_scale ? seq_scale[bt] : 1.0f) / (float)T;
#pragma unroll
    for (int i = 0; i < 8; ++i) dO[i] = d[i] * f;
  }
  float* s = sp[w];
  float* dp = sdp[w];
  // pass 1: scores and dP for every key (a group per key row, 8 rows per step)
  float mx = -INFINITY;
  for (int j0 = 0; j0 < seqlen; j0 += 8) {
    const int j = j0 + grp;
    const int jl = j < seqlen ? j : seqlen - 1;
    float k[8], v[8];
    load8f(base + key_row(jl) * ld + C + h * 64 + c * 8, k);
    load8f(base + key_row(jl) * ld + 2 * C + h * 64 + c * 8, v);
    float a = 0.f, e = 0.f;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      a = fmaf(q[i], k[i], a);
      e = fmaf(dO[i], v[i], e);
    }
    a += __shfl_xor(a, 1); a += __shfl_xor(a, 2); a += __shfl_xor(a, 4);
    e += __shfl_xor(e, 1); e += __shfl_xor(e, 2); e += __shfl_xor(e, 4);
    a *= scale;
    if (j < seqlen) {
      if (c == 0) { s[j] = a; dp[j] = e; }
      mx = fmaxf(mx, a);
    }
  }
#pragma unroll
  for (int o = 8; o < 64; o <<= 1) mx = fmaxf(mx, __shfl_xor(mx, o));
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  float sum = 0.f;
  for (int j = lane; j < seqlen; j += 64) {
    const float e = __expf(s[j] - mx);
    s[j] = e;
    sum += e;
  }
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) sum += __shfl_xor(sum, o);
  const float inv = 1.0f / sum;
  float D = 0.f;
  for (int j = lane; j < seqlen; j += 64) {
    const float pj = s[j] * inv;
    s[j] = pj;
    D = fmaf(pj, dp[j], D);
  }
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) D += __shfl_xor(D, o);
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  // pass 2: dk_j, dv_j of every key; dq accumulated per group
  float dq[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) dq[i] = 0.f;
  float* cw = ws + bt * ld;                                 // this sequence's CLS-row partials
  for (int j0 = 0; j0 < seqlen; j0 += 8) {
    const int j = j0 + grp;
    if (j < seqlen) {                                       // group-uniform branch
      const float pj = s[j], dsj = pj * (dp[j] - D);
      float k[8];
      load8f(base + key_row(j) * ld + C + h * 64 + c * 8, k);
      float dk[8], dv[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        dq[i] = fmaf(dsj, k[i], dq[i]);
        dk[i] = scale * dsj * q[i];
        dv[i] = pj * dO[i];
      }
      if (j == 0) {
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          cw[C + h * 64 + c * 8 + i] = dk[i];
          cw[2 * C + h * 64 + c * 8 + i] = dv[i];
        }
      } else {
        TI* dr = dqkv + (b * L + key_row(j)) * ld + h * 64 + c * 8;
        store4(dr, 0.f, 0.f, 0.f, 0.f);
        store4(dr + 4, 0.f, 0.f, 0.f, 0.f);
        store4(dr + C, dk[0], dk[1], dk[2], dk[3]);
        store4(dr + C + 4, dk[4], dk[5], dk[6], dk[7]);
        store4(dr + 2 * C, dv[0], dv[1], dv[2], dv[3]);
        store4(dr + 2 * C + 4, dv[4], dv[5], dv[6], dv[7]);
      }
    }
  }
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    dq[i] += __shfl_xor(dq[i], 8);
    dq[i] += __shfl_xor(dq[i], 16);
    dq[i] += __shfl_xor(dq[i], 32);
  }
  if (grp == 0) {
#pragma unroll
    for (int i = 0; i < 8; ++i) cw[h * 64 + c * 8 + i] = scale * dq[i];
  }
}

// CLS row of clip b: dqkv[b * L][:] = sum over t (in order) of ws[b * T + t][:]
template <typename TI>
__global__ __launch_bounds__(256) void attn_cls_bwd_reduce_kernel(const float* __restrict__ ws, TI* __restrict__ dqkv,
                                                                  int64_t B, int T, int64_t L, int64_t C3) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= B * C3) return;
  const int64_t b = i / C3, c = i % C3;
  float v = 0.f;
  for (int t = 0; t < T; ++t) v += ws[(b * T + t) * C3 + c];
  dqkv[b * L * C3 + c] = Elem<TI>::from_f(v);
}

int64_t attn_cls_bwd_ws_bytes(int64_t nseq, int64_t heads) { return nseq * heads * 64 * 3 * 4; }

hipError_t launch_attn_cls_bwd(int dtype, const void* qkv, const void* dout, void* dqkv, float* ws,
                               const float* seq_scale, int64_t B, int64_t T, int64_t L, int64_t heads, float scale,
                               hipStream_t s) {
  const int64_t seqlen = 1 + (L - 1) / T;
  if (seqlen > ATTN_CLS_BWD_MAX) return hipErrorInvalidValue;
  const int64_t items = B * T * heads, C3 = heads * 64 * 3;
  const unsigned g1 = (unsigned)((items + 3) / 4), g2 = (unsigned)((B * C3 + 255) / 256);
#define DSVT_CB(TI, TO) attn_cls_bwd_kernel<TI, TO><<<g1, 256, 0, s>>>((const TI*)qkv, (const TO*)dout, (TI*)dqkv, ws, \
                                                                       seq_scale, items, L, (int)T, (int)seqlen,       \
                                                                       (int)heads, scale)
  if (dtype == 0) {
    DSVT_CB(bf16_t, bf16_t);
    attn_cls_bwd_reduce_kernel<bf16_t><<<g2, 256, 0, s>>>(ws, (bf16_t*)dqkv, B, (int)T, L, C3);
  } else {
    DSVT_CB(float, float);
    attn_cls_bwd_reduce_kernel<float><<<g2, 256, 0, s>>>(ws, (float*)dqkv, B, (int)T, L, C3);
  }
#undef DSVT_CB
  return hipGetLastError();
}

}  // namespace dsvt
