// Shared device helpers for the DINO-SVT gfx950 kernels.
// Storage types: bf16 is carried as raw `unsigned short` bits (perf mode), float is the
// fp32 parity mode.  All accumulation is fp32.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "internal.h"

typedef unsigned short bf16_t;
typedef short sv8 __attribute__((ext_vector_type(8)));   // 8 x bf16 MFMA operand (4 VGPRs)
typedef short sv4 __attribute__((ext_vector_type(4)));   // 4 x bf16 (tr-read result)
typedef float fv4 __attribute__((ext_vector_type(4)));   // 4 x fp32 accumulator

#define LDS_PTR(p) ((__attribute__((address_space(3))) void*)(p))

__device__ __forceinline__ float bf2f(bf16_t u) { return __uint_as_float(((unsigned)u) << 16); }
__device__ __forceinline__ bf16_t f2bf(float f) {
  __bf16 h = (__bf16)f;  // v_cvt_pk_bf16_f32: round-to-nearest-even, NaN preserved
  return __builtin_bit_cast(bf16_t, h);
}

// packed bf16 pair (low half = lower address) <-> float
__device__ __forceinline__ float bf16_lo(unsigned u) { return __uint_as_float(u << 16); }
__device__ __forceinline__ float bf16_hi(unsigned u) { return __uint_as_float(u & 0xffff0000u); }
__device__ __forceinline__ unsigned pack_bf16x2(float a, float b) {
  return (unsigned)f2bf(a) | ((unsigned)f2bf(b) << 16);
}

// Two adjacent 16x16 fp32 fragments (cols 16j.. and 16(j+1).. of one row) -> 8 contiguous bf16
// per lane for ONE 16-byte store: a v_permlane16_swap per packed dword gives lane group g the
// columns {g0: 0-7, g1: 16-23, g2: 8-15, g3: 24-31} of the 32-column span (offset pair_off(g)).
// Cross-lane: call with the whole wave active; predicate only the store.
// two floats -> packed bf16 pair (low = a) in ONE v_cvt_pk_bf16_f32 (RNE)
__device__ __forceinline__ unsigned cvt_pk_bf16(float a, float b) {
  typedef float f2_t __attribute__((ext_vector_type(2)));
  typedef __bf16 b2_t __attribute__((ext_vector_type(2)));
  const b2_t h = __builtin_convertvector((f2_t){a, b}, b2_t);
  return __builtin_bit_cast(unsigned, h);
}
// same, from the four already-packed bf16 pairs (a0 = a[0..1], a1 = a[2..3], b0, b1)
__device__ __forceinline__ uint4 pack_pair_words(unsigned a0, unsigned a1, unsigned b0, unsigned b1) {
  const auto s0 = __builtin_amdgcn_permlane16_swap(a0, b0, false, false);
  const auto s1 = __builtin_amdgcn_permlane16_swap(a1, b1, false, false);
  return make_uint4(s0[0], s1[0], s0[1], s1[1]);
}
__device__ __forceinline__ uint4 pack_pair_bf16(fv4 a, fv4 b) {
  return pack_pair_words(cvt_pk_bf16(a[0], a[1]), cvt_pk_bf16(a[2], a[3]), cvt_pk_bf16(b[0], b[1]),
                         cvt_pk_bf16(b[2], b[3]));
}
__device__ __forceinline__ int pair_off(int g) { return ((g & 1) << 4) | ((g >> 1) << 3); }

// max over a lane's four 16-lane groups by the same two permlane swaps (every lane the same bits)
__device__ __forceinline__ float max_lane_groups(float v) {
  const auto a = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  v = fmaxf(__uint_as_float(a[0]), __uint_as_float(a[1]));
  const auto b = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return fmaxf(__uint_as_float(b[0]), __uint_as_float(b[1]));
}

// x0^2 + x1^2 + x2^2 + x3^2 as (fma(x0, x0, x1 x1)) + (fma(x2, x2, x3 x3)): written out so that no
// template instantiation can contract it differently (-ffp-contract=fast lets the compiler fuse a
// product into a neighbouring add where it likes; LayerNorm statistics must be the same bits
// whichever kernel instantiation -- full or ragged tile -- produced a row)
__device__ __forceinline__ float sumsq4(float x0, float x1, float x2, float x3) {
  return __builtin_fmaf(x0, x0, x1 * x1) + __builtin_fmaf(x2, x2, x3 * x3);
}

// sum over a lane's four 16-lane groups (lanes l, l ^ 16, l ^ 32, l ^ 48) by two VALU permlane
// swaps (no LDS traffic); every lane gets the same bits: (x0 + x2) + (x1 + x3) in one order
__device__ __forceinline__ float sum_lane_groups(float v) {
  const auto a = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  v = __uint_as_float(a[0]) + __uint_as_float(a[1]);
  const auto b = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(b[0]) + __uint_as_float(b[1]);
}

// Bias of a wave's 64 output columns cbase .. cbase+63 (cbase wave-uniform) as the lane's
// 4 x float4 (fragment j, columns cbase + 16j + 4g .. +3).  Read through the constant address
// space, i.e. SCALAR loads counted on lgkmcnt: a vector load here would sit on vmcnt behind
// the GEMM's in-flight LDS-DMA prefetches and stores, and its wait would drain them all.
__device__ __forceinline__ void bias_frag4(const float* bias, int64_t cbase, int g, float4 (&out)[4]) {
  if (!bias) {
#pragma unroll
    for (int j = 0; j < 4; ++j) out[j] = make_float4(0.f, 0.f, 0.f, 0.f);
    return;
  }
  typedef __attribute__((address_space(4))) const fv4* CF4;
  const CF4 bp = (CF4)(bias + cbase);
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const fv4 v0 = bp[4 * j], v1 = bp[4 * j + 1], v2 = bp[4 * j + 2], v3 = bp[4 * j + 3];
    const fv4 v = g == 0 ? v0 : g == 1 ? v1 : g == 2 ? v2 : v3;
    out[j] = make_float4(v[0], v[1], v[2], v[3]);
  }
}

// Generic element <-> float conversion for the two storage types.
template <typename T> struct Elem;
template <> struct Elem<bf16_t> {
  static constexpr int PER16 = 8;  // elements per 16-byte piece
  __device__ __forceinline__ static float to_f(bf16_t v) { return bf2f(v); }
  __device__ __forceinline__ static bf16_t from_f(float v) { return f2bf(v); }
};
template <> struct Elem<float> {
  static constexpr int PER16 = 4;
  __device__ __forceinline__ static float to_f(float v) { return v; }
  __device__ __forceinline__ static float from_f(float v) { return v; }
};

// Store 4 consecutive values (converted to T): 8 B for bf16, 16 B for fp32.
__device__ __forceinline__ void store4(bf16_t* p, float a, float b, float c, float d) {
  uint2 u;
  u.x = (unsigned)f2bf(a) | ((unsigned)f2bf(b) << 16);
  u.y = (unsigned)f2bf(c) | ((unsigned)f2bf(d) << 16);
  *reinterpret_cast<uint2*>(p) = u;
}
__device__ __forceinline__ void store4(float* p, float a, float b, float c, float d) {
  *reinterpret_cast<float4*>(p) = make_float4(a, b, c, d);
}
__device__ __forceinline__ void load4(const bf16_t* p, float* v) {
  uint2 u = *reinterpret_cast<const uint2*>(p);
  v[0] = __uint_as_float(u.x << 16); v[1] = __uint_as_float(u.x & 0xffff0000u);
  v[2] = __uint_as_float(u.y << 16); v[3] = __uint_as_float(u.y & 0xffff0000u);
}
__device__ __forceinline__ void load4(const float* p, float* v) {
  float4 f = *reinterpret_cast<const float4*>(p);
  v[0] = f.x; v[1] = f.y; v[2] = f.z; v[3] = f.w;
}

// Wait states covering the longest MFMA result latency before code that reads accumulators
// under control flow: the compiler's hazard recognizer has been seen to under-insert them on
// a branch target right after an MFMA (attention.hip, attn_short_bf16).  s_nop n = n+1 states.
__device__ __forceinline__ void mfma_result_fence() {
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 3");
  __builtin_amdgcn_sched_barrier(0);
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
// Sum over the 64 lanes without LDS round trips: DPP adds inside each 16-lane row (quad
// swaps, then row rotations by 4 and 8 -- every lane ends with its row's sum), then the four
// row sums through v_readlane.  ~20 cycles of latency against ~6 ds_bpermute round trips for
// wave_sum; the result is wave-uniform.  Summation order differs from wave_sum's butterfly.
__device__ __forceinline__ float wave_sum_dpp(float v) {
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0xB1, 0xF, 0xF, false));   // quad [1,0,3,2]
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x4E, 0xF, 0xF, false));   // quad [2,3,0,1]
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x124, 0xF, 0xF, false));  // row_ror:4
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x128, 0xF, 0xF, false));  // row_ror:8
  const float r0 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 0));
  const float r1 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 16));
  const float r2 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 32));
  const float r3 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 48));
  return (r0 + r1) + (r2 + r3);
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// Exact-erf GELU, 0.5 x (1 + erf(x / sqrt2)) (nn.GELU default).  erf by Abramowitz & Stegun
// 7.1.26 (|abs err| <= 1.5e-7): 1 - erf(z) = t P(t) exp(-z^2), t = 1 / (1 + 0.3275911 z), z >= 0.
// ~14 VALU ops (one v_rcp, one v_exp) instead of ~35 for the libm erff: this runs on every
// fc1 output element, in the epilogue of the largest GEMM.  1 + erf(-z) = t P(t) exp(-z^2) is
// formed directly for x < 0, so the negative tail has no cancellation.
__device__ __forceinline__ float gelu_erf(float x) {
  const float z = fabsf(x) * 0.70710678118654752f;
  const float t = __builtin_amdgcn_rcpf(fmaf(0.3275911f, z, 1.0f));
  float p = fmaf(t, 1.061405429f, -1.453152027f);
  p = fmaf(t, p, 1.421413741f);
  p = fmaf(t, p, -0.284496736f);
  p = fmaf(t, p, 0.254829592f);
  const float tail = p * t * __builtin_amdgcn_exp2f(-z * z * 1.4426950408889634f);  // 1 - erf(z)
  const float one_plus_erf = x >= 0.f ? 2.0f - tail : tail;
  return 0.5f * x * one_plus_erf;
}

// GELU for a bf16 OUTPUT (inference fc1 epilogue): x * sigmoid(x * P(x^2)) with P a quadratic in
// x^2 fitted minimax to the exact erf GELU on [-10, 10] (x^2 clamped at 100 outside, where the
// sigmoid has saturated): |error| <= 2.6e-5 absolute -- below half a bf16 ulp of the output for
// |GELU(x)| >= 0.013, and far below the 2^-9 relative rounding of the stored value elsewhere.
// 7 VALU + 2 transcendental ops against ~16 + 2 for gelu_erf: the fc1 epilogue is VALU-bound
// and runs with no MFMA beside it.  fp32 outputs (parity mode) and the training epilogues (whose
// backward differentiates gelu_erf) keep gelu_erf.  Coefficients pre-scaled by -log2(e).
__device__ __forceinline__ float gelu_bf16out(float x) {
  const float x2 = fminf(x * x, 100.0f);
  const float p = fmaf(fmaf(1.01426306e-03f, x2, -1.06775724e-01f), x2, -2.30112134e+00f);
  return x * __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(x * p));
}

// gelu_bf16out on a PAIR of values: the same operations, the non-transcendental ones as packed
// fp32 VALU (v_pk_mul / v_pk_fma / v_pk_add_f32: two lanes' worth per instruction) -- bitwise the
// scalar form's results, ~12 instead of 18 instructions per pair in the VALU-bound fc1 epilogue.
typedef float f2v __attribute__((ext_vector_type(2)));
__device__ __forceinline__ f2v gelu_bf16out2(f2v x) {
  f2v x2 = x * x;
  x2.x = fminf(x2.x, 100.0f);
  x2.y = fminf(x2.y, 100.0f);
  const f2v c0 = {1.01426306e-03f, 1.01426306e-03f}, c1 = {-1.06775724e-01f, -1.06775724e-01f};
  const f2v c2 = {-2.30112134e+00f, -2.30112134e+00f}, one = {1.0f, 1.0f};
  const f2v t = x * __builtin_elementwise_fma(__builtin_elementwise_fma(c0, x2, c1), x2, c2);
  const f2v d = one + f2v{__builtin_amdgcn_exp2f(t.x), __builtin_amdgcn_exp2f(t.y)};
  return x * f2v{__builtin_amdgcn_rcpf(d.x), __builtin_amdgcn_rcpf(d.y)};
}

// the inference GELU epilogue by output type: the fast form only when the result is stored in bf16
template <bool BF16_OUT>
__device__ __forceinline__ float gelu_out(float x) {
  if constexpr (BF16_OUT) return gelu_bf16out(x);
  else return gelu_erf(x);
}

// (GELU(x), GELU'(x)) in one evaluation: the erf tail and exp(-x^2/2) shared (the training fc1
// epilogue saves GELU'(pre) for the backward); .x is bitwise gelu_erf(x), .y gelu_erf_grad(x)
__device__ __forceinline__ float2 gelu_erf_and_grad(float x) {
  const float z = fabsf(x) * 0.70710678118654752f;
  const float t = __builtin_amdgcn_rcpf(fmaf(0.3275911f, z, 1.0f));
  float p = fmaf(t, 1.061405429f, -1.453152027f);
  p = fmaf(t, p, 1.421413741f);
  p = fmaf(t, p, -0.284496736f);
  p = fmaf(t, p, 0.254829592f);
  const float e = __builtin_amdgcn_exp2f(-z * z * 1.4426950408889634f);   // exp(-x^2/2)
  const float tail = p * t * e;                                            // 1 - erf(z)
  const float one_plus_erf = x >= 0.f ? 2.0f - tail : tail;
  const float cdf = 0.5f * one_plus_erf;
  return make_float2(0.5f * x * one_plus_erf, cdf + x * e * 0.3989422804014327f);
}
// d GELU / dx = Phi(x) + x phi(x) (same A&S 7.1.26 erf as gelu_erf): the Mlp.fc1 backward.
__device__ __forceinline__ float gelu_erf_grad(float x) {
  const float z = fabsf(x) * 0.70710678118654752f;
  const float t = __builtin_amdgcn_rcpf(fmaf(0.3275911f, z, 1.0f));
  float p = fmaf(t, 1.061405429f, -1.453152027f);
  p = fmaf(t, p, 1.421413741f);
  p = fmaf(t, p, -0.284496736f);
  p = fmaf(t, p, 0.254829592f);
  const float e = __builtin_amdgcn_exp2f(-z * z * 1.4426950408889634f);   // exp(-x^2/2)
  const float tail = p * t * e;                                            // 1 - erf(z)
  const float cdf = 0.5f * (x >= 0.f ? 2.0f - tail : tail);
  return cdf + x * e * 0.3989422804014327f;
}

// Output-row map used by every kernel that writes into the [B, L, C] token tensor:
//   row(m) = (m / rpg) * gstride + goff + (m % rpg)
// identity: rpg = huge, gstride = 0, goff = 0.
// (identity: one test; 32-bit operands: a 32-bit division instead of the ~50-op 64-bit one)
__device__ __forceinline__ long map_row(long m, long rpg, long gstride, long goff) {
  if (m < rpg) return goff + m;
  if (((unsigned long)m | (unsigned long)rpg) >> 31 == 0) {
    const unsigned q = (unsigned)m / (unsigned)rpg;
    return (long)q * gstride + goff + (long)((unsigned)m - q * (unsigned)rpg);
  }
  return (m / rpg) * gstride + goff + (m % rpg);
}
