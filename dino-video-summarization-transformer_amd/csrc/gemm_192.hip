// 256x192 bf16 MFMA GEMM with a phase-interleaved K loop (variant 30): the N = 768 residual
// GEMMs (attn.proj, the folded temporal proj . fc, fc2) over M = 13.8k-25.1k tokens.
//
// Why a second tile shape: at N = 768 the 256x256 kernel (gemm_8ph.hip) has 3 N-tiles, i.e. 297
// tiles for M = 25088 on 256 CUs -- 1.16 tiles per CU, run as two full tile times -- and each
// CU's fp32 X read-modify-write epilogue (640 KiB per tile) lands on HBM at the same moment
// as every other CU's.  A 192-column tile gives 4 N-tiles: 392 tiles = 1.53 tiles per CU of
// 0.75 the work each (1.5 tile times instead of 2), with 25 % less epilogue traffic per tile.
//
// Geometry: one 512-thread workgroup (8 waves, 4 x 2) per CU, 112 KiB of LDS = two K-tile
// buffers of BK = 64 (128-byte rows).  Wave (wr, wc) = (wave >> 1, wave & 1) owns the 64 x 96
// output block at (wr*64, wc*96): acc[4][6] 16x16 fragments in four quadrants
//   q0 = rows 0-31 x cols 0-47, q1 = rows 0-31 x cols 48-95, q2 = rows 32-63 x cols 48-95,
//   q3 = rows 32-63 x cols 0-47,
// one per PHASE of a K-tile (12 MFMA 16x16x32 per wave per phase).  The K-tile is staged as
//   AT = A rows {wr*64 + 0-31} (128 rows, 16 KiB), AB = A rows {wr*64 + 32-63},
//   BL = W rows {wc*96 + 0-47} (96 rows, 12 KiB),  BR = W rows {wc*96 + 48-95},
// in the stream order AT, BL, BR, AB like the 256x256 kernel (two K-tiles ahead of the reads of
// the same buffer; see gemm_8ph.hip for the phase protocol and the one-barrier stagger of the
// two waves of every SIMD).  An A half-tile is two global_load_lds_dwordx4 per thread; a B
// half-tile is one per thread plus one for waves 0-3 (its rows 64-95), so the vmcnt of the four
// half-tiles in flight is 8 for waves 0-3 and 6 for waves 4-7.
//
// The residual epilogue adds bias and X in registers (N % 192 == 0, so every wave column is
// full) and optionally writes the next LayerNorm's inputs (dsvt_gemm_resid_stats_fwd): the bf16
// row copy and the row's LN_PARTS partial sums -- a 192-column tile covers three 64-column
// slots, written as (sum of wave column 0, zero) and (sum of wave column 1), so every slot is
// written and the consumer's sum over all of them is the row sum.
#include "gemm_epi.h"

namespace dsvt {

namespace {

constexpr int Q_ROWB = 128;                 // bytes per LDS row: 64 bf16 of K
constexpr int Q_AH = 128 * Q_ROWB;          // A half-tile, 16 KiB
constexpr int Q_BH = 96 * Q_ROWB;           // B half-tile, 12 KiB
constexpr int Q_AT = 0, Q_AB = Q_AH, Q_BL = 2 * Q_AH, Q_BR = 2 * Q_AH + Q_BH;
constexpr int Q_BUF = 2 * Q_AH + 2 * Q_BH;  // one K-tile, 56 KiB

template <int N>
__device__ __forceinline__ void q_vm_wait() {
  static_assert(N >= 0 && N < 64, "vmcnt immediate");
  __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | 0x0F70);
}

__device__ __forceinline__ void q_barrier() {
  __builtin_amdgcn_sched_barrier(0);
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
}

// B half-tile row br (0-95) -> W row within the tile's BL half: wave column 0 rows 0-47, wave
// column 1 rows 96-143 (BR: + 48)
__device__ __forceinline__ int q_brow(int br) { return br >= 48 ? br + 48 : br; }

// X[row(m)] += acc + bias over the wave's 64 x 96 block, rows past M (FULL = false) skipped;
// STATS: also the bf16 copy and the LN partial slots of the row (see the header).  X rows run a
// rolling window of 2 rows of fragments ahead of their stores.
template <bool FULL, bool STATS>
__device__ __forceinline__ void resid192_rows(const GemmParams& p, fv4 (&acc)[4][6], int64_t rbase, int64_t cbase,
                                              int wc, int r16, int g) {
  constexpr int MI = 4, NJ = 6, W = 2;
  const bool ident = p.rpg >= p.M && p.goff == 0;
  auto orow_of = [&](int i) -> int64_t {
    int64_t m = rbase + i * 16 + r16;
    if constexpr (!FULL) m = m < p.M ? m : p.M - 1;
    return ident ? m : map_row(m, p.rpg, p.gstride, p.goff);
  };
  float4 x[W][NJ];
  auto load_row = [&](int i) {
    const float* src = resid_src(p) + orow_of(i) * p.ldo + cbase + 4 * g;
#pragma unroll
    for (int j = 0; j < NJ; ++j) x[i % W][j] = *reinterpret_cast<const float4*>(src + j * 16);
  };
#pragma unroll
  for (int i = 0; i < W; ++i) load_row(i);
  float4 bias4[NJ];
#pragma unroll
  for (int j = 0; j < NJ; ++j)
    bias4[j] = p.bias ? *reinterpret_cast<const float4*>(p.bias + cbase + j * 16 + 4 * g) : make_float4(0.f, 0.f, 0.f, 0.f);
  const int64_t slot = (cbase / 192) * 3 + 2 * wc;
#pragma unroll
  for (int i = 0; i < MI; ++i) {
    const int64_t orow = orow_of(i);
    // training DropPath (dsvt_gemm_resid_scaled_fwd): A carries the row's scale, the bias takes it here
    const float rs = p.row_scale ? row_scale_of(p, FULL ? rbase + i * 16 + r16 : min(rbase + i * 16 + r16, p.M - 1))
                                 : 1.0f;
    fv4 v[NJ];
    float s = 0.f, q = 0.f;
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const float4 xv = x[i % W][j];
      const float4 bb = bias4[j];
      // explicit fma: the same bits in the full- and ragged-tile instantiations
      v[j] = fv4{xv.x + __builtin_fmaf(bb.x, rs, acc[i][j][0]), xv.y + __builtin_fmaf(bb.y, rs, acc[i][j][1]),
                 xv.z + __builtin_fmaf(bb.z, rs, acc[i][j][2]), xv.w + __builtin_fmaf(bb.w, rs, acc[i][j][3])};
      if constexpr (STATS) {
        s += (v[j][0] + v[j][1]) + (v[j][2] + v[j][3]);
        q += sumsq4(v[j][0], v[j][1], v[j][2], v[j][3]);
      }
    }
    if (i + W < MI) load_row(i + W);
    if constexpr (STATS) {
      s = sum_lane_groups(s);
      q = sum_lane_groups(q);
    }
    const bool ok = FULL || rbase + i * 16 + r16 < p.M;
    if (ok) {
      float* dst = (float*)p.out + orow * p.ldo + cbase + 4 * g;
#pragma unroll
      for (int j = 0; j < NJ; ++j) *reinterpret_cast<fv4*>(dst + j * 16) = v[j];
      if constexpr (STATS) {
        bf16_t* xb = (bf16_t*)p.xb_out + orow * p.ldo + cbase;
#pragma unroll
        for (int j = 0; j < NJ; j += 2) store_pair_bf16(xb + j * 16, v[j], v[j + 1], g);
        // the four lanes of the row store the same bytes (no per-lane branch)
        float* sp = p.stats_out + (orow * LN_PARTS + slot) * 2;
        *reinterpret_cast<float2*>(sp) = make_float2(s, q);
        if (wc == 0) *reinterpret_cast<float2*>(sp + 2) = make_float2(0.f, 0.f);
      }
    }
  }
}

// bf16 out[row(m)] = acc + bias (GELU: then the bf16-output GELU, pairwise as gemm_8ph's) over the
// wave's 64 x 96 block (the backward's N = 768 dX GEMMs; config 4's fc1): 16-byte pair stores,
// rows past M clamped to M - 1 (their accumulators are row M - 1's: the A loads are clamped) so the
// stores are branch-free
template <bool GELU>
__device__ __forceinline__ void bias192_rows(const GemmParams& p, fv4 (&acc)[4][6], int64_t rbase, int64_t cbase,
                                             int r16, int g) {
  const bool ident = p.rpg >= p.M && p.goff == 0;
  float4 bias4[6];
#pragma unroll
  for (int j = 0; j < 6; ++j)
    bias4[j] = p.bias ? *reinterpret_cast<const float4*>(p.bias + cbase + j * 16 + 4 * g) : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    int64_t m = rbase + i * 16 + r16;
    m = m < p.M ? m : p.M - 1;
    const int64_t orow = ident ? m : map_row(m, p.rpg, p.gstride, p.goff);
#pragma unroll
    for (int j = 0; j < 6; ++j) {
      acc[i][j][0] += bias4[j].x; acc[i][j][1] += bias4[j].y; acc[i][j][2] += bias4[j].z; acc[i][j][3] += bias4[j].w;
      if constexpr (GELU) {
#pragma unroll
        for (int e = 0; e < 4; e += 2) {
          const f2v v = gelu_bf16out2(f2v{acc[i][j][e], acc[i][j][e + 1]});
          acc[i][j][e] = v.x;
          acc[i][j][e + 1] = v.y;
        }
      }
    }
#pragma unroll
    for (int j = 0; j < 6; j += 2) store_pair_bf16((bf16_t*)p.out + orow * p.ldo + cbase + j * 16, acc[i][j], acc[i][j + 1], g);
  }
}

// ---- T = 8 temporal attention in the epilogue (MODE_TATTN; timesformer.py:127-131 + Attention
// .forward :55-87 on the (b h w) t m sequences).  The tile is 256 rows = 32 temporal sequences of
// one head h = n0 / 192, its W rows head-interleaved (dsvt_ln_fold_weights with heads > 0): wave
// column wc holds q, k, v dims wc*32 .. wc*32+31 of head h as fragments j = 0-1, 2-3, 4-5.  Per
// 16-row fragment i (two sequences) and wave:
//   S_wc = Q_wc . K_wc^T   one MFMA 16x16x32 on the bf16 q / k accumulators as they sit (lane
//                         (r16, g) holds dims 4g+e and 16+4g+e of row r16: the k-slots of both
//                         operands in the same order); lane (query, g) gets keys 4g .. 4g+3
//   S = S_0 + S_1          the two wave columns' partial dot products through LDS (one barrier)
//   P = softmax(S * scale) fp32 over the 8 keys of the query's own sequence (lane pairs g, g^1)
//   O_wc = P . V_wc        one MFMA 16x16x32 per 16 dims: k-slots 0-15 = P_hi, 16-31 = P_lo
//                         (P = P_hi + P_lo, two bf16 terms) against V^T twice -- V^T fragments by
//                         ds_read_b64_tr_b16 from a per-wave [64 rows][32 dims] bf16 image
// and O (bf16) goes to out[m][h*64 + wc*32 + d].  q / k / v are the bf16 roundings the unfused
// qkv GEMM would store; the products accumulate in fp32 like attn_temporal_reg.
constexpr int Q_XCH = 2 * 1024;     // per wave: S partials of the 32 valid lanes x 4 fragments
constexpr int Q_VIM = 4 * 1024;     // per wave: V image [64][32] bf16

template <bool FULL>
__device__ __forceinline__ void tattn192(const GemmParams& p, fv4 (&acc)[4][6], int64_t rbase, int64_t n0, int wave,
                                         int wc, int r16, int g, char* xch, char* vim) {
  // S partials over this wave's 32 dims
  fv4 s[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    sv8 qa, kb;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      qa[e] = (short)f2bf(acc[i][0][e]); qa[4 + e] = (short)f2bf(acc[i][1][e]);
      kb[e] = (short)f2bf(acc[i][2][e]); kb[4 + e] = (short)f2bf(acc[i][3][e]);
    }
    s[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kb, qa, fv4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
  }
  // V image rows 16i + r16, dims 16jv + 4g .. +3 (row = 64 B)
  char* const vw = vim + wave * Q_VIM;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int jv = 0; jv < 2; ++jv) {
      const fv4 v = acc[i][4 + jv];
      *reinterpret_cast<uint2*>(vw + (16 * i + r16) * 64 + (16 * jv + 4 * g) * 2) =
          make_uint2(cvt_pk_bf16(v[0], v[1]), cvt_pk_bf16(v[2], v[3]));
    }
  // valid lanes: query and keys in the same sequence of the fragment (r16 < 8) == (g < 2)
  const bool valid = (r16 < 8) == (g < 2);
  const int xi = (r16 & 7) | ((g & 1) << 3) | ((r16 >> 3) << 4);
  if (valid) {
#pragma unroll
    for (int i = 0; i < 4; ++i) *reinterpret_cast<fv4*>(xch + wave * Q_XCH + (i * 32 + xi) * 16) = s[i];
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  q_barrier();
  fv4 so[4];
  if (valid) {
#pragma unroll
    for (int i = 0; i < 4; ++i) so[i] = *reinterpret_cast<const fv4*>(xch + (wave ^ 1) * Q_XCH + (i * 32 + xi) * 16);
  } else {
#pragma unroll
    for (int i = 0; i < 4; ++i) so[i] = fv4{0.f, 0.f, 0.f, 0.f};
  }
  const float sl2 = p.attn_scale * 1.4426950408889634f;
  const bool ksrc_own = g == 0 || g == 3, use_hi = g < 2;
  const bool kvalid = (g & 1) == (r16 >> 3);        // this lane's 8 k-slots are the query's keys
  const int64_t h = n0 / 192;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    // softmax over the query's 8 keys (this lane's 4 and lane g ^ 1's)
    float v[4], mx = -INFINITY;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      v[e] = (s[i][e] + so[i][e]) * sl2;
      mx = fmaxf(mx, v[e]);
    }
    {
      const auto t = __builtin_amdgcn_permlane16_swap(__float_as_uint(mx), __float_as_uint(mx), false, false);
      mx = fmaxf(__uint_as_float(t[0]), __uint_as_float(t[1]));
    }
    float sum = 0.f;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      v[e] = exp2f(v[e] - mx);
      sum += v[e];
    }
    {
      const auto t = __builtin_amdgcn_permlane16_swap(__float_as_uint(sum), __float_as_uint(sum), false, false);
      sum = __uint_as_float(t[0]) + __uint_as_float(t[1]);
    }
    const float inv = 1.0f / sum;
    // P of keys 8(g>>1) .. +7: own 4 + lane g ^ 1's 4 (permlane16 swap; element order: the
    // lower lane group's keys first), then the other half's 8 from lane g ^ 2 (permlane32 swap)
    float pk[8];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float pv = v[e] * inv;
      const auto t = __builtin_amdgcn_permlane16_swap(__float_as_uint(pv), __float_as_uint(pv), false, false);
      // t[0] / t[1]: the even / odd 16-lane row's value of the pair -- keys 4(g & ~1) + e / 4(g | 1) + e
      pk[e] = __uint_as_float(t[0]);
      pk[4 + e] = __uint_as_float(t[1]);
    }
    float px[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const auto t = __builtin_amdgcn_permlane32_swap(__float_as_uint(pk[e]), __float_as_uint(pk[e]), false, false);
      // t[0] / t[1]: the lower / upper 32-lane half's value
      const float own = pk[e], oth = (g < 2) ? __uint_as_float(t[1]) : __uint_as_float(t[0]);
      px[e] = ksrc_own ? own : oth;
    }
    sv8 pb;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float x = kvalid ? px[e] : 0.f;
      const float hi = __uint_as_float((unsigned)f2bf(x) << 16);
      pb[e] = (short)f2bf(use_hi ? x : x - hi);
    }
    // O = P . V over this wave's 32 dims: A = V^T (lane (d, g): keys 8(g & 1) .. +7 of dim d)
#pragma unroll
    for (int jv = 0; jv < 2; ++jv) {
      const int row0 = 16 * i + 8 * (g & 1) + (r16 >> 2), col = 16 * jv + 4 * (r16 & 3);
      const sv4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
          (__attribute__((address_space(3))) sv4*)(vw + row0 * 64 + col * 2));
      const sv4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
          (__attribute__((address_space(3))) sv4*)(vw + (row0 + 4) * 64 + col * 2));
      const sv8 va = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
      const fv4 o = __builtin_amdgcn_mfma_f32_16x16x32_bf16(va, pb, fv4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
      const int64_t m = rbase + 16 * i + r16;
      if (FULL || m < p.M)
        *reinterpret_cast<uint2*>((bf16_t*)p.out + m * p.ldo + h * 64 + wc * 32 + 16 * jv + 4 * g) =
            make_uint2(cvt_pk_bf16(o[0], o[1]), cvt_pk_bf16(o[2], o[3]));
    }
  }
}

}  // namespace

enum { MODE_RESID = 0, MODE_RESID_STATS = 1, MODE_TATTN = 2, MODE_BIAS = 3, MODE_GELU = 4 };

// MODE_RESID_STATS: the residual epilogue also writes the bf16 rows and LN partials (FUSE 2 of
// gemm_8ph); MODE_TATTN: the LayerNorm-folded A operand (FUSE 1 of gemm_8ph) and the temporal
// attention epilogue above
template <int MODE>
__global__ __launch_bounds__(512, 1) void gemm_192_kernel(GemmParams p) {
  constexpr bool STATS = MODE == MODE_RESID_STATS;
  // VMEM stores of a full-tile epilogue (the fewest any wave issues): the four phases after it
  // let them sit between the awaited half-tile and the younger stages (see gemm_8ph.hip)
  constexpr int S_EPI = MODE == MODE_TATTN ? 4 * 2 : (MODE == MODE_BIAS || MODE == MODE_GELU) ? 4 * 3 : STATS ? 4 * (6 + 3 + 1) : 4 * 6;
  __shared__ __attribute__((aligned(16))) char smem[2 * Q_BUF + (MODE == MODE_TATTN ? 8 * (Q_XCH + Q_VIM) : 0)];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wave >> 1, wc = wave & 1;
  const int sg = wave >> 2;                 // stagger group: the two waves of a SIMD differ
  const bool bsecond = sg == 0;             // issues the B half-tiles' second (32-row) piece
  const int r16 = lane & 15, g = lane >> 4;
  const int tilesN = (int)(p.N / 192);
  const int tiles = (int)((p.M + 255) >> 8) * tilesN;
  // XCD-contiguous tile ranges (block b runs on XCD b % 8; the grid is a multiple of 8)
  const int G = gridDim.x, b = blockIdx.x, xcd = b & 7, li = b >> 3, per_x = G >> 3;
  const int nk = (int)(p.K >> 6);
  const int tpx = (tiles + 7) >> 3;
  const int t_first = xcd * tpx + li;
  const int t_end = min(tiles, xcd * tpx + tpx);
  if (t_first >= t_end) return;
  const int tl_end = (t_end - t_first + per_x - 1) / per_x;
  const int J = tl_end * nk;
  auto adv = [&](int& tl, int& k) {
    if (++k == nk) { k = 0; ++tl; }
  };

  const char* A = (const char*)p.A;
  const char* W = (const char*)p.W;
  const int64_t lda_b = p.lda * 2, ldw_b = p.ldw * 2;
  const int srow = tid >> 3;
  const uint32_t schunk = (uint32_t)(((tid & 7) ^ ((tid >> 4) & 7)) << 4);
  uint32_t oAT[2], oAB[2], oBL[2], oBR[2];
  auto tile_mn = [&](int tl, int64_t& m0, int64_t& n0) {
    const int t = t_first + tl * per_x;
    m0 = (int64_t)(t / tilesN) * 256;
    n0 = (int64_t)(t % tilesN) * 192;
  };
  auto a_off = [&](int64_t gr) -> uint32_t {
    gr = gr < p.M ? gr : p.M - 1;
    if constexpr (MODE == MODE_TATTN) {    // the A row map (32-bit: rows < 2^31, host-checked)
      const uint32_t m = (uint32_t)gr, rpg = (uint32_t)(p.a_rpg < p.M ? p.a_rpg : p.M);
      gr = (int64_t)((m / rpg) * (uint32_t)p.a_gstride + (uint32_t)p.a_goff + m % rpg);
    }
    return (uint32_t)(gr * lda_b) + schunk;
  };
  auto b_off = [&](int64_t gr) -> uint32_t { return (uint32_t)(gr * ldw_b) + schunk; };
  auto set_atbl = [&](int tl) {
    int64_t m0, n0;
    tile_mn(tl, m0, n0);
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      oAT[q] = a_off(m0 + (2 * q + (srow >> 5)) * 64 + (srow & 31));
      oBL[q] = b_off(n0 + q_brow(min(q * 64 + srow, 95)));
    }
  };
  auto set_brab = [&](int tl) {
    int64_t m0, n0;
    tile_mn(tl, m0, n0);
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      oAB[q] = a_off(m0 + (2 * q + (srow >> 5)) * 64 + 32 + (srow & 31));
      oBR[q] = b_off(n0 + 48 + q_brow(min(q * 64 + srow, 95)));
    }
  };
#define Q_STAGE_A(H, OFF, BUFOFF, KB)                                                                          \
  {                                                                                                            \
    char* d_ = smem + (BUFOFF) + (H) + wave * 1024;                                                            \
    __builtin_amdgcn_global_load_lds((const void*)(A + (OFF[0] + (uint32_t)(KB))), LDS_PTR(d_), 16, 0, 0);     \
    __builtin_amdgcn_global_load_lds((const void*)(A + (OFF[1] + (uint32_t)(KB))), LDS_PTR(d_ + 64 * Q_ROWB), \
                                     16, 0, 0);                                                                \
  }
#define Q_STAGE_B(H, OFF, BUFOFF, KB)                                                                          \
  {                                                                                                            \
    char* d_ = smem + (BUFOFF) + (H) + wave * 1024;                                                            \
    __builtin_amdgcn_global_load_lds((const void*)(W + (OFF[0] + (uint32_t)(KB))), LDS_PTR(d_), 16, 0, 0);     \
    if (bsecond)                                                                                               \
      __builtin_amdgcn_global_load_lds((const void*)(W + (OFF[1] + (uint32_t)(KB))),                           \
                                       LDS_PTR(d_ + 64 * Q_ROWB), 16, 0, 0);                                   \
  }

  const int xs = (r16 >> 1) & 7;
  const int rdA = (wr * 32 + r16) * Q_ROWB, rdB = (wc * 48 + r16) * Q_ROWB;
  const int cs0 = (g ^ xs) << 4, cs1 = ((4 + g) ^ xs) << 4;
  sv8 fa[2][2], fbl[3][2], fbr[3][2];
#define Q_RD(DST, H, BASE, CB, N)                                                                      \
  _Pragma("unroll") for (int f_ = 0; f_ < (N); ++f_) {                                                \
    const char* s_ = smem + (CB) + (H) + (BASE) + f_ * 16 * Q_ROWB;                                   \
    DST[f_][0] = *reinterpret_cast<const sv8*>(s_ + cs0);                                             \
    DST[f_][1] = *reinterpret_cast<const sv8*>(s_ + cs1);                                             \
  }
#define Q_MFMA(I0, J0, FB)                                                                             \
  {                                                                                                    \
    __builtin_amdgcn_s_setprio(1);                                                                     \
    _Pragma("unroll") for (int s_ = 0; s_ < 2; ++s_)                                                   \
    _Pragma("unroll") for (int i_ = 0; i_ < 2; ++i_)                                                   \
    _Pragma("unroll") for (int j_ = 0; j_ < 3; ++j_)                                                   \
      acc[(I0) + i_][(J0) + j_] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(FB[j_][s_], fa[i_][s_],      \
                                                                      acc[(I0) + i_][(J0) + j_], 0, 0, 0); \
    __builtin_amdgcn_s_setprio(0);                                                                     \
  }
  // the four most recent half-tiles may stay in flight: 2 + 2 + 2 x (2 or 1) instructions
#define Q_WAIT(VALID)                                      \
  {                                                        \
    if (!(VALID)) q_vm_wait<0>();                          \
    else if (post) {                                       \
      if (bsecond) q_vm_wait<8 + S_EPI>();                 \
      else q_vm_wait<6 + S_EPI>();                         \
    } else if (bsecond) q_vm_wait<8>();                    \
    else q_vm_wait<6>();                                   \
  }
#define Q_COMPUTE(MFMA_STMT)                               \
  {                                                        \
    q_barrier();                                           \
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");     \
    __builtin_amdgcn_sched_barrier(0);                     \
    MFMA_STMT;                                             \
    q_barrier();                                           \
  }

  // ---- prologue: K-tile 0 complete, K-tile 1 parts AT / BL
  int tl1, k1, tl2, k2;
  bool post = false;                    // the previous K-tile ended with a full-tile epilogue
  set_atbl(0);
  set_brab(0);
  Q_STAGE_A(Q_AT, oAT, 0, 0);
  Q_STAGE_B(Q_BL, oBL, 0, 0);
  Q_STAGE_B(Q_BR, oBR, 0, 0);
  Q_STAGE_A(Q_AB, oAB, 0, 0);
  tl1 = 0; k1 = 0;
  adv(tl1, k1);
  tl2 = tl1; k2 = k1;
  adv(tl2, k2);
  if (J > 1) {
    set_atbl(tl1);
    Q_STAGE_A(Q_AT, oAT, Q_BUF, k1 * Q_ROWB);
    Q_STAGE_B(Q_BL, oBL, Q_BUF, k1 * Q_ROWB);
    Q_WAIT(true);                       // AT(0), BL(0) retired
  } else {
    q_vm_wait<0>();
  }
  set_brab(tl1);
  set_atbl(tl2);
  q_barrier();
  if (sg == 1) q_barrier();             // the second wave of every SIMD runs one barrier behind

  fv4 acc[4][6];
  auto init_acc = [&]() {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 6; ++j) acc[i][j] = fv4{0.f, 0.f, 0.f, 0.f};
  };
  init_acc();
  int tlc = 0, kc = 0;

  for (int j = 0; j < J; ++j) {
    const int cb = (j & 1) * Q_BUF, sb1 = cb ^ Q_BUF, sb2 = cb;
    const bool v1 = j + 1 < J, v2 = j + 2 < J;
    const int kb1 = k1 * Q_ROWB, kb2 = k2 * Q_ROWB;
    // phase 0: read BL + AT, stage BR(j+1), quadrant (AT, BL)
    Q_RD(fbl, Q_BL, rdB, cb, 3);
    __builtin_amdgcn_sched_barrier(0);
    Q_RD(fa, Q_AT, rdA, cb, 2);
    if (v1) Q_STAGE_B(Q_BR, oBR, sb1, kb1);
    Q_WAIT(v1);
    Q_COMPUTE(Q_MFMA(0, 0, fbl));
    // phase 1: read BR, stage AB(j+1), quadrant (AT, BR)
    Q_RD(fbr, Q_BR, rdB, cb, 3);
    if (v1) Q_STAGE_A(Q_AB, oAB, sb1, kb1);
    Q_WAIT(v1);
    Q_COMPUTE(Q_MFMA(0, 3, fbr));
    // phase 2: read AB, stage AT(j+2), quadrant (AB, BR)
    Q_RD(fa, Q_AB, rdA, cb, 2);
    if (v2) Q_STAGE_A(Q_AT, oAT, sb2, kb2);
    Q_WAIT(v2);
    Q_COMPUTE(Q_MFMA(2, 3, fbr));
    // phase 3: no reads, stage BL(j+2), quadrant (AB, BL)
    if (v2) Q_STAGE_B(Q_BL, oBL, sb2, kb2);
    Q_WAIT(v2);
    Q_COMPUTE(Q_MFMA(2, 0, fbl));

    post = false;
    if (++kc == nk) {                     // tile done: register epilogue
      int64_t m0, n0;
      tile_mn(tlc, m0, n0);
      const int64_t rbase = m0 + wr * 64, cbase = n0 + wc * 96;
      mfma_result_fence();
      post = rbase + 64 <= p.M;          // wave-uniform
      if constexpr (MODE == MODE_BIAS || MODE == MODE_GELU) {
        post = true;                     // clamped rows: every store issued
        bias192_rows<MODE == MODE_GELU>(p, acc, rbase, cbase, r16, g);
      } else if constexpr (MODE == MODE_TATTN) {
        ln_affine<4, 6>(p, acc, rbase, cbase, r16, g);
        __builtin_amdgcn_sched_barrier(0);
        char* const xch = smem + 2 * Q_BUF;
        if (post) tattn192<true>(p, acc, rbase, n0, wave, wc, r16, g, xch, xch + 8 * Q_XCH);
        else tattn192<false>(p, acc, rbase, n0, wave, wc, r16, g, xch, xch + 8 * Q_XCH);
      } else {
        if (post) resid192_rows<true, STATS>(p, acc, rbase, cbase, wc, r16, g);
        else resid192_rows<false, STATS>(p, acc, rbase, cbase, wc, r16, g);
      }
      kc = 0;
      ++tlc;
      __builtin_amdgcn_sched_barrier(0);
      init_acc();
    }
    { const int o = tl1; adv(tl1, k1); if (tl1 != o && tl1 < tl_end) set_brab(tl1); }
    { const int o = tl2; adv(tl2, k2); if (tl2 != o && tl2 < tl_end) set_atbl(tl2); }
  }
  if (sg == 0) q_barrier();             // balance the stagger barrier
#undef Q_STAGE_A
#undef Q_STAGE_B
#undef Q_RD
#undef Q_MFMA
#undef Q_WAIT
#undef Q_COMPUTE
}

// the fp32 residual epilogue (bias added in the epilogue, times the DropPath row scale when
// p.row_scale) or bf16 bias / bias + GELU without row scales, N a multiple of 192 with 16-byte aligned rows, K a multiple of 64, 32-bit LDS-DMA
// source offsets
bool gemm_192_ok(const GemmParams& p, int epi) {
  return (epi == EPI_RESID || ((epi == EPI_BIAS || epi == EPI_GELU) && !p.row_scale && !p.stats_out)) &&
         !(p.stats_out && p.row_scale) &&
         p.K >= 64 && p.K % 64 == 0 && p.M >= 1 && p.N >= 192 &&
         p.N % 192 == 0 && p.ldo % 8 == 0 && ((uintptr_t)p.out & 15) == 0 && ((uintptr_t)resid_src(p) & 15) == 0 &&
         (!p.bias || ((uintptr_t)p.bias & 15) == 0) && (p.M - 1) * p.lda * 2 + p.K * 2 <= (int64_t)UINT32_MAX &&
         (p.N - 1) * p.ldw * 2 + p.K * 2 <= (int64_t)UINT32_MAX;
}

static dim3 grid_192(const GemmParams& p) {
  const int64_t tiles = ((p.M + 255) / 256) * (p.N / 192);
  int64_t G = 256;                                    // one workgroup per CU (112 / 160 KiB LDS)
  const int64_t per_x = (tiles + 7) / 8;
  if (per_x * 8 < G) G = per_x * 8;
  return dim3((unsigned)G);
}

hipError_t launch_gemm_192(const GemmParams& p, int epi, int out_f32, hipStream_t s) {
  if (!gemm_192_ok(p, epi)) return hipErrorInvalidValue;
  if (epi == EPI_BIAS || epi == EPI_GELU) {          // bf16 out only (dX GEMMs, fc1)
    if (out_f32) return hipErrorInvalidValue;
    if (epi == EPI_GELU) gemm_192_kernel<MODE_GELU><<<grid_192(p), dim3(512), 0, s>>>(p);
    else gemm_192_kernel<MODE_BIAS><<<grid_192(p), dim3(512), 0, s>>>(p);
    return hipGetLastError();
  }                                                   // EPI_RESID: fp32 X whatever the flag says
  if (p.stats_out && (!p.xb_out || p.N != LN_PARTS * 64 || p.row_scale)) return hipErrorInvalidValue;
  if (p.stats_out) gemm_192_kernel<MODE_RESID_STATS><<<grid_192(p), dim3(512), 0, s>>>(p);
  else gemm_192_kernel<MODE_RESID><<<grid_192(p), dim3(512), 0, s>>>(p);
  return hipGetLastError();
}

// LayerNorm-folded temporal qkv GEMM with the T = 8 attention in its epilogue: A = the bf16 token
// rows through the A row map with their LN partials (p.ln_stats, ln_wsum, ln_eps, ln_invk), W / bias
// / wsum head-interleaved ([12 heads][q|k|v halves] rows of 192), out = O [M, ldo] bf16 (compact
// rows, heads * 64 columns); M a multiple of 8 (whole sequences)
bool gemm_tattn_ok(const GemmParams& p) {
  if (!(p.ln_stats && p.ln_wsum && p.bias && p.K == LN_PARTS * 64 && p.N % 192 == 0 && p.M >= 8 && p.M % 8 == 0 &&
        p.T == 8 && p.ldo >= p.N / 3 && p.ldo % 4 == 0 && ((uintptr_t)p.out & 7) == 0 && p.lda % 8 == 0 &&
        p.ldw % 8 == 0 && p.a_rpg >= 1 && p.a_gstride >= 0 && p.a_goff >= 0 && p.M < INT32_MAX))
    return false;
  const int64_t rpg = p.a_rpg < p.M ? p.a_rpg : p.M;
  const int64_t last_row = ((p.M - 1) / rpg) * p.a_gstride + p.a_goff + rpg - 1;   // >= every A row read
  return last_row < INT32_MAX && last_row * p.lda * 2 + p.K * 2 <= (int64_t)UINT32_MAX &&
         (p.N - 1) * p.ldw * 2 + p.K * 2 <= (int64_t)UINT32_MAX;
}

hipError_t launch_gemm_tattn(const GemmParams& p, hipStream_t s) {
  if (!gemm_tattn_ok(p)) return hipErrorInvalidValue;
  gemm_192_kernel<MODE_TATTN><<<grid_192(p), dim3(512), 0, s>>>(p);
  return hipGetLastError();
}

}  // namespace dsvt
