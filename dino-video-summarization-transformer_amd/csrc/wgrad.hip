// Weight gradients of every nn.Linear on the student's backward path (loss.backward(),
// train_ssl.py:538): G[n, k] (+)= sum_m dY[m, n] * X[m, k], bf16 operands, fp32 result, and
// optionally the bias gradient db[n] (+)= sum_m dY[m, n] of the same Linear, fused.
//
// Both operands are read along their ROWS (m), the reduction dimension: a stage of dY rows
// [32 m][256 n] and of X rows [32 m][256 k] is staged by LDS-DMA exactly as it lies in HBM
// (512-byte rows; 16-byte chunk' = chunk ^ ((row & 7) << 1) on the source address, so the 8
// rows one ds_read_b64_tr_b16 lane group touches land on 8 distinct 32-byte bank pairs), and
// both MFMA operands come out of LDS by transposed reads: lane (r16, g) of a 16-lane group gets
// one column of m-rows 4g..4g+3 and 16+4g..16+4g+3 of the 32-row stage -- the same permuted 8
// m-values for the X fragment (A operand: rows = k) and the dY fragment (B operand: columns =
// n), so the products pair up.  The output lane holds G[n = col][k = 4g .. 4g + 3]: one 16-byte
// store.
//
// 256 x 256 output tile per 512-thread workgroup (8 waves, 2 (k) x 4 (n) of 128 x 64), one
// workgroup per CU, a 4-stage LDS ring (128 KiB) with loads three stages ahead and a counted
// vmcnt wait: one barrier per 32-row stage.  M is split over S slices so that tiles x S fills
// the 256 CUs once; each slice writes an fp32 partial tile and wgrad_reduce_kernel sums the
// slices in a fixed order into G (deterministic; `accumulate` adds to G's old value).  Work is
// laid out slice-major over XCD-contiguous ranges (block b runs on XCD b % 8), so the tiles that
// share a slice's dY / X rows share one L2.  Rows past M are clamped on load and their dY values
// zeroed in registers in the last stage (the product and the column sum then get 0).
// The bias column sum rides on the dY fragments the k-tile-0 workgroups already hold: 4
// v_dot2_f32_bf16 against ones per fragment, reduced over the 4 lane groups at the end.
#include <stdlib.h>

#include "common.h"

namespace dsvt {

namespace {

constexpr int WG_BM = 32;                  // m rows per stage
constexpr int WG_T = 256;                  // output tile: 256 n x 256 k
constexpr int WG_ROWB = 512;               // bytes per staged row (256 bf16)
constexpr int WG_OP = WG_BM * WG_ROWB;     // 16 KiB per operand per stage
constexpr int WG_STAGE = 2 * WG_OP;        // [dY | X]
#ifndef DSVT_WG_NST
#define DSVT_WG_NST 4                      // A/B builds: 2 (train step 125.0 vs 127.7, tools/gpu_s28.sh)
#endif
constexpr int WG_NST = DSVT_WG_NST;        // ring depth (128 KiB; a power of two)

// byte offset of (row, column c) in a staged [32][256] operand (c % 4 == 0 for the 8-byte reads)
__device__ __forceinline__ int wg_off(int row, int c) {
  return row * WG_ROWB + ((((c >> 3) ^ ((row & 7) << 1))) << 4) + ((c & 7) << 1);
}

template <int N>
__device__ __forceinline__ void wg_vm_wait() {
  static_assert(N >= 0 && N < 64, "vmcnt immediate");
  __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | 0x0F70);
}

__device__ __forceinline__ void wg_barrier() {
  __builtin_amdgcn_sched_barrier(0);
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
}

typedef __bf16 bf2_t __attribute__((ext_vector_type(2)));

// ds_read_b64_tr_b16 as inline asm: the builtin makes the compiler drain every in-flight LDS-DMA
// (s_waitcnt vmcnt(0) -- the stages prefetched three ahead included) before the first read of each
// stage, which serialized the loads with the math; the asm form is not tracked, so the counted
// vmcnt waits above stay the only ones and wg_lgkm_wait orders the results before their use
__device__ __forceinline__ sv4 wg_tr_read(const char* lds) {
  sv4 r;
  const unsigned a = (unsigned)(uintptr_t)(__attribute__((address_space(3))) const char*)lds;
  asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(r) : "v"(a));
  return r;
}

// s_waitcnt lgkmcnt(0) tied to the 24 fragment halves, so no use of them is scheduled above it
__device__ __forceinline__ void wg_lgkm_wait(sv4 (&b)[8], sv4 (&a)[16]) {
  asm volatile("s_waitcnt lgkmcnt(0)"
               : "+v"(b[0]), "+v"(b[1]), "+v"(b[2]), "+v"(b[3]), "+v"(b[4]), "+v"(b[5]), "+v"(b[6]), "+v"(b[7]),
                 "+v"(a[0]), "+v"(a[1]), "+v"(a[2]), "+v"(a[3]), "+v"(a[4]), "+v"(a[5]), "+v"(a[6]), "+v"(a[7]),
                 "+v"(a[8]), "+v"(a[9]), "+v"(a[10]), "+v"(a[11]), "+v"(a[12]), "+v"(a[13]), "+v"(a[14]),
                 "+v"(a[15]));
}

}  // namespace

struct WgradParams {
  const bf16_t* dy; int64_t ldy;           // [M, N]
  const bf16_t* x; int64_t ldx;            // [M, K]
  float* out;                              // S > 1: partials [S][N][K]; else G (row stride K)
  float* db;                               // optional; S > 1: partials [S][N]; else db
  int64_t M, N, K;
  int S, tilesN, tilesK;
  int accumulate;                          // S == 1: G += / db += (else =)
};

// ABL (diagnostic builds, tools/wgrad_bench.py only; 0 = normal): bit 0 no loads after the
// prologue (stale stages), bit 1 no MFMA (fragments kept live), bit 2 no fragment reads.
// (Measured and dropped: staggering the two wave rows a barrier apart, 2 barriers per stage,
// -4 %; staging X through registers beside the LDS-DMA of dY, -6 %; r05, after the asm reads:
// each stage in two k-halves, the second half's reads in flight under the first half's MFMAs
// (lgkmcnt(8) / lgkmcnt(0)): qkv 127.4 vs 124.2 us, train step 134.8 / 135.0 vs 135.0 / 134.7;
// the gemm_8ph schedule -- two phases per stage, reads -> barrier -> 16 MFMA -> barrier, wave row
// 1 one barrier behind, the stage DMA in phase 1: qkv 140.4 vs 125.0 us, train 132.1 / 131.7 vs
// 134.6 / 134.8.  Alone the kernel runs ~0.45 of its MFMA time (PMC: MFMA busy 0.33 of the
// chip's SIMD cycles at 216 of 256 CUs, LDS array 15 % busy, 0 bank conflicts, 43 % of wave
// cycles in s_waitcnt); tools/pmc_wgrad.sh.)
template <int ABL = 0>
__global__ __launch_bounds__(512, 1) void wgrad_kernel(WgradParams p) {
  __shared__ __attribute__((aligned(16))) char smem[WG_NST * WG_STAGE];
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r16 = lane & 15, g = lane >> 4;
  const int wk = wave >> 2, wn = wave & 3;      // wave's block: k rows wk*128.., n cols wn*64..
  const int tiles = p.tilesN * p.tilesK;
  const int per_x = (int)(gridDim.x >> 3);
  const int t = (int)(blockIdx.x & 7) * per_x + (int)(blockIdx.x >> 3);
  if (t >= tiles * p.S) return;
  const int sl = t / tiles, tile = t - sl * tiles;
  const int64_t n0 = (int64_t)(tile / p.tilesK) * WG_T, k0 = (int64_t)(tile % p.tilesK) * WG_T;
  const int64_t steps = (p.M + WG_BM - 1) / WG_BM;
  const int64_t s_begin = sl * steps / p.S, s_end = (sl + 1) * steps / p.S;
  const int nst = (int)(s_end - s_begin);

  // DMA roles: a wave-instruction moves 2 rows x 512 B; lane -> (row in 2, physical chunk)
  int prow[2];
  int64_t cy[2], cx[2];
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    prow[q] = (wave * 2 + q) * 2 + (lane >> 5);
    const int lc = (lane & 31) ^ ((prow[q] & 7) << 1);    // logical chunk landing in physical chunk lane & 31
    const int64_t cn = n0 + lc * 8, ck = k0 + lc * 8;      // chunks past N / K re-read the last one
    cy[q] = cn < p.N ? cn : p.N - 8;
    cx[q] = ck < p.K ? ck : p.K - 8;
  }
  auto stage = [&](int buf, int64_t step) {
    const int64_t m0 = step * WG_BM;
    char* base = smem + buf * WG_STAGE;
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      int64_t m = m0 + prow[q];
      m = m < p.M ? m : p.M - 1;                             // clamped; zeroed in registers
      __builtin_amdgcn_global_load_lds((const void*)(p.dy + m * p.ldy + cy[q]),
                                       LDS_PTR(base + (wave * 2 + q) * 1024), 16, 0, 0);
      __builtin_amdgcn_global_load_lds((const void*)(p.x + m * p.ldx + cx[q]),
                                       LDS_PTR(base + WG_OP + (wave * 2 + q) * 1024), 16, 0, 0);
    }
  };

  fv4 acc[8][4];   // [k fragment][n fragment]
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = fv4{0.f, 0.f, 0.f, 0.f};
  const bool do_cs = p.db != nullptr && k0 == 0 && wk == 0;   // wave-uniform
  float cs[4] = {0.f, 0.f, 0.f, 0.f};
  const bf2_t ones = {(__bf16)1.0f, (__bf16)1.0f};

  for (int i = 0; i < WG_NST - 1 && i < nst; ++i) stage(i, s_begin + i);
  // lane (r16, g) supplies row 4g + (r16 >> 2) (+16) and columns 4 (r16 & 3) of each 16-column block
  const int ra = 4 * g + (r16 >> 2), rb = ra + 16, cq = 4 * (r16 & 3);
  for (int it = 0; it < nst; ++it) {
    const int later = min(nst - 1, it + WG_NST - 2) - it;   // stages issued beyond this one (<= 2)
    if (later >= 2) wg_vm_wait<8>();
    else if (later == 1) wg_vm_wait<4>();
    else wg_vm_wait<0>();
    wg_barrier();                 // stage `it` landed for every wave; stage it-1 read by every wave
    if (!(ABL & 1) && it + WG_NST - 1 < nst) stage((it + WG_NST - 1) & (WG_NST - 1), s_begin + it + WG_NST - 1);
    const char* ty = smem + (it & (WG_NST - 1)) * WG_STAGE;
    const char* tx = ty + WG_OP;
    sv8 fb[4], fa[8];
    if constexpr ((ABL & 4) != 0) {
#pragma unroll
      for (int j = 0; j < 4; ++j) fb[j] = sv8{(short)it, 1, 2, 3, 4, 5, 6, 7};
#pragma unroll
      for (int i = 0; i < 8; ++i) fa[i] = sv8{(short)i, 1, 2, 3, 4, 5, 6, (short)it};
    } else {
      sv4 hb[8], ha[16];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int c = wn * 64 + j * 16 + cq;
        hb[2 * j] = wg_tr_read(ty + wg_off(ra, c));
        hb[2 * j + 1] = wg_tr_read(ty + wg_off(rb, c));
      }
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int c = wk * 128 + i * 16 + cq;
        ha[2 * i] = wg_tr_read(tx + wg_off(ra, c));
        ha[2 * i + 1] = wg_tr_read(tx + wg_off(rb, c));
      }
      wg_lgkm_wait(hb, ha);
#pragma unroll
      for (int j = 0; j < 4; ++j) fb[j] = __builtin_shufflevector(hb[2 * j], hb[2 * j + 1], 0, 1, 2, 3, 4, 5, 6, 7);
#pragma unroll
      for (int i = 0; i < 8; ++i) fa[i] = __builtin_shufflevector(ha[2 * i], ha[2 * i + 1], 0, 1, 2, 3, 4, 5, 6, 7);
    }
    const int64_t m0 = (s_begin + it) * WG_BM;
    if (m0 + WG_BM > p.M) {                                   // last stage: dY rows past M -> 0
      const int valid = (int)(p.M - m0);
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const int row = (e < 4 ? 4 * g + e : 16 + 4 * g + e - 4);
          if (row >= valid) fb[j][e] = 0;
        }
    }
    if (do_cs) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const uint4 u = __builtin_bit_cast(uint4, fb[j]);
        float s = __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(bf2_t, u.x), ones, cs[j], false);
        s = __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(bf2_t, u.y), ones, s, false);
        s = __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(bf2_t, u.z), ones, s, false);
        cs[j] = __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(bf2_t, u.w), ones, s, false);
      }
    }
    if constexpr ((ABL & 2) != 0) {
#pragma unroll
      for (int i = 0; i < 8; ++i) asm volatile("" ::"v"(fa[i]));
#pragma unroll
      for (int j = 0; j < 4; ++j) asm volatile("" ::"v"(fb[j]));
    } else {
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i], fb[j], acc[i][j], 0, 0, 0);
      __builtin_amdgcn_s_setprio(0);
    }
  }

  // lane holds G[n = n0 + wn*64 + 16 j + r16][k = k0 + wk*128 + 16 i + 4 g .. + 3]
  mfma_result_fence();
  const bool direct = p.S == 1;
  float* out = p.out + (direct ? 0 : (int64_t)sl * p.N * p.K);
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int64_t n = n0 + wn * 64 + j * 16 + r16;
    if (n >= p.N) continue;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int64_t k = k0 + wk * 128 + i * 16 + 4 * g;
      if (k >= p.K) continue;
      float4* o = reinterpret_cast<float4*>(out + n * p.K + k);
      const fv4 a = acc[i][j];
      if (direct && p.accumulate) {
        const float4 old = *o;
        *o = make_float4(old.x + a[0], old.y + a[1], old.z + a[2], old.w + a[3]);
      } else {
        *o = make_float4(a[0], a[1], a[2], a[3]);
      }
    }
  }
  if (do_cs) {
    float* dbo = p.db + (direct ? 0 : (int64_t)sl * p.N);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      float v = cs[j];
      v += __shfl_xor(v, 16, 64);                          // the 4 lane groups hold disjoint rows
      v += __shfl_xor(v, 32, 64);
      const int64_t n = n0 + wn * 64 + j * 16 + r16;
      if (g == 0 && n < p.N) dbo[n] = (direct && p.accumulate) ? dbo[n] + v : v;
    }
  }
}

// Two workgroups per CU (DSVT_WGRAD_HALF): a 128 (k) x 256 (n) output tile per 256-thread
// workgroup -- 4 waves, each the same 128 x 64 block and fragment code as above, all on k rows
// 0..127 -- with a 3-stage ring of 24 KiB stages (X rows of 256 B, dY rows of 512 B), 72 KiB per
// workgroup.  The two workgroups of a CU synchronize only themselves, so one's fragment reads and
// loads run under the other's MFMAs instead of all eight waves of the 256 x 256 tile reading,
// then computing, between one barrier and the next.  1.5x the L2 -> LDS bytes per FLOP, which
// costs more than the overlap buys on the full-chip grids (qkv 133.4 vs 127.4 us, fc2 145.7 vs
// 137.8; train step 136.0 / 135.8 vs 137.1 / 137.8 with it everywhere) but not on the 768 x 768
// weights, whose 9 tiles x 8 slices hold 72 CUs: proj 90.8 vs 105.6 us.  Default (2): there only.
namespace {
constexpr int WH_K = 128, WH_N = 256;       // tile: k x n
constexpr int WH_XROWB = 256;               // bytes per staged X row (128 bf16)
constexpr int WH_XOP = WG_BM * WH_XROWB;    // 8 KiB
constexpr int WH_YOP = WG_BM * WG_ROWB;     // 16 KiB
constexpr int WH_STAGE = WH_YOP + WH_XOP;   // [dY | X] 24 KiB
constexpr int WH_NST = 3;

__device__ __forceinline__ int wh_xoff(int row, int c) {      // 256-B rows, 16 chunks, same XOR
  return row * WH_XROWB + ((((c >> 3) ^ ((row & 7) << 1))) << 4) + ((c & 7) << 1);
}
}  // namespace

__global__ __launch_bounds__(256, 2) void wgrad_half_kernel(WgradParams p) {
  __shared__ __attribute__((aligned(16))) char smem[WH_NST * WH_STAGE];
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r16 = lane & 15, g = lane >> 4;
  const int wn = wave;                          // the wave's n columns wn*64 ..
  const int tiles = p.tilesN * p.tilesK;
  const int per_x = (int)(gridDim.x >> 3);
  const int t = (int)(blockIdx.x & 7) * per_x + (int)(blockIdx.x >> 3);
  if (t >= tiles * p.S) return;
  const int sl = t / tiles, tile = t - sl * tiles;
  const int64_t n0 = (int64_t)(tile / p.tilesK) * WH_N, k0 = (int64_t)(tile % p.tilesK) * WH_K;
  const int64_t steps = (p.M + WG_BM - 1) / WG_BM;
  const int64_t s_begin = sl * steps / p.S, s_end = (sl + 1) * steps / p.S;
  const int nst = (int)(s_end - s_begin);

  // DMA roles: dY -- 4 wave-instructions of 2 rows x 512 B; X -- 2 of 4 rows x 256 B
  int yrow[4], xrow[2];
  int64_t cy[4], cx[2];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    yrow[q] = (wave * 4 + q) * 2 + (lane >> 5);
    const int lc = (lane & 31) ^ ((yrow[q] & 7) << 1);
    const int64_t cn = n0 + lc * 8;
    cy[q] = cn < p.N ? cn : p.N - 8;
  }
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    xrow[q] = (wave * 2 + q) * 4 + (lane >> 4);
    const int lc = (lane & 15) ^ ((xrow[q] & 7) << 1);
    const int64_t ck = k0 + lc * 8;
    cx[q] = ck < p.K ? ck : p.K - 8;
  }
  auto stage = [&](int buf, int64_t step) {
    const int64_t m0 = step * WG_BM;
    char* base = smem + buf * WH_STAGE;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      int64_t m = m0 + yrow[q];
      m = m < p.M ? m : p.M - 1;                               // clamped; zeroed in registers
      __builtin_amdgcn_global_load_lds((const void*)(p.dy + m * p.ldy + cy[q]),
                                       LDS_PTR(base + (wave * 4 + q) * 1024), 16, 0, 0);
    }
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      int64_t m = m0 + xrow[q];
      m = m < p.M ? m : p.M - 1;
      __builtin_amdgcn_global_load_lds((const void*)(p.x + m * p.ldx + cx[q]),
                                       LDS_PTR(base + WH_YOP + (wave * 2 + q) * 1024), 16, 0, 0);
    }
  };

  fv4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = fv4{0.f, 0.f, 0.f, 0.f};
  const bool do_cs = p.db != nullptr && k0 == 0;               // workgroup-uniform
  float cs[4] = {0.f, 0.f, 0.f, 0.f};
  const bf2_t ones = {(__bf16)1.0f, (__bf16)1.0f};

  for (int i = 0; i < WH_NST - 1 && i < nst; ++i) stage(i, s_begin + i);
  const int ra = 4 * g + (r16 >> 2), rb = ra + 16, cq = 4 * (r16 & 3);
  int buf = 0;
  for (int it = 0; it < nst; ++it) {
    if (it + 1 < nst) wg_vm_wait<6>();                         // stage it+1 may stay in flight
    else wg_vm_wait<0>();
    wg_barrier();                 // stage `it` landed for every wave; stage it-1 read by every wave
    if (it + WH_NST - 1 < nst) {
      const int nb = buf == 0 ? WH_NST - 1 : buf - 1;           // (it + 2) % 3
      stage(nb, s_begin + it + WH_NST - 1);
    }
    const char* ty = smem + buf * WH_STAGE;
    const char* tx = ty + WH_YOP;
    buf = buf == WH_NST - 1 ? 0 : buf + 1;
    sv4 hb[8], ha[16];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int c = wn * 64 + j * 16 + cq;
      hb[2 * j] = wg_tr_read(ty + wg_off(ra, c));
      hb[2 * j + 1] = wg_tr_read(ty + wg_off(rb, c));
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int c = i * 16 + cq;
      ha[2 * i] = wg_tr_read(tx + wh_xoff(ra, c));
      ha[2 * i + 1] = wg_tr_read(tx + wh_xoff(rb, c));
    }
    wg_lgkm_wait(hb, ha);
    sv8 fb[4], fa[8];
#pragma unroll
    for (int j = 0; j < 4; ++j) fb[j] = __builtin_shufflevector(hb[2 * j], hb[2 * j + 1], 0, 1, 2, 3, 4, 5, 6, 7);
#pragma unroll
    for (int i = 0; i < 8; ++i) fa[i] = __builtin_shufflevector(ha[2 * i], ha[2 * i + 1], 0, 1, 2, 3, 4, 5, 6, 7);
    const int64_t m0 = (s_begin + it) * WG_BM;
    if (m0 + WG_BM > p.M) {                                   // last stage: dY rows past M -> 0
      const int valid = (int)(p.M - m0);
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const int row = (e < 4 ? 4 * g + e : 16 + 4 * g + e - 4);
          if (row >= valid) fb[j][e] = 0;
        }
    }
    if (do_cs) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const uint4 u = __builtin_bit_cast(uint4, fb[j]);
        float s = __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(bf2_t, u.x), ones, cs[j], false);
        s = __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(bf2_t, u.y), ones, s, false);
        s = __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(bf2_t, u.z), ones, s, false);
        cs[j] = __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(bf2_t, u.w), ones, s, false);
      }
    }
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i], fb[j], acc[i][j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
  }

  mfma_result_fence();
  const bool direct = p.S == 1;
  float* out = p.out + (direct ? 0 : (int64_t)sl * p.N * p.K);
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int64_t n = n0 + wn * 64 + j * 16 + r16;
    if (n >= p.N) continue;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int64_t k = k0 + i * 16 + 4 * g;
      if (k >= p.K) continue;
      float4* o = reinterpret_cast<float4*>(out + n * p.K + k);
      const fv4 a = acc[i][j];
      if (direct && p.accumulate) {
        const float4 old = *o;
        *o = make_float4(old.x + a[0], old.y + a[1], old.z + a[2], old.w + a[3]);
      } else {
        *o = make_float4(a[0], a[1], a[2], a[3]);
      }
    }
  }
  if (do_cs) {
    float* dbo = p.db + (direct ? 0 : (int64_t)sl * p.N);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      float v = cs[j];
      v += __shfl_xor(v, 16, 64);
      v += __shfl_xor(v, 32, 64);
      const int64_t n = n0 + wn * 64 + j * 16 + r16;
      if (g == 0 && n < p.N) dbo[n] = (direct && p.accumulate) ? dbo[n] + v : v;
    }
  }
}

// dst (+)= sum over the S slices of the partials, in slice order (float4 per thread); the
// workgroups past `gblocks` do the same for the bias partials (one launch for both)
__global__ __launch_bounds__(256) void wgrad_reduce_kernel(const float* __restrict__ part, int64_t S, int64_t n4,
                                                           float* __restrict__ G, const float* __restrict__ dpart,
                                                           int64_t d4, float* __restrict__ db, int gblocks,
                                                           int accumulate) {
  const bool bias = (int)blockIdx.x >= gblocks;
  const float* src = bias ? dpart : part;
  float* dst = bias ? db : G;
  const int64_t n = bias ? d4 : n4;
  const int64_t b0 = bias ? blockIdx.x - gblocks : blockIdx.x, nb = bias ? gridDim.x - gblocks : gblocks;
  for (int64_t i = b0 * 256 + threadIdx.x; i < n; i += nb * 256) {
    float4 a = accumulate ? reinterpret_cast<const float4*>(dst)[i] : make_float4(0.f, 0.f, 0.f, 0.f);
    for (int64_t s = 0; s < S; ++s) {
      const float4 v = reinterpret_cast<const float4*>(src)[s * n + i];
      a.x += v.x; a.y += v.y; a.z += v.z; a.w += v.w;
    }
    reinterpret_cast<float4*>(dst)[i] = a;
  }
}

// M-slices: tiles x S <= 256 workgroups (one per CU, one round), each slice >= 8 stages, and
// at most 8 slices: every slice adds an N x K fp32 partial written and re-read, and in the
// training step these products run on a side stream beside the dX chain, so total traffic
// counts more than filling the chip (r04 train step: cap 8 > 6, 10, 12, 16 > uncapped (28 for the
// 768 x 768 weights) > 4 > 2; tools/train_step.py, DSVT_WGRAD_MAXS).  r05, after the kernel's
// drain fix (interleaved, tools/ab_train.sh): 12 137.5 / 137.6 / 137.6 / 137.5, 16 137.5 / 138.0,
// 8 136.5 / 136.9, 28 136.8 / 136.5, 6 133.9 / 134.2, 4 123.4 / 123.8 -> 12 (only the 768 x 768
// weights, 9 tiles, reach it; their grid stays on the two-per-CU kernel, 108 < 128 workgroups)
int64_t wgrad_slices(int64_t M, int64_t N, int64_t K) {
  const int64_t tiles = ((N + WG_T - 1) / WG_T) * ((K + WG_T - 1) / WG_T);
  const int64_t steps = (M + WG_BM - 1) / WG_BM;
  static const int64_t max_s = getenv("DSVT_WGRAD_MAXS") ? atoll(getenv("DSVT_WGRAD_MAXS")) : 12;
  int64_t S = 256 / tiles;
  if (S > max_s) S = max_s;
  if (S > steps / 8) S = steps / 8;
  return S < 1 ? 1 : S;
}

// workspace floats: the G partial slabs, then (with a bias) the db partial rows
int64_t wgrad_workspace_floats(int64_t M, int64_t N, int64_t K) {
  const int64_t S = wgrad_slices(M, N, K);
  return S > 1 ? S * N * K + S * N : 0;
}

hipError_t launch_wgrad(const bf16_t* dy, int64_t ldy, const bf16_t* x, int64_t ldx, float* G, float* db, int64_t M,
                        int64_t N, int64_t K, int accumulate, float* partial, hipStream_t s) {
  const int64_t S = wgrad_slices(M, N, K);
  float* dbp = db == nullptr ? nullptr : (S > 1 ? partial + S * N * K : db);
  static const int abl = getenv("DSVT_WGRAD_ABL") ? atoi(getenv("DSVT_WGRAD_ABL")) : 0;   // diagnostics only
#ifndef DSVT_WGRAD_HALF
#define DSVT_WGRAD_HALF 2   // A/B (train step, 3 interleaved rounds): 138.0 / 137.9 / 138.2 vs 137.4 / 136.8 / 136.7
#endif
  static const int half = getenv("DSVT_WGRAD_HALF") ? atoi(getenv("DSVT_WGRAD_HALF")) : DSVT_WGRAD_HALF;
  // 2: only where the 256 x 256 grid holds fewer than half the CUs (the 768 x 768 weights: 9 tiles)
  const int64_t tiles256 = ((N + WG_T - 1) / WG_T) * ((K + WG_T - 1) / WG_T);
  if (abl == 0 && (half == 1 || (half == 2 && tiles256 * S < 128))) {
    const int tilesN = (int)((N + WH_N - 1) / WH_N), tilesK = (int)((K + WH_K - 1) / WH_K);
    WgradParams p{dy, ldy, x, ldx, S > 1 ? partial : G, dbp, M, N, K, (int)S, tilesN, tilesK, accumulate};
    const int64_t total = (int64_t)tilesN * tilesK * S;
    wgrad_half_kernel<<<dim3((unsigned)((total + 7) / 8 * 8)), 256, 0, s>>>(p);
  } else {
  const int tilesN = (int)((N + WG_T - 1) / WG_T), tilesK = (int)((K + WG_T - 1) / WG_T);
  WgradParams p{dy, ldy, x, ldx, S > 1 ? partial : G, dbp, M, N, K, (int)S, tilesN, tilesK, accumulate};
  const int64_t total = (int64_t)tilesN * tilesK * S;
  const dim3 grid((unsigned)((total + 7) / 8 * 8));
  switch (abl) {
    case 1: wgrad_kernel<1><<<grid, 512, 0, s>>>(p); break;
    case 2: wgrad_kernel<2><<<grid, 512, 0, s>>>(p); break;
    case 3: wgrad_kernel<3><<<grid, 512, 0, s>>>(p); break;
    case 4: wgrad_kernel<4><<<grid, 512, 0, s>>>(p); break;
    case 6: wgrad_kernel<6><<<grid, 512, 0, s>>>(p); break;
    default: wgrad_kernel<0><<<grid, 512, 0, s>>>(p); break;
  }
  }
  if (S > 1) {
    const int64_t n4 = N * K / 4, d4 = db ? N / 4 : 0;
    int gblocks = (int)((n4 + 255) / 256);
    if (gblocks > 2048) gblocks = 2048;
    const int dblocks = (int)((d4 + 255) / 256);
    wgrad_reduce_kernel<<<gblocks + dblocks, 256, 0, s>>>(partial, S, n4, G, partial + S * N * K, d4, db, gblocks,
                                                          accumulate);
  }
  return hipGetLastError();
}

}  // namespace dsvt
