// 256x256 bf16 MFMA GEMM with a phase-interleaved K loop (variant 20), for the widest
// hot-path projections: qkv (N = 2304) and fc1 (N = 3072) over M = 13.9k-25.1k tokens, K = 768.
//
// Geometry: one 512-thread workgroup (8 waves, 2 x 4) per CU, 128 KiB of LDS = two K-tile
// buffers of BK = 64 (128-byte rows).  Wave (wr, wc) owns the 128 x 64 output block at
// (wr*128, wc*64): acc[8][4] 16x16 fragments, split in four quadrants
//   q0 = rows 0-63 x cols 0-31, q1 = rows 0-63 x cols 32-63, q2 = rows 64-127 x cols 32-63,
//   q3 = rows 64-127 x cols 0-31,
// and one K-tile is four PHASES, one quadrant each (16 MFMA 16x16x32 per wave per phase, issued
// k-half outer so that no two consecutive MFMAs share an accumulator).
// The K-tile is staged as four 16 KiB "half-tiles" grouped by the phase that first reads them:
//   AT = A rows {0-63, 128-191} (the q0/q1 rows of both wave rows), AB = A rows {64-127, 192-255},
//   BL = W rows {0-31, 64-95, 128-159, 192-223},                     BR = the other W rows,
// so phase 0 reads AT + BL, phase 1 BR, phase 2 AB, phase 3 nothing (all operands in registers).
// Every phase issues ONE half-tile of LDS-DMA (2 global_load_lds_dwordx4 per thread), in the
// stream order AT, BL, BR, AB of K-tile u at phases 4u-6 .. 4u-3, i.e. two K-tiles ahead of
// the reads of the same buffer, and waits `vmcnt(8)` (four half-tiles in flight) before its
// first barrier; a half-tile is read one phase after that wait and re-staged >= 2 phases after
// its last read (the two wave rows run one barrier apart, see below).
//
// Per phase: ds_read_b128 subtile -> issue stage -> s_waitcnt vmcnt -> s_barrier ->
// lgkmcnt(0) -> setprio(1) 16 x MFMA setprio(0) -> s_barrier.  Wave row 1 passes one extra
// barrier at the start (wave row 0 one at the end), so the LDS reads / load issue of one half of
// every SIMD's two waves overlap the MFMA cluster of the other half.
//
// The K-tile stream is continuous over all output tiles of the (persistent) workgroup: the
// loads of the next tile are already in flight while a tile's epilogue stores run.  Stores
// count on vmcnt in issue order, so the four phases after a full-tile epilogue wait
// vmcnt(8 + its store count).  LDS swizzle: 16-byte chunk' = chunk ^ ((row >> 1) & 7) of the
// 128-byte row (applied to the DMA source address and to the read address); the sixteen rows a
// 16-lane group reads then cover all 64 banks.
#include "gemm_epi.h"

#ifndef DSVT_8PH_GELU_NOFAST
#define DSVT_8PH_GELU_NOFAST 1   // the 16-byte pair-store path spills (201 VGPRs with the fast GELU too)
#endif

namespace dsvt {

namespace {

constexpr int P8_ROWB = 128;              // bytes per LDS row: 64 bf16 of K
constexpr int P8_HALF = 128 * P8_ROWB;    // one half-tile, 16 KiB
constexpr int P8_BUF = 4 * P8_HALF;       // one K-tile (AT, AB, BL, BR), 64 KiB
enum { H_AT = 0, H_AB = 1, H_BL = 2, H_BR = 3 };

// s_waitcnt vmcnt(N) for N <= 63 (gfx9 split vmcnt field), lgkmcnt / expcnt untouched
template <int N>
__device__ __forceinline__ void vm_wait() {
  static_assert(N >= 0 && N < 64, "vmcnt immediate");
  __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | 0x0F70);
}

__device__ __forceinline__ void p8_barrier() {
  __builtin_amdgcn_sched_barrier(0);
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
}

#ifndef DSVT_8PH_ASM_RD
#define DSVT_8PH_ASM_RD 1
#endif
// Fragment reads as inline-asm ds_read_b128 at an immediate offset (DSVT_8PH_ASM_RD, default):
// with plain LDS loads the compiler drained every in-flight LDS-DMA stage (s_waitcnt vmcnt(0),
// two K-tiles of prefetch) at the K-loop head of the residual / GELU-save instantiations.  The
// asm reads are not tracked: the phase's own counted vmcnt wait + barrier order them after the
// DMA they read, and p8_tie* (lgkmcnt(0) tied to the fragments) orders their use.
template <int OFF>
__device__ __forceinline__ sv8 p8_rd(unsigned a) {
  sv8 r;
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(r) : "v"(a), "i"(OFF));
  return r;
}
__device__ __forceinline__ unsigned p8_lds(const char* p) {
  return (unsigned)(uintptr_t)(__attribute__((address_space(3))) const char*)p;
}
__device__ __forceinline__ void p8_tie4(sv8 (&f)[2][2]) {
  asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(f[0][0]), "+v"(f[0][1]), "+v"(f[1][0]), "+v"(f[1][1]));
}
__device__ __forceinline__ void p8_tie8(sv8 (&f)[4][2]) {
  asm volatile("s_waitcnt lgkmcnt(0)"
               : "+v"(f[0][0]), "+v"(f[0][1]), "+v"(f[1][0]), "+v"(f[1][1]), "+v"(f[2][0]), "+v"(f[2][1]),
                 "+v"(f[3][0]), "+v"(f[3][1]));
}

}  // namespace

// ABL (diagnostic builds, benchmarking only; 0 = normal): bit 0 no wave-row stagger, bit 1 no
// loads after the prologue (stale tiles), bit 2 no MFMA (reads kept live), bit 3 no setprio,
// bit 4 no epilogue (accumulators kept live), bit 5 non-temporal output stores, bit 6 epilogue
// without its stores
// NFULL: N % 256 == 0 (every tile full in N), bias / GELU with a bf16 output -- the epilogue is
// the 16-byte store path alone for every tile (rows past M clamped, gemm_epi.h)
// FUSE 1 (dsvt_gemm_lnx_fwd, bias / GELU): the LayerNorm folded in -- A rows through the A row
// map, accumulators from zero, ln_affine before the epilogue; FUSE 2 (dsvt_gemm_resid_stats_fwd,
// residual): the epilogue also writes the bf16 copy and the LN partials of the updated rows.
template <int EPI, bool OUT_F32, int ABL = 0, bool NFULL = false, int FUSE = 0>
__global__ __launch_bounds__(512, 1) void gemm_8ph_kernel(GemmParams p) {
  constexpr bool CLAMPED = NFULL && (EPI == EPI_BIAS || EPI == EPI_GELU) && !OUT_F32;
  // VMEM instructions of a full-tile register epilogue: bf16 bias / GELU -> 16 pair stores
  constexpr int S_EPI = ((EPI == EPI_BIAS || CLAMPED) && !OUT_F32 && !(ABL & 64)) ? 16 : 0;
  __shared__ __attribute__((aligned(16))) char smem[2 * P8_BUF];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wave >> 2, wc = wave & 3;
  const int r16 = lane & 15, g = lane >> 4;
  const int tilesN = (int)((p.N + 255) >> 8);
  const int tiles = (int)((p.M + 255) >> 8) * tilesN;
  // XCD-contiguous tile ranges (block b runs on XCD b % 8; the grid is a multiple of 8)
  const int G = gridDim.x, b = blockIdx.x, xcd = b & 7, li = b >> 3, per_x = G >> 3;
  const int nk = (int)(p.K >> 6);
  // This workgroup's K-tile stream runs over its strided share of the tiles (XCD-contiguous
  // ranges): tiles t_first + tl * per_x, tl = 0 .. tl_end-1.
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
  // ---- LDS-DMA source offsets (32-bit, checked on the host) of the four half-tiles
  const int srow = tid >> 3;                                   // half-tile row within a 64-row piece
  const uint32_t schunk = (uint32_t)(((tid & 7) ^ ((tid >> 4) & 7)) << 4);
  uint32_t oAT[2], oAB[2], oBL[2], oBR[2];
  const int tilesM = (int)((p.M + 255) >> 8), GM = p.tile_group;
  auto tile_mn = [&](int tl, int64_t& m0, int64_t& n0) {
    const int t = t_first + tl * per_x;
    if (GM <= 0) {
      m0 = (int64_t)(t / tilesN) * 256;
      n0 = (int64_t)(t % tilesN) * 256;
    } else {                            // groups of GM m-tile rows, n-column-major inside
      const int grp = t / (GM * tilesN), w = t - grp * GM * tilesN;
      const int fm = grp * GM, gm = min(GM, tilesM - fm);
      m0 = (int64_t)(fm + w % gm) * 256;
      n0 = (int64_t)(w / gm) * 256;
    }
  };
  auto a_off = [&](int64_t gr) -> uint32_t {   // gr: row of the tile (rows past M clamped)
    gr = gr < p.M ? gr : p.M - 1;
    if constexpr (FUSE == 1) {             // the A row map (32-bit: rows < 2^31, host-checked)
      const uint32_t m = (uint32_t)gr, rpg = (uint32_t)(p.a_rpg < p.M ? p.a_rpg : p.M);
      gr = (int64_t)((m / rpg) * (uint32_t)p.a_gstride + (uint32_t)p.a_goff + m % rpg);
    }
    return (uint32_t)(gr * lda_b) + schunk;
  };
  auto b_off = [&](int64_t gr) -> uint32_t {
    gr = gr < p.N ? gr : p.N - 1;
    return (uint32_t)(gr * ldw_b) + schunk;
  };
  // stager of parts AT / BL (runs two K-tiles ahead of the compute) and of BR / AB (one ahead)
  auto set_atbl = [&](int tl) {
    int64_t m0, n0;
    tile_mn(tl, m0, n0);
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      oAT[q] = a_off(m0 + q * 128 + srow);
      oBL[q] = b_off(n0 + (2 * q + (srow >> 5)) * 64 + (srow & 31));
    }
  };
  auto set_brab = [&](int tl) {
    int64_t m0, n0;
    tile_mn(tl, m0, n0);
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      oAB[q] = a_off(m0 + q * 128 + 64 + srow);
      oBR[q] = b_off(n0 + (2 * q + (srow >> 5)) * 64 + 32 + (srow & 31));
    }
  };
#define P8_STAGE(H, OFF, SRC, BUFOFF, KB)                                                           \
  if (!(ABL & 2) || prologue_) {                                                                     \
    char* d_ = smem + (BUFOFF) + (H) * P8_HALF + wave * 1024;                                       \
    __builtin_amdgcn_global_load_lds((const void*)((SRC) + (OFF[0] + (uint32_t)(KB))), LDS_PTR(d_), \
                                     16, 0, 0);                                                     \
    __builtin_amdgcn_global_load_lds((const void*)((SRC) + (OFF[1] + (uint32_t)(KB))),             \
                                     LDS_PTR(d_ + 64 * P8_ROWB), 16, 0, 0);                         \
  }

  // ---- fragment read offsets (bytes within a half-tile)
  const int xs = (r16 >> 1) & 7;
  const int rdA = (wr * 64 + r16) * P8_ROWB, rdB = (wc * 32 + r16) * P8_ROWB;
  const int cs0 = (g ^ xs) << 4, cs1 = ((4 + g) ^ xs) << 4;
  sv8 fa[4][2], fbl[2][2], fbr[2][2];
#if DSVT_8PH_ASM_RD
#define P8_RD(DST, H, BASE, CB, N)                                                                     \
  {                                                                                                    \
    const unsigned b_ = p8_lds(smem + (CB) + (BASE)), a0_ = b_ + cs0, a1_ = b_ + cs1;                  \
    DST[0][0] = p8_rd<(H) * P8_HALF>(a0_);                                                             \
    DST[0][1] = p8_rd<(H) * P8_HALF>(a1_);                                                             \
    DST[1][0] = p8_rd<(H) * P8_HALF + 16 * P8_ROWB>(a0_);                                              \
    DST[1][1] = p8_rd<(H) * P8_HALF + 16 * P8_ROWB>(a1_);                                              \
    if constexpr ((N) == 4) {                                                                          \
      DST[(N) - 2][0] = p8_rd<(H) * P8_HALF + 32 * P8_ROWB>(a0_);                                      \
      DST[(N) - 2][1] = p8_rd<(H) * P8_HALF + 32 * P8_ROWB>(a1_);                                      \
      DST[(N) - 1][0] = p8_rd<(H) * P8_HALF + 48 * P8_ROWB>(a0_);                                      \
      DST[(N) - 1][1] = p8_rd<(H) * P8_HALF + 48 * P8_ROWB>(a1_);                                      \
    }                                                                                                  \
  }
#define P8_TIE(STMT) STMT
#else
#define P8_RD(DST, H, BASE, CB, N)                                                                     \
  _Pragma("unroll") for (int f_ = 0; f_ < (N); ++f_) {                                                \
    const char* s_ = smem + (CB) + (H) * P8_HALF + (BASE) + f_ * 16 * P8_ROWB;                        \
    DST[f_][0] = *reinterpret_cast<const sv8*>(s_ + cs0);                                             \
    DST[f_][1] = *reinterpret_cast<const sv8*>(s_ + cs1);                                             \
  }
#define P8_TIE(STMT)
#endif
#define P8_MFMA(I0, J0, FB)                                                                            \
  {                                                                                                    \
    if (!(ABL & 8)) __builtin_amdgcn_s_setprio(1);                                                     \
    _Pragma("unroll") for (int s_ = 0; s_ < 2; ++s_)                                                   \
    _Pragma("unroll") for (int i_ = 0; i_ < 4; ++i_)                                                   \
    _Pragma("unroll") for (int j_ = 0; j_ < 2; ++j_) {                                                 \
      if (ABL & 4) {                                                                                   \
        asm volatile("" ::"v"(FB[j_][s_]), "v"(fa[i_][s_]));                                           \
      } else {                                                                                         \
        acc[(I0) + i_][(J0) + j_] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(FB[j_][s_], fa[i_][s_],    \
                                                                        acc[(I0) + i_][(J0) + j_], 0, 0, 0); \
      }                                                                                                \
    }                                                                                                  \
    if (!(ABL & 8)) __builtin_amdgcn_s_setprio(0);                                                     \
  }
// wait for the half-tile the NEXT phase reads; VALID = this phase issued a stage.  After a
// full-tile epilogue its S_EPI stores sit between the awaited half-tile and the four younger
// stages (issue order), for the four phases of the next K-tile.
#define P8_WAIT(VALID)                                     \
  {                                                        \
    if (!(VALID)) vm_wait<0>();                            \
    else if (S_EPI > 0 && post) vm_wait<8 + S_EPI>();      \
    else vm_wait<8>();                                     \
  }
#define P8_COMPUTE(MFMA_STMT, TIE)                         \
  {                                                        \
    p8_barrier();                                          \
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");     \
    TIE;                                                   \
    __builtin_amdgcn_sched_barrier(0);                     \
    MFMA_STMT;                                             \
    p8_barrier();                                          \
  }

  // ---- prologue: K-tile 0 complete, K-tile 1 parts AT / BL
  int tl1, k1, tl2, k2;                 // stream positions u1 = j + 1 (BR, AB), u2 = j + 2 (AT, BL)
  bool prologue_ = true;
  set_atbl(0);
  set_brab(0);
  P8_STAGE(H_AT, oAT, A, 0, 0);
  P8_STAGE(H_BL, oBL, W, 0, 0);
  P8_STAGE(H_BR, oBR, W, 0, 0);
  P8_STAGE(H_AB, oAB, A, 0, 0);
  tl1 = 0; k1 = 0;
  adv(tl1, k1);
  tl2 = tl1; k2 = k1;
  adv(tl2, k2);
  if (J > 1) {
    set_atbl(tl1);
    P8_STAGE(H_AT, oAT, A, P8_BUF, k1 * P8_ROWB);
    P8_STAGE(H_BL, oBL, W, P8_BUF, k1 * P8_ROWB);
    vm_wait<8>();                       // AT(0), BL(0) retired
  } else {
    vm_wait<0>();
  }
  set_brab(tl1);
  set_atbl(tl2);
  p8_barrier();
  if (!(ABL & 1) && wr == 1) p8_barrier();  // wave row 1 runs one barrier behind

  // accumulators start from the bias of their columns (the epilogue adds none)
  constexpr bool BIAS_IN_ACC = EPI != EPI_DGELU;
  fv4 acc[8][4];
  auto init_acc = [&](int tl) {
    float4 b4[4];
    // (EPI_RESID with DropPath row scales: the epilogue adds s[m] * bias instead)
    int64_t bm0 = 0, bn0 = 0;
    tile_mn(tl, bm0, bn0);
    if (BIAS_IN_ACC && FUSE != 1 && p.bias && !(EPI == EPI_RESID && p.row_scale)) {
      const int64_t cbase = bn0 + wc * 64;
      if (cbase + 64 <= p.N) {
        bias_frag4(p.bias, cbase, g, b4);
      } else {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int64_t n = cbase + j * 16 + 4 * g;
          b4[j] = n < p.N ? *reinterpret_cast<const float4*>(p.bias + n) : make_float4(0.f, 0.f, 0.f, 0.f);
        }
      }
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j) b4[j] = make_float4(0.f, 0.f, 0.f, 0.f);
    }
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = fv4{b4[j].x, b4[j].y, b4[j].z, b4[j].w};
  };
  init_acc(0);
  prologue_ = false;
  int tlc = 0, kc = 0;                  // compute position
  bool post = false;                    // previous K-tile ended with a full-tile epilogue

  for (int j = 0; j < J; ++j) {
    const int cb = (j & 1) * P8_BUF, sb1 = cb ^ P8_BUF, sb2 = cb;
    const bool v1 = j + 1 < J, v2 = j + 2 < J;
    const int kb1 = k1 * P8_ROWB, kb2 = k2 * P8_ROWB;
    // phase 0: read BL + AT, stage BR(j+1), quadrant (AT, BL)
    P8_RD(fbl, H_BL, rdB, cb, 2);
    __builtin_amdgcn_sched_barrier(0);
    P8_RD(fa, H_AT, rdA, cb, 4);
    if (v1) P8_STAGE(H_BR, oBR, W, sb1, kb1);
    P8_WAIT(v1);
    P8_COMPUTE(P8_MFMA(0, 0, fbl), P8_TIE((p8_tie4(fbl), p8_tie8(fa))));
    // phase 1: read BR, stage AB(j+1), quadrant (AT, BR)
    P8_RD(fbr, H_BR, rdB, cb, 2);
    if (v1) P8_STAGE(H_AB, oAB, A, sb1, kb1);
    P8_WAIT(v1);
    P8_COMPUTE(P8_MFMA(0, 2, fbr), P8_TIE(p8_tie4(fbr)));
    // phase 2: read AB, stage AT(j+2), quadrant (AB, BR)
    P8_RD(fa, H_AB, rdA, cb, 4);
    if (v2) P8_STAGE(H_AT, oAT, A, sb2, kb2);
    P8_WAIT(v2);
    P8_COMPUTE(P8_MFMA(4, 2, fbr), P8_TIE(p8_tie8(fa)));
    // phase 3: no reads, stage BL(j+2), quadrant (AB, BL)
    if (v2) P8_STAGE(H_BL, oBL, W, sb2, kb2);
    P8_WAIT(v2);
    P8_COMPUTE(P8_MFMA(4, 0, fbl), );

    post = false;
    if (++kc == nk) {                     // tile done: register epilogue
      int64_t m0, n0;
      tile_mn(tlc, m0, n0);
      const int64_t rbase = m0 + wr * 128, cbase = n0 + wc * 64;
      mfma_result_fence();
      if constexpr ((ABL & 16) != 0) {
#pragma unroll
        for (int i = 0; i < 8; ++i)
#pragma unroll
          for (int jj = 0; jj < 4; ++jj) asm volatile("" ::"v"(acc[i][jj]));
      } else if constexpr (FUSE == 2) {
        epilogue_resid_stats<8, 4>(p, acc, rbase, cbase, r16, g);
      } else {
        if constexpr (FUSE == 1) {
          ln_affine<8, 4>(p, acc, rbase, cbase, r16, g);
          __builtin_amdgcn_sched_barrier(0);
        }
        epilogue_direct<8, 4, EPI, OUT_F32, (ABL & 32) ? 1 : (ABL & 128) ? 2 : 0, (ABL & 64) != 0, BIAS_IN_ACC, (EPI == EPI_GELU && DSVT_8PH_GELU_NOFAST), EPI == EPI_GELU_SAVE, NFULL, true>(p, acc, rbase, cbase,
                                                                                          r16, g);
      }
      post = S_EPI > 0 && (CLAMPED || (rbase + 128 <= p.M && cbase + 64 <= p.N));
      kc = 0;
      ++tlc;
      __builtin_amdgcn_sched_barrier(0);   // keep the next tile's bias loads after the stores
      if (tlc < tl_end) init_acc(tlc);
    }
    // advance the stagers
    { const int o = tl1; adv(tl1, k1); if (tl1 != o && tl1 < tl_end) set_brab(tl1); }
    { const int o = tl2; adv(tl2, k2); if (tl2 != o && tl2 < tl_end) set_atbl(tl2); }
  }
  if (!(ABL & 1) && wr == 0) p8_barrier();  // balance the stagger barrier
#undef P8_STAGE
#undef P8_RD
#undef P8_MFMA
#undef P8_WAIT
#undef P8_COMPUTE
#undef P8_TIE
}

// K a multiple of 64, 32-bit LDS-DMA source offsets, no patch-embed epilogue.  (The GELU
// epilogue takes the general per-fragment store path: with the 16-byte pair packing its 128
// erf-GELUs per lane do not fit beside the loop state without spilling.)
bool gemm_8ph_ok(const GemmParams& p, int epi) {
  return p.K >= 64 && p.K % 64 == 0 && p.M >= 1 && p.N >= 1 && epi != EPI_PATCH &&
         (p.M - 1) * p.lda * 2 + p.K * 2 <= (int64_t)UINT32_MAX && (p.N - 1) * p.ldw * 2 + p.K * 2 <= (int64_t)UINT32_MAX;
}

hipError_t launch_gemm_8ph(const GemmParams& p, int epi, int out_f32, hipStream_t s, int abl) {
  if (!gemm_8ph_ok(p, epi)) return hipErrorInvalidValue;
  const int64_t tiles = ((p.M + 255) / 256) * ((p.N + 255) / 256);
  int64_t G = 256;                                    // one workgroup per CU (128 KiB LDS)
  const int64_t per_x = (tiles + 7) / 8;
  if (per_x * 8 < G) G = per_x * 8;
  dim3 grid((unsigned)G), block(512);
#define DSVT_K(E, F) gemm_8ph_kernel<E, F><<<grid, block, 0, s>>>(p)
  if (abl) {                                          // diagnostic builds: EPI_BIAS, bf16 out
    if (abl == 16 && epi == EPI_RESID) {              // the residual GEMM's K loop alone (no epilogue)
      gemm_8ph_kernel<EPI_RESID, true, 16><<<grid, block, 0, s>>>(p);
      return hipGetLastError();
    }
    if (epi != EPI_BIAS || out_f32) return hipErrorInvalidValue;
    switch (abl) {
      case 1: gemm_8ph_kernel<EPI_BIAS, false, 1><<<grid, block, 0, s>>>(p); break;
      case 2: gemm_8ph_kernel<EPI_BIAS, false, 2><<<grid, block, 0, s>>>(p); break;
      case 4: gemm_8ph_kernel<EPI_BIAS, false, 4><<<grid, block, 0, s>>>(p); break;
      case 8: gemm_8ph_kernel<EPI_BIAS, false, 8><<<grid, block, 0, s>>>(p); break;
      case 16: gemm_8ph_kernel<EPI_BIAS, false, 16><<<grid, block, 0, s>>>(p); break;
      case 18: gemm_8ph_kernel<EPI_BIAS, false, 18><<<grid, block, 0, s>>>(p); break;
      case 32: gemm_8ph_kernel<EPI_BIAS, false, 32><<<grid, block, 0, s>>>(p); break;
      case 64: gemm_8ph_kernel<EPI_BIAS, false, 64><<<grid, block, 0, s>>>(p); break;
      default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
  }
  const bool nfull = p.N % 256 == 0 && !out_f32;
  if (p.ln_stats) {                                   // LayerNorm folded in (dsvt_gemm_lnx_fwd)
    if (!nfull || !p.ln_wsum) return hipErrorInvalidValue;
    if (epi == EPI_BIAS) gemm_8ph_kernel<EPI_BIAS, false, 0, true, 1><<<grid, block, 0, s>>>(p);
    else if (epi == EPI_GELU) gemm_8ph_kernel<EPI_GELU, false, 0, true, 1><<<grid, block, 0, s>>>(p);
    else return hipErrorInvalidValue;
    return hipGetLastError();
  }
  if (p.stats_out) {                                  // residual + LN inputs (dsvt_gemm_resid_stats_fwd)
    if (epi != EPI_RESID || p.row_scale || !p.xb_out || p.N % 64) return hipErrorInvalidValue;
    gemm_8ph_kernel<EPI_RESID, true, 0, false, 2><<<grid, block, 0, s>>>(p);
    return hipGetLastError();
  }
  switch (epi) {
    case EPI_BIAS:
      if (out_f32) DSVT_K(EPI_BIAS, true);
      else if (nfull) gemm_8ph_kernel<EPI_BIAS, false, 0, true><<<grid, block, 0, s>>>(p);
      else DSVT_K(EPI_BIAS, false);
      break;
    case EPI_RESID: DSVT_K(EPI_RESID, true); break;
    case EPI_GELU:
      if (out_f32) DSVT_K(EPI_GELU, true);
      else if (nfull) gemm_8ph_kernel<EPI_GELU, false, 0, true><<<grid, block, 0, s>>>(p);
      else DSVT_K(EPI_GELU, false);
      break;
    case EPI_GELU_SAVE: DSVT_K(EPI_GELU_SAVE, false); break;
    case EPI_DGELU: if (out_f32) DSVT_K(EPI_DGELU, true); else DSVT_K(EPI_DGELU, false); break;
    default: return hipErrorInvalidValue;
  }
#undef DSVT_K
  return hipGetLastError();
}

}  // namespace dsvt
