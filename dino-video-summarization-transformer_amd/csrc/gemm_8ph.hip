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
#include <stdlib.h>

#include "gemm_epi.h"

#ifndef DSVT_RESID_SEPI
#define DSVT_RESID_SEPI 0   // 55: leave the residual epilogue in flight (measured slower: fc2 171 vs 166 us)
#endif
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

}  // namespace

// ABL (diagnostic builds, benchmarking only; 0 = normal): bit 0 no wave-row stagger, bit 1 no
// loads after the prologue (stale tiles), bit 2 no MFMA (reads kept live), bit 3 no setprio,
// bit 4 no epilogue (accumulators kept live), bit 5 non-temporal output stores, bit 7 sc1 output
// stores (DSVT_8PH_SC1, full-N bias / GELU), bit 6 epilogue
// without its stores
// NFULL: N % 256 == 0 (every tile full in N), bias / GELU with a bf16 output -- the epilogue is
// the 16-byte store path alone for every tile (rows past M clamped, gemm_epi.h)
// SK (stream-K): the tiles x nk K-tiles form ONE iteration space split evenly over the grid
// (logical workgroup order XCD-major, so an XCD's workgroups walk adjacent tiles and share their
// A panels in L2); a range may start and end inside a tile.  Every partial segment of a tile
// stores its fp32 sums to its slot and counts itself in on the tile's counter; the workgroup
// that arrives last adds all slots in segment order (run-to-run deterministic) and runs the
// epilogue -- nobody waits on another workgroup, so concurrent launches on other streams cannot
// deadlock it.  No quantization tail: qkv at 25 104 rows is 891 tiles = 3.48 rounds of 256.
// XS (X stream, EPI_RESID only; N % 256 == 0, K >= 640, no row scales): the fp32 residual tile
// is NOT read in the epilogue.  It is streamed into the accumulators during the tile's K loop:
// in K-tiles [KS, KS + 8) (KS = nk - 9) every phase issues ONE LDS-DMA of a 16 x 16 fp32 X
// fragment (1 KiB per wave: lane = (row r16, 4 columns 4g), exactly the accumulator layout)
// into a per-wave 4-slot ring (32 KiB beside the 128 KiB K ring = the CU's 160 KiB), and the
// same phase of the next K-tile reads it back (ds_read_b128, conflict-free) and adds it into
// the accumulator -- of the quadrant two phases away, so the add never waits on an in-flight
// MFMA.  The stage waits count those DMAs (vm_wait<8 + c>, c = X DMAs of the three previous
// phases).  The epilogue is then 32 plain 16-B stores per lane, left in flight under the next
// tile's first K-tile (vm_wait<8 + 32>): no load -> wait -> store round trips, and the X reads
// overlap the MFMA loop instead of following it.
// SEG (grouped launch): the virtual m-tiles belong to up to MAX_SEG row segments of one A /
// one out buffer, each multiplied by its own W (+ bias) and written through its own row map --
// e.g. the teacher's and the student's calls of one layer as ONE launch (identical shapes,
// different weights), so their tiles share the rounds instead of each call paying a
// partly filled last round.  The stagers and the epilogue look the segment up per tile.
template <int EPI, bool OUT_F32, int ABL = 0, bool NFULL = false, bool SK = false, bool XS = false, bool SEG = false>
__global__ __launch_bounds__(512, 1) void gemm_8ph_kernel(GemmParams p) {
  static_assert(!XS || (EPI == EPI_RESID && !SK && ABL == 0), "X stream: residual epilogue only");
  static_assert(!SEG || (!SK && !XS && ABL == 0), "grouped launch: plain data-parallel kernel only");
  constexpr bool CLAMPED = NFULL && (EPI == EPI_BIAS || EPI == EPI_GELU) && !OUT_F32;
  // VMEM instructions of a full-tile register epilogue: bf16 bias / GELU -> 16 pair stores,
  // X-streamed residual -> 32 fp32 fragment stores
  // rolling-window residual (gemm_epi.h) -> 32 X loads + 32 fp32 stores; the waits can skip at
  // most 63 - 8 of them (a 6-bit vmcnt), so the oldest few still drain before the next K-tile
  constexpr int S_EPI = XS ? 32
                      : ((EPI == EPI_BIAS || CLAMPED) && !OUT_F32 && !(ABL & 64)) ? 16
                      : (EPI == EPI_RESID && ABL == 0 && !SK && DSVT_RESID_PIPE) ? DSVT_RESID_SEPI : 0;
  constexpr int XS_BYTES = XS ? 8 * 4096 : 0;           // 8 waves x 4 slots x 1 KiB
  constexpr int SMEM_BYTES = 2 * P8_BUF + XS_BYTES + (SK ? 16 : 0);
  __shared__ __attribute__((aligned(16))) char smem[SMEM_BYTES];
  int& sk_flag = *reinterpret_cast<int*>(smem + 2 * P8_BUF + XS_BYTES);

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wave >> 2, wc = wave & 3;
  const int r16 = lane & 15, g = lane >> 4;
  const int tilesN = (int)((p.N + 255) >> 8);
  const int tiles = (int)((p.M + 255) >> 8) * tilesN;
  // XCD-contiguous tile ranges (block b runs on XCD b % 8; the grid is a multiple of 8)
  const int G = gridDim.x, b = blockIdx.x, xcd = b & 7, li = b >> 3, per_x = G >> 3;
  const int nk = (int)(p.K >> 6);
  // This workgroup's K-tile stream runs over VIRTUAL tiles tl = 0 .. tl_end-1.  Plain: its
  // strided share of the tiles (XCD-contiguous ranges).  SK: the full rounds of tiles
  // [0, T0 = tiles / G * G) stay data-parallel with that mapping, and the last partial round --
  // the quantization tail -- is one iteration space of (tiles - T0) * nk K-tiles split evenly
  // over the grid; a workgroup streams its tail range FIRST (virtual tiles 0 .. n_tail-1, the
  // first starting at K-tile k0, the last ending at ke) and then its T0 / G whole tiles.
  int t_first, k0 = 0, ke = nk, n_tail = 0, tail_t0 = 0, tl_end, J, wl = 0;
  int64_t I_tail = 1, tail_base = 0;
  if constexpr (SK) {
    wl = xcd * per_x + li;
    const int T0 = tiles / G * G, ndp = T0 / G;
    t_first = xcd * (T0 >> 3) + li;
    I_tail = (int64_t)(tiles - T0) * nk;                 // >= G (host-checked): no empty range
    tail_base = (int64_t)T0 * nk;
    const int64_t a = tail_base + (int64_t)wl * I_tail / G, b = tail_base + (int64_t)(wl + 1) * I_tail / G;
    tail_t0 = (int)(a / nk);
    k0 = (int)(a % nk);
    ke = (int)((b - 1) % nk) + 1;
    n_tail = (int)((b - 1) / nk) - tail_t0 + 1;
    J = (int)(b - a) + ndp * nk;
    tl_end = n_tail + ndp;
  } else {
    const int tpx = (tiles + 7) >> 3;
    t_first = xcd * tpx + li;
    const int t_end = min(tiles, xcd * tpx + tpx);
    if (t_first >= t_end) return;
    tl_end = (t_end - t_first + per_x - 1) / per_x;
    J = tl_end * nk;
  }
  // K-tile range [seg_k0, seg_k1) of virtual tile tl, and the stream advance
  auto seg_k0 = [&](int tl) { return tl == 0 ? k0 : 0; };
  auto seg_k1 = [&](int tl) { return tl == n_tail - 1 ? ke : nk; };
  auto adv = [&](int& tl, int& k) {
    if (++k == seg_k1(tl)) { k = 0; ++tl; }
  };

  const char* A = (const char*)p.A;
  const char* W = (const char*)p.W;
  const int64_t lda_b = p.lda * 2, ldw_b = p.ldw * 2;
  // segment of the tile whose first virtual row is m0 (SEG); plain launches: one segment = p
  struct SegV { const char* W; const float* bias; int64_t vrow0, a_row0, M, rpg, gstride, goff; };
  auto seg_of = [&](int64_t m0) -> SegV {
    if constexpr (SEG) {
      const int64_t mt = m0 >> 8;
      int s = 0;
#pragma unroll
      for (int i = 1; i < GemmParams::MAX_SEG; ++i)
        if (i < p.nseg && mt >= p.seg[i].mtile0) s = i;
      const GemmParams::Seg& q = p.seg[s];
      return SegV{(const char*)q.W, q.bias, q.mtile0 * 256, q.a_row0, q.M, q.rpg, q.gstride, q.goff};
    } else {
      return SegV{(const char*)p.W, p.bias, 0, 0, p.M, p.rpg, p.gstride, p.goff};
    }
  };
  const char* Wa = W;                   // the W of the tile the AT / BL stager is on (SEG)
  const char* Wb = W;                   // ... and of the BR / AB stager's tile

  // ---- LDS-DMA source offsets (32-bit, checked on the host) of the four half-tiles
  const int srow = tid >> 3;                                   // half-tile row within a 64-row piece
  const uint32_t schunk = (uint32_t)(((tid & 7) ^ ((tid >> 4) & 7)) << 4);
  uint32_t oAT[2], oAB[2], oBL[2], oBR[2];
  const int tilesM = (int)((p.M + 255) >> 8), GM = p.tile_group;
  auto tile_mn = [&](int tl, int64_t& m0, int64_t& n0) {
    const int t = tl < n_tail ? tail_t0 + tl : t_first + (tl - n_tail) * per_x;
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
  auto a_off = [&](const SegV& sv, int64_t gr) -> uint32_t {   // gr: virtual row of the tile
    gr -= sv.vrow0;
    gr = gr < sv.M ? gr : sv.M - 1;
    return (uint32_t)((sv.a_row0 + gr) * lda_b) + schunk;
  };
  auto b_off = [&](int64_t gr) -> uint32_t {
    gr = gr < p.N ? gr : p.N - 1;
    return (uint32_t)(gr * ldw_b) + schunk;
  };
  // stager of parts AT / BL (runs two K-tiles ahead of the compute) and of BR / AB (one ahead)
  auto set_atbl = [&](int tl) {
    int64_t m0, n0;
    tile_mn(tl, m0, n0);
    const SegV sv = seg_of(m0);
    if constexpr (SEG) Wa = sv.W;
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      oAT[q] = a_off(sv, m0 + q * 128 + srow);
      oBL[q] = b_off(n0 + (2 * q + (srow >> 5)) * 64 + (srow & 31));
    }
  };
  auto set_brab = [&](int tl) {
    int64_t m0, n0;
    tile_mn(tl, m0, n0);
    const SegV sv = seg_of(m0);
    if constexpr (SEG) Wb = sv.W;
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      oAB[q] = a_off(sv, m0 + q * 128 + 64 + srow);
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
#define P8_RD(DST, H, BASE, CB, N)                                                                     \
  _Pragma("unroll") for (int f_ = 0; f_ < (N); ++f_) {                                                \
    const char* s_ = smem + (CB) + (H) * P8_HALF + (BASE) + f_ * 16 * P8_ROWB;                        \
    DST[f_][0] = *reinterpret_cast<const sv8*>(s_ + cs0);                                             \
    DST[f_][1] = *reinterpret_cast<const sv8*>(s_ + cs1);                                             \
  }
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
// XS: xc = X DMAs issued in the three phases before this one (the DMA of a phase is issued after
// its wait), so the half-tile four phases back -- and the X fragment of that phase -- are done.
#define P8_WAIT(VALID, PH)                                 \
  {                                                        \
    if (!(VALID)) vm_wait<0>();                            \
    else if (S_EPI > 0 && post) vm_wait<8 + S_EPI>();      \
    else if constexpr (XS) {                               \
      const int xc_ = xs_prev(PH);                         \
      if (xc_ == 3) vm_wait<11>();                         \
      else if (xc_ == 2) vm_wait<10>();                    \
      else if (xc_ == 1) vm_wait<9>();                     \
      else vm_wait<8>();                                   \
    } else vm_wait<8>();                                   \
  }
#define P8_COMPUTE(MFMA_STMT, PH)                          \
  {                                                        \
    p8_barrier();                                          \
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");     \
    __builtin_amdgcn_sched_barrier(0);                     \
    if constexpr (XS) {                                    \
      xs_add_rt(std::integral_constant<int, PH>{});        \
      xs_issue_rt(std::integral_constant<int, PH>{});      \
    }                                                      \
    __builtin_amdgcn_sched_barrier(0);                     \
    MFMA_STMT;                                             \
    p8_barrier();                                          \
  }

  // ---- prologue: K-tile 0 complete, K-tile 1 parts AT / BL
  int tl1, k1, tl2, k2;                 // stream positions u1 = j + 1 (BR, AB), u2 = j + 2 (AT, BL)
  bool prologue_ = true;
  set_atbl(0);
  set_brab(0);
  P8_STAGE(H_AT, oAT, A, 0, k0 * P8_ROWB);
  P8_STAGE(H_BL, oBL, Wa, 0, k0 * P8_ROWB);
  P8_STAGE(H_BR, oBR, Wb, 0, k0 * P8_ROWB);
  P8_STAGE(H_AB, oAB, A, 0, k0 * P8_ROWB);
  tl1 = 0; k1 = k0;
  adv(tl1, k1);
  tl2 = tl1; k2 = k1;
  adv(tl2, k2);
  if (J > 1) {
    set_atbl(tl1);
    P8_STAGE(H_AT, oAT, A, P8_BUF, k1 * P8_ROWB);
    P8_STAGE(H_BL, oBL, Wa, P8_BUF, k1 * P8_ROWB);
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
  auto init_acc = [&](int tl, bool with_bias) {   // SK: only a tile's k = 0 segment carries the bias
    float4 b4[4];
    // (EPI_RESID with DropPath row scales: the epilogue adds s[m] * bias instead)
    int64_t bm0 = 0, bn0 = 0;
    tile_mn(tl, bm0, bn0);
    const float* tbias = seg_of(bm0).bias;
    if (BIAS_IN_ACC && tbias && with_bias && !(EPI == EPI_RESID && p.row_scale)) {
      const int64_t cbase = bn0 + wc * 64;
      if (cbase + 64 <= p.N) {
        bias_frag4(tbias, cbase, g, b4);
      } else {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int64_t n = cbase + j * 16 + 4 * g;
          b4[j] = n < p.N ? *reinterpret_cast<const float4*>(tbias + n) : make_float4(0.f, 0.f, 0.f, 0.f);
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
  init_acc(0, k0 == 0);
  prologue_ = false;
  int tlc = 0, kc = k0;                 // compute position
  bool post = false;                    // previous K-tile ended with a full-tile epilogue

  // ---- X stream (XS): see the template comment.  Phase PH adds into the quadrant that phase
  // (PH + 2) % 4 computes: PH 0 -> (4, 2), 1 -> (4, 0), 2 -> (0, 0), 3 -> (0, 2); K-tile kx of
  // the window supplies its fragment (kx >> 1, kx & 1).
  const int KS = nk - 9;
  int64_t xrow0 = 0, xcol0 = 0;         // this wave's 128 x 64 block of the compute tile
  fv4 xv = {0.f, 0.f, 0.f, 0.f};
  char* const xslots = smem + 2 * P8_BUF + wave * 4096;
  auto xs_tile = [&](int tl) {
    int64_t m0, n0;
    tile_mn(tl, m0, n0);
    xrow0 = m0 + wr * 128;
    xcol0 = n0 + wc * 64;
  };
  auto xs_prev = [&](int ph) -> int {   // X DMAs in the three phases before phase ph of K-tile kc
    const int kx = kc - KS;
    return (kx >= 1 && kx <= 7) ? 3 : kx == 0 ? ph : kx == 8 ? 3 - ph : 0;
  };
#define XS_READ(PH)                                                                   \
  if constexpr (XS) {                                                                 \
    const int kx_ = kc - KS;                                                          \
    asm volatile("" ::: "memory");                                                    \
    if (kx_ >= 1 && kx_ <= 8) xv = *reinterpret_cast<const fv4*>(xslots + (PH) * 1024 + lane * 16); \
  }
  // (XI, XJ) of phase PH; the add targets acc[XI + (kk >> 1)][XJ + (kk & 1)]
// (the distinct asm tail keeps SimplifyCFG from sinking the eight adds into one dynamically
// indexed add, which would put acc in scratch)
#define XS_CASE(PH, KK)                                                                            \
  case KK:                                                                                         \
    acc[((PH) < 2 ? 4 : 0) + ((KK) >> 1)][(((PH) == 0 || (PH) == 3) ? 2 : 0) + ((KK) & 1)] += xv;  \
    asm volatile("; xs add " #PH " " #KK);                                                         \
    break;
  auto xs_add_rt = [&](auto ph_c) {
    constexpr int PH = decltype(ph_c)::value;
    const int kx = kc - KS;
    if (kx >= 1 && kx <= 8) {
      switch (kx - 1) { XS_CASE(PH, 0) XS_CASE(PH, 1) XS_CASE(PH, 2) XS_CASE(PH, 3)
                        XS_CASE(PH, 4) XS_CASE(PH, 5) XS_CASE(PH, 6) XS_CASE(PH, 7) }
    }
  };
  auto xs_issue_rt = [&](auto ph_c) {
    constexpr int PH = decltype(ph_c)::value;
    const int kx = kc - KS;
    if (kx >= 0 && kx <= 7) {
      const int fi = (PH < 2 ? 4 : 0) + (kx >> 1), fj = ((PH == 0 || PH == 3) ? 2 : 0) + (kx & 1);
      int64_t m = xrow0 + fi * 16 + r16;
      m = m < p.M ? m : p.M - 1;        // rows past M: row M - 1's X (never stored)
      const int64_t orow = (p.rpg >= p.M && p.goff == 0) ? m : map_row(m, p.rpg, p.gstride, p.goff);
      const float* src = resid_src(p) + orow * p.ldo + xcol0 + fj * 16 + 4 * g;
      __builtin_amdgcn_global_load_lds((const void*)src, LDS_PTR(xslots + PH * 1024), 16, 0, 0);
    }
  };
  if constexpr (XS) xs_tile(0);

  // SK: a partial segment of tail tile t (this workgroup's slot: 0 for its first tail tile, 1
  // for its last).  Returns true in the workgroup that arrives last, with the tile's full sums
  // in acc.  owner(it) = the workgroup whose tail range holds iteration it.
  auto owner = [&](int64_t it) -> int { return (int)(((it - tail_base + 1) * G - 1) / I_tail); };
  auto sk_combine = [&](int t, int slot) -> bool {
    if (!(ABL & 1) && wr == 0) p8_barrier();   // unstagger: the barriers below pair up in place
    // Hand-off without L2 write-back / invalidate fences (MI355X_MICROARCH.md, Valid forms, the
    // first table row): the slot is written by `sc1` (write-through) 16-B stores -- one wave
    // instruction covers 8 whole 128-B lines -- drained by every wave before the workgroup
    // barrier and the counter add; the workgroup whose add returns last reads the slots with
    // `sc1` loads after a barrier.  Inline-asm memory ops are invisible to the compiler's waits:
    // expcnt(0) after each store (its data VGPRs are read out after issue), and every load's
    // result passes through the vmcnt(0) below before use.
    const int64_t lane_off = (int64_t)wave * 32 * 64 + lane;
    fv4* mine = reinterpret_cast<fv4*>(p.sk_part) + (int64_t)(wl * 2 + slot) * 8 * 32 * 64 + lane_off;
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int jj = 0; jj < 4; ++jj)
        asm volatile("global_store_dwordx4 %0, %1, off sc1\n\ts_waitcnt expcnt(0)" ::"v"(mine + (i * 4 + jj) * 64),
                     "v"(acc[i][jj])
                     : "memory");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) sk_flag = __hip_atomic_fetch_add(p.sk_cnt + t, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __syncthreads();
    const int wa = owner((int64_t)t * nk), wb = owner((int64_t)(t + 1) * nk - 1);
    const bool last = sk_flag == wb - wa;            // workgroup-uniform
    if (last) {
      if (tid == 0) __hip_atomic_store(p.sk_cnt + t, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);   // next launch
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) acc[i][jj] = fv4{0.f, 0.f, 0.f, 0.f};
      for (int w = wa; w <= wb; ++w) {             // segment order: deterministic sums
        const int first_t = (int)((tail_base + (int64_t)w * I_tail / G) / nk);
        const fv4* src = reinterpret_cast<const fv4*>(p.sk_part) + (int64_t)(w * 2 + (t == first_t ? 0 : 1)) * 8 * 32 * 64 + lane_off;
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          fv4 v[4];
#pragma unroll
          for (int jj = 0; jj < 4; ++jj)
            asm volatile("global_load_dwordx4 %0, %1, off sc1" : "=v"(v[jj]) : "v"(src + (i * 4 + jj) * 64) : "memory");
          asm volatile("s_waitcnt vmcnt(0)" : "+v"(v[0]), "+v"(v[1]), "+v"(v[2]), "+v"(v[3])::"memory");
#pragma unroll
          for (int jj = 0; jj < 4; ++jj) acc[i][jj] += v[jj];
        }
      }
    }
    if (!(ABL & 1) && wr == 1) p8_barrier();   // re-stagger
    return last;
  };

  for (int j = 0; j < J; ++j) {
    const int cb = (j & 1) * P8_BUF, sb1 = cb ^ P8_BUF, sb2 = cb;
    const bool v1 = j + 1 < J, v2 = j + 2 < J;
    const int kb1 = k1 * P8_ROWB, kb2 = k2 * P8_ROWB;
    // phase 0: read BL + AT, stage BR(j+1), quadrant (AT, BL)
    P8_RD(fbl, H_BL, rdB, cb, 2);
    __builtin_amdgcn_sched_barrier(0);
    P8_RD(fa, H_AT, rdA, cb, 4);
    if (v1) P8_STAGE(H_BR, oBR, Wb, sb1, kb1);
    P8_WAIT(v1, 0);
    XS_READ(0);
    P8_COMPUTE(P8_MFMA(0, 0, fbl), 0);
    // phase 1: read BR, stage AB(j+1), quadrant (AT, BR)
    P8_RD(fbr, H_BR, rdB, cb, 2);
    if (v1) P8_STAGE(H_AB, oAB, A, sb1, kb1);
    P8_WAIT(v1, 1);
    XS_READ(1);
    P8_COMPUTE(P8_MFMA(0, 2, fbr), 1);
    // phase 2: read AB, stage AT(j+2), quadrant (AB, BR)
    P8_RD(fa, H_AB, rdA, cb, 4);
    if (v2) P8_STAGE(H_AT, oAT, A, sb2, kb2);
    P8_WAIT(v2, 2);
    XS_READ(2);
    P8_COMPUTE(P8_MFMA(4, 2, fbr), 2);
    // phase 3: no reads, stage BL(j+2), quadrant (AB, BL)
    if (v2) P8_STAGE(H_BL, oBL, Wa, sb2, kb2);
    P8_WAIT(v2, 3);
    XS_READ(3);
    P8_COMPUTE(P8_MFMA(4, 0, fbl), 3);

    post = false;
    if (++kc == seg_k1(tlc)) {            // tile (or SK tail segment) done: register epilogue
      int64_t m0, n0;
      tile_mn(tlc, m0, n0);
      // SEG: the tile's segment as a plain problem (its M, bias, row map) for the epilogue
      GemmParams pe = p;
      if constexpr (SEG) {
        const SegV sv = seg_of(m0);
        m0 -= sv.vrow0;
        pe.M = sv.M; pe.bias = sv.bias; pe.rpg = sv.rpg; pe.gstride = sv.gstride; pe.goff = sv.goff;
      }
      const int64_t rbase = m0 + wr * 128, cbase = n0 + wc * 64;
      mfma_result_fence();
      bool whole = true;
      if constexpr (SK) {
        if (tlc < n_tail && (seg_k0(tlc) != 0 || kc != nk)) whole = sk_combine(tail_t0 + tlc, tlc == 0 ? 0 : 1);
      }
      if (!whole) {
      } else if constexpr (XS) {          // X already in the accumulators: stores only
        const bool ident = p.rpg >= p.M && p.goff == 0;
        float* const out = (float*)p.out;
        if (rbase + 128 <= p.M) {
#pragma unroll
          for (int i = 0; i < 8; ++i) {
            const int64_t m = rbase + i * 16 + r16;
            float* o = out + (ident ? m : map_row(m, p.rpg, p.gstride, p.goff)) * p.ldo + cbase + 4 * g;
#pragma unroll
            for (int jj = 0; jj < 4; ++jj) *reinterpret_cast<fv4*>(o + jj * 16) = acc[i][jj];
          }
        } else {
#pragma unroll
          for (int i = 0; i < 8; ++i) {
            const int64_t m = rbase + i * 16 + r16;
            if (m >= p.M) continue;
            float* o = out + map_row(m, p.rpg, p.gstride, p.goff) * p.ldo + cbase + 4 * g;
#pragma unroll
            for (int jj = 0; jj < 4; ++jj) *reinterpret_cast<fv4*>(o + jj * 16) = acc[i][jj];
          }
        }
      } else if constexpr ((ABL & 16) != 0) {
#pragma unroll
        for (int i = 0; i < 8; ++i)
#pragma unroll
          for (int jj = 0; jj < 4; ++jj) asm volatile("" ::"v"(acc[i][jj]));
      } else {
        epilogue_direct<8, 4, EPI, OUT_F32, (ABL & 32) ? 1 : (ABL & 128) ? 2 : 0, (ABL & 64) != 0, BIAS_IN_ACC, (EPI == EPI_GELU && DSVT_8PH_GELU_NOFAST), EPI == EPI_GELU_SAVE, NFULL, true>(pe, acc, rbase, cbase,
                                                                                          r16, g);
      }
      post = whole && S_EPI > 0 && (CLAMPED || (rbase + 128 <= pe.M && cbase + 64 <= p.N)) &&
             (EPI != EPI_RESID || XS || !p.row_scale);
      kc = 0;
      ++tlc;
      __builtin_amdgcn_sched_barrier(0);   // keep the next tile's bias loads after the stores
      if (tlc < tl_end) {
        init_acc(tlc, true);
        if constexpr (XS) xs_tile(tlc);
      }
    }
    // advance the stagers
    { const int o = tl1; adv(tl1, k1); if (tl1 != o && tl1 < tl_end) set_brab(tl1); }
    { const int o = tl2; adv(tl2, k2); if (tl2 != o && tl2 < tl_end) set_atbl(tl2); }
  }
  if (!(ABL & 1) && wr == 0) p8_barrier();  // balance the stagger barrier
#undef XS_READ
#undef XS_CASE
#undef P8_STAGE
#undef P8_RD
#undef P8_MFMA
#undef P8_WAIT
#undef P8_COMPUTE
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
  GemmParams q = p;
  if (const char* e = getenv("DSVT_TILE_GROUP")) q.tile_group = atoi(e);
#define DSVT_K(E, F) gemm_8ph_kernel<E, F><<<grid, block, 0, s>>>(q)
  if (abl) {                                          // diagnostic builds: EPI_BIAS, bf16 out
    if (epi != EPI_BIAS || out_f32) return hipErrorInvalidValue;
    switch (abl) {
      case 1: gemm_8ph_kernel<EPI_BIAS, false, 1><<<grid, block, 0, s>>>(q); break;
      case 2: gemm_8ph_kernel<EPI_BIAS, false, 2><<<grid, block, 0, s>>>(q); break;
      case 4: gemm_8ph_kernel<EPI_BIAS, false, 4><<<grid, block, 0, s>>>(q); break;
      case 8: gemm_8ph_kernel<EPI_BIAS, false, 8><<<grid, block, 0, s>>>(q); break;
      case 16: gemm_8ph_kernel<EPI_BIAS, false, 16><<<grid, block, 0, s>>>(q); break;
      case 18: gemm_8ph_kernel<EPI_BIAS, false, 18><<<grid, block, 0, s>>>(q); break;
      case 32: gemm_8ph_kernel<EPI_BIAS, false, 32><<<grid, block, 0, s>>>(q); break;
      case 64: gemm_8ph_kernel<EPI_BIAS, false, 64><<<grid, block, 0, s>>>(q); break;
      default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
  }
  const bool nfull = p.N % 256 == 0 && !out_f32 && !getenv("DSVT_8PH_NO_NFULL");
  static const bool sc1 = [] {
    const char* e = getenv("DSVT_8PH_SC1");
    return e && atoi(e) == 1;
  }();
  if (nfull && sc1 && (epi == EPI_BIAS || epi == EPI_GELU)) {   // sc1 output stores
    if (epi == EPI_BIAS) gemm_8ph_kernel<EPI_BIAS, false, 128, true><<<grid, block, 0, s>>>(q);
    else gemm_8ph_kernel<EPI_GELU, false, 128, true><<<grid, block, 0, s>>>(q);
    return hipGetLastError();
  }
  switch (epi) {
    case EPI_BIAS:
      if (out_f32) DSVT_K(EPI_BIAS, true);
      else if (nfull) gemm_8ph_kernel<EPI_BIAS, false, 0, true><<<grid, block, 0, s>>>(q);
      else DSVT_K(EPI_BIAS, false);
      break;
    case EPI_RESID: DSVT_K(EPI_RESID, true); break;
    case EPI_GELU:
      if (out_f32) DSVT_K(EPI_GELU, true);
      else if (nfull) gemm_8ph_kernel<EPI_GELU, false, 0, true><<<grid, block, 0, s>>>(q);
      else DSVT_K(EPI_GELU, false);
      break;
    case EPI_GELU_SAVE: DSVT_K(EPI_GELU_SAVE, false); break;
    case EPI_DGELU: if (out_f32) DSVT_K(EPI_DGELU, true); else DSVT_K(EPI_DGELU, false); break;
    default: return hipErrorInvalidValue;
  }
#undef DSVT_K
  return hipGetLastError();
}

// ---- grouped launch: segments of rows with their own W / bias / row map (dsvt_gemm_grouped_fwd)
bool gemm_8ph_grouped_ok(const GemmParams& p, int epi, int out_f32) {
  if (p.nseg < 1 || p.nseg > GemmParams::MAX_SEG || !gemm_8ph_ok(p, epi) || p.row_scale || p.resid) return false;
  if (!(epi == EPI_BIAS || epi == EPI_GELU || epi == EPI_RESID)) return false;
  if (epi != EPI_RESID && out_f32) return false;
  int64_t mt = 0;
  for (int i = 0; i < p.nseg; ++i) {
    const GemmParams::Seg& q = p.seg[i];
    if (q.mtile0 != mt || q.M < 1 || !q.W) return false;
    if ((q.a_row0 + q.M - 1) * p.lda * 2 + p.K * 2 > (int64_t)UINT32_MAX) return false;
    if (((const char*)q.W - (const char*)nullptr) % 16) return false;
    mt += (q.M + 255) / 256;
  }
  return mt * 256 == p.M;
}

hipError_t launch_gemm_8ph_grouped(const GemmParams& p, int epi, int out_f32, hipStream_t s) {
  if (!gemm_8ph_grouped_ok(p, epi, out_f32)) return hipErrorInvalidValue;
  const int64_t tiles = (p.M / 256) * ((p.N + 255) / 256);
  int64_t G = 256;
  const int64_t per_x = (tiles + 7) / 8;
  if (per_x * 8 < G) G = per_x * 8;
  const bool nfull = p.N % 256 == 0;
  dim3 grid((unsigned)G), block(512);
  switch (epi) {
    case EPI_BIAS:
      if (nfull) gemm_8ph_kernel<EPI_BIAS, false, 0, true, false, false, true><<<grid, block, 0, s>>>(p);
      else gemm_8ph_kernel<EPI_BIAS, false, 0, false, false, false, true><<<grid, block, 0, s>>>(p);
      break;
    case EPI_GELU:
      if (nfull) gemm_8ph_kernel<EPI_GELU, false, 0, true, false, false, true><<<grid, block, 0, s>>>(p);
      else gemm_8ph_kernel<EPI_GELU, false, 0, false, false, false, true><<<grid, block, 0, s>>>(p);
      break;
    case EPI_RESID: gemm_8ph_kernel<EPI_RESID, true, 0, false, false, false, true><<<grid, block, 0, s>>>(p); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

// ---- X-streamed residual GEMM (variant 33): EPI_RESID, whole 256-column tiles, K-window of 8
// K-tiles after at least one more (nk >= 10), no DropPath row scales
bool gemm_8ph_xs_ok(const GemmParams& p, int epi) {
  return epi == EPI_RESID && gemm_8ph_ok(p, epi) && p.N % 256 == 0 && p.K / 64 >= 10 && !p.row_scale;
}

hipError_t launch_gemm_8ph_xs(const GemmParams& p, int epi, hipStream_t s) {
  if (!gemm_8ph_xs_ok(p, epi)) return hipErrorInvalidValue;
  const int64_t tiles = ((p.M + 255) / 256) * ((p.N + 255) / 256);
  int64_t G = 256;
  const int64_t per_x = (tiles + 7) / 8;
  if (per_x * 8 < G) G = per_x * 8;
  GemmParams q = p;
  if (const char* e = getenv("DSVT_TILE_GROUP")) q.tile_group = atoi(e);
  gemm_8ph_kernel<EPI_RESID, true, 0, false, false, true><<<dim3((unsigned)G), dim3(512), 0, s>>>(q);
  return hipGetLastError();
}

}  // namespace dsvt

namespace dsvt {

// ---- stream-K launch (variant 40): the kernel above with SK = true.  p.sk_part / p.sk_cnt point
// into the caller's workspace (gemm_sk_workspace_bytes; counters zero on entry, left zero).
bool gemm_sk_ok(const GemmParams& p, int epi, int out_f32) {
  if (!gemm_8ph_ok(p, epi)) return false;
  const int64_t tiles = ((p.M + 255) / 256) * ((p.N + 255) / 256);
  // a quantization tail to split, at least one tail K-tile per workgroup
  if (tiles > SK_MAX_TILES || tiles % 256 == 0 || (tiles % 256) * (p.K / 64) < 256) return false;
  if (epi == EPI_RESID) return true;                   // fp32 token rows whatever out_f32 says
  return (epi == EPI_BIAS || epi == EPI_GELU) && !out_f32 && p.N % 256 == 0;
}

hipError_t launch_gemm_sk(const GemmParams& p, int epi, int out_f32, hipStream_t s) {
  if (!gemm_sk_ok(p, epi, out_f32) || !p.sk_part || !p.sk_cnt) return hipErrorInvalidValue;
  dim3 grid(256), block(512);
  switch (epi) {
    case EPI_BIAS: gemm_8ph_kernel<EPI_BIAS, false, 0, true, true><<<grid, block, 0, s>>>(p); break;
    case EPI_GELU: gemm_8ph_kernel<EPI_GELU, false, 0, true, true><<<grid, block, 0, s>>>(p); break;
    case EPI_RESID: gemm_8ph_kernel<EPI_RESID, true, 0, false, true><<<grid, block, 0, s>>>(p); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

}  // namespace dsvt
