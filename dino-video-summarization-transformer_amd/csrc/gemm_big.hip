// Persistent 256x128 bf16 MFMA GEMM (variant 10: the training epilogues and the backward's dX
// GEMMs) and the K-split skinny GEMM (variant 50: the few-row GEMMs).
//
// Persistent kernel geometry: BM x BN output tile per workgroup (WM x WN waves), wave tile 128x64
// = MI x NJ MFMA 16x16x32 tiles, two workgroups per CU.  K advances 32 bf16 (64-byte rows) per
// stage; an NST-stage LDS ring keeps NST - 2 stages in flight behind the one being computed
// (global_load_lds_dwordx4 straight into LDS, counted `s_waitcnt vmcnt(N)` and one raw s_barrier
// per stage).  The LDS image is linear per 1 KB LDS-DMA piece (16 rows x 64 B); the swizzle
// chunk' = chunk ^ H[(row>>2)&3], H = {0,2,3,1}, is applied to the SOURCE address and to the
// ds_read_b128 address, which makes all four 16-lane groups of a fragment read bank-conflict free.
#include <stdlib.h>

#include <type_traits>

#include "gemm_epi.h"

namespace dsvt {

constexpr int BIG_ROWB = 64;   // bytes per tile row per stage (32 bf16)

__device__ __forceinline__ int swz64(int r) { return (0x78 >> (2 * ((r >> 2) & 3))) & 3; }

// s_waitcnt vmcnt(n) leaving lgkmcnt / expcnt untouched (gfx9 encoding: vmcnt[3:0] at bits 3:0,
// vmcnt[5:4] at bits 15:14; n < 64)
template <int N>
__device__ __forceinline__ void wait_vm() {
  static_assert(N >= 0 && N < 64, "vmcnt immediate");
  __builtin_amdgcn_s_waitcnt(0x0F70 | (N & 15) | ((N >> 4) << 14));
}

// s_waitcnt vmcnt(min(k, K) * PS) for a wave-uniform runtime k >= 0 (one immediate per depth)
template <int PS, int K>
__device__ __forceinline__ void wait_stages(int k) {
  static_assert(K * PS < 64, "vmcnt immediate");
  if constexpr (K == 0) {
    wait_vm<0>();
  } else {
    if (k >= K) { wait_vm<K * PS>(); return; }
    wait_stages<PS, K - 1>(k);
  }
}

// ---------------------------------------------------------------------------------------------
// Persistent variant: grid = 2 workgroups per CU; each walks tiles with a stride of the grid.
// Before storing tile t it issues the first stages of tile t+1 into the (free) LDS ring, so
// the loads fly under the store tail; STAGGER delays the second-resident half of the grid by
// ~half a tile so the two workgroups of a CU alternate MFMA loop and store tail.
// STATS (EPI_RESID, 64-column wave tiles): the residual epilogue that also writes the updated
// rows' bf16 copy and LayerNorm partials (dsvt_gemm_resid_stats_fwd; gemm_epi.h resid_stats_rows)
template <int BM, int BN, int WM, int WN, int NST, int EPI, bool OUT_F32, bool STAGGER, bool STATS = false>
__global__ __launch_bounds__(64 * WM * WN, 2) void gemm_persist_kernel(GemmParams p) {
  constexpr int NW = WM * WN;
  constexpr int A_BYTES = BM * BIG_ROWB, B_BYTES = BN * BIG_ROWB, ST_BYTES = A_BYTES + B_BYTES;
  constexpr int WTM = BM / WM, WTN = BN / WN, MI = WTM / 16, NJ = WTN / 16;
  constexpr int A_PIECES = A_BYTES / 1024 / NW, B_PIECES = B_BYTES / 1024 / NW;
  constexpr int PER_STAGE = A_PIECES + B_PIECES;
  static_assert(NST >= 3 && NST <= 16 && (NST - 2) * PER_STAGE < 64, "ring depth");
  __shared__ __attribute__((aligned(16))) char smem[NST * ST_BYTES];

  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / WN, wn = wave % WN;
  const int r16 = lane & 15, g = lane >> 4;
  const int tilesN = (int)((p.N + BN - 1) / BN);
  const int tiles = (int)((p.M + BM - 1) / BM) * tilesN;
  // XCD-contiguous tile ranges: block b runs on XCD b % 8 (round-robin dispatch, speed only)
  const int G = gridDim.x, b = blockIdx.x, xcd = b & 7, li = b >> 3, per_x = G >> 3;
  const int tpx = (tiles + 7) / 8;                       // tiles per XCD range
  const int t_begin = xcd * tpx, t_end = min(tiles, t_begin + tpx);
  const char* A = (const char*)p.A;
  const char* W = (const char*)p.W;
  const int64_t lda_b = p.lda * 2, ldw_b = p.ldw * 2;
  const int nk = (int)(p.K / 32);
  const int prow = lane >> 2, pch = lane & 3;
  const int frag_off = r16 * BIG_ROWB + ((g ^ swz64(r16)) << 4);
  const int a_base = wm * WTM * BIG_ROWB + frag_off;
  const int b_base = A_BYTES + wn * WTN * BIG_ROWB + frag_off;

  if (STAGGER && li >= per_x / 2) {                      // ~half a tile of delay for one resident half
    const int naps = nk / 2;
    for (int i = 0; i < naps; ++i) __builtin_amdgcn_s_sleep(8);
  }

  int64_t a_off[A_PIECES], b_off[B_PIECES];
  const int tilesM = (int)((p.M + BM - 1) / BM), GM = p.tile_group;
  auto set_tile = [&](int t, int64_t& m0, int64_t& n0) {
    if (GM <= 0) {
      m0 = (int64_t)(t / tilesN) * BM;
      n0 = (int64_t)(t % tilesN) * BN;
    } else {                            // groups of GM m-tile rows, n-column-major inside
      const int grp = t / (GM * tilesN), w = t - grp * GM * tilesN;
      const int fm = grp * GM, gm = min(GM, tilesM - fm);
      m0 = (int64_t)(fm + w % gm) * BM;
      n0 = (int64_t)(w / gm) * BN;
    }
#pragma unroll
    for (int i = 0; i < A_PIECES; ++i) {
      const int r = (wave * A_PIECES + i) * 16 + prow;
      int64_t gr = m0 + r;
      gr = gr < p.M ? gr : p.M - 1;
      a_off[i] = gr * lda_b + ((pch ^ swz64(r)) << 4);
    }
#pragma unroll
    for (int i = 0; i < B_PIECES; ++i) {
      const int r = (wave * B_PIECES + i) * 16 + prow;
      int64_t gr = n0 + r;
      gr = gr < p.N ? gr : p.N - 1;
      b_off[i] = gr * ldw_b + ((pch ^ swz64(r)) << 4);
    }
  };
#define DSVT_PISSUE(kt)                                                                            \
  {                                                                                                \
    char* st_ = smem + ((kt) % NST) * ST_BYTES;                                                    \
    const int64_t kb_ = (int64_t)(kt) * BIG_ROWB;                                                  \
    _Pragma("unroll") for (int i = 0; i < A_PIECES; ++i)                                           \
        __builtin_amdgcn_global_load_lds((const void*)(A + a_off[i] + kb_),                        \
                                         LDS_PTR(st_ + (wave * A_PIECES + i) * 1024), 16, 0, 0);   \
    _Pragma("unroll") for (int i = 0; i < B_PIECES; ++i)                                           \
        __builtin_amdgcn_global_load_lds((const void*)(W + b_off[i] + kb_),                        \
                                         LDS_PTR(st_ + A_BYTES + (wave * B_PIECES + i) * 1024),    \
                                         16, 0, 0);                                                \
  }

#define DSVT_PROLOGUE()                                       \
  {                                                          \
    _Pragma("unroll") for (int s_ = 0; s_ < NST - 1; ++s_)   \
      if (s_ < nk) DSVT_PISSUE(s_);                          \
  }
  int t = t_begin + li;
  if (t >= t_end) return;
  int64_t m0, n0;
  set_tile(t, m0, n0);
  DSVT_PROLOGUE();
  for (;;) {
    fv4 acc[MI][NJ];
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int j = 0; j < NJ; ++j) acc[i][j] = fv4{0.f, 0.f, 0.f, 0.f};
    sv8 fa[MI], fb[NJ];
    for (int kt = 0; kt < nk; ++kt) {
      const int ahead = nk - 1 - kt < NST - 2 ? nk - 1 - kt : NST - 2;
      wait_stages<PER_STAGE, NST - 2>(ahead);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      if (kt + NST - 1 < nk) DSVT_PISSUE(kt + NST - 1);
      const char* st_ = smem + (kt % NST) * ST_BYTES;
#pragma unroll
      for (int i = 0; i < MI; ++i) fa[i] = *reinterpret_cast<const sv8*>(st_ + a_base + i * 16 * BIG_ROWB);
#pragma unroll
      for (int j = 0; j < NJ; ++j) fb[j] = *reinterpret_cast<const sv8*>(st_ + b_base + j * 16 * BIG_ROWB);
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[j], fa[i], acc[i][j], 0, 0, 0);
    }
    // prefetch the next tile's first two stages under this tile's store tail
    const int64_t cm0 = m0, cn0 = n0;
    const int tn = t + per_x;
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();                         // all waves done reading the ring
    asm volatile("" ::: "memory");
    if (tn < t_end) {
      set_tile(tn, m0, n0);
      DSVT_PROLOGUE();
    }
    // ---- direct epilogue of tile (cm0, cn0)
    mfma_result_fence();
    if constexpr (STATS) {
      static_assert(EPI == EPI_RESID && NJ == 4, "the stats epilogue: residual, 64-column wave slabs");
      float4 b4[4];
      bias_frag4(p.bias, cn0 + wn * WTN, g, b4);           // N % BN == 0: every column valid
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
          acc[i][j][0] += b4[j].x; acc[i][j][1] += b4[j].y; acc[i][j][2] += b4[j].z; acc[i][j][3] += b4[j].w;
        }
#ifndef DSVT_PERSIST_STATS_W
#define DSVT_PERSIST_STATS_W 2   // rows of X in flight (3 spills)
#endif
      epilogue_resid_stats<MI, NJ, DSVT_PERSIST_STATS_W>(p, acc, cm0 + wm * WTM, cn0 + wn * WTN, r16, g);
    } else {
      epilogue_direct<MI, NJ, EPI, OUT_F32, false, false, false, false, true, false, false, true>(
          p, acc, cm0 + wm * WTM, cn0 + wn * WTN, r16, g);
    }
    if (tn >= t_end) break;
    t = tn;
  }
#undef DSVT_PISSUE
#undef DSVT_PROLOGUE
}

template <int BM, int BN, int WM, int WN, bool STAGGER, int NST = 3>
static hipError_t launch_persist_t(const GemmParams& p, int epi, int out_f32, hipStream_t s) {
  const int64_t tiles = ((p.M + BM - 1) / BM) * ((p.N + BN - 1) / BN);
  const int64_t lds = (int64_t)NST * (BM + BN) * BIG_ROWB;
  // resident workgroups: 1 or 2 per CU, up to 4 for the small-tile instantiations (LDS <= 40 KB)
  int64_t G = lds > 80 * 1024 ? 256 : lds > 40 * 1024 ? 512 : 1024;
  const int64_t per_x = (tiles + 7) / 8;
  if (per_x * 8 < G) G = per_x * 8;
  dim3 grid((unsigned)G), block(64 * WM * WN);
  GemmParams q = p;
  if (const char* e = getenv("DSVT_TILE_GROUP")) q.tile_group = atoi(e);
#define DSVT_K(E, F) gemm_persist_kernel<BM, BN, WM, WN, NST, E, F, STAGGER><<<grid, block, 0, s>>>(q)
  if (p.stats_out) {
    if constexpr (BN / WN == 64) {     // the stats epilogue: 64-column wave slabs
      if (epi != EPI_RESID || p.N % BN || p.row_scale || !p.xb_out) return hipErrorInvalidValue;
      gemm_persist_kernel<BM, BN, WM, WN, NST, EPI_RESID, true, STAGGER, true><<<grid, block, 0, s>>>(q);
      return hipGetLastError();
    }
    return hipErrorInvalidValue;
  }
  switch (epi) {
    case EPI_BIAS: if (out_f32) DSVT_K(EPI_BIAS, true); else DSVT_K(EPI_BIAS, false); break;
    case EPI_GELU: if (out_f32) DSVT_K(EPI_GELU, true); else DSVT_K(EPI_GELU, false); break;
    case EPI_RESID: DSVT_K(EPI_RESID, true); break;
    case EPI_PATCH: DSVT_K(EPI_PATCH, true); break;
    case EPI_GELU_SAVE: DSVT_K(EPI_GELU_SAVE, false); break;
    case EPI_DGELU: if (out_f32) DSVT_K(EPI_DGELU, true); else DSVT_K(EPI_DGELU, false); break;
    default: return hipErrorInvalidValue;
  }
#undef DSVT_K
  return hipGetLastError();
}

// variant 10 = the persistent staggered 256x128 kernel (2 WGs per CU); 20 = gemm_8ph.hip (21-29:
// its diagnostic ablation builds, tools/gemm_bench.py); 30 = gemm_192.hip
hipError_t launch_gemm_big(const GemmParams& p, int variant, int epi, int out_f32, hipStream_t s) {
  switch (variant) {
    case 10: return launch_persist_t<256, 128, 2, 2, true>(p, epi, out_f32, s);
    // small tiles for the small GEMMs (Video Swin stages 3-4: M = 784 / 3136 rows, 42-300 tiles of
    // 128x128 leave most CUs idle): 128x64 and 64x64, 5-stage rings
    case 11: return launch_persist_t<128, 64, 2, 2, false, 5>(p, epi, out_f32, s);
    case 12: return launch_persist_t<64, 64, 2, 2, false, 5>(p, epi, out_f32, s);
    // ... with deep rings (more bytes in flight per workgroup: a small grid has ~1 per CU)
    case 13: return launch_persist_t<64, 64, 2, 2, false, 10>(p, epi, out_f32, s);
    case 14: return launch_persist_t<128, 64, 2, 2, false, 6>(p, epi, out_f32, s);
    case 15: return launch_persist_t<64, 64, 2, 2, false, 14>(p, epi, out_f32, s);
    case 20: return launch_gemm_8ph(p, epi, out_f32, s);
    case 21: return launch_gemm_8ph(p, epi, out_f32, s, 1);
    case 22: return launch_gemm_8ph(p, epi, out_f32, s, 2);
    case 23: return launch_gemm_8ph(p, epi, out_f32, s, 4);
    case 25: return launch_gemm_8ph(p, epi, out_f32, s, 8);
    case 26: return launch_gemm_8ph(p, epi, out_f32, s, 16);
    case 27: return launch_gemm_8ph(p, epi, out_f32, s, 18);
    case 28: return launch_gemm_8ph(p, epi, out_f32, s, 32);
    case 29: return launch_gemm_8ph(p, epi, out_f32, s, 64);
    case 30: return launch_gemm_192(p, epi, out_f32, s);
    // 40 = gemm_4w.hip (41, 42, 44-46: its diagnostic ablation builds)
    case 40: return launch_gemm_4w(p, epi, out_f32, s);
    case 41: return launch_gemm_4w(p, epi, out_f32, s, 2);
    case 42: return launch_gemm_4w(p, epi, out_f32, s, 4);
    case 44: return launch_gemm_4w(p, epi, out_f32, s, 16);
    case 45: return launch_gemm_4w(p, epi, out_f32, s, 18);
    case 46: return launch_gemm_4w(p, epi, out_f32, s, 26);
    default: return hipErrorInvalidValue;
  }
}


// ---- skinny GEMM (variant 50): a few rows -- the CLS-only last block's Q / proj / fc1 / fc2 over
// the B clips' CLS rows and the DINO head's layers.  The 128x128 kernel runs these as N / 128
// workgroups that each walk all of K (6-24 busy CUs, 20-50 us per launch).  Here one 512-thread
// workgroup owns 32 output columns of a 64-row block and its 8 waves split K eight ways:
// N / 32 x ceil(M / 64) workgroups, each streaming its 32 rows of W once.  A row's result does
// not depend on M (the same K-split sums for every row), so a batch split over streams stays
// bitwise equal to the whole batch as long as the CALL SITE picks this kernel whatever M is
// (dsvt_set_gemm_skinny scopes, not an M threshold).  Operands go from HBM / L2
// straight to registers (16-B loads in the MFMA fragment layout; the few A rows are shared by
// every workgroup), the waves' partial sums are added in a fixed order through LDS (run-to-run
// deterministic), and wave 0 runs the register epilogue of the other kernels (bias, GELU, fp32
// residual through the output row map).  Rows past M are clamped on load and never stored.
constexpr int SKN_NW = 8, SKN_U = 4;
template <int EPI, bool OUT_F32>
__global__ __launch_bounds__(512, 1) void gemm_skinny_kernel(GemmParams p) {
  __shared__ fv4 red[SKN_NW - 1][4][2][64];   // waves 1..7: [m fragment][n fragment][lane], 56 KiB
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r16 = lane & 15, g = lane >> 4;
  const int64_t n0 = (int64_t)blockIdx.x * 32, r0 = (int64_t)blockIdx.y * 64;
  const int64_t kw = p.K / SKN_NW, k0 = wave * kw;
  const int ns = (int)(kw / 32);
  const bf16_t* ar[4];
  const bf16_t* wr[2];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int64_t m = r0 + i * 16 + r16;
    ar[i] = (const bf16_t*)p.A + (m < p.M ? m : p.M - 1) * p.lda + k0 + g * 8;
  }
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int64_t n = n0 + j * 16 + r16;
    wr[j] = (const bf16_t*)p.W + (n < p.N ? n : p.N - 1) * p.ldw + k0 + g * 8;
  }
  fv4 acc[4][2];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = fv4{0.f, 0.f, 0.f, 0.f};
  for (int s0 = 0; s0 < ns; s0 += SKN_U) {     // SKN_U k-steps of loads in flight, then their MFMAs
    sv8 a[SKN_U][4], b[SKN_U][2];
#pragma unroll
    for (int u = 0; u < SKN_U; ++u) {
      if (s0 + u < ns) {
#pragma unroll
        for (int j = 0; j < 2; ++j) b[u][j] = *reinterpret_cast<const sv8*>(wr[j] + (s0 + u) * 32);
#pragma unroll
        for (int i = 0; i < 4; ++i) a[u][i] = *reinterpret_cast<const sv8*>(ar[i] + (s0 + u) * 32);
      }
    }
#pragma unroll
    for (int u = 0; u < SKN_U; ++u) {
      if (s0 + u < ns) {
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b[u][j], a[u][i], acc[i][j], 0, 0, 0);
      }
    }
  }
  mfma_result_fence();
  if (wave > 0) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) red[wave - 1][i][j][lane] = acc[i][j];
  }
  __syncthreads();
  if (wave != 0) return;
#pragma unroll 1
  for (int w = 0; w < SKN_NW - 1; ++w)      // (not unrolled: all 56 partial fragments at once spill)
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) acc[i][j] += red[w][i][j][lane];
  epilogue_direct<4, 2, EPI, OUT_F32>(p, acc, r0, n0, r16, g);
}

bool gemm_skinny_ok(const GemmParams& p, int epi) {
  return p.M >= 1 && p.K >= 512 && p.K % (SKN_NW * 32) == 0 && p.N % 32 == 0 && p.lda % 8 == 0 && p.ldw % 8 == 0 &&
         (epi == EPI_BIAS || epi == EPI_GELU || epi == EPI_RESID) && !p.row_scale &&
         ((uintptr_t)p.A & 15) == 0 && ((uintptr_t)p.W & 15) == 0;
}

hipError_t launch_gemm_skinny(const GemmParams& p, int epi, int out_f32, hipStream_t s) {
  if (!gemm_skinny_ok(p, epi)) return hipErrorInvalidValue;
  const dim3 grid((unsigned)(p.N / 32), (unsigned)((p.M + 63) / 64)), block(512);
  switch (epi) {
    case EPI_BIAS:
      if (out_f32) gemm_skinny_kernel<EPI_BIAS, true><<<grid, block, 0, s>>>(p);
      else gemm_skinny_kernel<EPI_BIAS, false><<<grid, block, 0, s>>>(p);
      break;
    case EPI_GELU:
      if (out_f32) gemm_skinny_kernel<EPI_GELU, true><<<grid, block, 0, s>>>(p);
      else gemm_skinny_kernel<EPI_GELU, false><<<grid, block, 0, s>>>(p);
      break;
    case EPI_RESID: gemm_skinny_kernel<EPI_RESID, true><<<grid, block, 0, s>>>(p); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

}  // namespace dsvt
