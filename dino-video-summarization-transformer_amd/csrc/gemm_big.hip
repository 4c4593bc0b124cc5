// Large-tile bf16 MFMA GEMM for the big hot-path projections (M = tokens of a whole
// backbone call: 13.9k-25.1k rows; N = 768 / 2304 / 3072; K = 768 / 3072).
//
// Geometry: BM x BN output tile per 512-thread workgroup (8 waves as WM x WN), wave tile
// 128x64 (256x256) or 64x64 (256x128) = MI x NJ MFMA 16x16x32 tiles.  K advances 32 bf16
// (64-byte rows) per stage; a 4-stage LDS ring keeps THREE stages in flight behind the one
// being computed (global_load_lds_dwordx4 straight into LDS, counted `s_waitcnt vmcnt(N)`
// and one raw s_barrier per stage -- no vmcnt(0) drain in the loop).  The LDS image is
// linear per 1 KB LDS-DMA piece (16 rows x 64 B); the swizzle chunk' = chunk ^ H[(row>>2)&3],
// H = {0,2,3,1}, is applied to the SOURCE address and to the ds_read_b128 address, which makes
// all four 16-lane groups of a fragment read bank-conflict free.
#include <stdlib.h>

#include <type_traits>

#include "gemm_epi.h"

namespace dsvt {

constexpr int BIG_ROWB = 64;   // bytes per tile row per stage (32 bf16)

__device__ __forceinline__ int swz64(int r) { return (0x78 >> (2 * ((r >> 2) & 3))) & 3; }

// s_waitcnt vmcnt(n) leaving lgkmcnt / expcnt untouched (gfx9 encoding; n < 16)
template <int N>
__device__ __forceinline__ void wait_vm() {
  static_assert(N >= 0 && N < 16, "vmcnt immediate");
  __builtin_amdgcn_s_waitcnt(0x0F70 | N);
}

// s_waitcnt vmcnt(k * PS) for a runtime k in [0, 3] (instantiates only encodable immediates)
template <int PS>
__device__ __forceinline__ void wait_stages(int k) {
  if constexpr (3 * PS < 16) { if (k >= 3) { wait_vm<3 * PS>(); return; } }
  if constexpr (2 * PS < 16) { if (k >= 2) { wait_vm<2 * PS>(); return; } }
  if (k >= 1) { wait_vm<PS>(); return; }
  wait_vm<0>();
}

// ABL (diagnostic ablation builds, benchmarking only): 0 = normal, 1 = no MFMA (LDS reads
// kept live), 2 = no global loads after the prologue (MFMA + LDS reads on stale tiles).
template <int BM, int BN, int WM, int WN, int NST, bool STAGED, int EPI, bool OUT_F32, int ABL = 0, bool DB = true>
__global__ __launch_bounds__(64 * WM * WN, 2) void gemm_big_kernel(GemmParams p) {
  constexpr int NW = WM * WN;
  constexpr int A_BYTES = BM * BIG_ROWB, B_BYTES = BN * BIG_ROWB, ST_BYTES = A_BYTES + B_BYTES;
  constexpr int WTM = BM / WM, WTN = BN / WN, MI = WTM / 16, NJ = WTN / 16;
  constexpr int A_PIECES = A_BYTES / 1024 / NW, B_PIECES = B_BYTES / 1024 / NW;  // per wave per stage
  constexpr int PER_STAGE = A_PIECES + B_PIECES;
  static_assert(A_PIECES * NW * 1024 == A_BYTES && B_PIECES * NW * 1024 == B_BYTES, "piece split");
  static_assert((NST - 2) * PER_STAGE < 16, "vmcnt range");
  __shared__ __attribute__((aligned(16))) char smem[NST * ST_BYTES];

  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / WN, wn = wave % WN;
  const int r16 = lane & 15, g = lane >> 4;

  const int tilesN = (int)((p.N + BN - 1) / BN);
  const int nwg = gridDim.x, orig = blockIdx.x, xcd = orig & 7, q = nwg >> 3, rr = nwg & 7;
  const int wg = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + (orig >> 3);
  const int64_t m0 = (int64_t)(wg / tilesN) * BM;
  const int64_t n0 = (int64_t)(wg % tilesN) * BN;

  const char* A = (const char*)p.A;
  const char* W = (const char*)p.W;
  const int64_t lda_b = p.lda * 2, ldw_b = p.ldw * 2;
  const int nk = (int)(p.K / 32);

  // per-lane source rows / chunks of this wave's LDS-DMA pieces (fixed over the K loop)
  const int prow = lane >> 2, pch = lane & 3;
  int64_t a_off[A_PIECES], b_off[B_PIECES];
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

#define DSVT_ISSUE(kt)                                                                            \
  {                                                                                               \
    char* st_ = smem + ((kt) % NST) * ST_BYTES;                                                   \
    const int64_t kb_ = (int64_t)(kt) * BIG_ROWB;                                                 \
    _Pragma("unroll") for (int i = 0; i < A_PIECES; ++i)                                          \
        __builtin_amdgcn_global_load_lds((const void*)(A + a_off[i] + kb_),                       \
                                         LDS_PTR(st_ + (wave * A_PIECES + i) * 1024), 16, 0, 0);  \
    _Pragma("unroll") for (int i = 0; i < B_PIECES; ++i)                                          \
        __builtin_amdgcn_global_load_lds((const void*)(W + b_off[i] + kb_),                       \
                                         LDS_PTR(st_ + A_BYTES + (wave * B_PIECES + i) * 1024),   \
                                         16, 0, 0);                                               \
  }

  fv4 acc[MI][NJ];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j) acc[i][j] = fv4{0.f, 0.f, 0.f, 0.f};

  // fragment read offsets: row = base + r16, physical chunk = g ^ swz64(r16)
  // (declared before use by the pipeline macros below)
  const int frag_off = r16 * BIG_ROWB + ((g ^ swz64(r16)) << 4);
  const int a_base = wm * WTM * BIG_ROWB + frag_off;
  const int b_base = A_BYTES + wn * WTN * BIG_ROWB + frag_off;

  // Fragment double buffering: the ds_reads of stage kt+1 are in flight under the 32 MFMAs
  // of stage kt (whose fragments were read one iteration earlier).
#define DSVT_READ(FA, FB, kt)                                                                         \
  {                                                                                                   \
    const char* st_ = smem + ((kt) % NST) * ST_BYTES;                                                 \
    _Pragma("unroll") for (int i = 0; i < MI; ++i)                                                    \
        FA[i] = *reinterpret_cast<const sv8*>(st_ + a_base + i * 16 * BIG_ROWB);                      \
    _Pragma("unroll") for (int j = 0; j < NJ; ++j)                                                    \
        FB[j] = *reinterpret_cast<const sv8*>(st_ + b_base + j * 16 * BIG_ROWB);                      \
  }
#define DSVT_MMA(FA, FB)                                                                              \
  {                                                                                                   \
    if constexpr (ABL == 1) {                                                                         \
      _Pragma("unroll") for (int i = 0; i < MI; ++i) asm volatile("" ::"v"(FA[i]));                   \
      _Pragma("unroll") for (int j = 0; j < NJ; ++j) asm volatile("" ::"v"(FB[j]));                   \
    } else {                                                                                          \
      _Pragma("unroll") for (int i = 0; i < MI; ++i)                                                  \
          _Pragma("unroll") for (int j = 0; j < NJ; ++j)                                              \
              acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(FB[j], FA[i], acc[i][j], 0, 0, 0); \
    }                                                                                                 \
  }
  // one pipeline step: stage kt computed from (CA, CB), stage kt+1 read into (NA, NB)
#define DSVT_STEP(kt, CA, CB, NA, NB)                                                                 \
  {                                                                                                   \
    if ((kt) + 1 < nk) {                                                                              \
      const int ahead_ = nk - 2 - (kt) < NST - 2 ? nk - 2 - (kt) : NST - 2;                           \
      wait_stages<PER_STAGE>(ahead_);                                                                 \
    }                                                                                                 \
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");                                               \
    __builtin_amdgcn_s_barrier();                                                                     \
    asm volatile("" ::: "memory");                                                                    \
    if (ABL != 2 && (kt) + NST < nk) DSVT_ISSUE((kt) + NST);                                          \
    if ((kt) + 1 < nk) DSVT_READ(NA, NB, (kt) + 1);                                                   \
    DSVT_MMA(CA, CB);                                                                                 \
  }

  if constexpr (DB) {
    sv8 fa0[MI], fb0[NJ], fa1[MI], fb1[NJ];
    static_assert(NST == 3 || NST == 4, "ring depth");
    DSVT_ISSUE(0);
    if (nk > 1) DSVT_ISSUE(1);
    if (nk > 2) DSVT_ISSUE(2);
    if (NST == 4 && nk > 3) DSVT_ISSUE(3);
    wait_stages<PER_STAGE>((nk < NST ? nk : NST) - 1);   // stage 0 landed; the rest may fly
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    DSVT_READ(fa0, fb0, 0);
    int kt = 0;
    for (; kt + 1 < nk; kt += 2) {
      DSVT_STEP(kt, fa0, fb0, fa1, fb1);
      DSVT_STEP(kt + 1, fa1, fb1, fa0, fb0);
    }
    if (kt < nk) DSVT_STEP(kt, fa0, fb0, fa1, fb1);

  } else {
    // single fragment set: wait(stage kt) -> barrier -> issue kt+NST-1 -> read kt -> MMA kt
    sv8 fa[MI], fb[NJ];
    DSVT_ISSUE(0);
    if (nk > 1) DSVT_ISSUE(1);
    if (NST == 4 && nk > 2) DSVT_ISSUE(2);
    for (int kt = 0; kt < nk; ++kt) {
      // issued so far: stages <= kt + NST - 2; stage kt must land, the later ones may fly
      const int ahead = nk - 1 - kt < NST - 2 ? nk - 1 - kt : NST - 2;
      wait_stages<PER_STAGE>(ahead);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      if (ABL != 2 && kt + NST - 1 < nk) DSVT_ISSUE(kt + NST - 1);
      DSVT_READ(fa, fb, kt);
      DSVT_MMA(fa, fb);
    }
  }
#undef DSVT_STEP
#undef DSVT_MMA
#undef DSVT_READ
#undef DSVT_ISSUE

  mfma_result_fence();   // acc is read under the branches below
  // ---- epilogue.  Lane holds C[m = .. + r16][n = .. + 4g + 0..3] per (i, j) subtile.
  // Bias / GELU are applied on the way to LDS; the tile is staged through LDS in row chunks
  // (padded rows: conflict-free 8-/16-B writes), then written back as WHOLE rows with 16 B
  // per lane (full 128-B lines; the row map / residual / patch-embed adds are per row).
  if constexpr (ABL == 3) {
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int j = 0; j < NJ; ++j) asm volatile("" ::"v"(acc[i][j]));
    return;
  }
  using OutT = typename std::conditional<(EPI == EPI_RESID || EPI == EPI_PATCH || OUT_F32), float, bf16_t>::type;
  if constexpr (!STAGED) {
    epilogue_direct<MI, NJ, EPI, OUT_F32>(p, acc, m0 + wm * WTM, n0 + wn * WTN, r16, g);
    return;
  }
  // Wave-local staging: each wave transposes its own WTM x WTN sub-tile through a private LDS
  // slice (chunk' = chunk ^ ((row>>1)&7): conflict-free 8-/16-B writes), then stores whole
  // 128-B lines, 16 B per lane -- 8 full lines per store instruction instead of 16 partial ones.
  constexpr int ES = (int)sizeof(OutT);
  constexpr int RB = WTN * ES;                           // bytes per sub-tile row (128 or 256)
  constexpr int CPR = RB / 16;                           // 16-B chunks per row
  constexpr int SLICE0 = (NST * ST_BYTES / NW) < 16384 ? (NST * ST_BYTES / NW) : 16384;
  constexpr int SROWS0 = (SLICE0 / RB) / 16 * 16 < WTM ? (SLICE0 / RB) / 16 * 16 : WTM;
  constexpr int SROWS = (WTM % SROWS0 == 0) ? SROWS0 : 16;  // rows staged per pass
  constexpr int SLICE = SROWS * RB;
  static_assert(SROWS >= 16 && NW * SLICE <= NST * ST_BYTES, "wave slices fit the ring");
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();                          // the ring is no longer read by anyone
  asm volatile("" ::: "memory");
  char* wslice = smem + wave * SLICE;
#pragma unroll
  for (int ps = 0; ps < WTM / SROWS; ++ps) {
    // (1) this wave's rows [ps*SROWS, (ps+1)*SROWS) -> LDS (bias / GELU applied)
#pragma unroll
    for (int i = ps * (SROWS / 16); i < (ps + 1) * (SROWS / 16); ++i) {
      const int R = (i - ps * (SROWS / 16)) * 16 + r16;
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        const int col = j * 16 + 4 * g;                  // column inside the sub-tile
        float v0 = acc[i][j][0], v1 = acc[i][j][1], v2 = acc[i][j][2], v3 = acc[i][j][3];
        const int64_t n = n0 + wn * WTN + col;
        if (p.bias && n < p.N) {
          const float4 bb = *reinterpret_cast<const float4*>(p.bias + n);
          v0 += bb.x; v1 += bb.y; v2 += bb.z; v3 += bb.w;
        }
        if constexpr (EPI == EPI_GELU) {
          constexpr bool BO = std::is_same<OutT, bf16_t>::value;
          v0 = gelu_out<BO>(v0); v1 = gelu_out<BO>(v1); v2 = gelu_out<BO>(v2); v3 = gelu_out<BO>(v3);
        }
        const int byte = col * ES;
        const int chunk = (byte >> 4) ^ ((R >> 1) & 7 & (CPR - 1));
        store4(reinterpret_cast<OutT*>(wslice + R * RB + (chunk << 4) + (byte & 15)), v0, v1, v2, v3);
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    // (2) read back whole rows and store 16 B per lane
    constexpr int RPI = 64 / CPR;                        // rows per wave instruction
#pragma unroll
    for (int rr = 0; rr < SROWS; rr += RPI) {
      const int R = rr + lane / CPR, c = lane % CPR;
      const uint4 v = *reinterpret_cast<const uint4*>(wslice + R * RB + ((c ^ ((R >> 1) & 7 & (CPR - 1))) << 4));
      const int64_t m = m0 + wm * WTM + ps * SROWS + R;
      const int64_t n = n0 + wn * WTN + c * (16 / ES);
      if (m >= p.M || n >= p.N) continue;
      const int64_t orow = map_row(m, p.rpg, p.gstride, p.goff);
      if constexpr (EPI == EPI_BIAS || EPI == EPI_GELU) {
        *reinterpret_cast<uint4*>(reinterpret_cast<OutT*>(p.out) + orow * p.ldo + n) = v;
      } else if constexpr (EPI == EPI_RESID) {
        float4* xo = reinterpret_cast<float4*>(reinterpret_cast<float*>(p.out) + orow * p.ldo + n);
        float4 x = *reinterpret_cast<const float4*>(resid_src(p) + orow * p.ldo + n);
        x.x += __uint_as_float(v.x); x.y += __uint_as_float(v.y);
        x.z += __uint_as_float(v.z); x.w += __uint_as_float(v.w);
        *xo = x;
      } else {  // EPI_PATCH
        const int64_t rrw = m % p.rpg;
        const int64_t np = rrw / p.T, t = rrw % p.T;
        const float4 pe = *reinterpret_cast<const float4*>(p.pos + (1 + (int64_t)p.pidx[np]) * p.N + n);
        float4 o = make_float4(__uint_as_float(v.x) + pe.x, __uint_as_float(v.y) + pe.y,
                               __uint_as_float(v.z) + pe.z, __uint_as_float(v.w) + pe.w);
        if (p.temb) {
          const float4 te = *reinterpret_cast<const float4*>(p.temb + (int64_t)p.tidx[t] * p.N + n);
          o.x += te.x; o.y += te.y; o.z += te.z; o.w += te.w;
        }
        *reinterpret_cast<float4*>(reinterpret_cast<float*>(p.out) + orow * p.ldo + n) = o;
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // slice reads done before the next pass
  }
}

// ---------------------------------------------------------------------------------------------
// Persistent variant: grid = 2 workgroups per CU; each walks tiles with a stride of the grid.
// Before storing tile t it issues the first stages of tile t+1 into the (free) LDS ring, so
// the loads fly under the store tail; STAGGER delays the second-resident half of the grid by
// ~half a tile so the two workgroups of a CU alternate MFMA loop and store tail.
template <int BM, int BN, int WM, int WN, int NST, int EPI, bool OUT_F32, bool STAGGER>
__global__ __launch_bounds__(64 * WM * WN, 2) void gemm_persist_kernel(GemmParams p) {
  constexpr int NW = WM * WN;
  constexpr int A_BYTES = BM * BIG_ROWB, B_BYTES = BN * BIG_ROWB, ST_BYTES = A_BYTES + B_BYTES;
  constexpr int WTM = BM / WM, WTN = BN / WN, MI = WTM / 16, NJ = WTN / 16;
  constexpr int A_PIECES = A_BYTES / 1024 / NW, B_PIECES = B_BYTES / 1024 / NW;
  constexpr int PER_STAGE = A_PIECES + B_PIECES;
  static_assert(NST >= 3 && NST <= 5 && (NST - 2) * PER_STAGE < 16, "ring depth");
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
      wait_stages<PER_STAGE>(ahead);
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
    epilogue_direct<MI, NJ, EPI, OUT_F32, false, false, false, false, true>(p, acc, cm0 + wm * WTM, cn0 + wn * WTN,
                                                                          r16, g);
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
  int64_t G = lds > 80 * 1024 ? 256 : 512;           // resident workgroups: 1 or 2 per CU
  const int64_t per_x = (tiles + 7) / 8;
  if (per_x * 8 < G) G = per_x * 8;
  dim3 grid((unsigned)G), block(64 * WM * WN);
  GemmParams q = p;
  if (const char* e = getenv("DSVT_TILE_GROUP")) q.tile_group = atoi(e);
#define DSVT_K(E, F) gemm_persist_kernel<BM, BN, WM, WN, NST, E, F, STAGGER><<<grid, block, 0, s>>>(q)
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

template <int BM, int BN, int WM, int WN, int NST, bool STAGED, bool DB>
static hipError_t launch_big_t(const GemmParams& p, int epi, int out_f32, hipStream_t s) {
  const int64_t tiles = ((p.M + BM - 1) / BM) * ((p.N + BN - 1) / BN);
  dim3 grid((unsigned)tiles), block(64 * WM * WN);
#define DSVT_K(E, F) gemm_big_kernel<BM, BN, WM, WN, NST, STAGED, E, F, 0, DB><<<grid, block, 0, s>>>(p)
  switch (epi) {
    case EPI_BIAS: if (out_f32) DSVT_K(EPI_BIAS, true); else DSVT_K(EPI_BIAS, false); break;
    case EPI_GELU: if (out_f32) DSVT_K(EPI_GELU, true); else DSVT_K(EPI_GELU, false); break;
    case EPI_RESID: DSVT_K(EPI_RESID, true); break;
    case EPI_PATCH: DSVT_K(EPI_PATCH, true); break;
    default: return hipErrorInvalidValue;
  }
#undef DSVT_K
  return hipGetLastError();
}

// variant: 3 = 256x128 / 8 waves / 4 stages (fragment double-buffered);
// 4 = 256x128 / 4 waves (wave tile 128x64) / 3 stages = 72 KB LDS -> 2 WGs per CU, the
// epilogue of one overlaps the MFMA loop of the other; 5 = 128x256 / 4 waves / 3 stages.
hipError_t launch_gemm_big(const GemmParams& p, int variant, int epi, int out_f32, hipStream_t s) {
  switch (variant) {
    case 3: return launch_big_t<256, 128, 4, 2, 4, true, true>(p, epi, out_f32, s);
    case 4: return launch_big_t<256, 128, 2, 2, 3, false, false>(p, epi, out_f32, s);
    case 5: return launch_big_t<128, 256, 1, 4, 3, false, false>(p, epi, out_f32, s);
    case 6: return launch_big_t<256, 128, 2, 2, 3, true, false>(p, epi, out_f32, s);
    case 9: return launch_persist_t<256, 128, 2, 2, false>(p, epi, out_f32, s);
    case 10: return launch_persist_t<256, 128, 2, 2, true>(p, epi, out_f32, s);
    case 11: return launch_persist_t<128, 256, 1, 4, true>(p, epi, out_f32, s);
    case 12: return launch_persist_t<256, 256, 2, 4, false, 5>(p, epi, out_f32, s);
    case 13: return launch_persist_t<256, 256, 2, 4, false, 4>(p, epi, out_f32, s);
    case 20: return launch_gemm_8ph(p, epi, out_f32, s);
    case 21: return launch_gemm_8ph(p, epi, out_f32, s, 1);
    case 22: return launch_gemm_8ph(p, epi, out_f32, s, 2);
    case 23: return launch_gemm_8ph(p, epi, out_f32, s, 4);
    case 25: return launch_gemm_8ph(p, epi, out_f32, s, 8);
    case 26: return launch_gemm_8ph(p, epi, out_f32, s, 16);
    case 27: return launch_gemm_8ph(p, epi, out_f32, s, 18);
    case 28: return launch_gemm_8ph(p, epi, out_f32, s, 32);
    case 29: return launch_gemm_8ph(p, epi, out_f32, s, 64);
    case 33: return launch_gemm_8ph_xs(p, epi, s);
    default: break;
  }
  // ablation builds (EPI_BIAS, bf16 out only) of variant 4: 14 no-MFMA, 24 no-load, 34 no-epilogue
  dim3 grid((unsigned)(((p.M + 255) / 256) * ((p.N + 127) / 128))), block(256);
  switch (variant) {
    case 14: gemm_big_kernel<256, 128, 2, 2, 3, false, EPI_BIAS, false, 1, false><<<grid, block, 0, s>>>(p); break;
    case 24: gemm_big_kernel<256, 128, 2, 2, 3, false, EPI_BIAS, false, 2, false><<<grid, block, 0, s>>>(p); break;
    case 34: gemm_big_kernel<256, 128, 2, 2, 3, false, EPI_BIAS, false, 3, false><<<grid, block, 0, s>>>(p); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
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
         (epi == EPI_BIAS || epi == EPI_GELU || epi == EPI_RESID) && !p.row_scale && !p.nseg && !p.sk_part &&
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
