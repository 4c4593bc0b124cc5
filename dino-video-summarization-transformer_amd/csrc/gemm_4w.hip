// 256x256 bf16 MFMA GEMM with FOUR waves of 128x128 (variant 40): the wide hot-path projections
// (qkv N = 2304, fc1 N = 3072, the LayerNorm-folded forms of both) over M = 13.9k-25.1k tokens.
//
// Why a second 256x256 kernel.  The 8-wave gemm_8ph kernel (wave tile 128x64) reads 12 KiB of
// MFMA fragments from LDS per 524k FLOP and passes two barriers per 16-MFMA phase; with the loads
// and the epilogue compiled out its K loop still ran at only 0.54 of the bf16 peak
// (profiles/r05_gemm8ph_ablation.txt).  Here each wave owns a 128x128 output block: 64 fp32
// 16x16 accumulators = 256 registers, which at one wave per SIMD live in the AGPR half of the
// 512-entry register file, so the wave reads 16 KiB of fragments per 1M FLOP (64 FLOP / LDS
// byte instead of 44) and the four waves meet at ONE barrier per 32-deep K step.
//
// K loop.  The K dimension is staged in 32-deep STAGES (A 256 x 32 + W 256 x 32 bf16 = 32 KiB,
// 64-byte LDS rows) through a ring of W4_NBUF stage buffers filled by LDS-DMA
// (global_load_lds_dwordx4, 8 per wave per stage).  Step b computes stage b from registers:
//   boundary b:  s_waitcnt vmcnt(8 (NBUF - 2) [+ S])   this wave's DMA of stage b + 1 landed
//                s_waitcnt lgkmcnt(0)                   stage b's fragments are in registers
//                s_barrier                              ... for every wave
//   step b:      64 MFMA 16x16x32 on stage b's fragments, and interleaved between them
//                16 ds_read_b128 of stage b + 1's fragments (the other register set) and
//                8 LDS-DMA of stage b + NBUF into the buffer stage b just vacated.
// So every MFMA operand was read one step ahead, the DMA runs NBUF - 1 steps ahead, and the
// only wait on the MFMA path is the per-step barrier.  Two fragment register sets (2 x 64
// VGPRs) alternate, so the loop body is two steps; tiles have an even number of stages (K % 64
// == 0) and every tile starts on set 0.  Past the WG's last stage the stager keeps re-issuing
// its last stage (L2-hot) into the free buffers, so the vmcnt counts stay exact without
// branches; the tail drains with vmcnt(0) before the WG exits.
//
// LDS image: stage u in buffer u % NBUF, [A rows 0..255][64 B] then [W rows 0..255][64 B]; the
// 16-byte chunk c of row r sits at position c ^ swz((r >> 2) & 3), swz = {0, 2, 3, 1}, so each
// of ds_read_b128's four 16-lane groups ({0-3,12-15,20-27}, ...) covers the 16 slots of a 256-B
// bank row exactly once (rows r16 = lane & 15, chunk g = lane >> 4).  The DMA writes linearly
// (lane l -> row l >> 2, slot l & 3), so the permutation is applied to its SOURCE chunk.
//
// Epilogue (after a tile's last step, accumulators -> HBM) is the shared register epilogue of
// gemm_epi.h applied to the two 128 x 64 halves of the wave block.  Its stores sit on vmcnt
// between older and younger DMA stages: the bf16 store-only epilogue (CLAMPED) counts them into
// the next NBUF - 1 boundary waits exactly; epilogues that LOAD (LayerNorm statistics, the fp32
// residual) have already waited for every older stage, so those boundaries need no wait.
#include <utility>

#include "gemm_epi.h"

namespace dsvt {

namespace {

constexpr int W4_ROWB = 64;                 // bytes per LDS row: 32 bf16 of K
constexpr int W4_PART = 256 * W4_ROWB;      // one operand's stage image, 16 KiB
constexpr int W4_STAGE = 2 * W4_PART;       // A + W, 32 KiB
#ifndef DSVT_4W_NBUF
#define DSVT_4W_NBUF 4
#endif
constexpr int W4_NBUF = DSVT_4W_NBUF;       // stage buffers (4: 128 KiB, 5: 160 KiB)
static_assert(W4_NBUF >= 3 && W4_NBUF <= 5, "ring depth");
constexpr int W4_VM = 8 * (W4_NBUF - 2);    // DMA ops younger than the awaited stage

template <int N>
__device__ __forceinline__ void w4_vm_wait() {
  static_assert(N >= 0 && N < 64, "vmcnt immediate");
  __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | 0x0F70);
}

__device__ __forceinline__ void w4_barrier() {
  __builtin_amdgcn_sched_barrier(0);
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
}

// fragment read: inline asm so the compiler does not order it against the LDS-DMA (it would
// drain every in-flight stage with vmcnt(0) before a tracked LDS read); the boundary's counted
// vmcnt + barrier order it after the DMA it reads, w4_tie orders its use
template <int OFF>
__device__ __forceinline__ sv8 w4_rd(unsigned a) {
  sv8 r;
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(r) : "v"(a), "i"(OFF));
  return r;
}
__device__ __forceinline__ unsigned w4_lds(const char* p) {
  return (unsigned)(uintptr_t)(__attribute__((address_space(3))) const char*)p;
}
__device__ __forceinline__ void w4_tie(sv8 (&a)[8], sv8 (&b)[8]) {
  asm volatile("s_waitcnt lgkmcnt(0)"
               : "+v"(a[0]), "+v"(a[1]), "+v"(a[2]), "+v"(a[3]), "+v"(a[4]), "+v"(a[5]), "+v"(a[6]), "+v"(a[7]));
  asm volatile("" : "+v"(b[0]), "+v"(b[1]), "+v"(b[2]), "+v"(b[3]), "+v"(b[4]), "+v"(b[5]), "+v"(b[6]), "+v"(b[7]));
}
// acc += A . B with the accumulator pinned to AGPRs ("+a"): with the builtin the register
// allocator spread the 256 accumulator registers over both files and copied them through
// v_accvgpr_write before every MFMA.  As asm the MFMA is opaque to the hazard recognizer: the
// epilogue reads the accumulators only after mfma_result_fence(), and no MFMA of a step reads
// another's D.  w4_mfma0 starts a tile: C = 0 (inline constant).
__device__ __forceinline__ void w4_mfma(fv4& c, const sv8& a, const sv8& b) {
  asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(c) : "v"(a), "v"(b));
}
__device__ __forceinline__ void w4_mfma0(fv4& c, const sv8& a, const sv8& b) {
  asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, 0" : "=a"(c) : "v"(a), "v"(b));
}
// untracked global loads (inline asm): the compiler's own wait for a tracked load issued after
// LDS-DMA is vmcnt(0) -- it does not count the DMA in order with loads -- which drains every stage
// in flight; these are waited for by a counted w4_vm_wait at their use instead
typedef float f2v_t __attribute__((ext_vector_type(2)));
__device__ __forceinline__ f2v_t w4_gld2(const void* a) {
  f2v_t r;
  asm volatile("global_load_dwordx2 %0, %1, off" : "=v"(r) : "v"(a));
  return r;
}
__device__ __forceinline__ fv4 w4_gld4(const void* a) {
  fv4 r;
  asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(r) : "v"(a));
  return r;
}
// chunk position of row-quad q (rows 4q .. 4q+3 of a 16-row block): swz = {0, 2, 3, 1}
__device__ __forceinline__ int w4_swz(int q) { return (0x78 >> (2 * q)) & 3; }

template <typename F, int... Is>
__device__ __forceinline__ void w4_for_impl(F&& f, std::integer_sequence<int, Is...>) {
  (f(std::integral_constant<int, Is>{}), ...);
}
template <int N, typename F>
__device__ __forceinline__ void w4_for(F&& f) {
  w4_for_impl(f, std::make_integer_sequence<int, N>{});
}

}  // namespace

// ABL (diagnostic builds, tools/gemm_bench.py; 0 = normal): bit 1 no DMA after the prologue
// (stale stages), bit 2 no MFMA (fragments kept live), bit 3 no fragment reads after the
// prologue (stale registers), bit 4 no epilogue (accumulators kept live)
// NFULL: N % 256 == 0, bias / GELU with a bf16 output -- the 16-byte store path alone (rows past M
// clamped, gemm_epi.h); FUSE 1: LayerNorm folded in (dsvt_gemm_lnx_fwd); FUSE 2: residual + the
// next LayerNorm's inputs (dsvt_gemm_resid_stats_fwd)
template <int EPI, bool OUT_F32, int ABL = 0, bool NFULL = false, int FUSE = 0>
__global__ __launch_bounds__(256, 1) void gemm_4w_kernel(GemmParams p) {
  constexpr bool CLAMPED = NFULL && (EPI == EPI_BIAS || EPI == EPI_GELU) && !OUT_F32;
  // post-epilogue boundary waits: 0 = the 32 store instructions of the CLAMPED path counted in,
  // 1 = the epilogue loaded (and so waited for every older stage): no wait, 2 = conservative
  // (FUSE 1: its statistics / wsum / bias loads are prefetched in the tile's last step and consumed
  // before the epilogue's stores, so it is mode 0 too)
  // (plain EPI_RESID: 2 -- a wave whose 128 rows all lie past M loads nothing, so nothing of its
  // epilogue drains the stages in flight)
  constexpr int POST = ((FUSE == 0 || FUSE == 1) && CLAMPED) ? 0 : FUSE == 2 ? 1 : 2;
  constexpr int S_EPI = 32;
  // the bias comes in by the last step's prefetch (untracked loads, one counted wait) wherever the
  // wave's 128 columns are inside N: the scalar-load path (bias_frag4) serialized ~32 scalar
  // cache round trips per epilogue (30 of 101 us at the qkv shape)
  constexpr bool PRE_BIAS = CLAMPED || FUSE == 2;
  __shared__ __attribute__((aligned(16))) char smem[W4_NBUF * W4_STAGE];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wave >> 1, wc = wave & 1;
  const int r16 = lane & 15, g = lane >> 4;
  const int tilesN = (int)((p.N + 255) >> 8);
  const int tiles = (int)((p.M + 255) >> 8) * tilesN;
  // XCD-contiguous tile ranges (block b runs on XCD b % 8; the grid is a multiple of 8)
  const int G = gridDim.x, b = blockIdx.x, xcd = b & 7, li = b >> 3, per_x = G >> 3;
  const int nk = (int)(p.K >> 5);        // stages per tile (even)
  const int tpx = (tiles + 7) >> 3;
  const int t_first = xcd * tpx + li;
  const int t_end = min(tiles, xcd * tpx + tpx);
  if (t_first >= t_end) return;
  const int tl_end = (t_end - t_first + per_x - 1) / per_x;
  const int J = tl_end * nk;              // stages of this workgroup (even)

  const char* A = (const char*)p.A;
  const char* W = (const char*)p.W;
  const int64_t lda_b = p.lda * 2, ldw_b = p.ldw * 2;
  auto tile_mn = [&](int tl, int64_t& m0, int64_t& n0) {
    const int t = t_first + tl * per_x;
    m0 = (int64_t)(t / tilesN) * 256;
    n0 = (int64_t)(t % tilesN) * 256;
  };

  // ---- LDS-DMA sources: this wave's 4 A pieces and 4 W pieces (16 rows x 64 B each) of a stage
  const int prow = wave * 64 + (lane >> 2);   // + q * 16
  const uint32_t schunk = (uint32_t)(((lane & 3) ^ w4_swz((lane >> 4) & 3)) << 4);
  uint32_t oA[4], oB[4];
  auto set_src = [&](int tl) {
    int64_t m0, n0;
    tile_mn(tl, m0, n0);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      int64_t ga = m0 + prow + q * 16;
      ga = ga < p.M ? ga : p.M - 1;
      if constexpr (FUSE == 1) {           // the A row map (32-bit: rows < 2^31, host-checked)
        const uint32_t m = (uint32_t)ga, rpg = (uint32_t)(p.a_rpg < p.M ? p.a_rpg : p.M);
        ga = (int64_t)((m / rpg) * (uint32_t)p.a_gstride + (uint32_t)p.a_goff + m % rpg);
      }
      oA[q] = (uint32_t)(ga * lda_b) + schunk;
      int64_t gb = n0 + prow + q * 16;
      gb = gb < p.N ? gb : p.N - 1;
      oB[q] = (uint32_t)(gb * ldw_b) + schunk;
    }
  };
  int tl_s = 0, k_s = 0;                  // the stage the stager issues next
  auto stage = [&](int buf, int q) {      // DMA piece q (0-3: A, 4-7: W) of the stager's stage
    char* d = smem + buf * W4_STAGE + (q >> 2) * W4_PART + (wave * 64 + (q & 3) * 16) * W4_ROWB;
    const uint32_t o = ((q < 4) ? oA[q & 3] : oB[q & 3]) + (uint32_t)(k_s * W4_ROWB);
    __builtin_amdgcn_global_load_lds((const void*)(((q < 4) ? A : W) + o), LDS_PTR(d), 16, 0, 0);
  };
  auto adv_stager = [&]() {               // past the last stage: keep re-issuing it (L2-hot)
    if (k_s + 1 < nk) {
      ++k_s;
    } else if (tl_s + 1 < tl_end) {
      k_s = 0;
      set_src(++tl_s);
    }
  };

  // ---- fragment read addresses (stage buffer 0); fragment i: + i * 16 rows
  const uint32_t chunk = (uint32_t)((g ^ w4_swz((r16 >> 2) & 3)) << 4);
  const uint32_t rdA = w4_lds(smem) + (uint32_t)((wr * 128 + r16) * W4_ROWB) + chunk;
  const uint32_t rdB = w4_lds(smem) + (uint32_t)(W4_PART + (wc * 128 + r16) * W4_ROWB) + chunk;

  sv8 fa0[8], fb0[8], fa1[8], fb1[8];
  // acc[h][i][j]: rows i*16 + (lane & 15), columns h*64 + j*16 + 4g .. +3 of the wave block
  fv4 acc[2][8][4];
  // the first MFMA of a tile takes C = 0 (no accumulator initialisation: every accumulator is
  // defined and updated by AGPR-constrained asm only); the bias is added in the epilogue
  // read stage buffer `buf`'s fragments into (FA, FB)
  auto read_frag = [&](auto rc, sv8 (&FA)[8], sv8 (&FB)[8], uint32_t ba, uint32_t bb) {
    constexpr int r = decltype(rc)::value;         // 0-7: W fragment r, 8-15: A fragment r - 8
    if constexpr (r < 8) FB[r] = w4_rd<r * 16 * W4_ROWB>(bb);
    else FA[r - 8] = w4_rd<(r - 8) * 16 * W4_ROWB>(ba);
  };

  // ---- prologue: stages 0 .. NBUF-1 in flight, stage 0's fragments in set 0
  set_src(0);
  for (int u = 0; u < W4_NBUF; ++u) {
#pragma unroll
    for (int q = 0; q < 8; ++q) stage(u, q);
    adv_stager();
  }
  w4_vm_wait<8 * (W4_NBUF - 1)>();
  w4_barrier();
  w4_for<16>([&](auto rc) { read_frag(rc, fa0, fb0, rdA, rdB); });

  int post = 0;                          // boundaries left that follow an epilogue's stores

  // FUSE 1: the epilogue's loads (the rows' 3 LN partials per lane group, wsum and the folded bias
  // of the wave's columns), issued at the start of the tile's last step -- BEFORE that step's DMA
  // -- so waiting for them drains no stage the DMA issued since (an epilogue load after them
  // drained all NBUF - 1 stages in flight, like every load in the 256x256 kernel's epilogue)
  f2v_t pst[8][3];
  fv4 pws[2][4], pbf[2][4];
  auto prefetch = [&](int64_t rbase, int64_t cbase) {
    int le;
    asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(le));
    const int ge = le >> 4;
    if constexpr (FUSE != 1 && PRE_BIAS) {   // the bias of the wave's 128 columns (N % 256 == 0).
      // No branch around the loads (a join would let the compiler copy a pending register): without
      // a bias they read W's first N floats (valid memory: N * K bf16 >= N floats) and the epilogue
      // selects zeros
      const float* bsrc = p.bias ? p.bias : (const float*)p.W;
#pragma unroll
      for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int j = 0; j < 4; ++j) pbf[h][j] = w4_gld4(bsrc + cbase + h * 64 + j * 16 + 4 * ge);
    }
    if constexpr (FUSE == 1) {
      const int r16e = le & 15;
      const uint32_t a_rpg = (uint32_t)(p.a_rpg < p.M ? p.a_rpg : p.M), a_gs = (uint32_t)p.a_gstride;
      const uint32_t a_go = (uint32_t)p.a_goff, mlast = (uint32_t)(p.M - 1);
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        uint32_t m = (uint32_t)(rbase + i * 16 + r16e);
        m = m < mlast ? m : mlast;
        const uint32_t xr = (m / a_rpg) * a_gs + a_go + m % a_rpg;   // rows < 2^31 (host-checked)
        const float2* sp = reinterpret_cast<const float2*>(p.ln_stats) + (uint64_t)(xr * LN_PARTS + 3 * ge);
#pragma unroll
        for (int k = 0; k < 3; ++k) pst[i][k] = w4_gld2(sp + k);
      }
#pragma unroll
      for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int64_t n = cbase + h * 64 + j * 16 + 4 * ge;
          pws[h][j] = w4_gld4(p.ln_wsum + n);
          pbf[h][j] = w4_gld4(p.bias + n);
        }
    }
  };

  // one step: boundary, then 64 MFMAs on (FA, FB) with stage u + 1's reads into (NA, NB) and
  // stage u + NBUF's DMA into stage u's buffer interleaved
  auto step = [&](auto first, auto rd, int u, sv8 (&FA)[8], sv8 (&FB)[8], sv8 (&NA)[8], sv8 (&NB)[8],
                  int64_t pre_r = -1, int64_t pre_c = 0) {
    if (POST == 0 && post > 0) {
      --post;
      w4_vm_wait<W4_VM + S_EPI>();
    } else if (POST == 1 && post > 0) {
      --post;                            // the epilogue's loads waited for every older stage
    } else {
      w4_vm_wait<W4_VM>();
    }
    w4_tie(FA, FB);
    w4_barrier();
    // the tile's last step: the epilogue's loads (never in a build without the epilogue: an
    // untracked load must be waited for before its registers can be reused -- the ABL 16 build
    // that prefetched into dead registers faulted on the GPU)
    if constexpr (!decltype(rd)::value && (ABL & 16) == 0) {
      prefetch(pre_r, pre_c);
      __builtin_amdgcn_sched_barrier(0);
    }
    const int nbuf = (u + 1) % W4_NBUF, dbuf = u % W4_NBUF;
    const uint32_t na = rdA + (uint32_t)(nbuf * W4_STAGE), nb = rdB + (uint32_t)(nbuf * W4_STAGE);
    w4_for<64>([&](auto nc) {
      constexpr int n = decltype(nc)::value;
      constexpr int i = n >> 3, j = n & 7;
      if constexpr ((ABL & 4) != 0) {
        asm volatile("" ::"v"(FA[i]), "v"(FB[j]));
      } else {
        if constexpr (decltype(first)::value) w4_mfma0(acc[j >> 2][i][j & 3], FB[j], FA[i]);
        else w4_mfma(acc[j >> 2][i][j & 3], FB[j], FA[i]);
      }
      if constexpr (n % 3 == 0 && n / 3 < 16 && (ABL & 8) == 0 && decltype(rd)::value) {
        read_frag(std::integral_constant<int, n / 3>{}, NA, NB, na, nb);
      }
      if constexpr (n % 8 == 4 && (ABL & 2) == 0) stage(dbuf, n >> 3);
      __builtin_amdgcn_sched_barrier(0);
    });
    if constexpr ((ABL & 2) == 0) adv_stager();
  };

  int u = 0;
  for (int tlc = 0; tlc < tl_end; ++tlc) {   // tile loop; the K-stage stream runs on across tiles
    using T_ = std::true_type;
    using F_ = std::false_type;
    step(T_{}, T_{}, u, fa0, fb0, fa1, fb1);
    step(F_{}, T_{}, u + 1, fa1, fb1, fa0, fb0);
    u += 2;
    for (int kc = 2; kc < nk - 2; kc += 2, u += 2) {
      step(F_{}, T_{}, u, fa0, fb0, fa1, fb1);
      step(F_{}, T_{}, u + 1, fa1, fb1, fa0, fb0);
    }
    // the tile's last step leaves the next stage's fragments to after the epilogue (the
    // epilogue gets the 128 fragment registers)
    int64_t m0, n0;
    tile_mn(tlc, m0, n0);
    step(F_{}, T_{}, u, fa0, fb0, fa1, fb1);
    step(F_{}, F_{}, u + 1, fa1, fb1, fa0, fb0, m0 + wr * 128, n0 + wc * 128);
    u += 2;
    // tile done: register epilogue.  Its lane constants come from an opaque copy of the lane id,
    // so the compiler cannot hoist their (row-map, address) arithmetic out of the tile loop and
    // keep it live through the K loop -- that spilled.
    int lane_e;
    asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(lane_e));
    const int r16 = lane_e & 15, g = lane_e >> 4;
    const int64_t rbase = m0 + wr * 128, cbase = n0 + wc * 128;
    mfma_result_fence();
    if constexpr ((ABL & 16) != 0) {
#pragma unroll
      for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int i = 0; i < 8; ++i)
#pragma unroll
          for (int jj = 0; jj < 4; ++jj) asm volatile("" ::"a"(acc[h][i][jj]));
    } else {
      // the bias is not in the accumulators (every tile starts from C = 0): added a row at a time
      // as the rows are formed (one row's accumulators live in VGPRs at a time)
      auto bias_of = [&](int64_t cb, float4 (&b4)[4]) {
        // N % 256 == 0 (CLAMPED): always the scalar-load path.  A vector load on a path not taken
        // left pending at the join made the compiler drain vmcnt(0) -- every in-flight DMA stage --
        // in each epilogue half (33 of 102 us at the qkv shape)
        if (CLAMPED || cb + 64 <= p.N) {
          bias_frag4(p.bias, cb, g, b4);
        } else {
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const int64_t n = cb + j * 16 + 4 * g;
            b4[j] = (p.bias && n < p.N) ? *reinterpret_cast<const float4*>(p.bias + n) : make_float4(0.f, 0.f, 0.f, 0.f);
          }
        }
      };
      if constexpr (FUSE != 1 && PRE_BIAS) {   // the prefetched bias: only the last step's 8 DMA ops came after it
        asm volatile("s_waitcnt vmcnt(%8)"
                     : "+v"(pbf[0][0]), "+v"(pbf[0][1]), "+v"(pbf[0][2]), "+v"(pbf[0][3]), "+v"(pbf[1][0]),
                       "+v"(pbf[1][1]), "+v"(pbf[1][2]), "+v"(pbf[1][3])
                     : "i"((ABL & 2) ? 0 : 8));
        __builtin_amdgcn_sched_barrier(0);
      }
      const bool has_bias = p.bias != nullptr;   // kernel-argument uniform: a select, no branch
      auto bias_f4 = [&](int h, float4 (&b4)[4]) {
#pragma unroll
        for (int j = 0; j < 4; ++j)
          b4[j] = has_bias ? make_float4(pbf[h][j][0], pbf[h][j][1], pbf[h][j][2], pbf[h][j][3])
                           : make_float4(0.f, 0.f, 0.f, 0.f);
      };
      // FUSE 2 on a tile full in M (N % 256 == 0): the residual update X[row] += acc + bias, its
      // bf16 copy and LN partials (resid_stats_rows' arithmetic, bitwise), with the X loads as
      // untracked asm (a rolling window of W4_XW rows) and counted waits: the compiler's own waits
      // for them were vmcnt(0), 17 per tile.  Per row: 4 loads, then 7 stores (4 X, 2 bf16, 1 stats).
      auto resid_stats_full = [&](fv4 (&a)[8][4], int64_t rb, int64_t cb, int r16x, int gx, const float4 (&b4)[4]) {
        constexpr int XW = 4;
        int64_t rpg = p.rpg;
        asm volatile("" : "+s"(rpg));
        const bool ident = rpg >= p.M && p.goff == 0;
        const int part = (int)(cb >> 6);
        const float* xs = resid_src(p);
        auto orow_of = [&](int i) -> int64_t {
          const int64_t m = rb + i * 16 + r16x;
          return ident ? m : map_row(m, rpg, p.gstride, p.goff);
        };
        fv4 x[XW][4];
        auto load_row = [&](int i) {
          const float* src = xs + orow_of(i) * p.ldo + cb + 4 * gx;
#pragma unroll
          for (int j = 0; j < 4; ++j) x[i % XW][j] = w4_gld4(src + j * 16);
        };
#pragma unroll
        for (int i = 0; i < XW; ++i) load_row(i);
        w4_for<8>([&](auto ic) {
          constexpr int i = decltype(ic)::value;
          // VMEM ops issued after row i's loads when row i is consumed: the loads of rows i+1 ..
          // min(i+XW-1, 7) (4 each) and the 7 stores of each row k < i issued after them -- rows
          // 0 .. i-1 for a prologue row (i < XW), else the XW rows i-XW .. i-1 (row i's loads were
          // issued in row i-XW, before its stores).  Extra ops only make the wait longer.
          constexpr int later_loads = 4 * ((i + XW - 1 < 8 ? i + XW - 1 : 7) - i);
          constexpr int later_stores = 7 * (i < XW ? i : XW);
          w4_vm_wait<later_loads + later_stores>();
          asm volatile("" : "+v"(x[i % XW][0]), "+v"(x[i % XW][1]), "+v"(x[i % XW][2]), "+v"(x[i % XW][3]));
          const int64_t orow = orow_of(i);
          fv4 v[4];
          float sm = 0.f, q = 0.f;
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const fv4 xv = x[i % XW][j];
            fv4 av = a[i][j];
            av += fv4{b4[j].x, b4[j].y, b4[j].z, b4[j].w};
            v[j] = fv4{xv[0] + av[0], xv[1] + av[1], xv[2] + av[2], xv[3] + av[3]};
            sm += (v[j][0] + v[j][1]) + (v[j][2] + v[j][3]);
            q += sumsq4(v[j][0], v[j][1], v[j][2], v[j][3]);
          }
          if constexpr (i + XW < 8) load_row(i + XW);
          sm = sum_lane_groups(sm);
          q = sum_lane_groups(q);
          float* dst = (float*)p.out + orow * p.ldo + cb + 4 * gx;
#pragma unroll
          for (int j = 0; j < 4; ++j) *reinterpret_cast<fv4*>(dst + j * 16) = v[j];
          bf16_t* xbo = (bf16_t*)p.xb_out + orow * p.ldo + cb;
          store_pair_bf16(xbo, v[0], v[1], gx);
          store_pair_bf16(xbo + 32, v[2], v[3], gx);
          *reinterpret_cast<float2*>(p.stats_out + (orow * LN_PARTS + part) * 2) = make_float2(sm, q);
          __builtin_amdgcn_sched_barrier(0);
        });
      };
      if constexpr (FUSE == 1) {
        // acc <- rstd * (acc - mu * wsum[n]) + bias_f[n] (ln_affine, on the prefetched loads): wait
        // for them -- only the last step's 8 DMA ops were issued after them -- tied to every value
        asm volatile("s_waitcnt vmcnt(%24)"
                     : "+v"(pst[0][0]), "+v"(pst[0][1]), "+v"(pst[0][2]), "+v"(pst[1][0]), "+v"(pst[1][1]),
                       "+v"(pst[1][2]), "+v"(pst[2][0]), "+v"(pst[2][1]), "+v"(pst[2][2]), "+v"(pst[3][0]),
                       "+v"(pst[3][1]), "+v"(pst[3][2]), "+v"(pst[4][0]), "+v"(pst[4][1]), "+v"(pst[4][2]),
                       "+v"(pst[5][0]), "+v"(pst[5][1]), "+v"(pst[5][2]), "+v"(pst[6][0]), "+v"(pst[6][1]),
                       "+v"(pst[6][2]), "+v"(pst[7][0]), "+v"(pst[7][1]), "+v"(pst[7][2])
                     : "i"((ABL & 2) ? 0 : 8));
        asm volatile("" : "+v"(pws[0][0]), "+v"(pws[0][1]), "+v"(pws[0][2]), "+v"(pws[0][3]), "+v"(pws[1][0]),
                          "+v"(pws[1][1]), "+v"(pws[1][2]), "+v"(pws[1][3]), "+v"(pbf[0][0]), "+v"(pbf[0][1]),
                          "+v"(pbf[0][2]), "+v"(pbf[0][3]), "+v"(pbf[1][0]), "+v"(pbf[1][1]), "+v"(pbf[1][2]),
                          "+v"(pbf[1][3]));
        __builtin_amdgcn_sched_barrier(0);
        const float invk = p.ln_invk;
        float mu[8], rs[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          float sm = (pst[i][0].x + pst[i][1].x) + pst[i][2].x;
          float q = (pst[i][0].y + pst[i][1].y) + pst[i][2].y;
          sm = sum_lane_groups(sm);
          q = sum_lane_groups(q);
          const float m_ = sm * invk;
          const float var = fmaxf(__builtin_fmaf(-m_, m_, q * invk), 0.f);   // explicit: no contraction freedom
          rs[i] = 1.0f / sqrtf(var + p.ln_eps);
          mu[i] = -m_ * rs[i];
        }
#pragma unroll
        for (int h = 0; h < 2; ++h)
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const fv4 w4 = pws[h][j], b4 = pbf[h][j];
#pragma unroll
            for (int i = 0; i < 8; ++i) {
              acc[h][i][j][0] = fmaf(rs[i], acc[h][i][j][0], fmaf(mu[i], w4[0], b4[0]));
              acc[h][i][j][1] = fmaf(rs[i], acc[h][i][j][1], fmaf(mu[i], w4[1], b4[1]));
              acc[h][i][j][2] = fmaf(rs[i], acc[h][i][j][2], fmaf(mu[i], w4[2], b4[2]));
              acc[h][i][j][3] = fmaf(rs[i], acc[h][i][j][3], fmaf(mu[i], w4[3], b4[3]));
            }
          }
        __builtin_amdgcn_sched_barrier(0);
      }
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int64_t cb = cbase + 64 * h;
        if constexpr (FUSE == 2) {
          float4 b4[4];
          bias_f4(h, b4);
          if (rbase + 128 <= p.M) resid_stats_full(acc[h], rbase, cb, r16, g, b4);
          else {                          // an M-edge tile (rows past M): the shared epilogue, an
            GemmParams pe = p;            // opaque row-map divisor (not hoisted into the K loop)
            asm volatile("" : "+s"(pe.rpg));
            epilogue_resid_stats<8, 4, DSVT_STATS_W, true>(pe, acc[h], rbase, cb, r16, g, b4);
          }
        } else if constexpr (CLAMPED) {
          // bias / GELU, bf16 out, N % 256 == 0: 16-byte pair stores, rows past M clamped to M - 1
          // (their accumulators are row M - 1's: identical rewrites)
          float4 b4[4];
          if constexpr (FUSE == 1) {
#pragma unroll
            for (int j = 0; j < 4; ++j) b4[j] = make_float4(0.f, 0.f, 0.f, 0.f);
          } else {
            bias_f4(h, b4);
          }
          // (an opaque copy of the row map: its division constants are formed here, per tile, not
          // hoisted out of the tile loop and held -- or spilled -- through the K loop)
          int64_t rpg = p.rpg;
          asm volatile("" : "+s"(rpg));
          const bool ident = rpg >= p.M && p.goff == 0;
#pragma unroll
          for (int i = 0; i < 8; ++i) {
            int64_t m = rbase + i * 16 + r16;
            m = m < p.M ? m : p.M - 1;
            const int64_t orow = ident ? m : map_row(m, rpg, p.gstride, p.goff);
            fv4 v[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) v[j] = acc[h][i][j] + fv4{b4[j].x, b4[j].y, b4[j].z, b4[j].w};
            if constexpr (EPI == EPI_GELU) {
#pragma unroll
              for (int j = 0; j < 4; ++j)
#pragma unroll
                for (int e = 0; e < 4; e += 2) {
                  const f2v r = gelu_bf16out2(f2v{v[j][e], v[j][e + 1]});
                  v[j][e] = r.x;
                  v[j][e + 1] = r.y;
                }
            }
            bf16_t* const dst = (bf16_t*)p.out + orow * p.ldo + cb;
            store_pair_bf16(dst, v[0], v[1], g);
            store_pair_bf16(dst + 32, v[2], v[3], g);
            __builtin_amdgcn_sched_barrier(0);
          }
        } else {
          float4 b4[4];
          bias_of(cb, b4);
#pragma unroll
          for (int i = 0; i < 8; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j) acc[h][i][j] += fv4{b4[j].x, b4[j].y, b4[j].z, b4[j].w};
          epilogue_direct<8, 4, EPI, OUT_F32, 0, false, true, EPI == EPI_GELU, false, NFULL, true>(
              p, acc[h], rbase, cb, r16, g);
        }
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    post = W4_NBUF - 1;
    if constexpr (POST == 0) {           // a partial tile's stores are fewer: count none
      if (!(CLAMPED || (rbase + 128 <= p.M && cbase + 128 <= p.N))) post = 0;
    }
    __builtin_amdgcn_sched_barrier(0);
    if constexpr ((ABL & 8) == 0) {       // stage u's fragments (its DMA landed at boundary u - 1)
      const uint32_t o = (uint32_t)((u % W4_NBUF) * W4_STAGE);
      w4_for<16>([&](auto rc) { read_frag(rc, fa0, fb0, rdA + o, rdB + o); });
    }
  }
  w4_vm_wait<0>();                        // no LDS-DMA may land after the workgroup has left
}

// K a multiple of 64 with at least NBUF stages, 32-bit LDS-DMA source offsets; bias / GELU with a
// bf16 output and N % 256 == 0 (the 16-byte store path; a bias or none: prefetched unconditionally),
// or the fp32 residual (with a bias unless the statistics epilogue)
bool gemm_4w_ok(const GemmParams& p, int epi, int out_f32) {
  const bool nfull_bf16 = (epi == EPI_BIAS || epi == EPI_GELU) && !out_f32 && p.N % 256 == 0;
  if (p.stats_out && p.N % 256) return false;          // the 128-column wave slab of the stats epilogue
  return p.K >= 32 * W4_NBUF && p.K % 64 == 0 && p.M >= 1 && p.N >= 1 && (nfull_bf16 || epi == EPI_RESID) &&
         (p.bias != nullptr || nfull_bf16 || p.stats_out) &&
         !p.row_scale && (p.M - 1) * p.lda * 2 + p.K * 2 <= (int64_t)UINT32_MAX &&
         (p.N - 1) * p.ldw * 2 + p.K * 2 <= (int64_t)UINT32_MAX;
}

hipError_t launch_gemm_4w(const GemmParams& p, int epi, int out_f32, hipStream_t s, int abl) {
  if (!gemm_4w_ok(p, epi, out_f32)) return hipErrorInvalidValue;
  const int64_t tiles = ((p.M + 255) / 256) * ((p.N + 255) / 256);
  int64_t G = 256;                                    // one workgroup per CU (128-160 KiB LDS)
  const int64_t per_x = (tiles + 7) / 8;
  if (per_x * 8 < G) G = per_x * 8;
  dim3 grid((unsigned)G), block(256);
  if (abl) {                                          // diagnostic builds: EPI_BIAS, bf16 out
    if (epi != EPI_BIAS) return hipErrorInvalidValue;
    switch (abl) {
      case 2: gemm_4w_kernel<EPI_BIAS, false, 2, true><<<grid, block, 0, s>>>(p); break;
      case 4: gemm_4w_kernel<EPI_BIAS, false, 4, true><<<grid, block, 0, s>>>(p); break;
      case 16: gemm_4w_kernel<EPI_BIAS, false, 16, true><<<grid, block, 0, s>>>(p); break;
      case 18: gemm_4w_kernel<EPI_BIAS, false, 18, true><<<grid, block, 0, s>>>(p); break;
      case 26: gemm_4w_kernel<EPI_BIAS, false, 26, true><<<grid, block, 0, s>>>(p); break;
      default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
  }
  if (p.ln_stats) {                                   // LayerNorm folded in (dsvt_gemm_lnx_fwd)
    if (!p.ln_wsum) return hipErrorInvalidValue;
    if (epi == EPI_BIAS) gemm_4w_kernel<EPI_BIAS, false, 0, true, 1><<<grid, block, 0, s>>>(p);
    else gemm_4w_kernel<EPI_GELU, false, 0, true, 1><<<grid, block, 0, s>>>(p);
    return hipGetLastError();
  }
  if (p.stats_out) {                                  // residual + LN inputs (dsvt_gemm_resid_stats_fwd)
    if (epi != EPI_RESID || !p.xb_out || p.N % 256) return hipErrorInvalidValue;
    gemm_4w_kernel<EPI_RESID, true, 0, false, 2><<<grid, block, 0, s>>>(p);
    return hipGetLastError();
  }
  switch (epi) {
    case EPI_BIAS: gemm_4w_kernel<EPI_BIAS, false, 0, true><<<grid, block, 0, s>>>(p); break;
    case EPI_GELU: gemm_4w_kernel<EPI_GELU, false, 0, true><<<grid, block, 0, s>>>(p); break;
    case EPI_RESID: gemm_4w_kernel<EPI_RESID, true><<<grid, block, 0, s>>>(p); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

}  // namespace dsvt
