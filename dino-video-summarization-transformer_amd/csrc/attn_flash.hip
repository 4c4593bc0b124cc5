// Flash attention forward for CONTIGUOUS sequences (joint space-time attention, config 4:
// 1 + 196 x 16 = 3137 keys; space-only frames), bf16 perf mode, head_dim 64.
//   models/timesformer.py:55-87 (Attention.forward) under :120-123 (joint_space_time)
//
// Geometry: a wave owns QT 16-query tiles of one (sequence, head); a workgroup is either
//   4 waves x QT (QT = 1 or 2: 64 / 128 queries, 32 KiB LDS, three workgroups per CU), or
//   8 waves, waves 0-3 with QA tiles and waves 4-7 with QB (e.g. 3 + 2: 320 queries), one
//   workgroup per CU (64 KiB LDS; the register count keeps a second one out).  A SIMD then holds waves w and w + 4 of the workgroup, i.e.
//   QA + QB query tiles: the split is chosen so that the grid's per-SIMD work is even -- config 4
//   (2 clips x 12 heads x 197 tiles) as 240 workgroups of 5 tiles per SIMD instead of 600
//   workgroups of 2 tiles at three per CU (88 CUs carry 6 tiles per SIMD, the rest 4).
// K/V: 64-key tiles staged by LDS-DMA (global_load_lds_dwordx4, 1 KiB = 8 rows x 128 B per
// wave instruction) into an NBUF-deep ring (2 tiles for 4 waves, 4 for 8: measured optima),
// NBUF - 1 tiles ahead, one barrier per tile.  The
// rows of a sequence are contiguous token rows of the [rows, 3C] qkv tensor, so the per-lane
// DMA source offset carries the LDS swizzle (the same for every full tile: a scalar tile base +
// a per-lane 32-bit offset):
//   K rows: 16-B chunk' = chunk ^ ((row >> 1) & 7)  -- the 16-row ds_read_b128 of the S MFMA
//           A operand covers all 64 banks (the GEMM kernels' image);
//   V rows: chunk' = chunk ^ (row & 6)             -- the 8-row x 32-B ds_read_b64_tr_b16
//           reads of the P.V A operand (V^T) cover all 64 banks.
// Math per tile and wave (v_mfma_f32_16x16x32_bf16): S^T = K.Q^T (K as the A operand: a lane
// holds 16 scores of ONE query), online softmax in the exp2 domain, P^T straight from the score
// registers as the B operand of O^T += V^T.P^T (k order permuted to the tr-read V fragments).
// The kernel is VALU-ISSUE bound (rocprofv3: SQ_ACTIVE_INST_VALU ~2x the MFMA busy cycles), so the
// softmax is stripped to exp + convert per score:
//   * Q is pre-scaled by scale * log2(e) when its fragments are loaded (one extra bf16 rounding,
//     the size of P's own), and the running max enters as the MFMA's ACCUMULATOR INPUT (C = -m):
//     the MFMA emits s - m in the exp2 domain, no fma per score;
//   * the running max is LAZY: it is raised -- and O / l rescaled -- only when some lane's partial
//     max (its 16 scores, no cross-lane reduction) exceeds it by FA_LAZY (one compare + ballot per
//     tile); P <= 2^FA_LAZY is exact in fp32 and representable in bf16, the final 1 / l normalizes;
//   * the row sums l come out of the P.V MFMAs against an all-ones V^T block, not VALU adds;
//   * V^T fragments are read by inline-asm ds_read_b64_tr_b16 at immediate offsets: the builtin
//     made the compiler wait for EVERY in-flight LDS-DMA (vmcnt(0), the prefetches included)
//     before the first V read of each tile, and re-derive 16 addresses per tile.
// The LAST (possibly partial) key tile is processed FIRST, peeled out of the loop: it is the
// only tile that needs key masking, so the loop body is straight-line code (the
// MFMA -> VALU hazard rule: masking happens after mfma_result_fence(), outside the loop).
#include <math.h>

#include <type_traits>

#include "common.h"

namespace dsvt {

namespace {

constexpr int FA_ROWB = 128;                  // bytes per staged row: 64 bf16
constexpr int FA_TILE = 64 * FA_ROWB;         // one K or V tile, 8 KiB
constexpr float FA_LAZY = 8.0f;               // running-max slack, log2 units (P <= 2^8 before 1 / l)

template <int N>
__device__ __forceinline__ void fa_vmwait() {
  static_assert(N >= 0 && N < 64, "vmcnt immediate");
  __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | 0x0F70);
}

// wait until at most n (wave-uniform, <= MAXN) stages of VPS LDS-DMA instructions are in flight
template <int VPS, int MAXN>
__device__ __forceinline__ void fa_vmwait_stages(int n) {
  if constexpr (MAXN == 0) {
    fa_vmwait<0>();
  } else {
    if (n >= MAXN) fa_vmwait<VPS * MAXN>();
    else fa_vmwait_stages<VPS, MAXN - 1>(n);
  }
}

__device__ __forceinline__ void fa_barrier() {
  __builtin_amdgcn_sched_barrier(0);
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
}

// ds_read_b64_tr_b16 at an immediate offset; not tracked by the compiler (the caller waits lgkmcnt)
template <int OFF>
__device__ __forceinline__ sv4 fa_tr_read(unsigned a) {
  sv4 r;
  asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(r) : "v"(a), "i"(OFF));
  return r;
}

// s_waitcnt lgkmcnt(0) tied to the tr-read results, so no use of them is scheduled above it
__device__ __forceinline__ void fa_lgkm_wait(sv4 (&a)[4], sv4 (&b)[4]) {
  asm volatile("s_waitcnt lgkmcnt(0)"
               : "+v"(a[0]), "+v"(a[1]), "+v"(a[2]), "+v"(a[3]), "+v"(b[0]), "+v"(b[1]), "+v"(b[2]), "+v"(b[3]));
}

__device__ __forceinline__ unsigned lds_addr(const void* p) {
  return (unsigned)(uintptr_t)(__attribute__((address_space(3))) const char*)p;
}

// max of a lane's 16 scores
__device__ __forceinline__ float max16(const fv4 (&s)[4]) {
  float m = fmaxf(fmaxf(s[0][0], s[0][1]), s[0][2]);
  m = fmaxf(fmaxf(m, s[0][3]), s[1][0]);
  m = fmaxf(fmaxf(m, s[1][1]), s[1][2]);
  m = fmaxf(fmaxf(m, s[1][3]), s[2][0]);
  m = fmaxf(fmaxf(m, s[2][1]), s[2][2]);
  m = fmaxf(fmaxf(m, s[2][3]), s[3][0]);
  m = fmaxf(fmaxf(m, s[3][1]), s[3][2]);
  return fmaxf(m, s[3][3]);
}

// One wave's part of a workgroup: QT 16-query tiles from query qbase of (sequence blockIdx.z,
// head blockIdx.y), NW waves staging the K / V ring of NBUF 64-key tiles in smem.
template <int QT, int NW, int NBUF>
__device__ __forceinline__ void flash_run(const AttnParams& p, char* smem, const int wave, const int lane,
                                          const int64_t qbase) {
  constexpr int RW = 64 / NW;          // K / V rows this wave stages per tile
  constexpr int NI = RW / 8;           // LDS-DMA instructions per tensor per tile
  constexpr int VPS = 2 * NI;          // vmcnt per staged tile
  constexpr int D = NBUF - 1;          // tiles in flight ahead of the one computed
  static_assert(NI >= 1 && D >= 1, "ring geometry");
  const int r16 = lane & 15, g = lane >> 4;
  const int64_t seq = blockIdx.z;
  const int h = blockIdx.y;
  const int64_t L = p.seqlen;
  const int64_t ld = p.ld_qkv, C = p.C;
  const bf16_t* rows0 = (const bf16_t*)p.qkv + seq * p.L * ld;      // token row 0 of the sequence
  const int nt = (int)((L + 63) >> 6);
  const float sl2 = p.scale * 1.4426950408889634f;

  // ---- Q^T fragments (B operand), pre-scaled by scale * log2(e): query r16 of each tile, dims
  // 8g.. and 32 + 8g..
  sv8 qf[QT][2];
#pragma unroll
  for (int qt = 0; qt < QT; ++qt) {
    int64_t qi = qbase + qt * 16 + r16;
    qi = qi < L ? qi : L - 1;
    const bf16_t* qr = rows0 + qi * ld + h * 64 + g * 8;
#pragma unroll
    for (int half = 0; half < 2; ++half) {
      const sv8 raw = *reinterpret_cast<const sv8*>(qr + 32 * half);
      typedef unsigned uv4 __attribute__((ext_vector_type(4)));
      uv4 w;
#pragma unroll
      for (int e = 0; e < 4; ++e)
        w[e] = cvt_pk_bf16(bf2f((bf16_t)raw[2 * e]) * sl2, bf2f((bf16_t)raw[2 * e + 1]) * sl2);
      qf[qt][half] = __builtin_bit_cast(sv8, w);
    }
  }

  // ---- DMA roles: wave w stages rows [RW w, RW w + RW) of the K and the V tile, 8 per instruction
  const int prow = lane >> 3, pch = lane & 7;
  unsigned koff[NI], voff[NI];         // lane byte offsets inside a full tile (every tile but the first)
#pragma unroll
  for (int i = 0; i < NI; ++i) {
    const int r = wave * RW + i * 8 + prow;
    koff[i] = (unsigned)((r * ld + C + h * 64) * 2 + ((pch ^ ((r >> 1) & 7)) << 4));
    voff[i] = (unsigned)((r * ld + 2 * C + h * 64) * 2 + ((pch ^ (r & 6)) << 4));
  }
  // stream position j -> key tile: the last (partial) tile first, then 0, 1, ...
  auto stage = [&](int j, int slot) {
    char* kd = smem + slot * 2 * FA_TILE + wave * RW * FA_ROWB;
    if (j == 0) {
#pragma unroll
      for (int i = 0; i < NI; ++i) {
        const int r = wave * RW + i * 8 + prow;
        int64_t key = (int64_t)(nt - 1) * 64 + r;
        key = key < L ? key : L - 1;               // rows past the end: masked in the first tile
        const bf16_t* src = rows0 + key * ld + C + h * 64;
        __builtin_amdgcn_global_load_lds((const void*)(src + (pch ^ ((r >> 1) & 7)) * 8),
                                         LDS_PTR(kd + i * 8 * FA_ROWB), 16, 0, 0);
        __builtin_amdgcn_global_load_lds((const void*)(src + C + (pch ^ (r & 6)) * 8),
                                         LDS_PTR(kd + FA_TILE + i * 8 * FA_ROWB), 16, 0, 0);
      }
    } else {
      const char* tb = (const char*)rows0 + (int64_t)(j - 1) * 64 * ld * 2;   // uniform tile base
#pragma unroll
      for (int i = 0; i < NI; ++i) {
        __builtin_amdgcn_global_load_lds((const void*)(tb + koff[i]), LDS_PTR(kd + i * 8 * FA_ROWB), 16, 0, 0);
        __builtin_amdgcn_global_load_lds((const void*)(tb + voff[i]), LDS_PTR(kd + FA_TILE + i * 8 * FA_ROWB), 16,
                                         0, 0);
      }
    }
  };

  // ---- LDS fragment offsets
  const int xs = (r16 >> 1) & 7;
  const int krd0 = r16 * FA_ROWB + ((g ^ xs) << 4), krd1 = r16 * FA_ROWB + (((4 + g) ^ xs) << 4);
  // V^T tr-read of (st2, dt): row st2*32 + 4g + (r16 >> 2), bytes dt*32 + 8 (r16 & 3) of the
  // logical row; the chunk pair (2dt, 2dt + 1) ^ (row & 6) = 2 (dt ^ f2) + {0, 1}, f2 = (row & 6) / 2.
  // st2 adds 32 rows (4 KiB), the second 16-row half 2 KiB: immediate offsets
  const int vrow = 4 * g + (r16 >> 2), vf2 = (vrow & 6) >> 1;
  unsigned vl[4];
#pragma unroll
  for (int dt = 0; dt < 4; ++dt) vl[dt] = (unsigned)(vrow * FA_ROWB + ((r16 & 2) << 3) + 8 * (r16 & 1) + ((dt ^ vf2) << 5));
  const unsigned smem_lds = lds_addr(smem);

  float m2[QT];                         // running max per query (exp2 domain), lane-replicated
  fv4 cneg[QT], o[QT][4], lacc[QT];     // cneg = -m2 (the S MFMA accumulator input); lacc: row sums of P
  typedef short sv8_t __attribute__((ext_vector_type(8)));
  const sv8_t ones = {0x3F80, 0x3F80, 0x3F80, 0x3F80, 0x3F80, 0x3F80, 0x3F80, 0x3F80};   // bf16 1.0
#pragma unroll
  for (int qt = 0; qt < QT; ++qt) cneg[qt] = fv4{0.f, 0.f, 0.f, 0.f};

  // one 64-key tile from ring slot `slot`; FIRST: the peeled, masked tile that opens the stream
  auto tile = [&](int slot, auto first_c) {
    constexpr bool FIRST = decltype(first_c)::value;
    const char* Ks = smem + slot * 2 * FA_TILE;
    const unsigned vb = smem_lds + (unsigned)(slot * 2 * FA_TILE + FA_TILE);
    fv4 s[QT][4];
#pragma unroll
    for (int kt = 0; kt < 4; ++kt) {
      const sv8 k0 = *reinterpret_cast<const sv8*>(Ks + kt * 16 * FA_ROWB + krd0);
      const sv8 k1 = *reinterpret_cast<const sv8*>(Ks + kt * 16 * FA_ROWB + krd1);
#pragma unroll
      for (int qt = 0; qt < QT; ++qt) {
        s[qt][kt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(k0, qf[qt][0], cneg[qt], 0, 0, 0);
        s[qt][kt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(k1, qf[qt][1], s[qt][kt], 0, 0, 0);
      }
    }
    // V^T fragments of both 32-key steps: issued behind the S MFMAs, waited for before the P.V ones
    sv4 vlo[2][4], vhi[2][4];
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) {
      const unsigned a = vb + vl[dt];
      vlo[0][dt] = fa_tr_read<0>(a);
      vhi[0][dt] = fa_tr_read<16 * FA_ROWB>(a);
      vlo[1][dt] = fa_tr_read<32 * FA_ROWB>(a);
      vhi[1][dt] = fa_tr_read<48 * FA_ROWB>(a);
    }
    if constexpr (FIRST) {
      mfma_result_fence();
      const int lim = (int)(L - (int64_t)(nt - 1) * 64);     // valid keys of the last tile, 1..64
#pragma unroll
      for (int qt = 0; qt < QT; ++qt) {
#pragma unroll
        for (int kt = 0; kt < 4; ++kt)
#pragma unroll
          for (int jj = 0; jj < 4; ++jj)
            s[qt][kt][jj] = (kt * 16 + 4 * g + jj) < lim ? s[qt][kt][jj] : -INFINITY;
        const float mx = max_lane_groups(max16(s[qt]));
        m2[qt] = mx;
        cneg[qt] = fv4{-mx, -mx, -mx, -mx};
#pragma unroll
        for (int kt = 0; kt < 4; ++kt) s[qt][kt] -= mx;
#pragma unroll
        for (int dt = 0; dt < 4; ++dt) o[qt][dt] = fv4{0.f, 0.f, 0.f, 0.f};
        lacc[qt] = fv4{0.f, 0.f, 0.f, 0.f};
      }
    } else {
      // s already is score - m2.  Raise m2 (rescaling O / l) only when a lane's own 16 scores
      // exceed it by FA_LAZY: wave-uniform, rare after the first tiles
      float pm[QT];
      bool up = false;
#pragma unroll
      for (int qt = 0; qt < QT; ++qt) {
        pm[qt] = max16(s[qt]);
        up |= pm[qt] > FA_LAZY;
      }
      if (__builtin_amdgcn_ballot_w64(up) != 0) {
        mfma_result_fence();                // o / lacc are MFMA results read by VALU under a branch
#pragma unroll
        for (int qt = 0; qt < QT; ++qt) {
          const float d = fmaxf(max_lane_groups(pm[qt]), 0.f);
          const float alpha = __builtin_amdgcn_exp2f(-d);
#pragma unroll
          for (int dt = 0; dt < 4; ++dt) o[qt][dt] *= alpha;
          lacc[qt] *= alpha;
          m2[qt] += d;
          cneg[qt] = fv4{-m2[qt], -m2[qt], -m2[qt], -m2[qt]};
#pragma unroll
          for (int kt = 0; kt < 4; ++kt) s[qt][kt] -= d;
        }
      }
    }
#pragma unroll
    for (int qt = 0; qt < QT; ++qt)
#pragma unroll
      for (int kt = 0; kt < 4; ++kt)
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) s[qt][kt][jj] = __builtin_amdgcn_exp2f(s[qt][kt][jj]);
    fa_lgkm_wait(vlo[0], vhi[0]);
    fa_lgkm_wait(vlo[1], vhi[1]);
    // O^T += V^T . P^T over two 32-key steps; k-slot (g, jj): jj < 4 -> key tile 2 st2, else 2 st2 + 1
#pragma unroll
    for (int st2 = 0; st2 < 2; ++st2) {
      sv8 pb[QT];
#pragma unroll
      for (int qt = 0; qt < QT; ++qt) {
        const unsigned w0 = cvt_pk_bf16(s[qt][2 * st2][0], s[qt][2 * st2][1]);
        const unsigned w1 = cvt_pk_bf16(s[qt][2 * st2][2], s[qt][2 * st2][3]);
        const unsigned w2 = cvt_pk_bf16(s[qt][2 * st2 + 1][0], s[qt][2 * st2 + 1][1]);
        const unsigned w3 = cvt_pk_bf16(s[qt][2 * st2 + 1][2], s[qt][2 * st2 + 1][3]);
        typedef unsigned uv4 __attribute__((ext_vector_type(4)));
        pb[qt] = __builtin_bit_cast(sv8, (uv4{w0, w1, w2, w3}));
      }
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) {
        const sv8 vf = __builtin_shufflevector(vlo[st2][dt], vhi[st2][dt], 0, 1, 2, 3, 4, 5, 6, 7);
#pragma unroll
        for (int qt = 0; qt < QT; ++qt) o[qt][dt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(vf, pb[qt], o[qt][dt], 0, 0, 0);
      }
#pragma unroll
      for (int qt = 0; qt < QT; ++qt) lacc[qt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ones, pb[qt], lacc[qt], 0, 0, 0);
    }
  };

  // ---- stream: DMA D tiles ahead, one barrier per tile; tile j sits in slot j % NBUF
#pragma unroll
  for (int j = 0; j < D; ++j)
    if (j < nt) stage(j, j);
  int slot = 0;
  for (int j = 0; j < nt; ++j) {
    const int ahead = nt - 1 - j;
    fa_vmwait_stages<VPS, D - 1>(ahead < D - 1 ? ahead : D - 1);   // this wave's tile j landed
    fa_barrier();                            // every wave's tile j landed; tile j - 1 fully read
    if (j + D < nt) stage(j + D, slot == 0 ? NBUF - 1 : slot - 1);   // into the slot tile j - 1 used
    if (j == 0) tile(slot, std::true_type{});
    else tile(slot, std::false_type{});
    slot = slot + 1 == NBUF ? 0 : slot + 1;
  }

  mfma_result_fence();                       // accumulators read below, after the loop exit branch
  // lane holds O[query qbase + qt*16 + r16][d = dt*16 + 4g + 0..3]
#pragma unroll
  for (int qt = 0; qt < QT; ++qt) {
    const int64_t qo = qbase + qt * 16 + r16;
    if (qo < L) {
      const float inv = 1.0f / lacc[qt][0];   // every element of lacc holds the row sum
      bf16_t* dst = (bf16_t*)p.out + (seq * p.L + qo) * p.ld_out + h * 64 + 4 * g;
#pragma unroll
      for (int dt = 0; dt < 4; ++dt)
        store4(dst + dt * 16, o[qt][dt][0] * inv, o[qt][dt][1] * inv, o[qt][dt][2] * inv, o[qt][dt][3] * inv);
    }
  }
}

// 4-wave workgroups: a 2-tile ring (32 KiB; the registers allow three per CU): 2 clips forced to
// 64-query workgroups 86.3 vs 92.1 us with 3 tiles, 128-query 87.0 vs 87.5 (tools/gpu_s28.sh)
#ifndef DSVT_FA4_NBUF
#define DSVT_FA4_NBUF 2
#endif
constexpr int FA4_NBUF = DSVT_FA4_NBUF;
// 8-wave: a 4-tile ring (64 KiB; > 128 VGPRs keep one workgroup per CU).  Measured, interleaved on
// one box (tools/gpu_s27.sh): 2 clips 79.9 us at 4 tiles vs 83.3 / 84.0 / 83.4 / 85 at 3 / 5 / 6 / 9
#ifndef DSVT_FA8_NBUF
#define DSVT_FA8_NBUF 4
#endif
constexpr int FA8_NBUF = DSVT_FA8_NBUF;

}  // namespace

template <int QT>
__global__ __launch_bounds__(256, 2) void attn_flash_bf16(AttnParams p) {
  __shared__ __attribute__((aligned(16))) char smem[FA4_NBUF * 2 * FA_TILE];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  flash_run<QT, 4, FA4_NBUF>(p, smem, wave, lane, (int64_t)blockIdx.x * (64 * QT) + wave * (16 * QT));
}

// waves 0-3: QA query tiles each, waves 4-7: QB (a SIMD holds waves w and w + 4)
template <int QA, int QB>
__global__ __launch_bounds__(512, 1) void attn_flash8_bf16(AttnParams p) {
  __shared__ __attribute__((aligned(16))) char smem[FA8_NBUF * 2 * FA_TILE];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int64_t q0 = (int64_t)blockIdx.x * (64 * (QA + QB));
  if (wave < 4) flash_run<QA, 8, FA8_NBUF>(p, smem, wave, lane, q0 + wave * (16 * QA));
  else flash_run<QB, 8, FA8_NBUF>(p, smem, wave, lane, q0 + 64 * QA + (wave - 4) * (16 * QB));
}

bool attn_flash_ok(int dtype, const AttnParams& p) {
  return dtype == 0 && p.tok_stride == 1 && p.tin == 1 && !p.probs && !p.cls_aux && !p.seq_scale &&
         p.seqlen >= 1 && p.seqlen <= p.L && p.C >= 64 * p.heads && p.ld_qkv >= 3 * p.C;
}

namespace {

// workgroup shapes: 16-query tiles per SIMD-wave pair and per workgroup; `slots`: workgroups per CU
struct FlashShape {
  int cfg, tiles_simd, queries, slots;
};
constexpr FlashShape kShapes[] = {
    {1, 1, 64, 3},    // 4 waves x QT 1
    {2, 2, 128, 3},   // 4 waves x QT 2
    {3, 5, 320, 1},   // 8 waves, 3 + 2
    {4, 3, 192, 1},   // 8 waves, 2 + 1
    {5, 4, 256, 1},   // 8 waves, 2 + 2
};

}  // namespace

// cfg: 0 = automatic, else the kShapes entry.  Automatic: the shape with the least 16-query tiles
// on the busiest SIMD (ceil(workgroups / 256 CUs) x tiles per SIMD and workgroup, each CU's
// workgroups spread over its 4 SIMDs), ties to the larger per-wave tile count (fewer K/V reads
// per query; QT = 1 last).  Measured at L = 3137, 12 heads (tools/attn_joint_bench.py): DESIGN.md §3.
hipError_t launch_attn_flash(const AttnParams& p, hipStream_t s, int cfg) {
  const int64_t pairs = (int64_t)p.heads * p.nb;
  if (cfg == 0) {
    int64_t best = -1;
    for (const int c : {3, 2, 4, 5, 1}) {     // preference order on ties: more tiles per wave first
      const FlashShape& f = kShapes[c - 1];
      const int64_t wgs = (p.seqlen + f.queries - 1) / f.queries * pairs;
      const int64_t per_simd = (wgs + 255) / 256 * f.tiles_simd;
      if (best < 0 || per_simd < best) {
        best = per_simd;
        cfg = f.cfg;
      }
    }
  }
  if (cfg < 1 || cfg > 5) return hipErrorInvalidValue;
  const FlashShape& f = kShapes[cfg - 1];
  dim3 grid((unsigned)((p.seqlen + f.queries - 1) / f.queries), (unsigned)p.heads, (unsigned)p.nb);
  switch (cfg) {
    case 1: attn_flash_bf16<1><<<grid, 256, 0, s>>>(p); break;
    case 2: attn_flash_bf16<2><<<grid, 256, 0, s>>>(p); break;
    case 3: attn_flash8_bf16<3, 2><<<grid, 512, 0, s>>>(p); break;
    case 4: attn_flash8_bf16<2, 1><<<grid, 512, 0, s>>>(p); break;
    default: attn_flash8_bf16<2, 2><<<grid, 512, 0, s>>>(p); break;
  }
  return hipGetLastError();
}

}  // namespace dsvt
