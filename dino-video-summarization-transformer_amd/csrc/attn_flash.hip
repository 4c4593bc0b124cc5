// Flash attention forward for CONTIGUOUS sequences (joint space-time attention, config 4:
// 1 + 196 x 16 = 3137 keys; space-only frames), bf16 perf mode, head_dim 64.
//   models/timesformer.py:55-87 (Attention.forward) under :120-123 (joint_space_time)
//
// Geometry: one 256-thread workgroup = 4 waves x QT 16-query tiles (QT = 2: 128 queries of one
// (sequence, head)); three workgroups per CU (48 KiB LDS, <= 168 VGPRs each).
// K/V: 64-key tiles staged by LDS-DMA (global_load_lds_dwordx4, 1 KiB = 8 rows x 128 B per
// wave instruction, 4 per wave per tile) into a 3-deep ring, two tiles ahead, one barrier per
// tile.  The rows of a sequence are contiguous token rows of the [rows, 3C] qkv tensor, so the
// per-lane DMA source address carries the LDS swizzle:
//   K rows: 16-B chunk' = chunk ^ ((row >> 1) & 7)  -- the 16-row ds_read_b128 of the S MFMA
//           A operand covers all 64 banks (the GEMM kernels' image);
//   V rows: chunk' = chunk ^ (row & 6)             -- the 8-row x 32-B ds_read_b64_tr_b16
//           reads of the P.V A operand (V^T) cover all 64 banks.
// Math per tile and wave (v_mfma_f32_16x16x32_bf16): S^T = K.Q^T (K as the A operand: a lane
// holds 16 scores of ONE query, so the row max / sum are in-register + two lane xors), online
// softmax in the exp2 domain (scale * log2 e folded into one fma per score), P^T straight from
// the score registers as the B operand of O^T += V^T.P^T (k order permuted to the tr-read V
// fragments), 32 MFMAs per 64 keys x 32 queries.
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
constexpr int FA_NBUF = 3;
constexpr float FA_LAZY = 8.0f;               // running-max slack, log2 units (P <= 2^8 before 1 / l)

template <int N>
__device__ __forceinline__ void fa_vmwait() {
  static_assert(N >= 0 && N < 64, "vmcnt immediate");
  __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | 0x0F70);
}

__device__ __forceinline__ void fa_barrier() {
  __builtin_amdgcn_sched_barrier(0);
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
}

}  // namespace

template <int QT>
__global__ __launch_bounds__(256, 2) void attn_flash_bf16(AttnParams p) {
  __shared__ __attribute__((aligned(16))) char smem[FA_NBUF * 2 * FA_TILE];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r16 = lane & 15, g = lane >> 4;
  const int64_t seq = blockIdx.z;
  const int h = blockIdx.y;
  const int64_t L = p.seqlen;
  const int64_t ld = p.ld_qkv, C = p.C;
  const bf16_t* rows0 = (const bf16_t*)p.qkv + seq * p.L * ld;      // token row 0 of the sequence
  const int64_t qbase = (int64_t)blockIdx.x * (64 * QT) + wave * (16 * QT);
  const int nt = (int)((L + 63) >> 6);

  // ---- Q^T fragments (B operand): query r16 of each tile, dims 8g.. and 32 + 8g..
  sv8 qf[QT][2];
#pragma unroll
  for (int qt = 0; qt < QT; ++qt) {
    int64_t qi = qbase + qt * 16 + r16;
    qi = qi < L ? qi : L - 1;
    const bf16_t* qr = rows0 + qi * ld + h * 64 + g * 8;
    qf[qt][0] = *reinterpret_cast<const sv8*>(qr);
    qf[qt][1] = *reinterpret_cast<const sv8*>(qr + 32);
  }

  // ---- DMA roles: wave w stages rows [16w, 16w + 16) of the K and the V tile, 8 per instruction
  const int prow = lane >> 3, pch = lane & 7;
  // stream position j -> key tile: the last (partial) tile first, then 0, 1, ...
  auto key_tile = [&](int j) { return j == 0 ? nt - 1 : j - 1; };
  auto stage = [&](int j) {
    const int c = key_tile(j);
    char* kd = smem + (j % FA_NBUF) * 2 * FA_TILE;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      int64_t key = (int64_t)c * 64 + wave * 16 + i * 8 + prow;
      key = key < L ? key : L - 1;                 // rows past the end: masked in the first tile
      const bf16_t* src = rows0 + key * ld + C + h * 64;
      char* dk = kd + (wave * 16 + i * 8) * FA_ROWB;
      const int r = wave * 16 + i * 8 + prow;      // tile row: its K / V swizzles
      __builtin_amdgcn_global_load_lds((const void*)(src + (pch ^ ((r >> 1) & 7)) * 8), LDS_PTR(dk), 16, 0, 0);
      __builtin_amdgcn_global_load_lds((const void*)(src + C + (pch ^ (r & 6)) * 8), LDS_PTR(dk + FA_TILE), 16, 0,
                                       0);
    }
  };

  // ---- LDS fragment offsets
  const int xs = (r16 >> 1) & 7;
  const int krd0 = r16 * FA_ROWB + ((g ^ xs) << 4), krd1 = r16 * FA_ROWB + (((4 + g) ^ xs) << 4);
  // V^T tr-read of (st2, dt): row st2*32 + 4g + (r16 >> 2), bytes dt*32 + 8 (r16 & 3) of the
  // logical row; the chunk pair (2dt, 2dt + 1) ^ (row & 6) = 2 (dt ^ f2) + {0, 1}, f2 = (row & 6) / 2
  const int vrow = 4 * g + (r16 >> 2), vf2 = (vrow & 6) >> 1;
  const int vrd0 = vrow * FA_ROWB + ((r16 & 2) << 3) + 8 * (r16 & 1);
  auto vrd = [&](int st2, int dt) { return vrd0 + st2 * 32 * FA_ROWB + ((dt ^ vf2) << 5); };

  const float sl2 = p.scale * 1.4426950408889634f;
  float m2[QT];
  fv4 o[QT][4], lacc[QT];               // lacc: the row sums of P, accumulated by MFMA against ones
  typedef short sv8_t __attribute__((ext_vector_type(8)));
  const sv8_t ones = {0x3F80, 0x3F80, 0x3F80, 0x3F80, 0x3F80, 0x3F80, 0x3F80, 0x3F80};   // bf16 1.0

  // one 64-key tile from ring slot `buf`; FIRST: the peeled, masked tile that opens the stream
  auto tile = [&](int buf, auto first_c) {
    constexpr bool FIRST = decltype(first_c)::value;
    const char* Ks = smem + buf * 2 * FA_TILE;
    const char* Vs = Ks + FA_TILE;
    fv4 s[QT][4];
#pragma unroll
    for (int kt = 0; kt < 4; ++kt) {
      const sv8 k0 = *reinterpret_cast<const sv8*>(Ks + kt * 16 * FA_ROWB + krd0);
      const sv8 k1 = *reinterpret_cast<const sv8*>(Ks + kt * 16 * FA_ROWB + krd1);
#pragma unroll
      for (int qt = 0; qt < QT; ++qt) {
        const fv4 z = fv4{0.f, 0.f, 0.f, 0.f};
        s[qt][kt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(k0, qf[qt][0], z, 0, 0, 0);
        s[qt][kt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(k1, qf[qt][1], s[qt][kt], 0, 0, 0);
      }
    }
    if constexpr (FIRST) {
      mfma_result_fence();
      const int lim = (int)(L - (int64_t)(nt - 1) * 64);     // valid keys of the last tile, 1..64
#pragma unroll
      for (int qt = 0; qt < QT; ++qt)
#pragma unroll
        for (int kt = 0; kt < 4; ++kt)
#pragma unroll
          for (int jj = 0; jj < 4; ++jj)
            s[qt][kt][jj] = (kt * 16 + 4 * g + jj) < lim ? s[qt][kt][jj] : -INFINITY;
    }
    // online softmax (exp2 domain) with a LAZY running max: m2 is raised -- and O / l rescaled --
    // only when some query of the wave sees a score more than FA_LAZY (log2 units) above it, so
    // after the first tiles the rescale multiplies are skipped; P values up to 2^FA_LAZY are exact
    // in fp32 / representable in bf16 and the final 1 / l normalizes them.  s becomes P; the row
    // sums come out of the P.V MFMAs (an all-ones V^T block), not VALU adds.
#pragma unroll
    for (int qt = 0; qt < QT; ++qt) {
      float mx = -INFINITY;
#pragma unroll
      for (int kt = 0; kt < 4; ++kt)
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) mx = fmaxf(mx, s[qt][kt][jj]);
      mx = max_lane_groups(mx) * sl2;       // VALU permlane swaps, no LDS-crossbar round trip
      if constexpr (FIRST) {
        m2[qt] = mx;
#pragma unroll
        for (int dt = 0; dt < 4; ++dt) o[qt][dt] = fv4{0.f, 0.f, 0.f, 0.f};
        lacc[qt] = fv4{0.f, 0.f, 0.f, 0.f};
      } else if (__builtin_amdgcn_ballot_w64(mx > m2[qt] + FA_LAZY) != 0) {   // wave-uniform, rare
        mfma_result_fence();                // o / lacc are MFMA results read by VALU under a branch
        const float mn = fmaxf(m2[qt], mx);
        const float alpha = __builtin_amdgcn_exp2f(m2[qt] - mn);
#pragma unroll
        for (int dt = 0; dt < 4; ++dt) o[qt][dt] *= alpha;
        lacc[qt] *= alpha;
        m2[qt] = mn;
      }
#pragma unroll
      for (int kt = 0; kt < 4; ++kt)
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) s[qt][kt][jj] = __builtin_amdgcn_exp2f(fmaf(s[qt][kt][jj], sl2, -m2[qt]));
    }
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
        const sv4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
            (__attribute__((address_space(3))) sv4*)(Vs + vrd(st2, dt)));
        const sv4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
            (__attribute__((address_space(3))) sv4*)(Vs + vrd(st2, dt) + 16 * FA_ROWB));
        const sv8 vf = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
#pragma unroll
        for (int qt = 0; qt < QT; ++qt) o[qt][dt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(vf, pb[qt], o[qt][dt], 0, 0, 0);
      }
#pragma unroll
      for (int qt = 0; qt < QT; ++qt) lacc[qt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ones, pb[qt], lacc[qt], 0, 0, 0);
    }
  };

  // ---- stream: DMA two tiles ahead, one barrier per tile
  stage(0);
  if (nt > 1) stage(1);
  for (int j = 0; j < nt; ++j) {
    if (j + 1 < nt) fa_vmwait<4>();          // this wave's tile j landed (tile j + 1 in flight)
    else fa_vmwait<0>();
    fa_barrier();                            // every wave's tile j landed; tile j - 1 fully read
    if (j + 2 < nt) stage(j + 2);            // into the slot tile j - 1 used
    if (j == 0) tile(0, std::true_type{});
    else tile(j % FA_NBUF, std::false_type{});
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

bool attn_flash_ok(int dtype, const AttnParams& p) {
  return dtype == 0 && p.tok_stride == 1 && p.tin == 1 && !p.probs && !p.cls_aux && !p.seq_scale &&
         p.seqlen >= 1 && p.seqlen <= p.L && p.C >= 64 * p.heads && p.ld_qkv >= 3 * p.C;
}

// qt: 0 = automatic -- 128 queries per workgroup (QT = 2) when that grid gives every CU two
// workgroups, else 64 (QT = 1: twice the workgroups for the same keys).  Measured at L = 3137, 12
// heads (tools/attn_joint_bench.py): one clip (300 workgroups at QT = 2) 77.0 vs 84.7 us, two
// clips (600) 121.2 vs 113.2 us.
hipError_t launch_attn_flash(const AttnParams& p, hipStream_t s, int qt) {
  const int64_t blocks2 = (p.seqlen + 127) / 128 * p.heads * p.nb;
  if (qt == 0) qt = blocks2 >= 2 * 256 ? 2 : 1;
  if (qt == 2) {
    dim3 grid((unsigned)((p.seqlen + 127) / 128), (unsigned)p.heads, (unsigned)p.nb);
    attn_flash_bf16<2><<<grid, 256, 0, s>>>(p);
  } else {
    dim3 grid((unsigned)((p.seqlen + 63) / 64), (unsigned)p.heads, (unsigned)p.nb);
    attn_flash_bf16<1><<<grid, 256, 0, s>>>(p);
  }
  return hipGetLastError();
}

}  // namespace dsvt
