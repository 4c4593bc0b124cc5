// MFMA GEMM with fused epilogues for every nn.Linear / Conv2d(k=s=16) on the hot path.
//
//   out = A[M,K] . W[N,K]^T  (+ bias, GELU, residual add into the fp32 token tensor X,
//                             or the patch-embed pos/time-embed add)
//
// Tiling (gfx950): 128x128 output tile per 256-thread workgroup (4 waves as 2x2, each a
// 64x64 sub-tile = 4x4 MFMA 16x16 tiles).  K advances 128 BYTES per stage (64 bf16 or
// 32 fp32), staged global->LDS with `global_load_lds_dwordx4` (16 B/lane, no VGPR round
// trip) into a 2-stage ring (64 KB LDS), XOR-swizzled on the SOURCE address so the
// ds_read_b128 fragment reads are bank-conflict free (chunk' = chunk ^ ((row>>1)&7)).
//
// bf16: v_mfma_f32_16x16x32_bf16.  fp32 parity mode: v_mfma_f32_16x16x4_f32 (exact fp32
// products), with the K order inside a stage permuted (lane group g owns k = 8g..8g+7).
//
// The MFMA is issued "swapped" (W fragment as the A operand) so each lane ends with 4
// CONSECUTIVE output columns of one row: the epilogue does 16-B (fp32) / 8-B (bf16)
// vector loads/stores.  Workgroup ids are remapped so the N-tiles of one M-tile run on the
// same XCD (its A panel then stays in that XCD's L2).
#include "common.h"

namespace dsvt {

constexpr int BM = 128, BN = 128, BKB = 128;  // tile rows, tile cols, K bytes per stage
constexpr int TILE_BYTES = BM * BKB;           // 16 KB per operand per stage
constexpr int STAGE_BYTES = 2 * TILE_BYTES;    // A + W

__device__ __forceinline__ int swz(int r) { return (r >> 1) & 7; }

// Issue the global->LDS copy of one [128 rows][128 bytes] tile (16 x 1 KB pieces, 4 per
// wave).  Rows beyond `rows` re-read the last row (results masked in the epilogue).
__device__ __forceinline__ void stage_tile(const char* __restrict__ g, int64_t ld_bytes,
                                           int64_t row0, int64_t rows, int64_t kbyte0,
                                           char* lds_tile, int wave, int lane) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int piece = wave * 4 + i;
    const int r = piece * 8 + (lane >> 3);
    const int cl = lane & 7;
    int64_t gr = row0 + r;
    gr = gr < rows ? gr : rows - 1;
    const char* src = g + gr * ld_bytes + kbyte0 + ((cl ^ swz(r)) << 4);
    __builtin_amdgcn_global_load_lds((const void*)src, LDS_PTR(lds_tile + piece * 1024), 16, 0, 0);
  }
}

__device__ __forceinline__ const char* lds_chunk(const char* tile, int r, int c) {
  return tile + r * BKB + ((c ^ swz(r)) << 4);
}

template <typename T> struct TileMMA;

template <> struct TileMMA<bf16_t> {
  __device__ __forceinline__ static void run(const char* At, const char* Wt, fv4 (&acc)[4][4],
                                             int wm, int wn, int lane) {
    const int r16 = lane & 15, g = lane >> 4;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      sv8 a[4], b[4];
#pragma unroll
      for (int i = 0; i < 4; ++i)
        a[i] = *reinterpret_cast<const sv8*>(lds_chunk(At, wm * 64 + i * 16 + r16, ks * 4 + g));
#pragma unroll
      for (int j = 0; j < 4; ++j)
        b[j] = *reinterpret_cast<const sv8*>(lds_chunk(Wt, wn * 64 + j * 16 + r16, ks * 4 + g));
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b[j], a[i], acc[i][j], 0, 0, 0);
    }
  }
};

template <> struct TileMMA<float> {
  __device__ __forceinline__ static void run(const char* At, const char* Wt, fv4 (&acc)[4][4],
                                             int wm, int wn, int lane) {
    const int r16 = lane & 15, g = lane >> 4;
    fv4 a[4][2], b[4][2];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int r = wm * 64 + i * 16 + r16;
      a[i][0] = *reinterpret_cast<const fv4*>(lds_chunk(At, r, 2 * g));
      a[i][1] = *reinterpret_cast<const fv4*>(lds_chunk(At, r, 2 * g + 1));
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int r = wn * 64 + j * 16 + r16;
      b[j][0] = *reinterpret_cast<const fv4*>(lds_chunk(Wt, r, 2 * g));
      b[j][1] = *reinterpret_cast<const fv4*>(lds_chunk(Wt, r, 2 * g + 1));
    }
#pragma unroll
    for (int s = 0; s < 8; ++s)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(b[j][s >> 2][s & 3], a[i][s >> 2][s & 3],
                                                          acc[i][j], 0, 0, 0);
  }
};

// The fp32 residual tile of one wave (full tiles): 16 float4 loads, issued by gemm_kernel two
// K steps before the end of its main loop (PREF) so their latency runs under the last MFMAs.
__device__ __forceinline__ void resid_load(const GemmParams& p, int64_t m0, int64_t n0, int wm, int wn, int lane,
                                           float4 (&add)[4][4]) {
  const int r16 = lane & 15, g = lane >> 4;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int64_t orow = map_row(m0 + wm * 64 + i * 16 + r16, p.rpg, p.gstride, p.goff);
#pragma unroll
    for (int j = 0; j < 4; ++j)
      add[i][j] = *reinterpret_cast<const float4*>(resid_src(p) + orow * p.ldo + n0 + wn * 64 + j * 16 + 4 * g);
  }
}

template <typename T, int EPI, bool OUT_F32, bool CHECK, bool PRE = false>
__device__ __forceinline__ void epilogue_128(const GemmParams& p, fv4 (&acc)[4][4], int64_t m0, int64_t n0, int wm,
                                             int wn, int lane, const float4 (*pre)[4] = nullptr) {
  const int r16 = lane & 15, g = lane >> 4;
  int64_t orow[4];
  bool vrow[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int64_t m = m0 + wm * 64 + i * 16 + r16;
    vrow[i] = !CHECK || m < p.M;
    orow[i] = map_row(vrow[i] ? m : p.M - 1, p.rpg, p.gstride, p.goff);
  }
  float4 bias4[4];
  if (!CHECK || n0 + wn * 64 + 64 <= p.N) {
    bias_frag4(p.bias, n0 + wn * 64, g, bias4);         // scalar loads (lgkmcnt)
  } else {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int64_t n = n0 + wn * 64 + j * 16 + 4 * g;
      bias4[j] = (p.bias && n < p.N) ? *reinterpret_cast<const float4*>(p.bias + n) : make_float4(0.f, 0.f, 0.f, 0.f);
    }
  }
  float4 add[4][4];                    // residual / embedding addend per fragment
  if constexpr (PRE) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) add[i][j] = pre[i][j];
  } else if constexpr (EPI == EPI_RESID || EPI == EPI_PATCH) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int64_t m = m0 + wm * 64 + i * 16 + r16;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int64_t n = n0 + wn * 64 + j * 16 + 4 * g;
        add[i][j] = make_float4(0.f, 0.f, 0.f, 0.f);
        if (CHECK && (!vrow[i] || n >= p.N)) continue;
        if constexpr (EPI == EPI_RESID) {
          add[i][j] = *reinterpret_cast<const float4*>(resid_src(p) + orow[i] * p.ldo + n);
        } else {
          const int64_t rr = m % p.rpg;
          const int64_t np = rr / p.T, t = rr % p.T;
          float4 o = *reinterpret_cast<const float4*>(p.pos + (1 + (int64_t)p.pidx[np]) * p.N + n);
          if (p.temb) {
            const float4 te = *reinterpret_cast<const float4*>(p.temb + (int64_t)p.tidx[t] * p.N + n);
            o.x += te.x; o.y += te.y; o.z += te.z; o.w += te.w;
          }
          add[i][j] = o;
        }
      }
    }
  }
  float rsc[4];                        // DropPath row scales (EPI_BIAS / EPI_GELU_SAVE: the output;
#pragma unroll                         // EPI_RESID: the bias term only)
  for (int i = 0; i < 4; ++i) {
    rsc[i] = 1.0f;
    if constexpr (EPI == EPI_BIAS || EPI == EPI_GELU_SAVE || EPI == EPI_RESID)
      if (p.row_scale) rsc[i] = row_scale_of(p, m0 + wm * 64 + i * 16 + r16);
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    if (CHECK && !vrow[i]) continue;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int64_t n = n0 + wn * 64 + j * 16 + 4 * g;
      if (CHECK && n >= p.N) continue;
      float4 bb = bias4[j];
      if constexpr (EPI == EPI_RESID) {  // x + A.W^T + s[m] * bias (A already carries the scale)
        bb.x *= rsc[i]; bb.y *= rsc[i]; bb.z *= rsc[i]; bb.w *= rsc[i];
      }
      float v0 = acc[i][j][0] + bb.x, v1 = acc[i][j][1] + bb.y, v2 = acc[i][j][2] + bb.z, v3 = acc[i][j][3] + bb.w;
      if constexpr (EPI == EPI_GELU_SAVE) {
        store4((T*)p.aux + orow[i] * p.ld_aux + n, v0, v1, v2, v3);
      }
      if constexpr (EPI == EPI_GELU) {
        constexpr bool BO = !OUT_F32 && std::is_same<T, bf16_t>::value;
        v0 = gelu_out<BO>(v0); v1 = gelu_out<BO>(v1); v2 = gelu_out<BO>(v2); v3 = gelu_out<BO>(v3);
      }
      if constexpr (EPI == EPI_GELU_SAVE) {
        v0 = gelu_erf(v0); v1 = gelu_erf(v1); v2 = gelu_erf(v2); v3 = gelu_erf(v3);
      }
      if constexpr (EPI == EPI_BIAS || EPI == EPI_GELU_SAVE) {
        v0 *= rsc[i]; v1 *= rsc[i]; v2 *= rsc[i]; v3 *= rsc[i];
      }
      if constexpr (EPI == EPI_DGELU) {
        float pre[4];
        load4((const T*)p.aux + orow[i] * p.ld_aux + n, pre);
        v0 = acc[i][j][0] * gelu_erf_grad(pre[0]); v1 = acc[i][j][1] * gelu_erf_grad(pre[1]);
        v2 = acc[i][j][2] * gelu_erf_grad(pre[2]); v3 = acc[i][j][3] * gelu_erf_grad(pre[3]);
      }
      if constexpr (EPI == EPI_BIAS || EPI == EPI_GELU || EPI == EPI_GELU_SAVE || EPI == EPI_DGELU) {
        if constexpr (OUT_F32)
          store4((float*)p.out + orow[i] * p.ldo + n, v0, v1, v2, v3);
        else
          store4((T*)p.out + orow[i] * p.ldo + n, v0, v1, v2, v3);
      } else {  // EPI_RESID / EPI_PATCH: fp32 token rows
        const float4 a = add[i][j];
        store4((float*)p.out + orow[i] * p.ldo + n, v0 + a.x, v1 + a.y, v2 + a.z, v3 + a.w);
      }
    }
  }
}

template <typename T, int EPI, bool OUT_F32, bool PREF = false>
__global__ __launch_bounds__(256, 2) void gemm_kernel(GemmParams p) {
  __shared__ __attribute__((aligned(16))) char smem[2 * STAGE_BYTES];
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 1, wn = wave & 1;

  // XCD-aware bijective remap: consecutive workgroup ids of one XCD walk the N-tiles of
  // one M-tile (blocks b and b+8 share an XCD under round-robin dispatch).
  const int tilesN = (int)((p.N + BN - 1) / BN);
  const int nwg = gridDim.x, orig = blockIdx.x, xcd = orig & 7, q = nwg >> 3, r = nwg & 7;
  const int wg = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (orig >> 3);
  const int64_t m0 = (int64_t)(wg / tilesN) * BM;
  const int64_t n0 = (int64_t)(wg % tilesN) * BN;

  const char* A = (const char*)p.A;
  const char* W = (const char*)p.W;
  const int64_t lda_b = p.lda * (int64_t)sizeof(T), ldw_b = p.ldw * (int64_t)sizeof(T);
  const int nk = (int)((p.K * (int64_t)sizeof(T)) / BKB);

  fv4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = fv4{0.f, 0.f, 0.f, 0.f};

  stage_tile(A, lda_b, m0, p.M, 0, smem, wave, lane);
  stage_tile(W, ldw_b, n0, p.N, 0, smem + TILE_BYTES, wave, lane);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  // PREF (fp32 residual, full tiles): the last two K steps are peeled; the residual tile's 16
  // loads are issued right after the last stage's loads, and that step waits with vmcnt(16) --
  // for the stage, not for them -- so their latency runs under the last two steps' MFMAs.
  const bool full = m0 + BM <= p.M && n0 + BN <= p.N;
  const bool peel = PREF && full && nk >= 2;
  const int nmain = peel ? nk - 2 : nk;
  for (int kt = 0; kt < nmain; ++kt) {
    char* cur = smem + (kt & 1) * STAGE_BYTES;
    if (kt + 1 < nk) {
      char* nxt = smem + ((kt + 1) & 1) * STAGE_BYTES;
      stage_tile(A, lda_b, m0, p.M, (int64_t)(kt + 1) * BKB, nxt, wave, lane);
      stage_tile(W, ldw_b, n0, p.N, (int64_t)(kt + 1) * BKB, nxt + TILE_BYTES, wave, lane);
    }
    TileMMA<T>::run(cur, cur + TILE_BYTES, acc, wm, wn, lane);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }
  if constexpr (PREF) {
    if (peel) {
      char* cur = smem + ((nk - 2) & 1) * STAGE_BYTES;
      char* nxt = smem + ((nk - 1) & 1) * STAGE_BYTES;
      stage_tile(A, lda_b, m0, p.M, (int64_t)(nk - 1) * BKB, nxt, wave, lane);
      stage_tile(W, ldw_b, n0, p.N, (int64_t)(nk - 1) * BKB, nxt + TILE_BYTES, wave, lane);
      __builtin_amdgcn_sched_barrier(0);
      float4 xpre[4][4];
      resid_load(p, m0, n0, wm, wn, lane, xpre);
      __builtin_amdgcn_sched_barrier(0);
      TileMMA<T>::run(cur, cur + TILE_BYTES, acc, wm, wn, lane);
      asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
      __syncthreads();
      TileMMA<T>::run(nxt, nxt + TILE_BYTES, acc, wm, wn, lane);
      mfma_result_fence();
      epilogue_128<T, EPI, OUT_F32, false, true>(p, acc, m0, n0, wm, wn, lane, xpre);
      return;
    }
  }

  // ---- epilogue: lane holds C[m = .. + (lane&15)][n = .. + 4*(lane>>4) + 0..3]
  // Every global load of the epilogue (bias, residual X, pos/time embeddings) is issued
  // before the first store: stores to the row-mapped X may alias later loads as far as the
  // compiler knows, so a load/add/store loop would pay one HBM round trip per fragment.
  // Full tiles (uniform per workgroup) take a branch-free path: no per-lane bounds branches,
  // so the compiler's vmcnt waits stay exact instead of draining after every store.
  mfma_result_fence();   // acc is read under the branches below
  if (full) epilogue_128<T, EPI, OUT_F32, false>(p, acc, m0, n0, wm, wn, lane);
  else epilogue_128<T, EPI, OUT_F32, true>(p, acc, m0, n0, wm, wn, lane);
}

// ---- variant 2: the same 128x128 bf16 tile on a 4-deep LDS-DMA ring with counted waits.
// One MFMA k-step (64 B of K) per stage, 16 KB per stage, 64 KB per workgroup (2 per CU).
// Stage kt+3 is issued right after the barrier that retires stage kt-1, so three stages are
// in flight and each wave waits only for its own oldest stage (vmcnt 8 / 4 / 0) -- no
// vmcnt(0) drain per K step.  The k-steps run in the same order as variant 1's, so the two
// produce bitwise-identical results.  Row r of a stage holds its four 16-B K chunks at
// slot = chunk ^ pswz(r), pswz(r) = -(r >> 2) mod 4: the 16 lanes of every ds_read_b128
// lane group then cover all 64 banks.
// Measured on MI355X (tools/gemm_bench.py, same box, interleaved): 10-17 % SLOWER than
// variant 1 on every hot-path shape (proj 62.7 vs 58.3 us, fc2 160 vs 138 us): twice the
// barriers per K and 64-B row segments per load cost more than the drain they remove, since
// variant 1's second resident workgroup already covers it.  Kept opt-in (DSVT_GEMM_VARIANT=2).
constexpr int PB = 64;                        // K bytes per stage
constexpr int P_TILE = BM * PB;               // 8 KB per operand per stage
constexpr int P_STAGE = 2 * P_TILE;
constexpr int P_NST = 4;

__device__ __forceinline__ int pswz(int r) { return (4 - ((r >> 2) & 3)) & 3; }

__device__ __forceinline__ void stage_tile64(const char* __restrict__ g, int64_t ld_bytes, int64_t row0, int64_t rows,
                                             int64_t kbyte0, char* lds_tile, int wave, int lane) {
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int piece = wave * 2 + i;           // 8 pieces of 16 rows x 64 B, lane-linear in LDS
    const int r = piece * 16 + (lane >> 2), cl = lane & 3;
    int64_t gr = row0 + r;
    gr = gr < rows ? gr : rows - 1;
    const char* src = g + gr * ld_bytes + kbyte0 + ((cl ^ pswz(r)) << 4);
    __builtin_amdgcn_global_load_lds((const void*)src, LDS_PTR(lds_tile + piece * 1024), 16, 0, 0);
  }
}

template <int N>
__device__ __forceinline__ void p_vm_wait() {
  static_assert(N >= 0 && N < 64, "vmcnt immediate");
  __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | 0x0F70);
}

template <int EPI, bool OUT_F32>
__global__ __launch_bounds__(256, 2) void gemm_pipe_kernel(GemmParams p) {
  __shared__ __attribute__((aligned(16))) char smem[P_NST * P_STAGE];
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 1, wn = wave & 1, r16 = lane & 15, g = lane >> 4;
  const int tilesN = (int)((p.N + BN - 1) / BN);
  const int nwg = gridDim.x, orig = blockIdx.x, xcd = orig & 7, q = nwg >> 3, r = nwg & 7;
  const int wg = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (orig >> 3);
  const int64_t m0 = (int64_t)(wg / tilesN) * BM;
  const int64_t n0 = (int64_t)(wg % tilesN) * BN;
  const char* A = (const char*)p.A;
  const char* W = (const char*)p.W;
  const int64_t lda_b = p.lda * 2, ldw_b = p.ldw * 2;
  const int nk = (int)(p.K * 2 / PB);

  fv4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = fv4{0.f, 0.f, 0.f, 0.f};

#pragma unroll
  for (int st = 0; st < P_NST - 1; ++st) {
    if (st < nk) {
      stage_tile64(A, lda_b, m0, p.M, (int64_t)st * PB, smem + st * P_STAGE, wave, lane);
      stage_tile64(W, ldw_b, n0, p.N, (int64_t)st * PB, smem + st * P_STAGE + P_TILE, wave, lane);
    }
  }
  for (int kt = 0; kt < nk; ++kt) {
    const int later = nk - 1 - kt;            // stages issued beyond kt (at most 2 here)
    if (later >= 2) p_vm_wait<8>();
    else if (later == 1) p_vm_wait<4>();
    else p_vm_wait<0>();
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();             // stage kt landed for all waves; stage kt-1 read by all
    __builtin_amdgcn_sched_barrier(0);
    if (kt + P_NST - 1 < nk) {
      char* nxt = smem + ((kt + P_NST - 1) & (P_NST - 1)) * P_STAGE;
      stage_tile64(A, lda_b, m0, p.M, (int64_t)(kt + P_NST - 1) * PB, nxt, wave, lane);
      stage_tile64(W, ldw_b, n0, p.N, (int64_t)(kt + P_NST - 1) * PB, nxt + P_TILE, wave, lane);
    }
    const char* At = smem + (kt & (P_NST - 1)) * P_STAGE;
    const char* Wt = At + P_TILE;
    sv8 a[4], b[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int row = wm * 64 + i * 16 + r16;
      a[i] = *reinterpret_cast<const sv8*>(At + row * PB + ((g ^ pswz(row)) << 4));
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int row = wn * 64 + j * 16 + r16;
      b[j] = *reinterpret_cast<const sv8*>(Wt + row * PB + ((g ^ pswz(row)) << 4));
    }
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b[j], a[i], acc[i][j], 0, 0, 0);
  }
  mfma_result_fence();
  if (m0 + BM <= p.M && n0 + BN <= p.N) epilogue_128<bf16_t, EPI, OUT_F32, false>(p, acc, m0, n0, wm, wn, lane);
  else epilogue_128<bf16_t, EPI, OUT_F32, true>(p, acc, m0, n0, wm, wn, lane);
}

static bool gemm_pipe_ok(const GemmParams& p) { return p.K % 32 == 0 && p.K >= 32; }

static hipError_t launch_pipe(const GemmParams& p, int epi, int out_f32, hipStream_t s) {
  const int64_t tiles = ((p.M + BM - 1) / BM) * ((p.N + BN - 1) / BN);
  dim3 grid((unsigned)tiles), block(256);
  switch (epi) {
    case EPI_BIAS:
      if (out_f32) gemm_pipe_kernel<EPI_BIAS, true><<<grid, block, 0, s>>>(p);
      else gemm_pipe_kernel<EPI_BIAS, false><<<grid, block, 0, s>>>(p);
      break;
    case EPI_GELU:
      if (out_f32) gemm_pipe_kernel<EPI_GELU, true><<<grid, block, 0, s>>>(p);
      else gemm_pipe_kernel<EPI_GELU, false><<<grid, block, 0, s>>>(p);
      break;
    case EPI_RESID: gemm_pipe_kernel<EPI_RESID, true><<<grid, block, 0, s>>>(p); break;
    case EPI_GELU_SAVE: gemm_pipe_kernel<EPI_GELU_SAVE, false><<<grid, block, 0, s>>>(p); break;
    case EPI_DGELU:
      if (out_f32) gemm_pipe_kernel<EPI_DGELU, true><<<grid, block, 0, s>>>(p);
      else gemm_pipe_kernel<EPI_DGELU, false><<<grid, block, 0, s>>>(p);
      break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

template <typename T>
static hipError_t launch_t(const GemmParams& p, int epi, int out_f32, hipStream_t s) {
  const int64_t tiles = ((p.M + BM - 1) / BM) * ((p.N + BN - 1) / BN);
  dim3 grid((unsigned)tiles), block(256);
  switch (epi) {
    case EPI_BIAS:
      if (out_f32) gemm_kernel<T, EPI_BIAS, true><<<grid, block, 0, s>>>(p);
      else gemm_kernel<T, EPI_BIAS, false><<<grid, block, 0, s>>>(p);
      break;
    case EPI_GELU:
      if (out_f32) gemm_kernel<T, EPI_GELU, true><<<grid, block, 0, s>>>(p);
      else gemm_kernel<T, EPI_GELU, false><<<grid, block, 0, s>>>(p);
      break;
    case EPI_RESID: {
      static const int pref = getenv("DSVT_RESID_PREF") ? atoi(getenv("DSVT_RESID_PREF")) : 1;   // tuning only
      if (pref && sizeof(T) == 2) gemm_kernel<T, EPI_RESID, true, true><<<grid, block, 0, s>>>(p);
      else gemm_kernel<T, EPI_RESID, true><<<grid, block, 0, s>>>(p);
      break;
    }
    case EPI_PATCH: gemm_kernel<T, EPI_PATCH, true><<<grid, block, 0, s>>>(p); break;
    case EPI_GELU_SAVE: gemm_kernel<T, EPI_GELU_SAVE, false><<<grid, block, 0, s>>>(p); break;
    case EPI_DGELU:
      if (out_f32) gemm_kernel<T, EPI_DGELU, true><<<grid, block, 0, s>>>(p);
      else gemm_kernel<T, EPI_DGELU, false><<<grid, block, 0, s>>>(p);
      break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

static thread_local int g_gemm_variant = 0; // 0 = auto; otherwise forced (tools/gemm_bench.py, tests)

void set_gemm_variant(int v) { g_gemm_variant = v; }
// call-site scope (dsvt_set_gemm_skinny): the few-row GEMMs of the CLS-only tail and the DINO head
static thread_local int g_skinny_scope = 0;
void set_gemm_skinny(int on) { g_skinny_scope = on; }

// Kernel choice (0 = fp32 128x128, 1 = bf16 128x128, >= 2: gemm_big.hip variants, 20:
// gemm_8ph.hip).
// Measured on MI355X (tools/gemm_bench.py): every big bf16 projection with K <= 1024 (qkv
// N=2304, fc1 N=3072, proj / folded temporal fc N=768) -> persistent staggered 256x128 (v10:
// 2 WGs/CU, the epilogue of one overlaps the MFMA loop of the other, the next tile's loads fly
// under the store tail); K = 3072 (fc2), small M (DINO head) and the patch GEMM -> 128x128.
// Stream-K (variant 40) for the calls that pass a workspace (dsvt_gemm_sk_fwd): DSVT_SK = 0
// (default) never, 1 bias / GELU projections, 2 also the fp32 residual ones.  Opt-in: measured
// slower than the data-parallel kernels on every hot-path shape (qkv 118 vs 104 us, fc2 172 vs
// 137 us): writing and re-reading 256 KB fp32 partial tiles costs more than the tail round.
static bool sk_auto(int epi) {
  static const int mode = [] {
    const char* e = getenv("DSVT_SK");
    return e ? atoi(e) : 0;
  }();
  return mode >= 2 || (mode == 1 && epi != EPI_RESID);
}

// the residual GEMMs' X stream (variant 33) in the auto choice: DSVT_RESID_XS = 1 on, 0 off
static bool xs_auto() {
  static const int mode = [] {
    const char* e = getenv("DSVT_RESID_XS");
    return e ? atoi(e) : 0;
  }();
  return mode != 0;
}

int gemm_variant_for(const GemmParams& p, int dtype, int epi, int out_f32) {
  if (dtype != 0) return 0;
  if (epi == EPI_PATCH) return 1;
  if (p.sk_part && !p.row_scale && gemm_sk_ok(p, epi, out_f32) &&
      (g_gemm_variant == 40 || (g_gemm_variant == 0 && sk_auto(epi))))
    return 40;
  // forced stream-K on an ineligible shape, or 41 (auto + tail split): the automatic choice
  const int gv = (g_gemm_variant == 40 || g_gemm_variant == 41 || g_gemm_variant == 50) ? 0 : g_gemm_variant;
  // inside a dsvt_set_gemm_skinny scope (the CLS-only tail's and the DINO head's few-row GEMMs,
  // chosen by call site so that a batch split over streams picks the same kernel as the whole
  // batch): the K-split skinny kernel (variant 50 forces it where eligible) -- bench 397.7-398.7
  // vs 395.1-396.0 clips/s with the 128x128 kernel (same box, three interleaved rounds;
  // DSVT_SKINNY=0 turns the scopes off for A/B)
  static const int skinny = getenv("DSVT_SKINNY") ? atoi(getenv("DSVT_SKINNY")) : 1;
  if ((g_gemm_variant == 50 || (g_gemm_variant == 0 && skinny && g_skinny_scope)) && gemm_skinny_ok(p, epi)) return 50;
  // training fc1 (GELU with the pre-activation saved, DropPath row scales or not) and the dX of
  // fc2 through GELU': the 256x256 kernel with the branch-free training epilogue -- measured
  // 195 vs 254 us (persistent 256x128) and 215 vs 231 us at 25104 x 3072 x 768 (tools/aux_bench.py)
  if ((epi == EPI_GELU_SAVE || epi == EPI_DGELU) && (gv == 0 || gv == 20) && p.M >= 4096 && p.N % 256 == 0 &&
      gemm_8ph_ok(p, epi))
    return 20;
  // 256x256 kernel for the big N = 768 GEMMs: see the residual / N = 768 rules below
  static const int64_t min_t = getenv("DSVT_8PH_MIN_TILES") ? atoll(getenv("DSVT_8PH_MIN_TILES")) : 128;
  const bool big8 = p.M >= 4096 && ((p.M + 255) / 256) * ((p.N + 255) / 256) >= min_t;
  static const int r8 = getenv("DSVT_RESID_8PH") ? atoi(getenv("DSVT_RESID_8PH")) : 2;
  // training DropPath residual GEMMs (s[m] * bias in the epilogue) likewise
  // (the row-scaled ones are opt-in, DSVT_RESID_RS_8PH=1: 117.1 / 117.2 vs 117.4 / 117.6 train
  // clips/s on the same box -- no gain, the 128x128 kernel stays their default)
  static const int rs8 = getenv("DSVT_RESID_RS_8PH") ? atoi(getenv("DSVT_RESID_RS_8PH")) : 0;
  if (epi == EPI_RESID && p.row_scale && gemm_8ph_ok(p, epi) &&
      (gv == 20 || (gv == 0 && rs8 && r8 && big8 && (r8 >= 2 || p.K >= 2048))))
    return 20;
  if (p.row_scale)              // DropPath row scales: the 128x128 and persistent kernels only
    return (epi != EPI_RESID && p.M >= 2048 && p.N % 128 == 0 && p.K <= 1024) ? 10 : 1;
  if (gv >= 20 && gv <= 29) return gemm_8ph_ok(p, epi) ? gv : 1;
  if (gv == 33) return gemm_8ph_xs_ok(p, epi) ? 33 : gemm_8ph_ok(p, epi) ? 20 : 1;
  if (gv == 2) return (gemm_pipe_ok(p) && epi != EPI_PATCH) ? 2 : 1;
  if (epi >= EPI_GELU_SAVE) {   // training epilogues: 128x128 or the persistent kernel only
    if (gv == 1 || gv == 9 || gv == 10) return gv;
    return (p.M >= 2048 && p.N % 128 == 0 && p.K <= 1024) ? 10 : 1;
  }
  if (gv) return gv;
  // wide bias-only projections with a bf16 output (qkv, N = 2304): the 256x256 phase-interleaved
  // kernel (v20) -- measured 895 vs 828 TF/s (global crops) and 933 vs 786 (local crops)
  // fc1 + GELU likewise (728 vs 709 TF/s global crops; its epilogue uses the general store path)
  if ((epi == EPI_BIAS || epi == EPI_GELU) && !out_f32 && p.M >= 4096 && p.N >= 1024 && gemm_8ph_ok(p, epi))
    return 20;
  // fp32 residual GEMMs (N = 768: proj / temporal fc / fc2): the 256x256 kernel.  ALONE it is
  // the slower one (proj 73.6 vs 57.6 us, fc2 165 vs 138 us against the 128x128 kernel: 297
  // tiles on 256 CUs leave a 1.16-round tail), but the forward runs three backbone calls on
  // concurrent streams whose kernels fill that tail, and there its higher per-tile rate wins:
  // 379.7 / 380.0 vs 360.6 / 359.7 clips/s on the bench line (same box, two interleaved rounds;
  // DSVT_RESID_8PH = 0 -> 128x128, 1 -> only K >= 2048, 2 -> all, the default).
  // Below ~half a round of 256x256 tiles (config 4's single 2-clip call: 75 tiles) the 128x128
  // kernel's 4x more tiles win even with other streams beside it (DSVT_8PH_MIN_TILES).
  if (epi == EPI_RESID) {
    if (r8 && big8 && gemm_8ph_ok(p, epi) && (r8 >= 2 || p.K >= 2048)) return xs_auto() && gemm_8ph_xs_ok(p, epi) ? 33 : 20;
    return 1;
  }
  // N = 768 bias-only (the split residual path's proj / temporal fc, the backward's dX GEMMs):
  // the 128x128 kernel -- 43.4 vs 53.8 us (persistent 256x128) at 25104 x 768 x 768 alone;
  // DSVT_N768_8PH = 1 (A/B knob) puts them on the 256x256 kernel like the residual GEMMs.
  if (epi == EPI_BIAS && p.N < 1024) {
    static const int n8 = getenv("DSVT_N768_8PH") ? atoi(getenv("DSVT_N768_8PH")) : 1;
    if (n8 && big8 && gemm_8ph_ok(p, epi)) return 20;
    return 1;
  }
  return (p.M >= 2048 && p.N % 128 == 0 && p.K <= 1024) ? 10 : 1;
}

// Tail split (DSVT_TAIL_SPLIT=1, opt-in): a 256x256 launch whose last round of tiles is at most
// half full -- the global-crop residual GEMMs: 297 tiles = one round + 41; qkv: 891 = three
// rounds + 123 -- runs its full rounds on the 256x256 kernel and the rows of the last round on the
// 128x128 kernel (4x the tiles for the same rows: the tail round's work spread over more CUs).
// Alone it is faster (proj 72.4 -> 61.1 us, fc2 163 -> 134 us, qkv unchanged), inside the DINO
// step slower (374 vs 385 clips/s, three interleaved rounds): the three concurrent backbone
// calls already fill the tail round, and the second launch waits for the whole first one.
// Bias / plain residual epilogues only (no row scales, no aux operand); with a row map the split
// falls on a row-group boundary so the second launch's map is the first's shifted by whole groups.
// Returns the first launch's row count, 0 = no split.
static int64_t tail_split_rows(const GemmParams& p, int epi) {
  static const int on = getenv("DSVT_TAIL_SPLIT") ? atoi(getenv("DSVT_TAIL_SPLIT")) : 0;
  // variant 41 = the automatic choice with the tail split (tests, A/B on one thread)
  if (!(g_gemm_variant == 41 || (on && g_gemm_variant == 0)) || p.row_scale || p.nseg || p.sk_part ||
      !(epi == EPI_BIAS || epi == EPI_RESID))
    return 0;
  const int64_t tn = (p.N + 255) / 256, tiles = ((p.M + 255) / 256) * tn, full = tiles / 256;
  const int64_t rem = tiles - full * 256;
  if (full < 1 || rem == 0 || rem * 2 > 256) return 0;
  int64_t rows_a = (full * 256 / tn) * 256;
  const bool ident = p.rpg >= p.M && p.goff == 0;
  if (!ident) rows_a = p.rpg > 0 ? rows_a / p.rpg * p.rpg : 0;
  return (rows_a > 0 && rows_a < p.M) ? rows_a : 0;
}

hipError_t launch_gemm(const GemmParams& p, int dtype, int epi, int out_f32, hipStream_t s) {
  const int v = gemm_variant_for(p, dtype, epi, out_f32);
  if (v == 20) {
    if (const int64_t ra = tail_split_rows(p, epi)) {
      GemmParams a = p, b = p;
      a.M = ra;
      if (hipError_t e = launch_gemm_8ph(a, epi, out_f32, s)) return e;
      b.M = p.M - ra;
      b.A = (const char*)p.A + ra * p.lda * 2;
      if (p.rpg >= p.M && p.goff == 0) {            // identity map: shift the output rows
        const int64_t osz = (epi == EPI_RESID || out_f32) ? 4 : 2;
        b.out = (char*)p.out + ra * p.ldo * osz;
        if (p.resid) b.resid = p.resid + ra * p.ldo;
        b.rpg = b.M;
      } else {                                      // row groups: shift the map by ra / rpg groups
        b.goff = p.goff + (ra / p.rpg) * p.gstride;
      }
      return launch_t<bf16_t>(b, epi, out_f32, s);
    }
  }
  if (v == 40) return launch_gemm_sk(p, epi, out_f32, s);
  if (v == 50) return launch_gemm_skinny(p, epi, out_f32, s);
  if (v == 2) return launch_pipe(p, epi, out_f32, s);
  if (v >= 2) return launch_gemm_big(p, v, epi, out_f32, s);
  if (v == 1) return launch_t<bf16_t>(p, epi, out_f32, s);
  return launch_t<float>(p, epi, out_f32, s);
}

}  // namespace dsvt
