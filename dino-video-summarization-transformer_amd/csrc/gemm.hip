// MFMA GEMM with fused epilogues for every nn.Linear / Conv2d(k=s=16) on the hot path.
//
//   out = A[M,K] . W[N,K]^T  (+ bias, GELU, residual add into the fp32 token tensor X,
//                             or the patch-embed pos/time-embed add)
//
// Tiling (gfx950): 128x128 output tile per 256-thread workgroup (4 waves as 2x2, each a
// 64x64 sub-tile = 4x4 MFMA 16x16 tiles); the bf16 residual epilogue also as 160x128 (MI = 5
// fragments per wave along M: variant 3, config 4's N = 768 GEMMs, one round of 240 tiles where
// 128x128 needs 294 = a 1.15-round grid).  K advances 128 BYTES per stage (64 bf16 or
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
#include "gemm_epi.h"

namespace dsvt {

constexpr int BM = 128, BN = 128, BKB = 128;  // tile rows, tile cols, K bytes per stage
constexpr int TILE_BYTES = BM * BKB;           // 16 KB per operand per stage
constexpr int STAGE_BYTES = 2 * TILE_BYTES;    // A + W

__device__ __forceinline__ int swz(int r) { return (r >> 1) & 7; }

// Issue the global->LDS copy of one [32 NP rows][128 bytes] tile (4 NP x 1 KB pieces, NP per
// wave).  Rows beyond `rows` re-read the last row (results masked in the epilogue).
template <int NP = 4>
__device__ __forceinline__ void stage_tile(const char* __restrict__ g, int64_t ld_bytes,
                                           int64_t row0, int64_t rows, int64_t kbyte0,
                                           char* lds_tile, int wave, int lane) {
#pragma unroll
  for (int i = 0; i < NP; ++i) {
    const int piece = wave * NP + i;
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
  template <int MI>
  __device__ __forceinline__ static void run(const char* At, const char* Wt, fv4 (&acc)[MI][4],
                                             int wm, int wn, int lane) {
    const int r16 = lane & 15, g = lane >> 4;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      sv8 a[MI], b[4];
#pragma unroll
      for (int i = 0; i < MI; ++i)
        a[i] = *reinterpret_cast<const sv8*>(lds_chunk(At, wm * 16 * MI + i * 16 + r16, ks * 4 + g));
#pragma unroll
      for (int j = 0; j < 4; ++j)
        b[j] = *reinterpret_cast<const sv8*>(lds_chunk(Wt, wn * 64 + j * 16 + r16, ks * 4 + g));
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b[j], a[i], acc[i][j], 0, 0, 0);
    }
  }
};

template <> struct TileMMA<float> {
  template <int MI>
  __device__ __forceinline__ static void run(const char* At, const char* Wt, fv4 (&acc)[MI][4],
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

// The fp32 residual tile of one wave (full tiles): 4 MI float4 loads, issued by gemm_kernel two
// K steps before the end of its main loop (PREF) so their latency runs under the last MFMAs.
template <int MI>
__device__ __forceinline__ void resid_load(const GemmParams& p, int64_t m0, int64_t n0, int wm, int wn, int lane,
                                           float4 (&add)[MI][4]) {
  const int r16 = lane & 15, g = lane >> 4;
#pragma unroll
  for (int i = 0; i < MI; ++i) {
    const int64_t orow = map_row(m0 + wm * 16 * MI + i * 16 + r16, p.rpg, p.gstride, p.goff);
#pragma unroll
    for (int j = 0; j < 4; ++j)
      add[i][j] = *reinterpret_cast<const float4*>(resid_src(p) + orow * p.ldo + n0 + wn * 64 + j * 16 + 4 * g);
  }
}

template <typename T, int EPI, bool OUT_F32, bool CHECK, bool PRE = false, int MI = 4>
__device__ __forceinline__ void epilogue_128(const GemmParams& p, fv4 (&acc)[MI][4], int64_t m0, int64_t n0, int wm,
                                             int wn, int lane, const float4 (*pre)[4] = nullptr) {
  const int r16 = lane & 15, g = lane >> 4;
  int64_t orow[MI];
  bool vrow[MI];
#pragma unroll
  for (int i = 0; i < MI; ++i) {
    const int64_t m = m0 + wm * 16 * MI + i * 16 + r16;
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
  float4 add[MI][4];                   // residual / embedding addend per fragment
  if constexpr (PRE) {
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) add[i][j] = pre[i][j];
  } else if constexpr (EPI == EPI_RESID || EPI == EPI_PATCH) {
#pragma unroll
    for (int i = 0; i < MI; ++i) {
      const int64_t m = m0 + wm * 16 * MI + i * 16 + r16;
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
  float rsc[MI];                       // DropPath row scales (EPI_BIAS / EPI_GELU_SAVE: the output;
#pragma unroll                         // EPI_RESID: the bias term only)
  for (int i = 0; i < MI; ++i) {
    rsc[i] = 1.0f;
    if constexpr (EPI == EPI_BIAS || EPI == EPI_GELU_SAVE || EPI == EPI_RESID)
      if (p.row_scale) rsc[i] = row_scale_of(p, m0 + wm * 16 * MI + i * 16 + r16);
  }
#pragma unroll
  for (int i = 0; i < MI; ++i) {
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
      if constexpr (EPI == EPI_GELU_SAVE) {   // aux = GELU'(pre): the DGELU epilogue's multiplier
        store4((T*)p.aux + orow[i] * p.ld_aux + n, gelu_erf_grad(v0), gelu_erf_grad(v1), gelu_erf_grad(v2),
               gelu_erf_grad(v3));
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
        v0 = acc[i][j][0] * pre[0]; v1 = acc[i][j][1] * pre[1];
        v2 = acc[i][j][2] * pre[2]; v3 = acc[i][j][3] * pre[3];
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

template <int N>
__device__ __forceinline__ void gk_vmwait() {
  static_assert(N >= 0 && N < 64, "vmcnt immediate");
  __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | 0x0F70);
}

// STATS (EPI_RESID, bf16, N % 128 == 0; dsvt_gemm_resid_stats_fwd): the residual epilogue that
// also writes the updated rows' bf16 copy and LayerNorm partials (gemm_epi.h resid_stats_rows:
// one partial per 64-column wave slab)
template <typename T, int EPI, bool OUT_F32, bool PREF = false, int MI = 4, bool STATS = false>
__global__ __launch_bounds__(256, MI == 4 ? 2 : 1) void gemm_kernel(GemmParams p) {
  constexpr int BMv = 32 * MI;                       // tile rows
  constexpr int A_BYTES = BMv * BKB, SBYTES = A_BYTES + TILE_BYTES;
  // 160x128 (one workgroup per CU): a 3-stage ring, loads two K steps ahead; 128x128: 2 stages
  // (two workgroups per CU hide each other's waits)
  constexpr int NST = MI == 5 ? 3 : 2;
  constexpr int LPS = MI + 4;                        // LDS-DMA instructions per wave per stage
  __shared__ __attribute__((aligned(16))) char smem[NST * SBYTES];
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 1, wn = wave & 1;

  // XCD-aware bijective remap: consecutive workgroup ids of one XCD walk the N-tiles of
  // one M-tile (blocks b and b+8 share an XCD under round-robin dispatch).
  const int tilesN = (int)((p.N + BN - 1) / BN);
  const int nwg = gridDim.x, orig = blockIdx.x, xcd = orig & 7, q = nwg >> 3, r = nwg & 7;
  const int wg = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (orig >> 3);
  const int64_t m0 = (int64_t)(wg / tilesN) * BMv;
  const int64_t n0 = (int64_t)(wg % tilesN) * BN;

  const char* A = (const char*)p.A;
  const char* W = (const char*)p.W;
  const int64_t lda_b = p.lda * (int64_t)sizeof(T), ldw_b = p.ldw * (int64_t)sizeof(T);
  const int nk = (int)((p.K * (int64_t)sizeof(T)) / BKB);

  fv4 acc[MI][4];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = fv4{0.f, 0.f, 0.f, 0.f};

  auto stage_k = [&](int k, char* buf) {
    stage_tile<MI>(A, lda_b, m0, p.M, (int64_t)k * BKB, buf, wave, lane);
    stage_tile(W, ldw_b, n0, p.N, (int64_t)k * BKB, buf + A_BYTES, wave, lane);
  };
  if constexpr (NST == 3) {
    const bool full3 = m0 + BMv <= p.M && n0 + BN <= p.N;
    const bool peel3 = PREF && full3 && nk >= 2;
    const int nmain3 = peel3 ? nk - 2 : nk;
    stage_k(0, smem);
    if (nk > 1) {
      stage_k(1, smem + SBYTES);
      gk_vmwait<LPS>();
    } else {
      gk_vmwait<0>();
    }
    __syncthreads();
    // at the top of step kt its stage has landed for every wave; stage kt + 2 goes into the slot
    // step kt - 1 read (released by that step's barrier)
    for (int kt = 0; kt < nmain3; ++kt) {
      char* cur = smem + (kt % 3) * SBYTES;
      if (kt + 2 < nk) stage_k(kt + 2, smem + ((kt + 2) % 3) * SBYTES);
      TileMMA<T>::run(cur, cur + A_BYTES, acc, wm, wn, lane);
      if (kt + 2 < nk) gk_vmwait<LPS>();           // stage kt + 1 landed, kt + 2 in flight
      else gk_vmwait<0>();
      __syncthreads();
    }
    if constexpr (PREF) {
      if (peel3) {                                 // stages nk - 2 (landed) and nk - 1 (issued)
        char* cur = smem + ((nk - 2) % 3) * SBYTES;
        char* nxt = smem + ((nk - 1) % 3) * SBYTES;
        __builtin_amdgcn_sched_barrier(0);
        float4 xpre[MI][4];
        resid_load(p, m0, n0, wm, wn, lane, xpre);
        __builtin_amdgcn_sched_barrier(0);
        TileMMA<T>::run(cur, cur + A_BYTES, acc, wm, wn, lane);
        gk_vmwait<4 * MI>();                       // stage nk - 1, not the residual loads
        __syncthreads();
        TileMMA<T>::run(nxt, nxt + A_BYTES, acc, wm, wn, lane);
        mfma_result_fence();
        epilogue_128<T, EPI, OUT_F32, false, true, MI>(p, acc, m0, n0, wm, wn, lane, xpre);
        return;
      }
    }
    mfma_result_fence();
    if (full3) epilogue_128<T, EPI, OUT_F32, false, false, MI>(p, acc, m0, n0, wm, wn, lane);
    else epilogue_128<T, EPI, OUT_F32, true, false, MI>(p, acc, m0, n0, wm, wn, lane);
    return;
  }

  stage_k(0, smem);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  // PREF (fp32 residual, full tiles): the last two K steps are peeled; the residual tile's 16
  // loads are issued right after the last stage's loads, and that step waits with vmcnt(16) --
  // for the stage, not for them -- so their latency runs under the last two steps' MFMAs.
  const bool full = m0 + BMv <= p.M && n0 + BN <= p.N;
  const bool peel = PREF && !STATS && full && nk >= 2;
  const int nmain = peel ? nk - 2 : nk;
  for (int kt = 0; kt < nmain; ++kt) {
    char* cur = smem + (kt & 1) * SBYTES;
    if (kt + 1 < nk) {
      char* nxt = smem + ((kt + 1) & 1) * SBYTES;
      stage_tile<MI>(A, lda_b, m0, p.M, (int64_t)(kt + 1) * BKB, nxt, wave, lane);
      stage_tile(W, ldw_b, n0, p.N, (int64_t)(kt + 1) * BKB, nxt + A_BYTES, wave, lane);
    }
    TileMMA<T>::run(cur, cur + A_BYTES, acc, wm, wn, lane);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }
  if constexpr (PREF) {
    if (peel) {
      char* cur = smem + ((nk - 2) & 1) * SBYTES;
      char* nxt = smem + ((nk - 1) & 1) * SBYTES;
      stage_tile<MI>(A, lda_b, m0, p.M, (int64_t)(nk - 1) * BKB, nxt, wave, lane);
      stage_tile(W, ldw_b, n0, p.N, (int64_t)(nk - 1) * BKB, nxt + A_BYTES, wave, lane);
      __builtin_amdgcn_sched_barrier(0);
      float4 xpre[MI][4];
      resid_load(p, m0, n0, wm, wn, lane, xpre);
      __builtin_amdgcn_sched_barrier(0);
      TileMMA<T>::run(cur, cur + A_BYTES, acc, wm, wn, lane);
      if constexpr (MI == 4) asm volatile("s_waitcnt vmcnt(16)" ::: "memory");   // the residual loads
      else asm volatile("s_waitcnt vmcnt(20)" ::: "memory");
      __syncthreads();
      TileMMA<T>::run(nxt, nxt + A_BYTES, acc, wm, wn, lane);
      mfma_result_fence();
      epilogue_128<T, EPI, OUT_F32, false, true, MI>(p, acc, m0, n0, wm, wn, lane, xpre);
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
  if constexpr (STATS) {
    static_assert(EPI == EPI_RESID && MI == 4, "the stats epilogue: residual, 64-row wave tiles");
    const int g = lane >> 4;
    float4 b4[4];
    bias_frag4(p.bias, n0 + wn * 64, g, b4);          // N % 128 == 0: every column valid
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        acc[i][j][0] += b4[j].x; acc[i][j][1] += b4[j].y; acc[i][j][2] += b4[j].z; acc[i][j][3] += b4[j].w;
      }
    epilogue_resid_stats<MI, 4>(p, acc, m0 + wm * 16 * MI, n0 + wn * 64, lane & 15, g);
    return;
  }
  if (full) epilogue_128<T, EPI, OUT_F32, false, false, MI>(p, acc, m0, n0, wm, wn, lane);
  else epilogue_128<T, EPI, OUT_F32, true, false, MI>(p, acc, m0, n0, wm, wn, lane);
}

// 160x128 tiles: the bf16 residual epilogue only
static hipError_t launch_resid160(const GemmParams& p, int epi, hipStream_t s) {
  if (epi != EPI_RESID) return hipErrorInvalidValue;
  const int64_t tiles = ((p.M + 159) / 160) * ((p.N + BN - 1) / BN);
  gemm_kernel<bf16_t, EPI_RESID, true, true, 5><<<dim3((unsigned)tiles), dim3(256), 0, s>>>(p);
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
    case EPI_RESID:   // bf16: the instantiation with the residual-tile prefetch (PREF)
      if (sizeof(T) == 2 && p.stats_out) {
        if (p.N % 128 || p.row_scale || !p.xb_out) return hipErrorInvalidValue;
        gemm_kernel<bf16_t, EPI_RESID, true, false, 4, true><<<grid, block, 0, s>>>(p);
      } else if (sizeof(T) == 2) gemm_kernel<T, EPI_RESID, true, true><<<grid, block, 0, s>>>(p);
      else gemm_kernel<T, EPI_RESID, true><<<grid, block, 0, s>>>(p);
      break;
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

static thread_local int g_gemm_variant = 0; // 0 = auto; otherwise forced (dsvt_debug.h: tools, tests)

void set_gemm_variant(int v) { g_gemm_variant = v; }

// Kernel choice (0 = fp32 128x128, 1 = bf16 128x128, 3 = bf16 160x128 (residual epilogue), 10 = persistent staggered 256x128
// (gemm_big.hip; 11-15 its 128x64 / 64x64 instantiations), 20 = 256x256 phase-interleaved (gemm_8ph.hip), 50 = K-split skinny).
// Measured on MI355X (tools/gemm_bench.py and same-box A/Bs of the whole step).
int gemm_variant_for(const GemmParams& p, int dtype, int epi, int out_f32) {
  // the index-mapped residual epilogue (dsvt_gemm_resid_rows_fwd): the 64x64 persistent kernel
  if (p.row_idx) return (dtype == 0 && epi == EPI_RESID && p.K % 32 == 0 && !p.stats_out && !p.ln_stats) ? 12 : -1;
  if (dtype != 0) return 0;
  // K % 64 != 0 (Video Swin's C = 96 stage without K padding): only the persistent kernels step K
  // by 32 -- the 64x64 one, or the 256x128 one where a variant of that family is forced
  if (p.K % 64) {
    if (p.ln_stats || p.stats_out) return -1;
    return (g_gemm_variant >= 10 && g_gemm_variant <= 15) ? g_gemm_variant : 12;
  }
  if (epi == EPI_PATCH) return 1;
  int gv = g_gemm_variant;
  if (gv == 30 && !(!p.ln_stats && gemm_192_ok(p, epi) && (epi == EPI_RESID || !out_f32))) gv = 0;   // forced, ineligible: auto
  // DSVT_GEMM_FEW_ROWS call sites (the CLS-only tail's and the DINO head's few-row GEMMs, chosen
  // by call site so that a batch split over streams picks the same kernel as the whole batch):
  // the K-split skinny kernel (variant 50 forces it where eligible) -- bench 397.7-398.7 vs
  // 395.1-396.0 clips/s with the 128x128 kernel (same box, three interleaved rounds)
  if ((gv == 50 || (gv == 0 && p.few_rows)) && gemm_skinny_ok(p, epi)) return 50;
  if (gv == 30) return 30;
  // fp32 residual GEMMs with N % 192 == 0 (the N = 768 proj / temporal fc / fc2): the 256x192 kernel
#ifndef DSVT_RESID192
#define DSVT_RESID192 0
#endif
  if (DSVT_RESID192 && gv == 0 && !p.ln_stats && p.M >= 4096 && gemm_192_ok(p, epi))
    return 30;
  // the LayerNorm-folded A operand (dsvt_gemm_lnx_fwd): the 256x256 kernel only; the residual
  // epilogue that writes the next LayerNorm's row statistics (dsvt_gemm_resid_stats_fwd): the
  // 256x256 kernel or (DSVT_RESID_STATS_V = 1, A/B builds; forced variant 1) the 128x128 one
#ifndef DSVT_RESID_STATS_V
#define DSVT_RESID_STATS_V 20
#endif
  if (p.stats_out && (gv == 1 || (gv == 0 && DSVT_RESID_STATS_V == 1)) && p.N % 128 == 0) return 1;
  if (p.stats_out && (gv == 10 || (gv == 0 && DSVT_RESID_STATS_V == 10)) && p.N % 128 == 0) return 10;
  if (gv >= 40 && gv <= 49) return gemm_4w_ok(p, epi, out_f32) ? gv : (p.ln_stats || p.stats_out) ? 20 : 1;
  // the 4-wave 256x256 kernel (gemm_4w.hip, r06) where it takes the call: the LayerNorm-folded
  // qkv / fc1 and the plain bias / GELU GEMMs below -- tools/gemm4w_bench.py, same box: lnx qkv
  // 97.0 vs 110.8 us, lnx fc1 137.2 vs 157.5, qkv 90.7 vs 106.8, fc1 125.7 vs 140.8 (global rows);
  // fwd+loss (tools/r5_ab.sh, two interleaved rounds) 410.0 / 408.7 clips/s with the folded GEMMs on
  // it vs 405.3 / 404.8 without.  The residual + statistics GEMMs stay on the 8-wave kernel: alone
  // on par (proj + stats 76.1 vs 80.2 us, fc2 + stats 174.8 vs 173.4), in the step 397.0 / 397.6
  // with them on the 4-wave kernel -- its epilogue keeps fewer X loads in flight per CU
#ifndef DSVT_GEMM4W
#define DSVT_GEMM4W 5
#endif
  // (A/B builds: DSVT_GEMM4W is a mask -- 1 the LayerNorm-folded GEMMs, 2 the residual + statistics
  // GEMMs, 4 the plain bias / GELU GEMMs)
  const bool use4w = DSVT_GEMM4W && gv == 0 && p.M >= 4096 && gemm_4w_ok(p, epi, out_f32) &&
                     (DSVT_GEMM4W & (p.ln_stats ? 1 : p.stats_out ? 2 : 4));
  if ((p.ln_stats || p.stats_out) && use4w) return 40;
  if (p.ln_stats || p.stats_out) return 20;
  // small GEMMs -- Video Swin's stages 3-4 (M = 3136 / 784 rows: 42-300 tiles of 128x128 leave most
  // CUs idle) and its narrow stage 1-2 layers (N = 96-576): the persistent kernel with 64x64 tiles
  // (variant 12).  tools/r6_swin_gemm.sh, same box, us: stage-3 qkv 10.8 vs 14.5, fc2 13.6 vs 19.2,
  // stage-4 fc2 20.1 vs 38.8, proj 8.3 vs 12.5, stage-1 qkv 15.9 vs 23.0, fc1 17.9 vs 24.2.  Not
  // the DINO ViT's GEMMs (M >= 4096 and N >= 768) nor its head (M < 512 rows)
#ifndef DSVT_SMALL_GEMM
#define DSVT_SMALL_GEMM 1
#endif
#ifndef DSVT_SMALL_MIN_M
#define DSVT_SMALL_MIN_M 512
#endif
  if (DSVT_SMALL_GEMM && gv == 0 && !p.row_scale && p.K % 32 == 0 && p.M >= DSVT_SMALL_MIN_M && (p.M < 4096 || p.N <= 576) &&
      (epi == EPI_BIAS || epi == EPI_GELU || epi == EPI_RESID))
    return 12;
  // training fc1 (GELU with the pre-activation saved, DropPath row scales or not) and the dX of
  // fc2 through GELU': the 256x256 kernel with the branch-free training epilogue -- measured
  // 195 vs 254 us (persistent 256x128) and 215 vs 231 us at 25104 x 3072 x 768 (tools/aux_bench.py)
  if ((epi == EPI_GELU_SAVE || epi == EPI_DGELU) && (gv == 0 || gv == 20) && p.M >= 4096 && p.N % 256 == 0 &&
      gemm_8ph_ok(p, epi))
    return 20;
  // 256x256 kernel for the big N = 768 GEMMs: see the residual / N = 768 rules below
  const bool big8 = p.M >= 4096 && ((p.M + 255) / 256) * ((p.N + 255) / 256) >= 128;
  if (epi == EPI_RESID && p.row_scale && gv == 20 && gemm_8ph_ok(p, epi)) return 20;
#ifndef DSVT_RESID_RS
// the training residual GEMMs with DropPath row scales: the 256x256 kernel (20) since r05's
// K-loop drain fix and the forward's group fork (train step 140.2 / 140.8 vs 139.6 / 139.7 on
// the 128x128 kernel, 1; neutral before the fork)
#define DSVT_RESID_RS 20
#endif
  if (p.row_scale) {            // DropPath row scales: the 128x128 and persistent kernels
    if (epi == EPI_RESID && DSVT_RESID_RS == 20 && p.M >= 4096 && gemm_8ph_ok(p, epi)) return 20;
    if (epi == EPI_RESID && DSVT_RESID_RS == 3) return 3;
    return (epi != EPI_RESID && p.M >= 2048 && p.N % 128 == 0 && p.K <= 1024) ? 10 : 1;
  }
  if (gv >= 20 && gv <= 29) return gemm_8ph_ok(p, epi) ? gv : 1;
  if (epi >= EPI_GELU_SAVE) {   // training epilogues: 128x128 or the persistent kernel only
    if (gv == 1 || gv == 10) return gv;
    return (p.M >= 2048 && p.N % 128 == 0 && p.K <= 1024) ? 10 : 1;
  }
  if (gv == 3 && epi != EPI_RESID) return 1;   // 160x128: the residual epilogue only
  if (gv) return gv == 50 ? 1 : gv;   // forced skinny on a shape it does not take: 128x128
  // wide bias-only projections with a bf16 output (qkv, N = 2304): the 256x256 phase-interleaved
  // kernel (v20) -- measured 895 vs 828 TF/s (global crops) and 933 vs 786 (local crops)
  // fc1 + GELU likewise (728 vs 709 TF/s global crops; its epilogue uses the general store path)
  // ... unless the 256x256 grid ends in a short second round that the 256x192 kernel's tiles fill:
  // config 4's fc1 (M = 6274, N = 3072: 300 tiles of 256x256 -> two rounds, 400 of 256x192 -> two
  // rounds of 3/4 the tile), chosen on ceil(tiles / 256 CUs) x tile area with a 20 % margin (no
  // shape of the three-stream config-2 forward qualifies)
  if ((epi == EPI_BIAS || epi == EPI_GELU) && !out_f32 && p.M >= 4096 && p.N >= 1024 && gemm_8ph_ok(p, epi)) {
    const int64_t mt = (p.M + 255) / 256;
    const int64_t c256 = (mt * ((p.N + 255) / 256) + 255) / 256 * 256, c192 = (mt * (p.N / 192) + 255) / 256 * 192;
    if (gv == 0 && gemm_192_ok(p, epi) && c192 * 5 < c256 * 4) return 30;
    return use4w ? 40 : 20;
  }
  // fp32 residual GEMMs (N = 768: proj / temporal fc / fc2): the 256x256 kernel.  ALONE it is
  // the slower one (proj 73.6 vs 57.6 us, fc2 165 vs 138 us against the 128x128 kernel: 297
  // tiles on 256 CUs leave a 1.16-round tail), but the forward runs three backbone calls on
  // concurrent streams whose kernels fill that tail, and there its higher per-tile rate wins:
  // 379.7 / 380.0 vs 360.6 / 359.7 clips/s on the bench line (same box, two interleaved rounds).
  // Below ~half a round of 256x256 tiles (config 4's single 2-clip call: 75 tiles) the 128x128
  // kernel's 4x more tiles win even with other streams beside it.
  // Below that, 128x128 tiles -- or 160x128 where their grid is a round shorter: config 4's
  // M = 6274 (294 tiles of 128x128 = 1.15 rounds on 256 CUs -> 240 of 160x128, one round)
  if (epi == EPI_RESID) {
    if (big8 && gemm_8ph_ok(p, epi)) return 20;
    const int64_t tn = (p.N + 127) / 128;
    const int64_t c128 = (((p.M + 127) / 128) * tn + 255) / 256 * 128, c160 = (((p.M + 159) / 160) * tn + 255) / 256 * 160;
    return c160 < c128 ? 3 : 1;
  }
  // N = 768 bias-only (the backward's dX GEMMs): the 256x256 kernel on big calls
#ifndef DSVT_DX192
#define DSVT_DX192 0
#endif
  if (DSVT_DX192 && epi == EPI_BIAS && !out_f32 && big8 && gemm_192_ok(p, epi)) return 30;
  if (epi == EPI_BIAS && p.N < 1024) return (big8 && use4w) ? 40 : (big8 && gemm_8ph_ok(p, epi)) ? 20 : 1;
  return (p.M >= 2048 && p.N % 128 == 0 && p.K <= 1024) ? 10 : 1;
}

hipError_t launch_gemm(const GemmParams& p, int dtype, int epi, int out_f32, hipStream_t s) {
  const int v = gemm_variant_for(p, dtype, epi, out_f32);
  if (v < 0 || (p.row_idx && (v < 10 || v > 15))) return hipErrorInvalidValue;
  if ((p.ln_stats && v != 20 && v != 40) || (p.stats_out && v != 20 && v != 30 && v != 1 && v != 10 && v != 40))
    return hipErrorInvalidValue;
  if (v == 50) return launch_gemm_skinny(p, epi, out_f32, s);
  if (v == 3) return launch_resid160(p, epi, s);
  if (v >= 2) return launch_gemm_big(p, v, epi, out_f32, s);
  if (v == 1) return launch_t<bf16_t>(p, epi, out_f32, s);
  return launch_t<float>(p, epi, out_f32, s);
}

}  // namespace dsvt
