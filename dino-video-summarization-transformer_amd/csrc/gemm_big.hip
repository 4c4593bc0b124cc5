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
#include "common.h"

namespace dsvt {

constexpr int BIG_NST = 4;     // LDS stages
constexpr int BIG_ROWB = 64;   // bytes per tile row per stage (32 bf16)

__device__ __forceinline__ int swz64(int r) { return (0x78 >> (2 * ((r >> 2) & 3))) & 3; }

// s_waitcnt vmcnt(n) leaving lgkmcnt / expcnt untouched (gfx9 encoding; n < 16)
template <int N>
__device__ __forceinline__ void wait_vm() {
  static_assert(N >= 0 && N < 16, "vmcnt immediate");
  __builtin_amdgcn_s_waitcnt(0x0F70 | N);
}

template <int BM, int BN, int WM, int WN, int EPI, bool OUT_F32>
__global__ __launch_bounds__(512) void gemm_big_kernel(GemmParams p) {
  constexpr int A_BYTES = BM * BIG_ROWB, B_BYTES = BN * BIG_ROWB, ST_BYTES = A_BYTES + B_BYTES;
  constexpr int WTM = BM / WM, WTN = BN / WN, MI = WTM / 16, NJ = WTN / 16;
  constexpr int A_PIECES = A_BYTES / 1024 / 8, B_PIECES = B_BYTES / 1024 / 8;  // per wave per stage
  constexpr int PER_STAGE = A_PIECES + B_PIECES;
  static_assert(WM * WN == 8, "8 waves");
  static_assert(3 * PER_STAGE < 16, "vmcnt range");
  __shared__ __attribute__((aligned(16))) char smem[BIG_NST * ST_BYTES];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
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
    char* st_ = smem + ((kt) % BIG_NST) * ST_BYTES;                                               \
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
  const int frag_off = r16 * BIG_ROWB + ((g ^ swz64(r16)) << 4);
  const int a_base = wm * WTM * BIG_ROWB + frag_off;
  const int b_base = A_BYTES + wn * WTN * BIG_ROWB + frag_off;

  DSVT_ISSUE(0);
  if (nk > 1) DSVT_ISSUE(1);
  if (nk > 2) DSVT_ISSUE(2);
  for (int kt = 0; kt < nk; ++kt) {
    const int rem = nk - 1 - kt;
    if (rem >= 2) wait_vm<2 * PER_STAGE>();
    else if (rem == 1) wait_vm<PER_STAGE>();
    else wait_vm<0>();
    asm volatile("" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (kt + 3 < nk) DSVT_ISSUE(kt + 3);
    const char* st = smem + (kt % BIG_NST) * ST_BYTES;
    sv8 a[MI], b[NJ];
#pragma unroll
    for (int i = 0; i < MI; ++i) a[i] = *reinterpret_cast<const sv8*>(st + a_base + i * 16 * BIG_ROWB);
#pragma unroll
    for (int j = 0; j < NJ; ++j) b[j] = *reinterpret_cast<const sv8*>(st + b_base + j * 16 * BIG_ROWB);
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int j = 0; j < NJ; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b[j], a[i], acc[i][j], 0, 0, 0);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // this stage's LDS reads retired (WAR)
  }
#undef DSVT_ISSUE

  // ---- epilogue: lane holds C[m = .. + r16][n = .. + 4g + 0..3]
#pragma unroll
  for (int i = 0; i < MI; ++i) {
    const int64_t m = m0 + wm * WTM + i * 16 + r16;
    if (m >= p.M) continue;
    const int64_t orow = map_row(m, p.rpg, p.gstride, p.goff);
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int64_t n = n0 + wn * WTN + j * 16 + 4 * g;
      if (n >= p.N) continue;
      float v0 = acc[i][j][0], v1 = acc[i][j][1], v2 = acc[i][j][2], v3 = acc[i][j][3];
      if (p.bias) {
        const float4 bb = *reinterpret_cast<const float4*>(p.bias + n);
        v0 += bb.x; v1 += bb.y; v2 += bb.z; v3 += bb.w;
      }
      if constexpr (EPI == EPI_GELU) {
        v0 = gelu_erf(v0); v1 = gelu_erf(v1); v2 = gelu_erf(v2); v3 = gelu_erf(v3);
      }
      if constexpr (EPI == EPI_BIAS || EPI == EPI_GELU) {
        if constexpr (OUT_F32)
          store4((float*)p.out + orow * p.ldo + n, v0, v1, v2, v3);
        else
          store4((bf16_t*)p.out + orow * p.ldo + n, v0, v1, v2, v3);
      } else if constexpr (EPI == EPI_RESID) {
        float4* xo = reinterpret_cast<float4*>((float*)p.out + orow * p.ldo + n);
        float4 x = *xo;
        x.x += v0; x.y += v1; x.z += v2; x.w += v3;
        *xo = x;
      } else {  // EPI_PATCH
        const int64_t rrw = m % p.rpg;
        const int64_t np = rrw / p.T, t = rrw % p.T;
        const float4 pe = *reinterpret_cast<const float4*>(p.pos + (1 + (int64_t)p.pidx[np]) * p.N + n);
        v0 += pe.x; v1 += pe.y; v2 += pe.z; v3 += pe.w;
        if (p.temb) {
          const float4 te = *reinterpret_cast<const float4*>(p.temb + (int64_t)p.tidx[t] * p.N + n);
          v0 += te.x; v1 += te.y; v2 += te.z; v3 += te.w;
        }
        store4((float*)p.out + orow * p.ldo + n, v0, v1, v2, v3);
      }
    }
  }
}

template <int BM, int BN, int WM, int WN>
static hipError_t launch_big_t(const GemmParams& p, int epi, int out_f32, hipStream_t s) {
  const int64_t tiles = ((p.M + BM - 1) / BM) * ((p.N + BN - 1) / BN);
  dim3 grid((unsigned)tiles), block(512);
  switch (epi) {
    case EPI_BIAS:
      if (out_f32) gemm_big_kernel<BM, BN, WM, WN, EPI_BIAS, true><<<grid, block, 0, s>>>(p);
      else gemm_big_kernel<BM, BN, WM, WN, EPI_BIAS, false><<<grid, block, 0, s>>>(p);
      break;
    case EPI_GELU:
      if (out_f32) gemm_big_kernel<BM, BN, WM, WN, EPI_GELU, true><<<grid, block, 0, s>>>(p);
      else gemm_big_kernel<BM, BN, WM, WN, EPI_GELU, false><<<grid, block, 0, s>>>(p);
      break;
    case EPI_RESID: gemm_big_kernel<BM, BN, WM, WN, EPI_RESID, true><<<grid, block, 0, s>>>(p); break;
    case EPI_PATCH: gemm_big_kernel<BM, BN, WM, WN, EPI_PATCH, true><<<grid, block, 0, s>>>(p); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

hipError_t launch_gemm_big(const GemmParams& p, int variant, int epi, int out_f32, hipStream_t s) {
  if (variant == 2) return launch_big_t<256, 256, 2, 4>(p, epi, out_f32, s);
  return launch_big_t<256, 128, 4, 2>(p, epi, out_f32, s);
}

}  // namespace dsvt
