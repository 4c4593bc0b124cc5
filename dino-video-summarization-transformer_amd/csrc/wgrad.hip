// Weight gradients of every nn.Linear on the student's backward path (loss.backward(),
// train_ssl.py:538): G[n, k] (+)= sum_m dY[m, n] * X[m, k], bf16 operands, fp32 result.
//
// Both operands are read along their ROWS (m), the reduction dimension: a tile of dY rows
// [64 m][128 n] and of X rows [64 m][128 k] is staged by LDS-DMA exactly as it lies in HBM
// (256-byte rows, 16-byte chunks XOR-swizzled by ((row & 3) << 2) | ((row >> 2) & 3) on the
// source address), and both MFMA operands come out of LDS by ds_read_b64_tr_b16 transposed
// reads: lane (r16, g) of a 16-lane group gets one column of 4 consecutive m-rows, twice (rows
// 4g.. and 16 + 4g.. of a 32-row block), i.e. the same permuted 8 m-values for the X fragment
// (A operand: rows = k) and the dY fragment (B operand: columns = n), so the products pair up.
// The output lane then holds G[n = col][k = 4g .. 4g + 3]: one 16-byte store.
//
// 128 x 128 output tile per 256-thread workgroup (2 x 2 waves of 64 x 64), 2-stage LDS ring
// (64 KiB: 2 workgroups per CU).  M is split over gridDim.y slices (a few hundred workgroups
// for the 768..3072-wide weights); each slice writes an fp32 partial tile and a second kernel
// sums the slices in a fixed order into G (deterministic; `accumulate` adds to G's old value).
// Rows past M are zeroed in the X tile of the last step (the product then contributes 0).
#include "common.h"

namespace dsvt {

namespace {

constexpr int WG_BM = 64;                  // m rows per step
constexpr int WG_TN = 128, WG_TK = 128;    // output tile: n x k
constexpr int WG_ROWB = 256;               // bytes per staged row (128 bf16)
constexpr int WG_TILE = WG_BM * WG_ROWB;   // 16 KiB per operand per stage

__device__ __forceinline__ int wg_swz(int row) { return ((row & 3) << 2) | ((row >> 2) & 3); }

// byte offset of (row, column c) in a staged [64][128] tile (c % 4 == 0 for the 8-byte reads)
__device__ __forceinline__ int wg_off(int row, int c) { return row * WG_ROWB + (((c >> 3) ^ wg_swz(row)) << 4) + ((c & 7) << 1); }

typedef __attribute__((address_space(3))) sv4* LDS4;

}  // namespace

struct WgradParams {
  const bf16_t* dy; int64_t ldy;           // [M, N]
  const bf16_t* x; int64_t ldx;            // [M, K]
  float* out; int64_t ldo;                 // slices > 1: partials [S][N][K] (ldo = K); else G
  int64_t M, N, K;
  int accumulate;                          // single slice: G += (else G =)
};

__global__ __launch_bounds__(256, 2) void wgrad_kernel(WgradParams p) {
  __shared__ __attribute__((aligned(16))) char smem[2][2 * WG_TILE];   // [stage][dY | X]
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r16 = lane & 15, g = lane >> 4;
  const int wk = wave >> 1, wn = wave & 1;      // wave's 64 x 64 block: k rows wk*64.., n cols wn*64..
  const int tilesK = (int)((p.K + WG_TK - 1) / WG_TK);
  const int64_t n0 = (int64_t)(blockIdx.x / tilesK) * WG_TN, k0 = (int64_t)(blockIdx.x % tilesK) * WG_TK;
  const int64_t steps = (p.M + WG_BM - 1) / WG_BM, S = gridDim.y, sl = blockIdx.y;
  const int64_t s_begin = sl * steps / S, s_end = (sl + 1) * steps / S;

  // DMA roles: a wave-instruction moves 4 rows x 256 B; lane -> (row in 4, physical chunk)
  const int prow = lane >> 4, pch = lane & 15;
  auto stage = [&](int st, int64_t step) {
    const int64_t m0 = step * WG_BM;
#pragma unroll
    for (int i = 0; i < 4; ++i) {                  // 16 pieces per operand, 4 per wave
      const int row = (wave * 4 + i) * 4 + prow;
      int64_t m = m0 + row;
      m = m < p.M ? m : p.M - 1;                   // clamped; the X rows are zeroed below
      const int lc = pch ^ wg_swz(row);            // logical chunk landing in physical chunk pch
      int64_t cn = n0 + lc * 8, ck = k0 + lc * 8;  // column chunks past N / K re-read the last one
      cn = cn < p.N ? cn : p.N - 8;
      ck = ck < p.K ? ck : p.K - 8;
      __builtin_amdgcn_global_load_lds((const void*)(p.dy + m * p.ldy + cn),
                                       LDS_PTR(smem[st] + (wave * 4 + i) * 1024), 16, 0, 0);
      __builtin_amdgcn_global_load_lds((const void*)(p.x + m * p.ldx + ck),
                                       LDS_PTR(smem[st] + WG_TILE + (wave * 4 + i) * 1024), 16, 0, 0);
    }
  };

  fv4 acc[4][4];   // [k fragment][n fragment]
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = fv4{0.f, 0.f, 0.f, 0.f};

  if (s_begin < s_end) stage(0, s_begin);
  for (int64_t step = s_begin; step < s_end; ++step) {
    const int st = (int)((step - s_begin) & 1);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (step + 1 < s_end) stage(st ^ 1, step + 1);
    if ((step + 1) * WG_BM > p.M) {                 // tail step: zero the X rows past M
      const int r0 = (int)(p.M - step * WG_BM);
      for (int e = tid; e < (WG_BM - r0) * 16; e += 256) {
        const int row = r0 + e / 16;
        *reinterpret_cast<uint4*>(smem[st] + WG_TILE + row * WG_ROWB + (e % 16) * 16) = make_uint4(0, 0, 0, 0);
      }
      __syncthreads();
    }
    const char* ty = smem[st];
    const char* tx = smem[st] + WG_TILE;
#pragma unroll
    for (int kb = 0; kb < WG_BM / 32; ++kb) {
      // lane (r16, g) supplies row 4g + (r16 >> 2) (+16) and columns 4 (r16 & 3) of each 16-column block
      const int ra = kb * 32 + 4 * g + (r16 >> 2), rb = ra + 16;
      const int cq = 4 * (r16 & 3);
      sv8 fa[4], fb[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int c = wk * 64 + i * 16 + cq;
        const sv4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS4)(tx + wg_off(ra, c)));
        const sv4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS4)(tx + wg_off(rb, c)));
        fa[i] = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int c = wn * 64 + j * 16 + cq;
        const sv4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS4)(ty + wg_off(ra, c)));
        const sv4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS4)(ty + wg_off(rb, c)));
        fb[j] = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
      }
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i], fb[j], acc[i][j], 0, 0, 0);
    }
  }

  // lane holds G[n = n0 + wn*64 + 16 j + r16][k = k0 + wk*64 + 16 i + 4 g .. + 3]
  mfma_result_fence();
  float* out = p.out + (S > 1 ? sl * p.N * p.ldo : 0);
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int64_t n = n0 + wn * 64 + j * 16 + r16;
    if (n >= p.N) continue;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int64_t k = k0 + wk * 64 + i * 16 + 4 * g;
      if (k >= p.K) continue;
      float4* o = reinterpret_cast<float4*>(out + n * p.ldo + k);
      const fv4 a = acc[i][j];
      if (S == 1 && p.accumulate) {
        const float4 old = *o;
        *o = make_float4(old.x + a[0], old.y + a[1], old.z + a[2], old.w + a[3]);
      } else {
        *o = make_float4(a[0], a[1], a[2], a[3]);
      }
    }
  }
}

// G (+)= sum over the S slices of the partials, in slice order (float4 per thread)
__global__ __launch_bounds__(256) void wgrad_reduce_kernel(const float* __restrict__ part, int64_t S, int64_t n4,
                                                           float* __restrict__ G, int accumulate) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n4; i += (int64_t)gridDim.x * 256) {
    float4 a = accumulate ? reinterpret_cast<const float4*>(G)[i] : make_float4(0.f, 0.f, 0.f, 0.f);
    for (int64_t s = 0; s < S; ++s) {
      const float4 v = reinterpret_cast<const float4*>(part)[s * n4 + i];
      a.x += v.x; a.y += v.y; a.z += v.z; a.w += v.w;
    }
    reinterpret_cast<float4*>(G)[i] = a;
  }
}

// M-slices: enough workgroups for 2 per CU over the output tiles, each slice >= 8 steps
int64_t wgrad_slices(int64_t M, int64_t N, int64_t K) {
  const int64_t tiles = ((N + WG_TN - 1) / WG_TN) * ((K + WG_TK - 1) / WG_TK);
  const int64_t steps = (M + WG_BM - 1) / WG_BM;
  int64_t S = (512 + tiles - 1) / tiles;
  if (S > steps / 8) S = steps / 8;
  return S < 1 ? 1 : S;
}

hipError_t launch_wgrad(const bf16_t* dy, int64_t ldy, const bf16_t* x, int64_t ldx, float* G, int64_t M, int64_t N,
                        int64_t K, int accumulate, float* partial, hipStream_t s) {
  const int64_t S = wgrad_slices(M, N, K);
  WgradParams p{dy, ldy, x, ldx, S > 1 ? partial : G, K, M, N, K, accumulate};
  const int64_t tiles = ((N + WG_TN - 1) / WG_TN) * ((K + WG_TK - 1) / WG_TK);
  wgrad_kernel<<<dim3((unsigned)tiles, (unsigned)S), 256, 0, s>>>(p);
  if (S > 1) {
    const int64_t n4 = N * K / 4;
    unsigned blocks = (unsigned)((n4 + 255) / 256);
    if (blocks > 2048) blocks = 2048;
    wgrad_reduce_kernel<<<blocks, 256, 0, s>>>(partial, S, n4, G, accumulate);
  }
  return hipGetLastError();
}

}  // namespace dsvt
