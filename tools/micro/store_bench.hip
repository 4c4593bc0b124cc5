// Store-pattern microbenchmark: time writing a [M, N] bf16 matrix with
//  (a) coalesced rows, 16 B/lane (1 KB contiguous per wave instruction)
//  (b) the MFMA-fragment pattern: lane (r16, g) writes 8 B at row r16, cols 16j + 4g (16 rows x 32 B)
//  (c) same as (b) but 16 B per lane (16 rows x 64 B)
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

__global__ void coalesced(uint4* out, int64_t n16) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n16; i += (int64_t)gridDim.x * blockDim.x)
    out[i] = make_uint4(i, i, i, i);
}
// one workgroup = 256 threads = 4 waves = a 128x128 bf16 tile (like a GEMM tile epilogue)
template <int W>
__global__ void frag(unsigned short* out, int64_t M, int64_t N) {
  const int tilesN = N / 128;
  const int64_t m0 = (int64_t)(blockIdx.x / tilesN) * 128, n0 = (int64_t)(blockIdx.x % tilesN) * 128;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, r16 = lane & 15, g = lane >> 4;
  const int wm = wave >> 1, wn = wave & 1;
  for (int i = 0; i < 4; ++i)
    for (int j = 0; j < 4 / (W / 8); ++j) {
      const int64_t m = m0 + wm * 64 + i * 16 + r16;
      const int64_t n = n0 + wn * 64 + j * 16 * (W / 8) + (W / 2) * g;
      if (W == 8) *reinterpret_cast<uint2*>(out + m * N + n) = make_uint2(m, n);
      else *reinterpret_cast<uint4*>(out + m * N + n) = make_uint4(m, n, m, n);
    }
}

int main() {
  const int64_t M = 25104, N = 2304;
  unsigned short* buf;
  hipMalloc(&buf, M * N * 2);
  hipEvent_t e0, e1;
  hipEventCreate(&e0); hipEventCreate(&e1);
  float ms;
  for (int rep = 0; rep < 2; ++rep) {
    hipEventRecord(e0);
    for (int k = 0; k < 10; ++k) coalesced<<<4096, 256>>>((uint4*)buf, M * N * 2 / 16);
    hipEventRecord(e1); hipEventSynchronize(e1); hipEventElapsedTime(&ms, e0, e1);
    printf("coalesced 16B/lane: %.1f us  %.2f TB/s\n", ms * 100, M * N * 2 / (ms / 10 * 1e-3) / 1e12);
    const int tiles = (M / 128) * (N / 128);
    hipEventRecord(e0);
    for (int k = 0; k < 10; ++k) frag<8><<<tiles, 256>>>(buf, M, N);
    hipEventRecord(e1); hipEventSynchronize(e1); hipEventElapsedTime(&ms, e0, e1);
    printf("fragment 8B/lane (16 rows x 32 B): %.1f us  %.2f TB/s\n", ms * 100, (M / 128 * 128) * N * 2 / (ms / 10 * 1e-3) / 1e12);
    hipEventRecord(e0);
    for (int k = 0; k < 10; ++k) frag<16><<<tiles, 256>>>(buf, M, N);
    hipEventRecord(e1); hipEventSynchronize(e1); hipEventElapsedTime(&ms, e0, e1);
    printf("fragment 16B/lane (16 rows x 64 B): %.1f us  %.2f TB/s\n", ms * 100, (M / 128 * 128) * N * 2 / (ms / 10 * 1e-3) / 1e12);
  }
  return 0;
}
