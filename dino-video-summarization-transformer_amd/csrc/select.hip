// Score -> frame-index selection (datasets_custom/frame_selection_loader.py:115-166, the
// "adaptive" method) and the row gather that picks the selected frames, on the device where
// the frame scores already live (dsvt/scoring.py keeps them there).
//
// Bit-exact with the reference's numpy float64 arithmetic:
//   pdf = loss / np.sum(loss)      np.sum = numpy's pairwise summation (8-way unrolled leaves of
//                                  <= 128 elements, halved at multiples of 8) per 8192-element
//                                  ufunc buffer, buffers added left to right
//   cdf = np.cumsum(pdf)           sequential
//   idx = argmin |cdf - i / N|     first index of the minimum
// then the reference's collision walk (already-taken index -> next multiple of the pre-sampling
// rate; past the end -> the previous multiple and the last frame).  The loss values are the
// float64 numbers of the scores JSON.  One workgroup: the sums and the walk are inherently
// sequential (one lane), the N arg-min scans are parallel.
#include "common.h"

namespace dsvt {

namespace {

constexpr int SEL_THREADS = 256;
constexpr int64_t NP_BUFSIZE = 8192;   // numpy ufunc buffer (np.getbufsize())

// numpy pairwise_sum for one contiguous run of n doubles (numpy/_core/src/umath/loops_utils.h.src)
// (one lane; the explicit evaluation stack lives in LDS -- no scratch)
struct PwFrame { int64_t off, n; };
__device__ double np_pairwise(const double* a, int64_t n, PwFrame* st, double* vals) {
  int sp = 0, vp = 0;
  // post-order evaluation: push (off, n); a frame with n > 128 is replaced by its two halves and
  // a marker (n = -1) that adds the two results it finds on the value stack
  st[sp++] = PwFrame{0, n};
  while (sp > 0) {
    const PwFrame f = st[--sp];
    if (f.n < 0) {
      const double r = vals[--vp];
      const double l = vals[--vp];
      vals[vp++] = l + r;
      continue;
    }
    const double* p = a + f.off;
    const int64_t m = f.n;
    if (m < 8) {
      double res = 0.0;
      for (int64_t i = 0; i < m; ++i) res += p[i];
      vals[vp++] = res;
    } else if (m <= 128) {
      double r[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) r[k] = p[k];
      int64_t i = 8;
      for (; i < m - (m % 8); i += 8) {
#pragma unroll
        for (int k = 0; k < 8; ++k) r[k] += p[i + k];
      }
      double res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
      for (; i < m; ++i) res += p[i];
      vals[vp++] = res;
    } else {
      int64_t n2 = m / 2;
      n2 -= n2 % 8;
      st[sp++] = PwFrame{0, -1};              // combine after both halves
      st[sp++] = PwFrame{f.off + n2, m - n2}; // right half evaluated second
      st[sp++] = PwFrame{f.off, n2};          // left half first
    }
  }
  return vals[0];
}

__device__ double np_sum(const double* a, int64_t n, PwFrame* st, double* vals) {
  double res = 0.0;
  for (int64_t s = 0; s < n; s += NP_BUFSIZE) {
    const int64_t m = n - s < NP_BUFSIZE ? n - s : NP_BUFSIZE;
    const double c = np_pairwise(a + s, m, st, vals);
    res = s == 0 ? c : res + c;
  }
  return res;
}

__global__ __launch_bounds__(SEL_THREADS) void select_frames_kernel(const double* loss, int64_t n, int64_t n_frames,
                                                                    int64_t n_unsampled, int64_t rate, int64_t N,
                                                                    int64_t* indices, int32_t* frame_pos, double* cdf,
                                                                    unsigned* taken) {
  __shared__ double s_best[SEL_THREADS];
  __shared__ int64_t s_idx[SEL_THREADS];
  __shared__ double s_sum;
  __shared__ PwFrame s_stack[64];
  __shared__ double s_vals[64];
  const int tid = threadIdx.x;
  const int64_t nwords = (n_unsampled + 31) / 32;
  for (int64_t w = tid; w < nwords; w += SEL_THREADS) taken[w] = 0u;
  if (tid == 0) s_sum = np_sum(loss, n, s_stack, s_vals);
  __syncthreads();
  const double S = s_sum;
  // pdf (elementwise, any order), then the sequential cumsum on one lane
  for (int64_t k = tid; k < n; k += SEL_THREADS) cdf[k] = loss[k] / S;
  __syncthreads();
  if (tid == 0) {
    double c = cdf[0];
    for (int64_t k = 1; k < n; ++k) {
      c = c + cdf[k];
      cdf[k] = c;
    }
  }
  __syncthreads();
  for (int64_t i = 0; i < N; ++i) {
    const double q = (double)i / (double)N;
    double best = __builtin_huge_val();
    int64_t bidx = INT64_MAX;
    for (int64_t k = tid; k < n; k += SEL_THREADS) {
      const double d = fabs(cdf[k] - q);
      if (d < best) { best = d; bidx = k; }      // k increases: first minimum kept
    }
    s_best[tid] = best;
    s_idx[tid] = bidx;
    __syncthreads();
    for (int o = SEL_THREADS / 2; o > 0; o >>= 1) {
      if (tid < o) {
        const double b2 = s_best[tid + o];
        const int64_t i2 = s_idx[tid + o];
        if (b2 < s_best[tid] || (b2 == s_best[tid] && i2 < s_idx[tid])) {
          s_best[tid] = b2;
          s_idx[tid] = i2;
        }
      }
      __syncthreads();
    }
    if (tid == 0) {
      const int64_t idx = s_idx[0];
      const int64_t scaled = idx * rate;
      auto is_taken = [&](int64_t v) { return (taken[v >> 5] >> (v & 31)) & 1u; };
      auto take = [&](int64_t v) { taken[v >> 5] |= 1u << (v & 31); };
      if (!is_taken(scaled)) {
        take(scaled);
        indices[i] = scaled;
        frame_pos[i] = (int32_t)idx;
      } else {
        int64_t t = scaled + rate;
        for (;;) {
          if (t < n_unsampled && !is_taken(t)) {
            take(t);
            indices[i] = t;
            frame_pos[i] = (int32_t)idx;        // the reference appends frames[idx] here
            break;
          }
          if (t >= n_unsampled) {
            take(t - rate);
            indices[i] = t - rate;
            frame_pos[i] = (int32_t)(n_frames - 1);   // frames[-1]
            break;
          }
          t += rate;
        }
      }
    }
    __syncthreads();
  }
}

// dst[r] = src[idx[r]] for rows of row_bytes bytes (16-byte pieces when aligned)
__global__ void gather_rows_kernel(const char* src, int64_t row_bytes, const int32_t* idx, int64_t rows, char* dst) {
  const int64_t r = blockIdx.y;
  const char* s = src + (int64_t)idx[r] * row_bytes;
  char* d = dst + r * row_bytes;
  if ((row_bytes & 15) == 0 && (((uintptr_t)src | (uintptr_t)dst) & 15) == 0) {
    const int64_t n16 = row_bytes >> 4;
    for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < n16; k += (int64_t)gridDim.x * blockDim.x)
      reinterpret_cast<uint4*>(d)[k] = reinterpret_cast<const uint4*>(s)[k];
  } else {
    for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < row_bytes; k += (int64_t)gridDim.x * blockDim.x)
      d[k] = s[k];
  }
}

}  // namespace

int64_t select_frames_ws_bytes(int64_t n, int64_t n_unsampled) {
  return ((n * 8 + 255) / 256) * 256 + (((n_unsampled + 31) / 32) * 4 + 255) / 256 * 256;
}

hipError_t launch_select_frames(const double* loss, int64_t n, int64_t n_frames, int64_t n_unsampled, int64_t rate,
                                int64_t N, int64_t* indices, int32_t* frame_pos, double* cdf_out, void* ws,
                                hipStream_t s) {
  double* cdf = cdf_out ? cdf_out : (double*)ws;
  unsigned* taken = (unsigned*)((char*)ws + ((n * 8 + 255) / 256) * 256);
  select_frames_kernel<<<1, SEL_THREADS, 0, s>>>(loss, n, n_frames, n_unsampled, rate, N, indices, frame_pos, cdf,
                                                 taken);
  return hipGetLastError();
}

hipError_t launch_gather_rows(const void* src, int64_t row_bytes, const int32_t* idx, int64_t rows, void* dst,
                              hipStream_t s) {
  const int64_t per = (row_bytes & 15) == 0 ? row_bytes / 16 : row_bytes;
  int64_t bx = (per + 255) / 256;
  if (bx > 1024) bx = 1024;
  dim3 grid((unsigned)(bx < 1 ? 1 : bx), (unsigned)rows), block(256);
  gather_rows_kernel<<<grid, block, 0, s>>>((const char*)src, row_bytes, idx, rows, (char*)dst);
  return hipGetLastError();
}

}  // namespace dsvt
