// Video DINO augmentation of one crop (datasets_custom/transform.py:661-749) as two fused
// passes over the output pixels, on frames that stay in HBM in their decoded layout:
//
//   x = frames / 255 (uint8) | frames (fp32)                         VideoDataAugmentationDINO.__call__
//   x = bicubic(crop(x, y0, x0, h, w), S x S), align_corners=False,  random_resized_crop :134-173,
//       A = -0.75, border taps clamped (F.interpolate)               resize :66-76
//   x = flip_W(x)                                                    horizontal_flip :176-203
//   for op in order: brightness x*a + 0*(1-a) | contrast x*a + mean(gray(x))*(1-a)
//                    | saturation x*a + gray(x)*(1-a)                color_jitter :371-461
//   x = gray(x) (all channels)                                       grayscale :349-368
//   y = (x - mean_c) / std_c                                         color_normalization :494-516
//
// gray(x) = 0.299*x[2] + 0.587*x[1] + 0.114*x[0] (the reference's BGR convention), every
// product / sum rounded separately as the reference's tensor ops do (no FMA contraction).  The
// contrast mean is a per-frame reduction of the image AT that point of the chain, so a crop
// whose chain contains "contrast" first runs pass 1: the chain up to contrast, gray, per-block
// partial sums (fp64); pass 2 then reduces the frame's partials in a fixed order and writes
// the output, [T, C, S, S] or [C, T, S, S].  Random parameters are drawn on the host with the
// reference's own RNG calls (dsvt/augment.py).
#include "common.h"

#include "../../include/dsvt.h"

namespace dsvt {

namespace {

constexpr int AUG_THREADS = 256;

__device__ __forceinline__ float fmul(float a, float b) { return __fmul_rn(a, b); }
__device__ __forceinline__ float fadd(float a, float b) { return __fadd_rn(a, b); }

// PyTorch's cubic convolution coefficients (A = -0.75) for fractional offset t
__device__ __forceinline__ void cubic_coeffs(float t, float (&c)[4]) {
  const float A = -0.75f;
  const float x1 = t + 1.0f, x2 = t, x3 = 1.0f - t, x4 = 2.0f - t;
  c[0] = ((A * x1 - 5.0f * A) * x1 + 8.0f * A) * x1 - 4.0f * A;
  c[1] = ((A + 2.0f) * x2 - (A + 3.0f)) * x2 * x2 + 1.0f;
  c[2] = ((A + 2.0f) * x3 - (A + 3.0f)) * x3 * x3 + 1.0f;
  c[3] = ((A * x4 - 5.0f * A) * x4 + 8.0f * A) * x4 - 4.0f * A;
}

struct AugIn {
  const void* frames; int u8;
  int64_t sT, sC, sH, sW;     // element strides of the frame tensor
  int64_t H, W;
  const int32_t* fidx;        // output frame t reads input frame fidx[t] (nullable: identity)
  int64_t T_in;               // frames in the input (indices are clamped into it)
};

__device__ __forceinline__ int64_t in_frame(const AugIn& in, int64_t t) {
  int64_t f = in.fidx ? (int64_t)in.fidx[t] : t;
  return f < 0 ? 0 : (f >= in.T_in ? in.T_in - 1 : f);
}

__device__ __forceinline__ float pix(const AugIn& in, int64_t t, int c, int64_t y, int64_t x) {
  const int64_t o = t * in.sT + c * in.sC + y * in.sH + x * in.sW;
  if (in.u8) return __fdiv_rn((float)((const uint8_t*)in.frames)[o], 255.0f);
  return ((const float*)in.frames)[o];
}

// bicubic sample of the crop at output pixel (oy, ox) for all three channels
__device__ __forceinline__ void resized(const AugIn& in, const dsvt_aug_params& p, int64_t t, int oy, int ox,
                                        float (&v)[3]) {
  const float sy = (float)p.h / (float)p.size, sx = (float)p.w / (float)p.size;
  const float ry = sy * ((float)oy + 0.5f) - 0.5f, rx = sx * ((float)ox + 0.5f) - 0.5f;
  const float fy = floorf(ry), fx = floorf(rx);
  float cy[4], cx[4];
  cubic_coeffs(ry - fy, cy);
  cubic_coeffs(rx - fx, cx);
  int64_t ys[4], xs[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    int64_t yy = (int64_t)fy - 1 + k, xx = (int64_t)fx - 1 + k;
    yy = yy < 0 ? 0 : (yy > p.h - 1 ? p.h - 1 : yy);
    xx = xx < 0 ? 0 : (xx > p.w - 1 ? p.w - 1 : xx);
    ys[k] = p.y0 + yy;
    xs[k] = p.x0 + xx;
  }
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    float acc = 0.f;
#pragma unroll
    for (int a = 0; a < 4; ++a) {
      float row = 0.f;
#pragma unroll
      for (int b = 0; b < 4; ++b) row += pix(in, t, c, ys[a], xs[b]) * cx[b];
      acc += row * cy[a];
    }
    v[c] = acc;
  }
}

__device__ __forceinline__ float gray_of(const float (&v)[3]) {
  return fadd(fadd(fmul(0.299f, v[2]), fmul(0.587f, v[1])), fmul(0.114f, v[0]));
}

// apply ops [from, to) of the jitter chain (contrast uses `cmean`)
__device__ __forceinline__ void jitter(const dsvt_aug_params& p, int from, int to, float cmean, float (&v)[3]) {
  for (int k = from; k < to; ++k) {
    const float a = p.alpha[k], b = p.beta[k];
    if (p.op[k] == DSVT_AUG_BRIGHTNESS) {
#pragma unroll
      for (int c = 0; c < 3; ++c) v[c] = fadd(fmul(v[c], a), fmul(0.0f, b));
    } else if (p.op[k] == DSVT_AUG_CONTRAST) {
      const float m = fmul(cmean, b);
#pragma unroll
      for (int c = 0; c < 3; ++c) v[c] = fadd(fmul(v[c], a), m);
    } else {
      const float g = fmul(gray_of(v), b);
#pragma unroll
      for (int c = 0; c < 3; ++c) v[c] = fadd(fmul(v[c], a), g);
    }
  }
}

__device__ __forceinline__ int contrast_pos(const dsvt_aug_params& p) {
  for (int k = 0; k < p.n_ops; ++k)
    if (p.op[k] == DSVT_AUG_CONTRAST) return k;
  return -1;
}

// pass 1: per-block partial sums of gray(chain[0:contrast)(x)) for frame blockIdx.y
__global__ __launch_bounds__(AUG_THREADS) void aug_gray_partials_kernel(AugIn in, dsvt_aug_params p, double* partial) {
  __shared__ double red[AUG_THREADS];
  const int64_t t = blockIdx.y;
  const int64_t tin = in_frame(in, t);
  const int64_t npix = (int64_t)p.size * p.size;
  const int64_t pidx = (int64_t)blockIdx.x * AUG_THREADS + threadIdx.x;
  const int cpos = contrast_pos(p);
  double s = 0.0;
  if (pidx < npix) {
    const int oy = (int)(pidx / p.size), ox = (int)(pidx % p.size);
    float v[3];
    resized(in, p, tin, oy, p.flip ? p.size - 1 - ox : ox, v);
    jitter(p, 0, cpos, 0.f, v);
    s = (double)gray_of(v);
  }
  red[threadIdx.x] = s;
  __syncthreads();
  for (int o = AUG_THREADS / 2; o > 0; o >>= 1) {
    if (threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) partial[t * gridDim.x + blockIdx.x] = red[0];
}

// pass 2: the whole chain + normalization, one thread per output pixel (3 channels)
__global__ __launch_bounds__(AUG_THREADS) void aug_apply_kernel(AugIn in, dsvt_aug_params p, const double* partial,
                                                                int nparts, float* out, int64_t T, int layout) {
  __shared__ float s_mean;
  const int64_t t = blockIdx.y;
  const int64_t tin = in_frame(in, t);
  const int64_t npix = (int64_t)p.size * p.size;
  const int cpos = contrast_pos(p);
  if (cpos >= 0) {
    if (threadIdx.x == 0) {
      double s = 0.0;
      for (int k = 0; k < nparts; ++k) s += partial[t * nparts + k];
      s_mean = (float)(s / (double)npix);
    }
    __syncthreads();
  }
  const int64_t pidx = (int64_t)blockIdx.x * AUG_THREADS + threadIdx.x;
  if (pidx >= npix) return;
  const int oy = (int)(pidx / p.size), ox = (int)(pidx % p.size);
  float v[3];
  resized(in, p, tin, oy, p.flip ? p.size - 1 - ox : ox, v);
  jitter(p, 0, p.n_ops, cpos >= 0 ? s_mean : 0.f, v);
  if (p.gray) {
    const float g = gray_of(v);
    v[0] = v[1] = v[2] = g;
  }
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    const float y = __fdiv_rn(__fsub_rn(v[c], p.mean[c]), p.std[c]);
    const int64_t o = layout == 0 ? ((t * 3 + c) * npix + pidx) : (((int64_t)c * T + t) * npix + pidx);
    out[o] = y;
  }
}

}  // namespace

int64_t augment_ws_bytes(int64_t T, int64_t size) {
  const int64_t nparts = (size * size + AUG_THREADS - 1) / AUG_THREADS;
  return T * nparts * 8;
}

hipError_t launch_video_augment(const void* frames, int u8, int64_t T_in, int64_t T, const int32_t* fidx, int64_t H,
                                int64_t W, int64_t sT, int64_t sC, int64_t sH, int64_t sW, const dsvt_aug_params& p,
                                float* out, int layout, void* ws, hipStream_t s) {
  AugIn in{frames, u8, sT, sC, sH, sW, H, W, fidx, T_in};
  const int64_t npix = (int64_t)p.size * p.size;
  const int nparts = (int)((npix + AUG_THREADS - 1) / AUG_THREADS);
  dim3 grid((unsigned)nparts, (unsigned)T), block(AUG_THREADS);
  bool contrast = false;
  for (int k = 0; k < p.n_ops; ++k) contrast |= p.op[k] == DSVT_AUG_CONTRAST;
  if (contrast) {
    aug_gray_partials_kernel<<<grid, block, 0, s>>>(in, p, (double*)ws);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  aug_apply_kernel<<<grid, block, 0, s>>>(in, p, (const double*)ws, nparts, out, T, layout);
  return hipGetLastError();
}

}  // namespace dsvt
