// BatchNorm1d + GELU of DINOHead(use_bn=True) (vision_transformer.py:255-262: Linear ->
// BatchNorm1d -> GELU per hidden layer; train_ssl.py:319-321 converts them to SyncBatchNorm).
// The head's rows are a few crops' CLS tokens (R in the tens to hundreds, D = 2048 hidden), so
// every kernel here is a column pass: one thread per column, rows looped, column sums in fp64.
//
//   forward:  sums[D | D] = (sum x, sum x^2) over the rows        bn_colsum2
//             (SyncBatchNorm: the caller all-reduces sums and the row count across ranks)
//             mean / rstd (+ running-stat update in training)    bn_finalize
//             y = GELU((x - mean) * rstd * gamma + beta), xhat and GELU'(.) saved for the backward
//   backward: sums[D | D] = (sum dz, sum dz * xhat)               bn_bwd_sums (all-reduced for SyncBN)
//             dx = gamma * rstd * (dz - sum dz / n - xhat * sum(dz xhat) / n) from the reduced sums,
//             dgamma, dbeta from the local ones
// where dz = dL/d(BatchNorm output) (the GELU' already applied by the DGELU GEMM epilogue).
#include "common.h"
#include "internal.h"

namespace dsvt {

namespace {

template <typename T>
__device__ __forceinline__ float ld_el(const T* p, int64_t i) {
  return Elem<T>::to_f(p[i]);
}

__global__ void bn_colsum2_kernel(const float* __restrict__ x, int64_t R, int64_t D, double* __restrict__ sums) {
  const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= D) return;
  double s = 0.0, q = 0.0;
  for (int64_t r = 0; r < R; ++r) {
    const double v = x[r * D + j];
    s += v;
    q += v * v;
  }
  sums[j] = s;
  sums[D + j] = q;
}

// training: batch statistics (biased variance normalises, unbiased variance enters the running
// estimate, torch's BatchNorm semantics) and running = (1 - momentum) * running + momentum * batch;
// eval: the running statistics
__global__ void bn_finalize_kernel(const double* __restrict__ sums, double count, int64_t D, float eps,
                                   float momentum, int training, float* __restrict__ run_mean,
                                   float* __restrict__ run_var, float* __restrict__ mean, float* __restrict__ rstd) {
  const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= D) return;
  if (training) {
    const double mu = sums[j] / count;
    const double var = fmax(sums[D + j] / count - mu * mu, 0.0);
    mean[j] = (float)mu;
    rstd[j] = (float)(1.0 / sqrt(var + (double)eps));
    if (run_mean) run_mean[j] = (1.0f - momentum) * run_mean[j] + momentum * (float)mu;
    if (run_var) run_var[j] = (1.0f - momentum) * run_var[j] + momentum * (float)(var * count / fmax(count - 1.0, 1.0));
  } else {
    mean[j] = run_mean[j];
    rstd[j] = 1.0f / sqrtf(run_var[j] + eps);
  }
}

template <typename T>
__global__ void bn_gelu_kernel(const float* __restrict__ x, const float* __restrict__ mean,
                               const float* __restrict__ rstd, const float* __restrict__ gamma,
                               const float* __restrict__ beta, T* __restrict__ y, T* __restrict__ gelu_grad,
                               float* __restrict__ xhat, int64_t R, int64_t D) {
  const int64_t n = R * D;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t j = i % D;
    const float xh = (x[i] - mean[j]) * rstd[j];
    const float v = fmaf(xh, gamma ? gamma[j] : 1.0f, beta ? beta[j] : 0.0f);
    const float2 r = gelu_erf_and_grad(v);
    y[i] = Elem<T>::from_f(r.x);
    if (gelu_grad) gelu_grad[i] = Elem<T>::from_f(r.y);
    if (xhat) xhat[i] = xh;
  }
}

template <typename T>
__global__ void bn_bwd_sums_kernel(const T* __restrict__ dz, const float* __restrict__ xhat, int64_t R, int64_t D,
                                   double* __restrict__ sums) {
  const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= D) return;
  double s = 0.0, q = 0.0;
  for (int64_t r = 0; r < R; ++r) {
    const double g = ld_el(dz, r * D + j);
    s += g;
    q += g * (double)xhat[r * D + j];
  }
  sums[j] = s;
  sums[D + j] = q;
}

template <typename T>
__global__ void bn_bwd_dx_kernel(const T* __restrict__ dz, const float* __restrict__ xhat,
                                 const double* __restrict__ sums, double count, const float* __restrict__ gamma,
                                 const float* __restrict__ rstd, float* __restrict__ dx, int64_t R, int64_t D) {
  const int64_t n = R * D;
  const double inv = 1.0 / count;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t j = i % D;
    const float g = (gamma ? gamma[j] : 1.0f) * rstd[j];
    const float mdz = (float)(sums[j] * inv), mdzx = (float)(sums[D + j] * inv);
    dx[i] = g * (ld_el(dz, i) - mdz - xhat[i] * mdzx);
  }
}

// dgamma (+)= sum dz * xhat, dbeta (+)= sum dz -- from this process's own sums under SyncBatchNorm
// (torch's SyncBatchNorm returns local weight / bias gradients; DDP averages them)
__global__ void bn_param_grads_kernel(const double* __restrict__ sums, int64_t D, float* __restrict__ dgamma,
                                      float* __restrict__ dbeta, int accumulate) {
  const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= D) return;
  if (dgamma) dgamma[j] = (accumulate ? dgamma[j] : 0.f) + (float)sums[D + j];
  if (dbeta) dbeta[j] = (accumulate ? dbeta[j] : 0.f) + (float)sums[j];
}

unsigned cols_grid(int64_t D) { return (unsigned)((D + 255) / 256); }
unsigned elems_grid(int64_t n) {
  const int64_t b = (n + 255) / 256;
  return (unsigned)(b < 4096 ? b : 4096);
}

}  // namespace

hipError_t launch_bn_colsum2(const float* x, int64_t R, int64_t D, double* sums, hipStream_t s) {
  bn_colsum2_kernel<<<cols_grid(D), 256, 0, s>>>(x, R, D, sums);
  return hipGetLastError();
}

hipError_t launch_bn_finalize(const double* sums, double count, int64_t D, float eps, float momentum, int training,
                              float* run_mean, float* run_var, float* mean, float* rstd, hipStream_t s) {
  bn_finalize_kernel<<<cols_grid(D), 256, 0, s>>>(sums, count, D, eps, momentum, training, run_mean, run_var, mean,
                                                  rstd);
  return hipGetLastError();
}

hipError_t launch_bn_gelu(int dtype, const float* x, const float* mean, const float* rstd, const float* gamma,
                          const float* beta, void* y, void* gelu_grad, float* xhat, int64_t R, int64_t D,
                          hipStream_t s) {
  if (dtype == 0)
    bn_gelu_kernel<bf16_t><<<elems_grid(R * D), 256, 0, s>>>(x, mean, rstd, gamma, beta, (bf16_t*)y,
                                                             (bf16_t*)gelu_grad, xhat, R, D);
  else
    bn_gelu_kernel<float><<<elems_grid(R * D), 256, 0, s>>>(x, mean, rstd, gamma, beta, (float*)y, (float*)gelu_grad,
                                                            xhat, R, D);
  return hipGetLastError();
}

hipError_t launch_bn_bwd_sums(int dtype, const void* dz, const float* xhat, int64_t R, int64_t D, double* sums,
                              hipStream_t s) {
  if (dtype == 0) bn_bwd_sums_kernel<bf16_t><<<cols_grid(D), 256, 0, s>>>((const bf16_t*)dz, xhat, R, D, sums);
  else bn_bwd_sums_kernel<float><<<cols_grid(D), 256, 0, s>>>((const float*)dz, xhat, R, D, sums);
  return hipGetLastError();
}

hipError_t launch_bn_bwd_dx(int dtype, const void* dz, const float* xhat, const double* sums,
                            const double* param_sums, double count,
                            const float* gamma, const float* rstd, float* dx, float* dgamma, float* dbeta,
                            int accumulate, int64_t R, int64_t D, hipStream_t s) {
  if (dtype == 0)
    bn_bwd_dx_kernel<bf16_t><<<elems_grid(R * D), 256, 0, s>>>((const bf16_t*)dz, xhat, sums, count, gamma, rstd, dx,
                                                               R, D);
  else
    bn_bwd_dx_kernel<float><<<elems_grid(R * D), 256, 0, s>>>((const float*)dz, xhat, sums, count, gamma, rstd, dx,
                                                              R, D);
  if (dgamma || dbeta) bn_param_grads_kernel<<<cols_grid(D), 256, 0, s>>>(param_sums, D, dgamma, dbeta, accumulate);
  return hipGetLastError();
}

}  // namespace dsvt
