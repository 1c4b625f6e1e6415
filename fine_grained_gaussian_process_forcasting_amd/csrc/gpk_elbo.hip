// ELBO terms of the variational path as single launches (fp32, fixed-order sums).
//
// Reference: the ELBO at forecast_denoising.py:86-89 --
//   DeepApproximateMLL(VariationalELBO(likelihood, model, num_data=d))(dist, y)
// whose terms are upstream GaussianLikelihood.expected_log_prob (summed over the points)
// and MeanFieldVariationalDistribution's KL(q(u) || N(0, I)) (whitened):
//   ell_r = sum_i -0.5 [((y_ri - m_ri)^2 + v_ri) / noise + log noise + log 2 pi]
//   kl    = 0.5 [sum s^2 + sum m^2 - M - sum log s^2]
// In the reference (and eagerly) each is a chain of ~10 elementwise kernels forward and
// as many backward; here one kernel each way.
#include "gpk_common.h"
#include "gpk_elbo.h"

namespace {

constexpr float kLog2Pi = 1.8378770664093453f;

// 256 threads: sum over the workgroup, result valid in thread 0 (fixed order)
GPK_DEVICE float block_sum(float v, float* red) {
  v = wave_sum(v);
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) red[w] = v;
  __syncthreads();
  float s = 0.f;
  if (threadIdx.x == 0) s = (red[0] + red[1]) + (red[2] + red[3]);
  __syncthreads();
  return s;
}

// one workgroup per row r
__global__ void __launch_bounds__(256)
gpk_ell_kernel(const float* __restrict__ y, const float* __restrict__ mean, const float* __restrict__ var,
               const float* __restrict__ noise, int N, float* __restrict__ ell) {
  __shared__ float red[4];
  const size_t base = (size_t)blockIdx.x * N;
  const float nz = noise[0], inv = 1.f / nz, cst = __logf(nz) + kLog2Pi;
  float acc = 0.f;
  for (int i = threadIdx.x; i < N; i += 256) {
    const float d = y[base + i] - mean[base + i];
    acc += (d * d + var[base + i]) * inv + cst;
  }
  const float s = block_sum(acc, red);
  if (threadIdx.x == 0) ell[blockIdx.x] = -0.5f * s;
}

// d/d{y, mean, var} of sum_r gell_r ell_r, and per-row partials of d/dnoise
__global__ void __launch_bounds__(256)
gpk_ell_grad_kernel(const float* __restrict__ y, const float* __restrict__ mean,
                    const float* __restrict__ var, const float* __restrict__ noise,
                    const float* __restrict__ gell, int N, float* __restrict__ dy,
                    float* __restrict__ dmean, float* __restrict__ dvar, float* __restrict__ dnoise_part) {
  __shared__ float red[4];
  const size_t base = (size_t)blockIdx.x * N;
  const float nz = noise[0], inv = 1.f / nz, g = gell[blockIdx.x];
  float acc = 0.f;
  for (int i = threadIdx.x; i < N; i += 256) {
    const float d = y[base + i] - mean[base + i];
    const float q = d * d + var[base + i];
    if (dmean != nullptr) dmean[base + i] = g * d * inv;
    if (dy != nullptr) dy[base + i] = -g * d * inv;
    if (dvar != nullptr) dvar[base + i] = -0.5f * g * inv;
    acc += q * inv * inv - inv;
  }
  const float s = block_sum(acc, red);
  if (threadIdx.x == 0 && dnoise_part != nullptr) dnoise_part[blockIdx.x] = 0.5f * g * s;
}

// KL of the mean-field q(u) against N(0, I): one workgroup; gkl != nullptr -> backward
__global__ void __launch_bounds__(256)
gpk_kl_kernel(const float* __restrict__ m, const float* __restrict__ s, int M, float* __restrict__ kl,
              const float* __restrict__ gkl, float* __restrict__ dm, float* __restrict__ ds) {
  __shared__ float red[4];
  if (gkl != nullptr) {
    const float g = gkl[0];
    for (int i = threadIdx.x; i < M; i += 256) {
      dm[i] = g * m[i];
      ds[i] = g * (s[i] - 1.f / s[i]);
    }
    return;
  }
  float acc = 0.f;
  for (int i = threadIdx.x; i < M; i += 256) {
    const float s2 = s[i] * s[i];
    acc += s2 + m[i] * m[i] - 1.f - __logf(s2);
  }
  const float t = block_sum(acc, red);
  if (threadIdx.x == 0) kl[0] = 0.5f * t;
}

}  // namespace

int gpk_launch_ell(const float* y, const float* mean, const float* var, const float* noise, int R,
                   int N, float* ell, hipStream_t stream) {
  hipLaunchKernelGGL(gpk_ell_kernel, dim3(R), dim3(256), 0, stream, y, mean, var, noise, N, ell);
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? 0 : (int)e;
}

int gpk_launch_ell_grad(const float* y, const float* mean, const float* var, const float* noise,
                        const float* gell, int R, int N, float* dy, float* dmean, float* dvar,
                        float* dnoise_part, hipStream_t stream) {
  hipLaunchKernelGGL(gpk_ell_grad_kernel, dim3(R), dim3(256), 0, stream, y, mean, var, noise, gell, N,
                     dy, dmean, dvar, dnoise_part);
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? 0 : (int)e;
}

int gpk_launch_kl(const float* m, const float* s, int M, float* kl, const float* gkl, float* dm,
                  float* ds, hipStream_t stream) {
  hipLaunchKernelGGL(gpk_kl_kernel, dim3(1), dim3(256), 0, stream, m, s, M, kl, gkl, dm, ds);
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? 0 : (int)e;
}
