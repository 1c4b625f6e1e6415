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

// ---------------------------------------------------------------------------
// Verdict of one recorded numerical check of a HIP-graph replay (graphs.GraphedStep):
// ring[slot][item] = {max info, max(-info, 0), NaN in the inputs} (kind 0: a
// psd_safe_cholesky info vector) or {flag, 0, 0} (kind 1: the variance-clamp flag word),
// slot = counter % slots; sticky |= (max info > 0) for kind 0; kind 2 only bumps the replay
// counter (the step's end). The NaN scan runs only for a failed factorisation. One
// workgroup: replaces ~10 small torch reductions per recorded check.
// ---------------------------------------------------------------------------
namespace {
__global__ void __launch_bounds__(256)
gpk_verdict_kernel(const int* __restrict__ info, int n, const float* __restrict__ in0, long long n0,
                   const float* __restrict__ in1, long long n1, int kind, int* __restrict__ ring,
                   long long* __restrict__ counter, int slots, int item, int items, int* __restrict__ sticky,
                   int advance) {
  __shared__ int red[3][4];
  __shared__ int fail;
  const int tid = threadIdx.x;
  if (kind == 2) {   // the step's end: advance the replay counter only
    if (tid == 0) counter[0] = counter[0] + 1;
    return;
  }
  int mx = -2147483647, mn = 0, nan = 0;
  if (kind == 0) {
    for (int i = tid; i < n; i += 256) {
      const int v = info[i];
      mx = v > mx ? v : mx;
      mn = -v > mn ? -v : mn;
    }
  } else if (tid == 0) {
    mx = info[0];
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    mx = max(mx, __shfl_xor(mx, off, 64));
    mn = max(mn, __shfl_xor(mn, off, 64));
  }
  if ((tid & 63) == 0) {
    red[0][tid >> 6] = mx;
    red[1][tid >> 6] = mn;
  }
  __syncthreads();
  if (tid == 0) {
    for (int w = 1; w < 4; ++w) {
      mx = max(mx, red[0][w]);
      mn = max(mn, red[1][w]);
    }
    fail = kind == 0 && mx > 0;
  }
  __syncthreads();
  if (fail) {   // NaN scan of the inputs only for a failed factorisation (as the eager check)
    for (long long i = tid; i < n0; i += 256) nan |= (in0[i] != in0[i]);
    for (long long i = tid; i < n1; i += 256) nan |= (in1[i] != in1[i]);
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) nan |= __shfl_xor(nan, off, 64);
    if ((tid & 63) == 0) red[2][tid >> 6] = nan;
    __syncthreads();
    if (tid == 0) nan = (red[2][0] | red[2][1]) | (red[2][2] | red[2][3]);
  }
  if (tid == 0) {
    const long long cnt = counter[0];
    int* dst = ring + ((size_t)(cnt % slots) * items + item) * 3;
    dst[0] = mx;
    dst[1] = kind == 0 ? mn : 0;
    dst[2] = kind == 0 ? nan : 0;
    if (kind == 0 && mx > 0) sticky[0] = 1;
    if (advance) counter[0] = cnt + 1;
  }
}
}  // namespace

int gpk_launch_verdict(const int* info, int n, const float* in0, long long n0, const float* in1,
                       long long n1, int kind, int* ring, long long* counter, int slots, int item,
                       int items, int* sticky, int advance, hipStream_t stream) {
  hipLaunchKernelGGL(gpk_verdict_kernel, dim3(1), dim3(256), 0, stream, info, n, in0, n0, in1, n1, kind,
                     ring, counter, slots, item, items, sticky, advance);
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? 0 : (int)e;
}
