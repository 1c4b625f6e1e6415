// Internal launch descriptors shared by the kernels and the C-ABI shim.
#pragma once
#include <hip/hip_runtime.h>

struct GpkExactArgs {
  const float* X;      // (B, N, D) row-major
  const float* y;      // (B, N)
  const float* hyp;    // device: [outputscale, noise, mean_constant, lengthscale[n_ls]]
  int n_ls;            // 1 (shared lengthscale, GPModel.py:8) or D (ARD)
  int B, N, D;
  double jitter;       // first rung of the jitter ladder (fp32: 1e-6)
  int max_tries;       // ladder length (3)
  float* L;            // (B, N, N) or nullptr
  float* z;            // (B, N) or nullptr: L^{-1}(y - c)
  float* mll;          // (B,)
  int* info;           // (B,)
};

int gpk_launch_exact(const GpkExactArgs& a, hipStream_t stream);
int gpk_launch_exact_stamps(const GpkExactArgs& a, unsigned long long* stamps, hipStream_t stream);
