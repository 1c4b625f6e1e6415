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

struct GpkExactGradArgs {
  const float* X;      // (B, N, D)
  const float* L;      // (B, N, N) forward factor
  const float* z;      // (B, N) forward L^{-1}(y - c)
  const float* hyp;    // as GpkExactArgs
  int n_ls;
  int B, N, D;
  const float* gout;   // (B,) d(objective)/d(mll_b)
  float* ws;           // gpk_exact_grad_ws_floats(B, N) floats
  float* dX;           // (B, N, D) or nullptr
  float* dy;           // (B, N) or nullptr
  float* dhyp;         // (B, 3 + n_ls): per-window d/d{s2, noise, c, lengthscale...}
};

size_t gpk_exact_grad_ws_floats(int B, int N);
int gpk_launch_exact_grad(const GpkExactGradArgs& a, hipStream_t stream);
int gpk_launch_exact_stamps(const GpkExactArgs& a, unsigned long long* stamps, hipStream_t stream);

struct GpkKzzArgs {
  const float* Z;      // (M, D)
  const float* hyp;    // device: [outputscale, lengthscale[D]]
  int M, D;
  float jitter_var;    // VariationalStrategy jitter added to K_ZZ in fp32 (1e-4)
  double jitter_chol;  // fp64 psd_safe_cholesky ladder base (1e-8)
  int max_tries;
  double* L;           // (M, M) out
  double* Linv;        // (M, M) out
  int* info;           // (1,) out
};

struct GpkVarArgs {
  const float* X;      // (B, N, D)
  const float* Z;      // (M, D)
  const double* Linv;  // (M, M)
  const float* vmean;  // (M,)
  const float* vstd;   // (M,)
  const float* hyp;    // device: [outputscale, noise, jitter, bias, weights[D], lengthscale[D]]
  const float* y;      // (B, N) or nullptr
  int B, N, M, D;
  float* mean;         // (B, N)
  float* var;          // (B, N)
  float* ell;          // (B,) or nullptr: sum_i expected log prob
  float* saved;        // training: gpk_var_saved_bytes(B, N, M, D) bytes of state for the adjoint, or nullptr
};

struct GpkVarAdjArgs {
  const float* X;      // (B, N, D)
  const float* Z;      // (M, D)
  const double* Linv;  // (M, M)
  const float* vmean;  // (M,)
  const float* vstd;   // (M,)
  const float* hyp;    // as GpkVarArgs
  const float* gmean;  // (B, N)
  const float* gvar;   // (B, N)
  int B, N, M, D;
  void* ws;            // gpk_var_adjoint_ws_bytes(B, N, M, D) bytes (saved: gpk_var_adjoint_saved_ws_bytes)
  float* dX;           // (B, N, D) out
  double* dLinv;       // (M, M) out (lower; upper zero)
  float* dZ;           // (M, D) out: the K_ZX part of dZ
  float* dpar;         // (2M + 2D + 2) out: dvmean, dvstd, ds2, dlengthscale, dweights, dbias
  const float* saved;  // the training forward's state (gpk_var_saved_bytes), or nullptr: recompute
};


struct GpkKzzGradArgs {
  const double* dLinv; // (M, M) lower: dObjective/dLinv summed over the calls sharing the factor
  const double* L;     // (M, M) gpk_kzz_chol_f64 factor (lower, zero upper)
  const double* Linv;  // (M, M) its inverse (lower, zero upper)
  const float* Z;      // (M, D)
  const float* hyp;    // device: [outputscale, lengthscale[D]]
  int M, D;
  void* ws;            // gpk_kzz_grad_ws_bytes(M, D) bytes
  float* dZ;           // (M, D) out
  float* dhyp;         // (1 + D) out: {ds2, dlengthscale[D]}
};

size_t gpk_kzz_grad_ws_bytes(int M, int D);
int gpk_launch_kzz_grad(const GpkKzzGradArgs& a, hipStream_t stream);

size_t gpk_var_adjoint_ws_bytes(int B, int N, int M, int D);
size_t gpk_var_saved_bytes(int B, int N, int M, int D);
size_t gpk_var_adjoint_saved_ws_bytes(int B, int N, int M, int D);
int gpk_launch_var_adjoint(const GpkVarAdjArgs& a, hipStream_t stream);
int gpk_launch_var(const GpkVarArgs& a, int* flags, hipStream_t stream);

int gpk_launch_window_gather(const float* table, int F, const long long* rows, int B, int n_enc,
                             int n_dec, int pred_len, int tcol, float* enc, float* dec, float* y,
                             hipStream_t stream);

struct GpkPostArgs {
  const float* X;      // (B, N, D) training inputs
  const float* L;      // (B, N, N) training factor chol(K + noise I (+ jitter)), lower
  const float* z;      // (B, N) L^{-1}(y - c)
  const float* hyp;    // as GpkExactArgs: [outputscale, noise, mean_constant, lengthscale[n_ls]]
  int n_ls;
  const float* Xs;     // (B, Ns, D) test inputs
  int B, N, Ns, D;
  float* mean;         // (B, Ns) posterior mean of f
  float* var;          // (B, Ns) posterior variance of f (unclamped)
};

size_t gpk_post_lds_bytes(int N, int D);

// 256 < N <= 800 (gpk_exact_large.hip): blocked kernels with the window's matrix in HBM.
constexpr int kGpkExactRegMaxN = 256;     // largest N of the register / LDS-resident kernels
constexpr int kGpkExactMaxN = 800;        // GPyTorch settings.max_cholesky_size
size_t gpk_exact_large_grad_ws_floats(int B, int N);
int gpk_launch_exact_large(const GpkExactArgs& a, hipStream_t stream);
int gpk_launch_exact_large_grad(const GpkExactGradArgs& a, hipStream_t stream);
int gpk_launch_exact_large_posterior(const GpkPostArgs& a, hipStream_t stream);
int gpk_launch_exact_posterior(const GpkPostArgs& a, hipStream_t stream);
