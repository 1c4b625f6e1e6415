/*
 * gpk.h — C ABI of the MI355X-native GP blur/denoise kernels (libgpk.so).
 *
 * Plain pointers and sizes only; every buffer is DEVICE memory owned by the
 * caller (contiguous, row-major). `stream` is a hipStream_t passed as void*
 * (0 = legacy default stream); all work is enqueued on it, nothing
 * synchronises, nothing is allocated. The library keeps no pointer after a
 * call returns and holds no mutable global state (safe for concurrent callers,
 * e.g. Optuna's n_jobs=4 threads in reference train.py:86).
 *
 * Return codes: 0 = success; <0 = invalid argument (-k: k-th argument, LAPACK
 * style); >0 = a hipError_t from the launch. Per-window numerical status goes
 * to info[b] (see each function).
 */
#ifndef GPK_H_
#define GPK_H_
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Library version (major*10000 + minor*100 + patch). */
int gpk_version(void);

/* Human-readable text for a return code of any gpk_* function. */
const char* gpk_strerror(int code);

/* Largest N gpk_exact_mll_f32 accepts (padded to 16, register-resident). */
int gpk_exact_max_n(void);

/*
 * Exact GP marginal log likelihood, fused per window b in [0, B):
 *   K_hat = s2 * exp(-0.5*||(x_i - x_j)/l||^2) + noise * I
 *   L     = psd_safe_cholesky(K_hat) with the fp32 jitter ladder
 *           jitter * 10^t (t < max_tries), applied to failing windows only
 *   z     = L^{-1} (y - c)
 *   mll   = -0.5 * (|z|^2 + 2 sum_i log L_ii + N log 2pi) / N
 *
 * Replaces (reference): ExactGPModel.forward (denoising_model/GPModel.py:10-13)
 * + ExactMarginalLogLikelihood(likelihood, model)(output, y) — the canonical
 * GPyTorch partner of GPModel.py (upstream mlls/exact_marginal_log_likelihood.py,
 * linear_operator utils/cholesky.py::psd_safe_cholesky); SURVEY.md §8a rows a1-a7.
 *
 * X    : (B, N, D) float     y : (B, N) float
 * hyp  : device float[3 + n_lengthscale] =
 *        {outputscale s2, noise, mean_constant c, lengthscale[n_lengthscale]}
 *        (constrained values: softplus already applied by the caller)
 * n_lengthscale : 1 (GPModel.py:8) or D (ARD)
 * jitter, max_tries : ladder (GPyTorch defaults 1e-6 and 3 for fp32)
 * L    : (B, N, N) float out, lower factor with zeroed upper triangle; may be NULL
 * z    : (B, N) float out; may be NULL
 * mll  : (B,) float out
 * info : (B,) int out: 0 = factored without jitter; -t = factored after t
 *        ladder steps (caller emits GPyTorch's NumericalWarning); k > 0 = still
 *        not positive definite at column k after max_tries (caller raises
 *        NotPSDError, or NanError if the inputs hold NaN).
 */
int gpk_exact_mll_f32(const float* X, const float* y, const float* hyp,
                      int n_lengthscale, int B, int N, int D, double jitter,
                      int max_tries, float* L, float* z, float* mll, int* info,
                      void* stream);

#ifdef __cplusplus
}
#endif
#endif /* GPK_H_ */
