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

/* Largest N the exact entry points accept: 800, GPyTorch's settings.max_cholesky_size (the
 * exact MLL leaves Cholesky for CG / Lanczos above it). N <= 256 runs the fused register /
 * LDS-resident kernels; 256 < N <= 800 the blocked kernels of gpk_exact_large.hip, which
 * factor in place in L (so L is required there) and need D <= 64. */
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
 * L    : (B, N, N) float out, lower factor with zeroed upper triangle; may be NULL for
 *        N <= 256 (required above: the blocked path's working storage, -10 if NULL)
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

/*
 * Analytic backward of gpk_exact_mll_f32 (per window b, objective sum_b gout[b] mll[b]):
 *   G = gout (alpha alpha^T - K_hat^{-1}) / (2N),  alpha = K_hat^{-1} (y - c) = L^{-T} z
 *   dhyp[b] = {sum G o E, tr G, gout sum(alpha)/N, dl...}  (E = K / s2, l: 1 or D entries)
 *   dX = dK/dX contracted with G,  dy = -gout alpha / N
 * from the forward's L and z (nothing is refactored).
 *
 * Replaces (reference): the autograd backward that train.py:166 (loss.backward())
 * runs through GPyTorch's ExactMarginalLogLikelihood for ExactGPModel
 * (denoising_model/GPModel.py:5-13; upstream linear_operator inv_quad_logdet /
 * psd_safe_cholesky backward, kernels/rbf_kernel.py backward); SURVEY.md §8f row 1.
 *
 * L : (B, N, N) float, z : (B, N) float (gpk_exact_mll_f32 outputs)   gout : (B,) float
 * workspace : gpk_exact_grad_workspace_bytes(B, N) bytes of device memory (the lower block
 *             tiles of K_hat^{-1} per window, ~145 KB at N = 256, plus small vectors; for
 *             N > 256, L^{-1} and K_hat^{-1} as Np x Np each, Np = N rounded up to 32)
 * dX : (B, N, D) float out or NULL (D <= 64)   dy : (B, N) float out or NULL
 * dhyp : (B, 3 + n_lengthscale) float out (per window; the caller sums over b)
 */
size_t gpk_exact_grad_workspace_bytes(int B, int N);
int gpk_exact_mll_grad_f32(const float* X, const float* L, const float* z, const float* hyp,
                           int n_lengthscale, int B, int N, int D, const float* gout, void* workspace,
                           float* dX, float* dy, float* dhyp, void* stream);

/*
 * Exact-GP posterior at new inputs (eval mode), per window b, from the training
 * factor of gpk_exact_mll_f32 (nothing is refactored):
 *   K*   = s2 * exp(-0.5 ||(x_n - xs_t)/l||^2)       (N x Ns, training x test)
 *   V    = L^{-1} K*
 *   mean = c + V^T z          = c + K*^T K_hat^{-1} (y - c)
 *   var  = s2 - colsum(V o V) = diag(K** - K*^T K_hat^{-1} K*)   (latent f, unclamped)
 *
 * Replaces (reference): ExactGPModel in eval mode (denoising_model/GPModel.py:10-13;
 * SURVEY.md §3.3) -> upstream models/exact_gp.py __call__ ->
 * exact_prediction_strategies.py exact_predictive_mean / exact_predictive_covar (diag).
 *
 * X : (B, N, D) float training inputs   L : (B, N, N) float   z : (B, N) float
 * hyp : as gpk_exact_mll_f32   Xs : (B, Ns, D) float test inputs (D <= 64, N <= 800)
 * mean, var : (B, Ns) float out
 */
int gpk_exact_posterior_f32(const float* X, const float* L, const float* z, const float* hyp,
                            int n_lengthscale, const float* Xs, int B, int N, int Ns, int D,
                            float* mean, float* var, void* stream);

/*
 * Shared inducing-point factorisation of the whitened VariationalStrategy:
 *   A    = K_ZZ + jitter (fp32 add, as K_ZZ.add_jitter), then upcast to fp64
 *   L    = psd_safe_cholesky(A) with the fp64 ladder chol_jitter * 10^t
 *   Linv = L^{-1}
 * K_ZZ = s2 * exp(-0.5 ||(z_i - z_j)/l||^2) with ARD lengthscales (GPyTorch's centred
 * GEMM-form squared distance, diagonal not zeroed: Z requires grad in the reference).
 * Factor: ONE workgroup (16 waves: 15 hold the upper triangle as fp64-MFMA register tiles,
 * a diagonal wave factors each 16 x 16 diagonal block one step ahead; 16-column right-looking
 * steps; the fp64 ladder restarted in-kernel); inverse: one workgroup per 16-column block
 * column (block forward substitution on fp64 MFMA), the block columns on different CUs.
 *
 * Replaces (reference): the per-window (b-fold redundant) fp64 Cholesky that
 * VariationalStrategy._cholesky_factor runs for ToyDeepGPHiddenLayer
 * (denoising_model/DeepGP.py:33-38, inducing points expanded to the batch by
 * upstream _expand_inputs); SURVEY.md §8a rows a7/a9.
 *
 * Z   : (M, D) float (M <= 256, D <= 64)     hyp : device float[1 + D] = {s2, lengthscale[D]}
 * L, Linv : (M, M) double out (lower, zero upper)   info : (1,) int out, codes as above
 */
int gpk_kzz_chol_f64(const float* Z, const float* hyp, int M, int D, float jitter,
                     double chol_jitter, int max_tries, double* L, double* Linv, int* info,
                     void* stream);

/*
 * Adjoint of gpk_kzz_chol_f64, once per optimizer step for all GP calls that shared the
 * factor (fp64 throughout):
 *   Lbar = -tril(Linv^T G Linv^T),  S = Linv^T Phi(L^T Lbar) Linv,  Kbar = (S + S^T)/2
 *   (Phi = lower triangle with the diagonal halved), then the RBF adjoint over K_ZZ
 *   (without its jitter): W = Kbar o K, dZ = 2 (W zs - zs o W1)/l, dl, ds2 = sum W / s2.
 * Five fp64-MFMA tile GEMM launches + a W-tile kernel + one fixed-order reduction
 * (run-to-run deterministic).
 *
 * Replaces (reference): the autograd backward of psd_safe_cholesky + the triangular solve
 * inside upstream VariationalStrategy (denoising_model/DeepGP.py:33-38) that train.py:166
 * runs -- b times per GP call in the reference (Z expanded over the batch), once per step
 * here; SURVEY.md §8f rows 1 and 3.
 *
 * dLinv : (M, M) double, lower (G = dObjective/dLinv)   L, Linv : gpk_kzz_chol_f64 outputs
 * Z : (M, D) float   hyp : device float[1 + D] = {s2, lengthscale[D]} (as gpk_kzz_chol_f64)
 * workspace : gpk_kzz_backward_workspace_bytes(M, D) bytes of device memory
 * dZ : (M, D) float out    dhyp : (1 + D) float out = {ds2, dlengthscale[D]}
 */
size_t gpk_kzz_backward_workspace_bytes(int M, int D);
int gpk_kzz_backward_f64(const double* dLinv, const double* L, const double* Linv, const float* Z,
                         const float* hyp, int M, int D, void* workspace, float* dZ, float* dhyp,
                         void* stream);

/*
 * ELBO terms of the variational path, one launch each way (fixed-order sums):
 *   ell_r = sum_i -0.5 [((y_ri - mean_ri)^2 + var_ri) / noise + log noise + log 2 pi]
 *   kl    = 0.5 [sum s^2 + sum m^2 - M - sum log s^2]         (whitened mean-field q(u))
 * gpk_gauss_ell_grad_f32: for the objective sum_r gell_r ell_r -> dy, dmean, dvar (each
 * (R, N) or NULL) and dnoise_part (R,) per-row partials of d/dnoise (or NULL).
 * gpk_meanfield_kl_f32: gkl == NULL -> kl (1,) out; else the backward dm = gkl m,
 * ds = gkl (s - 1/s).
 *
 * Replaces (reference): upstream GaussianLikelihood.expected_log_prob (summed over the
 * points by VariationalELBO._log_likelihood_term) and
 * MeanFieldVariationalDistribution.kl_divergence, as the ELBO at forecast_denoising.py:86-89
 * evaluates them, and their autograd backward (train.py:166); SURVEY.md §8a row a14.
 *
 * y, mean, var : (R, N) float;  noise : device float[1];  ell, gell : (R,) float
 * m, s : (M,) float (variational mean / stddev);  kl, gkl : (1,) float
 */
int gpk_gauss_ell_f32(const float* y, const float* mean, const float* var, const float* noise, int R,
                      int N, float* ell, void* stream);
int gpk_gauss_ell_grad_f32(const float* y, const float* mean, const float* var, const float* noise,
                           const float* gell, int R, int N, float* dy, float* dmean, float* dvar,
                           float* dnoise_part, void* stream);
int gpk_meanfield_kl_f32(const float* m, const float* s, int M, float* kl, const float* gkl,
                         float* dm, float* ds, void* stream);

/*
 * The per-row ELBO of VariationalELBO (combine_terms, one whitened mean-field layer) in one
 * launch each way:
 *   elbo_r = ell_r / N - kl_scale * KL(N(m, diag s^2) || N(0, I)),  kl_scale = beta / num_data
 *   ell_r  = sum_i -0.5 [((y_ri - mean_ri)^2 + var_ri) / noise + log noise + log 2 pi]
 * Rows r of y / mean / var start at r * ld (ld >= N: a point slice of a joint output needs no
 * copy). clamp_flag (or NULL): set to 1 if any var_ri <= min_var (the kernel-clamped entries:
 * MultivariateNormal.variance's NumericalWarning). The backward (objective sum_r g_r elbo_r)
 * writes dmean, dvar (R, N contiguous), per-row d/dnoise partials and dm, ds (M). R = 0 is
 * accepted by both (the forward writes nothing; the backward zero-fills dm and ds).
 *
 * Replaces (reference): DeepApproximateMLL(VariationalELBO(likelihood, model, num_data=d))
 * at forecast_denoising.py:86-89 (upstream mlls/variational_elbo.py +
 * _approximate_mll.py: expected_log_prob(...).sum(-1).div(N) - kl.div(num_data / beta))
 * and its autograd backward (train.py:166); SURVEY.md §8a row a14.
 */
int gpk_variational_elbo_f32(const float* y, long long ldy, const float* mean, long long ldm,
                             const float* var, long long ldv, const float* noise, const float* m,
                             const float* s, int M, int R, int N, float kl_scale, float min_var,
                             float* elbo, int* clamp_flag, void* stream);
int gpk_variational_elbo_grad_f32(const float* y, long long ldy, const float* mean, long long ldm,
                                  const float* var, long long ldv, const float* noise, const float* m,
                                  const float* s, int M, int R, int N, float kl_scale, const float* gelbo,
                                  float* dmean, float* dvar, float* dnoise_part, float* dm, float* ds,
                                  void* stream);

/*
 * Condensed verdict of one host-side numerical check inside a captured HIP graph
 * (graphs.GraphedStep): kind 0 = a psd_safe_cholesky info vector (n entries; in0 / in1 =
 * the factorised inputs, scanned for NaN only when a factorisation failed), kind 1 = the
 * variance-clamp flag word, kind 2 = end of the step (advance the replay counter).
 *   ring[(counter % slots) * items + item] = {max info, max(-info, 0), NaN in the inputs}
 *   sticky |= (max info > 0)
 * so the host reads the verdicts of a block of replays with one copy and warns / raises
 * per replay exactly as GPyTorch's eager psd_safe_cholesky / MultivariateNormal.variance
 * checks (linear_operator utils/cholesky.py).
 * ring : (slots, items, 3) int device;  counter : (1,) int64 device;  sticky : (1,) int device
 */
int gpk_record_check(const int* info, int n, const float* in0, long long n0, const float* in1,
                     long long n1, int kind, int* ring, long long* counter, int slots, int item,
                     int items, int* sticky, void* stream);

/*
 * Batched variational predictive distribution and expected log likelihood:
 *   K_ZX = s2 * exp(-0.5 ||(z_m - x_i)/l||^2)       (fp32, GPyTorch's centred GEMM form)
 *   A    = Linv @ K_ZX                              (fp64, then cast to fp32)
 *   mean = A^T m + x @ w + b0                       (LinearMean)
 *   var  = max(s2 + jitter + sum_m A_mi^2 (s_m^2 - 1), 1e-6)
 *   ell  = sum_i -0.5 [((y_i - mean_i)^2 + var_i)/noise + log noise + log 2pi]
 *
 * Replaces (reference): DeepGPp.predict / ToyDeepGPHiddenLayer.__call__
 * (denoising_model/DeepGP.py:51-99) via upstream VariationalStrategy.forward,
 * DeepGPLayer.__call__, GaussianLikelihood.expected_log_prob as used by
 * denoise_model_2.add_gp_noise (denoise_model_2.py:32-40) and the ELBO at
 * forecast_denoising.py:86-89; SURVEY.md §8a rows a9-a14.
 *
 * X : (B, N, D) float (D <= 64)  Z : (M, D)  Linv : (M, M) double (gpk_kzz_chol_f64)
 * vmean, vstd : (M,) float (MeanFieldVariationalDistribution mean / stddev)
 * hyp : device float[4 + 2D] = {s2, noise, jitter, bias, weights[D], lengthscale[D]}
 * y : (B, N) float or NULL;  mean, var : (B, N) float out;  ell : (B,) float out or NULL
 * (needs y)   flags : (1,) int out or NULL: bit 0 set when the variance clamp fired
 * (the caller emits GPyTorch's NumericalWarning from MultivariateNormal.variance).
 */
int gpk_variational_f32(const float* X, const float* Z, const double* Linv, const float* vmean,
                        const float* vstd, const float* hyp, const float* y, int B, int N, int M,
                        int D, float* mean, float* var, float* ell, int* flags, void* stream);

/*
 * Adjoint of gpk_variational_f32 for the objective sum(gmean * mean) + sum(gvar * var)
 * (var's clamp at 1e-6 passes no gradient), everything but the K_ZZ factor:
 *   dA    = gmean_i m_m + 2 gvar_i (s_m^2 - 1) A_mi         (fp32, as the reference's dA)
 *   dK    = Linv^T dA,  Q = dK o K_ZX
 *   dX    (B, N, D) float out: RBF adjoint + gmean_i w
 *   dLinv (M, M) double out: sum over all points of dA K_ZX^T (lower, upper zero) -- the
 *         caller back-propagates it through the shared K_ZZ factor once per step
 *   dZ    (M, D) float out: the K_ZX part of dZ
 *   dpar  (2M + 2D + 2) float out: {dvmean (M), dvstd (M), ds2 (K_ZX and variance parts),
 *         dl (D, K_ZX part), dweights (D), dbias}  (LinearMean: dweights = X^T gmean)
 * workspace : gpk_variational_adjoint_workspace_bytes(B, N, M, D) bytes of device memory.
 * All sums are in a fixed order (run-to-run deterministic).
 *
 * Replaces (reference): the autograd backward that train.py:166 runs through
 * VariationalStrategy / DeepGPLayer for DeepGPp (denoising_model/DeepGP.py:51-99,
 * forecast_denoising.py:86-104); SURVEY.md §8f row 1.
 */
size_t gpk_variational_adjoint_workspace_bytes(int B, int N, int M, int D);
int gpk_variational_adjoint_f32(const float* X, const float* Z, const double* Linv,
                                const float* vmean, const float* vstd, const float* hyp,
                                const float* gmean, const float* gvar, int B, int N, int M, int D,
                                void* workspace, float* dX, double* dLinv, float* dZ, float* dpar,
                                void* stream);

/*
 * Training pair of the variational path for M > 64 (the reference's DeepGP default M = 256,
 * denoising_model/DeepGP.py:15): the forward keeps state the adjoint consumes, so the adjoint
 * neither repeats the forward's A = Linv K_ZX GEMM nor round-trips dA / K_ZX through HBM.
 *   gpk_variational_saved_bytes(B, N, M, D): bytes of that state; 0 when the shape is served
 *     by the recompute adjoint only (M <= 64, or the saved path's LDS plan does not fit).
 *   gpk_variational_train_f32: gpk_variational_f32 + `saved` (device, saved_bytes bytes; may be
 *     NULL only when saved_bytes is 0, else -16): A (fp32, as the reference casts it) and the
 *     variance clamp mask of every point.
 *   gpk_variational_adjoint_saved_f32: gpk_variational_adjoint_f32 from that state (same
 *     outputs, same argument meaning; saved = argument 9, -12 when saved_bytes is 0 for the
 *     shape), workspace of gpk_variational_adjoint_saved_workspace_bytes(B, N, M, D) bytes.
 *     dLinv = sum_i dA_i K_i^T is formed as m u^T + 2 diag(s^2 - 1) G' with u = K_ZX gmean and
 *     G' = A diag(gvar) K_ZX^T on the saved fp32 A (products exact on f32 MFMA), i.e. the
 *     reference's own fp32 dA, without a dA / K_ZX workspace.
 * Replaces (reference): the same forward / autograd backward as the two functions above.
 */
size_t gpk_variational_saved_bytes(int B, int N, int M, int D);
int gpk_variational_train_f32(const float* X, const float* Z, const double* Linv, const float* vmean,
                              const float* vstd, const float* hyp, const float* y, int B, int N, int M,
                              int D, float* mean, float* var, float* ell, int* flags, void* saved,
                              void* stream);
size_t gpk_variational_adjoint_saved_workspace_bytes(int B, int N, int M, int D);
int gpk_variational_adjoint_saved_f32(const float* X, const float* Z, const double* Linv,
                                      const float* vmean, const float* vstd, const float* hyp,
                                      const float* gmean, const float* gvar, const void* saved, int B,
                                      int N, int M, int D, void* workspace, float* dX, double* dLinv,
                                      float* dZ, float* dpar, void* stream);

/*
 * GPU-resident training-window gather:
 *   for window b with first row r = rows[b] of the (id, time)-sorted table:
 *     enc[b] = table[r      : r + n_enc]                  (n_enc, F)
 *     dec[b] = table[r + n_enc : r + T - pred_len]        (T - n_enc - pred_len, F)
 *     y[b]   = table[r + T - pred_len : r + T, target_col] (pred_len,)
 *   r = -1 gives an all-zero window (the reference's zero-filled tail when max_samples
 *   exceeds the valid sampling locations). Bit-exact copies (float32 table).
 *
 * Replaces (reference): the host NumPy windowing of Utils/base_train.py:29-97
 * (sample_train_val_test; windows chosen as in batch_sampled_data :100-153) and the
 * per-step host->device copies of train.py:160-161; the window CHOICE stays on the host
 * (the reference's np.random sequence, reproduced by the caller).
 *
 * table : (n_rows, F) float, device    rows : (B,) int64, device (each r + T <= n_rows, or -1)
 * enc : (B, n_enc, F) float out   dec : (B, T - n_enc - pred_len, F) float out   y : (B, pred_len) float out
 */
int gpk_window_gather_f32(const float* table, long long n_rows, int F, const long long* rows, int B,
                          int T, int n_enc, int pred_len, int target_col, float* enc, float* dec,
                          float* y, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* GPK_H_ */
