// C-ABI shim: argument validation + dispatch to the gfx950 kernels.
// Declarations and the reference interfaces each entry point replaces: include/gpk.h.
#include "../../include/gpk.h"
#include "gpk_internal.h"
#include "gpk_elbo.h"
#include "gpk_kzz.h"

extern "C" {

int gpk_version(void) { return 100; }

const char* gpk_strerror(int code) {
  if (code == 0) return "success";
  if (code < 0) {
    switch (code) {
      case -6: return "gpk: N exceeds the supported maximum (gpk_exact_max_n)";
      case -7: return "gpk: D too large for the LDS staging layout";
      default: return "gpk: invalid argument (negative code = argument index)";
    }
  }
  return hipGetErrorString((hipError_t)code);
}

int gpk_exact_max_n(void) { return kGpkExactMaxN; }

int gpk_exact_mll_f32(const float* X, const float* y, const float* hyp, int n_lengthscale,
                      int B, int N, int D, double jitter, int max_tries, float* L, float* z,
                      float* mll, int* info, void* stream) {
  if (X == nullptr) return -1;
  if (y == nullptr) return -2;
  if (hyp == nullptr) return -3;
  if (n_lengthscale != 1 && n_lengthscale != D) return -4;
  if (B < 0) return -5;
  if (N < 1) return -6;
  if (D < 1) return -7;
  if (!(jitter >= 0.0)) return -8;
  if (max_tries < 0 || max_tries > 12) return -9;
  if (mll == nullptr) return -12;
  if (info == nullptr) return -13;
  if (N > gpk_exact_max_n()) return -6;
  if (N > kGpkExactRegMaxN && L == nullptr) return -10;   // the blocked path factors in L
  if (N > kGpkExactRegMaxN && D > 64) return -7;
  if (B == 0) return 0;
  GpkExactArgs a{X, y, hyp, n_lengthscale, B, N, D, jitter, max_tries, L, z, mll, info};
  if (N > kGpkExactRegMaxN) return gpk_launch_exact_large(a, (hipStream_t)stream);
  return gpk_launch_exact(a, (hipStream_t)stream);
}

size_t gpk_exact_grad_workspace_bytes(int B, int N) {
  if (B < 0 || N < 1 || N > gpk_exact_max_n()) return 0;
  if (N > kGpkExactRegMaxN) return gpk_exact_large_grad_ws_floats(B, N) * sizeof(float);
  return gpk_exact_grad_ws_floats(B, N) * sizeof(float);
}

int gpk_exact_mll_grad_f32(const float* X, const float* L, const float* z, const float* hyp,
                           int n_lengthscale, int B, int N, int D, const float* gout, void* workspace,
                           float* dX, float* dy, float* dhyp, void* stream) {
  if (X == nullptr) return -1;
  if (L == nullptr) return -2;
  if (z == nullptr) return -3;
  if (hyp == nullptr) return -4;
  if (n_lengthscale != 1 && n_lengthscale != D) return -5;
  if (B < 0) return -6;
  if (N < 1 || N > gpk_exact_max_n()) return -7;
  if (D < 1 || D > 64) return -8;
  if (gout == nullptr) return -9;
  if (workspace == nullptr && B > 0 && gpk_exact_grad_workspace_bytes(B, N) > 0) return -10;
  if (dhyp == nullptr) return -13;
  if (B == 0) return 0;
  GpkExactGradArgs a{X, L, z, hyp, n_lengthscale, B, N, D, gout, (float*)workspace, dX, dy, dhyp};
  if (N > kGpkExactRegMaxN) return gpk_launch_exact_large_grad(a, (hipStream_t)stream);
  return gpk_launch_exact_grad(a, (hipStream_t)stream);
}

int gpk_exact_posterior_f32(const float* X, const float* L, const float* z, const float* hyp,
                            int n_lengthscale, const float* Xs, int B, int N, int Ns, int D,
                            float* mean, float* var, void* stream) {
  if (X == nullptr) return -1;
  if (L == nullptr) return -2;
  if (z == nullptr) return -3;
  if (hyp == nullptr) return -4;
  if (n_lengthscale != 1 && n_lengthscale != D) return -5;
  if (Xs == nullptr) return -6;
  if (B < 0) return -7;
  if (N < 1 || N > gpk_exact_max_n()) return -8;
  if (Ns < 0) return -9;
  if (D < 1 || D > 64) return -10;
  if (mean == nullptr) return -11;
  if (var == nullptr) return -12;
  if (B == 0 || Ns == 0) return 0;
  GpkPostArgs a{X, L, z, hyp, n_lengthscale, Xs, B, N, Ns, D, mean, var};
  if (N > kGpkExactRegMaxN) return gpk_launch_exact_large_posterior(a, (hipStream_t)stream);
  return gpk_launch_exact_posterior(a, (hipStream_t)stream);
}

int gpk_kzz_chol_f64(const float* Z, const float* hyp, int M, int D, float jitter,
                     double chol_jitter, int max_tries, double* L, double* Linv, int* info,
                     void* stream) {
  if (Z == nullptr) return -1;
  if (hyp == nullptr) return -2;
  if (M < 1 || M > 256) return -3;
  if (D < 1 || D > 64) return -4;
  if (max_tries < 0 || max_tries > 12) return -7;
  if (L == nullptr) return -8;
  if (Linv == nullptr) return -9;
  if (info == nullptr) return -10;
  GpkKzzArgs a{Z, hyp, M, D, jitter, chol_jitter, max_tries, L, Linv, info};
  return gpk_launch_kzz16(a, (hipStream_t)stream);
}

size_t gpk_kzz_backward_workspace_bytes(int M, int D) {
  if (M < 1 || M > 256 || D < 1 || D > 64) return 0;
  return gpk_kzz_grad_ws_bytes(M, D);
}

int gpk_kzz_backward_f64(const double* dLinv, const double* L, const double* Linv, const float* Z,
                         const float* hyp, int M, int D, void* workspace, float* dZ, float* dhyp,
                         void* stream) {
  if (dLinv == nullptr) return -1;
  if (L == nullptr) return -2;
  if (Linv == nullptr) return -3;
  if (Z == nullptr) return -4;
  if (hyp == nullptr) return -5;
  if (M < 1 || M > 256) return -6;
  if (D < 1 || D > 64) return -7;
  if (workspace == nullptr) return -8;
  if (dZ == nullptr) return -9;
  if (dhyp == nullptr) return -10;
  GpkKzzGradArgs a{dLinv, L, Linv, Z, hyp, M, D, workspace, dZ, dhyp};
  return gpk_launch_kzz_grad(a, (hipStream_t)stream);
}

int gpk_gauss_ell_f32(const float* y, const float* mean, const float* var, const float* noise, int R,
                      int N, float* ell, void* stream) {
  if (y == nullptr) return -1;
  if (mean == nullptr) return -2;
  if (var == nullptr) return -3;
  if (noise == nullptr) return -4;
  if (R < 0) return -5;
  if (N < 1) return -6;
  if (ell == nullptr) return -7;
  if (R == 0) return 0;
  return gpk_launch_ell(y, mean, var, noise, R, N, ell, (hipStream_t)stream);
}

int gpk_gauss_ell_grad_f32(const float* y, const float* mean, const float* var, const float* noise,
                           const float* gell, int R, int N, float* dy, float* dmean, float* dvar,
                           float* dnoise_part, void* stream) {
  if (y == nullptr) return -1;
  if (mean == nullptr) return -2;
  if (var == nullptr) return -3;
  if (noise == nullptr) return -4;
  if (gell == nullptr) return -5;
  if (R < 0) return -6;
  if (N < 1) return -7;
  if (R == 0) return 0;
  return gpk_launch_ell_grad(y, mean, var, noise, gell, R, N, dy, dmean, dvar, dnoise_part,
                             (hipStream_t)stream);
}

int gpk_meanfield_kl_f32(const float* m, const float* s, int M, float* kl, const float* gkl,
                         float* dm, float* ds, void* stream) {
  if (m == nullptr) return -1;
  if (s == nullptr) return -2;
  if (M < 1) return -3;
  if (gkl == nullptr && kl == nullptr) return -4;
  if (gkl != nullptr && (dm == nullptr || ds == nullptr)) return -6;
  return gpk_launch_kl(m, s, M, kl, gkl, dm, ds, (hipStream_t)stream);
}

int gpk_variational_elbo_f32(const float* y, long long ldy, const float* mean, long long ldm,
                             const float* var, long long ldv, const float* noise, const float* m,
                             const float* s, int M, int R, int N, float kl_scale, float min_var,
                             float* elbo, int* clamp_flag, void* stream) {
  if (y == nullptr) return -1;
  if (ldy < N) return -2;
  if (mean == nullptr) return -3;
  if (ldm < N) return -4;
  if (var == nullptr) return -5;
  if (ldv < N) return -6;
  if (noise == nullptr) return -7;
  if (m == nullptr) return -8;
  if (s == nullptr) return -9;
  if (M < 1) return -10;
  if (R < 0) return -11;
  if (N < 1) return -12;
  if (elbo == nullptr) return -15;
  if (R == 0) return 0;
  return gpk_launch_elbo(y, ldy, mean, ldm, var, ldv, noise, m, s, M, R, N, kl_scale, min_var, elbo,
                         clamp_flag, (hipStream_t)stream);
}

int gpk_variational_elbo_grad_f32(const float* y, long long ldy, const float* mean, long long ldm,
                                  const float* var, long long ldv, const float* noise, const float* m,
                                  const float* s, int M, int R, int N, float kl_scale, const float* gelbo,
                                  float* dmean, float* dvar, float* dnoise_part, float* dm, float* ds,
                                  void* stream) {
  if (y == nullptr) return -1;
  if (ldy < N) return -2;
  if (mean == nullptr) return -3;
  if (ldm < N) return -4;
  if (var == nullptr) return -5;
  if (ldv < N) return -6;
  if (noise == nullptr) return -7;
  if (m == nullptr) return -8;
  if (s == nullptr) return -9;
  if (M < 1) return -10;
  if (R < 0) return -11;
  if (N < 1) return -12;
  if (R > 0 && gelbo == nullptr) return -14;
  if (dm == nullptr || ds == nullptr || (R > 0 && (dmean == nullptr || dvar == nullptr || dnoise_part == nullptr)))
    return -15;
  if (R == 0) {
    // an empty batch (the forward's no-op): no rows, and the KL enters scaled by sum g = 0
    hipError_t e = hipMemsetAsync(dm, 0, sizeof(float) * (size_t)M, (hipStream_t)stream);
    if (e == hipSuccess) e = hipMemsetAsync(ds, 0, sizeof(float) * (size_t)M, (hipStream_t)stream);
    return e == hipSuccess ? 0 : (int)e;
  }
  return gpk_launch_elbo_grad(y, ldy, mean, ldm, var, ldv, noise, m, s, M, R, N, kl_scale, gelbo, dmean,
                              dvar, dnoise_part, dm, ds, (hipStream_t)stream);
}

int gpk_record_check(const int* info, int n, const float* in0, long long n0, const float* in1,
                     long long n1, int kind, int* ring, long long* counter, int slots, int item,
                     int items, int* sticky, void* stream) {
  if (kind < 0 || kind > 2) return -7;
  if (kind != 2 && info == nullptr) return -1;
  if (kind == 0 && (n < 1 || (n0 > 0 && in0 == nullptr) || (n1 > 0 && in1 == nullptr))) return -2;
  if (ring == nullptr && kind != 2) return -8;
  if (counter == nullptr) return -9;
  if (slots < 1) return -10;
  if (kind != 2 && (item < 0 || item >= items)) return -11;
  if (kind == 0 && sticky == nullptr) return -13;
  return gpk_launch_verdict(info, n, in0, n0, in1, n1, kind, ring, counter, slots, item, items, sticky,
                            kind == 2, (hipStream_t)stream);
}

int gpk_variational_f32(const float* X, const float* Z, const double* Linv, const float* vmean,
                        const float* vstd, const float* hyp, const float* y, int B, int N, int M,
                        int D, float* mean, float* var, float* ell, int* flags, void* stream) {
  if (X == nullptr) return -1;
  if (Z == nullptr) return -2;
  if (Linv == nullptr) return -3;
  if (vmean == nullptr) return -4;
  if (vstd == nullptr) return -5;
  if (hyp == nullptr) return -6;
  if (B < 0) return -8;
  if (N < 1) return -9;
  if (M < 1 || M > 256) return -10;
  if (D < 1 || D > 64) return -11;
  if (mean == nullptr) return -12;
  if (var == nullptr) return -13;
  if (ell != nullptr && y == nullptr) return -7;
  if (B == 0) return 0;
  GpkVarArgs a{X, Z, Linv, vmean, vstd, hyp, y, B, N, M, D, mean, var, ell};
  return gpk_launch_var(a, flags, (hipStream_t)stream);
}

size_t gpk_variational_saved_bytes(int B, int N, int M, int D) {
  if (B < 1 || N < 1 || M < 1 || M > 256 || D < 1 || D > 64) return 0;
  return gpk_var_saved_bytes(B, N, M, D);
}
int gpk_variational_train_f32(const float* X, const float* Z, const double* Linv, const float* vmean,
                              const float* vstd, const float* hyp, const float* y, int B, int N, int M,
                              int D, float* mean, float* var, float* ell, int* flags, void* saved,
                              void* stream) {
  if (X == nullptr) return -1;
  if (Z == nullptr) return -2;
  if (Linv == nullptr) return -3;
  if (vmean == nullptr) return -4;
  if (vstd == nullptr) return -5;
  if (hyp == nullptr) return -6;
  if (B < 0) return -8;
  if (N < 1) return -9;
  if (M < 1 || M > 256) return -10;
  if (D < 1 || D > 64) return -11;
  if (mean == nullptr) return -12;
  if (var == nullptr) return -13;
  if (ell != nullptr && y == nullptr) return -7;
  if (saved == nullptr && gpk_var_saved_bytes(B, N, M, D) > 0) return -16;
  if (B == 0) return 0;
  GpkVarArgs a{X, Z, Linv, vmean, vstd, hyp, y, B, N, M, D, mean, var, ell, (float*)saved};
  return gpk_launch_var(a, flags, (hipStream_t)stream);
}
size_t gpk_variational_adjoint_saved_workspace_bytes(int B, int N, int M, int D) {
  if (B < 1 || N < 1 || M < 1 || M > 256 || D < 1 || D > 64) return 0;
  return gpk_var_adjoint_saved_ws_bytes(B, N, M, D);
}
int gpk_variational_adjoint_saved_f32(const float* X, const float* Z, const double* Linv,
                                      const float* vmean, const float* vstd, const float* hyp,
                                      const float* gmean, const float* gvar, const void* saved, int B,
                                      int N, int M, int D, void* workspace, float* dX, double* dLinv,
                                      float* dZ, float* dpar, void* stream) {
  if (X == nullptr) return -1;
  if (Z == nullptr) return -2;
  if (Linv == nullptr) return -3;
  if (vmean == nullptr) return -4;
  if (vstd == nullptr) return -5;
  if (hyp == nullptr) return -6;
  if (gmean == nullptr) return -7;
  if (gvar == nullptr) return -8;
  if (saved == nullptr) return -9;
  if (B < 1) return -10;
  if (N < 1) return -11;
  if (M < 1 || M > 256) return -12;
  if (D < 1 || D > 64) return -13;
  if (gpk_var_saved_bytes(B, N, M, D) == 0) return -12;
  if (workspace == nullptr) return -14;
  if (dX == nullptr) return -15;
  if (dLinv == nullptr) return -16;
  if (dZ == nullptr) return -17;
  if (dpar == nullptr) return -18;
  GpkVarAdjArgs a{X, Z, Linv, vmean, vstd, hyp, gmean, gvar, B, N, M, D, workspace, dX, dLinv, dZ, dpar,
                  (const float*)saved};
  return gpk_launch_var_adjoint(a, (hipStream_t)stream);
}
size_t gpk_variational_adjoint_workspace_bytes(int B, int N, int M, int D) {
  if (B < 1 || N < 1 || M < 1 || M > 256 || D < 1 || D > 64) return 0;
  return gpk_var_adjoint_ws_bytes(B, N, M, D);
}

int gpk_variational_adjoint_f32(const float* X, const float* Z, const double* Linv,
                                const float* vmean, const float* vstd, const float* hyp,
                                const float* gmean, const float* gvar, int B, int N, int M, int D,
                                void* workspace, float* dX, double* dLinv, float* dZ, float* dpar,
                                void* stream) {
  if (X == nullptr) return -1;
  if (Z == nullptr) return -2;
  if (Linv == nullptr) return -3;
  if (vmean == nullptr) return -4;
  if (vstd == nullptr) return -5;
  if (hyp == nullptr) return -6;
  if (gmean == nullptr) return -7;
  if (gvar == nullptr) return -8;
  if (B < 1) return -9;
  if (N < 1) return -10;
  if (M < 1 || M > 256) return -11;
  if (D < 1 || D > 64) return -12;
  if (workspace == nullptr) return -13;
  if (dX == nullptr) return -14;
  if (dLinv == nullptr) return -15;
  if (dZ == nullptr) return -16;
  if (dpar == nullptr) return -17;
  GpkVarAdjArgs a{X, Z, Linv, vmean, vstd, hyp, gmean, gvar, B, N, M, D, workspace, dX, dLinv, dZ, dpar};
  return gpk_launch_var_adjoint(a, (hipStream_t)stream);
}

int gpk_window_gather_f32(const float* table, long long n_rows, int F, const long long* rows, int B,
                          int T, int n_enc, int pred_len, int target_col, float* enc, float* dec,
                          float* y, void* stream) {
  if (table == nullptr) return -1;
  if (n_rows < 0) return -2;
  if (F < 1) return -3;
  if (rows == nullptr && B > 0) return -4;
  if (B < 0) return -5;
  if (T < 1) return -6;
  if (n_enc < 0 || n_enc > T) return -7;
  if (pred_len < 0 || n_enc + pred_len > T) return -8;
  if (target_col < 0 || target_col >= F) return -9;
  if (enc == nullptr && B > 0 && n_enc > 0) return -10;
  if (dec == nullptr && B > 0 && T - n_enc - pred_len > 0) return -11;
  if (y == nullptr && B > 0 && pred_len > 0) return -12;
  if (B == 0) return 0;
  return gpk_launch_window_gather(table, F, rows, B, n_enc, T - n_enc - pred_len, pred_len,
                                  target_col, enc, dec, y, (hipStream_t)stream);
}

// Diagnostic (not part of the product ABI): same as gpk_exact_mll_f32 for N in
// (240, 256], plus per-workgroup phase clocks and a per-step timeline (32 + 1024 x u64 per window) in `stamps`.
int gpk_debug_exact_stamps(const float* X, const float* y, const float* hyp, int n_lengthscale,
                           int B, int N, int D, double jitter, int max_tries, float* L, float* z,
                           float* mll, int* info, unsigned long long* stamps, void* stream) {
  GpkExactArgs a{X, y, hyp, n_lengthscale, B, N, D, jitter, max_tries, L, z, mll, info};
  return gpk_launch_exact_stamps(a, stamps, (hipStream_t)stream);
}

}  // extern "C"
