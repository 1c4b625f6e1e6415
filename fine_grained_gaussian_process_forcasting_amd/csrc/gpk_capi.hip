// C-ABI shim: argument validation + dispatch to the gfx950 kernels.
// Declarations and the reference interfaces each entry point replaces: include/gpk.h.
#include "../../include/gpk.h"
#include "gpk_internal.h"

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

int gpk_exact_max_n(void) { return 256; }

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
  if (B == 0) return 0;
  GpkExactArgs a{X, y, hyp, n_lengthscale, B, N, D, jitter, max_tries, L, z, mll, info};
  return gpk_launch_exact(a, (hipStream_t)stream);
}

// Diagnostic (not part of the product ABI): same as gpk_exact_mll_f32 for N in
// (240, 256], plus per-workgroup phase clocks (16 x u64 per window) in `stamps`.
int gpk_debug_exact_stamps(const float* X, const float* y, const float* hyp, int n_lengthscale,
                           int B, int N, int D, double jitter, int max_tries, float* L, float* z,
                           float* mll, int* info, unsigned long long* stamps, void* stream) {
  GpkExactArgs a{X, y, hyp, n_lengthscale, B, N, D, jitter, max_tries, L, z, mll, info};
  return gpk_launch_exact_stamps(a, stamps, (hipStream_t)stream);
}

}  // extern "C"
