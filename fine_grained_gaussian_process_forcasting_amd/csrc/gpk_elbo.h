// Launchers of gpk_elbo.hip (the ELBO terms), for the C-ABI shim.
#pragma once
#include <hip/hip_runtime.h>

int gpk_launch_ell(const float* y, const float* mean, const float* var, const float* noise, int R,
                   int N, float* ell, hipStream_t stream);
int gpk_launch_ell_grad(const float* y, const float* mean, const float* var, const float* noise,
                        const float* gell, int R, int N, float* dy, float* dmean, float* dvar,
                        float* dnoise_part, hipStream_t stream);
int gpk_launch_kl(const float* m, const float* s, int M, float* kl, const float* gkl, float* dm,
                  float* ds, hipStream_t stream);
int gpk_launch_verdict(const int* info, int n, const float* in0, long long n0, const float* in1,
                       long long n1, int kind, int* ring, long long* counter, int slots, int item,
                       int items, int* sticky, int advance, hipStream_t stream);
int gpk_launch_elbo(const float* y, long long ldy, const float* mean, long long ldm, const float* var,
                    long long ldv, const float* noise, const float* m, const float* s, int M, int R, int N,
                    float kl_scale, float min_var, float* elbo, int* clamp_flag, hipStream_t stream);
int gpk_launch_elbo_grad(const float* y, long long ldy, const float* mean, long long ldm, const float* var,
                         long long ldv, const float* noise, const float* m, const float* s, int M, int R,
                         int N, float kl_scale, const float* g, float* dmean, float* dvar, float* dnoise_part,
                         float* dm, float* ds, hipStream_t stream);
