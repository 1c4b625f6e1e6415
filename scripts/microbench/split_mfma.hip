// Accuracy check of the split-f16 tile product (gpk_common.h::mma_tn_split)
// against mma_tn (f32 MFMA) and an fp64 host reference. Diagnostic only.
#include "../../fine_grained_gaussian_process_forcasting_amd/csrc/gpk_common.h"
#include <cstdio>
#include <cstdlib>
#include <cmath>
#include <vector>

__global__ void k(const float* Q, const float* P, float* Df, float* Ds, float* Dr) {
  __shared__ float tq[256], tp[256];
  const int lane = threadIdx.x, c = lane & 15, g = lane >> 4;
  f32x4 q, p;
  for (int r = 0; r < 4; ++r) { q[r] = Q[(4 * g + r) * 16 + c]; p[r] = P[(4 * g + r) * 16 + c]; }
  f32x4 df = mma_tn(q, p, f32x4{0, 0, 0, 0});
  store_split_f16(tq, lane, q);
  store_split_f16(tp, lane, p);
  __syncthreads();
  f32x4 ds = mma_tn_split(load_split_hl(tq, lane), load_split_lh(tp, lane), f32x4{0, 0, 0, 0});
  // reconstructed operand (hi + lo) to measure representation error
  half8_t h = load_split_hl(tq, lane);
  for (int r = 0; r < 4; ++r) {
    Df[(4 * g + r) * 16 + c] = df[r];
    Ds[(4 * g + r) * 16 + c] = ds[r];
    Dr[(4 * g + r) * 16 + c] = (float)h[r] + (float)h[4 + r];
  }
}

int main(int argc, char** argv) {
  srand(1);
  const float amp = argc > 1 ? atof(argv[1]) : 200.f;
  const int T = 20;
  double emax_f = 0, emax_s = 0, erep = 0;
  for (int t = 0; t < T; ++t) {
    std::vector<float> Q(256), P(256);
    for (int i = 0; i < 256; ++i) {
      Q[i] = (rand() / (float)RAND_MAX - 0.5f) * amp;
      P[i] = (rand() / (float)RAND_MAX - 0.5f) * amp;
    }
    float *dQ, *dP, *dF, *dS, *dR;
    hipMalloc(&dQ, 1024); hipMalloc(&dP, 1024); hipMalloc(&dF, 1024); hipMalloc(&dS, 1024); hipMalloc(&dR, 1024);
    hipMemcpy(dQ, Q.data(), 1024, hipMemcpyHostToDevice);
    hipMemcpy(dP, P.data(), 1024, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, dQ, dP, dF, dS, dR);
    std::vector<float> F(256), S(256), R(256);
    hipMemcpy(F.data(), dF, 1024, hipMemcpyDeviceToHost);
    hipMemcpy(S.data(), dS, 1024, hipMemcpyDeviceToHost);
    hipMemcpy(R.data(), dR, 1024, hipMemcpyDeviceToHost);
    double nrm = 0;
    for (int m = 0; m < 16; ++m)
      for (int n = 0; n < 16; ++n) {
        double ref = 0;
        for (int kk = 0; kk < 16; ++kk) ref += (double)Q[kk * 16 + m] * P[kk * 16 + n];
        nrm = fmax(nrm, fabs(ref));
        emax_f = fmax(emax_f, fabs(F[m * 16 + n] - ref));
        emax_s = fmax(emax_s, fabs(S[m * 16 + n] - ref));
        if (t == 0 && m < 2 && n < 3) printf("ref %.9g f32 %.9g split %.9g\n", ref, F[m * 16 + n], S[m * 16 + n]);
      }
    for (int i = 0; i < 256; ++i) erep = fmax(erep, fabs(R[i] - Q[i]) / fabs(Q[i]));
    emax_f /= 1.0; 
    if (t == 0) printf("scale (max |ref|) %.3g\n", nrm);
    hipFree(dQ); hipFree(dP); hipFree(dF); hipFree(dS); hipFree(dR);
  }
  printf("amp %g: max abs err: f32 %.3e  split %.3e   max rel repr err (hi+lo vs x) %.3e\n", amp, emax_f, emax_s, erep);
  return 0;
}
