// Microbenchmark: cycles of one 16x16 diagonal-tile factorisation in one wave.
// Build: hipcc -O3 --offload-arch=gfx950 -I../../include -I../../fine_grained_gaussian_process_forcasting_amd/csrc diag_mb.hip -o diag_mb
#include "gpk_common.h"
#include <cstdio>
#include <vector>

#define DIAG_ONLY
namespace mb {
#include "diag_factor_impl.inc"
#include "diag_dpp.inc"
}
__global__ void kern_dpp(const float* in, float* out, unsigned long long* cyc, int reps) {
  const int lane = threadIdx.x & 63;
  const int c = lane & 15, grp = lane >> 4;
  float v[16];
  for (int i = 0; i < 16; ++i) v[i] = in[(lane * 4 + i) & 255];
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int r = 0; r < reps; ++r) {
    mb::dsweep<0>(v);
    v[0] += 1e-30f;
  }
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  float s = 0; for (int i = 0; i < 16; ++i) s += v[i];
  out[lane] = s;
  if (lane == 0) cyc[blockIdx.x] = (t1 - t0) / reps;
}

__global__ void kern(const float* in, float* out, unsigned long long* cyc, int reps) {
  __shared__ __attribute__((aligned(16))) float dsc[256];
  __shared__ __attribute__((aligned(16))) float wbuf[256];
  const int lane = threadIdx.x & 63;
  f32x4 a = *(const f32x4*)&in[lane * 4];
  float logdet = 0.f;
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  int f = 0;
  for (int r = 0; r < reps; ++r) {
    f += mb::diag_factor(a, dsc, wbuf, nullptr, 256, 0, logdet);
    a[0] += wbuf[lane] * 1e-30f;
  }
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  out[lane] = logdet + f + wbuf[lane];
  if (lane == 0) cyc[blockIdx.x] = (t1 - t0) / reps;
}

int main() {
  // SPD tile: T = I*16 + small symmetric, given negated in acc layout
  std::vector<float> T(256), acc(256);
  for (int i = 0; i < 16; ++i) for (int j = 0; j < 16; ++j) T[i * 16 + j] = (i == j ? 16.f : 0.f) + 0.1f / (1 + i + j);
  for (int l = 0; l < 64; ++l) for (int r = 0; r < 4; ++r) acc[l * 4 + r] = -T[(4 * (l >> 4) + r) * 16 + (l & 15)];
  float *din, *dout; unsigned long long* dc;
  hipMalloc(&din, 1024); hipMalloc(&dout, 1024); hipMalloc(&dc, 8 * 1024);
  hipMemcpy(din, acc.data(), 1024, hipMemcpyHostToDevice);
  for (int blocks : {1, 256, 1024}) {
    hipLaunchKernelGGL(kern, dim3(blocks), dim3(64), 0, 0, din, dout, dc, 100);
    hipDeviceSynchronize();
    std::vector<unsigned long long> c(blocks);
    hipMemcpy(c.data(), dc, 8 * blocks, hipMemcpyDeviceToHost);
    double s = 0; for (auto v : c) s += v;
    printf("blocks=%d avg cycles per diag_factor: %.0f\n", blocks, s / blocks);
    hipLaunchKernelGGL(kern_dpp, dim3(blocks), dim3(64), 0, 0, din, dout, dc, 100);
    hipDeviceSynchronize();
    hipMemcpy(c.data(), dc, 8 * blocks, hipMemcpyDeviceToHost);
    s = 0; for (auto v : c) s += v;
    printf("blocks=%d avg cycles per dpp sweep only: %.0f\n", blocks, s / blocks);
  }
  return 0;
}
