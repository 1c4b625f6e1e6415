// Calibration: cycles of readlane / dpp / fma / pk_fma streams for one wave.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float f32x2 __attribute__((ext_vector_type(2)));
template <int I> __device__ __forceinline__ float rl(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), I));
}
template <int I> __device__ __forceinline__ float bc(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0x150 + I, 0xf, 0xf, true));
}
#define R16(X) X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7) X(8) X(9) X(10) X(11) X(12) X(13) X(14) X(15)
__global__ void k_readlane(float* o, unsigned long long* cyc, int reps) {
  float a = threadIdx.x * 0.001f, v[16];
  for (int i = 0; i < 16; ++i) v[i] = i * 0.5f + a;
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int r = 0; r < reps; ++r) {
    float s[16];
#define X(I) s[I] = rl<I>(a);
    R16(X)
#undef X
    asm volatile("" : "+s"(s[0]), "+s"(s[1]), "+s"(s[2]), "+s"(s[3]), "+s"(s[4]), "+s"(s[5]), "+s"(s[6]), "+s"(s[7]), "+s"(s[8]), "+s"(s[9]), "+s"(s[10]), "+s"(s[11]), "+s"(s[12]), "+s"(s[13]), "+s"(s[14]), "+s"(s[15]));
    for (int i = 0; i < 16; ++i) v[i] = __builtin_fmaf(-s[i], a, v[i]);
    a = v[r & 15] * 0.5f;
  }
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  float acc = 0; for (int i = 0; i < 16; ++i) acc += v[i];
  o[threadIdx.x] = acc;
  if (threadIdx.x == 0) cyc[0] = (t1 - t0) / reps;
}
__global__ void k_dpp(float* o, unsigned long long* cyc, int reps) {
  float a = threadIdx.x * 0.001f, v[16];
  for (int i = 0; i < 16; ++i) v[i] = i * 0.5f + a;
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int r = 0; r < reps; ++r) {
    float s[16];
#define X(I) s[I] = bc<I>(a);
    R16(X)
#undef X
    for (int i = 0; i < 16; i += 2) {
      f32x2 vv = {v[i], v[i + 1]}; f32x2 ss = {-s[i], -s[i + 1]}; f32x2 aa = {a, a};
      vv = __builtin_elementwise_fma(ss, aa, vv); v[i] = vv[0]; v[i + 1] = vv[1];
    }
    a = v[r & 15] * 0.5f;
  }
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  float acc = 0; for (int i = 0; i < 16; ++i) acc += v[i];
  o[threadIdx.x] = acc;
  if (threadIdx.x == 0) cyc[0] = (t1 - t0) / reps;
}
__global__ void k_fma(float* o, unsigned long long* cyc, int reps) {
  float a = threadIdx.x * 0.001f, v[16];
  for (int i = 0; i < 16; ++i) v[i] = i * 0.5f + a;
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int r = 0; r < reps; ++r) {
    for (int i = 0; i < 16; ++i) v[i] = __builtin_fmaf(v[(i + 1) & 15], a, v[i]);
    a = v[r & 15] * 0.5f;
  }
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  float acc = 0; for (int i = 0; i < 16; ++i) acc += v[i];
  o[threadIdx.x] = acc;
  if (threadIdx.x == 0) cyc[0] = (t1 - t0) / reps;
}
__global__ void k_rsq(float* o, unsigned long long* cyc, int reps) {
  float a = threadIdx.x * 0.001f + 1.f;
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int r = 0; r < reps; ++r) {
    float p = rl<3>(a);
    float rs = __builtin_amdgcn_rsqf(p);
    a = a * rs + 1.0f;
  }
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  o[threadIdx.x] = a;
  if (threadIdx.x == 0) cyc[0] = (t1 - t0) / reps;
}
int main() {
  float* d; unsigned long long* c; hipMalloc(&d, 4096); hipMalloc(&c, 64);
  unsigned long long h;
  const int reps = 1000;
  hipLaunchKernelGGL(k_readlane, dim3(1), dim3(64), 0, 0, d, c, reps); hipMemcpy(&h, c, 8, hipMemcpyDeviceToHost);
  printf("16 readlane + 16 fma: %llu cycles/iter\n", h);
  hipLaunchKernelGGL(k_dpp, dim3(1), dim3(64), 0, 0, d, c, reps); hipMemcpy(&h, c, 8, hipMemcpyDeviceToHost);
  printf("16 dpp-bcast + 8 pk_fma: %llu cycles/iter\n", h);
  hipLaunchKernelGGL(k_fma, dim3(1), dim3(64), 0, 0, d, c, reps); hipMemcpy(&h, c, 8, hipMemcpyDeviceToHost);
  printf("16 dependent-ish fma: %llu cycles/iter\n", h);
  hipLaunchKernelGGL(k_rsq, dim3(1), dim3(64), 0, 0, d, c, reps); hipMemcpy(&h, c, 8, hipMemcpyDeviceToHost);
  printf("readlane->rsq->fma chain: %llu cycles/iter\n", h);
  return 0;
}
