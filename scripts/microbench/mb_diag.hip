// Microbenchmark: cycles of the exact kernel's 16x16 diagonal-tile sweep
// (diag_sweep<0>, readlane form) and of the DPP/permlane form, for one wave
// alone and beside "hog" waves on the same / other SIMDs.
// Build: hipcc -O3 -std=c++17 --offload-arch=gfx950 -I../../include mb_diag.hip -o mb_diag
#include "../../fine_grained_gaussian_process_forcasting_amd/csrc/gpk_exact.hip"
#include <cstdio>
#include <vector>

namespace mbd {
template <int I>
GPK_DEVICE float bcast_row(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0x150 + I, 0xf, 0xf, true));
}
GPK_DEVICE float rep01(float v) {
  auto r = __builtin_amdgcn_permlane16_swap(__builtin_bit_cast(int, v), __builtin_bit_cast(int, v), false, false);
  return __builtin_bit_cast(float, (int)r[0]);
}
template <int I, int M>
GPK_DEVICE void dupd(float (&v)[16], float r) {
  if constexpr (I < 16) {
    const float b = bcast_row<I>(r);
    v[I] = __builtin_fmaf(-b, v[M], v[I]);
    dupd<I + 1, M>(v, r);
  }
}
template <int M>
GPK_DEVICE void dsweep(float (&v)[16]) {
  __builtin_amdgcn_sched_barrier(0);
  const float rowm = rep01(v[M]);
  const float piv = bcast_row<M>(rowm);
  const float rs = __builtin_amdgcn_rsqf(piv);
  const float r = rowm * rs;
  v[M] = v[M] * rs;
  dupd<M + 1, M>(v, r);
#pragma unroll
  for (int i = M; i < 16; ++i) asm volatile("" : "+v"(v[i]));
  if constexpr (M < 15) dsweep<M + 1>(v);
}
}  // namespace mbd

// hog kinds: 0 none, 1 back-to-back f16 MFMA (4 chains), 2 MFMA + LDS reads, 3 VALU exp/fma
template <int SWEEP>
__global__ void __launch_bounds__(1024) kdiag(const float* in, float* out, unsigned long long* cyc,
                                              unsigned* hw, int reps, int hog_kind, int hog_sel, int prio) {
  __shared__ int simd_of[16];
  __shared__ volatile int done;
  __shared__ __attribute__((aligned(16))) float lbuf[4096];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const unsigned hwid = __builtin_amdgcn_s_getreg(4 | (31 << 11));
  const int simd = (hwid >> 4) & 3;
  if (lane == 0) {
    simd_of[wave] = simd;
    hw[blockIdx.x * 16 + wave] = hwid;
  }
  for (int i = threadIdx.x; i < 4096; i += blockDim.x) lbuf[i] = 0.001f * (i & 63);
  if (threadIdx.x == 0) done = 0;
  __syncthreads();
  if (wave == 0) {
    if (prio) __builtin_amdgcn_s_setprio(3);
    const int c = lane & 15, grp = lane >> 4;
    float v[16];
    for (int i = 0; i < 16; ++i) {
      const float t = in[(4 * i + c) & 255];
      v[i] = (grp == 0 || grp == 2) ? t + (i == c ? 16.f : 0.f) : (i == c ? 1.f : 0.f);
    }
    for (int i = 0; i < 16; ++i) v[i] = (grp == 0 || grp == 2) ? (v[i] + in[(4 * c + i) & 255]) * 0.5f + (i == c ? 16.f : 0.f) : v[i];
    unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int r = 0; r < reps; ++r) {
      float w[16];
      for (int i = 0; i < 16; ++i) w[i] = v[i];
      if constexpr (SWEEP == 0) diag_sweep<0>(w);
      else if constexpr (SWEEP == 1) mbd::dsweep<0>(w);
      else diag_sweep_dpp(w);
      v[0] += w[15] * 1e-30f;
    }
    unsigned long long t1 = __builtin_amdgcn_s_memtime();
    if (lane == 0) cyc[blockIdx.x] = (t1 - t0) / reps;
    done = 1;
    float s = 0.f;
    for (int i = 0; i < 16; ++i) s += v[i];
    out[blockIdx.x * 64 + lane] = s;
    __builtin_amdgcn_s_setprio(0);
    return;
  }
  bool hog = false;
  if (hog_sel == 0) hog = true;                       // every other wave
  else if (hog_sel == 1) hog = simd == simd_of[0];    // same SIMD as the sweep wave
  else hog = simd != simd_of[0];                      // other SIMDs only
  if (!hog || hog_kind == 0) return;
  f32x4 a0 = {0, 0, 0, 0}, a1 = a0, a2 = a0, a3 = a0;
  half8_t x = {(_Float16)0.01f, (_Float16)0.02f, (_Float16)0.01f, (_Float16)0.02f,
               (_Float16)0.01f, (_Float16)0.02f, (_Float16)0.01f, (_Float16)0.02f};
  float e = lane * 1e-3f;
  for (int it = 0; it < (1 << 20); ++it) {
    if (done) break;
    if (hog_kind == 1) {
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        a0 = __builtin_amdgcn_mfma_f32_16x16x32_f16(x, x, a0, 0, 0, 0);
        a1 = __builtin_amdgcn_mfma_f32_16x16x32_f16(x, x, a1, 0, 0, 0);
        a2 = __builtin_amdgcn_mfma_f32_16x16x32_f16(x, x, a2, 0, 0, 0);
        a3 = __builtin_amdgcn_mfma_f32_16x16x32_f16(x, x, a3, 0, 0, 0);
      }
    } else if (hog_kind == 2) {
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const half8_t p = *(const half8_t*)&lbuf[((u * 64 + lane) * 4) & 4095];
        const half8_t q = *(const half8_t*)&lbuf[((u * 64 + lane + 512) * 4) & 4095];
        a0 = __builtin_amdgcn_mfma_f32_16x16x32_f16(p, q, a0, 0, 0, 0);
        a0 = __builtin_amdgcn_mfma_f32_16x16x32_f16(q, p, a0, 0, 0, 0);
      }
    } else {
#pragma unroll
      for (int u = 0; u < 16; ++u) e = __builtin_fmaf(__builtin_amdgcn_exp2f(e), 1e-3f, 0.5f);
    }
  }
  out[4096 + blockIdx.x * 1024 + threadIdx.x] = a0[0] + a1[1] + a2[2] + a3[3] + e;
}

int main() {
  std::vector<float> hin(256);
  for (int i = 0; i < 256; ++i) hin[i] = 0.1f / (1 + (i % 17));
  float *din, *dout;
  unsigned long long* dc;
  unsigned* dhw;
  const int BL = 256;
  hipMalloc(&din, 1024);
  hipMalloc(&dout, (4096 + BL * 1024) * 4);
  hipMalloc(&dc, 8 * BL);
  hipMalloc(&dhw, 4 * 16 * BL);
  hipMemcpy(din, hin.data(), 1024, hipMemcpyHostToDevice);
  const char* hogn[] = {"none", "mfma", "mfma+lds", "valu-exp"};
  const char* seln[] = {"all", "same-simd", "other-simd"};
  for (int sweep = 0; sweep < 3; ++sweep) {
    for (int prio = 0; prio < 1; ++prio) {
      for (int kind = 0; kind < 4; ++kind) {
        for (int sel = 0; sel < 3; ++sel) {
          if (kind == 0 && sel > 0) continue;
          const int threads = kind == 0 ? 64 : 1024;
          for (int rep = 0; rep < 2; ++rep) {
            if (sweep == 0)
              hipLaunchKernelGGL(kdiag<0>, dim3(BL), dim3(threads), 0, 0, din, dout, dc, dhw, 200, kind, sel, prio);
            else if (sweep == 1)
              hipLaunchKernelGGL(kdiag<1>, dim3(BL), dim3(threads), 0, 0, din, dout, dc, dhw, 200, kind, sel, prio);
            else
              hipLaunchKernelGGL(kdiag<2>, dim3(BL), dim3(threads), 0, 0, din, dout, dc, dhw, 200, kind, sel, prio);
          }
          hipDeviceSynchronize();
          std::vector<unsigned long long> c(BL);
          hipMemcpy(c.data(), dc, 8 * BL, hipMemcpyDeviceToHost);
          double s = 0;
          for (auto v : c) s += v;
          printf("sweep=%d prio=%d hog=%-9s sel=%-10s cycles/sweep %.0f\n", sweep, prio,
                 hogn[kind], seln[sel], s / BL);
        }
      }
    }
  }
  // SIMD mapping of a 16-wave block
  std::vector<unsigned> hw(16 * BL);
  hipLaunchKernelGGL(kdiag<0>, dim3(BL), dim3(1024), 0, 0, din, dout, dc, dhw, 2, 0, 0, 0);
  hipDeviceSynchronize();
  hipMemcpy(hw.data(), dhw, 4 * 16 * BL, hipMemcpyDeviceToHost);
  for (int b = 0; b < 4; ++b) {
    printf("block %d simd per wave:", b);
    for (int w = 0; w < 16; ++w) printf(" %u", (hw[b * 16 + w] >> 4) & 3);
    printf("\n");
  }
  // numeric check: both sweeps on the same tile
  float* o2;
  hipMalloc(&o2, (4096 + BL * 1024) * 4);
  hipLaunchKernelGGL(kdiag<0>, dim3(1), dim3(64), 0, 0, din, dout, dc, dhw, 1, 0, 0, 0);
  hipLaunchKernelGGL(kdiag<2>, dim3(1), dim3(64), 0, 0, din, o2, dc, dhw, 1, 0, 0, 0);
  hipDeviceSynchronize();
  std::vector<float> r0(64), r1(64);
  hipMemcpy(r0.data(), dout, 256, hipMemcpyDeviceToHost);
  hipMemcpy(r1.data(), o2, 256, hipMemcpyDeviceToHost);
  double md = 0;
  for (int l = 0; l < 32; ++l) md = fmax(md, fabs(r0[l] - r1[l]));
  printf("readlane vs asm-dpp max |diff| over lanes 0-31: %.3e (lane0 %.6f %.6f)\n", md, r0[0], r1[0]);
  return 0;
}
