// Shared inducing-point factorisation K_ZZ + jitter = L L^T (fp64) and L^{-1}, once per
// optimizer step (include/gpk.h::gpk_kzz_chol_f64).
//
// Reference: VariationalStrategy._cholesky_factor -> psd_safe_cholesky (fp64 ladder 1e-8 x10^t)
// for ToyDeepGPHiddenLayer (denoising_model/DeepGP.py:33-38 via upstream
// variational_strategy.py); the reference runs it b times per GP call (Z expanded over the
// batch). oracle/gp_oracle.py::kzz_factor restates it.
//
// gpk_kzz16_kernel<NS>: ONE workgroup of 8 waves; the UPPER triangle of K_ZZ (padded to
// T 16-blocks, identity padding) is held as 16 x 16 fp64 tiles in v_mfma_f64_16x16x4f64
// accumulators (acc layout: lane (c, g), reg r <-> row g + 4r, column c), NS tiles per
// wave, for the whole factorisation. Blocked right-looking Cholesky of R = L^T in 16-column
// steps (T steps instead of the 4-column kernel's 4T):
//   diag   the owner wave of tile (k,k) factors it in ONE readlane-broadcast sweep of the
//          augmented [T_kk | I] (lanes 0-15: columns of T_kk -> rows of L_kk, lanes 16-31:
//          identity columns -> columns of L_kk^{-1}); L_kk^{-1} -> LDS;
//   TRSM   owners of block row k: R_kj = L_kk^{-1} T'_kj (4 f64 MFMAs, the register tile is
//          the B operand) -> LDS panel + L's block (j, k);
//   update every tile (i, j), k < i <= j: T'_ij -= R_ki^T R_kj (4 f64 MFMAs, both operands
//          read from the LDS panel in acc layout: conflict-free).
// Two workgroup barriers per step. GPyTorch's fp64 ladder restarts in-kernel (info = -t).
// gpk_kzz_inv_kernel: L^{-1}, one workgroup per 16-column block column (block forward
// substitution on fp64 MFMA), the block columns on different CUs.
#include "gpk_common.h"
#include "gpk_internal.h"
#include "gpk_kzz.h"

#include <mutex>

namespace {

GPK_DEVICE f64x4 mfma64(double a, double b, f64x4 c) {
  return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
}
GPK_DEVICE f32x4 mfma32(float a, float b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}
GPK_DEVICE double rsq64(double x) {   // 1/sqrt(x), x > 0: hardware estimate + 2 Newton steps
  double y = __builtin_amdgcn_rsq(x);
  y = y * (1.5 - 0.5 * x * y * y);
  y = y * (1.5 - 0.5 * x * y * y);
  return y;
}
GPK_DEVICE double rcp64(double x) {   // 1/x: hardware estimate + 2 Newton steps
  double y = __builtin_amdgcn_rcp(x);
  y = y * (2.0 - x * y);
  y = y * (2.0 - x * y);
  return y;
}
GPK_DEVICE double readlane_d(double v, int lane) {
  const unsigned long long u = __builtin_bit_cast(unsigned long long, v);
  const unsigned lo = __builtin_amdgcn_readlane((unsigned)u, lane);
  const unsigned hi = __builtin_amdgcn_readlane((unsigned)(u >> 32), lane);
  return __builtin_bit_cast(double, ((unsigned long long)hi << 32) | lo);
}

constexpr int KT = 512;   // 8 waves
__host__ __device__ inline int kzz_zstride(int D) { return ((D + 15) & ~15) + 4; }
constexpr int kLinvStride = 17;   // L_kk^{-1} rows in LDS (odd: conflict-free column reads)

template <int NS>
__global__ void __launch_bounds__(KT, 1)
gpk_kzz16_kernel(const float* __restrict__ Z, const float* __restrict__ hyp, int M, int D,
                 float jitter_var, double jitter_chol, int max_tries, double* __restrict__ L,
                 int* __restrict__ info) {
  extern __shared__ __attribute__((aligned(16))) double dsm[];
  const int T = (M + 15) >> 4, Mp = 16 * T;
  double* panel = dsm;                 // (T - 1) tiles x 256, [slot][reg][lane]
  double* dbuf = panel + (size_t)(T > 1 ? T - 1 : 1) * 256;   // 256: the diagonal tile
  double* linv = dbuf + 256;           // 16 x 17: L_kk^{-1}
  int* status = (int*)(linv + 16 * kLinvStride);              // [0]: failed column + 1
  float* zt = (float*)(status + 4);    // M x ZS  Z / l, centred (zero padded)
  const int ZS = kzz_zstride(D);
  const int D16 = (D + 15) & ~15;
  float* zn = zt + M * ZS;             // M
  float* cm = zn + M;                  // D
  const int tid = threadIdx.x, lane = tid & 63, c = lane & 15, g = lane >> 4;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const float s2 = hyp[0];
  const float* ls = hyp + 1;

  for (int base = 0; base < M * ZS; base += 8 * KT) {   // 8 loads in flight per thread
    float v[8], l[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int e = base + u * KT + tid, m = e / ZS, d = e - m * ZS;
      const bool ok = e < M * ZS && d < D;
      v[u] = Z[ok ? m * D + d : 0];
      l[u] = ls[ok ? d : 0];
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int e = base + u * KT + tid, d = e % ZS;
      if (e < M * ZS) zt[e] = d < D ? v[u] / l[u] : 0.f;
    }
  }
  lds_barrier();
  // column means in a fixed order: 8 partial sums per column (one per wave), then 8 -> 1
  for (int d = wave; d < D; d += KT / 64) {
    float sm = 0.f;
    for (int m = lane; m < M; m += 64) sm += zt[m * ZS + d];
    sm = wave_sum(sm);
    if (lane == 0) cm[d] = sm / (float)M;
  }
  lds_barrier();
  for (int e = tid; e < M * ZS; e += KT) {
    const int d = e % ZS;
    if (d < D) zt[e] -= cm[d];
  }
  lds_barrier();
  for (int m = tid; m < M; m += KT) {
    float sm = 0.f;
    for (int d = 0; d < D; ++d) sm = __builtin_fmaf(zt[m * ZS + d], zt[m * ZS + d], sm);
    zn[m] = sm;
  }
  lds_barrier();

  // upper tiles (it <= jt), column-major t = jt (jt + 1) / 2 + it, dealt round-robin
  const int ntile = T * (T + 1) / 2;
  int its[NS], jts[NS];
#pragma unroll
  for (int q = 0; q < NS; ++q) {
    const int t = wave + 8 * q;
    int it = T, jt = T;   // no tile: coordinates past the end (skipped everywhere)
    if (t < ntile) tile_of(t, T, it, jt);
    its[q] = __builtin_amdgcn_readfirstlane(it);
    jts[q] = __builtin_amdgcn_readfirstlane(jt);
  }
  f64x4 acc[NS];
  int result = 0;
  for (int attempt = 0; attempt <= max_tries; ++attempt) {
    double ladder = 0.0;  // GPyTorch adds (jitter_new - jitter_prev) cumulatively
    {
      double prev = 0.0, p10 = 1.0;
      for (int q = 0; q < attempt; ++q) {
        const double jn = jitter_chol * p10;
        ladder += jn - prev;
        prev = jn;
        p10 *= 10.0;
      }
    }
    // K_ZZ tiles: fp32 Gram on MFMA (A rows fed in the order pi(x) = (x >> 2) + 4 (x & 3) so the
    // fp32 accumulator lands in the fp64 acc layout), fp32 kernel + jitter, -> fp64 + ladder
#pragma unroll
    for (int q = 0; q < NS; ++q) {
      asm volatile("" : "+s"(its[q]), "+s"(jts[q]));
      const int j = 16 * jts[q] + c;
      f32x4 gram = {0.f, 0.f, 0.f, 0.f};
      if (its[q] < T) {
        const int ia = 16 * its[q] + (c >> 2) + 4 * (c & 3);
        const float* za = zt + (ia < M ? ia : 0) * ZS + 4 * g;
        const float* zb = zt + (j < M ? j : 0) * ZS + 4 * g;
        for (int d0 = 0; d0 < D16; d0 += 16) {
          const float4 av = *(const float4*)(za + d0);
          const float4 bv = *(const float4*)(zb + d0);
          gram = mfma32(av.x, bv.x, gram);
          gram = mfma32(av.y, bv.y, gram);
          gram = mfma32(av.z, bv.z, gram);
          gram = mfma32(av.w, bv.w, gram);
        }
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int i = 16 * its[q] + g + 4 * r;
        double v = (i == j) ? 1.0 : 0.0;
        if (its[q] < T && i < M && j < M) {
          float dist = zn[i] + zn[j] - 2.f * gram[r];
          dist = dist < 0.f ? 0.f : dist;
          float kv = s2 * __expf(-0.5f * dist);
          if (i == j) kv = kv + jitter_var;
          v = (double)kv;
          if (i == j) v += ladder;
        }
        acc[q][r] = v;
      }
    }
    if (tid == 0) status[0] = 0;
    int failed = 0;
    for (int k = 0; k < T; ++k) {
#pragma unroll
      for (int q = 0; q < NS; ++q) asm volatile("" : "+s"(its[q]), "+s"(jts[q]));
      // ---- diagonal block: the owner wave of tile (k, k) ----
      const int tkk = k * (k + 1) / 2 + k;
      if (wave == (tkk & 7)) {
#pragma unroll
        for (int q = 0; q < NS; ++q) {
          if (its[q] == k && jts[q] == k) {
#pragma unroll
            for (int r = 0; r < 4; ++r) dbuf[(g + 4 * r) * 16 + c] = acc[q][r];
          }
        }
        wave_lds_sync();
        // augmented [T_kk | I]: lane c < 16 holds column c of T_kk, lane 16 + c column c of I
        double v[16];
        const bool left = lane < 16;
#pragma unroll
        for (int i = 0; i < 16; ++i) v[i] = left ? dbuf[i * 16 + c] : ((lane - 16 == i) ? 1.0 : 0.0);
        int bad = 0;
#pragma unroll
        for (int q = 0; q < 16; ++q) {
          const double p = readlane_d(v[q], q);
          if (!(p > 0.0) && bad == 0) bad = q + 1;
          const double s = rsq64(p > 0.0 ? p : 1.0);
          const double sq = s * s;
          const double vq = v[q];
          v[q] = vq * s;
#pragma unroll
          for (int i = q + 1; i < 16; ++i) v[i] = __builtin_fma(-readlane_d(v[i], q) * sq, vq, v[i]);
        }
        // lanes 0-15: v[i] = L_kk[c][i] (i <= c); lanes 16-31: v[i] = L_kk^{-1}[i][c]
        const int row = 16 * k + c;
        if (left) {
          if (row < M) {
#pragma unroll
            for (int i = 0; i < 16; ++i)
              if (i <= c) L[(size_t)row * M + 16 * k + i] = v[i];
          }
        } else if (lane < 32) {
#pragma unroll
          for (int i = 0; i < 16; ++i) linv[i * kLinvStride + (lane - 16)] = v[i];
        }
        if (lane == 0) status[0] = bad == 0 ? 0 : 16 * k + bad;
      }
      lds_barrier();
      failed = status[0];
      if (failed) break;
      // ---- TRSM of block row k: R_kj = L_kk^{-1} T'_kj -> registers, LDS panel, L ----
      double la[4];
#pragma unroll
      for (int kk = 0; kk < 4; ++kk) la[kk] = linv[c * kLinvStride + g + 4 * kk];
#pragma unroll
      for (int q = 0; q < NS; ++q) {
        if (its[q] == k && jts[q] > k && jts[q] < T) {
          f64x4 x = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
          for (int kk = 0; kk < 4; ++kk) x = mfma64(la[kk], acc[q][kk], x);
          acc[q] = x;
          double* pt = panel + (size_t)(jts[q] - k - 1) * 256;
#pragma unroll
          for (int r = 0; r < 4; ++r) pt[r * 64 + lane] = x[r];
          // L block (j, k) = R_kj^T: L[16 j + c][16 k + g + 4 r] = R_kj[g + 4 r][c]
          const int row = 16 * jts[q] + c;
          if (row < M) {
#pragma unroll
            for (int r = 0; r < 4; ++r) L[(size_t)row * M + 16 * k + g + 4 * r] = x[r];
          }
        }
      }
      lds_barrier();
      // ---- trailing update: T'_ij -= R_ki^T R_kj for k < i <= j ----
#pragma unroll
      for (int q = 0; q < NS; ++q) {
        if (its[q] > k && its[q] < T) {
          const double* pa = panel + (size_t)(its[q] - k - 1) * 256;
          const double* pb = panel + (size_t)(jts[q] - k - 1) * 256;
#pragma unroll
          for (int kk = 0; kk < 4; ++kk) acc[q] = mfma64(-pa[kk * 64 + lane], pb[kk * 64 + lane], acc[q]);
        }
      }
    }
    if (!failed) {
      result = attempt > 0 ? -attempt : 0;
      break;
    }
    result = failed;
    lds_barrier();
  }
  for (int i = wave; i < M; i += KT / 64) {   // strict upper triangle of L: one row per wave
    for (int j = i + 1 + lane; j < M; j += 64) L[(size_t)i * M + j] = 0.0;
  }
  if (tid == 0) info[0] = result;
}

// L^{-1} of the K_ZZ factor: one workgroup per 16-column block column jb (grid T16), so
// the block columns run concurrently on different CUs. Block forward substitution,
// right-looking, on fp64 MFMA:
//   T_u = L_uu^{-1} (the diagonal blocks the column needs, formed in the workgroup),
//   X_jb = T_jb;  for k = jb ..: S_u += -L_uk X_k (u > k), X_{k+1} = T_{k+1} S_{k+1}.
// k-order of every MFMA: q = g + 4 kk, so a tile held in acc layout (reg r <-> row g + 4r)
// is the B operand of k-step kk straight from register kk. S tiles dealt over the 4 waves
// (u = wave mod 4); the L tiles of the next step are prefetched from L2 during this one.
constexpr int KIT = 256;
__global__ void __launch_bounds__(KIT)
gpk_kzz_inv_kernel(const double* __restrict__ L, int M, const int* __restrict__ info,
                   double* __restrict__ Linv) {
  extern __shared__ __attribute__((aligned(16))) double dsm[];
  const int Mp = (M + 15) & ~15, T16 = Mp >> 4;
  const int jb = blockIdx.x;
  const int nb = T16 - jb;            // block rows jb .. T16-1 of this block column
  double* Tv = dsm;                   // nb x 256: T_{jb+u}, row-major [row][col]
  double* Xs = Tv + nb * 256;         // nb x 256: X_{jb+u}, row-major
  const int tid = threadIdx.x, lane = tid & 63, c = lane & 15, g = lane >> 4;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  if (info[0] > 0) return;           // no factor (the op raises NotPSDError)
  auto Lat = [&](int i, int j) -> double {   // L with identity padding beyond M
    if (i < M && j < M) return L[(size_t)i * M + j];
    return i == j ? 1.0 : 0.0;
  };
  for (int e = tid; e < 16 * jb * 16; e += KIT) {   // block rows above the diagonal: zero
    const int i = e >> 4, j = 16 * jb + (e & 15);
    if (i < M && j < M) Linv[(size_t)i * M + j] = 0.0;
  }
  // diagonal-block inverses: lane group g of wave w takes block u = 4 w + g (+ 16 ...),
  // lane c its column c by forward substitution
  for (int u = 4 * wave + g; u < nb; u += 16) {
    const int b0 = 16 * (jb + u);
    double lr[16][16];
#pragma unroll
    for (int r = 0; r < 16; ++r)
#pragma unroll
      for (int q = 0; q <= r; ++q) lr[r][q] = Lat(b0 + r, b0 + q);
    double x[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      double v = (r == c) ? 1.0 : 0.0;
#pragma unroll
      for (int q = 0; q < r; ++q) v = __builtin_fma(-lr[r][q], x[q], v);
      x[r] = (r >= c) ? v * rcp64(lr[r][r]) : 0.0;
    }
#pragma unroll
    for (int r = 0; r < 16; ++r) Tv[u * 256 + r * 16 + c] = x[r];
  }
  lds_barrier();
  for (int e = tid; e < 256; e += KIT) {      // X_jb = T_jb
    Xs[e] = Tv[e];
    const int i = 16 * jb + (e >> 4), j = 16 * jb + (e & 15);
    if (i < M && j < M) Linv[(size_t)i * M + j] = Tv[e];
  }
  lds_barrier();
  f64x4 S[4];
#pragma unroll
  for (int t = 0; t < 4; ++t) S[t] = f64x4{0.0, 0.0, 0.0, 0.0};
  // A operands of step k: -L_{jb+u, jb+k}[c][g + 4kk] for the wave's tiles u = wave + 4t
  double an[4][4];
  auto load_a = [&](int k, double (&dst)[4][4]) {
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const int u = wave + 4 * t;
#pragma unroll
      for (int kk = 0; kk < 4; ++kk)
        dst[t][kk] = (u > k && u < nb) ? -Lat(16 * (jb + u) + c, 16 * (jb + k) + g + 4 * kk) : 0.0;
    }
  };
  load_a(0, an);
  for (int k = 0; k + 1 < nb; ++k) {
    double a[4][4];
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int kk = 0; kk < 4; ++kk) a[t][kk] = an[t][kk];
    if (k + 2 < nb) load_a(k + 1, an);
    double xb[4];
#pragma unroll
    for (int kk = 0; kk < 4; ++kk) xb[kk] = Xs[k * 256 + (g + 4 * kk) * 16 + c];
    const int tn = (k + 1) >> 2;          // slot of S_{k+1} in its owner wave
    const bool own = wave == ((k + 1) & 3);
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const int u = wave + 4 * t;
      if (u > k && u < nb) {
#pragma unroll
        for (int kk = 0; kk < 4; ++kk) S[t] = mfma64(a[t][kk], xb[kk], S[t]);
      }
    }
    if (own) {                            // X_{k+1} = T_{k+1} S_{k+1}
      f64x4 sv = S[0];
#pragma unroll
      for (int t = 1; t < 4; ++t) sv = (t == tn) ? S[t] : sv;
      f64x4 xv = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
      for (int kk = 0; kk < 4; ++kk) xv = mfma64(Tv[(k + 1) * 256 + c * 16 + g + 4 * kk], sv[kk], xv);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        Xs[(k + 1) * 256 + (g + 4 * r) * 16 + c] = xv[r];
        const int i = 16 * (jb + k + 1) + g + 4 * r, j = 16 * jb + c;
        if (i < M && j < M) Linv[(size_t)i * M + j] = xv[r];
      }
    }
    lds_barrier();
  }
}

template <auto Kernel>
void set_lds_once() {
  static std::once_flag once;  // one flag per kernel instantiation
  std::call_once(once, [] {
    (void)hipFuncSetAttribute((const void*)Kernel, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    (void)hipGetLastError();
  });
}

template <int NS>
int launch_kzz16(const GpkKzzArgs& a, hipStream_t stream) {
  const int T = (a.M + 15) >> 4;
  const size_t lds = (size_t)((T > 1 ? T - 1 : 1) * 256 + 256 + 16 * kLinvStride) * sizeof(double) +
                     4 * sizeof(int) + (size_t)(a.M * kzz_zstride(a.D) + a.M + a.D) * sizeof(float);
  if (lds > 160 * 1024) return -4;
  set_lds_once<gpk_kzz16_kernel<NS>>();
  hipLaunchKernelGGL((gpk_kzz16_kernel<NS>), dim3(1), dim3(KT), lds, stream, a.Z, a.hyp, a.M, a.D,
                     a.jitter_var, a.jitter_chol, a.max_tries, a.L, a.info);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return (int)e;
  set_lds_once<gpk_kzz_inv_kernel>();
  hipLaunchKernelGGL(gpk_kzz_inv_kernel, dim3(T), dim3(KIT), (size_t)2 * T * 256 * sizeof(double),
                     stream, a.L, a.M, a.info, a.Linv);
  e = hipGetLastError();
  return e == hipSuccess ? 0 : (int)e;
}

}  // namespace

int gpk_launch_kzz16(const GpkKzzArgs& a, hipStream_t stream) {
  const int T = (a.M + 15) >> 4;
  const int ns = (T * (T + 1) / 2 + 7) / 8;   // tiles per wave
  if (ns <= 2) return launch_kzz16<2>(a, stream);
  if (ns <= 5) return launch_kzz16<5>(a, stream);
  if (ns <= 10) return launch_kzz16<10>(a, stream);
  if (ns <= 17) return launch_kzz16<17>(a, stream);
  return -3;
}
