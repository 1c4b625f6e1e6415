// Variational (DeepGP) hot path for gfx950.
//
// Reference (oracle/gp_oracle.py::variational_forward):
//   ToyDeepGPHiddenLayer / DeepGPp (denoising_model/DeepGP.py:15-99) driven through
//   upstream variational/variational_strategy.py (whitened):
//     K_ZZ + jitter (fp32) -> fp64 -> L = psd_safe_cholesky (fp64 ladder 1e-8 x10^i)
//     A    = L^{-1} K_ZX        (fp64, cast to fp32)
//     mean = A^T m + x w + b0   (LinearMean, DeepGP.py:42-45)
//     var  = s2 + jitter + sum_m A_mi^2 (s_m^2 - 1), clamped >= 1e-6 (MVN.variance)
//     ELL  = sum_i -0.5 [((y_i - mean_i)^2 + var_i)/noise + log noise + log 2pi]
//
// Two launches per call:
//   gpk_kzz_kernel: ONE workgroup builds K_ZZ for the shared inducing points and
//     factors it in fp64 together with L^{-1} (forward elimination of [K | I]);
//     the reference does this b times (Z is expanded over the batch), we do it once.
//   gpk_var_kernel: one workgroup per window; each wave owns 16-point column
//     blocks, builds K_ZX columns in fp32 directly in the B-operand layout of
//     v_mfma_f64_16x16x4_f64 and accumulates A = L^{-1} K_ZX in fp64 tiles
//     (triangular L^{-1}: only k-steps p <= m), then reduces mean / var / ELL.
#include "gpk_common.h"
#include "gpk_internal.h"

namespace {

constexpr float kLog2PiF = 1.8378770664093453f;

GPK_DEVICE void barrier_all() { __syncthreads(); }

// ---------------------------------------------------------------------------
// K_ZZ build + fp64 Cholesky + inverse, one workgroup. L and Linv are the
// caller's output buffers (M x M fp64) and double as the working matrices.
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(1024)
gpk_kzz_kernel(const float* __restrict__ Z, const float* __restrict__ hyp, int M, int D,
               float jitter_var, double jitter_chol, int max_tries, double* __restrict__ L,
               double* __restrict__ Linv, int* __restrict__ info) {
  extern __shared__ __attribute__((aligned(16))) float vsm[];
  float* zt = vsm;                 // M x D   Z / l, centred
  float* zn = zt + M * D;          // M       squared norms
  float* cm = zn + M;              // D       column means
  double* bc = (double*)(((uintptr_t)(cm + D) + 15) & ~(uintptr_t)15);  // broadcast slots
  int* st = (int*)(bc + 4);
  double* colk = bc + 8;           // 4 x M: columns k, k+1 of L; rows k, k+1 of L^{-1}
  const int tid = threadIdx.x, T = blockDim.x;
  const float s2 = hyp[0];
  const float* ls = hyp + 1;  // D lengthscales (ARD, DeepGP.py:46-49)

  for (int e = tid; e < M * D; e += T) zt[e] = Z[e] / ls[e % D];
  barrier_all();
  for (int d = tid; d < D; d += T) {
    float s = 0.f;
    for (int m = 0; m < M; ++m) s += zt[m * D + d];
    cm[d] = s / (float)M;
  }
  barrier_all();
  for (int e = tid; e < M * D; e += T) zt[e] -= cm[e % D];
  barrier_all();
  for (int m = tid; m < M; m += T) {
    float s = 0.f;
    for (int d = 0; d < D; ++d) s = __builtin_fmaf(zt[m * D + d], zt[m * D + d], s);
    zn[m] = s;
  }
  barrier_all();

  int status = 0;
  for (int attempt = 0; attempt <= max_tries; ++attempt) {
    // (re)build A = K_ZZ + jitter (fp32) -> fp64 (+ fp64 ladder), B = I
    for (int e = tid; e < M * M; e += T) {
      const int i = e / M, j = e - i * M;
      double a = 0.0;
      if (j <= i) {
        float dot = 0.f;
        for (int d = 0; d < D; ++d) dot = __builtin_fmaf(zt[i * D + d], zt[j * D + d], dot);
        float dist = zn[i] + zn[j] - 2.f * dot;
        dist = dist < 0.f ? 0.f : dist;
        float kv = s2 * __expf(-0.5f * dist);
        if (i == j) kv = kv + jitter_var;
        a = (double)kv;
        if (i == j) {
          // GPyTorch adds (jitter_new - jitter_prev) cumulatively to Aprime
          double acc = a;
          double prev = 0.0;
          for (int q = 0; q < attempt; ++q) {
            double p10 = 1.0;
            for (int u = 0; u < q; ++u) p10 *= 10.0;
            const double jn = jitter_chol * p10;
            acc += jn - prev;
            prev = jn;
          }
          a = acc;
        }
      }
      L[e] = a;
      Linv[e] = (i == j) ? 1.0 : 0.0;
    }
    if (tid == 0) st[0] = 0;
    barrier_all();
    // column k of the trailing matrix and row k of L^{-1} live in LDS (cur / currow):
    // the threads that update column k+1 / row k+1 also write them there (nxt /
    // nxtrow), so a step never waits on a global load for its pivot or its scaling.
    double* cur = colk;
    double* nxt = colk + M;
    double* currow = colk + 2 * M;
    double* nxtrow = colk + 3 * M;
    for (int i = tid; i < M; i += T) {
      cur[i] = L[(size_t)i * M];
      currow[i] = (i == 0) ? 1.0 : 0.0;
    }
    barrier_all();
    int failed = 0;
    const int wv = tid >> 6, ln = tid & 63, NWV = T >> 6;
    for (int k = 0; k < M; ++k) {
      const double piv = cur[k];
      if (!(piv > 0.0)) { failed = k + 1; break; }  // uniform: every thread reads the same LDS word
      const double lkk = __builtin_sqrt(piv);
      const double inv = 1.0 / lkk;
      if (tid == 0) L[(size_t)k * M + k] = lkk;
      for (int i = k + 1 + tid; i < M; i += T) {
        const double v = cur[i] * inv;
        L[(size_t)i * M + k] = v;
        cur[i] = v;
      }
      for (int j = tid; j <= k; j += T) {
        const double v = currow[j] * inv;
        Linv[(size_t)k * M + j] = v;
        currow[j] = v;
      }
      barrier_all();
      // rank-1 update of the trailing lower triangle and of L^{-1}'s rows below k:
      // one row per wave at a time, lanes along the row (coalesced)
      for (int i = k + 1 + wv; i < M; i += NWV) {
        const double lik = cur[i];
        double* Li = L + (size_t)i * M;
        for (int j = k + 1 + ln; j <= i; j += 64) {
          const double v = Li[j] - lik * cur[j];
          Li[j] = v;
          if (j == k + 1) nxt[i] = v;
        }
        double* Ii = Linv + (size_t)i * M;
        for (int j = ln; j <= k; j += 64) {
          const double v = Ii[j] - lik * currow[j];
          Ii[j] = v;
          if (i == k + 1) nxtrow[j] = v;
        }
      }
      if (tid == 0 && k + 1 < M) nxtrow[k + 1] = 1.0;  // B = I: row k+1's diagonal is untouched
      barrier_all();
      double* t = cur; cur = nxt; nxt = t;
      t = currow; currow = nxtrow; nxtrow = t;
    }
    if (!failed) {
      status = attempt > 0 ? -attempt : 0;
      break;
    }
    status = failed;
    barrier_all();
  }
  // zero the strictly-upper triangles
  for (int e = tid; e < M * M; e += T) {
    const int i = e / M, j = e - i * M;
    if (j > i) { L[e] = 0.0; Linv[e] = 0.0; }
  }
  if (tid == 0) info[0] = status;
}

// ---------------------------------------------------------------------------
// Blocked K_ZZ factorisation (one workgroup, 1024 threads, KR = 32-column blocks).
// Same arithmetic as gpk_kzz_kernel (K_ZZ fp32 -> fp64, GPyTorch's cumulative fp64
// ladder, L and L^{-1} of [K | I] by forward elimination) but per block of KR columns:
//   (1) the KR x KR diagonal block and an identity are eliminated in LDS (one
//       element per thread, one barrier per column) -> L11, L11^{-1};
//   (2) V = L11^{-1} [Linv rows k.. (cols < k+KR) | A21^T] in LDS, one column per
//       thread -> the final rows of L^{-1} and the final L21 (written to L2/HBM);
//   (3) ONE trailing update of every remaining row i: target[i][c] -= sum_p V[p][i]
//       V[p][c] (c < k+KR: L^{-1}; k+KR <= c <= i: the Schur complement), 4 x 4
//       register tiles, lanes along c (coalesced), operands from LDS.
// M/KR block steps instead of M serial column steps through L2.
// ---------------------------------------------------------------------------
constexpr int KR = 32;

__global__ void __launch_bounds__(1024)
gpk_kzz_blocked_kernel(const float* __restrict__ Z, const float* __restrict__ hyp, int M, int D,
                       float jitter_var, double jitter_chol, int max_tries,
                       double* __restrict__ L, double* __restrict__ Linv, int* __restrict__ info) {
  extern __shared__ __attribute__((aligned(16))) float vsm[];
  const int Mp = (M + 3) & ~3;
  double* V = (double*)vsm;                  // KR x Mp
  double* dg = V + KR * Mp;                  // KR x 2KR  [A11 | I] elimination
  double* li = dg + KR * 2 * KR;             // KR x KR   L11^{-1}
  float* zt = (float*)(li + KR * KR);        // M x D     Z / l, centred
  float* zn = zt + M * D;                    // M
  float* cm = zn + M;                        // D
  const int tid = threadIdx.x, T = blockDim.x;
  const float s2 = hyp[0];
  const float* ls = hyp + 1;

  for (int e = tid; e < M * D; e += T) zt[e] = Z[e] / ls[e % D];
  __syncthreads();
  for (int d = tid; d < D; d += T) {
    float s = 0.f;
    for (int m = 0; m < M; ++m) s += zt[m * D + d];
    cm[d] = s / (float)M;
  }
  __syncthreads();
  for (int e = tid; e < M * D; e += T) zt[e] -= cm[e % D];
  __syncthreads();
  for (int m = tid; m < M; m += T) {
    float s = 0.f;
    for (int d = 0; d < D; ++d) s = __builtin_fmaf(zt[m * D + d], zt[m * D + d], s);
    zn[m] = s;
  }
  __syncthreads();

  const int jr = tid >> 5, jc = tid & 31;  // (row, column) of this thread in a KR x KR block
  int status = 0;
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
    for (int e = tid; e < M * M; e += T) {
      const int i = e / M, j = e - i * M;
      double a = 0.0;
      if (j <= i) {
        float dot = 0.f;
        for (int d = 0; d < D; ++d) dot = __builtin_fmaf(zt[i * D + d], zt[j * D + d], dot);
        float dist = zn[i] + zn[j] - 2.f * dot;
        dist = dist < 0.f ? 0.f : dist;
        float kv = s2 * __expf(-0.5f * dist);
        if (i == j) kv = kv + jitter_var;
        a = (double)kv;
        if (i == j) a += ladder;
      }
      L[e] = a;
      Linv[e] = (i == j) ? 1.0 : 0.0;
    }
    __syncthreads();

    int failed = 0;
    for (int k = 0; k < M && !failed; k += KR) {
      const int r = M - k < KR ? M - k : KR;
      // (1) diagonal block, symmetric fill from the lower storage, identity padding
      {
        double a;
        if (jr < r && jc < r) {
          const int hi = jr > jc ? jr : jc, lo = jr > jc ? jc : jr;
          a = L[(size_t)(k + hi) * M + k + lo];
        } else {
          a = (jr == jc) ? 1.0 : 0.0;
        }
        dg[jr * 2 * KR + jc] = a;
        dg[jr * 2 * KR + KR + jc] = (jr == jc) ? 1.0 : 0.0;
      }
      __syncthreads();
      for (int j = 0; j < r; ++j) {
        const double piv = dg[j * 2 * KR + j];
        if (!(piv > 0.0)) { failed = k + j + 1; break; }  // uniform (same LDS word)
        if (jr > j) {
          const double f = dg[jr * 2 * KR + j] / piv;
          if (jc > j) dg[jr * 2 * KR + jc] -= f * dg[j * 2 * KR + jc];
          if (jc <= j) dg[jr * 2 * KR + KR + jc] -= f * dg[j * 2 * KR + KR + jc];
        }
        __syncthreads();
      }
      if (failed) break;
      {
        const double s = 1.0 / __builtin_sqrt(dg[jr * 2 * KR + jr]);
        // L11[jc][jr] = U[jr][jc] for jc >= jr
        if (jr < r && jc < r && jc >= jr) L[(size_t)(k + jc) * M + k + jr] = dg[jr * 2 * KR + jc] * s;
        li[jr * KR + jc] = (jr < r && jc <= jr) ? dg[jr * 2 * KR + KR + jc] * s : 0.0;
      }
      // (2) stage V = [Linv rows k..k+r (cols < k+r) | A21^T]
      for (int e = tid; e < KR * M; e += T) {
        const int p = e / M, c = e - p * M;
        double v = 0.0;
        if (p < r) v = c < k + r ? Linv[(size_t)(k + p) * M + c] : L[(size_t)c * M + k + p];
        V[p * Mp + c] = v;
      }
      __syncthreads();
      for (int c = tid; c < M; c += T) {
        double vin[KR];
#pragma unroll
        for (int p = 0; p < KR; ++p) vin[p] = V[p * Mp + c];
#pragma unroll
        for (int j = 0; j < KR; ++j) {
          double acc = 0.0;
#pragma unroll
          for (int p = 0; p <= j; ++p) acc = __builtin_fma(li[j * KR + p], vin[p], acc);
          V[j * Mp + c] = acc;
          if (j < r) {
            if (c < k + r) Linv[(size_t)(k + j) * M + c] = acc;
            else L[(size_t)c * M + k + j] = acc;
          }
        }
      }
      __syncthreads();
      // (3) trailing update of rows k+r .. M-1
      const int i0 = k + r;
      const int nrt = (M - i0 + 3) >> 2, nct = Mp >> 2;
      for (int t = tid; t < nrt * nct; t += T) {
        const int rt = t / nct, ct = t - rt * nct;
        const int ib = i0 + 4 * rt, cb = 4 * ct;
        if (cb > ib + 3) continue;  // tile entirely above the diagonal
        double acc[4][4];
#pragma unroll
        for (int u = 0; u < 4; ++u)
#pragma unroll
          for (int w = 0; w < 4; ++w) acc[u][w] = 0.0;
#pragma unroll 8
        for (int p = 0; p < KR; ++p) {
          const double* vr = V + p * Mp;
          double a[4], b[4];
#pragma unroll
          for (int u = 0; u < 4; ++u) { a[u] = vr[ib + u < Mp ? ib + u : 0]; b[u] = vr[cb + u]; }
#pragma unroll
          for (int u = 0; u < 4; ++u)
#pragma unroll
            for (int w = 0; w < 4; ++w) acc[u][w] = __builtin_fma(a[u], b[w], acc[u][w]);
        }
        double* tgt = cb < i0 ? Linv : L;
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int i = ib + u;
          if (i >= M) continue;
#pragma unroll
          for (int w = 0; w < 4; ++w) {
            const int c = cb + w;
            if (c <= i && c < M) tgt[(size_t)i * M + c] -= acc[u][w];
          }
        }
      }
      __syncthreads();
    }
    if (!failed) {
      status = attempt > 0 ? -attempt : 0;
      break;
    }
    status = failed;
    __syncthreads();
  }
  for (int e = tid; e < M * M; e += T) {
    const int i = e / M, j = e - i * M;
    if (j > i) { L[e] = 0.0; Linv[e] = 0.0; }
  }
  if (tid == 0) info[0] = status;
}

// ---------------------------------------------------------------------------
// Batched predictive mean / variance / expected log-likelihood.
// MB = number of 16-row blocks of the inducing dimension (M <= 16 MB),
// DMAX = register capacity for one data point's coordinates (D <= DMAX).
// ---------------------------------------------------------------------------
template <int MB, int DMAX>
__global__ void __launch_bounds__(256)
gpk_var_kernel(const float* __restrict__ X, const float* __restrict__ Z,
               const double* __restrict__ Linv, const float* __restrict__ vmean,
               const float* __restrict__ vstd, const float* __restrict__ hyp,
               const float* __restrict__ y, int N, int M, int D, float* __restrict__ mean_out,
               float* __restrict__ var_out, float* __restrict__ ell_out) {
  extern __shared__ __attribute__((aligned(16))) float vsm[];
  float* zt = vsm;               // 16MB x D   centred Z / l (zero-padded rows)
  float* cm = zt + 16 * MB * D;  // D
  float* vm = cm + D;            // 16MB  variational mean
  float* sm1 = vm + 16 * MB;     // 16MB  s^2 - 1
  float* red = sm1 + 16 * MB;    // 8
  const int tid = threadIdx.x, T = blockDim.x;
  const int lane = tid & 63, c = lane & 15, g = lane >> 4;
  const int wave = tid >> 6, NW = T >> 6;
  const int b = blockIdx.x;
  // hyp: [s2, noise, jitter, b0, w[D], ls[D]]
  const float s2 = hyp[0], noise = hyp[1], jit = hyp[2], b0 = hyp[3];
  const float* w = hyp + 4;
  const float* ls = hyp + 4 + D;

  for (int e = tid; e < 16 * MB * D; e += T) {
    const int m = e / D;
    zt[e] = (m < M) ? Z[e] / ls[e % D] : 0.f;
  }
  for (int m = tid; m < 16 * MB; m += T) {
    vm[m] = (m < M) ? vmean[m] : 0.f;
    const float sd = (m < M) ? vstd[m] : 1.f;
    sm1[m] = sd * sd - 1.f;
  }
  __syncthreads();
  for (int d = tid; d < D; d += T) {
    float s = 0.f;
    for (int m = 0; m < M; ++m) s += zt[m * D + d];
    cm[d] = s / (float)M;  // GPyTorch _sq_dist centres by x1 = Z
  }
  __syncthreads();
  for (int e = tid; e < M * D; e += T) zt[e] -= cm[e % D];
  __syncthreads();

  const float* Xb = X + (size_t)b * N * D;
  float ell_acc = 0.f;
  const float log_noise = __logf(noise);
  const float nhalf_log2e = -0.72134752044448170f;
  const int NBLK = (N + 15) / 16;
  for (int nb = wave; nb < NBLK; nb += NW) {
    const int i = 16 * nb + c;
    float xr[DMAX];
#pragma unroll
    for (int d = 0; d < DMAX; ++d)
      xr[d] = (d < D && i < N) ? Xb[(size_t)i * D + d] / ls[d] - cm[d] : 0.f;
    f64x4 acc[MB];
#pragma unroll
    for (int mb = 0; mb < MB; ++mb) acc[mb] = f64x4{0.0, 0.0, 0.0, 0.0};
    for (int s = 0; s < 4 * MB; ++s) {
      const int p = 4 * s + g;  // inducing point of this lane's B-operand row
      float dist = 0.f;
#pragma unroll
      for (int d = 0; d < DMAX; ++d) {
        if (d < D) {
          const float df = zt[p * D + d] - xr[d];
          dist = __builtin_fmaf(df, df, dist);
        }
      }
      const float kv = (p < M && i < N) ? s2 * __builtin_amdgcn_exp2f(nhalf_log2e * dist) : 0.f;
      const double kd = (double)kv;
      const int mb0 = (4 * s) >> 4;  // L^{-1}[m][p] = 0 for m < p
#pragma unroll
      for (int mb = 0; mb < MB; ++mb) {
        if (mb >= mb0) {
          const int m = 16 * mb + c;  // A-operand: lane holds Linv[m][4s + g]
          const double a = (m < M && p < M) ? Linv[(size_t)m * M + p] : 0.0;
          acc[mb] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, kd, acc[mb], 0, 0, 0);
        }
      }
    }
    // acc[mb][r] = A[16 mb + g + 4 r][16 nb + c]  (f64 16x16x4 C/D layout)
    float mpart = 0.f, vpart = 0.f;
#pragma unroll
    for (int mb = 0; mb < MB; ++mb) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = 16 * mb + g + 4 * r;
        const float a32 = (float)acc[mb][r];
        mpart = __builtin_fmaf(a32, vm[m], mpart);
        vpart = __builtin_fmaf(a32 * a32, sm1[m], vpart);
      }
    }
    mpart += __shfl_xor(mpart, 16, 64);
    mpart += __shfl_xor(mpart, 32, 64);
    vpart += __shfl_xor(vpart, 16, 64);
    vpart += __shfl_xor(vpart, 32, 64);
    if (g == 0 && i < N) {
      float mu = b0;
      float lin = 0.f;
      for (int d = 0; d < D; ++d) lin = __builtin_fmaf(Xb[(size_t)i * D + d], w[d], lin);
      const float mean_i = mpart + (lin + mu);
      float var_i = s2 + jit + vpart;
      var_i = var_i < 1e-6f ? 1e-6f : var_i;  // MVN.variance clamp (fp32 min_variance)
      mean_out[(size_t)b * N + i] = mean_i;
      var_out[(size_t)b * N + i] = var_i;
      if (y != nullptr) {
        const float dy = y[(size_t)b * N + i] - mean_i;
        ell_acc += -0.5f * ((dy * dy + var_i) / noise + log_noise + kLog2PiF);
      }
    }
  }
  if (ell_out != nullptr) {
    ell_acc = wave_sum(ell_acc);
    if (lane == 0) red[wave] = ell_acc;
    __syncthreads();
    if (tid == 0) {
      float s = 0.f;
      for (int q = 0; q < NW; ++q) s += red[q];
      ell_out[b] = s;
    }
  }
}

// ---------------------------------------------------------------------------
// Adjoint of gpk_var_kernel (variational path). Per window and
// 16-point block it recomputes K_ZX (fp32) and A = L^{-1} K_ZX (fp64 MFMA) exactly
// as the forward, then with the incoming gmean / gvar (gvar masked where the
// variance was clamped, MVN.variance):
//   dA   = gmean_i m_m + 2 gvar_i (s_m^2 - 1) A_mi                 (fp64)
//   dK   = L^{-T} dA   (fp64 MFMA, triangular k-steps only)
//   Q    = dK o K_ZX   (the RBF adjoint's only per-entry quantity)
// and writes dA (fp64), K_ZX and Q (fp32) as (B, M, N) plus per-window partial
// sums dm = sum_i gmean A, dsm1 = sum_i gvar A^2 and sum_i gvar. The contractions
// over points / windows (dL^{-1} = sum dA K^T, Q x / Q z) are plain GEMMs done by
// the caller (rocBLAS through torch), and the M x M K_ZZ adjoint once per call.
// ---------------------------------------------------------------------------
template <int MB, int DMAX>
__global__ void __launch_bounds__(256)
gpk_var_adjoint_kernel(const float* __restrict__ X, const float* __restrict__ Z,
                       const double* __restrict__ Linv, const float* __restrict__ vmean,
                       const float* __restrict__ vstd, const float* __restrict__ hyp,
                       const float* __restrict__ gmean, const float* __restrict__ gvar, int N,
                       int M, int D, double* __restrict__ dA_out, float* __restrict__ K_out,
                       float* __restrict__ Q_out, float* __restrict__ part_out) {
  extern __shared__ __attribute__((aligned(16))) float vsm[];
  float* zt = vsm;               // 16MB x D   centred Z / l (zero-padded rows)
  float* cm = zt + 16 * MB * D;  // D
  float* vm = cm + D;            // 16MB  variational mean
  float* sm1 = vm + 16 * MB;     // 16MB  s^2 - 1
  float* dm = sm1 + 16 * MB;     // 16MB  partial sum_i gmean A
  float* ds = dm + 16 * MB;      // 16MB  partial sum_i gvar A^2
  float* ksm = ds + 16 * MB;     // 4 waves x 16MB x 16  K_ZX of the wave's block
  float* red = ksm + 4 * 16 * MB * 16;  // 8
  const int tid = threadIdx.x, T = blockDim.x;
  const int lane = tid & 63, c = lane & 15, g = lane >> 4;
  const int wave = tid >> 6, NW = T >> 6;
  const int b = blockIdx.x;
  const float s2 = hyp[0], jit = hyp[2];
  const float* ls = hyp + 4 + D;
  const size_t MN = (size_t)M * N;

  for (int e = tid; e < 16 * MB * D; e += T) {
    const int m = e / D;
    zt[e] = (m < M) ? Z[e] / ls[e % D] : 0.f;
  }
  for (int m = tid; m < 16 * MB; m += T) {
    vm[m] = (m < M) ? vmean[m] : 0.f;
    const float sd = (m < M) ? vstd[m] : 1.f;
    sm1[m] = sd * sd - 1.f;
    dm[m] = 0.f;
    ds[m] = 0.f;
  }
  __syncthreads();
  for (int d = tid; d < D; d += T) {
    float s = 0.f;
    for (int m = 0; m < M; ++m) s += zt[m * D + d];
    cm[d] = s / (float)M;
  }
  __syncthreads();
  for (int e = tid; e < M * D; e += T) zt[e] -= cm[e % D];
  __syncthreads();

  const float* Xb = X + (size_t)b * N * D;
  float* kw = ksm + wave * 16 * MB * 16;
  float gvsum = 0.f;
  const float nhalf_log2e = -0.72134752044448170f;
  const int NBLK = (N + 15) / 16;
  for (int nb = wave; nb < NBLK; nb += NW) {
    const int i = 16 * nb + c;
    float xr[DMAX];
#pragma unroll
    for (int d = 0; d < DMAX; ++d)
      xr[d] = (d < D && i < N) ? Xb[(size_t)i * D + d] / ls[d] - cm[d] : 0.f;
    f64x4 acc[MB];
#pragma unroll
    for (int mb = 0; mb < MB; ++mb) acc[mb] = f64x4{0.0, 0.0, 0.0, 0.0};
    for (int s = 0; s < 4 * MB; ++s) {
      const int p = 4 * s + g;
      float dist = 0.f;
#pragma unroll
      for (int d = 0; d < DMAX; ++d) {
        if (d < D) {
          const float df = zt[p * D + d] - xr[d];
          dist = __builtin_fmaf(df, df, dist);
        }
      }
      const float kv = (p < M && i < N) ? s2 * __builtin_amdgcn_exp2f(nhalf_log2e * dist) : 0.f;
      kw[p * 16 + c] = kv;
      if (p < M && i < N) K_out[(size_t)b * MN + (size_t)p * N + i] = kv;
      const double kd = (double)kv;
      const int mb0 = (4 * s) >> 4;
#pragma unroll
      for (int mb = 0; mb < MB; ++mb) {
        if (mb >= mb0) {
          const int m = 16 * mb + c;
          const double a = (m < M && p < M) ? Linv[(size_t)m * M + p] : 0.0;
          acc[mb] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, kd, acc[mb], 0, 0, 0);
        }
      }
    }
    // acc[mb][r] = A[16 mb + g + 4 r][16 nb + c]; the variance (for the clamp mask)
    float vpart = 0.f;
#pragma unroll
    for (int mb = 0; mb < MB; ++mb) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float a32 = (float)acc[mb][r];
        vpart = __builtin_fmaf(a32 * a32, sm1[16 * mb + g + 4 * r], vpart);
      }
    }
    vpart += __shfl_xor(vpart, 16, 64);
    vpart += __shfl_xor(vpart, 32, 64);
    const float var_i = s2 + jit + vpart;
    const float gm = (i < N) ? gmean[(size_t)b * N + i] : 0.f;
    float gv = (i < N) ? gvar[(size_t)b * N + i] : 0.f;
    if (var_i < 1e-6f) gv = 0.f;  // clamp_min(1e-6): no gradient below the clamp
    if (g == 0) gvsum += gv;
    // dA (fp64, C layout of A), partial sums for dm / ds, dA out
#pragma unroll
    for (int mb = 0; mb < MB; ++mb) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = 16 * mb + g + 4 * r;
        const double a = acc[mb][r];
        const float a32 = (float)a;
        const double da = (double)gm * (double)vm[m] + 2.0 * (double)gv * (double)sm1[m] * (double)a32;
        acc[mb][r] = da;
        float pm = gm * a32, ps = gv * a32 * a32;
#pragma unroll
        for (int off = 1; off < 16; off <<= 1) {  // sum over the 16 points of the block
          pm += __shfl_xor(pm, off, 64);
          ps += __shfl_xor(ps, off, 64);
        }
        if (c == 0 && m < M) {
          (void)__hip_atomic_fetch_add(&dm[m], pm, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
          (void)__hip_atomic_fetch_add(&ds[m], ps, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
        if (m < M && i < N) dA_out[(size_t)b * MN + (size_t)m * N + i] = da;
      }
    }
    // dK = L^{-T} dA: output block pb, k-steps s >= 4 pb (L^{-1}[m][p] = 0 for m < p);
    // the B operand of k-step s is dA[4s + g][c] = acc[s / 4][s % 4]
#pragma unroll
    for (int pb = 0; pb < MB; ++pb) {
      f64x4 dk = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
      for (int s = 4 * pb; s < 4 * MB; ++s) {
        const int m = 4 * s + g, p = 16 * pb + c;
        const double a = (m < M && p < M) ? Linv[(size_t)m * M + p] : 0.0;
        dk = __builtin_amdgcn_mfma_f64_16x16x4f64(a, acc[s >> 2][s & 3], dk, 0, 0, 0);
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int p = 16 * pb + g + 4 * r;
        if (p < M && i < N) Q_out[(size_t)b * MN + (size_t)p * N + i] = (float)dk[r] * kw[p * 16 + c];
      }
    }
  }
  gvsum = wave_sum(gvsum);
  if (lane == 0) red[wave] = gvsum;
  __syncthreads();
  // per-window partials: [dm (M), ds (M), sum gvar]
  float* po = part_out + (size_t)b * (2 * M + 1);
  for (int m = tid; m < M; m += T) {
    po[m] = dm[m];
    po[M + m] = ds[m];
  }
  if (tid == 0) {
    float s = 0.f;
    for (int q = 0; q < NW; ++q) s += red[q];
    po[2 * M] = s;
  }
}

template <int MB, int DMAX>
int launch_var_adj(const GpkVarAdjArgs& a, hipStream_t stream) {
  const size_t lds = (size_t)(16 * MB * a.D + a.D + 4 * 16 * MB + 4 * 16 * MB * 16 + 8) * sizeof(float);
  if (lds > 160 * 1024) return -10;
  if (lds > 64 * 1024)
    (void)hipFuncSetAttribute((const void*)gpk_var_adjoint_kernel<MB, DMAX>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  hipLaunchKernelGGL((gpk_var_adjoint_kernel<MB, DMAX>), dim3(a.B), dim3(256), lds, stream, a.X,
                     a.Z, a.Linv, a.vmean, a.vstd, a.hyp, a.gmean, a.gvar, a.N, a.M, a.D, a.dA,
                     a.K, a.Q, a.part);
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? 0 : (int)e;
}

template <int DMAX>
int launch_var_adj_d(const GpkVarAdjArgs& a, hipStream_t stream) {
  switch ((a.M + 15) / 16) {
#define GPK_VCASE(mb) case mb: return launch_var_adj<mb, DMAX>(a, stream);
    GPK_VCASE(1) GPK_VCASE(2) GPK_VCASE(3) GPK_VCASE(4) GPK_VCASE(5) GPK_VCASE(6)
    GPK_VCASE(7) GPK_VCASE(8) GPK_VCASE(9) GPK_VCASE(10) GPK_VCASE(11) GPK_VCASE(12)
    GPK_VCASE(13) GPK_VCASE(14) GPK_VCASE(15) GPK_VCASE(16)
#undef GPK_VCASE
    default: return -10;
  }
}

template <int MB, int DMAX>
int launch_var(const GpkVarArgs& a, hipStream_t stream) {
  const size_t lds = (size_t)(16 * MB * a.D + a.D + 2 * 16 * MB + 8) * sizeof(float);
  if (lds > 64 * 1024)
    (void)hipFuncSetAttribute((const void*)gpk_var_kernel<MB, DMAX>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  hipLaunchKernelGGL((gpk_var_kernel<MB, DMAX>), dim3(a.B), dim3(256), lds, stream, a.X, a.Z,
                     a.Linv, a.vmean, a.vstd, a.hyp, a.y, a.N, a.M, a.D, a.mean, a.var, a.ell);
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? 0 : (int)e;
}

template <int DMAX>
int launch_var_d(const GpkVarArgs& a, hipStream_t stream) {
  switch ((a.M + 15) / 16) {
#define GPK_VCASE(mb) case mb: return launch_var<mb, DMAX>(a, stream);
    GPK_VCASE(1) GPK_VCASE(2) GPK_VCASE(3) GPK_VCASE(4) GPK_VCASE(5) GPK_VCASE(6)
    GPK_VCASE(7) GPK_VCASE(8) GPK_VCASE(9) GPK_VCASE(10) GPK_VCASE(11) GPK_VCASE(12)
    GPK_VCASE(13) GPK_VCASE(14) GPK_VCASE(15) GPK_VCASE(16)
#undef GPK_VCASE
    default: return -9;
  }
}

}  // namespace

int gpk_launch_kzz(const GpkKzzArgs& a, hipStream_t stream) {
  const size_t lds = (size_t)(a.M * a.D + a.M + a.D + 16) * sizeof(float) + 64 + 4 * a.M * sizeof(double) + 64;
  if (lds > 160 * 1024) return -4;
  if (lds > 64 * 1024)
    (void)hipFuncSetAttribute((const void*)gpk_kzz_kernel,
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  hipLaunchKernelGGL(gpk_kzz_kernel, dim3(1), dim3(1024), lds, stream, a.Z, a.hyp, a.M, a.D,
                     a.jitter_var, a.jitter_chol, a.max_tries, a.L, a.Linv, a.info);
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? 0 : (int)e;
}

int gpk_launch_var_adjoint(const GpkVarAdjArgs& a, hipStream_t stream) {
  if (a.D <= 16) return launch_var_adj_d<16>(a, stream);
  if (a.D <= 32) return launch_var_adj_d<32>(a, stream);
  if (a.D <= 64) return launch_var_adj_d<64>(a, stream);
  return -11;
}

int gpk_launch_var(const GpkVarArgs& a, hipStream_t stream) {
  if (a.D <= 16) return launch_var_d<16>(a, stream);
  if (a.D <= 32) return launch_var_d<32>(a, stream);
  if (a.D <= 64) return launch_var_d<64>(a, stream);
  return -8;
}
