// Adjoint of the shared K_ZZ factor (fp64), once per optimizer step.
//
// Reference: the autograd backward that train.py:166 runs through GPyTorch's
// VariationalStrategy._cholesky_factor (psd_safe_cholesky of K_ZZ + jitter in fp64) and
// the triangular solve L^{-1} K_ZX (denoising_model/DeepGP.py:33-38 via upstream
// variational_strategy.py); oracle/gp_oracle.py restates the forward.
//
// Given G = dObjective/dLinv (lower, summed over every GP call that used the factor):
//   T1   = G Linv^T                      (full)
//   Lbar = -tril(Linv^T T1)              (= dObjective/dL)
//   P    = Phi(L^T Lbar)                 (tril, diagonal halved)
//   U    = P Linv                        (lower)
//   S    = Linv^T U                      (full; Kbar = (S + S^T) / 2)
//   W    = Kbar o s2 exp(-d2/2),  w1 = W 1,  Wz = W zs  (zs = Z / l, fp64)
//   dZ   = 2 (Wz - zs o w1) / l,  dl_d = 2 (sum_i w1_i zs_id^2 - Wz_id zs_id) / l_d,
//   ds2  = sum W / s2.
// Kernels: gpk_kzzg_gemm_kernel<MODE> (one workgroup per 16 x 16 output tile, its k-blocks
// split over the 4 waves, all operands requested up front from L2, fp64 MFMA; triangular
// k-ranges), gpk_kzzg_rbf_kernel (one wave per 16 x 16 tile of W: partial w1 / Wz per row
// and column block), gpk_kzzg_rows_kernel (per 16-row block: fixed-order totals -> dZ and
// the block's dl / ds2 partials) + gpk_kzzg_fin_kernel (fixed-order sum of the T block
// partials -> ds2, dl): deterministic.
#include "gpk_common.h"
#include "gpk_internal.h"


namespace {

GPK_DEVICE f64x4 mfma64(double a, double b, f64x4 c) {
  return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
}

// lower tiles row-major: tile t -> (it, jt), jt <= it
GPK_DEVICE void tri_tile(int t, int& it, int& jt) {
  int r = (int)((__builtin_sqrtf(8.f * (float)t + 1.f) - 1.f) * 0.5f);
  while ((r + 1) * (r + 2) / 2 <= t) ++r;
  while (r * (r + 1) / 2 > t) --r;
  it = r;
  jt = t - r * (r + 1) / 2;
}

// MODE 1: C = G Linv^T        A(i,k) = G[i][k] (k <= i)   B(k,j) = Linv[j][k]   kb in [0, min(ib, jb)]  full
// MODE 2: C = -tril(Linv^T T1) A(i,k) = -Linv[k][i]        B(k,j) = T1[k][j]     kb in [ib, T)           lower
// MODE 3: C = Phi(L^T Lbar)   A(i,k) = L[k][i]             B(k,j) = Lbar[k][j]   kb in [ib, T)           lower, diag / 2
// MODE 4: C = P Linv          A(i,k) = P[i][k]             B(k,j) = Linv[k][j]   kb in [jb, ib]          lower
// MODE 5: C = Linv^T U        A(i,k) = Linv[k][i]          B(k,j) = U[k][j]      kb in [max(ib,jb), T)   full
template <int MODE>
struct KzzGemm {
  static constexpr bool kFull = MODE == 1 || MODE == 5;
  static constexpr bool kTA = MODE == 2 || MODE == 3 || MODE == 5;   // A(i,k) read as X[k][i]
};

// One workgroup per output tile; its k-blocks are dealt to the 4 waves (kb = k_lo + w,
// + 4, ...), every wave requests ALL its operands up front (<= 4 k-blocks at M = 256: one
// L2 latency instead of one per k-block), and the 4 partial tiles are summed in LDS in a
// fixed order.
template <int MODE>
__global__ void __launch_bounds__(256)
gpk_kzzg_gemm_kernel(const double* __restrict__ Am, const double* __restrict__ Bm, int M,
                     double* __restrict__ C) {
  using G = KzzGemm<MODE>;
  __shared__ double red[3][256];
  const int T = (M + 15) >> 4;
  const int t = blockIdx.x;
  int ib, jb;
  if (G::kFull) {
    ib = t / T;
    jb = t - ib * T;
  } else {
    tri_tile(t, ib, jb);
  }
  const int lane = threadIdx.x & 63, c = lane & 15, g = lane >> 4;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  int k_lo, k_hi;   // k-blocks [k_lo, k_hi]
  if (MODE == 1) { k_lo = 0; k_hi = ib < jb ? ib : jb; }
  else if (MODE == 4) { k_lo = jb; k_hi = ib; }
  else { k_lo = ib > jb ? ib : jb; k_hi = T - 1; }
  const int i = 16 * ib + c;          // A row of this lane
  const int j = 16 * jb + c;          // B column of this lane
  const bool iok = i < M, jok = j < M;
  constexpr int KPW = 4;              // k-blocks per wave (T <= 16)
  double a[KPW][4], b[KPW][4];
#pragma unroll
  for (int u = 0; u < KPW; ++u) {
    const int kb = k_lo + wave + 4 * u;
#pragma unroll
    for (int s = 0; s < 4; ++s) {     // step s of k-block kb uses k = 16 kb + 4 s + g
      const int k = 16 * kb + 4 * s + g;
      const bool kok = kb <= k_hi && k < M;
      const int kc = kok ? k : 0, ic = iok ? i : 0, jc = jok ? j : 0;
      double av = G::kTA ? Am[(size_t)kc * M + ic] : Am[(size_t)ic * M + kc];
      double bv = MODE == 1 ? Bm[(size_t)jc * M + kc] : Bm[(size_t)kc * M + jc];
      if (MODE == 1 && k > i) av = 0.0;          // G = tril(dLinv)
      a[u][s] = (iok && kok) ? (MODE == 2 ? -av : av) : 0.0;
      b[u][s] = (jok && kok) ? bv : 0.0;
    }
  }
  // every operand in registers before the first MFMA: the loads above are all in flight
  // together (the scheduler would otherwise interleave them with the MFMA chain)
#pragma unroll
  for (int u = 0; u < KPW; ++u)
#pragma unroll
    for (int s = 0; s < 4; ++s) asm volatile("" : "+v"(a[u][s]), "+v"(b[u][s]));
  f64x4 acc = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
  for (int u = 0; u < KPW; ++u)
#pragma unroll
    for (int s = 0; s < 4; ++s) acc = mfma64(a[u][s], b[u][s], acc);
  if (wave > 0) {
#pragma unroll
    for (int r = 0; r < 4; ++r) red[wave - 1][r * 64 + lane] = acc[r];
  }
  __syncthreads();
  if (wave != 0) return;
  // lane (c, g), reg r <-> C[16 ib + g + 4 r][16 jb + c]
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int ii = 16 * ib + g + 4 * r;
    if (ii >= M || !jok) continue;
    double v = ((acc[r] + red[0][r * 64 + lane]) + red[1][r * 64 + lane]) + red[2][r * 64 + lane];
    if (!G::kFull && ib == jb) {
      if (j > ii) v = 0.0;
      if (MODE == 3 && j == ii) v *= 0.5;
    }
    C[(size_t)ii * M + j] = v;
  }
}

// W tile (ib, jb): W_ij = (S_ij + S_ji)/2 * s2 exp(-d2_ij / 2). Per row i of the tile the
// partial sums over j of this column block: part[(jb * M + i) * (D + 1) + {0: w1, 1 + d: Wz_d}].
// One wave per tile; zs rows of both blocks staged in LDS as fp64.
constexpr int kRbfMaxD = 64;
__global__ void __launch_bounds__(64)
gpk_kzzg_rbf_kernel(const double* __restrict__ S, const float* __restrict__ Z,
                    const float* __restrict__ hyp, int M, int D, double* __restrict__ part) {
  __shared__ double zi[16][kRbfMaxD + 1];
  __shared__ double zj[16][kRbfMaxD + 1];
  __shared__ double w[16][17];
  const int T = (M + 15) >> 4;
  const int ib = blockIdx.x / T, jb = blockIdx.x - (blockIdx.x / T) * T;
  const int lane = threadIdx.x;
  const double s2 = (double)hyp[0];
  for (int e = lane; e < 16 * D; e += 64) {
    const int r = e / D, d = e - r * D;
    const int ii = 16 * ib + r, jj = 16 * jb + r;
    const double l = (double)hyp[1 + d];
    zi[r][d] = ii < M ? (double)Z[(size_t)ii * D + d] / l : 0.0;
    zj[r][d] = jj < M ? (double)Z[(size_t)jj * D + d] / l : 0.0;
  }
  __syncthreads();
  // 256 entries, 4 per lane: row r = lane >> 2 ... (entry e = lane + 64 q)
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int e = lane + 64 * q, r = e >> 4, cc = e & 15;
    const int ii = 16 * ib + r, jj = 16 * jb + cc;
    double v = 0.0;
    if (ii < M && jj < M) {
      double d2 = 0.0;
      for (int d = 0; d < D; ++d) {
        const double df = zi[r][d] - zj[cc][d];
        d2 = __builtin_fma(df, df, d2);
      }
      const double kbar = 0.5 * (S[(size_t)ii * M + jj] + S[(size_t)jj * M + ii]);
      v = kbar * s2 * exp(-0.5 * d2);
    }
    w[r][cc] = v;
  }
  __syncthreads();
  // row r = lane & 15, dims d = (lane >> 4) + 4 u
  const int r = lane & 15, q4 = lane >> 4;
  const int ii = 16 * ib + r;
  if (ii >= M) return;
  double* out = part + ((size_t)jb * M + ii) * (D + 1);
  if (q4 == 0) {
    double s = 0.0;
#pragma unroll
    for (int cc = 0; cc < 16; ++cc) s += w[r][cc];
    out[0] = s;
  }
  for (int d = q4; d < D; d += 4) {
    double s = 0.0;
#pragma unroll
    for (int cc = 0; cc < 16; ++cc) s = __builtin_fma(w[r][cc], zj[cc][d], s);
    out[1 + d] = s;
  }
}

// One workgroup per 16-row block ib (16 rows x 16 threads): w1_i and Wz_id summed over the
// column blocks in a fixed order, dZ of those rows, and the block's fixed-order partials
// rpart[ib] = {sum_i w1_i, sum_i (w1_i z_id^2 - Wz_id z_id) for each d} (rows in order).
// (Round 4 ran the row totals and ONE 256-thread workgroup over all M rows: 5 + 19 us.)
__global__ void __launch_bounds__(256)
gpk_kzzg_rows_kernel(const double* __restrict__ part, const float* __restrict__ Z,
                     const float* __restrict__ hyp, int M, int D, float* __restrict__ dZ,
                     double* __restrict__ rpart) {
  __shared__ double cs[16][kRbfMaxD + 1];
  __shared__ double w1s[16];
  const int T = (M + 15) >> 4;
  const int ib = blockIdx.x, tid = threadIdx.x, r = tid >> 4, q = tid & 15;
  const int i = 16 * ib + r;
  const bool iok = i < M;
  const int ic = iok ? i : 0;
  // the T <= 16 column-block partials of a row: all loads issued together (clamped, fixed
  // count), then the fixed-order sum -- a runtime-bounded load + add loop waited per load
  auto colsum = [&](int o) {
    double v[16];
#pragma unroll
    for (int jb = 0; jb < 16; ++jb) v[jb] = part[((size_t)(jb < T ? jb : 0) * M + ic) * (D + 1) + o];
    double t = 0.0;
#pragma unroll
    for (int jb = 0; jb < 16; ++jb) t += jb < T ? v[jb] : 0.0;
    return t;
  };
  const double w1 = iok ? colsum(0) : 0.0;
  if (q == 0) w1s[r] = w1;
  for (int d = q; d < D; d += 16) {
    double c = 0.0;
    if (iok) {
      const double wz = colsum(1 + d);
      const double l = (double)hyp[1 + d];
      const double z = (double)Z[(size_t)i * D + d] / l;
      dZ[(size_t)i * D + d] = (float)(2.0 * (wz - z * w1) / l);
      c = w1 * z * z - wz * z;
    }
    cs[r][d] = c;
  }
  __syncthreads();
  double* out = rpart + (size_t)ib * (D + 1);
  if (tid < D) {
    double s = 0.0;
#pragma unroll
    for (int rr = 0; rr < 16; ++rr) s += cs[rr][tid];
    out[1 + tid] = s;
  } else if (tid == D) {
    double s = 0.0;
#pragma unroll
    for (int rr = 0; rr < 16; ++rr) s += w1s[rr];
    out[0] = s;
  }
}

// dhyp = {ds2 = sum w1 / s2, dl_d = 2 / l_d sum_i (...)} from the row-block partials, summed
// over the blocks in a fixed order. One wave per output group.
__global__ void __launch_bounds__(128)
gpk_kzzg_fin_kernel(const double* __restrict__ rpart, const float* __restrict__ hyp, int M, int D,
                    float* __restrict__ dhyp) {
  const int e = threadIdx.x;
  if (e > D) return;
  const int T = (M + 15) >> 4;
  double v[16];
#pragma unroll
  for (int ib = 0; ib < 16; ++ib) v[ib] = rpart[(size_t)(ib < T ? ib : 0) * (D + 1) + e];
  double s = 0.0;
#pragma unroll
  for (int ib = 0; ib < 16; ++ib) s += ib < T ? v[ib] : 0.0;
  dhyp[e] = e == 0 ? (float)(s / (double)hyp[0]) : (float)(2.0 * s / (double)hyp[e]);
}

template <int MODE>
hipError_t launch_gemm(const double* A, const double* B, int M, double* C, hipStream_t stream) {
  const int T = (M + 15) >> 4;
  const int ntile = KzzGemm<MODE>::kFull ? T * T : T * (T + 1) / 2;
  hipLaunchKernelGGL((gpk_kzzg_gemm_kernel<MODE>), dim3(ntile), dim3(256), 0, stream, A, B, M, C);
  return hipGetLastError();
}

}  // namespace

size_t gpk_kzz_grad_ws_bytes(int M, int D) {
  const int T = (M + 15) >> 4;
  return (2 * (size_t)M * M + (size_t)(T + 1) * M * (D + 1)) * sizeof(double);
}

int gpk_launch_kzz_grad(const GpkKzzGradArgs& a, hipStream_t stream) {
  const int M = a.M, D = a.D;
  double* b0 = (double*)a.ws;
  double* b1 = b0 + (size_t)M * M;
  double* part = b1 + (size_t)M * M;
  hipError_t e;
  if ((e = launch_gemm<1>(a.dLinv, a.Linv, M, b0, stream)) != hipSuccess) return (int)e;   // T1
  if ((e = launch_gemm<2>(a.Linv, b0, M, b1, stream)) != hipSuccess) return (int)e;        // Lbar
  if ((e = launch_gemm<3>(a.L, b1, M, b0, stream)) != hipSuccess) return (int)e;           // P
  if ((e = launch_gemm<4>(b0, a.Linv, M, b1, stream)) != hipSuccess) return (int)e;        // U
  if ((e = launch_gemm<5>(a.Linv, b1, M, b0, stream)) != hipSuccess) return (int)e;        // S
  const int T = (M + 15) >> 4;
  hipLaunchKernelGGL(gpk_kzzg_rbf_kernel, dim3(T * T), dim3(64), 0, stream, b0, a.Z, a.hyp, M, D, part);
  if ((e = hipGetLastError()) != hipSuccess) return (int)e;
  double* rpart = part + (size_t)T * M * (D + 1);
  hipLaunchKernelGGL(gpk_kzzg_rows_kernel, dim3(T), dim3(256), 0, stream, part, a.Z, a.hyp, M, D, a.dZ,
                     rpart);
  if ((e = hipGetLastError()) != hipSuccess) return (int)e;
  hipLaunchKernelGGL(gpk_kzzg_fin_kernel, dim3(1), dim3(128), 0, stream, rpart, a.hyp, M, D, a.dhyp);
  e = hipGetLastError();
  return e == hipSuccess ? 0 : (int)e;
}
