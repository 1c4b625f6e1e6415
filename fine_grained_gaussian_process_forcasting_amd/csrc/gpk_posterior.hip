// Exact-GP posterior at new inputs (eval mode) for gfx950.
//
// Replaces, per window b, GPyTorch's exact prediction strategy behind
// ExactGPModel in eval mode (reference denoising_model/GPModel.py:10-13; upstream
// models/exact_gp.py __call__ -> models/exact_prediction_strategies.py
// exact_predictive_mean / exact_predictive_covar), given the training factor
// L = chol(K_hat) and z = L^{-1}(y - c) that gpk_exact_mll_f32 already produced
// (GPyTorch's mean_cache = K_hat^{-1}(y - c) = L^{-T} z):
//   K*   = s2 * exp(-0.5 ||(x_n - x*_t)/l||^2)                 (N x Ns)
//   V    = L^{-1} K*
//   mean = c + V^T z                                          (= c + K*^T K_hat^{-1}(y - c))
//   var  = s2 - colsum(V o V)                                 (= diag(K** - K*^T K_hat^{-1} K*))
// (latent f; the likelihood adds the noise, the MVN clamps at min_variance).
//
// Design: one workgroup of 4 waves per (window, 64 test points); each wave owns
// 16 test columns and runs the blocked forward substitution down the NB block
// rows of L with its V tiles held in REGISTERS (acc layout, gpk_common.h):
//   C_i  = K*_i - sum_{j<i} L_ij V_j     (fp32 MFMA; L_ij read as one 16-B load
//                                         per lane: A[c][4g+r] = L[16i+c][16j+4g+r])
//   V_i  = (L_ii)^{-1} C_i               (fp32 MFMA; the 16 diagonal-block inverses
//                                         are formed once per workgroup into LDS)
// K*_i comes from a centred fp32-MFMA Gram against the LDS-staged training inputs.
// No barrier after the prologue: the waves never exchange data.
#include "gpk_common.h"
#include "gpk_internal.h"

#include <mutex>

namespace {

constexpr int kPostWaves = 4;
constexpr int kPostCols = 16 * kPostWaves;   // test points per workgroup

struct PostLds {
  int xtr, nrm, zv, dinv, ltmp, red, total;   // float offsets
};

__host__ __device__ inline PostLds post_lds_layout(int NB, int DP) {
  PostLds o;
  const int NP = 16 * NB;
  o.xtr = 0;                                  // NP x (DP + 4), scaled by 1/l, centred
  o.nrm = o.xtr + NP * (DP + 4);              // ||x_n||^2
  o.zv = o.nrm + NP;                          // z (padded with zeros)
  o.dinv = o.zv + NP;                         // NB x 16 x 16 inverses of the diagonal blocks
  o.ltmp = o.dinv + NB * 256;                 // NB x 16 x 16 diagonal blocks of L
  o.red = o.ltmp + NB * 256;                  // column-mean partials (256) + means (DP)
  o.total = o.red + 256 + 64;
  return o;
}

GPK_DEVICE f32x4 mfma4(const f32x4 a, const f32x4 b, f32x4 d) {
  d = __builtin_amdgcn_mfma_f32_16x16x4f32(a[0], b[0], d, 0, 0, 0);
  d = __builtin_amdgcn_mfma_f32_16x16x4f32(a[1], b[1], d, 0, 0, 0);
  d = __builtin_amdgcn_mfma_f32_16x16x4f32(a[2], b[2], d, 0, 0, 0);
  d = __builtin_amdgcn_mfma_f32_16x16x4f32(a[3], b[3], d, 0, 0, 0);
  return d;
}

// NB = ceil(N/16) block rows, DQ = DP/16 (DP = D padded to 16/32/64), FULL: N == 16*NB.
template <int NB, int DQ, bool FULL>
__global__ __launch_bounds__(256) void gpk_post_kernel(GpkPostArgs a) {
  extern __shared__ float smem[];
  constexpr int DP = 16 * DQ;
  constexpr int XS = DP + 4;
  constexpr int NP = 16 * NB;
  const PostLds lay = post_lds_layout(NB, DP);
  const int N = FULL ? NP : a.N;
  const int D = a.D, Ns = a.Ns;
  const int T = (Ns + kPostCols - 1) / kPostCols;
  // XCD-aware order: the test tiles of one window go to the same XCD (shared L2 for L)
  const int total = a.B * T;
  int id = blockIdx.x;
  if ((total & 7) == 0) id = (id & 7) * (total >> 3) + (id >> 3);
  const int b = id / T, tile = id - b * T;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int c = lane & 15, g = lane >> 4;

  const float s2 = a.hyp[0];
  const float c0 = a.hyp[2];
  const float* ls = a.hyp + 3;
  const bool ard = a.n_ls > 1;
  float* xtr = smem + lay.xtr;
  float* nrm = smem + lay.nrm;
  float* zv = smem + lay.zv;
  float* dinv = smem + lay.dinv;
  float* ltmp = smem + lay.ltmp;
  float* red = smem + lay.red;
  const float* Xb = a.X + (size_t)b * N * D;
  const float* Lb = a.L + (size_t)b * N * N;

  // ---- prologue: training inputs / l into LDS (zero padded), z, diagonal blocks of L
  // 8 unconditional loads (clamped addresses) in flight per thread, then the stores: a
  // predicated load per loop iteration would cost one full memory latency each
  for (int base = 0; base < NP * DP; base += 8 * 256) {
    float v[8], l[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int e = base + u * 256 + tid, n = e / DP, d = e - n * DP;
      const bool ok = e < NP * DP && n < N && d < D;
      v[u] = Xb[ok ? (size_t)n * D + d : 0];
      l[u] = ls[(ok && ard) ? d : 0];
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int e = base + u * 256 + tid, n = e / DP, d = e - n * DP;
      if (e < NP * DP) xtr[n * XS + d] = (n < N && d < D) ? v[u] / l[u] : 0.f;
    }
  }
  for (int n = tid; n < NP; n += 256) zv[n] = n < N ? a.z[(size_t)b * N + n] : 0.f;
  {
    const int bi = tid >> 4, m = tid & 15;   // tile bi, row m (NB <= 16 -> 256 rows)
    if (bi < NB) {
      const int row = 16 * bi + m;
      float lv[16];
#pragma unroll
      for (int k = 0; k < 16; ++k) {   // unconditional (clamped) loads, all in flight
        const bool ok = k <= m && row < N;
        lv[k] = Lb[ok ? (size_t)row * N + 16 * bi + k : 0];
      }
#pragma unroll
      for (int k = 0; k < 16; ++k) {
        const int col = 16 * bi + k;
        float v = (row == col) ? 1.f : 0.f;  // identity on padded rows
        if (k <= m && row < N) v = lv[k];
        ltmp[bi * 256 + m * 16 + k] = v;
      }
    }
  }
  lds_barrier();
  // column means over the N real rows (GPyTorch centres the Gram; here by the training mean)
  {
    constexpr int P = 256 / DP;
    const int d = tid % DP, part = tid / DP;
    float s = 0.f;
    for (int n = part; n < N; n += P) s += xtr[n * XS + d];
    red[tid] = s;
  }
  // inverses of the diagonal blocks: thread = (block, column), forward substitution
  {
    const int bi = tid >> 4, cc = tid & 15;
    if (bi < NB) {
      const float* Lt = ltmp + bi * 256;
      float x[16];
#pragma unroll
      for (int m = 0; m < 16; ++m) {
        float s = (m == cc) ? 1.f : 0.f;
#pragma unroll
        for (int k = 0; k < m; ++k) s = __builtin_fmaf(-Lt[m * 16 + k], x[k], s);
        x[m] = (m < cc) ? 0.f : s / Lt[m * 16 + m];
      }
#pragma unroll
      for (int m = 0; m < 16; ++m) dinv[bi * 256 + m * 16 + cc] = x[m];
    }
  }
  lds_barrier();
  if (tid < DP) {
    float s = 0.f;
    for (int p = 0; p < 256 / DP; ++p) s += red[p * DP + tid];
    red[256 + tid] = s / (float)N;
  }
  lds_barrier();
  for (int e = tid; e < N * DP; e += 256) {
    const int n = e / DP, d = e - n * DP;
    if (d < D) xtr[n * XS + d] -= red[256 + d];
  }
  lds_barrier();
  for (int n = tid; n < NP; n += 256) {
    float s = 0.f;
#pragma unroll 8
    for (int d = 0; d < DP; ++d) s = __builtin_fmaf(xtr[n * XS + d], xtr[n * XS + d], s);
    nrm[n] = s;
  }
  lds_barrier();

  // ---- this lane's test point (column c of wave w): B operand of the Gram, k = 16q + 4g + r
  const int col = tile * kPostCols + 16 * w + c;
  const bool live = col < Ns;
  f32x4 xs[DQ];
  float nxs = 0.f;
  {
    // all DQ*4 coordinates requested before any is used: clamped in-bounds addresses,
    // the dead lanes/coordinates masked afterwards
    const float* xrow = a.Xs + ((size_t)b * Ns + (live ? col : 0)) * D;
    float raw[DQ][4];
#pragma unroll
    for (int q = 0; q < DQ; ++q)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int d = 16 * q + 4 * g + r;
        raw[q][r] = xrow[d < D ? d : 0];
      }
#pragma unroll
    for (int q = 0; q < DQ; ++q) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int d = 16 * q + 4 * g + r;
        float v = 0.f;
        if (live && d < D) v = raw[q][r] / (ard ? ls[d] : ls[0]) - red[256 + d];
        xs[q][r] = v;
        nxs = __builtin_fmaf(v, v, nxs);
      }
    }
  }
  nxs += __shfl_xor(nxs, 16, 64);
  nxs += __shfl_xor(nxs, 32, 64);

  constexpr float nhalf_log2e = -0.72134752044448170f;
  f32x4 V[NB];
  float mp = 0.f, vp = 0.f;
#pragma unroll
  for (int i = 0; i < NB; ++i) {
    // FULL: this lane's L row-block operands for the update below, all requested up front
    // (they come from L2: one latency per block row, hidden under the Gram tile and exp2;
    // fetching them a block row earlier measured no faster). The ragged path keeps
    // per-element predicated loads at their use (hoisting 4 scalars per block would double
    // its register footprint).
    const int lrow = 16 * i + c;
    f32x4 la[NB > 1 ? NB - 1 : 1];
    if (FULL) {
#pragma unroll
      for (int j = 0; j < i; ++j) la[j] = *(const f32x4*)&Lb[(size_t)lrow * N + 16 * j + 4 * g];
      __builtin_amdgcn_sched_barrier(0);   // keep the loads issued here, ahead of the Gram
    }
    // K*_i (acc layout: reg r = row 16i + 4g + r, column c)
    f32x4 G = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int q = 0; q < DQ; ++q) {
      const f32x4 xa = *(const f32x4*)&xtr[(16 * i + c) * XS + 16 * q + 4 * g];
      G = mfma4(xa, xs[q], G);
    }
    f32x4 Cm;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int row = 16 * i + 4 * g + r;
      const float d2 = __builtin_fmaxf(nrm[row] + nxs - 2.f * G[r], 0.f);
      float k = s2 * __builtin_amdgcn_exp2f(d2 * nhalf_log2e);
      if (!FULL && row >= N) k = 0.f;
      Cm[r] = k;
    }
    // - sum_{j<i} L_ij V_j (two accumulators: halves the dependent MFMA chain)
    f32x4 U0 = {0.f, 0.f, 0.f, 0.f}, U1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int j = 0; j < i; ++j) {
      f32x4 lj;
      if (FULL) {
        lj = la[j];
      } else {
#pragma unroll
        for (int r = 0; r < 4; ++r) lj[r] = lrow < N ? Lb[(size_t)lrow * N + 16 * j + 4 * g + r] : 0.f;
      }
      if (j & 1) U1 = mfma4(lj, V[j], U1);
      else U0 = mfma4(lj, V[j], U0);
    }
    Cm = Cm - U0 - U1;
    const f32x4 di = *(const f32x4*)&dinv[i * 256 + c * 16 + 4 * g];
    const f32x4 z0 = {0.f, 0.f, 0.f, 0.f};
    V[i] = mfma4(di, Cm, z0);
    const f32x4 zz = *(const f32x4*)&zv[16 * i + 4 * g];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      mp = __builtin_fmaf(V[i][r], zz[r], mp);
      vp = __builtin_fmaf(V[i][r], V[i][r], vp);
    }
  }
  mp += __shfl_xor(mp, 16, 64);
  mp += __shfl_xor(mp, 32, 64);
  vp += __shfl_xor(vp, 16, 64);
  vp += __shfl_xor(vp, 32, 64);
  if (g == 0 && live) {
    a.mean[(size_t)b * Ns + col] = c0 + mp;
    a.var[(size_t)b * Ns + col] = s2 - vp;
  }
}

template <int NB, int DQ>
int launch_post(const GpkPostArgs& a, hipStream_t stream) {
  const PostLds lay = post_lds_layout(NB, 16 * DQ);
  const size_t lds = (size_t)lay.total * sizeof(float);
  const int T = (a.Ns + kPostCols - 1) / kPostCols;
  const long long grid = (long long)a.B * T;
  if (grid > 0x7fffffff) return -6;
  if (a.N == 16 * NB) {
    static std::once_flag once;
    std::call_once(once, [&] {
      (void)hipFuncSetAttribute((const void*)gpk_post_kernel<NB, DQ, true>,
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
      (void)hipGetLastError();
    });
    hipLaunchKernelGGL((gpk_post_kernel<NB, DQ, true>), dim3((unsigned)grid), dim3(256), lds, stream, a);
  } else {
    static std::once_flag once;
    std::call_once(once, [&] {
      (void)hipFuncSetAttribute((const void*)gpk_post_kernel<NB, DQ, false>,
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
      (void)hipGetLastError();
    });
    hipLaunchKernelGGL((gpk_post_kernel<NB, DQ, false>), dim3((unsigned)grid), dim3(256), lds, stream, a);
  }
  return (int)hipGetLastError();
}

template <int NB>
int launch_post_nb(const GpkPostArgs& a, hipStream_t stream) {
  if (a.D <= 16) return launch_post<NB, 1>(a, stream);
  if (a.D <= 32) return launch_post<NB, 2>(a, stream);
  return launch_post<NB, 4>(a, stream);
}

}  // namespace

size_t gpk_post_lds_bytes(int N, int D) {
  const int NB = (N + 15) / 16;
  const int DP = D <= 16 ? 16 : (D <= 32 ? 32 : 64);
  return (size_t)post_lds_layout(NB, DP).total * sizeof(float);
}

int gpk_launch_exact_posterior(const GpkPostArgs& a, hipStream_t stream) {
  switch ((a.N + 15) / 16) {
#define GPK_POST_CASE(nb) case nb: return launch_post_nb<nb>(a, stream);
    GPK_POST_CASE(1) GPK_POST_CASE(2) GPK_POST_CASE(3) GPK_POST_CASE(4)
    GPK_POST_CASE(5) GPK_POST_CASE(6) GPK_POST_CASE(7) GPK_POST_CASE(8)
    GPK_POST_CASE(9) GPK_POST_CASE(10) GPK_POST_CASE(11) GPK_POST_CASE(12)
    GPK_POST_CASE(13) GPK_POST_CASE(14) GPK_POST_CASE(15) GPK_POST_CASE(16)
#undef GPK_POST_CASE
    default: return -6;
  }
}
