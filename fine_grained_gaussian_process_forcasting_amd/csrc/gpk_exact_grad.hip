// Analytic backward of the exact-GP marginal log likelihood (gfx950), per window b:
//
//   mll   = -0.5 (r^T K^-1 r + log|K| + N log 2pi) / N,  r = y - c,  K = K_hat (+ jitter)
//   G     = dmll/dK = g (alpha alpha^T - K^-1) / (2N),    alpha = K^-1 r = L^-T z
//   ds2   = sum_ij G_ij E_ij            (E = exp(-d/2), K = s2 E + noise I)
//   dnoise= sum_i G_ii
//   dc    = g sum_i alpha_i / N,   dy = -g alpha / N
//   W     = G o (s2 E) (zero diagonal),  w1 = W 1,  Wx = W xs  (xs = x / l, centred)
//   dxs_i = -2 (xs_i w1_i - Wx_i),   dx = dxs / l,
//   dl_d  = (2 / l_d) sum_i xs_id (xs_id w1_i - Wx_id)   (summed over d for a scalar l)
//
// which is what torch autograd produces through GPyTorch's ExactMarginalLogLikelihood
// (reference GPModel.py:5-13; upstream mlls/exact_marginal_log_likelihood.py,
// linear_operator inv_quad_logdet + psd_safe_cholesky backward) when train.py:166
// calls loss.backward(); oracle: oracle/gp_oracle.py::exact_mll_grads.
//
// Inputs are the forward's outputs (L, z), so nothing is refactored. One workgroup
// (8 waves) per window, three phases separated by workgroup barriers:
//   0. inverses of the 16 diagonal blocks of L (forward substitution, one lane
//      per column, L entries read as uniform scalars);
//   1. L^-1 by block columns (wave w owns columns J = w mod 8):
//      Linv_IJ = -Linv_II sum_{K=J}^{I-1} L_IK Linv_KJ   (fp32 MFMA 16x16x4),
//      tiles kept in a caller workspace in acc layout (one float4 per lane);
//   2. alpha = Linv^T z; then for every tile (I <= J): K^-1_IJ = sum_K Linv_KI^T
//      Linv_KJ, G, the RBF recomputed from xs (MFMA Gram), and the reductions:
//      ds2 / dnoise in registers, w1 and Wx = W xs (both MFMA orientations) as
//      LDS float atomics;
//   3. per-row dx, dy and the lengthscale sums.
#include "gpk_common.h"
#include "gpk_internal.h"

namespace {

constexpr int kNW = 8;           // waves per workgroup (one window)
constexpr int kT = 64 * kNW;

// acc-layout tile of L^T for block (I, K): lane (g, c) reg r <- L[16I + c][16K + 4g + r]
// (padding beyond N is the identity).
GPK_DEVICE f32x4 load_LT(const float* Lb, int N, int I, int K, int lane) {
  const int c = lane & 15, g = lane >> 4;
  const int row = 16 * I + c, col = 16 * K + 4 * g;
  f32x4 v;
  if ((N & 3) == 0 && row < N && col + 3 < N) {
    v = *(const f32x4*)&Lb[(size_t)row * N + col];
  } else {
#pragma unroll
    for (int r = 0; r < 4; ++r)
      v[r] = (row < N && col + r < N) ? Lb[(size_t)row * N + col + r] : (row == col + r ? 1.f : 0.f);
  }
  return v;
}

GPK_DEVICE f32x4 ws_load(const float* ws, int NB, int I, int J, int lane) {
  return *(const f32x4*)&ws[((size_t)(I * NB + J) * 64 + lane) * 4];
}
GPK_DEVICE void ws_store(float* ws, int NB, int I, int J, int lane, const f32x4 v) {
  *(f32x4*)&ws[((size_t)(I * NB + J) * 64 + lane) * 4] = v;
}

GPK_DEVICE void lds_add(float* p, float v) {
  (void)__hip_atomic_fetch_add(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// Sum over the 16 lanes of each row (lanes sharing g), DPP only.
GPK_DEVICE float row16_sum(float v) {
#define GPK_DPP_ADD(ctrl) \
  v += __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), ctrl, 0xf, 0xf, false));
  GPK_DPP_ADD(0xB1) GPK_DPP_ADD(0x4E) GPK_DPP_ADD(0x141) GPK_DPP_ADD(0x140)
#undef GPK_DPP_ADD
  return v;
}

template <int NB>
__global__ void __launch_bounds__(kT, 1)
gpk_exact_grad_kernel(const float* __restrict__ X, const float* __restrict__ Lg,
                      const float* __restrict__ zg, const float* __restrict__ hyp, int n_ls,
                      int N, int D, int DP, const float* __restrict__ gout,
                      float* __restrict__ ws_all, float* __restrict__ dX, float* __restrict__ dy,
                      float* __restrict__ dhyp) {
  constexpr int NP = NB * 16;
  extern __shared__ __attribute__((aligned(16))) float smem[];
  float* dinvT = smem;                 // NB tiles: acc layout of Linv_II^T
  float* xs = dinvT + NB * 256;        // NP x DP, centred x / l
  float* Wx = xs + NP * DP;            // NP x DP
  float* w1 = Wx + NP * DP;            // NP
  float* alpha = w1 + NP;              // NP
  float* nrm = alpha + NP;             // NP
  float* scr = nrm + NP;               // kNW waves x 256 (transposes)
  float* part = scr + kNW * 256;       // kT partial sums
  float* red = part + kT;              // 3 * kNW

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int c = lane & 15, g = lane >> 4;
  const int b = blockIdx.x;
  const float* Lb = Lg + (size_t)b * N * N;
  float* ws = ws_all + (size_t)b * NB * NB * 256;
  const float s2 = hyp[0];
  const float gw = gout[b];
  const float gs = gw / (2.f * (float)N);

  // ---- 0. diagonal block inverses: lane c < 16 solves column c of L_II X = I
  for (int I = wave; I < NB; I += kNW) {
    if (lane < 16) {
      float x[16];
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int gi = 16 * I + i;
        float s = (i == c) ? 1.f : 0.f;
#pragma unroll
        for (int k = 0; k < i; ++k) {
          const int gk = 16 * I + k;
          const float lik = (gi < N && gk < N) ? Lb[(size_t)gi * N + gk] : 0.f;
          s = __builtin_fmaf(-lik, x[k], s);
        }
        const float lii = (gi < N) ? Lb[(size_t)gi * N + gi] : 1.f;
        x[i] = s / lii;
      }
      // Linv_II (acc layout) -> workspace; Linv_II^T (acc layout) -> LDS
      float* t = dinvT + I * 256;
#pragma unroll
      for (int i = 0; i < 16; ++i) t[(16 * (c >> 2) + i) * 4 + (c & 3)] = x[i];  // X^T[c][i]
#pragma unroll
      for (int i = 0; i < 16; ++i)
        ws[((size_t)(I * NB + I) * 64 + 16 * (i >> 2) + c) * 4 + (i & 3)] = x[i];  // X[i][c]
    }
  }
  __syncthreads();

  // ---- 1. block columns of L^-1
  for (int J = wave; J < NB; J += kNW) {
    for (int I = J + 1; I < NB; ++I) {
      f32x4 s0 = {0.f, 0.f, 0.f, 0.f}, s1 = {0.f, 0.f, 0.f, 0.f};
      int K = J;
      for (; K + 1 < I; K += 2) {
        const f32x4 a0 = load_LT(Lb, N, I, K, lane), p0 = ws_load(ws, NB, K, J, lane);
        const f32x4 a1 = load_LT(Lb, N, I, K + 1, lane), p1 = ws_load(ws, NB, K + 1, J, lane);
        s0 = mma_tn(a0, p0, s0);
        s1 = mma_tn(a1, p1, s1);
      }
      if (K < I) s0 = mma_tn(load_LT(Lb, N, I, K, lane), ws_load(ws, NB, K, J, lane), s0);
      const f32x4 qt = *(const f32x4*)&dinvT[I * 256 + lane * 4];
      const f32x4 v = mma_tn(qt, s0 + s1, f32x4{0.f, 0.f, 0.f, 0.f});
      ws_store(ws, NB, I, J, lane, -v);
    }
  }
  // ---- 2a. xs = x / l (centred over the N real rows), norms, zeroed accumulators
  for (int q = tid; q < NP * DP; q += kT) {
    const int n = q / DP, d = q - n * DP;
    float v = 0.f;
    if (n < N && d < D) v = X[((size_t)b * N + n) * D + d] / hyp[3 + (n_ls == 1 ? 0 : d)];
    xs[q] = v;
    Wx[q] = 0.f;
  }
  for (int q = tid; q < NP; q += kT) w1[q] = 0.f;
  __syncthreads();  // also publishes the workspace tiles of phase 1
  {
    const int parts = kT / DP;
    const int p = tid / DP, d = tid - p * DP;
    if (p < parts) {
      float s = 0.f;
      for (int n = p; n < N; n += parts) s += xs[n * DP + d];
      part[p * DP + d] = s;
    }
    __syncthreads();
    if (tid < DP) {
      float s = 0.f;
      for (int q = 0; q < parts; ++q) s += part[q * DP + tid];
      part[kT - DP + tid] = s / (float)N;  // (only read after the barrier below)
    }
    __syncthreads();
    for (int q = tid; q < N * DP; q += kT) {
      const int d = q % DP;
      if (d < D) xs[q] -= part[kT - DP + d];
    }
    __syncthreads();
    for (int n = tid; n < NP; n += kT) {
      float s = 0.f;
      for (int d = 0; d < DP; ++d) s = __builtin_fmaf(xs[n * DP + d], xs[n * DP + d], s);
      nrm[n] = s;
    }
  }
  // alpha = L^-T z (block rows I = wave mod 4); column 0 of each Z tile is live
  for (int I = wave; I < NB; I += kNW) {
    f32x4 a = {0.f, 0.f, 0.f, 0.f};
    for (int K = I; K < NB; ++K) {
      f32x4 zt;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = 16 * K + 4 * g + r;
        zt[r] = (c == 0 && row < N) ? zg[(size_t)b * N + row] : 0.f;
      }
      a = mma_tn(ws_load(ws, NB, K, I, lane), zt, a);
    }
    if (c == 0) {
#pragma unroll
      for (int r = 0; r < 4; ++r) alpha[16 * I + 4 * g + r] = a[r];
    }
  }
  __syncthreads();

  // ---- 2b. tiles (I <= J)
  float ds2 = 0.f, dnz = 0.f;
  float* sc = scr + wave * 256;
  int t = 0;
  for (int J = 0; J < NB; ++J) {
    for (int I = 0; I <= J; ++I, ++t) {
      if (t % kNW != wave) continue;
      // K^-1_IJ
      f32x4 k0 = {0.f, 0.f, 0.f, 0.f}, k1 = {0.f, 0.f, 0.f, 0.f};
      int K = J;
      for (; K + 1 < NB; K += 2) {
        const f32x4 a0 = ws_load(ws, NB, K, I, lane), b0 = ws_load(ws, NB, K, J, lane);
        const f32x4 a1 = ws_load(ws, NB, K + 1, I, lane), b1 = ws_load(ws, NB, K + 1, J, lane);
        k0 = mma_tn(a0, b0, k0);
        k1 = mma_tn(a1, b1, k1);
      }
      if (K < NB) k0 = mma_tn(ws_load(ws, NB, K, I, lane), ws_load(ws, NB, K, J, lane), k0);
      const f32x4 kinv = k0 + k1;
      // Gram of xs rows (contraction over d in chunks of 16)
      f32x4 gr = {0.f, 0.f, 0.f, 0.f};
      for (int dd = 0; dd < DP; dd += 16) {
        const f32x4 qi = *(const f32x4*)&xs[(16 * I + c) * DP + dd + 4 * g];
        const f32x4 qj = *(const f32x4*)&xs[(16 * J + c) * DP + dd + 4 * g];
        gr = mma_tn(qi, qj, gr);
      }
      const int col = 16 * J + c;
      const float aj = alpha[col], nj = nrm[col];
      f32x4 W;
      float csum = 0.f;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = 16 * I + 4 * g + r;
        float G = (alpha[row] * aj - kinv[r]) * gs;
        if (row >= N || col >= N) G = 0.f;
        float dist = nrm[row] + nj - 2.f * gr[r];
        dist = dist < 0.f ? 0.f : dist;
        if (row == col) dist = 0.f;
        const float E = __expf(-0.5f * dist);
        ds2 += (I == J ? 1.f : 2.f) * G * E;
        if (row == col) dnz += G;
        float w = G * s2 * E;
        if (row == col) w = 0.f;
        W[r] = w;
        csum += w;
      }
      // w1: row sums (rows of block I) and, off the diagonal, column sums (rows of J)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float rs = row16_sum(W[r]);
        if (c == 0) lds_add(&w1[16 * I + 4 * g + r], rs);
      }
      if (I != J) lds_add(&w1[col], csum);
      // Wx_J += W^T xs_I ; Wx_I += W xs_J (I != J)
      *(f32x4*)&sc[lane * 4] = W;  // for the transpose below
      for (int dd = 0; dd < DP; dd += 16) {
        f32x4 pi;
#pragma unroll
        for (int r = 0; r < 4; ++r) pi[r] = xs[(16 * I + 4 * g + r) * DP + dd + c];
        const f32x4 o = mma_tn(W, pi, f32x4{0.f, 0.f, 0.f, 0.f});  // rows j, dims dd + c
#pragma unroll
        for (int r = 0; r < 4; ++r) lds_add(&Wx[(16 * J + 4 * g + r) * DP + dd + c], o[r]);
      }
      if (I != J) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront", "local");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront", "local");
        f32x4 wt;  // acc layout of W^T: W^T[4g + r][c] = W[c][4g + r]
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int a = c, bb = 4 * g + r;  // element W[a][bb]
          wt[r] = sc[(16 * (a >> 2) + bb) * 4 + (a & 3)];
        }
        for (int dd = 0; dd < DP; dd += 16) {
          f32x4 pj;
#pragma unroll
          for (int r = 0; r < 4; ++r) pj[r] = xs[(16 * J + 4 * g + r) * DP + dd + c];
          const f32x4 o = mma_tn(wt, pj, f32x4{0.f, 0.f, 0.f, 0.f});  // rows i
#pragma unroll
          for (int r = 0; r < 4; ++r) lds_add(&Wx[(16 * I + 4 * g + r) * DP + dd + c], o[r]);
        }
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront", "local");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront", "local");
    }
  }
  ds2 = wave_sum(ds2);
  dnz = wave_sum(dnz);
  if (lane == 0) {
    red[wave] = ds2;
    red[kNW + wave] = dnz;
  }
  __syncthreads();

  // ---- 3. per-row outputs and the lengthscale / constant sums
  const float invN = 1.f / (float)N;
  float asum = 0.f;
  for (int n = tid; n < N; n += kT) {
    const float an = alpha[n];
    asum += an;
    if (dy != nullptr) dy[(size_t)b * N + n] = -gw * an * invN;
  }
  // thread (row n) accumulates xs_nd (xs_nd w1_n - Wx_nd) per d into part[d] via atomics
  for (int q = tid; q < DP; q += kT) part[q] = 0.f;
  __syncthreads();
  for (int n = tid; n < N; n += kT) {
    const float wn = w1[n];
    for (int d = 0; d < D; ++d) {
      const float x = xs[n * DP + d];
      const float e = x * wn - Wx[n * DP + d];  // = -dxs / 2
      const float l = hyp[3 + (n_ls == 1 ? 0 : d)];
      if (dX != nullptr) dX[((size_t)b * N + n) * D + d] = -2.f * e / l;
      lds_add(&part[d], x * e);
    }
  }
  asum = wave_sum(asum);
  if (lane == 0) red[2 * kNW + wave] = asum;
  __syncthreads();
  if (tid == 0) {
    float* o = dhyp + (size_t)b * (3 + n_ls);
    float a0 = 0.f, a1 = 0.f, a2 = 0.f;
    for (int w = 0; w < kNW; ++w) {
      a0 += red[w];
      a1 += red[kNW + w];
      a2 += red[2 * kNW + w];
    }
    o[0] = a0;
    o[1] = a1;
    o[2] = gw * a2 * invN;
    if (n_ls == 1) {
      float s = 0.f;
      for (int d = 0; d < D; ++d) s += part[d];
      o[3] = 2.f * s / hyp[3];
    } else {
      for (int d = 0; d < D; ++d) o[3 + d] = 2.f * part[d] / hyp[3 + d];
    }
  }
}

template <int NB>
int launch_grad_nb(const GpkExactGradArgs& a, hipStream_t stream) {
  const int DP = (a.D + 15) / 16 * 16;
  if (DP > 64) return -7;
  const size_t lds = sizeof(float) * ((size_t)NB * 256 + 2 * (size_t)NB * 16 * DP + 3 * NB * 16 + kNW * 256 + kT + 3 * kNW);
  if (lds > 160 * 1024) return -7;
  if (lds > 64 * 1024)
    (void)hipFuncSetAttribute((const void*)gpk_exact_grad_kernel<NB>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  hipLaunchKernelGGL((gpk_exact_grad_kernel<NB>), dim3(a.B), dim3(kT), lds, stream, a.X, a.L, a.z,
                     a.hyp, a.n_ls, a.N, a.D, DP, a.gout, a.ws, a.dX, a.dy, a.dhyp);
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? 0 : (int)e;
}

}  // namespace

size_t gpk_exact_grad_ws_floats(int B, int N) {
  const size_t NB = (size_t)(N + 15) / 16;
  return (size_t)B * NB * NB * 256;
}

int gpk_launch_exact_grad(const GpkExactGradArgs& a, hipStream_t stream) {
  const int NB = (a.N + 15) / 16;
  switch (NB) {
#define GPK_CASE(nb) case nb: return launch_grad_nb<nb>(a, stream);
    GPK_CASE(1) GPK_CASE(2) GPK_CASE(3) GPK_CASE(4) GPK_CASE(5) GPK_CASE(6)
    GPK_CASE(7) GPK_CASE(8) GPK_CASE(9) GPK_CASE(10) GPK_CASE(11) GPK_CASE(12)
    GPK_CASE(13) GPK_CASE(14) GPK_CASE(15) GPK_CASE(16)
#undef GPK_CASE
    default: return -6;
  }
}
