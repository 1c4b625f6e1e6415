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
// Three launches, inputs are the forward's L and z (nothing is refactored):
//   gpk_grad_solve_kernel  one workgroup (16 waves) per window: alpha = L^-T z, dy, and the
//       lower block tiles of K^-1: wave J solves block column J with its tiles in registers
//         forward   V_I = -Linv_II sum_{K=J}^{I-1} L_IK V_K       (I > J, V_J = Linv_JJ)
//         backward  U_I =  Linv_II^T (V_I - sum_{K>I} L_KI^T U_K)  (I = NB-1 .. J)
//       fp32 MFMA; all waves step together and each step's block row / column of L is
//       staged once in LDS by the workgroup, fetched two steps ahead (double buffer);
//       the diagonal-block inverses Linv_II live in LDS. U_I = K^-1_IJ -> workspace.
//   gpk_grad_gram_kernel   one wave per (window, block row I), no atomics: for every J the
//       tile K^-1_JI (stored, or the transpose of the stored K^-1_IJ), the RBF tile
//       recomputed from xs (fp32-MFMA Gram), G, W and Wx_I += W_JI^T xs_J (MFMA), w1_I;
//       then dX of rows I and the block row's partials of ds2, dnoise, dl.
//   gpk_grad_fin_kernel    fixed-order sums of the partials -> dhyp (deterministic).
#include "gpk_common.h"
#include "gpk_internal.h"

#include <mutex>

// Timing experiments only (A/B builds of the solve kernel; results are wrong when set):
// bit 1 skips the phase-1 tile math, 2 the phase-2 tile math, 4 the L staging, 8 the
// K^-1 tile stores, 16 the alpha wave, 32 the phase-2 staging stores.
#ifndef GPK_GRAD_SKIP
#define GPK_GRAD_SKIP 0
#endif

namespace {

constexpr int kSW = 16;          // waves of the solve kernel (one block column each)
constexpr int kST = 64 * kSW;
constexpr int kMaxD = 64;

// ---- workspace layout (floats, per window) -------------------------------------------
struct GradWs {
  int NB, NT, kinv, alpha, mean, asum, part, per;
};
__host__ __device__ inline GradWs grad_ws(int N) {
  GradWs w;
  w.NB = (N + 15) / 16;
  w.NT = w.NB * (w.NB + 1) / 2;
  w.kinv = 0;                           // NT tiles x 256: lower tiles (I >= J), row-major
                                        // tile order, each in acc layout (lane-major float4)
  w.alpha = w.kinv + w.NT * 256;        // NP
  w.mean = w.alpha + 16 * w.NB;         // kMaxD: column means of x / l
  w.asum = w.mean + kMaxD;              // 4: sum(alpha)
  w.part = w.asum + 4;                  // NB x (2 + kMaxD): ds2, dnoise, dl[d] per block row
  w.per = w.part + w.NB * (2 + kMaxD);
  w.per = (w.per + 63) & ~63;
  return w;
}
GPK_DEVICE int tile_index(int I, int J) { return I * (I + 1) / 2 + J; }

GPK_DEVICE f32x4 mfma4(const f32x4 a, const f32x4 b, f32x4 d) {
  d = __builtin_amdgcn_mfma_f32_16x16x4f32(a[0], b[0], d, 0, 0, 0);
  d = __builtin_amdgcn_mfma_f32_16x16x4f32(a[1], b[1], d, 0, 0, 0);
  d = __builtin_amdgcn_mfma_f32_16x16x4f32(a[2], b[2], d, 0, 0, 0);
  d = __builtin_amdgcn_mfma_f32_16x16x4f32(a[3], b[3], d, 0, 0, 0);
  return d;
}

// Uniform value the compiler must treat as unknown at this point: keeps per-tile
// addresses from being hoisted out of their step (live addresses would spill).
GPK_DEVICE int opaque_s(int v) {
  asm volatile("" : "+s"(v));
  return v;
}

// Sum over the 16 lanes of each row (lanes sharing g), DPP only.
GPK_DEVICE float row16_sum(float v) {
#define GPK_DPP_ADD(ctrl) \
  v += __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), ctrl, 0xf, 0xf, false));
  GPK_DPP_ADD(0xB1) GPK_DPP_ADD(0x4E) GPK_DPP_ADD(0x141) GPK_DPP_ADD(0x140)
#undef GPK_DPP_ADD
  return v;
}

// ======================================================================================
// 1. solve: alpha, dy and the lower tiles of K^-1
// ======================================================================================
struct SolveLds {
  int dinv, stg, sv, alpha, red, total;
};
__host__ __device__ inline SolveLds solve_lds(int NB) {
  SolveLds o;
  const int TS = (NB > 1 ? NB - 1 : 1) * 256;
  const int stg = 2 * TS > NB * 256 ? 2 * TS : NB * 256;   // (prologue: diagonal blocks of L)
  o.dinv = 0;                     // NB x 16 x 16 row-major Linv_II
  o.stg = o.dinv + NB * 256;
  o.sv = o.stg + stg;             // NP
  o.alpha = o.sv + 16 * NB;       // NP
  o.red = o.alpha + 16 * NB;      // kST column-sum partials + 64
  o.total = o.red + kST + 64;
  return o;
}

template <int NB, bool FULL>
__global__ void __launch_bounds__(kST, 1) gpk_grad_solve_kernel(GpkExactGradArgs a) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  constexpr int NP = 16 * NB;
  constexpr int TS = (NB > 1 ? NB - 1 : 1) * 256;
  const SolveLds lay = solve_lds(NB);
  float* dinv = smem + lay.dinv;
  float* stg = smem + lay.stg;
  float* sv = smem + lay.sv;
  float* alpha = smem + lay.alpha;
  float* red = smem + lay.red;
  const int N = FULL ? NP : a.N;
  const int D = a.D;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int c = lane & 15, g = lane >> 4;
  const int b = blockIdx.x;
  const float* Lb = a.L + (size_t)b * N * N;
  const GradWs ws = grad_ws(N);
  float* wsb = a.ws + (size_t)b * ws.per;
  const float* hyp = a.hyp;
  const int n_ls = a.n_ls;

  // ---- prologue: diagonal blocks of L (staged in stg), z, column sums of x / l
  {
    const int bi = tid >> 6, m = (tid >> 2) & 15, kq = (tid & 3) * 4;   // one float4 per thread
    if (bi < NB) {
      const int row = 16 * bi + m, col0 = 16 * bi + kq;
      f32x4 v;
      if (FULL) {
        v = *(const f32x4*)&Lb[(size_t)row * N + col0];
      } else {
#pragma unroll
        for (int j = 0; j < 4; ++j) v[j] = (row < N && col0 + j < N) ? Lb[(size_t)row * N + col0 + j] : 0.f;
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        if (kq + j > m) v[j] = 0.f;
        if (kq + j == m && row >= N) v[j] = 1.f;   // identity padding
      }
      *(f32x4*)&stg[bi * 256 + m * 16 + kq] = v;
    }
  }
  for (int n = tid; n < NP; n += kST) sv[n] = n < N ? a.z[(size_t)b * N + n] : 0.f;
  {
    const int d = tid & 63, part = tid >> 6;
    float s = 0.f;
    if (d < D) {
      const float inv_l = 1.f / hyp[3 + (n_ls == 1 ? 0 : d)];
      for (int n = part; n < N; n += kST / 64) s += a.X[((size_t)b * N + n) * D + d] * inv_l;
    }
    red[tid] = s;
  }
  lds_barrier();
  {
    const int bi = tid >> 4, cc = tid & 15;
    if (bi < NB) {
      const float* Lt = stg + bi * 256;
      float x[16];
#pragma unroll
      for (int m = 0; m < 16; ++m) {
        float t = (m == cc) ? 1.f : 0.f;
#pragma unroll
        for (int k = 0; k < m; ++k) t = __builtin_fmaf(-Lt[m * 16 + k], x[k], t);
        x[m] = (m < cc) ? 0.f : t / Lt[m * 16 + m];
      }
#pragma unroll
      for (int m = 0; m < 16; ++m) dinv[bi * 256 + m * 16 + cc] = x[m];
    }
    if (tid < kMaxD) {
      float s = 0.f;
      for (int p = 0; p < kST / 64; ++p) s += red[p * 64 + tid];
      wsb[ws.mean + tid] = s / (float)N;
    }
  }
  lds_barrier();
  // ---- block columns of K^-1 (lower part): wave J owns column J; all waves step
  //      together through 2 NB steps with the step's L tiles staged in LDS
  const int J = wave;
  const bool live = J < NB;
  constexpr int AW = NB < kSW ? NB : kSW - 1;   // the wave that also solves alpha
  const float gw = a.gout[b];
  const float invN = 1.f / (float)N;
  float asum = 0.f;
  const f32x4 z4 = {0.f, 0.f, 0.f, 0.f};
  auto fetch_row = [&](const int I) -> f32x4 {    // tiles (I, K < I), row-major
    if (tid >= I * 64 || (GPK_GRAD_SKIP & 4)) return z4;
    const int K = tid >> 6, q = tid & 63, m = q >> 2, cg = (q & 3) * 4;
    const int row = 16 * I + m, col0 = 16 * K + cg;
    if (FULL) return *(const f32x4*)&Lb[(size_t)row * N + col0];
    f32x4 v;
#pragma unroll
    for (int j = 0; j < 4; ++j) v[j] = (row < N && col0 + j < N) ? Lb[(size_t)row * N + col0 + j] : 0.f;
    return v;
  };
  auto put_row = [&](float* buf, const int I, const f32x4 v) {
    if (tid >= I * 64) return;
    const int K = tid >> 6, q = tid & 63, m = q >> 2, cg = (q & 3) * 4;
    *(f32x4*)&buf[K * 256 + m * 16 + cg] = v;
  };
  auto fetch_col = [&](const int I) -> f32x4 {    // tiles (K > I, I), read by rows
    if (tid >= (NB - 1 - I) * 64 || (GPK_GRAD_SKIP & 4)) return z4;
    const int sl = tid >> 6, q = tid & 63, k = q >> 2, cg = (q & 3) * 4;
    const int row = 16 * (I + 1 + sl) + k, col0 = 16 * I + cg;
    if (FULL) return *(const f32x4*)&Lb[(size_t)row * N + col0];
    f32x4 v;
#pragma unroll
    for (int j = 0; j < 4; ++j) v[j] = (row < N && col0 + j < N) ? Lb[(size_t)row * N + col0 + j] : 0.f;
    return v;
  };
  auto put_col = [&](float* buf, const int I, const f32x4 v) {   // stored transposed
    if (tid >= (NB - 1 - I) * 64) return;
    const int sl = tid >> 6, q = tid & 63, k = q >> 2, cg = (q & 3) * 4;
#pragma unroll
    for (int j = 0; j < 4; ++j) buf[sl * 256 + (cg + j) * 16 + k] = v[j];
  };
  f32x4 X[NB];
  // Step s reads buffer s & 1: phase 1 step I (s = I) block row I, phase 2 step I
  // (s = 2NB-1-I) block column I. The tiles of step s+2 are fetched during step s and
  // written into buffer s & 1 after the step's barrier (everyone is done reading it).
  if (NB > 1) put_row(stg + TS, 1, fetch_row(1));
  lds_barrier();
#pragma unroll
  for (int I = 0; I < NB; ++I) {
    const f32x4 nxt = (I + 2 < NB) ? fetch_row(I + 2) : ((I + 2 == NB + 1 && NB >= 2) ? fetch_col(NB - 2) : z4);
    const float* buf = stg + (I & 1) * TS;
    const int I16 = opaque_s(16 * I);
    if (live && !(GPK_GRAD_SKIP & 1)) {
      if (I == J) {
#pragma unroll
        for (int r = 0; r < 4; ++r) X[I][r] = dinv[I16 * 16 + (4 * g + r) * 16 + c];
      } else if (I > J) {
        f32x4 s[4] = {z4, z4, z4, z4};   // 4 independent MFMA chains
#pragma unroll
        for (int K = 0; K < I; ++K) {
          if (K >= J) {
            const f32x4 la = *(const f32x4*)&buf[K * 256 + c * 16 + 4 * g];
            s[K & 3] = mfma4(la, X[K], s[K & 3]);
          }
        }
        const f32x4 di = *(const f32x4*)&dinv[I16 * 16 + c * 16 + 4 * g];
        X[I] = -mfma4(di, (s[0] + s[1]) + (s[2] + s[3]), z4);
      }
    }
    lds_barrier();
    if (I + 2 < NB) put_row(stg + (I & 1) * TS, I + 2, nxt);
    else if (I + 2 == NB + 1 && NB >= 2) put_col(stg + (I & 1) * TS, NB - 2, nxt);   // step 2NB-1-(NB-2)
  }
  lds_barrier();
#pragma unroll
  for (int I = NB - 1; I >= 0; --I) {
    const int st = 2 * NB - 1 - I;
    const f32x4 nxt = (I > 1) ? fetch_col(I - 2) : z4;
    const float* buf = stg + (st & 1) * TS;
    const int I16 = opaque_s(16 * I);
    if (live && I >= J && !(GPK_GRAD_SKIP & 2)) {
      f32x4 s[4] = {z4, z4, z4, z4};   // 4 independent MFMA chains
#pragma unroll
      for (int K = I + 1; K < NB; ++K) {
        const f32x4 la = *(const f32x4*)&buf[(K - I - 1) * 256 + c * 16 + 4 * g];
        s[K & 3] = mfma4(la, X[K], s[K & 3]);
      }
      const f32x4 t = X[I] - ((s[0] + s[1]) + (s[2] + s[3]));
      f32x4 dt;
#pragma unroll
      for (int r = 0; r < 4; ++r) dt[r] = dinv[I16 * 16 + (4 * g + r) * 16 + c];
      const f32x4 U = mfma4(dt, t, z4);
      X[I] = U;
      if (!(GPK_GRAD_SKIP & 8)) *(f32x4*)&wsb[ws.kinv + (size_t)tile_index(I, J) * 256 + lane * 4] = U;
    }
    // alpha = L^-T z by the same back substitution (right-hand side z in column 0 of the
    // tiles), run by wave AW: an idle wave when NB < 16, else wave 15 once its own
    // column (one tile, step NB-1) is done
    if (wave == AW && !(GPK_GRAD_SKIP & 18)) {
      if (I == NB - 1) {
#pragma unroll
        for (int K = 0; K < NB; ++K)
#pragma unroll
          for (int r = 0; r < 4; ++r) X[K][r] = c == 0 ? sv[16 * K + 4 * g + r] : 0.f;
      }
      f32x4 s[4] = {z4, z4, z4, z4};   // 4 independent MFMA chains
#pragma unroll
      for (int K = I + 1; K < NB; ++K) {
        const f32x4 la = *(const f32x4*)&buf[(K - I - 1) * 256 + c * 16 + 4 * g];
        s[K & 3] = mfma4(la, X[K], s[K & 3]);
      }
      const f32x4 t = X[I] - ((s[0] + s[1]) + (s[2] + s[3]));
      f32x4 dt;
#pragma unroll
      for (int r = 0; r < 4; ++r) dt[r] = dinv[I16 * 16 + (4 * g + r) * 16 + c];
      X[I] = mfma4(dt, t, z4);
      if (c == 0) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int n = 16 * I + 4 * g + r;
          const float an = X[I][r];
          wsb[ws.alpha + n] = an;
          if (FULL || n < N) {
            asum += an;
            if (a.dy != nullptr) a.dy[(size_t)b * N + n] = -gw * an * invN;
          }
        }
      }
    }
    lds_barrier();
    if (I > 1 && !(GPK_GRAD_SKIP & 32)) put_col(stg + (st & 1) * TS, I - 2, nxt);
  }
  if (wave == AW) {
    asum = wave_sum(asum);
    if (lane == 0) wsb[ws.asum] = asum;
  }
}

// ======================================================================================
// 2. contractions per (window, block row I): W, w1, Wx, dX and the partials.
//    One workgroup (16 waves) per window: xs = x / l - mean, ||xs||^2 and alpha are
//    staged in LDS once; wave I owns block row I and visits every block column J.
// ======================================================================================
constexpr int kGW = 16;

template <int DQ, bool FULL>
__global__ void __launch_bounds__(64 * kGW, DQ == 4 ? 4 : 8) gpk_grad_gram_kernel(GpkExactGradArgs a) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  constexpr int DP = 16 * DQ, XS = DP + 4;
  const int N = a.N, D = a.D;
  const GradWs ws = grad_ws(N);
  const int NB = ws.NB, NP = 16 * NB;
  const int tid = threadIdx.x, lane = tid & 63, I = tid >> 6;
  const int c = lane & 15, g = lane >> 4;
  const int b = blockIdx.x;
  const float* Xb = a.X + (size_t)b * N * D;
  const float* wsb = a.ws + (size_t)b * ws.per;
  const float* hyp = a.hyp;
  const bool ard = a.n_ls > 1;
  float* xs = smem;                  // NP x XS
  float* nrm = xs + NP * XS;         // NP
  float* al = nrm + NP;              // NP
  // loads of 4 iterations in flight (clamped unconditional addresses), then the stores
  for (int base = 0; base < NP * DP; base += 4 * 64 * kGW) {
    float v[4], l[4], mu[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int e = base + u * 64 * kGW + tid, n = e / DP, d = e - n * DP;
      const bool ok = e < NP * DP && (FULL || n < N) && d < D;
      v[u] = Xb[ok ? (size_t)n * D + d : 0];
      l[u] = hyp[3 + ((ok && ard) ? d : 0)];
      mu[u] = wsb[ws.mean + (ok ? d : 0)];
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int e = base + u * 64 * kGW + tid, n = e / DP, d = e - n * DP;
      if (e < NP * DP) xs[n * XS + d] = ((FULL || n < N) && d < D) ? v[u] / l[u] - mu[u] : 0.f;
    }
  }
  for (int n = tid; n < NP; n += 64 * kGW) al[n] = wsb[ws.alpha + n];
  lds_barrier();
  for (int n = tid; n < NP; n += 64 * kGW) {
    float t = 0.f;
#pragma unroll
    for (int d = 0; d < DP; ++d) t = __builtin_fmaf(xs[n * XS + d], xs[n * XS + d], t);
    nrm[n] = t;
  }
  lds_barrier();
  if (I >= NB) return;   // wave-uniform; no barriers below
  const float s2 = hyp[0];
  const float gw = a.gout[b];
  const float gs = gw / (2.f * (float)N);
  constexpr float nhalf_log2e = -0.72134752044448170f;

  // Gram B operand for the columns i = 16I + c: xs[i][16q + 4g .. +3]
  f32x4 bi[DQ];
#pragma unroll
  for (int q = 0; q < DQ; ++q) bi[q] = *(const f32x4*)&xs[(16 * I + c) * XS + 16 * q + 4 * g];
  const int col = 16 * I + c;
  const float ni = nrm[col], ai = al[col];
  f32x4 wx[DQ];
#pragma unroll
  for (int q = 0; q < DQ; ++q) wx[q] = f32x4{0.f, 0.f, 0.f, 0.f};
  float w1p = 0.f, ds2 = 0.f, dnz = 0.f;
  // K^-1_JI in acc layout (rows j, cols i): stored when J >= I, else the transpose of K^-1_IJ
  auto load_T = [&](int J) -> f32x4 {
    f32x4 T;
    if (J >= I) {
      T = *(const f32x4*)&wsb[ws.kinv + (size_t)tile_index(J, I) * 256 + lane * 4];
    } else {
      const float* t = wsb + ws.kinv + (size_t)tile_index(I, J) * 256;
#pragma unroll
      for (int r = 0; r < 4; ++r) T[r] = t[((c >> 2) * 16 + 4 * g + r) * 4 + (c & 3)];
    }
    return T;
  };
  f32x4 Tn = load_T(0);
  for (int J = 0; J < NB; ++J) {
    const f32x4 T = Tn;
    if (J + 1 < NB) Tn = load_T(J + 1);      // one tile ahead: the L2 latency overlaps this one
    const int j0 = 16 * J;
    f32x4 gr = {0.f, 0.f, 0.f, 0.f}, pj[DQ];
#pragma unroll
    for (int q = 0; q < DQ; ++q) {
      gr = mfma4(*(const f32x4*)&xs[(j0 + c) * XS + 16 * q + 4 * g], bi[q], gr);
#pragma unroll
      for (int r = 0; r < 4; ++r) pj[q][r] = xs[(j0 + 4 * g + r) * XS + 16 * q + c];
    }
    const f32x4 aj = *(const f32x4*)&al[j0 + 4 * g];
    const f32x4 nj = *(const f32x4*)&nrm[j0 + 4 * g];
    f32x4 W;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int row = j0 + 4 * g + r;
      float G = (aj[r] * ai - T[r]) * gs;
      if (!FULL && (row >= N || col >= N)) G = 0.f;
      float d2 = __builtin_fmaxf(nj[r] + ni - 2.f * gr[r], 0.f);
      if (row == col) d2 = 0.f;
      const float E = __builtin_amdgcn_exp2f(d2 * nhalf_log2e);
      ds2 = __builtin_fmaf(G, E, ds2);
      if (row == col) dnz += G;
      W[r] = (row == col) ? 0.f : G * s2 * E;
    }
    w1p += (W[0] + W[1]) + (W[2] + W[3]);
    // Wx_I += W_JI^T xs_J  (rows i, dims)
#pragma unroll
    for (int q = 0; q < DQ; ++q) wx[q] = mfma4(W, pj[q], wx[q]);
  }
  // w1 of row 16I + c (column sums of the W_JI tiles)
  w1p += __shfl_xor(w1p, 16, 64);
  w1p += __shfl_xor(w1p, 32, 64);
  // rows of the Wx accumulator are 16I + 4g + r; their w1 lives in lane 4g + r
  float w1r[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) w1r[r] = __shfl(w1p, 4 * g + r, 64);
  float* part = a.ws + (size_t)b * ws.per + ws.part + I * (2 + kMaxD);
#pragma unroll
  for (int q = 0; q < DQ; ++q) {
    const int d = 16 * q + c;
    const float ilq = d < D ? 1.f / hyp[3 + (ard ? d : 0)] : 0.f;
    float lp = 0.f;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int row = 16 * I + 4 * g + r;
      const float x = xs[row * XS + d];
      const float e = x * w1r[r] - wx[q][r];   // = -dxs / 2
      if ((FULL || row < N) && d < D) {
        if (a.dX != nullptr) a.dX[((size_t)b * N + row) * D + d] = -2.f * e * ilq;
        lp = __builtin_fmaf(x, e, lp);
      }
    }
    lp += __shfl_xor(lp, 16, 64);
    lp += __shfl_xor(lp, 32, 64);
    if (g == 0) part[2 + d] = lp;          // (d >= D: 0)
  }
  ds2 = wave_sum(ds2);
  dnz = wave_sum(dnz);
  if (lane == 0) {
    part[0] = ds2;
    part[1] = dnz;
  }
}

// ======================================================================================
// 3. fixed-order sums of the block-row partials -> dhyp
// ======================================================================================
__global__ void __launch_bounds__(128) gpk_grad_fin_kernel(GpkExactGradArgs a, int DP) {
  const int N = a.N, D = a.D;
  const GradWs ws = grad_ws(N);
  const int b = blockIdx.x, t = threadIdx.x;
  const float* wsb = a.ws + (size_t)b * ws.per;
  const float* part = wsb + ws.part;
  float* o = a.dhyp + (size_t)b * (3 + a.n_ls);
  const float* hyp = a.hyp;
  // thread t < 64: dl_t (t < D); 64: ds2, 65: dnoise, 66: dc
  const int f = t < 64 ? (t < D ? 2 + t : -1) : (t == 64 ? 0 : (t == 65 ? 1 : -1));
  float s = 0.f;
  if (f >= 0)
    for (int I = 0; I < ws.NB; ++I) s += part[I * (2 + kMaxD) + f];
  if (t == 64) o[0] = s;
  if (t == 65) o[1] = s;
  if (t == 66) o[2] = a.gout[b] * wsb[ws.asum] / (float)N;
  if (t < 64) {
    if (a.n_ls == 1) {
      const float tot = wave_sum(s);   // fixed-order butterfly over the dims
      if (t == 0) o[3] = 2.f * tot / hyp[3];
    } else if (t < D) {
      o[3 + t] = 2.f * s / hyp[3 + t];
    }
  }
  (void)DP;
}

template <int NB>
int launch_solve(const GpkExactGradArgs& a, hipStream_t stream) {
  const size_t lds = (size_t)solve_lds(NB).total * sizeof(float);
  if (lds > 160 * 1024) return -7;
  static std::once_flag once;
  std::call_once(once, [&] {
    (void)hipFuncSetAttribute((const void*)gpk_grad_solve_kernel<NB, true>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    (void)hipFuncSetAttribute((const void*)gpk_grad_solve_kernel<NB, false>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    (void)hipGetLastError();
  });
  if (a.N == 16 * NB)
    hipLaunchKernelGGL((gpk_grad_solve_kernel<NB, true>), dim3(a.B), dim3(kST), lds, stream, a);
  else
    hipLaunchKernelGGL((gpk_grad_solve_kernel<NB, false>), dim3(a.B), dim3(kST), lds, stream, a);
  return (int)hipGetLastError();
}

template <int DQ>
int launch_gram(const GpkExactGradArgs& a, hipStream_t stream) {
  const int NB = (a.N + 15) / 16;
  const size_t lds = sizeof(float) * (size_t)(16 * NB) * (16 * DQ + 4 + 2);
  static std::once_flag once;
  std::call_once(once, [&] {
    (void)hipFuncSetAttribute((const void*)gpk_grad_gram_kernel<DQ, true>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    (void)hipFuncSetAttribute((const void*)gpk_grad_gram_kernel<DQ, false>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    (void)hipGetLastError();
  });
  if (a.N == 16 * NB)
    hipLaunchKernelGGL((gpk_grad_gram_kernel<DQ, true>), dim3(a.B), dim3(64 * kGW), lds, stream, a);
  else
    hipLaunchKernelGGL((gpk_grad_gram_kernel<DQ, false>), dim3(a.B), dim3(64 * kGW), lds, stream, a);
  return (int)hipGetLastError();
}

}  // namespace

size_t gpk_exact_grad_ws_floats(int B, int N) {
  return (size_t)B * grad_ws(N).per;
}

int gpk_launch_exact_grad(const GpkExactGradArgs& a, hipStream_t stream) {
  int rc;
  switch ((a.N + 15) / 16) {
#define GPK_CASE(nb) case nb: rc = launch_solve<nb>(a, stream); break;
    GPK_CASE(1) GPK_CASE(2) GPK_CASE(3) GPK_CASE(4) GPK_CASE(5) GPK_CASE(6)
    GPK_CASE(7) GPK_CASE(8) GPK_CASE(9) GPK_CASE(10) GPK_CASE(11) GPK_CASE(12)
    GPK_CASE(13) GPK_CASE(14) GPK_CASE(15) GPK_CASE(16)
#undef GPK_CASE
    default: return -7;
  }
  if (rc != 0) return rc;
  rc = a.D <= 16 ? launch_gram<1>(a, stream) : (a.D <= 32 ? launch_gram<2>(a, stream) : launch_gram<4>(a, stream));
  if (rc != 0) return rc;
  hipLaunchKernelGGL(gpk_grad_fin_kernel, dim3(a.B), dim3(128), 0, stream, a, 0);
  return (int)hipGetLastError();
}
