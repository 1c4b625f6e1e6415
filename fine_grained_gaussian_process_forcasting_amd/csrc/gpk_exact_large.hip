// Exact-GP path for 256 < N <= 800 on gfx950: forward MLL, analytic backward and eval
// posterior. GPyTorch keeps the exact MLL on Cholesky up to settings.max_cholesky_size = 800
// (linear_operator inv_quad_logdet; above it CG / Lanczos, a different algorithm), and the
// reference's ExactGPModel (denoising_model/GPModel.py:4-13) takes whatever N its caller
// hands it. The N <= 256 kernels keep a window's whole factor in LDS + registers; at
// N = 800 the lower triangle alone is 1.28 MB, so here a window's matrix lives in HBM (the
// caller's L buffer, L2 / MALL resident while its workgroup runs) and the kernels are blocked:
//
//   gpk_lg_exact_kernel  (one workgroup of 16 waves per window) -- K_hat = s2 RBF + noise I
//     built straight into L by an f32-MFMA Gram of the centred inputs (GPyTorch _sq_dist
//     form), then a right-looking blocked Cholesky with 32-wide panels: the diagonal block
//     factored by one wave with a row per lane (v_readlane broadcasts, no LDS round trips),
//     its inverse formed column per lane from an LDS copy, the panel below by TRSM-as-GEMM
//     (A L_kk^-T, one wave per 16-row tile) into an LDS-resident panel, the trailing update
//     A_IJ -= L_Ik L_Jk^T on f32 MFMA in 32x32 units from that panel; z = L^-1 (y - c) and
//     log|L| ride along per panel. The psd_safe_cholesky
//     ladder (jitter * 10^t, failing windows only, cumulative fp32 diagonal adds) restarts the
//     window in-kernel: one launch, no host sync.
//   gpk_lg_grad_kernel   (one workgroup per window) -- X = L^-1 by blocked forward
//     substitution (diagonal-block inverses, then block rows X_i = -X_ii sum_p L_ip X_p),
//     K_hat^-1 = X^T X on MFMA, alpha = X^T z, then per block row of G = g(alpha alpha^T -
//     K_hat^-1)/(2N): W = G o K (K recomputed), w1 = W 1, Wx = W xs on MFMA, and the same
//     dX / dy / dhyp formulas as the N <= 256 backward (gpk_exact_grad.hip), partial sums
//     reduced in a fixed order (deterministic).
//   gpk_lg_post_kernel   (one workgroup per (window, 16 test points)) -- V = L^-1 K* by
//     blocked forward substitution with V in LDS (two waves form R = K*_k - L_k,<k V, a third
//     forms L_kk^-1 meanwhile, V_k = L_kk^-1 R on MFMA), mean = c + V^T z, var = s2 - colsum(V o V).
//
// Tile conventions: gpk_common.h ("acc layout"). Operands of a K = 32 product are fed with
// the k order k = 8q + s (lane l: q = l >> 4 picks the MFMA k slot, s the instruction), so a
// lane's 8 operand values are 8 consecutive floats of one row.
#include "gpk_common.h"
#include "gpk_internal.h"

#include <math.h>
#include <mutex>

namespace {

#ifndef GPK_LG_WAVES
#define GPK_LG_WAVES 16
#endif
// Timing-only knockouts of the forward's phases (bit 1 trailing update, 2 panel TRSM, 4 the
// diagonal block's factor / inverse / z, 8 the K_hat build); failures are ignored. Never set
// in a product build.
#ifndef GPK_LG_KO
#define GPK_LG_KO 0
#endif
// Software-pipelined trailing update (the next unit's loads before this unit's MFMAs):
// measured slower (16 waves: 110 VGPRs of spills, N = 800: 1.755 / 4.435 ms at B = 64 / 512
// vs 1.673 / 4.209 ms without; 8 waves: 1.783 / 4.144), so off.
// Timing-only knockouts of the backward (bit 1 block-row substitution of L^-1, 2 X^T X,
// 4 the gram); never set in a product build.
#ifndef GPK_LG_GKO
#define GPK_LG_GKO 0
#endif
#ifndef GPK_LG_PIPE
#define GPK_LG_PIPE 0
#endif
constexpr int kLgWaves = GPK_LG_WAVES;   // waves per window workgroup (forward, backward)
constexpr int kLgThreads = 64 * kLgWaves;
constexpr int kPostThreads = 192;   // posterior: 2 waves for R, 1 for L_kk^-1
constexpr int kPS = 36;          // LDS row stride of a 32-wide panel / block (floats; 16-B rows)
constexpr int kVS = 17;          // LDS row stride of 16-column scratch (V, T)
constexpr float kLog2PiL = 1.8378770664093453f;

__host__ __device__ inline int lg_np(int N) { return (N + 31) & ~31; }

GPK_DEVICE f32x4 mfma4(float a, float b, f32x4 d) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, d, 0, 0, 0);
}

// p -> (i, j), j <= i, in row-major order of a lower triangle (wave-uniform p).
GPK_DEVICE void tri_decode(int p, int& i, int& j) {
  int t = (int)((sqrtf(8.f * (float)p + 1.f) - 1.f) * 0.5f);
  while ((t + 1) * (t + 2) / 2 <= p) ++t;
  while (t * (t + 1) / 2 > p) --t;
  i = t;
  j = p - t * (t + 1) / 2;
}

// Cholesky of a 32x32 SPD block held one ROW per lane: lane c (of 0..31; lanes 32..63 mirror
// them and are never stored) has v[i] = A[c][i] for i <= c. Column j: the pivot A[j][j] is
// lane j's v[j]; every lane scales its own v[j] (= A[c][j], the column entry it owns) to
// L[c][j], then updates v[i] -= L[c][j] L[i][j] for i > j with L[i][j] broadcast from lane i
// by v_readlane (static register, static lane). Entries i > c are carried but never used.
// Returns the first failing column (0-based; pivot <= 0 or NaN) or -1; adds log L_jj to ld.
GPK_DEVICE int lg_chol32(float (&v)[32], int c, float& ld) {
  int fail = -1;
#pragma unroll
  for (int j = 0; j < 32; ++j) {
    const float p = readlane_f(v[j], j);
    if (fail < 0 && !(p > 0.f)) fail = j;
    const float ljj = sqrtf(p);
    ld += logf(ljj);
    const float rl = 1.f / ljj;
    v[j] = (c == j) ? ljj : v[j] * rl;
#pragma unroll
    for (int i = j + 1; i < 32; ++i) v[i] = fmaf(-readlane_f(v[j], i), v[j], v[i]);
  }
  return fail;
}

// Row c of the factor (lane c < 32) into a 32 x kPS LDS block, zeros above the diagonal.
GPK_DEVICE void lg_rows_to_lds(const float (&v)[32], int c, int lane, float* Lsh) {
  if (lane < 32) {
#pragma unroll
    for (int i = 0; i < 32; ++i) Lsh[c * kPS + i] = i <= c ? v[i] : 0.f;
  }
  wave_lds_sync();
}

// X = L^-1 of the 32x32 lower factor in LDS (Lsh, row-major, stride kPS): lane m forms column
// m by forward substitution, x[i] = X[i][m] (zero above the diagonal). The L entries are
// uniform-address LDS reads (broadcasts): as v_readlane broadcasts of a fixed register block
// the compiler hoists all 496 of them into SGPRs and spills.
GPK_DEVICE void lg_inv32(const float* Lsh, int m, float (&x)[32]) {
#pragma unroll
  for (int i = 0; i < 32; ++i) {
    float s = (i == m) ? 1.f : 0.f;
#pragma unroll
    for (int p = 0; p < i; ++p) s = fmaf(-Lsh[i * kPS + p], x[p], s);
    x[i] = s / Lsh[i * kPS + i];
  }
}

// Row c of the 32x32 diagonal block at (r0, r0) of a row-major matrix with leading dimension
// ld (elements i <= c); rows at or beyond N are identity rows (the padding of the last block:
// L stays block-diagonal with an identity tail, log 1 = 0, z = 0 there).
GPK_DEVICE void lg_load_diag_row(const float* __restrict__ A, int ld, int r0, int c, int N,
                                 float (&v)[32]) {
  const int row = r0 + c;
#pragma unroll
  for (int i = 0; i < 32; ++i) {
    float e = (i == c) ? 1.f : 0.f;
    if (row < N && i <= c) e = A[(size_t)row * ld + r0 + i];
    v[i] = e;
  }
}

// Centring mean of x / l over the N training rows (GPyTorch _sq_dist: adj = x1.mean(-2)),
// 1 / l, and the squared norms of the centred rows: mu[D], ils[D], nrm[Np] in LDS (rows >= N
// get 0). The column sums are split over every thread of the workgroup (row groups of a
// dimension, 8 loads in flight each), then summed over the groups in a fixed order; `part`
// is nthreads floats of LDS scratch. Inputs are scaled by 1 / l like the N <= 256 kernels.
GPK_DEVICE void lg_centre(const float* __restrict__ X, const float* __restrict__ hyp, int n_ls,
                          int N, int Np, int D, float* mu, float* ils, float* nrm, float* part,
                          int tid, int nthreads) {
  const int ngrp = nthreads / D;            // D <= 64 <= nthreads
  if (tid < ngrp * D) {
    const int d = tid % D, grp = tid / D;
    const float il = 1.f / hyp[3 + (n_ls == 1 ? 0 : d)];
    float s = 0.f;
#pragma unroll 8
    for (int i = grp; i < N; i += ngrp) s += X[(size_t)i * D + d] * il;
    part[tid] = s;
    if (grp == 0) ils[d] = il;
  }
  __syncthreads();
  if (tid < D) {
    float s = 0.f;
    for (int grp = 0; grp < ngrp; ++grp) s += part[grp * D + tid];
    mu[tid] = s / (float)N;
  }
  __syncthreads();
  for (int i = tid; i < Np; i += nthreads) {
    float s = 0.f;
    if (i < N)
#pragma unroll 8
      for (int d = 0; d < D; ++d) {
        const float a = X[(size_t)i * D + d] * ils[d] - mu[d];
        s = fmaf(a, a, s);
      }
    nrm[i] = s;
  }
  __syncthreads();
}

// Centred, scaled input (x / l - mu)[row][d]; 0 outside the matrix.
GPK_DEVICE float lg_xs(const float* __restrict__ X, const float* mu, const float* ils, int row,
                       int d, int N, int D) {
  return (row < N && d < D) ? X[(size_t)row * D + d] * ils[d] - mu[d] : 0.f;
}

// clamp_min(0) of a squared distance, NaN-propagating like torch (fmaxf would drop a NaN).
GPK_DEVICE float lg_clamp0(float d) { return d < 0.f ? 0.f : d; }

// Dot products a_i . a_j of a 16x16 tile (rows of X1 from r0, rows of X2 from c0) in acc
// layout, on f32 MFMA (k = d = 4t + q).
GPK_DEVICE f32x4 lg_gram_tile(const float* __restrict__ X1, int N1, int r0,
                              const float* __restrict__ X2, int N2, int c0, const float* mu,
                              const float* ils, int D, int lane) {
  const int i = lane & 15, q = lane >> 4;
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  for (int t = 0; 4 * t < D; ++t) {
    const int d = 4 * t + q;
    acc = mfma4(lg_xs(X1, mu, ils, r0 + i, d, N1, D), lg_xs(X2, mu, ils, c0 + i, d, N2, D), acc);
  }
  return acc;
}

// The same tile from centred inputs staged in LDS (row stride 33 floats, D <= 32).
GPK_DEVICE f32x4 lg_gram_tile_lds(const float* xsl, int r0, int c0, int D, int lane) {
  const int i = lane & 15, q = lane >> 4;
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int t = 0; t < 8; ++t)
    if (4 * t < D) acc = mfma4(xsl[(r0 + i) * 33 + 4 * t + q], xsl[(c0 + i) * 33 + 4 * t + q], acc);
  return acc;
}

// =========================================================================================
// Forward: K_hat -> L (in the caller's buffer), z, mll, info.
// =========================================================================================
struct LgFwdLds {
  int panel, linv, lkk, rv, zb, nrm, mu, ils, misc, total;
};
__host__ __device__ inline LgFwdLds lg_fwd_layout(int Np) {
  LgFwdLds o{};
  o.panel = 0;                      // Np x kPS: L[:, 32k : 32k + 32] of the current panel
  o.linv = o.panel + Np * kPS;      // 32 x kPS: L_kk^-1
  o.lkk = o.linv + 32 * kPS;        // 32 x kPS: L_kk
  o.rv = o.lkk + 32 * kPS;          // Np: y - c, reduced panel by panel
  o.zb = o.rv + Np;                 // Np: z = L^-1 (y - c)
  o.nrm = o.zb + Np;                // Np: squared norms of the centred rows
  o.mu = o.nrm + Np;                // 64
  o.ils = o.mu + 64;                 // 64
  o.misc = o.ils + 64;               // 8 ints: [0] failing column (1-based) of this attempt
  o.total = o.misc + 8;
  return o;
}

__global__ void __launch_bounds__(kLgThreads, 1) gpk_lg_exact_kernel(GpkExactArgs a) {
  extern __shared__ float smem[];
  const int b = blockIdx.x, tid = threadIdx.x, lane = tid & 63;
  const int wave = wave_id_uniform();
  const int N = a.N, D = a.D, Np = lg_np(N), nb = Np / 32, nsub = Np / 16;
  const LgFwdLds lay = lg_fwd_layout(Np);
  float* panel = smem + lay.panel;
  float* linv = smem + lay.linv;
  float* lkk = smem + lay.lkk;
  float* rv = smem + lay.rv;
  float* zb = smem + lay.zb;
  float* nrm = smem + lay.nrm;
  float* mu = smem + lay.mu;
  float* ils = smem + lay.ils;   // 1 / lengthscale
  volatile int* misc = (volatile int*)(smem + lay.misc);
  const float* X = a.X + (size_t)b * N * D;
  const float* y = a.y + (size_t)b * N;
  float* Lg = a.L + (size_t)b * N * N;
  const float s2 = a.hyp[0], noise = a.hyp[1], cmean = a.hyp[2];
  const int g = lane >> 4, c = lane & 15, q = lane >> 4, il = lane & 15;

  lg_centre(X, a.hyp, a.n_ls, N, Np, D, mu, ils, nrm, panel, tid, kLgThreads);
  // the strict upper triangle of L is zero and never touched again
  for (int i = wave; i < N; i += kLgWaves)
    for (int j = i + 1 + lane; j < N; j += 64) Lg[(size_t)i * N + j] = 0.f;

  float diagval = s2 + noise;   // K_ii = s2 exp(0) (_sq_dist zeroes the diagonal) + noise
  double jit_prev = 0.0;
  int info_w = 0;
  float ld = 0.f;               // sum log L_jj (wave 0; uniform)
  for (int attempt = 0; attempt <= a.max_tries; ++attempt) {
    if (attempt > 0) {
      double p10 = 1.0;
      for (int t = 1; t < attempt; ++t) p10 *= 10.0;
      const double jn = a.jitter * p10;
      diagval = diagval + (float)(jn - jit_prev);   // psd_safe_cholesky: diag += jn - jprev
      jit_prev = jn;
    }
    __syncthreads();   // every wave has read the previous attempt's verdict
    if (tid == 0) misc[0] = 0;
    // ---- K_hat (lower 16x16 tiles, diagonal tiles whole) into L. For D <= 32 the centred
    //      inputs are staged in the panel's LDS (free until the first panel): the Gram's
    //      strided global loads were the build's whole cost.
    const bool xs_lds = D <= 32;
    if (xs_lds) {
      for (int e = tid; e < Np * 32; e += kLgThreads) {
        const int i = e >> 5, d = e & 31;
        panel[i * 33 + d] = lg_xs(X, mu, ils, i, d, N, D);
      }
      __syncthreads();
    }
    const int npair = nsub * (nsub + 1) / 2;
    for (int p = wave; p < npair && !(GPK_LG_KO & 8); p += kLgWaves) {
      int I, J;
      tri_decode(p, I, J);
      if (16 * I >= N) continue;
      const f32x4 dot = xs_lds ? lg_gram_tile_lds(panel, 16 * I, 16 * J, D, lane)
                               : lg_gram_tile(X, N, 16 * I, X, N, 16 * J, mu, ils, D, lane);
      const int col = 16 * J + c;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = 16 * I + 4 * g + r;
        if (row < N && col < N) {
          const float dd = lg_clamp0(fmaf(-2.f, dot[r], nrm[row]) + nrm[col]);
          Lg[(size_t)row * N + col] = row == col ? diagval : s2 * expf(dd * -0.5f);
        }
      }
    }
    for (int i = tid; i < Np; i += kLgThreads) rv[i] = i < N ? y[i] - cmean : 0.f;
    __syncthreads();

    int fail = 0;
    ld = 0.f;
    for (int k = 0; k < nb; ++k) {
      const int r0 = 32 * k;
      // ---- 1. diagonal block (wave 0): factor, write back, inverse, z_k
      if (wave == 0) {
        const int cr = lane & 31;
        float v[32];
        lg_load_diag_row(Lg, N, r0, cr, N, v);
        const int f = (GPK_LG_KO & 4) ? -1 : lg_chol32(v, cr, ld);
        if (f >= 0 && !GPK_LG_KO) {
          if (lane == 0) misc[0] = r0 + f + 1;
        } else {
          const int row = r0 + cr;
          if (lane < 32 && row < N) {
#pragma unroll
            for (int i = 0; i < 32; ++i)
              if (r0 + i < N) Lg[(size_t)row * N + r0 + i] = i <= cr ? v[i] : 0.f;
          }
          lg_rows_to_lds(v, cr, lane, lkk);
          float x[32];
          if (GPK_LG_KO & 4) {
#pragma unroll
            for (int i = 0; i < 32; ++i) x[i] = v[i];
          } else {
            lg_inv32(lkk, cr, x);
          }
          if (lane < 32) {
#pragma unroll
            for (int i = 0; i < 32; ++i) linv[i * kPS + cr] = x[i];
          }
          // z_k = L_kk^-1 r_k (forward substitution, LAPACK strsv order: divide by L_pp)
          float rr = rv[r0 + cr], zc = 0.f;
#pragma unroll
          for (int p = 0; p < 32; ++p) {
            const float zp = readlane_f(rr, p) / lkk[p * kPS + p];
            if (cr == p) zc = zp;
            if (cr > p) rr = fmaf(-lkk[cr * kPS + p], zp, rr);
          }
          if (lane < 32) zb[r0 + cr] = zc;
        }
      }
      __syncthreads();
      if (misc[0] != 0) { fail = misc[0]; break; }
      // ---- 2. panel below the block: L_Ik = A_Ik L_kk^-T, one 16-row tile per wave (both
      //      16-column halves: A_Ik is read in place and overwritten by L_Ik, so one wave
      //      must own the whole 32-wide row segment)
      const int s0 = 2 * (k + 1);
      for (int I = s0 + wave; I < nsub && !(GPK_LG_KO & 2); I += kLgWaves) {
        if (16 * I >= N) break;
        const int row = 16 * I + il;
        const float* arow = Lg + (size_t)row * N + r0 + 8 * q;
        float av[8];
#pragma unroll
        for (int s = 0; s < 8; ++s) av[s] = row < N ? arow[s] : 0.f;
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const float* brow = linv + (16 * h + il) * kPS + 8 * q;
          f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
          for (int s = 0; s < 8; ++s) acc = mfma4(av[s], brow[s], acc);
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int rr = 16 * I + 4 * g + r;
            panel[rr * kPS + 16 * h + c] = acc[r];
            if (rr < N) Lg[(size_t)rr * N + r0 + 16 * h + c] = acc[r];
          }
        }
      }
      __syncthreads();
      // ---- 3. r_i -= L_ik z_k below the block; trailing update A_IJ -= L_Ik L_Jk^T
      for (int i = r0 + 32 + tid; i < Np; i += kLgThreads) {
        float s = 0.f;
#pragma unroll
        for (int m = 0; m < 32; ++m) s = fmaf(panel[i * kPS + m], zb[r0 + m], s);
        rv[i] -= s;
      }
      // 32x32 units (four 16x16 tiles: 16 loads in flight per lane, the panel operands read
      // once per unit; a diagonal unit skips its upper tile), software-pipelined: the next
      // unit's loads are issued before this unit's MFMAs. Units never overlap, and every
      // unit's first row block is real (32 (nb - 1) < N).
      const int mb = nb - (k + 1), nbp = mb * (mb + 1) / 2;
      auto unit_of = [&](int p, int& I0, int& J0, bool& dg) {
        int bi, bj;
        tri_decode(p, bi, bj);
        I0 = s0 + 2 * bi;
        J0 = s0 + 2 * bj;
        dg = bi == bj;
      };
      auto load_unit = [&](int I0, int J0, f32x4 (&acc)[2][2]) {
#pragma unroll
        for (int ti = 0; ti < 2; ++ti)
#pragma unroll
          for (int tj = 0; tj < 2; ++tj) {
            const int col = 16 * (J0 + tj) + c;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const int row = 16 * (I0 + ti) + 4 * g + r;
              acc[ti][tj][r] = (row < N && col < N) ? Lg[(size_t)row * N + col] : 0.f;
            }
          }
      };
      int p = wave, I0 = 0, J0 = 0;
      bool dg = false;
      f32x4 cur[2][2];
      if (p < nbp && !(GPK_LG_KO & 1)) {
        unit_of(p, I0, J0, dg);
        load_unit(I0, J0, cur);
      }
      for (; p < nbp && !(GPK_LG_KO & 1); p += kLgWaves) {
        const int pn = p + kLgWaves;
        int nI0 = 0, nJ0 = 0;
        bool ndg = false;
        f32x4 nxt[2][2];
        if (GPK_LG_PIPE && pn < nbp) {
          unit_of(pn, nI0, nJ0, ndg);
          load_unit(nI0, nJ0, nxt);
        }
        f32x4 ao[2][2], bo[2][2];
#pragma unroll
        for (int t = 0; t < 2; ++t) {
          ao[t][0] = *(const f32x4*)&panel[(16 * (I0 + t) + il) * kPS + 8 * q];
          ao[t][1] = *(const f32x4*)&panel[(16 * (I0 + t) + il) * kPS + 8 * q + 4];
          bo[t][0] = *(const f32x4*)&panel[(16 * (J0 + t) + il) * kPS + 8 * q];
          bo[t][1] = *(const f32x4*)&panel[(16 * (J0 + t) + il) * kPS + 8 * q + 4];
        }
#pragma unroll
        for (int ti = 0; ti < 2; ++ti)
#pragma unroll
          for (int tj = 0; tj < 2; ++tj) {
#pragma unroll
            for (int s = 0; s < 4; ++s) cur[ti][tj] = mfma4(-ao[ti][0][s], bo[tj][0][s], cur[ti][tj]);
#pragma unroll
            for (int s = 0; s < 4; ++s) cur[ti][tj] = mfma4(-ao[ti][1][s], bo[tj][1][s], cur[ti][tj]);
          }
#pragma unroll
        for (int ti = 0; ti < 2; ++ti)
#pragma unroll
          for (int tj = 0; tj < 2; ++tj) {
            if (dg && ti == 0 && tj == 1) continue;   // above the diagonal
            const int col = 16 * (J0 + tj) + c;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const int row = 16 * (I0 + ti) + 4 * g + r;
              if (row < N && col < N) Lg[(size_t)row * N + col] = cur[ti][tj][r];
            }
          }
        if (GPK_LG_PIPE) {
#pragma unroll
          for (int ti = 0; ti < 2; ++ti)
#pragma unroll
            for (int tj = 0; tj < 2; ++tj) cur[ti][tj] = nxt[ti][tj];
          I0 = nI0;
          J0 = nJ0;
          dg = ndg;
        } else if (pn < nbp) {
          unit_of(pn, I0, J0, dg);
          load_unit(I0, J0, cur);
        }
      }
      __syncthreads();
    }
    if (fail == 0) { info_w = attempt > 0 ? -attempt : 0; break; }
    info_w = fail;
  }
  // ---- MLL = -0.5 (|z|^2 + 2 sum log L_jj + N log 2 pi) / N
  if (wave == 0) {
    float s = 0.f;
    for (int i = lane; i < N; i += 64) s = fmaf(zb[i], zb[i], s);
    s = wave_sum(s);
    if (lane == 0) {
      a.info[b] = info_w;
      a.mll[b] = info_w > 0 ? __builtin_nanf("")
                            : -0.5f * (s + 2.f * ld + (float)N * kLog2PiL) / (float)N;
    }
  }
  if (a.z != nullptr)
    for (int i = tid; i < N; i += kLgThreads) a.z[(size_t)b * N + i] = zb[i];
}

// =========================================================================================
// Backward: X = L^-1, K_hat^-1 = X^T X (workspace), then the gram contractions.
// =========================================================================================
struct LgGradLds {
  int alpha, zb, nrm, mu, ils, scr, red, lrow, total;
};
constexpr int kRedStride = 2 + 64;
__host__ __device__ inline LgGradLds lg_grad_layout(int Np) {
  LgGradLds o{};
  o.alpha = 0;                          // Np: alpha = K_hat^-1 (y - c) = X^T z
  o.zb = o.alpha + Np;                  // Np
  o.nrm = o.zb + Np;                    // Np
  o.mu = o.nrm + Np;                    // 64
  o.ils = o.mu + 64;                     // 64
  o.scr = o.ils + 64;                    // waves x 32 x kVS: the T block of a row step
  o.red = o.scr + kLgWaves * 32 * kVS;  // waves x kRedStride fp64 partial sums (2 floats each)
  o.lrow = o.red + 2 * kLgWaves * kRedStride;   // 32 x (Np + 4): the row step's block row of L
                                                // (phase 1: the waves' L_kk, 32 x kPS each)
  const int lrow_n = 32 * (Np + 4), lkk_n = kLgWaves * 32 * kPS;
  o.total = o.lrow + (lrow_n > lkk_n ? lrow_n : lkk_n);
  return o;
}

__global__ void __launch_bounds__(kLgThreads, 1) gpk_lg_grad_kernel(GpkExactGradArgs a) {
  extern __shared__ float smem[];
  const int b = blockIdx.x, tid = threadIdx.x, lane = tid & 63;
  const int wave = wave_id_uniform();
  const int N = a.N, D = a.D, Np = lg_np(N), nb = Np / 32, nsub = Np / 16;
  const LgGradLds lay = lg_grad_layout(Np);
  float* alpha = smem + lay.alpha;
  float* zb = smem + lay.zb;
  float* nrm = smem + lay.nrm;
  float* mu = smem + lay.mu;
  float* ils = smem + lay.ils;   // 1 / lengthscale
  float* scr = smem + lay.scr + wave * (32 * kVS);
  float* lrow = smem + lay.lrow;
  const int LS = Np + 4;
  double* red = (double*)(smem + lay.red);
  const float* X = a.X + (size_t)b * N * D;
  const float* Lg = a.L + (size_t)b * N * N;
  float* Xw = a.ws + (size_t)b * 2 * Np * Np;   // L^-1 (lower 16x16 tiles; row stride Np)
  float* Kw = Xw + (size_t)Np * Np;             // K_hat^-1 (lower 16x16 tiles)
  const int g = lane >> 4, c = lane & 15, q = lane >> 4, il = lane & 15;

  lg_centre(X, a.hyp, a.n_ls, N, Np, D, mu, ils, nrm, smem + lay.scr, tid, kLgThreads);
  for (int i = tid; i < Np; i += kLgThreads) zb[i] = i < N ? a.z[(size_t)b * N + i] : 0.f;
  // ---- 1. diagonal-block inverses X_kk = L_kk^-1
  for (int k = wave; k < nb; k += kLgWaves) {
    const int cr = lane & 31;
    float x[32];
    {
      float v[32];
      lg_load_diag_row(Lg, N, 32 * k, cr, N, v);
      lg_rows_to_lds(v, cr, lane, lrow + wave * (32 * kPS));
    }
    lg_inv32(lrow + wave * (32 * kPS), cr, x);
    if (lane < 32) {
#pragma unroll
      for (int i = 0; i < 32; ++i) Xw[(size_t)(32 * k + i) * Np + 32 * k + cr] = x[i];
    }
  }
  __syncthreads();
  // ---- 2. block rows: X_iJ = -X_ii sum_{p = J/2}^{i-1} L_ip X_pJ (16-column tiles J). The
  //      step's block row L[32i .. 32i+31][0 .. 32i) is staged in LDS once (coalesced) and read
  //      as the A operand by every tile J (a lane's 8 values: two 16-byte reads); the X_pJ
  //      operands come from the workspace, two 32-row chunks in flight.
  for (int i = 1; i < nb && !(GPK_LG_GKO & 1); ++i) {
    for (int e = tid; e < 32 * 8 * i; e += kLgThreads) {   // float4 pieces of the block row
      const int r = e / (8 * i), c4 = e - r * (8 * i), row = 32 * i + r;
      f32x4 v = {0.f, 0.f, 0.f, 0.f};
      if (row < N) {
#pragma unroll
        for (int t = 0; t < 4; ++t) v[t] = Lg[(size_t)row * N + 4 * c4 + t];
      }
      *(f32x4*)&lrow[r * LS + 4 * c4] = v;
    }
    __syncthreads();
    for (int J = wave; J < 2 * i; J += kLgWaves) {
      f32x4 t0 = {0.f, 0.f, 0.f, 0.f}, t1 = {0.f, 0.f, 0.f, 0.f};
      auto chunk = [&](int p, const float (&bv)[8]) {
        const f32x4 a00 = *(const f32x4*)&lrow[il * LS + 32 * p + 8 * q];
        const f32x4 a01 = *(const f32x4*)&lrow[il * LS + 32 * p + 8 * q + 4];
        const f32x4 a10 = *(const f32x4*)&lrow[(16 + il) * LS + 32 * p + 8 * q];
        const f32x4 a11 = *(const f32x4*)&lrow[(16 + il) * LS + 32 * p + 8 * q + 4];
#pragma unroll
        for (int s = 0; s < 4; ++s) {
          t0 = mfma4(a00[s], bv[s], t0);
          t1 = mfma4(a10[s], bv[s], t1);
        }
#pragma unroll
        for (int s = 0; s < 4; ++s) {
          t0 = mfma4(a01[s], bv[4 + s], t0);
          t1 = mfma4(a11[s], bv[4 + s], t1);
        }
      };
      auto xload = [&](int p, float (&bv)[8]) {
#pragma unroll
        for (int s = 0; s < 8; ++s) bv[s] = Xw[(size_t)(32 * p + 8 * q + s) * Np + 16 * J + il];
      };
      int p = J >> 1;
      for (; p + 1 < i; p += 2) {
        float b0[8], b1[8];
        xload(p, b0);
        xload(p + 1, b1);
        chunk(p, b0);
        chunk(p + 1, b1);
      }
      if (p < i) {
        float b0[8];
        xload(p, b0);
        chunk(p, b0);
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        scr[(4 * g + r) * kVS + c] = t0[r];
        scr[(16 + 4 * g + r) * kVS + c] = t1[r];
      }
      wave_lds_sync();
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const float* xrow = Xw + (size_t)(32 * i + 16 * h + il) * Np + 32 * i + 8 * q;
        f32x4 yv = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int s = 0; s < 8; ++s) yv = mfma4(-xrow[s], scr[(8 * q + s) * kVS + il], yv);
#pragma unroll
        for (int r = 0; r < 4; ++r) Xw[(size_t)(32 * i + 16 * h + 4 * g + r) * Np + 16 * J + c] = yv[r];
      }
      wave_lds_sync();
    }
    __syncthreads();
  }
  // ---- 3. K_hat^-1 = X^T X (lower tiles, in 32x32 units: the four tiles share each 16-row
  //      step's X loads) and alpha = X^T z
  const int nbp = nb * (nb + 1) / 2;
  for (int p = wave; p < nbp && !(GPK_LG_GKO & 2); p += kLgWaves) {
    int bi, bj;
    tri_decode(p, bi, bj);
    const int I0 = 2 * bi, J0 = 2 * bj;
    if (16 * I0 >= N) continue;
    f32x4 acc[2][2];
#pragma unroll
    for (int ti = 0; ti < 2; ++ti)
#pragma unroll
      for (int tj = 0; tj < 2; ++tj) acc[ti][tj] = f32x4{0.f, 0.f, 0.f, 0.f};
    for (int pp = I0; pp < nsub && 16 * pp < N; ++pp) {
      f32x4 qv[2], pv[2];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const size_t row = (size_t)(16 * pp + 4 * g + r) * Np;
        qv[0][r] = Xw[row + 16 * I0 + c];
        qv[1][r] = Xw[row + 16 * I0 + 16 + c];
        pv[0][r] = Xw[row + 16 * J0 + c];
        pv[1][r] = Xw[row + 16 * J0 + 16 + c];
      }
#pragma unroll
      for (int ti = 0; ti < 2; ++ti)
#pragma unroll
        for (int tj = 0; tj < 2; ++tj) acc[ti][tj] = mma_tn(qv[ti], pv[tj], acc[ti][tj]);
    }
#pragma unroll
    for (int ti = 0; ti < 2; ++ti)
#pragma unroll
      for (int tj = 0; tj < 2; ++tj) {
        if (bi == bj && ti == 0 && tj == 1) continue;
#pragma unroll
        for (int r = 0; r < 4; ++r)
          Kw[(size_t)(16 * (I0 + ti) + 4 * g + r) * Np + 16 * (J0 + tj) + c] = acc[ti][tj][r];
      }
  }
  for (int j = tid; j < Np; j += kLgThreads) {
    float s = 0.f;
    for (int i = j; i < N; ++i) s = fmaf(Xw[(size_t)i * Np + j], zb[i], s);
    alpha[j] = j < N ? s : 0.f;
  }
  __syncthreads();
  // ---- 4. gram: per 16-point block I (one wave), tiles (rows J, cols I) of
  //      G = g (alpha alpha^T - K_hat^-1) / (2N), E = K / s2, W = G o K (zero diagonal)
  const float gout = a.gout[b];
  const float gsc = gout / (2.f * (float)N);
  const float s2 = a.hyp[0];
  const int nDQ = (D + 15) / 16;
  // the hyper-parameter sums cancel heavily (sum G o E of a well-fit model is ~1e-3 of its
  // terms): fp64 accumulators, fixed-order reduction
  double p_s2 = 0.0, p_tr = 0.0, p_dl[4] = {0.0, 0.0, 0.0, 0.0};
  for (int I = wave; I < nsub && 16 * I < N && !(GPK_LG_GKO & 4); I += kLgWaves) {
    float bI[16];
#pragma unroll
    for (int t = 0; t < 16; ++t) bI[t] = 4 * t < D ? lg_xs(X, mu, ils, 16 * I + il, 4 * t + q, N, D) : 0.f;
    f32x4 wx[4];
#pragma unroll
    for (int dc = 0; dc < 4; ++dc) wx[dc] = f32x4{0.f, 0.f, 0.f, 0.f};
    float w1p = 0.f;
    const int ci = 16 * I + c;
    for (int J = 0; J < nsub && 16 * J < N; ++J) {
      f32x4 dot = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int t = 0; t < 16; ++t)
        if (4 * t < D) dot = mfma4(lg_xs(X, mu, ils, 16 * J + il, 4 * t + q, N, D), bI[t], dot);
      f32x4 wt;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int rj = 16 * J + 4 * g + r;
        float w = 0.f;
        if (rj < N && ci < N) {
          const float kin = J >= I ? Kw[(size_t)rj * Np + ci] : Kw[(size_t)ci * Np + rj];
          float dd = lg_clamp0(fmaf(-2.f, dot[r], nrm[rj]) + nrm[ci]);
          if (rj == ci) dd = 0.f;
          const float e = expf(dd * -0.5f);
          const float gg = gsc * (alpha[rj] * alpha[ci] - kin);
          p_s2 += (double)(gg * e);
          if (rj == ci) p_tr += (double)gg;
          else w = gg * (s2 * e);
        }
        wt[r] = w;
        w1p += w;
      }
#pragma unroll
      for (int dc = 0; dc < 4; ++dc)
        if (dc < nDQ) {
          f32x4 xj;
#pragma unroll
          for (int r = 0; r < 4; ++r) xj[r] = lg_xs(X, mu, ils, 16 * J + 4 * g + r, 16 * dc + c, N, D);
          wx[dc] = mma_tn(wt, xj, wx[dc]);   // Wx[16I + 4g + r][16dc + c] += sum_j W_ij xs_j
        }
    }
    // w1 of point 16I + c (sum over the four lane groups), then per (point, dim)
    float w1c = w1p + __shfl_xor(w1p, 16, 64);
    w1c += __shfl_xor(w1c, 32, 64);
#pragma unroll
    for (int dc = 0; dc < 4; ++dc)
      if (dc < nDQ) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float w1r = __shfl(w1c, 4 * g + r, 64);
          const int pt = 16 * I + 4 * g + r, d = 16 * dc + c;
          if (pt < N && d < D) {
            const float xs = lg_xs(X, mu, ils, pt, d, N, D);
            const float t = fmaf(xs, w1r, -wx[dc][r]);   // xs w1 - Wx
            if (a.dX != nullptr) a.dX[((size_t)b * N + pt) * D + d] = -2.f * t * ils[d];
            p_dl[dc] += (double)(xs * t);
          }
        }
      }
  }
  p_s2 = wave_sum_d(p_s2);
  p_tr = wave_sum_d(p_tr);
#pragma unroll
  for (int dc = 0; dc < 4; ++dc) {
    p_dl[dc] += __shfl_xor(p_dl[dc], 16, 64);
    p_dl[dc] += __shfl_xor(p_dl[dc], 32, 64);
  }
  if (lane == 0) {
    red[wave * kRedStride + 0] = p_s2;
    red[wave * kRedStride + 1] = p_tr;
  }
  if (lane < 16) {
#pragma unroll
    for (int dc = 0; dc < 4; ++dc) red[wave * kRedStride + 2 + 16 * dc + lane] = p_dl[dc];
  }
  __syncthreads();
  if (a.dy != nullptr)
    for (int i = tid; i < N; i += kLgThreads) a.dy[(size_t)b * N + i] = -gout * alpha[i] / (float)N;
  const int nh = 3 + a.n_ls;
  if (tid < nh) {
    double v = 0.0;
    if (tid == 0 || tid == 1) {
      for (int w = 0; w < kLgWaves; ++w) v += red[w * kRedStride + tid];
    } else if (tid == 2) {
      for (int i = 0; i < N; ++i) v += (double)alpha[i];
      v = (double)gout * v / (double)N;
    } else if (a.n_ls == 1) {
      for (int d = 0; d < D; ++d)
        for (int w = 0; w < kLgWaves; ++w) v += red[w * kRedStride + 2 + d];
      v = 2.0 * v * (double)ils[0];
    } else {
      const int d = tid - 3;
      for (int w = 0; w < kLgWaves; ++w) v += red[w * kRedStride + 2 + d];
      v = 2.0 * v * (double)ils[d];
    }
    a.dhyp[(size_t)b * nh + tid] = (float)v;
  }
}

// =========================================================================================
// Posterior: V = L^-1 K* (16 test points per workgroup), mean and latent variance.
// =========================================================================================
struct LgPostLds {
  int V, lkk, linv, zb, nrm, mu, ils, tn, red, total;
};
__host__ __device__ inline LgPostLds lg_post_layout(int Np) {
  LgPostLds o{};
  o.V = 0;                    // Np x kVS
  o.lkk = o.V + Np * kVS;     // 32 x kPS: L_kk (identity-padded)
  o.linv = o.lkk + 32 * kPS;  // 32 x kPS: L_kk^-1
  o.zb = o.linv + 32 * kPS;   // Np
  o.nrm = o.zb + Np;          // Np
  o.mu = o.nrm + Np;          // 64
  o.ils = o.mu + 64;           // 64
  o.tn = o.ils + 64;           // 16: test-point norms
  o.red = o.tn + 16;           // 2 x 32: per-wave mean / variance partials
  o.total = o.red + 64;
  return o;
}

__global__ void __launch_bounds__(kPostThreads) gpk_lg_post_kernel(GpkPostArgs a) {
  extern __shared__ float smem[];
  const int b = blockIdx.y, t0 = 16 * blockIdx.x, tid = threadIdx.x, lane = tid & 63;
  const int wave = wave_id_uniform();
  const int N = a.N, Ns = a.Ns, D = a.D, Np = lg_np(N), nb = Np / 32;
  const LgPostLds lay = lg_post_layout(Np);
  float* V = smem + lay.V;
  float* lkk = smem + lay.lkk;
  float* linv = smem + lay.linv;
  float* zb = smem + lay.zb;
  float* nrm = smem + lay.nrm;
  float* mu = smem + lay.mu;
  float* ils = smem + lay.ils;   // 1 / lengthscale
  float* tn = smem + lay.tn;
  float* red = smem + lay.red;
  const float* X = a.X + (size_t)b * N * D;
  const float* Xs = a.Xs + (size_t)b * Ns * D;
  const float* Lg = a.L + (size_t)b * N * N;
  const float s2 = a.hyp[0], cmean = a.hyp[2];
  const int g = lane >> 4, c = lane & 15, q = lane >> 4, il = lane & 15;

  lg_centre(X, a.hyp, a.n_ls, N, Np, D, mu, ils, nrm, V, tid, kPostThreads);
  if (tid < 16) {
    float s = 0.f;
    for (int d = 0; d < D; ++d) {
      const float v = lg_xs(Xs, mu, ils, t0 + tid, d, Ns, D);
      s = fmaf(v, v, s);
    }
    tn[tid] = s;
  }
  for (int i = tid; i < Np; i += kPostThreads) zb[i] = i < N ? a.z[(size_t)b * N + i] : 0.f;
  float mp = 0.f, vp = 0.f;   // waves 0, 1: partials of column c over this wave's rows
  for (int k = 0; k < nb; ++k) {
    const int r0 = 32 * k;
    for (int e = tid; e < 32 * 32; e += kPostThreads) {
      const int i = e >> 5, m = e & 31, row = r0 + i;
      float v = m == i ? 1.f : 0.f;
      if (row < N) v = m <= i ? Lg[(size_t)row * N + r0 + m] : 0.f;
      lkk[i * kPS + m] = v;
    }
    __syncthreads();   // (also: tn / zb / the previous step's V rows)
    if (wave < 2) {
      // R = K*[rows r0 + 16 wave, cols t0..] - L[rows, :r0] V[:r0, :]  -> V rows (LDS)
      const int rows = r0 + 16 * wave;
      const f32x4 dot = lg_gram_tile(X, N, rows, Xs, Ns, t0, mu, ils, D, lane);
      f32x4 acc;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = rows + 4 * g + r, col = t0 + c;
        float v = 0.f;
        if (row < N && col < Ns) {
          const float dd = lg_clamp0(fmaf(-2.f, dot[r], nrm[row]) + tn[c]);
          v = s2 * expf(dd * -0.5f);
        }
        acc[r] = v;
      }
      // k order kk = 16p + 4q + t: a lane's four A values are consecutive floats of its L
      // row (one 16-byte load when the rows are 16-byte aligned), two chunks in flight
      const int ra = rows + il;
      const float* lrow = Lg + (size_t)ra * N;
      const bool vec = (N & 3) == 0;
      auto lrow4 = [&](int p) -> f32x4 {
        const int k0 = 16 * p + 4 * q;
        if (ra >= N) return f32x4{0.f, 0.f, 0.f, 0.f};
        if (vec) return *(const f32x4*)&lrow[k0];
        return f32x4{lrow[k0], lrow[k0 + 1], lrow[k0 + 2], lrow[k0 + 3]};
      };
      int p = 0;
      for (; p + 1 < 2 * k; p += 2) {
        const f32x4 l0 = lrow4(p), l1 = lrow4(p + 1);
#pragma unroll
        for (int t = 0; t < 4; ++t) acc = mfma4(-l0[t], V[(16 * p + 4 * q + t) * kVS + il], acc);
#pragma unroll
        for (int t = 0; t < 4; ++t) acc = mfma4(-l1[t], V[(16 * p + 16 + 4 * q + t) * kVS + il], acc);
      }
      if (p < 2 * k) {
        const f32x4 l0 = lrow4(p);
#pragma unroll
        for (int t = 0; t < 4; ++t) acc = mfma4(-l0[t], V[(16 * p + 4 * q + t) * kVS + il], acc);
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) V[(rows + 4 * g + r) * kVS + c] = acc[r];
    } else {
      // wave 2, meanwhile: L_kk^-1 (column per lane) for the MFMA solve below
      const int cr = lane & 31;
      float x[32];
      lg_inv32(lkk, cr, x);
      if (lane < 32) {
#pragma unroll
        for (int i = 0; i < 32; ++i) linv[i * kPS + cr] = x[i];
      }
    }
    __syncthreads();
    // V_k = L_kk^-1 R: rows 16 wave of the block, K = 32 (A: L_kk^-1 rows, B: R columns)
    f32x4 yv = {0.f, 0.f, 0.f, 0.f};
    if (wave < 2) {
#pragma unroll
      for (int s = 0; s < 8; ++s)
        yv = mfma4(linv[(16 * wave + il) * kPS + 8 * q + s], V[(r0 + 8 * q + s) * kVS + il], yv);
    }
    __syncthreads();   // every wave is done reading R before V_k overwrites it
    if (wave < 2) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = r0 + 16 * wave + 4 * g + r;
        V[row * kVS + c] = yv[r];
        mp = fmaf(yv[r], zb[row], mp);
        vp = fmaf(yv[r], yv[r], vp);
      }
    }
  }
  // per-column totals: the four lane groups of each wave, then the two waves, in order
  mp += __shfl_xor(mp, 16, 64);
  mp += __shfl_xor(mp, 32, 64);
  vp += __shfl_xor(vp, 16, 64);
  vp += __shfl_xor(vp, 32, 64);
  if (wave < 2 && lane < 16) {
    red[wave * 32 + lane] = mp;
    red[wave * 32 + 16 + lane] = vp;
  }
  __syncthreads();
  if (tid < 16 && t0 + tid < Ns) {
    a.mean[(size_t)b * Ns + t0 + tid] = cmean + (red[tid] + red[32 + tid]);
    a.var[(size_t)b * Ns + t0 + tid] = s2 - (red[16 + tid] + red[48 + tid]);
  }
}

}  // namespace

size_t gpk_exact_large_grad_ws_floats(int B, int N) {
  const size_t np = (size_t)lg_np(N);
  return (size_t)B * 2 * np * np;
}

int gpk_launch_exact_large(const GpkExactArgs& a, hipStream_t stream) {
  if (a.L == nullptr) return -10;   // N > 256: L is the factor's storage
  if (a.D > 64) return -7;
  const size_t lds = (size_t)lg_fwd_layout(lg_np(a.N)).total * sizeof(float);
  static std::once_flag once;
  std::call_once(once, [] {
    (void)hipFuncSetAttribute((const void*)gpk_lg_exact_kernel,
                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    (void)hipGetLastError();
  });
  hipLaunchKernelGGL(gpk_lg_exact_kernel, dim3(a.B), dim3(kLgThreads), lds, stream, a);
  return (int)hipGetLastError();
}

int gpk_launch_exact_large_grad(const GpkExactGradArgs& a, hipStream_t stream) {
  const size_t lds = (size_t)lg_grad_layout(lg_np(a.N)).total * sizeof(float);
  static std::once_flag once;
  std::call_once(once, [] {
    (void)hipFuncSetAttribute((const void*)gpk_lg_grad_kernel,
                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    (void)hipGetLastError();
  });
  hipLaunchKernelGGL(gpk_lg_grad_kernel, dim3(a.B), dim3(kLgThreads), lds, stream, a);
  return (int)hipGetLastError();
}

int gpk_launch_exact_large_posterior(const GpkPostArgs& a, hipStream_t stream) {
  const size_t lds = (size_t)lg_post_layout(lg_np(a.N)).total * sizeof(float);
  static std::once_flag once;
  std::call_once(once, [] {
    (void)hipFuncSetAttribute((const void*)gpk_lg_post_kernel,
                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    (void)hipGetLastError();
  });
  hipLaunchKernelGGL(gpk_lg_post_kernel, dim3((a.Ns + 15) / 16, a.B), dim3(kPostThreads), lds,
                     stream, a);
  return (int)hipGetLastError();
}
