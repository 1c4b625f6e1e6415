// Exact-GP hot path for gfx950: per-window RBF Gram + jittered Cholesky +
// forward solve + marginal log likelihood, fused into ONE kernel launch.
//
// Replaces, per window b (reference semantics: oracle/gp_oracle.py::exact_mll):
//   K_hat = s2 * exp(-0.5 * ||(x_i - x_j)/l||^2) + sigma2 * I   (GPModel.py:7-13,
//           upstream kernels/rbf_kernel.py + likelihoods/gaussian_likelihood.py)
//   L     = psd_safe_cholesky(K_hat)                          (upstream linear_operator
//           utils/cholesky.py: jitter ladder 1e-6,1e-5,1e-4 applied per window)
//   mll   = -0.5 * (||L^{-1}(y-c)||^2 + 2 sum log L_ii + N log 2pi) / N
//           (upstream mlls/exact_marginal_log_likelihood.py, MVN.log_prob)
//
// Design: one workgroup of W waves per window. The padded
// K_hat (NB x NB tiles of 16x16, upper triangle, plus one right-hand-side
// block column holding y - c) lives in REGISTERS as MFMA accumulators (acc
// layout, see gpk_common.h); tile t is owned by wave t % W. The blocked
// right-looking Cholesky works on R = L^T:
//   A(k): owner of (k,k) factors its tile (readlane-broadcast column steps)
//         and publishes -R_kk^{-1} (acc layout) through LDS.
//   B(k): owners of (k,j) compute R_kj = R_kk^{-T} T_kj with 4 MFMAs and
//         publish R_kj through an LDS panel; the RHS block yields z.
//   C(k): every owner of (i,j), i > k, accumulates  R_ki^T R_kj  (4 MFMAs).
// The MFMA accumulators hold -T, so every update is a plain MFMA accumulate.
#include "gpk_common.h"
#include "gpk_internal.h"

namespace {

constexpr float kLog2Pi = 1.8378770664093453f;

// (i | j << 8) for upper tiles i <= j < 16 in column-major order t = j(j+1)/2 + i.
struct TileTable {
  int v[136];
  constexpr TileTable() : v() {
    int t = 0;
    for (int j = 0; j < 16; ++j)
      for (int i = 0; i <= j; ++i) v[t++] = i | (j << 8);
  }
};
__constant__ TileTable c_tile_tbl = TileTable();
#define c_tile_ij (c_tile_tbl.v)

struct ExactLds {
  // offsets in floats
  int xf, nrm, rv, panel, rinv, dsc, red, total;
};

__host__ __device__ inline ExactLds exact_lds_layout(int NB, int DC, int W) {
  ExactLds o;
  o.xf = 0;
  o.nrm = o.xf + NB * DC * 256;
  o.rv = o.nrm + NB * 16;
  o.panel = o.rv + NB * 16;
  int panel_sz = (NB + 1) * 256;
  if (panel_sz < 64 * W) panel_sz = 64 * W;  // reused for centring partials
  o.rinv = o.panel + panel_sz;
  o.dsc = o.rinv + 256;
  o.red = o.dsc + 256;
  o.total = o.red + 4 * W + 16;
  return o;
}

GPK_DEVICE int frag_index(int n, int d, int DC) {
  const int blk = n >> 4, c = n & 15, dd = d >> 4, g = (d >> 2) & 3, r = d & 3;
  return ((blk * DC + dd) * 64 + 16 * g + c) * 4 + r;
}

// Factor one 16x16 diagonal tile (given as -T in acc layout) in a single wave.
// Writes L's diagonal block (row-major, ld = N) when Lrow != nullptr, publishes
// -R^{-1} in acc layout to rinv_out, returns the 1-based failing column or 0.
GPK_DEVICE int diag_factor(const f32x4 a, float* dsc, float* rinv_out, float* Lblk,
                           int N, int row0, float& logdet) {
  // Launder the lane id so the per-lane compare masks below are not hoisted out
  // of the caller's loops (they would each pin an SGPR pair for the whole kernel).
  int lane = threadIdx.x & 63;
  asm volatile("" : "+v"(lane));
  const int c = lane & 15, grp = lane >> 4;
  *(f32x4*)&dsc[lane * 4] = a;
  wave_lds_sync();
  float col[16];
#pragma unroll
  for (int g = 0; g < 4; ++g) {
    const f32x4 v = *(const f32x4*)&dsc[(16 * g + c) * 4];
#pragma unroll
    for (int r = 0; r < 4; ++r) col[4 * g + r] = -v[r];
  }
  int fail = 0;
#pragma unroll
  for (int m = 0; m < 16; ++m) {
    __builtin_amdgcn_sched_barrier(0);
    const float piv = readlane_f(col[m], m);
    if (!(piv > 0.f) && fail == 0) fail = m + 1;
    const float rowv = col[m] * __builtin_amdgcn_rsqf(piv);
    col[m] = rowv;
#pragma unroll
    for (int i = m + 1; i < 16; ++i) {
      const float s = readlane_f(rowv, i);
      col[i] = __builtin_fmaf(-s, rowv, col[i]);
    }
    // Pin the right-looking order: materialise every column update now so the
    // compiler does not sink the FMAs (which keeps 100+ readlane SGPRs live).
#pragma unroll
    for (int i = m; i < 16; ++i) asm volatile("" : "+v"(col[i]));
    asm volatile("" : "+v"(fail));
  }
  // log|T| = sum_c log R[c][c]^2 (GPyTorch: _chol_diag.pow(2).log().sum())
  {
    float dg = col[0];
#pragma unroll
    for (int i = 1; i < 16; ++i) dg = (c == i) ? col[i] : dg;
    float lg = (lane < 16) ? __builtin_amdgcn_logf(dg * dg) : 0.f;
#pragma unroll
    for (int off = 8; off > 0; off >>= 1) lg += __shfl_xor(lg, off, 64);
    logdet += readlane_f(lg, 0) * 0.69314718055994531f;  // v_log_f32 is log2
  }
#pragma unroll
  for (int i = 0; i < 16; ++i)
    if (i > c) col[i] = 0.f;
  // L diagonal block: L[row0 + c][row0 + i] = R[i][c] = col[i]
  if (Lblk != nullptr) {
    const f32x4 o = pick_group4(col, grp);
    const int row = row0 + c, colg = row0 + 4 * grp;
    if (row < N) {
      if (((N & 3) == 0) && colg + 3 < N) {
        *(f32x4*)&Lblk[(size_t)row * N + colg] = o;
      } else {
#pragma unroll
        for (int r = 0; r < 4; ++r)
          if (colg + r < N) Lblk[(size_t)row * N + colg + r] = o[r];
      }
    }
  }
  // In-place upper-triangular inverse, column c per lane: X = R^{-1}.
#pragma unroll
  for (int i = 15; i >= 0; --i) {
    __builtin_amdgcn_sched_barrier(0);
    const float rii = readlane_f(col[i], i);
    float acc = (c == i) ? 1.f : 0.f;
#pragma unroll
    for (int p = i + 1; p < 16; ++p) {
      const float s = readlane_f(col[i], p);  // R[i][p]
      acc = __builtin_fmaf(-s, col[p], acc);
    }
    col[i] = acc * __builtin_amdgcn_rcpf(rii);
    asm volatile("" : "+v"(col[i]));
  }
  f32x4 q = pick_group4(col, grp);
  q = -q;
  *(f32x4*)&rinv_out[lane * 4] = q;
  return fail;
}

// Tile held by slot s of wave wv (t = wv + W*s, see tile_of in gpk_common.h).
// Called with a laundered wave id inside every phase so the compiler cannot
// hoist per-slot coordinates/addresses out of the factorisation loop (they
// would pin ~2 SGPRs + 2 VGPRs per slot for the whole kernel).
template <int NB, int W>
GPK_DEVICE void slot_tile(int wv, int s, int& i, int& j) {
  constexpr int NTU = NB * (NB + 1) / 2, NT = NTU + NB;
  const int t = wv + W * s;
  if (t < NTU) { const int v = c_tile_ij[t]; i = v & 255; j = v >> 8; }
  else if (t < NT) { i = t - NTU; j = NB; }
  else { i = -1; j = -1; }
}

GPK_DEVICE int launder_s(int v) { asm volatile("" : "+s"(v)); return v; }

GPK_DEVICE void store_block(float* L, int N, int row, int colg, const f32x4 v) {
  if (row >= N) return;
  if (((N & 3) == 0) && colg + 3 < N) {
    *(f32x4*)&L[(size_t)row * N + colg] = v;
  } else {
#pragma unroll
    for (int r = 0; r < 4; ++r)
      if (colg + r < N) L[(size_t)row * N + colg + r] = v[r];
  }
}

template <int NB, int W>
__global__ void __launch_bounds__(64 * W, 4)
gpk_exact_kernel(const float* __restrict__ X, const float* __restrict__ y,
                 const float* __restrict__ hyp, int n_ls, int N, int D, int DC,
                 double jitter0, int max_tries, float* __restrict__ Lout,
                 float* __restrict__ zout, float* __restrict__ mll,
                 int* __restrict__ info) {
  constexpr int NTU = NB * (NB + 1) / 2;
  constexpr int NT = NTU + NB;
  constexpr int SLOTS = (NT + W - 1) / W;
  constexpr int T = 64 * W;
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const ExactLds lay = exact_lds_layout(NB, DC, W);
  float* xf = smem + lay.xf;
  float* nrm = smem + lay.nrm;
  float* rv = smem + lay.rv;
  float* panel = smem + lay.panel;
  float* rinv = smem + lay.rinv;
  float* dsc = smem + lay.dsc;
  float* red = smem + lay.red;
  int* flag = (int*)(red + 4 * W);

  const int tid = threadIdx.x;
  const int lane = tid & 63, c = lane & 15, grp = lane >> 4;
  const int wave = wave_id_uniform();
  const int b = blockIdx.x;
  const int DP = DC * 16;
  const int NP = NB * 16;

  const float s2 = hyp[0];
  const float noise = hyp[1];
  const float cmean = hyp[2];

  // ---- 1. stage X / l into LDS in fragment layout (zero padded) ----------
  const float* Xb = X + (size_t)b * N * D;
  for (int idx = tid; idx < NP * DP; idx += T) {
    const int n = idx / DP, d = idx - n * DP;
    float v = 0.f;
    if (n < N && d < D) v = Xb[(size_t)n * D + d] / hyp[3 + (n_ls == 1 ? 0 : d)];
    xf[frag_index(n, d, DC)] = v;
  }
  __syncthreads();
  // ---- 2. centre columns by the mean over the N real rows (GPyTorch _sq_dist)
  {
    const int parts = T / DP;  // DP divides T (host guarantees DP <= T, power-of-2 chunking)
    const int part = tid / DP, d = tid - part * DP;
    if (part < parts) {
      float s = 0.f;
      for (int n = part; n < N; n += parts) s += xf[frag_index(n, d, DC)];
      panel[part * DP + d] = s;
    }
    __syncthreads();
    if (tid < DP) {
      float s = 0.f;
      for (int p = 0; p < parts; ++p) s += panel[p * DP + tid];
      rinv[tid] = s / (float)N;
    }
    __syncthreads();
    for (int idx = tid; idx < N * DP; idx += T) {
      const int n = idx / DP, d = idx - n * DP;
      if (d < D) xf[frag_index(n, d, DC)] -= rinv[d];
    }
    __syncthreads();
  }
  // ---- 3. squared norms and residual r = y - c ---------------------------
  for (int n = tid; n < NP; n += T) {
    float s = 0.f;
    for (int d = 0; d < D; ++d) {
      const float v = xf[frag_index(n, d, DC)];
      s = __builtin_fmaf(v, v, s);
    }
    nrm[n] = s;
    rv[n] = (n < N) ? (y[(size_t)b * N + n] - cmean) : 0.f;
  }

  float* Lb = Lout ? Lout + (size_t)b * N * N : nullptr;
  // ---- zero the strictly-upper 16x16 blocks of L once (never rewritten) ----
  if (Lb != nullptr) {
    const int vec = ((N & 3) == 0);
    for (int row = wave; row < N; row += W) {
      const int c0 = ((row >> 4) + 1) << 4;  // first column of the next block column
      if (vec) {
        for (int cc = c0 + 4 * lane; cc < N; cc += 256)
          *(f32x4*)&Lb[(size_t)row * N + cc] = f32x4{0.f, 0.f, 0.f, 0.f};
      } else {
        for (int cc = c0 + lane; cc < N; cc += 64) Lb[(size_t)row * N + cc] = 0.f;
      }
    }
  }
  const float nhalf_log2e = -0.72134752044448170f;  // -0.5 * log2(e)
  float diagval = s2 + noise;
  double jit_prev = 0.0;
  int info_w = 0;
  f32x4 acc[SLOTS];

  for (int attempt = 0; attempt <= max_tries; ++attempt) {
    if (attempt > 0) {
      double p10 = 1.0;
      for (int q = 1; q < attempt; ++q) p10 *= 10.0;
      const double jn = jitter0 * p10;
      diagval = diagval + (float)(jn - jit_prev);
      jit_prev = jn;
    }
    if (tid == 0) flag[0] = 0;
    __syncthreads();

    // ---- 4. RBF tiles straight into the accumulators (negated) -----------
    const int wv0 = launder_s(wave);
#pragma unroll
    for (int s = 0; s < SLOTS; ++s) {
      int i, j;
      slot_tile<NB, W>(wv0, s, i, j);
      if (i < 0) continue;
      if (j < NB) {
        f32x4 g = {0.f, 0.f, 0.f, 0.f};
        for (int dd = 0; dd < DC; ++dd) {
          const f32x4 xa = *(const f32x4*)&xf[((i * DC + dd) * 64 + lane) * 4];
          const f32x4 xb = *(const f32x4*)&xf[((j * DC + dd) * 64 + lane) * 4];
          g = mma_tn(xa, xb, g);
        }
        const f32x4 nr = *(const f32x4*)&nrm[16 * i + 4 * grp];
        const int col = 16 * j + c;
        const float nc = nrm[col];
        f32x4 o;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int row = 16 * i + 4 * grp + r;
          float dist = nr[r] + nc - 2.f * g[r];
          dist = dist < 0.f ? 0.f : dist;  // clamp_min(0), NaN-propagating like torch
          float v = s2 * __builtin_amdgcn_exp2f(nhalf_log2e * dist);
          if (row == col) v = diagval;
          if (row >= N || col >= N) v = (row == col) ? 1.f : 0.f;
          o[r] = -v;
        }
        acc[s] = o;
      } else {
        const f32x4 rr = *(const f32x4*)&rv[16 * i + 4 * grp];
        acc[s] = (c == 0) ? -rr : f32x4{0.f, 0.f, 0.f, 0.f};
      }
    }

    float logdet = 0.f, sumz2 = 0.f;
    int failed = 0;
    for (int k = 0; k < NB; ++k) {
      // ---- A(k): factor the diagonal tile --------------------------------
      {
        const int t = k * (k + 1) / 2 + k;
        if (wave == t % W) {
          f32x4 a = {0.f, 0.f, 0.f, 0.f};
          const int slot = t / W;
#pragma unroll
          for (int s = 0; s < SLOTS; ++s)
            if (s == slot) a = acc[s];
          const int f = diag_factor(a, dsc, rinv, Lb, N, 16 * k, logdet);
          if (f != 0 && lane == 0) flag[0] = 16 * k + f;
        }
      }
      __syncthreads();
      if (flag[0] != 0) { failed = flag[0]; break; }
      // ---- B(k): panel TRSM  R_kj = R_kk^{-T} T_kj ----------------------
      {
        const f32x4 q = *(const f32x4*)&rinv[lane * 4];
        const int wv = launder_s(wave);
#pragma unroll
        for (int s = 0; s < SLOTS; ++s) {
          int i, j;
          slot_tile<NB, W>(wv, s, i, j);
          if (i != k || j <= k) continue;
          const f32x4 rkj = mma_tn(q, acc[s], f32x4{0.f, 0.f, 0.f, 0.f});
          acc[s] = rkj;
          *(f32x4*)&panel[j * 256 + lane * 4] = rkj;
          if (j < NB) {
            if (Lb != nullptr) {
              // L[16j + c][16k + 4g + r] = R_kj[4g + r][c]; zero mirror block.
              store_block(Lb, N, 16 * j + c, 16 * k + 4 * grp, rkj);
            }
          } else if (c == 0) {
#pragma unroll
            for (int r = 0; r < 4; ++r) sumz2 = __builtin_fmaf(rkj[r], rkj[r], sumz2);
            if (zout != nullptr) {
              const int row = 16 * k + 4 * grp;
#pragma unroll
              for (int r = 0; r < 4; ++r)
                if (row + r < N) zout[(size_t)b * N + row + r] = rkj[r];
            }
          }
        }
      }
      __syncthreads();
      // ---- C(k): trailing update  -T_ij += R_ki^T R_kj ---------------------
      {
      const int wv = launder_s(wave);
#pragma unroll
      for (int s = 0; s < SLOTS; ++s) {
        int i, j;
        slot_tile<NB, W>(wv, s, i, j);
        if (i <= k) continue;
        const f32x4 pi = *(const f32x4*)&panel[i * 256 + lane * 4];
        const f32x4 pj = *(const f32x4*)&panel[j * 256 + lane * 4];
        acc[s] = mma_tn(pi, pj, acc[s]);
      }
      }
    }
    if (!failed) {
      info_w = attempt > 0 ? -attempt : 0;
      // ---- 5. reduce logdet / |z|^2 over waves, write the MLL -----------
      if (lane == 0) red[wave] = logdet;
      const float z2 = wave_sum(sumz2);
      if (lane == 0) red[W + wave] = z2;
      __syncthreads();
      if (tid == 0) {
        float ld = 0.f, zz = 0.f;
        for (int w = 0; w < W; ++w) { ld += red[w]; zz += red[W + w]; }
        mll[b] = -0.5f * (zz + ld + (float)N * kLog2Pi) / (float)N;
        info[b] = info_w;
      }
      return;
    }
    info_w = failed;
    __syncthreads();
  }
  if (tid == 0) {
    info[b] = info_w;
    mll[b] = __builtin_nanf("");
  }
}

template <int NB>
int launch_exact_nb(const GpkExactArgs& a, hipStream_t stream) {
  constexpr int W = NB >= 6 ? 8 : 4;
  const int DC = (a.D + 15) / 16;
  const ExactLds lay = exact_lds_layout(NB, DC, W);
  const size_t lds = (size_t)lay.total * sizeof(float);
  if (DC * 16 > 64 * W || DC * 16 > 256) return -7;
  if (lds > 160 * 1024) return -7;
  static bool attr_done = false;  // benign race: idempotent attribute set
  if (!attr_done && lds > 64 * 1024) {
    (void)hipFuncSetAttribute((const void*)gpk_exact_kernel<NB, W>,
                        hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    attr_done = true;
  }
  hipLaunchKernelGGL((gpk_exact_kernel<NB, W>), dim3(a.B), dim3(64 * W), lds, stream,
                     a.X, a.y, a.hyp, a.n_ls, a.N, a.D, DC, a.jitter, a.max_tries,
                     a.L, a.z, a.mll, a.info);
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? 0 : (int)e;
}

}  // namespace

int gpk_launch_exact(const GpkExactArgs& a, hipStream_t stream) {
  const int NB = (a.N + 15) / 16;
  switch (NB) {
#define GPK_CASE(nb) case nb: return launch_exact_nb<nb>(a, stream);
    GPK_CASE(1) GPK_CASE(2) GPK_CASE(3) GPK_CASE(4) GPK_CASE(5) GPK_CASE(6)
    GPK_CASE(7) GPK_CASE(8) GPK_CASE(9) GPK_CASE(10) GPK_CASE(11) GPK_CASE(12)
    GPK_CASE(13) GPK_CASE(14) GPK_CASE(15) GPK_CASE(16)
#undef GPK_CASE
    default: return -6;
  }
}
