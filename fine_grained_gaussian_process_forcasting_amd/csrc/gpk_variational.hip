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
// Kernels (the shared K_ZZ factor and its adjoint: gpk_kzz.hip, gpk_kzz_grad.hip):
//   gpk_var_fwd_kernel  the per-point work as ONE column-tiled GEMM A = L^{-1} [K_ZX(b=0) | ...]:
//                       a workgroup owns a chunk of TW points of one window and all M rows of A;
//                       K_ZX chunk from an f32-MFMA Gram (GPyTorch's centred _sq_dist form) in
//                       LDS, A in fp64 MFMA accumulators (v_mfma_f64_16x16x4f64, triangular
//                       k-range per row tile), mean / variance reduced in the epilogue.
//   gpk_var_ell_kernel  per-window ELL sum from the written mean / var (fixed order: deterministic).
//   gpk_var_adj_kernel  adjoint, same tiling: recomputes K_ZX, A; dA; dK = L^{-T} dA (fp64 MFMA);
//                       Q = dK o K_ZX; dX per point, and per-workgroup partials of
//                       Q X (M x D), sum_i Q, dvmean, dvstd, ds2, dl (deterministic, no atomics);
//                       dA and K_ZX (fp32, as the reference's fp32 dA) go to the workspace for
//   gpk_dlinv_kernel    dL^{-1} = sum_points dA K_ZX^T: split-K fp64-MFMA GEMM, 64 x 64 lower tiles;
//   gpk_var_red_kernel / gpk_var_fin_kernel  fixed-order sums of the partials -> outputs.
#include "gpk_common.h"
#include "gpk_internal.h"

#include <mutex>

// Timing experiments only (A/B builds of the adjoint; results are wrong when set): bit 1
// skips A = L^-1 K_ZX, 2 dK = L^-T dA, 4 the dA / K_ZX workspace stores, 8 the Q / Q^T zs /
// QX section, 16 the q column sums, 32 the dX loop.
#ifndef GPK_VAR_SKIP
#define GPK_VAR_SKIP 0
#endif


namespace {

constexpr float kLog2PiF = 1.8378770664093453f;
constexpr float kNHalfLog2e = -0.72134752044448170f;  // -0.5 * log2(e)

#define GPK_HOST_DEVICE_INLINE __host__ __device__ __forceinline__

GPK_DEVICE f64x4 mfma64(double a, double b, f64x4 c) {
  return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
}
GPK_DEVICE f32x4 mfma32(float a, float b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}
// Sum over the 16 lanes of a row (lanes sharing g), DPP only.
GPK_DEVICE float row16_sum_f(float v) {
#define GPK_DPP_ADD(ctrl) \
  v += __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), ctrl, 0xf, 0xf, false));
  GPK_DPP_ADD(0xB1) GPK_DPP_ADD(0x4E) GPK_DPP_ADD(0x141) GPK_DPP_ADD(0x140)
#undef GPK_DPP_ADD
  return v;
}

// Add v into an LDS accumulator that only the calling wave updates, without a round trip: a
// no-return LDS add (no wait, where `*p += v` costs a read, a full LDS-latency wait and a
// write). One wave's LDS operations execute in issue order, so the adds land in program
// order: the sums stay deterministic.
GPK_DEVICE void lds_acc(float* p, float v) {
  (void)__hip_atomic_fetch_add(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
}

// Order of the per-wave scratch transposes: one wave's LDS operations execute in issue order,
// so a code-motion barrier is enough between a tile's writes, its reads and the next tile's
// writes (GPK_ADJ_LDS_WAIT=1: the waitcnt-draining wave_lds_sync instead, for A/B builds)
#ifndef GPK_ADJ_LDS_WAIT
#define GPK_ADJ_LDS_WAIT 0
#endif
GPK_DEVICE void adj_lds_order() {
#if GPK_ADJ_LDS_WAIT
  wave_lds_sync();
#else
  __builtin_amdgcn_wave_barrier();
#endif
}

// Per-chunk LDS base the compiler must treat as new on every iteration: the staged
// operands (L^{-1}, zs, norms) and their per-lane addresses would otherwise be hoisted out of the chunk loop as
// loop-invariant loads and pinned in (hundreds of) registers.
GPK_DEVICE const float* fresh_lds(const float* p) {
  int z = 0;
  asm volatile("" : "+s"(z));
  return p + z;
}
// The same for a global pointer whose per-lane addresses would be loop-invariant.
template <typename T>
GPK_DEVICE const T* fresh_ptr(const T* p) {
  asm volatile("" : "+s"(p));
  return p;
}

// ---------------------------------------------------------------------------
// Column-tile geometry shared by the forward and adjoint kernels.
//   MB  = 16-row blocks of the inducing dimension (M <= 16 MB <= 256)
//   4 waves = WR (along rows of A) x WC (along points); a wave owns row tiles
//   {wr + WR j} (interleaved: balances the triangular k-range) and CT = 2 column tiles.
//   TW  = points per chunk; a workgroup walks the chunks {part, part + S, ...} of window b.
// ---------------------------------------------------------------------------
template <int MB>
struct VarGeo {
  static constexpr int WR = MB <= 4 ? 1 : (MB <= 8 ? 2 : 4);
  static constexpr int WC = 4 / WR;
  static constexpr int RT = (MB + WR - 1) / WR;
  static constexpr int CT = 2;
  static constexpr int TW = 16 * CT * WC;
  static constexpr int MP = 16 * MB;
  static constexpr int QST = (MP % 32 == 0) ? MP + 16 : MP;  // Q^T row stride (bank spread)
};

// D padded to a power of two >= 16 (<= 64): MFMA k-steps and d-tiles, and 256 % Dq == 0.
GPK_HOST_DEVICE_INLINE int dq_of(int D) { return D <= 16 ? 16 : (D <= 32 ? 32 : 64); }

// Column means of zs (rows 0..M-1, columns 0..Dq-1, row stride ds) in ONE fixed order for
// every kernel that centres the inducing points (stage_inducing, gpk_var_fin_kernel): 8
// partial sums per column over the rows m = k (mod 8), ascending, then k = 0..7 (a serial
// sum over all M rows per column was ~20K cycles of dependent LDS reads at M = 256).
// scr: >= 8 Dq floats of free LDS. Ends with a barrier.
constexpr int kCmParts = 8;
GPK_DEVICE void col_means(const float* zs, int M, int D, int Dq, int ds, float* scr, float* cm) {
  const int tid = threadIdx.x, T = blockDim.x;
  for (int e = tid; e < kCmParts * Dq; e += T) {
    const int d = e % Dq, k = e / Dq;
    float a = 0.f;
    for (int m = k; m < M; m += kCmParts) a += zs[m * ds + d];
    scr[e] = a;
  }
  lds_barrier();
  for (int d = tid; d < Dq; d += T) {
    float a = 0.f;
#pragma unroll
    for (int k = 0; k < kCmParts; ++k) a += scr[k * Dq + d];
    cm[d] = d < D ? a / (float)M : 0.f;   // GPyTorch _sq_dist centres by x1 = Z
  }
  lds_barrier();
}

// Stage the centred, scaled inducing points zs = Z/l - mean(Z/l) (rows >= M and
// columns >= D zero), their squared norms, the q(u) mean and s^2 - 1. scr: >= 8 Dq floats
// of LDS that is free during the staging.
GPK_DEVICE void stage_inducing(const float* __restrict__ Z, const float* __restrict__ ls,
                               const float* __restrict__ vmean, const float* __restrict__ vstd,
                               int M, int D, int MP, int Dq, int ds, float* zs, float* zn, float* cm,
                               float* vm, float* sm1, float* scr) {
  const int tid = threadIdx.x, T = blockDim.x;
  // 8 unconditional loads (clamped addresses) in flight per thread, then the stores:
  // a predicated load per loop iteration costs one full memory latency each
  for (int base = 0; base < MP * Dq; base += 8 * T) {
    float v[8], l[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int e = base + u * T + tid, m = e / Dq, d = e - m * Dq;
      const bool ok = e < MP * Dq && m < M && d < D;
      v[u] = Z[ok ? m * D + d : 0];
      l[u] = ls[ok ? d : 0];
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int e = base + u * T + tid, m = e / Dq, d = e - m * Dq;
      if (e < MP * Dq) zs[m * ds + d] = (m < M && d < D) ? v[u] / l[u] : 0.f;
    }
  }
  for (int m = tid; m < MP; m += T) {
    vm[m] = (m < M) ? vmean[m] : 0.f;
    const float sd = (m < M) ? vstd[m] : 1.f;
    sm1[m] = sd * sd - 1.f;
  }
  lds_barrier();
  col_means(zs, M, D, Dq, ds, scr, cm);
  for (int e = tid; e < M * Dq; e += T) {
    const int m = e / Dq, d = e - m * Dq;
    zs[m * ds + d] -= cm[d];
  }
  lds_barrier();
  for (int m = tid; m < MP; m += T) {
    float s = 0.f;
    for (int d = 0; d < Dq; ++d) s = __builtin_fmaf(zs[m * ds + d], zs[m * ds + d], s);
    zn[m] = s;
  }
}

// Stage the chunk's points xs = x/l - cm (invalid columns zero) and their norms.
GPK_DEVICE void stage_points(const float* __restrict__ Xw, const float* __restrict__ ls, int nvalid,
                             int D, int TW, int Dq, int ds, const float* cm, float* xs, float* xn) {
  const int tid = threadIdx.x, T = blockDim.x;
  for (int base = 0; base < TW * Dq; base += 4 * T) {   // loads in flight together (stage_inducing)
    float v[4], l[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int e = base + u * T + tid, j = e / Dq, d = e - j * Dq;
      const bool ok = e < TW * Dq && j < nvalid && d < D;
      v[u] = Xw[ok ? (size_t)j * D + d : 0];
      l[u] = ls[ok ? d : 0];
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int e = base + u * T + tid, j = e / Dq, d = e - j * Dq;
      if (e < TW * Dq) xs[j * ds + d] = (j < nvalid && d < D) ? v[u] / l[u] - cm[d] : 0.f;
    }
  }
  lds_barrier();
  for (int j = tid; j < TW; j += T) {
    float s = 0.f;
    for (int d = 0; d < Dq; ++d) s = __builtin_fmaf(xs[j * ds + d], xs[j * ds + d], s);
    xn[j] = s;
  }
}

// K_ZX chunk (MP x TW, LDS) = s2 exp(-0.5 clamp(|zs|^2 + |xs|^2 - 2 zs.xs, 0)) on f32 MFMA.
template <int MB, int TW>
GPK_DEVICE void build_kzx(const float* zs, const float* xs, const float* zn, const float* xn,
                          int M, int nvalid, int Dq, int ds, float s2, float* Kl) {
  const int lane = threadIdx.x & 63, c = lane & 15, g = lane >> 4;
  const int wave = threadIdx.x >> 6;
  constexpr int NCT = TW / 16;
  for (int t = wave; t < MB * NCT; t += 4) {
    const int rt = t / NCT, ct = t - rt * NCT;
    const float* za = zs + (16 * rt + c) * ds + g;
    const float* xb = xs + (16 * ct + c) * ds + g;
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    for (int k = 0; k < Dq / 4; ++k) acc = mfma32(za[4 * k], xb[4 * k], acc);
    const int col = 16 * ct + c;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int p = 16 * rt + 4 * g + r;
      float dist = zn[p] + xn[col] - 2.f * acc[r];
      dist = dist < 0.f ? 0.f : dist;
      Kl[p * TW + col] = (p < M && col < nvalid) ? s2 * __builtin_amdgcn_exp2f(kNHalfLog2e * dist) : 0.f;
    }
  }
}

// A = L^{-1} K_ZX for the wave's row tiles (fp64 MFMA). acc[j][q][r] = A[16 rt_j + g + 4r][16 ct_q + c].
// The contraction runs in k-blocks of 16 inducing points; inside a block MFMA step u
// takes p = 16 kb + 4 g + u on lane group g (any consistent k-order is legal), so a
// lane's four A operands of a block are 4 consecutive doubles of one L^{-1} row. The
// whole next block's A operands are loaded while the current block's MFMAs run (row
// tile rt only needs blocks kb <= rt: L^{-1} is lower triangular).
template <int MB>
GPK_DEVICE void gemm_linv_k(const double* __restrict__ Linv, const float* Kl, int M,
                            f64x4 (&acc)[VarGeo<MB>::RT][VarGeo<MB>::CT]) {
  using G = VarGeo<MB>;
  const int lane = threadIdx.x & 63, c = lane & 15, g = lane >> 4;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wr = wave / G::WC, wc = wave - wr * G::WC;
#pragma unroll
  for (int j = 0; j < G::RT; ++j)
#pragma unroll
    for (int q = 0; q < G::CT; ++q) acc[j][q] = f64x4{0.0, 0.0, 0.0, 0.0};
  int last = 0;
#pragma unroll
  for (int j = 0; j < G::RT; ++j)
    if (wr + G::WR * j < MB) last = wr + G::WR * j;
  double an[G::RT][4];
  auto load_blk = [&](int kb, double (&dst)[G::RT][4]) {
#pragma unroll
    for (int j = 0; j < G::RT; ++j) {
      const int rt = wr + G::WR * j;
      const int m = 16 * rt + c;
      const bool ok = rt < MB && kb <= rt && m < M;
      const double* row = Linv + (size_t)(ok ? m : 0) * M;
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int p = 16 * kb + 4 * g + u;
        dst[j][u] = (ok && p < M) ? row[p] : 0.0;
      }
    }
  };
  load_blk(0, an);
  for (int kb = 0; kb <= last; ++kb) {
    double a[G::RT][4];
#pragma unroll
    for (int j = 0; j < G::RT; ++j)
#pragma unroll
      for (int u = 0; u < 4; ++u) a[j][u] = an[j][u];
    if (kb < last) load_blk(kb + 1, an);
    float bf[G::CT][4];
#pragma unroll
    for (int q = 0; q < G::CT; ++q)
#pragma unroll
      for (int u = 0; u < 4; ++u) bf[q][u] = Kl[(16 * kb + 4 * g + u) * G::TW + 16 * (wc * G::CT + q) + c];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
#pragma unroll
      for (int j = 0; j < G::RT; ++j) {
        const int rt = wr + G::WR * j;
        if (rt < MB && kb <= rt) {
#pragma unroll
          for (int q = 0; q < G::CT; ++q) acc[j][q] = mfma64(a[j][u], (double)bf[q][u], acc[j][q]);
        }
      }
    }
  }
}

// ---------------------------------------------------------------------------
// Forward: mean / variance of q(f) for every point (workgroups walk the chunk list).
// ---------------------------------------------------------------------------
template <int MB>
__global__ void __launch_bounds__(256)
gpk_var_fwd_kernel(const float* __restrict__ X, const float* __restrict__ Z,
                   const double* __restrict__ Linv, const float* __restrict__ vmean,
                   const float* __restrict__ vstd, const float* __restrict__ hyp, int N, int M,
                   int D, int nchunks, float* __restrict__ mean_out, float* __restrict__ var_out,
                   int* __restrict__ flags) {
  using G = VarGeo<MB>;
  constexpr int TW = G::TW, MP = G::MP;
  extern __shared__ __attribute__((aligned(16))) float vsm[];
  const int Dq = dq_of(D), ds = Dq + 2;
  float* zs = vsm;                 // MP x ds
  float* xs = zs + MP * ds;        // TW x ds
  float* zn = xs + TW * ds;        // MP
  float* xn = zn + MP;             // TW
  float* vm = xn + TW;             // MP
  float* sm1 = vm + MP;            // MP
  float* cm = sm1 + MP;            // Dq
  float* Kl = cm + Dq;             // MP x TW
  float* redm = Kl + MP * TW;      // WR x TW
  float* redv = redm + G::WR * TW; // WR x TW
  const int tid = threadIdx.x;
  const int lane = tid & 63, c = lane & 15, g = lane >> 4;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wave / G::WC, wc = wave - wr * G::WC;
  // hyp: [s2, noise, jitter, b0, w[D], ls[D]]
  const float s2 = hyp[0], jit = hyp[2], b0 = hyp[3];
  const float* w = hyp + 4;
  const float* ls = hyp + 4 + D;

  stage_inducing(Z, ls, vmean, vstd, M, D, MP, Dq, ds, zs, zn, cm, vm, sm1, Kl);
  const int nch = (N + TW - 1) / TW;
  int clamped = 0;
  // grid-stride over (window, chunk) pairs: the inducing-point staging is paid once
  for (int t = blockIdx.x; t < nchunks; t += gridDim.x) {
    const int b = t / nch, ch = t - b * nch;
    const int i0 = ch * TW;
    const int nvalid = N - i0 < TW ? N - i0 : TW;
    const float* Xw = X + ((size_t)b * N + i0) * D;
    lds_barrier();  // previous chunk done with xs / Kl / red; zs staged
    stage_points(Xw, ls, nvalid, D, TW, Dq, ds, cm, xs, xn);
    lds_barrier();
    build_kzx<MB, TW>(zs, xs, zn, xn, M, nvalid, Dq, ds, s2, Kl);
    lds_barrier();
    f64x4 acc[G::RT][G::CT];
    gemm_linv_k<MB>(Linv, Kl, M, acc);
    // epilogue: partial sum_m A m_m and sum_m A^2 (s_m^2 - 1) over the wave's rows
#pragma unroll
    for (int q = 0; q < G::CT; ++q) {
      float mp = 0.f, vp = 0.f;
#pragma unroll
      for (int j = 0; j < G::RT; ++j) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int row = 16 * (wr + G::WR * j) + g + 4 * r;
          const float a32 = (float)acc[j][q][r];  // A is cast to fp32 (reference)
          const int rr = row < MP ? row : 0;
          mp = __builtin_fmaf(a32, row < MP ? vm[rr] : 0.f, mp);
          vp = __builtin_fmaf(a32 * a32, row < MP ? sm1[rr] : 0.f, vp);
        }
      }
      mp += __shfl_xor(mp, 16, 64);
      mp += __shfl_xor(mp, 32, 64);
      vp += __shfl_xor(vp, 16, 64);
      vp += __shfl_xor(vp, 32, 64);
      if (g == 0) {
        redm[wr * TW + 16 * (wc * G::CT + q) + c] = mp;
        redv[wr * TW + 16 * (wc * G::CT + q) + c] = vp;
      }
    }
    lds_barrier();
    for (int col = tid; col < nvalid; col += blockDim.x) {
      float mm = 0.f, vv = 0.f;
#pragma unroll
      for (int q = 0; q < G::WR; ++q) {
        mm += redm[q * TW + col];
        vv += redv[q * TW + col];
      }
      const float* xr = Xw + (size_t)col * D;
      float lin = 0.f;
      for (int d = 0; d < D; ++d) lin = __builtin_fmaf(xr[d], w[d], lin);
      const float mean_i = mm + (lin + b0);
      float var_i = s2 + jit + vv;
      if (var_i < 1e-6f) { var_i = 1e-6f; clamped = 1; }  // MVN.variance clamp (fp32)
      mean_out[(size_t)b * N + i0 + col] = mean_i;
      var_out[(size_t)b * N + i0 + col] = var_i;
    }
  }
  if (flags != nullptr && clamped)
    (void)__hip_atomic_fetch_or(flags, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Per-window ELL sum (fixed summation order: run-to-run deterministic).
__global__ void __launch_bounds__(256)
gpk_var_ell_kernel(const float* __restrict__ mean, const float* __restrict__ var,
                   const float* __restrict__ y, const float* __restrict__ hyp, int N,
                   float* __restrict__ ell) {
  __shared__ float red[4];
  const int b = blockIdx.x, tid = threadIdx.x;
  const float noise = hyp[1];
  const float log_noise = __logf(noise);
  float acc = 0.f;
  for (int i = tid; i < N; i += 256) {
    const size_t o = (size_t)b * N + i;
    const float dy = y[o] - mean[o];
    acc += -0.5f * ((dy * dy + var[o]) / noise + log_noise + kLog2PiF);
  }
  acc = wave_sum(acc);
  if ((tid & 63) == 0) red[tid >> 6] = acc;
  lds_barrier();
  if (tid == 0) ell[b] = (red[0] + red[1]) + (red[2] + red[3]);
}

// ---------------------------------------------------------------------------
// Forward for M > 64 (cfg-3 shape M = 256): L^{-1} held in REGISTERS for the whole launch.
// A persistent workgroup of NWV = ceil(MB/2) waves; wave w owns the row tiles rA = w and
// rB = MB-1-w, i.e. MB+1 16x16 blocks of the lower triangle of L^{-1} (the same count for
// every wave: balanced), loaded once as f64 MFMA A operands: slot s holds, on lane (c, g)
// at MFMA step u, L^{-1}[16 rt + c][16 kb + 4 g + u]. Per 32-point chunk:
//   stage   xs = x/l - mean(Z/l), |xs|^2 and x.w (16 threads per point, DPP row sums);
//   Gram    the K_ZX tiles of the wave's own row tiles on f32 MFMA -- the f32 C layout
//           (reg r <-> row 4g + r) IS the f64 B-operand layout of step u = r, so each tile is
//           one b128 LDS store, read back by every wave as one b128 per (kb, column tile);
//   GEMM    A[rt] += L^{-1}[rt, kb] K_ZX[kb] over the wave's MB+1 blocks (fp64 MFMA);
//   reduce  per-wave partials of sum_m A m and sum_m A^2 (s^2 - 1) -> LDS, one wave finishes
//           mean / variance while the others stage the next chunk (its points were loaded
//           into registers during this chunk's GEMM).
// The LDS-tiled kernel above re-read the L^{-1} triangle (272 KB) from L2 for every chunk.
// ---------------------------------------------------------------------------
constexpr int LTW = 32;   // points per chunk (2 column tiles)

// Per-chunk block of the state the training forward keeps for the adjoint (M > 64):
// A = L^{-1} K_ZX of the chunk cast to fp32 (MB x 2 tiles, element u of lane (c, g) of tile
// (rt, ct) <-> row 16 rt + g + 4u, point 16 ct + c), then the clamp mask of its LTW points
// (1: var_i >= 1e-6, 0: clamped or padding).
template <int MB>
struct LSaved {
  static constexpr int tiles = MB * 2 * 256;
  static constexpr int blk = tiles + LTW;
};

// A[rA] / A[rB] of one chunk for the wave with rA = RA: slots 0..RA are blocks (RA, s),
// slots RA+1..MB blocks (MB-1-RA, s-RA-1). The next slot's K_ZX operands (one b128 per
// column tile) are read while this slot's 8 MFMAs run; a scheduling fence per slot keeps
// the reads from all being hoisted.
template <int MB, int RA>
GPK_DEVICE void lreg_gemm(const double (&Lr)[MB + 1][4], const float* Kl, int lane,
                          f64x4 (&aA)[2], f64x4 (&aB)[2]) {
  constexpr int RB = MB - 1 - RA;
  constexpr int NS = RB == RA ? RA + 1 : MB + 1;
  f64x4 acc[2] = {f64x4{0.0, 0.0, 0.0, 0.0}, f64x4{0.0, 0.0, 0.0, 0.0}};
  f32x4 k0 = *(const f32x4*)(Kl + (0 * 64 + lane) * 4);
  f32x4 k1 = *(const f32x4*)(Kl + (1 * 64 + lane) * 4);
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    if (s == RA + 1) {
      aA[0] = acc[0];
      aA[1] = acc[1];
      acc[0] = acc[1] = f64x4{0.0, 0.0, 0.0, 0.0};
    }
    f32x4 n0 = k0, n1 = k1;
    if (s + 1 < NS) {
      const int kbn = s + 1 <= RA ? s + 1 : s - RA;
      n0 = *(const f32x4*)(Kl + ((kbn * 2 + 0) * 64 + lane) * 4);
      n1 = *(const f32x4*)(Kl + ((kbn * 2 + 1) * 64 + lane) * 4);
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      acc[0] = mfma64(Lr[s][u], (double)k0[u], acc[0]);
      acc[1] = mfma64(Lr[s][u], (double)k1[u], acc[1]);
    }
    k0 = n0;
    k1 = n1;
    __builtin_amdgcn_sched_barrier(0);
  }
  if (RB == RA) {
    aA[0] = acc[0];
    aA[1] = acc[1];
    aB[0] = aB[1] = f64x4{0.0, 0.0, 0.0, 0.0};
  } else {
    aB[0] = acc[0];
    aB[1] = acc[1];
  }
}
template <int MB, int RA>
GPK_DEVICE void lreg_gemm_for(int wave, const double (&Lr)[MB + 1][4], const float* Kl, int lane,
                              f64x4 (&aA)[2], f64x4 (&aB)[2]) {
  if constexpr (RA < (MB + 1) / 2) {
    if (wave == RA) lreg_gemm<MB, RA>(Lr, Kl, lane, aA, aB);
    else lreg_gemm_for<MB, RA + 1>(wave, Lr, Kl, lane, aA, aB);
  }
}

template <int MB, int DQ>
struct LGeo {
  static constexpr int NWV = (MB + 1) / 2;              // waves
  static constexpr int NT = 64 * NWV;
  static constexpr int MP = 16 * MB;
  static constexpr int DS = DQ + 2;                     // zs / xs row stride (floats)
  static constexpr int NPASS = (LTW * 16 + NT - 1) / NT; // point-staging passes (16 thr / point)
  static constexpr int DV = DQ / 16;                    // dims per staging thread
  // LDS (floats): Kl first (b128 aligned)
  static constexpr int oKl = 0;                          // MB x 2 tiles x 64 lanes x 4
  static constexpr int oRed = oKl + MP * LTW;            // NWV x 2 x LTW
  static constexpr int oZs = oRed + NWV * 2 * LTW;       // MP x DS
  static constexpr int oZn = oZs + MP * DS;
  static constexpr int oVm = oZn + MP;
  static constexpr int oSm1 = oVm + MP;
  static constexpr int oCm = oSm1 + MP;                  // DQ
  static constexpr int oXs = oCm + DQ;                   // LTW x DS
  static constexpr int oXn = oXs + LTW * DS;             // LTW
  static constexpr int oLin = oXn + LTW;                 // 2 x LTW (chunk parity)
  static constexpr int total = oLin + 2 * LTW;
};

template <int MB, int DQ>
__global__ void __launch_bounds__(64 * ((MB + 1) / 2), 2)
gpk_var_fwd_l_kernel(const float* __restrict__ X, const float* __restrict__ Z,
                     const double* __restrict__ Linv, const float* __restrict__ vmean,
                     const float* __restrict__ vstd, const float* __restrict__ hyp, int N, int M,
                     int D, int nchunks, float* __restrict__ mean_out, float* __restrict__ var_out,
                     int* __restrict__ flags, float* __restrict__ saved) {
  using G = LGeo<MB, DQ>;
  constexpr int NWV = G::NWV, NT = G::NT, DS = G::DS, NPASS = G::NPASS, DV = G::DV;
  extern __shared__ __attribute__((aligned(16))) float vsm[];
  const int tid = threadIdx.x, lane = tid & 63, c = lane & 15, g = lane >> 4, sub = tid & 15;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int rA = wave, rB = MB - 1 - wave;   // rB == rA: the middle wave of an odd MB
  // hyp: [s2, noise, jitter, b0, w[D], ls[D]]
  const float s2 = hyp[0], jit = hyp[2], b0 = hyp[3];
  const float* w = hyp + 4;
  const float* ls = hyp + 4 + D;
  const int nch = (N + LTW - 1) / LTW;

  // the wave's L^{-1} blocks -> registers. M % 16 == 0: two row bases, every slot one
  // 32-byte run at an immediate offset (no per-load address registers or masks -- with
  // them the 68 loads in flight at M = 256 overflowed the register file); otherwise
  // masked loads from clamped addresses, 4 slots in flight at a time.
  double Lr[MB + 1][4];
  if ((M & 15) == 0) {
    const double* baseA = Linv + (size_t)(16 * rA + c) * M + 4 * g;
    const double* baseB = Linv + (size_t)(16 * rB + c) * M + 4 * g - 16 * (rA + 1);
#pragma unroll
    for (int s = 0; s <= MB; ++s) {
      const bool isA = s <= rA;
      if (isA || rB != rA) {
        const double* src = (isA ? baseA : baseB) + 16 * s;
        const double2 v0 = *(const double2*)src, v1 = *(const double2*)(src + 2);
        Lr[s][0] = v0.x; Lr[s][1] = v0.y; Lr[s][2] = v1.x; Lr[s][3] = v1.y;
      } else {
#pragma unroll
        for (int u = 0; u < 4; ++u) Lr[s][u] = 0.0;
      }
    }
  } else {
#pragma unroll
    for (int s = 0; s <= MB; ++s) {
      const bool isA = s <= rA;
      const int rt = isA ? rA : rB, kb = isA ? s : s - rA - 1;
      const bool ok = isA || rB != rA;
      const int m = 16 * rt + c;
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int p = 16 * kb + 4 * g + u;
        const bool in = ok && m < M && p < M;
        const double v = Linv[in ? (size_t)m * M + p : 0];
        Lr[s][u] = in ? v : 0.0;
      }
      if ((s & 3) == 3) __builtin_amdgcn_sched_barrier(0);
    }
  }
  // per-thread staging constants: dims d = sub + 16 v
  float lsr[DV], wr[DV];
#pragma unroll
  for (int v = 0; v < DV; ++v) {
    const int d = sub + 16 * v;
    lsr[v] = ls[d < D ? d : 0];
    wr[v] = d < D ? w[d] : 0.f;
  }
  float xr[NPASS][DV];
  auto load_x = [&](int t) {
    const int b = t / nch, i0 = (t - b * nch) * LTW;
#pragma unroll
    for (int q = 0; q < NPASS; ++q) {
      const int j = (tid >> 4) + q * (NT / 16), i = i0 + j;
      const bool ok = t < nchunks && j < LTW && i < N;
#pragma unroll
      for (int v = 0; v < DV; ++v) {
        const int d = sub + 16 * v;
        const bool okd = ok && d < D;
        const float x = X[okd ? ((size_t)b * N + i) * D + d : 0];
        xr[q][v] = okd ? x : 0.f;
      }
    }
  };
  load_x(blockIdx.x);
  stage_inducing(Z, ls, vmean, vstd, M, D, G::MP, DQ, DS, vsm + G::oZs, vsm + G::oZn, vsm + G::oCm,
                 vsm + G::oVm, vsm + G::oSm1, vsm + G::oKl);
  lds_barrier();
  float cmr[DV];
#pragma unroll
  for (int v = 0; v < DV; ++v) cmr[v] = vsm[G::oCm + sub + 16 * v];
  int clamped = 0, par = 0;

  for (int t = blockIdx.x; t < nchunks; t += gridDim.x, par ^= 1) {
    const int b = t / nch, i0 = (t - b * nch) * LTW;
    const int nvalid = N - i0 < LTW ? N - i0 : LTW;
    // every LDS address re-derived per chunk (hoisted, they pinned ~100 registers)
    float* sm = (float*)fresh_lds(vsm);
    float* Kl = sm + G::oKl;
    float* red = sm + G::oRed;
    const float* zs = sm + G::oZs;
    const float* zn = sm + G::oZn;
    const float* vm = sm + G::oVm;
    const float* sm1 = sm + G::oSm1;
    float* xs = sm + G::oXs;
    float* xn = sm + G::oXn;
    float* lin = sm + G::oLin + par * LTW;
    // stage the chunk's points (xs of the previous chunk was last read by its Gram, before
    // the previous GEMM barrier; lin is double-buffered against the finishing wave)
#pragma unroll
    for (int q = 0; q < NPASS; ++q) {
      const int j = (tid >> 4) + q * (NT / 16);
      float nrm = 0.f, lp = 0.f;
      const bool okj = j < nvalid;
#pragma unroll
      for (int v = 0; v < DV; ++v) {
        const int d = sub + 16 * v;
        const float xv = (okj && d < D) ? xr[q][v] / lsr[v] - cmr[v] : 0.f;
        nrm = __builtin_fmaf(xv, xv, nrm);
        lp = __builtin_fmaf(xr[q][v], wr[v], lp);
        if (j < LTW) xs[j * DS + d] = xv;
      }
      nrm = row16_sum_f(nrm);
      lp = row16_sum_f(lp);
      if (sub == 0 && j < LTW) {    // (row16_sum_f leaves the sum on all 16 lanes)
        xn[j] = nrm;
        lin[j] = lp;
      }
    }
    lds_barrier();
    // K_ZX tiles of the wave's row tiles
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int rt = h == 0 ? rA : rB;
      if (h == 1 && rB == rA) break;
#pragma unroll
      for (int ct = 0; ct < 2; ++ct) {
        const float* za = zs + (16 * rt + c) * DS + g;
        const float* xb = xs + (16 * ct + c) * DS + g;
        f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int k = 0; k < DQ / 4; ++k) acc = mfma32(za[4 * k], xb[4 * k], acc);
        const int col = 16 * ct + c;
        const float xnc = xn[col];
        f32x4 o;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int p = 16 * rt + 4 * g + r;
          float dist = zn[p] + xnc - 2.f * acc[r];
          dist = dist < 0.f ? 0.f : dist;
          o[r] = (p < M && col < nvalid) ? s2 * __builtin_amdgcn_exp2f(kNHalfLog2e * dist) : 0.f;
        }
        *(f32x4*)(Kl + ((rt * 2 + ct) * 64 + lane) * 4) = o;
      }
    }
    if (t + (int)gridDim.x < nchunks) load_x(t + gridDim.x);   // next chunk's points
    lds_barrier();
    // A = L^{-1} K_ZX on the wave's row tiles (code specialised per wave: the slot -> row
    // tile switch at rA is then static -- as a runtime test it was if-converted into
    // selects that doubled the accumulators)
    f64x4 aA[2], aB[2];
    lreg_gemm_for<MB, 0>(wave, Lr, Kl, lane, aA, aB);
    if (saved != nullptr) {
      // training: A (fp32, as the reference casts it) in the adjoint's LDS tile layout, so
      // gpk_var_adjs_l_kernel needs neither the forward GEMM nor the K_ZX Gram again
      float* sb = saved + (size_t)t * LSaved<MB>::blk;
#pragma unroll
      for (int ct = 0; ct < 2; ++ct) {
        *(f32x4*)(sb + ((rA * 2 + ct) * 64 + lane) * 4) =
            f32x4{(float)aA[ct][0], (float)aA[ct][1], (float)aA[ct][2], (float)aA[ct][3]};
        if (rB != rA)
          *(f32x4*)(sb + ((rB * 2 + ct) * 64 + lane) * 4) =
              f32x4{(float)aB[ct][0], (float)aB[ct][1], (float)aB[ct][2], (float)aB[ct][3]};
      }
    }
    // partials over the wave's rows (A cast to fp32 as the reference does)
#pragma unroll
    for (int ct = 0; ct < 2; ++ct) {
      float mp = 0.f, vp = 0.f;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int rowA = 16 * rA + g + 4 * r;
        const float a = (float)aA[ct][r];
        mp = __builtin_fmaf(a, vm[rowA], mp);
        vp = __builtin_fmaf(a * a, sm1[rowA], vp);
      }
      if (rB != rA) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int rowB = 16 * rB + g + 4 * r;
          const float a = (float)aB[ct][r];
          mp = __builtin_fmaf(a, vm[rowB], mp);
          vp = __builtin_fmaf(a * a, sm1[rowB], vp);
        }
      }
      mp += __shfl_xor(mp, 16, 64);
      mp += __shfl_xor(mp, 32, 64);
      vp += __shfl_xor(vp, 16, 64);
      vp += __shfl_xor(vp, 32, 64);
      if (g == 0) {
        red[(wave * 2 + 0) * LTW + 16 * ct + c] = mp;
        red[(wave * 2 + 1) * LTW + 16 * ct + c] = vp;
      }
    }
    lds_barrier();
    if (tid < nvalid) {
      float mm = 0.f, vv = 0.f;
#pragma unroll
      for (int q = 0; q < NWV; ++q) {
        mm += red[(q * 2 + 0) * LTW + tid];
        vv += red[(q * 2 + 1) * LTW + tid];
      }
      const float mean_i = mm + (lin[tid] + b0);
      float var_i = s2 + jit + vv;
      const bool clamp = var_i < 1e-6f;
      if (clamp) { var_i = 1e-6f; clamped = 1; }  // MVN.variance clamp (fp32)
      mean_out[(size_t)b * N + i0 + tid] = mean_i;
      var_out[(size_t)b * N + i0 + tid] = var_i;
      // the clamp passes no gradient: the adjoint masks gvar with this
      if (saved != nullptr) saved[(size_t)t * LSaved<MB>::blk + LSaved<MB>::tiles + tid] = clamp ? 0.f : 1.f;
    } else if (saved != nullptr && tid < LTW) {
      saved[(size_t)t * LSaved<MB>::blk + LSaved<MB>::tiles + tid] = 0.f;
    }
  }
  if (flags != nullptr && clamped)
    (void)__hip_atomic_fetch_or(flags, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// ---------------------------------------------------------------------------
// Adjoint of the forward for the objective sum(gmean * mean) + sum(gvar * var).
// Per chunk (same tiling as the forward):
//   K_ZX (LDS), A = L^{-1} K_ZX (fp64 MFMA), var -> clamp mask on gvar,
//   dA = gmean_i m_m + 2 gvar_i (s_m^2 - 1) A_mi   (fp32: the reference's dA is the
//        gradient of an fp32 tensor), dA and K_ZX -> workspace for dL^{-1},
//   dK = L^{-T} dA (fp64 MFMA), Q = dK o K_ZX,
//   dX_i = (sum_p Q_pi zs_p - xs_i sum_p Q_pi) / l + gmean_i w     (written per point)
//   partials per workgroup: QX_p = sum_i Q_pi xs_i, q_p = sum_i Q_pi, sum_i gmean A,
//   sum_i gvar A^2, sum_i r_i xs_i^2, sum Q, sum gvar (reduced by gpk_var_red_kernel).
// ---------------------------------------------------------------------------
template <int MB, int DQ>
__global__ void __launch_bounds__(256, 1)
gpk_var_adj_kernel(const float* __restrict__ X, const float* __restrict__ Z,
                   const double* __restrict__ Linv, const float* __restrict__ vmean,
                   const float* __restrict__ vstd, const float* __restrict__ hyp,
                   const float* __restrict__ gmean, const float* __restrict__ gvar, int N, int M,
                   int D, int nchunks, long long BN, float* __restrict__ wsdA, float* __restrict__ wsK,
                   float* __restrict__ wspart, float* __restrict__ dX) {
  using G = VarGeo<MB>;
  constexpr int TW = G::TW, MP = G::MP, QST = G::QST;
  constexpr int Dq = DQ, ds = DQ + 2, NDT = DQ / 16;
  extern __shared__ __attribute__((aligned(16))) float vsm[];
  float* zs = vsm;                    // MP x ds
  float* xs = zs + MP * ds;           // TW x ds
  float* zn = xs + TW * ds;           // MP
  float* xn = zn + MP;                // TW
  float* vm = xn + TW;                // MP
  float* sm1 = vm + MP;               // MP
  float* cm = sm1 + MP;               // Dq
  float* gmc = cm + Dq;               // TW
  float* gvc = gmc + TW;              // TW
  float* rcol = gvc + TW;             // TW   r_i = sum_p Q_pi
  float* qacc = rcol + TW;            // MP   sum_i Q_pi (this workgroup)
  float* dvma = qacc + MP;            // WC x MP
  float* dsma = dvma + G::WC * MP;    // WC x MP
  float* rx2 = dsma + G::WC * MP;     // 256  per-thread sum r_i xs_i^2 (thread -> one d)
  float* gxa = rx2 + 256;             // 256  per-thread sum gmean_i xs_i (thread -> one d)
  float* redw = gxa + 256;            // 2 x WR x TW
  float* Kl = redw + 2 * G::WR * TW;  // MP x TW     (later: Q^T zs partials, WR x TW x Dq)
  constexpr int KLN = MP * TW > G::WR * TW * DQ ? MP * TW : G::WR * TW * DQ;
  float* dAl = Kl + KLN;              // MP x TW dA  (later: Q^T, TW x QST)
  const int tid = threadIdx.x;
  const int lane = tid & 63, c = lane & 15, g = lane >> 4;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wave / G::WC, wc = wave - wr * G::WC;
  const float s2 = hyp[0], jit = hyp[2];
  const float* w = hyp + 4;
  const float* ls = hyp + 4 + D;

  stage_inducing(Z, ls, vmean, vstd, M, D, MP, Dq, ds, zs, zn, cm, vm, sm1, Kl);
  for (int m = tid; m < MP; m += blockDim.x) {
    qacc[m] = 0.f;
    for (int q = 0; q < G::WC; ++q) { dvma[q * MP + m] = 0.f; dsma[q * MP + m] = 0.f; }
  }
  rx2[tid] = 0.f;
  gxa[tid] = 0.f;
  float sumQ = 0.f, sumgv = 0.f, sumgm = 0.f;
  // persistent f32 accumulators of QX = sum_i Q_pi xs_i: tiles (pt, dt) dealt over the waves
  constexpr int MAXQT = (MB * NDT + 3) / 4;  // QX tiles (MB x NDT) dealt over 4 waves
  f32x4 qx[MAXQT];
#pragma unroll
  for (int u = 0; u < MAXQT; ++u) qx[u] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nch = (N + TW - 1) / TW;
#pragma unroll 1
  for (int t = blockIdx.x; t < nchunks; t += gridDim.x) {
    const int b = t / nch, ch = t - b * nch;
    const int i0 = ch * TW;
    const int nvalid = N - i0 < TW ? N - i0 : TW;
    const size_t col0 = (size_t)b * N + i0;
    const float* Xw = X + col0 * D;
    lds_barrier();
    stage_points(Xw, ls, nvalid, D, TW, Dq, ds, cm, xs, xn);
    for (int j = tid; j < TW; j += blockDim.x) {
      gmc[j] = j < nvalid ? gmean[col0 + j] : 0.f;
      gvc[j] = j < nvalid ? gvar[col0 + j] : 0.f;
    }
    lds_barrier();
    build_kzx<MB, TW>(zs, xs, zn, xn, M, nvalid, Dq, ds, s2, Kl);
    lds_barrier();
    f64x4 acc[G::RT][G::CT];
    if (!(GPK_VAR_SKIP & 1)) gemm_linv_k<MB>(Linv, Kl, M, acc);
    else {
#pragma unroll
      for (int j = 0; j < G::RT; ++j)
#pragma unroll
        for (int q = 0; q < G::CT; ++q) acc[j][q] = f64x4{0.1, 0.1, 0.1, 0.1};
    }
    // variance -> clamp mask (no gradient below the clamp)
#pragma unroll
    for (int q = 0; q < G::CT; ++q) {
      float vp = 0.f;
#pragma unroll
      for (int j = 0; j < G::RT; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int row = 16 * (wr + G::WR * j) + g + 4 * r;
          const float a32 = (float)acc[j][q][r];
          vp = __builtin_fmaf(a32 * a32, row < MP ? sm1[row] : 0.f, vp);
        }
      vp += __shfl_xor(vp, 16, 64);
      vp += __shfl_xor(vp, 32, 64);
      if (g == 0) redw[wr * TW + 16 * (wc * G::CT + q) + c] = vp;
    }
    lds_barrier();
    for (int col = tid; col < TW; col += blockDim.x) {
      float vv = 0.f;
      for (int q = 0; q < G::WR; ++q) vv += redw[q * TW + col];
      if (s2 + jit + vv < 1e-6f) gvc[col] = 0.f;  // clamp_min(1e-6): gradient masked
      sumgv += gvc[col];
      sumgm += gmc[col];
    }
    lds_barrier();
    // dA (fp32) -> LDS + workspace; partial sums for dvmean / dvstd
#pragma unroll
    for (int j = 0; j < G::RT; ++j) {
      const int rt = wr + G::WR * j;
      if (rt >= MB) continue;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = 16 * rt + g + 4 * r;
        float pm = 0.f, ps = 0.f;
#pragma unroll
        for (int q = 0; q < G::CT; ++q) {
          const int col = 16 * (wc * G::CT + q) + c;
          const float a32 = (float)acc[j][q][r];
          const float gm = gmc[col], gv = gvc[col];
          const float da = gm * vm[row] + 2.f * gv * sm1[row] * a32;
          dAl[row * TW + col] = da;
          if (row < M && col < nvalid && !(GPK_VAR_SKIP & 4)) wsdA[(size_t)row * BN + col0 + col] = da;
          pm = __builtin_fmaf(gm, a32, pm);
          ps = __builtin_fmaf(gv, a32 * a32, ps);
        }
#pragma unroll
        for (int off = 1; off < 16; off <<= 1) {
          pm += __shfl_xor(pm, off, 64);
          ps += __shfl_xor(ps, off, 64);
        }
        if (c == 0) {
          dvma[wc * MP + row] += pm;
          dsma[wc * MP + row] += ps;
        }
      }
    }
    // K_ZX -> workspace (row-major M x BN, coalesced along points)
    for (int e = tid; e < M * TW && !(GPK_VAR_SKIP & 4); e += blockDim.x) {
      const int p = e / TW, col = e - p * TW;
      if (col < nvalid) wsK[(size_t)p * BN + col0 + col] = Kl[p * TW + col];
    }
    lds_barrier();
    // dK = L^{-T} dA (fp64 MFMA): output rows p = the wave's row tiles, k = m >= p, in
    // k-blocks of 16 (k-order m = 16 kb + 4 g + u), next block's operands prefetched
    {
      int first = MB;
#pragma unroll
      for (int j = 0; j < G::RT; ++j) {
        const int rt = wr + G::WR * j;
        if (rt < MB) first = rt < first ? rt : first;
      }
#pragma unroll
      for (int j = 0; j < G::RT; ++j)
#pragma unroll
        for (int q = 0; q < G::CT; ++q) acc[j][q] = f64x4{0.0, 0.0, 0.0, 0.0};
      double an[G::RT][4];
      auto load_blk = [&](int kb, double (&dst)[G::RT][4]) {
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int m = 16 * kb + 4 * g + u;
          const double* row = Linv + (size_t)(m < M ? m : 0) * M;
#pragma unroll
          for (int j = 0; j < G::RT; ++j) {
            const int rt = wr + G::WR * j;
            const int p = 16 * rt + c;
            dst[j][u] = (rt < MB && kb >= rt && m < M && p < M) ? row[p] : 0.0;
          }
        }
      };
      load_blk(first, an);
      for (int kb = first; kb < MB && !(GPK_VAR_SKIP & 2); ++kb) {
        double a[G::RT][4];
#pragma unroll
        for (int j = 0; j < G::RT; ++j)
#pragma unroll
          for (int u = 0; u < 4; ++u) a[j][u] = an[j][u];
        if (kb + 1 < MB) load_blk(kb + 1, an);
        float bf[G::CT][4];
#pragma unroll
        for (int q = 0; q < G::CT; ++q)
#pragma unroll
          for (int u = 0; u < 4; ++u) bf[q][u] = dAl[(16 * kb + 4 * g + u) * TW + 16 * (wc * G::CT + q) + c];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
#pragma unroll
          for (int j = 0; j < G::RT; ++j) {
            const int rt = wr + G::WR * j;
            if (rt < MB && kb >= rt) {
#pragma unroll
              for (int q = 0; q < G::CT; ++q) acc[j][q] = mfma64(a[j][u], (double)bf[q][u], acc[j][q]);
            }
          }
        }
      }
    }
    lds_barrier();  // every wave is done reading dAl
    // Q = dK o K_ZX: Q^T -> LDS (over dAl), sum Q, r_i partials, and Q^T zs on f32 MFMA
    f32x4 xz[G::CT][NDT];
#pragma unroll
    for (int q = 0; q < G::CT; ++q)
#pragma unroll
      for (int dt = 0; dt < NDT; ++dt) xz[q][dt] = f32x4{0.f, 0.f, 0.f, 0.f};
    float rp[G::CT] = {};
#pragma unroll
    for (int j = 0; j < G::RT; ++j) {
      const int rt = wr + G::WR * j;
      if (rt >= MB || (GPK_VAR_SKIP & 8)) continue;
#pragma unroll
      for (int q = 0; q < G::CT; ++q) {
        const int col = 16 * (wc * G::CT + q) + c;
        float qv[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int row = 16 * rt + g + 4 * r;
          qv[r] = (float)acc[j][q][r] * Kl[row * TW + col];
          dAl[col * QST + row] = qv[r];
          sumQ += qv[r];
          rp[q] += qv[r];
        }
        // (Q^T zs)[col][d] += sum over this tile's rows (k-order g + 4r)
#pragma unroll
        for (int dt = 0; dt < NDT; ++dt) {
#pragma unroll
          for (int r = 0; r < 4; ++r)
            xz[q][dt] = mfma32(qv[r], zs[(16 * rt + g + 4 * r) * ds + 16 * dt + c], xz[q][dt]);
        }
      }
    }
#pragma unroll
    for (int q = 0; q < G::CT; ++q) {
      float v = rp[q];
      v += __shfl_xor(v, 16, 64);
      v += __shfl_xor(v, 32, 64);
      if (g == 0) redw[wr * TW + 16 * (wc * G::CT + q) + c] = v;
    }
    lds_barrier();  // Q^T complete, K_ZX no longer needed, r partials in redw
    // Q^T zs partials -> LDS (over Kl): [wr][col][d]; xz[q][dt][r] = (Q^T zs)[16ct + 4g + r][16dt + c]
#pragma unroll
    for (int q = 0; q < G::CT; ++q)
#pragma unroll
      for (int dt = 0; dt < NDT; ++dt) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int col = 16 * (wc * G::CT + q) + 4 * g + r;
          Kl[(wr * TW + col) * Dq + 16 * dt + c] = xz[q][dt][r];
        }
      }
    for (int col = tid; col < TW; col += blockDim.x) {
      float v = 0.f;
      for (int q = 0; q < G::WR; ++q) v += redw[q * TW + col];
      rcol[col] = v;
    }
    // QX += sum_i Q_pi xs_i (f32 MFMA, A = Q from Q^T, B = xs); tiles dealt over the waves
#pragma unroll
    for (int u = 0; u < MAXQT; ++u) {
      const int tq = wave + 4 * u;
      if (tq < MB * NDT && !(GPK_VAR_SKIP & 8)) {
        const int pt = tq / NDT, dt = tq - pt * NDT;
        for (int k = 0; k < TW / 4; ++k)
          qx[u] = mfma32(dAl[(4 * k + g) * QST + 16 * pt + c], xs[(4 * k + g) * ds + 16 * dt + c], qx[u]);
      }
    }
    for (int p = tid; p < MP && !(GPK_VAR_SKIP & 16); p += blockDim.x) {
      float v = 0.f;
      for (int i = 0; i < TW; ++i) v += dAl[i * QST + p];
      qacc[p] += v;
    }
    lds_barrier();  // Q^T zs partials and r complete
    // dX per point; sum_i r_i xs_i^2 per d (thread tid always sees d = tid % Dq)
    for (int e = tid; e < TW * Dq && !(GPK_VAR_SKIP & 32); e += blockDim.x) {
      const int col = e / Dq, d = e - col * Dq;
      float v = 0.f;
      for (int q = 0; q < G::WR; ++q) v += Kl[(q * TW + col) * Dq + d];
      const float xv = xs[col * ds + d];
      const float r = rcol[col];
      if (col < nvalid && d < D) {
        dX[(col0 + col) * D + d] = (v - xv * r) / ls[d] + gmc[col] * w[d];
        rx2[tid] += r * xv * xv;
        gxa[tid] += gmc[col] * xv;   // LinearMean: dw = l (sum gmean xs + cm sum gmean)
      }
    }
  }
  lds_barrier();
  // per-workgroup partials:
  //   [QX (M x D) | q (M) | dvm (M) | dsm (M) | rx2 (D) | sumQ | sumgv | gx (D) | sumgm]
  const int P = M * D + 3 * M + 2 * D + 3;
  float* po = wspart + (size_t)blockIdx.x * P;
#pragma unroll
  for (int u = 0; u < MAXQT; ++u) {
    const int tq = wave + 4 * u;
    if (tq < MB * NDT) {
      const int pt = tq / NDT, dt = tq - pt * NDT;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int p = 16 * pt + 4 * g + r, d = 16 * dt + c;
        if (p < M && d < D) po[p * D + d] = qx[u][r];
      }
    }
  }
  for (int m = tid; m < M; m += blockDim.x) {
    float a = 0.f, s = 0.f;
    for (int q = 0; q < G::WC; ++q) { a += dvma[q * MP + m]; s += dsma[q * MP + m]; }
    po[M * D + m] = qacc[m];
    po[M * D + M + m] = a;
    po[M * D + 2 * M + m] = s;
  }
  // sum r xs^2 and gmean xs over the threads that accumulated the same d (d = tid % Dq)
  for (int d = tid; d < D; d += blockDim.x) {
    float v = 0.f, u = 0.f;
    for (int t = d; t < 256; t += Dq) { v += rx2[t]; u += gxa[t]; }
    po[M * D + 3 * M + d] = v;
    po[M * D + 3 * M + D + 2 + d] = u;
  }
  sumQ = wave_sum(sumQ);
  if (lane == 0) redw[wave] = sumQ;
  lds_barrier();  // rx2 / gxa read, sumQ partials out
  rx2[tid] = sumgv;  // accumulated by the column threads
  gxa[tid] = sumgm;
  lds_barrier();
  if (tid == 0) {
    float v = 0.f, u = 0.f;
    for (int t = 0; t < 256; ++t) { v += rx2[t]; u += gxa[t]; }
    po[M * D + 3 * M + D] = (redw[0] + redw[1]) + (redw[2] + redw[3]);
    po[M * D + 3 * M + D + 1] = v;
    po[M * D + 3 * M + 2 * D + 2] = u;
  }
}

// ---------------------------------------------------------------------------
// Adjoint for M > 64 (cfg-3 shape M = 256) in the forward's register-resident layout
// (gpk_var_fwd_l_kernel), split in two persistent kernels over the same chunk list:
//   gpk_var_adja_l_kernel  wave w holds the L^{-1} ROW blocks of row tiles rA = w,
//                          rB = MB-1-w: K (Gram), A = L^{-1} K, the variance clamp mask,
//                          dA = gmean m + 2 gvar (s^2 - 1) A -> the workspace with K (for
//                          dL^{-1} = sum dA K^T, gpk_dlinv_kernel, and for the next kernel);
//                          dvmean / dvstd row sums.
//   gpk_var_adjk_l_kernel  wave w holds the L^{-1} COLUMN blocks of block rows pA = w,
//                          pB = MB-1-w: dK = L^{-T} dA from the chunk's dA / K tiles (LDS),
//                          Q = dK o K, q_p, r_i, Q^T zs, QX += Q xs, dX.
// (Both layouts at once would need 272 of the 256 registers; one fused kernel streaming the
// column blocks from L2 spilled heavily.) k-order of every contraction over inducing
// points: m = g + 4u, the f64 C layout, so accumulator tiles are the next product's B
// operands directly; the Gram feeds the zs rows in the order pi(c) = (c >> 2) + 4 (c & 3)
// to land in it. LDS tiles of K / dA: one b128 per lane, (rt, ct) tile at ((rt*2+ct)*64 +
// lane)*4, element u <-> row 16 rt + g + 4u, point 16 ct + c.
// Both kernels write disjoint fields of the same per-workgroup partial rows (the same grid).
// ---------------------------------------------------------------------------
GPK_DEVICE int pi16(int c) { return (c >> 2) + 4 * (c & 3); }

// Buffer descriptors for the (M x BN) workspace arrays: a 32-bit lane offset plus a
// wave-uniform SGPR offset per row step, where flat addressing pinned a 64-bit address per
// load in flight (the host keeps M BN 4 < 2^31 on this path).
GPK_DEVICE __amdgpu_buffer_rsrc_t ws_rsrc(const float* p, long long elems) {
  return __builtin_amdgcn_make_buffer_rsrc((void*)p, 0, (int)(elems * 4), 0x00020000);
}
GPK_DEVICE float buf_ld(__amdgpu_buffer_rsrc_t r, int voff, int soff) {
  return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, voff, soff, 0));
}
GPK_DEVICE void buf_st(float v, __amdgpu_buffer_rsrc_t r, int voff, int soff) {
  __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, v), r, voff, soff, 0);
}

template <int MB, int DQ>
struct LAdjGeo {
  static constexpr int NWV = (MB + 1) / 2, NT = 64 * NWV, MP = 16 * MB, DS = DQ + 2;
  static constexpr int NPASS = (LTW * 16 + NT - 1) / NT, DV = DQ / 16, NDT = DQ / 16;
  // gpk_var_adja_l_kernel
  static constexpr int aKl = 0;                          // MP x LTW
  static constexpr int aRed = aKl + MP * LTW;            // NWV x LTW
  static constexpr int aZs = aRed + NWV * LTW;           // MP x DS
  static constexpr int aZn = aZs + MP * DS;
  static constexpr int aVm = aZn + MP;
  static constexpr int aSm1 = aVm + MP;
  static constexpr int aCm = aSm1 + MP;                  // DQ
  static constexpr int aRows = aCm + DQ;                 // 2 x MP: dvm | dsm
  static constexpr int aXs = aRows + 2 * MP;             // LTW x DS
  static constexpr int aXn = aXs + LTW * DS;             // LTW
  static constexpr int aGm = aXn + LTW;                  // 2 x LTW (chunk parity)
  static constexpr int aGv = aGm + 2 * LTW;              // 2 x LTW
  static constexpr int a_total = aGv + 2 * LTW;
  // gpk_var_adjk_l_kernel
  static constexpr int kKl = 0;                          // MP x LTW
  static constexpr int kdA = kKl + MP * LTW;             // MP x LTW
  static constexpr int kXz = kdA + MP * LTW;             // NWV x LTW x DQ  Q^T zs partials
  static constexpr int kRed = kXz + NWV * LTW * DQ;      // NWV x LTW       r partials
  static constexpr int kZs = kRed + NWV * LTW;           // MP x DS
  static constexpr int kZn = kZs + MP * DS;
  static constexpr int kVm = kZn + MP;
  static constexpr int kSm1 = kVm + MP;
  static constexpr int kCm = kSm1 + MP;                  // DQ
  static constexpr int kQ = kCm + DQ;                    // MP  q_p
  static constexpr int kScr = kQ + MP;                   // NWV x 320 transpose scratch
  static constexpr int kXs = kScr + NWV * 320;           // 2 x LTW x DS (chunk parity)
  static constexpr int kGm = kXs + 2 * LTW * DS;         // 2 x LTW
  static constexpr int kMisc = kGm + 2 * LTW;            // 2 NT + NWV
  static constexpr int k_total = kMisc + 2 * NT + NWV;
  static constexpr bool fits = (size_t)a_total * 4 <= 160 * 1024 && (size_t)k_total * 4 <= 160 * 1024;
};

// dK of the wave with pA = RA from its column-block registers: slots 0..NA-1 are blocks
// (rt = RA + s, RA), the rest (rt = RB + s - NA, RB); B operands dA[rt] from LDS.
template <int MB, int RA>
GPK_DEVICE void lcol_gemm(const double (&Lc)[MB + 1][4], const float* dAl, int lane,
                          f64x4 (&dKa)[2], f64x4 (&dKb)[2]) {
  constexpr int RB = MB - 1 - RA;
  constexpr int NA = MB - RA;
  constexpr int NS = RB == RA ? NA : MB + 1;
  f64x4 acc[2] = {f64x4{0.0, 0.0, 0.0, 0.0}, f64x4{0.0, 0.0, 0.0, 0.0}};
  f32x4 k0 = *(const f32x4*)(dAl + ((RA * 2 + 0) * 64 + lane) * 4);
  f32x4 k1 = *(const f32x4*)(dAl + ((RA * 2 + 1) * 64 + lane) * 4);
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    if (s == NA) {
      dKa[0] = acc[0];
      dKa[1] = acc[1];
      acc[0] = acc[1] = f64x4{0.0, 0.0, 0.0, 0.0};
    }
    f32x4 n0 = k0, n1 = k1;
    if (s + 1 < NS) {
      const int rtn = s + 1 < NA ? RA + s + 1 : RB + (s + 1 - NA);
      n0 = *(const f32x4*)(dAl + ((rtn * 2 + 0) * 64 + lane) * 4);
      n1 = *(const f32x4*)(dAl + ((rtn * 2 + 1) * 64 + lane) * 4);
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      acc[0] = mfma64(Lc[s][u], (double)k0[u], acc[0]);
      acc[1] = mfma64(Lc[s][u], (double)k1[u], acc[1]);
    }
    k0 = n0;
    k1 = n1;
    __builtin_amdgcn_sched_barrier(0);
  }
  if (RB == RA) {
    dKa[0] = acc[0];
    dKa[1] = acc[1];
    dKb[0] = dKb[1] = f64x4{0.0, 0.0, 0.0, 0.0};
  } else {
    dKb[0] = acc[0];
    dKb[1] = acc[1];
  }
}
template <int MB, int RA>
GPK_DEVICE void lcol_gemm_for(int wave, const double (&Lc)[MB + 1][4], const float* dAl, int lane,
                              f64x4 (&dKa)[2], f64x4 (&dKb)[2]) {
  if constexpr (RA < (MB + 1) / 2) {
    if (wave == RA) lcol_gemm<MB, RA>(Lc, dAl, lane, dKa, dKb);
    else lcol_gemm_for<MB, RA + 1>(wave, Lc, dAl, lane, dKa, dKb);
  }
}

// The chunk's points (16 threads per point, dims sub + 16 v) -> xs (and |xs|^2 -> xn if given).
template <int NPASS, int DV, int NT, int DS>
GPK_DEVICE void lstage_points(const float (&xr)[NPASS][DV], const float (&lsr)[DV], const float (&cmr)[DV],
                              int D, int nvalid, float* xs, float* xn) {
  const int tid = threadIdx.x, sub = tid & 15;
#pragma unroll
  for (int q = 0; q < NPASS; ++q) {
    const int j = (tid >> 4) + q * (NT / 16);
    float nrm = 0.f;
    const bool okj = j < nvalid;
#pragma unroll
    for (int v = 0; v < DV; ++v) {
      const int d = sub + 16 * v;
      const float xv = (okj && d < D) ? xr[q][v] / lsr[v] - cmr[v] : 0.f;
      nrm = __builtin_fmaf(xv, xv, nrm);
      if (j < LTW) xs[j * DS + d] = xv;
    }
    if (xn != nullptr) {
      nrm = row16_sum_f(nrm);
      if (sub == 0 && j < LTW) xn[j] = nrm;
    }
  }
}
template <int NPASS, int DV, int NT>
GPK_DEVICE void lload_points(const float* X, int t, int nchunks, int nch, int N, int D, float (&xr)[NPASS][DV]) {
  const int tid = threadIdx.x, sub = tid & 15;
  const int b = t / nch, i0 = (t - b * nch) * LTW;
#pragma unroll
  for (int q = 0; q < NPASS; ++q) {
    const int j = (tid >> 4) + q * (NT / 16), i = i0 + j;
    const bool ok = t < nchunks && j < LTW && i < N;
#pragma unroll
    for (int v = 0; v < DV; ++v) {
      const int d = sub + 16 * v;
      const bool okd = ok && d < D;
      const float x = X[okd ? ((size_t)b * N + i) * D + d : 0];
      xr[q][v] = okd ? x : 0.f;
    }
  }
}

template <int MB, int DQ>
__global__ void __launch_bounds__(64 * ((MB + 1) / 2), 2)
gpk_var_adja_l_kernel(const float* __restrict__ X, const float* __restrict__ Z,
                      const double* __restrict__ Linv, const float* __restrict__ vmean,
                      const float* __restrict__ vstd, const float* __restrict__ hyp,
                      const float* __restrict__ gmean, const float* __restrict__ gvar, int N, int M,
                      int D, int nchunks, long long BN, float* __restrict__ wsdA,
                      float* __restrict__ wsK, float* __restrict__ wspart) {
  using G = LAdjGeo<MB, DQ>;
  constexpr int NWV = G::NWV, NT = G::NT, DS = G::DS, NPASS = G::NPASS, DV = G::DV;
  extern __shared__ __attribute__((aligned(16))) float vsm[];
  const int tid = threadIdx.x, lane = tid & 63, c = lane & 15, g = lane >> 4, sub = tid & 15;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int rA = wave, rB = MB - 1 - wave;
  const bool two = rB != rA;
  const float s2 = hyp[0], jit = hyp[2];
  const float* ls = hyp + 4 + D;
  const int nch = (N + LTW - 1) / LTW;

  // L^{-1} row blocks, k-order g + 4u: Lr[s][u] = L^{-1}[16 rt + c][16 kb + g + 4u]
  double Lr[MB + 1][4];
  {
    const bool full = (M & 15) == 0;
#pragma unroll
    for (int s = 0; s <= MB; ++s) {
      const bool isA = s <= rA;
      const int rt = isA ? rA : rB, kb = isA ? s : s - rA - 1;
      const bool ok = isA || two;
      const int m = 16 * rt + c;
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int p = 16 * kb + g + 4 * u;
        const bool in = ok && (full || (m < M && p < M));
        const double v = Linv[in ? (size_t)m * M + p : 0];
        Lr[s][u] = in ? v : 0.0;
      }
      if ((s & 3) == 3) __builtin_amdgcn_sched_barrier(0);
    }
  }
  float lsr[DV];
#pragma unroll
  for (int v = 0; v < DV; ++v) lsr[v] = ls[sub + 16 * v < D ? sub + 16 * v : 0];
  float xr[NPASS][DV];
  lload_points<NPASS, DV, NT>(X, blockIdx.x, nchunks, nch, N, D, xr);
  stage_inducing(Z, ls, vmean, vstd, M, D, G::MP, DQ, DS, vsm + G::aZs, vsm + G::aZn, vsm + G::aCm,
                 vsm + G::aVm, vsm + G::aSm1, vsm + G::aKl);
  for (int e = tid; e < 2 * G::MP; e += NT) vsm[G::aRows + e] = 0.f;
  lds_barrier();
  float cmr[DV];
#pragma unroll
  for (int v = 0; v < DV; ++v) cmr[v] = vsm[G::aCm + sub + 16 * v];
  float sumgv = 0.f;
  int par = 0;
  const __amdgpu_buffer_rsrc_t rdA = ws_rsrc(wsdA, (long long)M * BN), rK = ws_rsrc(wsK, (long long)M * BN);

  for (int t = blockIdx.x; t < nchunks; t += gridDim.x, par ^= 1) {
    const int b = t / nch, i0 = (t - b * nch) * LTW;
    const int nvalid = N - i0 < LTW ? N - i0 : LTW;
    const long long col0 = (long long)b * N + i0;
    float* sm = (float*)fresh_lds(vsm);
    float* Kl = sm + G::aKl;
    float* red = sm + G::aRed;
    const float* zs = sm + G::aZs;
    const float* zn = sm + G::aZn;
    const float* vm = sm + G::aVm;
    const float* sm1 = sm + G::aSm1;
    float* rows = sm + G::aRows;
    float* xs = sm + G::aXs;
    float* xn = sm + G::aXn;
    float* gmc = sm + G::aGm + par * LTW;
    float* gvc = sm + G::aGv + par * LTW;
    lstage_points<NPASS, DV, NT, DS>(xr, lsr, cmr, D, nvalid, xs, xn);
    if (tid < LTW) {
      const bool ok = tid < nvalid;
      const float gm = gmean[ok ? col0 + tid : 0], gv = gvar[ok ? col0 + tid : 0];
      gmc[tid] = ok ? gm : 0.f;
      gvc[tid] = ok ? gv : 0.f;
    }
    lds_barrier();
    // K tiles of the wave's rows (rows fed in the order pi: acc row g + 4r)
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int rt = h == 0 ? rA : rB;
      if (h == 1 && !two) break;
#pragma unroll
      for (int ct = 0; ct < 2; ++ct) {
        const float* za = zs + (16 * rt + pi16(c)) * DS + g;
        const float* xb = xs + (16 * ct + c) * DS + g;
        f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int k = 0; k < DQ / 4; ++k) acc = mfma32(za[4 * k], xb[4 * k], acc);
        const int col = 16 * ct + c;
        const float xnc = xn[col];
        f32x4 o;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int p = 16 * rt + g + 4 * r;
          float dist = zn[p] + xnc - 2.f * acc[r];
          dist = dist < 0.f ? 0.f : dist;
          o[r] = (p < M && col < nvalid) ? s2 * __builtin_amdgcn_exp2f(kNHalfLog2e * dist) : 0.f;
        }
        *(f32x4*)(Kl + ((rt * 2 + ct) * 64 + lane) * 4) = o;
      }
    }
    if (t + (int)gridDim.x < nchunks) lload_points<NPASS, DV, NT>(X, t + gridDim.x, nchunks, nch, N, D, xr);
    lds_barrier();
    f32x4 Af[2][2];
    {
      f64x4 aA[2], aB[2];
      lreg_gemm_for<MB, 0>(wave, Lr, Kl, lane, aA, aB);
#pragma unroll
      for (int ct = 0; ct < 2; ++ct)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          Af[0][ct][r] = (float)aA[ct][r];
          Af[1][ct][r] = (float)aB[ct][r];
        }
    }
#pragma unroll
    for (int ct = 0; ct < 2; ++ct) {
      float vp = 0.f;
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        if (h == 1 && !two) break;
        const int rt = h == 0 ? rA : rB;
#pragma unroll
        for (int r = 0; r < 4; ++r) vp = __builtin_fmaf(Af[h][ct][r] * Af[h][ct][r], sm1[16 * rt + g + 4 * r], vp);
      }
      vp += __shfl_xor(vp, 16, 64);
      vp += __shfl_xor(vp, 32, 64);
      if (g == 0) red[wave * LTW + 16 * ct + c] = vp;
    }
    lds_barrier();
    // clamp mask (the same fixed-order total on every wave), dA, row sums, workspace
    float gmq[2], gvq[2];
#pragma unroll
    for (int ct = 0; ct < 2; ++ct) {
      const int col = 16 * ct + c;
      float vv = 0.f;
#pragma unroll
      for (int q = 0; q < NWV; ++q) vv += red[q * LTW + col];
      gmq[ct] = gmc[col];
      gvq[ct] = (s2 + jit + vv < 1e-6f) ? 0.f : gvc[col];   // clamp_min(1e-6): gradient masked
      if (wave == 0 && g == 0) sumgv += gvq[ct];
    }
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      if (h == 1 && !two) break;
      const int rt = h == 0 ? rA : rB;
      const int voff = (int)(((long long)(16 * rt + g) * BN + col0 + c) * 4);
#pragma unroll
      for (int ct = 0; ct < 2; ++ct) {
        const f32x4 kv = *(const f32x4*)(Kl + ((rt * 2 + ct) * 64 + lane) * 4);
        const bool okc = 16 * ct + c < nvalid;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int p = 16 * rt + g + 4 * r;
          const float da = gmq[ct] * vm[p] + 2.f * gvq[ct] * sm1[p] * Af[h][ct][r];
          if (p < M && okc) {
            buf_st(da, rdA, voff + 64 * ct, (int)(16 * r * BN));
            buf_st(kv[r], rK, voff + 64 * ct, (int)(16 * r * BN));
          }
        }
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float pm = 0.f, ps = 0.f;
#pragma unroll
        for (int ct = 0; ct < 2; ++ct) {
          pm = __builtin_fmaf(gmq[ct], Af[h][ct][r], pm);
          ps = __builtin_fmaf(gvq[ct], Af[h][ct][r] * Af[h][ct][r], ps);
        }
        pm = row16_sum_f(pm);
        ps = row16_sum_f(ps);
        if (c == 0) {
          const int p = 16 * rt + g + 4 * r;
          rows[p] += pm;
          rows[G::MP + p] += ps;
        }
      }
    }
  }
  lds_barrier();
  // partial fields of this kernel: dvm (M) | dsm (M) | sumgv
  const int P = M * D + 3 * M + 2 * D + 3;
  float* po = wspart + (size_t)blockIdx.x * P;
  for (int m = tid; m < M; m += NT) {
    po[M * D + M + m] = vsm[G::aRows + m];
    po[M * D + 2 * M + m] = vsm[G::aRows + G::MP + m];
  }
  if (wave == 0) {
    const float v = row16_sum_f(sumgv);   // accumulated on lanes 0..15 only
    if (lane == 0) po[M * D + 3 * M + D + 1] = v;
  }
}

template <int MB, int DQ>
__global__ void __launch_bounds__(64 * ((MB + 1) / 2), 2)
gpk_var_adjk_l_kernel(const float* __restrict__ X, const float* __restrict__ Z,
                      const double* __restrict__ Linv, const float* __restrict__ vmean,
                      const float* __restrict__ vstd, const float* __restrict__ hyp,
                      const float* __restrict__ gmean, int N, int M, int D, int nchunks,
                      long long BN, const float* __restrict__ wsdA, const float* __restrict__ wsK,
                      float* __restrict__ wspart, float* __restrict__ dX) {
  using G = LAdjGeo<MB, DQ>;
  constexpr int NWV = G::NWV, NT = G::NT, DS = G::DS, NPASS = G::NPASS, DV = G::DV, NDT = G::NDT;
  constexpr int NLD = G::MP * LTW / NT;   // workspace elements per thread per array
  extern __shared__ __attribute__((aligned(16))) float vsm[];
  const int tid = threadIdx.x, lane = tid & 63, c = lane & 15, g = lane >> 4, sub = tid & 15;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int pA = wave, pB = MB - 1 - wave;
  const bool two = pB != pA;
  const float* w = hyp + 4;
  const float* ls = hyp + 4 + D;
  const int nch = (N + LTW - 1) / LTW;

  // L^{-1} column blocks, k-order g + 4u: slot s < MB - pA: (rt = pA + s, P = pA), then
  // (rt = pB + s', P = pB);  Lc[s][u] = L^{-1}[16 rt + g + 4u][16 P + c]
  double Lc[MB + 1][4];
  {
    const bool full = (M & 15) == 0;
    const int NA = MB - pA;
#pragma unroll
    for (int s = 0; s <= MB; ++s) {
      const bool isA = s < NA;
      const int P = isA ? pA : pB, rt = isA ? pA + s : pB + (s - NA);
      const bool ok = isA || (two && rt < MB);
      const int col = 16 * P + c;
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int row = 16 * rt + g + 4 * u;
        const bool in = ok && (full || (row < M && col < M));
        const double v = Linv[in ? (size_t)row * M + col : 0];
        Lc[s][u] = in ? v : 0.0;
      }
      if ((s & 3) == 3) __builtin_amdgcn_sched_barrier(0);
    }
  }
  float lsr[DV];
#pragma unroll
  for (int v = 0; v < DV; ++v) lsr[v] = ls[sub + 16 * v < D ? sub + 16 * v : 0];
  float xr[NPASS][DV];
  lload_points<NPASS, DV, NT>(X, blockIdx.x, nchunks, nch, N, D, xr);
  stage_inducing(Z, ls, vmean, vstd, M, D, G::MP, DQ, DS, vsm + G::kZs, vsm + G::kZn, vsm + G::kCm,
                 vsm + G::kVm, vsm + G::kSm1, vsm + G::kKl);
  for (int e = tid; e < G::MP; e += NT) vsm[G::kQ + e] = 0.f;
  lds_barrier();
  float cmr[DV];
#pragma unroll
  for (int v = 0; v < DV; ++v) cmr[v] = vsm[G::kCm + sub + 16 * v];
  const __amdgpu_buffer_rsrc_t rdA = ws_rsrc(wsdA, (long long)M * BN), rK = ws_rsrc(wsK, (long long)M * BN);
  const int dd = tid % DQ;   // the dX phase's dim for this thread (NT % DQ == 0)
  const float il_dd = dd < D ? 1.f / ls[dd < D ? dd : 0] : 0.f;
  const float w_dd = dd < D ? w[dd < D ? dd : 0] : 0.f;
  float rx2 = 0.f, gxa = 0.f, sumQ = 0.f, sumgm = 0.f;
  f32x4 qx[2][NDT];   // QX rows of the wave's blocks (p = 16 blk + 4g + r, d = 16 dt + c)
#pragma unroll
  for (int h = 0; h < 2; ++h)
#pragma unroll
    for (int dt = 0; dt < NDT; ++dt) qx[h][dt] = f32x4{0.f, 0.f, 0.f, 0.f};
  int par = 0;

  for (int t = blockIdx.x; t < nchunks; t += gridDim.x, par ^= 1) {
    const int b = t / nch, i0 = (t - b * nch) * LTW;
    const int nvalid = N - i0 < LTW ? N - i0 : LTW;
    const long long col0 = (long long)b * N + i0;
    float* sm = (float*)fresh_lds(vsm);
    float* Kl = sm + G::kKl;
    float* dAl = sm + G::kdA;
    float* xzl = sm + G::kXz;
    float* red = sm + G::kRed;
    const float* zs = sm + G::kZs;
    float* qrow = sm + G::kQ;
    float* scr = sm + G::kScr + wave * 320;
    float* xs = sm + G::kXs + par * LTW * DS;
    float* gmc = sm + G::kGm + par * LTW;
    // ---- the chunk's dA / K rows (coalesced along points) -> LDS tiles; points; gmean
    {
      // thread -> point j = tid % 32 of rows m = tid / 32 + q NT / 32: one lane offset, the
      // row step in the SGPR offset (rows >= M read past the array: zero by the bounds check)
      // (two halves: 16 values per array in flight at most)
      constexpr int NH = NLD > 8 ? 2 : 1, NQ = NLD / NH;
      const int j = tid & (LTW - 1);
      const int voff = (int)(((long long)(tid / LTW) * BN + col0 + j) * 4);
#pragma unroll
      for (int hh = 0; hh < NH; ++hh) {
        float va[NQ], vk[NQ];
#pragma unroll
        for (int qq = 0; qq < NQ; ++qq) {
          const int so = (int)((long long)(hh * NQ + qq) * (NT / LTW) * BN * 4);
          va[qq] = buf_ld(rdA, voff, so);
          vk[qq] = buf_ld(rK, voff, so);
        }
#pragma unroll
        for (int qq = 0; qq < NQ; ++qq) {
          const int q = hh * NQ + qq;
          const int m = tid / LTW + q * (NT / LTW);
          const bool ok = m < M && j < nvalid;
          const int rt = m >> 4, mm = m & 15, ct = j >> 4, cc = j & 15;
          const int o = ((rt * 2 + ct) * 64 + (mm & 3) * 16 + cc) * 4 + (mm >> 2);
          dAl[o] = ok ? va[qq] : 0.f;
          Kl[o] = ok ? vk[qq] : 0.f;
        }
      }
    }
    lstage_points<NPASS, DV, NT, DS>(xr, lsr, cmr, D, nvalid, xs, nullptr);
    if (tid < LTW) {
      const bool ok = tid < nvalid;
      const float gm = gmean[ok ? col0 + tid : 0];
      gmc[tid] = ok ? gm : 0.f;
      sumgm += ok ? gm : 0.f;
    }
    if (t + (int)gridDim.x < nchunks) lload_points<NPASS, DV, NT>(X, t + gridDim.x, nchunks, nch, N, D, xr);
    lds_barrier();
    // ---- dK = L^{-T} dA on the wave's block rows; Q = dK o K
    f32x4 Qt[2][2];
    {
      f64x4 dK[2][2];
      lcol_gemm_for<MB, 0>(wave, Lc, dAl, lane, dK[0], dK[1]);
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int rt = h == 0 ? pA : pB;
#pragma unroll
        for (int ct = 0; ct < 2; ++ct) {
          const f32x4 kv = *(const f32x4*)(Kl + ((rt * 2 + ct) * 64 + lane) * 4);
#pragma unroll
          for (int r = 0; r < 4; ++r) Qt[h][ct][r] = (h == 1 && !two) ? 0.f : (float)dK[h][ct][r] * kv[r];
        }
      }
    }
    // q_p row sums (rows owned by this wave), r_i partials, sum Q
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      if (h == 1 && !two) break;
      const int rt = h == 0 ? pA : pB;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float v = row16_sum_f(Qt[h][0][r] + Qt[h][1][r]);
        if (c == 0) qrow[16 * rt + g + 4 * r] += v;
      }
    }
#pragma unroll
    for (int ct = 0; ct < 2; ++ct) {
      float v = 0.f;
#pragma unroll
      for (int h = 0; h < 2; ++h) v += (Qt[h][ct][0] + Qt[h][ct][1]) + (Qt[h][ct][2] + Qt[h][ct][3]);
      sumQ += v;
      v += __shfl_xor(v, 16, 64);
      v += __shfl_xor(v, 32, 64);
      if (g == 0) red[wave * LTW + 16 * ct + c] = v;
    }
    // Q^T zs (k = p, rows g + 4r): xz[ct][dt][r'] = sum_p Q[p][16 ct + 4g + r'] zs[p][16 dt + c]
    {
      f32x4 xz[2][NDT];
#pragma unroll
      for (int ct = 0; ct < 2; ++ct)
#pragma unroll
        for (int dt = 0; dt < NDT; ++dt) xz[ct][dt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        if (h == 1 && !two) break;
        const int rt = h == 0 ? pA : pB;
#pragma unroll
        for (int r = 0; r < 4; ++r)
#pragma unroll
          for (int dt = 0; dt < NDT; ++dt) {
            const float zb = zs[(16 * rt + g + 4 * r) * DS + 16 * dt + c];
#pragma unroll
            for (int ct = 0; ct < 2; ++ct) xz[ct][dt] = mfma32(Qt[h][ct][r], zb, xz[ct][dt]);
          }
      }
#pragma unroll
      for (int ct = 0; ct < 2; ++ct)
#pragma unroll
        for (int dt = 0; dt < NDT; ++dt)
#pragma unroll
          for (int r = 0; r < 4; ++r)
            xzl[(wave * LTW + 16 * ct + 4 * g + r) * DQ + 16 * dt + c] = xz[ct][dt][r];
    }
    // QX_p += sum_i Q_pi xs_i: each Q tile transposed through the wave's scratch (k = point)
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      if (h == 1 && !two) break;
#pragma unroll
      for (int ct = 0; ct < 2; ++ct) {
#pragma unroll
        for (int r = 0; r < 4; ++r) scr[lane * 5 + r] = Qt[h][ct][r];
        adj_lds_order();
        float aq[4];
#pragma unroll
        for (int s = 0; s < 4; ++s) aq[s] = scr[((c & 3) * 16 + 4 * s + g) * 5 + (c >> 2)];
        adj_lds_order();   // the next tile overwrites scr
#pragma unroll
        for (int dt = 0; dt < NDT; ++dt)
#pragma unroll
          for (int s = 0; s < 4; ++s)
            qx[h][dt] = mfma32(aq[s], xs[(16 * ct + 4 * s + g) * DS + 16 * dt + c], qx[h][dt]);
      }
    }
    lds_barrier();   // Q^T zs and r partials complete
    // ---- dX_i = ((Q^T zs)_i - xs_i r_i) / l + gmean_i w; sum_i r_i xs_i^2, gmean_i xs_i
    for (int e = tid; e < LTW * DQ; e += NT) {
      const int col = e / DQ;
      float v = 0.f, r = 0.f;
#pragma unroll
      for (int q = 0; q < NWV; ++q) {
        v += xzl[(q * LTW + col) * DQ + dd];
        r += red[q * LTW + col];
      }
      const float xv = xs[col * DS + dd];
      if (col < nvalid && dd < D) {
        dX[(col0 + col) * D + dd] = (v - xv * r) * il_dd + gmc[col] * w_dd;
        rx2 = __builtin_fmaf(r * xv, xv, rx2);
        gxa = __builtin_fmaf(gmc[col], xv, gxa);
      }
    }
  }
  lds_barrier();
  // partial fields of this kernel: QX (M x D) | q (M) | rx2 (D) | sumQ | gx (D) | sumgm
  const int P = M * D + 3 * M + 2 * D + 3;
  float* po = wspart + (size_t)blockIdx.x * P;
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    if (h == 1 && !two) break;
    const int rt = h == 0 ? pA : pB;
#pragma unroll
    for (int dt = 0; dt < NDT; ++dt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int p = 16 * rt + 4 * g + r, d = 16 * dt + c;
        if (p < M && d < D) po[p * D + d] = qx[h][dt][r];
      }
  }
  for (int m = tid; m < M; m += NT) po[M * D + m] = vsm[G::kQ + m];
  float* misc = vsm + G::kMisc;
  misc[tid] = rx2;
  misc[NT + tid] = gxa;
  sumQ = wave_sum(sumQ);
  if (lane == 0) misc[2 * NT + wave] = sumQ;
  lds_barrier();
  for (int d = tid; d < D; d += NT) {
    float v = 0.f, u = 0.f;
    for (int q = d; q < NT; q += DQ) { v += misc[q]; u += misc[NT + q]; }
    po[M * D + 3 * M + d] = v;
    po[M * D + 3 * M + D + 2 + d] = u;
  }
  if (tid == 0) {
    float v = 0.f;
    for (int q = 0; q < NWV; ++q) v += misc[2 * NT + q];
    po[M * D + 3 * M + D] = v;
  }
  if (wave == 0) {
    const float u = wave_sum(sumgm);   // accumulated on lanes 0..LTW-1
    if (lane == 0) po[M * D + 3 * M + 2 * D + 2] = u;
  }
}


// ---------------------------------------------------------------------------
// dL^{-1} of the saved-state adjoint (M > 64), from the forward's A instead of a dA / K_ZX
// workspace: with dA = gmean m + 2 gvar (s^2 - 1) A,
//   dL^{-1} = sum_i dA_i K_i^T = m u^T + 2 diag(s^2 - 1) G',   u = sum_i gmean_i K_i,
//   G' = sum_i gvar_i A_i K_i^T            (lower part only: dL^{-1} is lower triangular)
// (the same arithmetic as the reference's fp32 dA: A is the saved fp32 A, products exact on f32
// MFMA, no L^{-1} product -- a form through G = K diag(gvar) K^T would multiply G's rounding by
// L^{-1}'s conditioning). gpk_var_kgram_l_kernel: per workgroup over its chunks, wave w owns the
// G' tile rows I = w and MB-1-w (MB + 1 lower tiles for every wave, f32 MFMA accumulators). Per
// chunk: the saved A block -> LDS rows [p][point], K_ZX recomputed (f32 MFMA Gram, fp32 exp) ->
// LDS rows, gvar masked by the saved clamp mask; each tile product is 8 mfma_f32_16x16x4_f32
// with both operands read as two b128 per lane (the k index of step j on lane (c, g) is point
// 8 g + j). Partials gpart[wg] = G' tiles (acc layout) | u, summed in a fixed order afterwards
// (gpk_var_red_kernel), then var_gdl_elem (extra blocks of gpk_var_fin_kernel) forms dL^{-1}
// elementwise.
// ---------------------------------------------------------------------------
#ifndef GPK_KGRAM_SPL
#define GPK_KGRAM_SPL 2   // waves per G' tile-row pair (1: 8 waves x 17 tiles, 209 VGPRs, 2 waves/SIMD)
#endif
template <int MB, int DQ, int SPL = GPK_KGRAM_SPL>
struct LGramGeo {
  static constexpr int NWV = SPL * ((MB + 1) / 2), NT = 64 * NWV, MP = 16 * MB, DS = DQ + 2;
  static constexpr int HS = (MB + 1 + SPL - 1) / SPL;      // G' slots per wave (of the pair's MB + 1)
  static constexpr int NPASS = (LTW * 16 + NT - 1) / NT, DV = DQ / 16;
  static constexpr int KS = LTW + 4;                       // row stride of the A / K blocks (floats)
  static constexpr int NTILE = MB * (MB + 1) / 2;
  static constexpr int PG = NTILE * 256 + MP;              // partial row: tiles | u
  static constexpr int oA = 0;                             // MP x KS  A[p][point]
  static constexpr int oK = oA + MP * KS;                  // MP x KS  K[p][point]
  static constexpr int oZs = oK + MP * KS;                 // MP x DS
  static constexpr int oZn = oZs + MP * DS;
  static constexpr int oVm = oZn + MP;
  static constexpr int oSm1 = oVm + MP;
  static constexpr int oCm = oSm1 + MP;                    // DQ
  static constexpr int oXs = oCm + DQ;                     // LTW x DS
  static constexpr int oXn = oXs + LTW * DS;               // LTW
  static constexpr int oGm = oXn + LTW;                    // LTW
  static constexpr int oGv = oGm + LTW;                    // LTW
  static constexpr int total = oGv + LTW;
};

template <int MB, int DQ>
__global__ void __launch_bounds__(64 * GPK_KGRAM_SPL * ((MB + 1) / 2), GPK_KGRAM_SPL == 1 ? 2 : 4)
gpk_var_kgram_l_kernel(const float* __restrict__ X, const float* __restrict__ Z,
                       const float* __restrict__ vmean, const float* __restrict__ vstd,
                       const float* __restrict__ hyp, const float* __restrict__ gmean,
                       const float* __restrict__ gvar, const float* __restrict__ saved, int N, int M,
                       int D, int nchunks, float* __restrict__ gpart) {
  using G = LGramGeo<MB, DQ>;
  using SV = LSaved<MB>;
  constexpr int NT = G::NT, DS = G::DS, NPASS = G::NPASS, DV = G::DV, KS = G::KS;
  constexpr int SPL = GPK_KGRAM_SPL, HS = G::HS;
  constexpr int NU = SV::tiles / 4;                 // f32x4 units of A per chunk
  static_assert(NU % NT == 0, "A block: whole passes");
  extern __shared__ __attribute__((aligned(16))) float vsm[];
  const int tid = threadIdx.x, lane = tid & 63, c = lane & 15, g = lane >> 4, sub = tid & 15;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  // the tile-row pair (IA, IB) of this wave and its share of the pair's slots
  // (slot s <= IA: tile (IA, s); slot IA + 1 + s': tile (IB, s')), [s0, s0 + HS)
  const int pr = wave / SPL, hf = wave - pr * SPL;
  const int IA = pr, IB = MB - 1 - pr;
  const bool two = IB != IA;
  const int nslot = two ? MB + 1 : IA + 1, s0 = hf * HS;
  const float s2 = hyp[0];
  const float* ls = hyp + 4 + D;
  const int nch = (N + LTW - 1) / LTW;
  float lsr[DV];
#pragma unroll
  for (int v = 0; v < DV; ++v) lsr[v] = ls[sub + 16 * v < D ? sub + 16 * v : 0];
  float xr[NPASS][DV];
  lload_points<NPASS, DV, NT>(X, blockIdx.x, nchunks, nch, N, D, xr);
  stage_inducing(Z, ls, vmean, vstd, M, D, G::MP, DQ, DS, vsm + G::oZs, vsm + G::oZn, vsm + G::oCm,
                 vsm + G::oVm, vsm + G::oSm1, vsm + G::oA);
  lds_barrier();
  float cmr[DV];
#pragma unroll
  for (int v = 0; v < DV; ++v) cmr[v] = vsm[G::oCm + sub + 16 * v];
  f32x4 gacc[HS];
#pragma unroll
  for (int s = 0; s < HS; ++s) gacc[s] = f32x4{0.f, 0.f, 0.f, 0.f};
  f32x4 uacc[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
  // the chunk's A units (4 rows of one point each): loaded one chunk ahead (registers)
  f32x4 au[NU / NT];
  auto load_a = [&](int t) {
    const float* sb = saved + (size_t)(t < nchunks ? t : 0) * SV::blk;
#pragma unroll
    for (int q = 0; q < NU / NT; ++q) au[q] = *(const f32x4*)(sb + 4 * (tid + q * NT));
  };
  load_a(blockIdx.x);

  for (int t = blockIdx.x; t < nchunks; t += gridDim.x) {
    const int b = t / nch, i0 = (t - b * nch) * LTW;
    const int nvalid = N - i0 < LTW ? N - i0 : LTW;
    const long long col0 = (long long)b * N + i0;
    float* sm = (float*)fresh_lds(vsm);
    float* Ar = sm + G::oA;
    float* Kr = sm + G::oK;
    const float* zs = sm + G::oZs;
    const float* zn = sm + G::oZn;
    float* xs = sm + G::oXs;
    float* xn = sm + G::oXn;
    float* gmc = sm + G::oGm;
    float* gvc = sm + G::oGv;
    const float* sb = saved + (size_t)t * SV::blk;
    lds_barrier();   // the previous chunk's reads are done
#pragma unroll
    for (int q = 0; q < NU / NT; ++q) {
      // unit e: tile (rt, ct) = e / 64, lane' = e % 64 -> rows 16 rt + g' + 4u, point 16 ct + c'
      const int e = tid + q * NT, tl = e >> 6, ln = e & 63, rt = tl >> 1, ct = tl & 1;
      const int col = 16 * ct + (ln & 15), r0 = 16 * rt + (ln >> 4);
#pragma unroll
      for (int u = 0; u < 4; ++u) Ar[(r0 + 4 * u) * KS + col] = au[q][u];
    }
    lstage_points<NPASS, DV, NT, DS>(xr, lsr, cmr, D, nvalid, xs, xn);
    if (tid < LTW) {
      const bool ok = tid < nvalid;
      const float gm = gmean[ok ? col0 + tid : 0], gv = gvar[ok ? col0 + tid : 0];
      const float keep = sb[SV::tiles + tid];
      gmc[tid] = ok ? gm : 0.f;
      gvc[tid] = (ok && keep != 0.f) ? gv : 0.f;   // the variance clamp passes no gradient
    }
    if (t + (int)gridDim.x < nchunks) {
      lload_points<NPASS, DV, NT>(X, t + gridDim.x, nchunks, nch, N, D, xr);
      load_a(t + gridDim.x);   // (au was consumed by the LDS stores above)
    }
    lds_barrier();
    // K_ZX of the wave's rows -> Kr[row][point]; u partials (SPL = 2: half 0 row IA, half 1 IB)
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      if (h == 1 && !two) break;
      if (SPL == 2 && h != hf) continue;
      const int rt = h == 0 ? IA : IB;
#pragma unroll
      for (int ct = 0; ct < 2; ++ct) {
        const float* za = zs + (16 * rt + c) * DS + g;
        const float* xb = xs + (16 * ct + c) * DS + g;
        f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int k = 0; k < DQ / 4; ++k) acc = mfma32(za[4 * k], xb[4 * k], acc);
        const int col = 16 * ct + c;
        const float xnc = xn[col], gmv = gmc[col];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int p = 16 * rt + 4 * g + r;
          float dist = zn[p] + xnc - 2.f * acc[r];
          dist = dist < 0.f ? 0.f : dist;
          const float kv = (p < M && col < nvalid) ? s2 * __builtin_amdgcn_exp2f(kNHalfLog2e * dist) : 0.f;
          Kr[p * KS + col] = kv;
          uacc[h][r] = __builtin_fmaf(gmv, kv, uacc[h][r]);
        }
      }
    }
    lds_barrier();
    // G' tiles (I >= J): A[16 I + c][8 g + j] gvar_(8 g + j) and K[16 J + c][8 g + j]
    {
      const f32x4 gv0 = *(const f32x4*)(gvc + 8 * g), gv1 = *(const f32x4*)(gvc + 8 * g + 4);
      auto rowop = [&](const float* base, int rt, float (&o)[8]) {
        const f32x4 a0 = *(const f32x4*)(base + (16 * rt + c) * KS + 8 * g);
        const f32x4 a1 = *(const f32x4*)(base + (16 * rt + c) * KS + 8 * g + 4);
#pragma unroll
        for (int q = 0; q < 4; ++q) { o[q] = a0[q]; o[4 + q] = a1[q]; }
      };
      float aA[8], aB[8];
      rowop(Ar, IA, aA);
      rowop(Ar, two ? IB : IA, aB);
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        aA[q] *= gv0[q]; aA[4 + q] *= gv1[q];
        aB[q] *= gv0[q]; aB[4 + q] *= gv1[q];
      }
#pragma unroll
      for (int ls = 0; ls < HS; ++ls) {
        const int s = s0 + ls;
        if (s >= nslot) break;
        const bool isA = s <= IA;
        const int J = isA ? s : s - IA - 1;
        float bo[8];
        rowop(Kr, J, bo);
#pragma unroll
        for (int q = 0; q < 8; ++q) gacc[ls] = mfma32(isA ? aA[q] : aB[q], bo[q], gacc[ls]);
        __builtin_amdgcn_sched_barrier(0);
      }
    }
  }
  // partials: tile (I, J) at (I (I + 1) / 2 + J) * 256 + lane * 4 + r (acc layout) | u
  float* po = gpart + (size_t)blockIdx.x * G::PG;
#pragma unroll
  for (int ls = 0; ls < HS; ++ls) {
    const int s = s0 + ls;
    if (s >= nslot) break;
    const bool isA = s <= IA;
    const int I = isA ? IA : IB, J = isA ? s : s - IA - 1;
    *(f32x4*)(po + (I * (I + 1) / 2 + J) * 256 + lane * 4) = gacc[ls];
  }
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    if (h == 1 && !two) break;
    if (SPL == 2 && h != hf) continue;
    const int rt = h == 0 ? IA : IB;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float v = row16_sum_f(uacc[h][r]);
      if (c == 0) po[G::NTILE * 256 + 16 * rt + 4 * g + r] = v;
    }
  }
}

// ---------------------------------------------------------------------------
// Adjoint for M > 64 from the training forward's saved state (gpk_variational_train_f32):
// ONE kernel in the adjk layout (wave w holds the L^{-1} COLUMN blocks of block rows
// pA = w, pB = MB-1-w). Per chunk: A (fp32, LSaved layout) straight into the LDS dA tiles by
// LDS-DMA (double-buffered), the clamp mask onto gvar; each wave turns ITS rows of A into
// dA = gmean m + 2 gvar (s^2 - 1) A in place (with the dvmean / dvstd row sums); then
// dK = L^{-T} dA on f32 MFMA from an fp32 copy of the wave's L^{-1} column blocks (round 6; the
// reference's dK is fp64: 68 instead of 136 VGPRs and twice the MFMA rate, 0.229 -> 0.180 ms at
// N = 192; the gradients stay within ~1e-6 of the fp64 oracle), K_ZX of the
// wave's rows recomputed (f32 MFMA, natural row order: every f32 MFMA output here is in the f32
// C layout, lane (g, c) reg r <-> row 4 g + r), Q = dK o K and the Q^T zs / QX contractions, dX
// per point and the fixed-order partials. dL^{-1} comes from gpk_var_kgram_l_kernel (G' = A
// diag(gvar) K_ZX^T from the same saved A, below). (Accumulating dL^{-1} = sum dA K^T in this
// pass as well -- the wave's tile columns are its K rows -- needs 68 more VGPRs than the 256 of
// two waves per SIMD: 98 VGPRs of spills, L^{-1} reloaded from scratch inside the GEMM, measured
// 0.232 ms; not kept.)
// ---------------------------------------------------------------------------
// dK of the wave with pA = RA from its fp32 column-block registers: slots 0..NA-1 are blocks
// (rt = RA + s, RA), the rest (rt = RB + s - NA, RB); B operands dA[rt] from LDS (the next slot's
// read while this slot's 8 MFMAs run).
template <int MB, int RA>
GPK_DEVICE void lcol_gemm32(const float (&Lc)[MB + 1][4], const float* dAl, int lane,
                            f32x4 (&dKa)[2], f32x4 (&dKb)[2]) {
  constexpr int RB = MB - 1 - RA;
  constexpr int NA = MB - RA;
  constexpr int NS = RB == RA ? NA : MB + 1;
  f32x4 acc[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
  f32x4 k0 = *(const f32x4*)(dAl + ((RA * 2 + 0) * 64 + lane) * 4);
  f32x4 k1 = *(const f32x4*)(dAl + ((RA * 2 + 1) * 64 + lane) * 4);
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    if (s == NA) {
      dKa[0] = acc[0];
      dKa[1] = acc[1];
      acc[0] = acc[1] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
    f32x4 n0 = k0, n1 = k1;
    if (s + 1 < NS) {
      const int rtn = s + 1 < NA ? RA + s + 1 : RB + (s + 1 - NA);
      n0 = *(const f32x4*)(dAl + ((rtn * 2 + 0) * 64 + lane) * 4);
      n1 = *(const f32x4*)(dAl + ((rtn * 2 + 1) * 64 + lane) * 4);
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      acc[0] = mfma32(Lc[s][u], k0[u], acc[0]);
      acc[1] = mfma32(Lc[s][u], k1[u], acc[1]);
    }
    k0 = n0;
    k1 = n1;
    __builtin_amdgcn_sched_barrier(0);
  }
  if (RB == RA) {
    dKa[0] = acc[0];
    dKa[1] = acc[1];
    dKb[0] = dKb[1] = f32x4{0.f, 0.f, 0.f, 0.f};
  } else {
    dKb[0] = acc[0];
    dKb[1] = acc[1];
  }
}
template <int MB, int RA>
GPK_DEVICE void lcol_gemm32_for(int wave, const float (&Lc)[MB + 1][4], const float* dAl, int lane,
                                f32x4 (&dKa)[2], f32x4 (&dKb)[2]) {
  if constexpr (RA < (MB + 1) / 2) {
    if (wave == RA) lcol_gemm32<MB, RA>(Lc, dAl, lane, dKa, dKb);
    else lcol_gemm32_for<MB, RA + 1>(wave, Lc, dAl, lane, dKa, dKb);
  }
}

template <int MB, int DQ>
__global__ void __launch_bounds__(64 * ((MB + 1) / 2), 2)
gpk_var_adjs_l_kernel(const float* __restrict__ X, const float* __restrict__ Z,
                      const double* __restrict__ Linv, const float* __restrict__ vmean,
                      const float* __restrict__ vstd, const float* __restrict__ hyp,
                      const float* __restrict__ gmean, const float* __restrict__ gvar,
                      const float* __restrict__ saved, int N, int M, int D, int nchunks,
                      float* __restrict__ wspart, float* __restrict__ dX, float* __restrict__ cm_out) {
  using G = LAdjGeo<MB, DQ>;
  using SV = LSaved<MB>;
  constexpr int NWV = G::NWV, NT = G::NT, DS = G::DS, NPASS = G::NPASS, DV = G::DV, NDT = G::NDT;
  constexpr int NU = SV::tiles / 4;                 // f32x4 units of A per chunk
  static_assert(NU % NT == 0, "A block: whole passes");
  static_assert(MB % 2 == 0, "two distinct column blocks per wave");   // (MB in {6, 8, 12, 16})
  extern __shared__ __attribute__((aligned(16))) float vsm[];
  const int tid = threadIdx.x, lane = tid & 63, c = lane & 15, g = lane >> 4, sub = tid & 15;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int pA = wave, pB = MB - 1 - wave;
  const float s2 = hyp[0];
  const float* w = hyp + 4;
  const float* ls = hyp + 4 + D;
  const int nch = (N + LTW - 1) / LTW;
  constexpr int oRows = G::kMisc, oXn = G::kMisc + 2 * G::MP, oGv = oXn + 2 * LTW;
  static_assert(2 * G::MP + 4 * LTW <= 2 * NT + NWV, "misc area");

  // L^{-1} column blocks (k-order g + 4u, as gpk_var_adjs_l_kernel), rounded to fp32
  float Lc[MB + 1][4];
  {
    const bool full = (M & 15) == 0;
    const int NA = MB - pA;
#pragma unroll
    for (int s = 0; s <= MB; ++s) {
      const bool isA = s < NA;
      const int P = isA ? pA : pB, rt = isA ? pA + s : pB + (s - NA);
      const bool ok = isA || rt < MB;
      const int col = 16 * P + c;
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int row = 16 * rt + g + 4 * u;
        const bool in = ok && (full || (row < M && col < M));
        const double v = Linv[in ? (size_t)row * M + col : 0];
        Lc[s][u] = in ? (float)v : 0.f;
      }
      if ((s & 3) == 3) __builtin_amdgcn_sched_barrier(0);
    }
  }
  float lsr[DV];
#pragma unroll
  for (int v = 0; v < DV; ++v) lsr[v] = ls[sub + 16 * v < D ? sub + 16 * v : 0];
  float xr[NPASS][DV];
  lload_points<NPASS, DV, NT>(X, blockIdx.x, nchunks, nch, N, D, xr);
  stage_inducing(Z, ls, vmean, vstd, M, D, G::MP, DQ, DS, vsm + G::kZs, vsm + G::kZn, vsm + G::kCm,
                 vsm + G::kVm, vsm + G::kSm1, vsm + G::kKl);
  for (int e = tid; e < G::MP; e += NT) vsm[G::kQ + e] = 0.f;
  for (int e = tid; e < 2 * G::MP; e += NT) vsm[oRows + e] = 0.f;
  auto copy_a = [&](int t, float* buf) {
    const float* sb = saved + (size_t)t * SV::blk;
#pragma unroll
    for (int q = 0; q < NU / NT; ++q) {
      const int u0 = (q * NWV + wave) * 64;
      __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(sb + 4 * (u0 + lane)),
                                       (__attribute__((address_space(3))) void*)(buf + 4 * u0), 16, 0, 0);
    }
  };
  copy_a(blockIdx.x, vsm + G::kdA);
  lds_barrier();
  if (blockIdx.x == 0 && tid < D) cm_out[tid] = vsm[G::kCm + tid];
  float cmr[DV];
#pragma unroll
  for (int v = 0; v < DV; ++v) cmr[v] = vsm[G::kCm + sub + 16 * v];
  const int dd = tid % DQ;
  const float il_dd = dd < D ? 1.f / ls[dd < D ? dd : 0] : 0.f;
  const float w_dd = dd < D ? w[dd < D ? dd : 0] : 0.f;
  float rx2 = 0.f, gxa = 0.f, sumQ = 0.f, sumgm = 0.f, sumgv = 0.f;
  f32x4 qx[2][NDT];
#pragma unroll
  for (int h = 0; h < 2; ++h)
#pragma unroll
    for (int dt = 0; dt < NDT; ++dt) qx[h][dt] = f32x4{0.f, 0.f, 0.f, 0.f};
  int par = 0;

  for (int t = blockIdx.x; t < nchunks; t += gridDim.x, par ^= 1) {
    const int b = t / nch, i0 = (t - b * nch) * LTW;
    const int nvalid = N - i0 < LTW ? N - i0 : LTW;
    const long long col0 = (long long)b * N + i0;
    float* sm = (float*)fresh_lds(vsm);
    float* dAl = sm + (par ? G::kKl : G::kdA);
    float* xzl = sm + G::kXz;
    float* red = sm + G::kRed;
    const float* zs = sm + G::kZs;
    const float* zn = sm + G::kZn;
    const float* vm = sm + G::kVm;
    const float* sm1 = sm + G::kSm1;
    float* qrow = sm + G::kQ;
    float* scr = sm + G::kScr + wave * 320;
    float* xs = sm + G::kXs + par * LTW * DS;
    float* xn = sm + oXn + par * LTW;
    float* gmc = sm + G::kGm + par * LTW;
    float* gvc = sm + oGv + par * LTW;
    float* rows = sm + oRows;
    {
      const float* sb = saved + (size_t)t * SV::blk;
      if (tid < LTW) {
        const bool ok = tid < nvalid;
        const float keep = sb[SV::tiles + tid];
        const float gm = gmean[ok ? col0 + tid : 0], gv = gvar[ok ? col0 + tid : 0];
        const float gvk = (ok && keep != 0.f) ? gv : 0.f;
        gmc[tid] = ok ? gm : 0.f;
        gvc[tid] = gvk;
        sumgm += ok ? gm : 0.f;
        sumgv += gvk;
      }
    }
    lstage_points<NPASS, DV, NT, DS>(xr, lsr, cmr, D, nvalid, xs, xn);
    if (t + (int)gridDim.x < nchunks) lload_points<NPASS, DV, NT>(X, t + gridDim.x, nchunks, nch, N, D, xr);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // this wave's A copy has landed
    lds_barrier();
    // ---- the wave's own rows: row sums of A, A -> dA in place
    {
      float gmq[2], gvq[2];
#pragma unroll
      for (int ct = 0; ct < 2; ++ct) {
        gmq[ct] = gmc[16 * ct + c];
        gvq[ct] = gvc[16 * ct + c];
      }
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int rt = h == 0 ? pA : pB;
        float pm[4] = {0.f, 0.f, 0.f, 0.f}, ps[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int ct = 0; ct < 2; ++ct) {
          float* at = dAl + ((rt * 2 + ct) * 64 + lane) * 4;
          const f32x4 av = *(const f32x4*)at;
          f32x4 da;
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int p = 16 * rt + g + 4 * r;
            pm[r] = __builtin_fmaf(gmq[ct], av[r], pm[r]);
            ps[r] = __builtin_fmaf(gvq[ct], av[r] * av[r], ps[r]);
            da[r] = gmq[ct] * vm[p] + 2.f * gvq[ct] * sm1[p] * av[r];
          }
          *(f32x4*)at = da;
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float a = row16_sum_f(pm[r]), q = row16_sum_f(ps[r]);
          if (c == 0) {
            const int p = 16 * rt + g + 4 * r;
            lds_acc(rows + p, a);
            lds_acc(rows + G::MP + p, q);
          }
        }
      }
    }
    lds_barrier();
    // ---- dK = L^{-T} dA (f32 MFMA) on the wave's block rows; K_ZX of those rows; Q = dK o K
    f32x4 Qt[2][2];
    {
      f32x4 dK[2][2];
      if (t + (int)gridDim.x < nchunks) copy_a(t + gridDim.x, sm + (par ? G::kdA : G::kKl));
      lcol_gemm32_for<MB, 0>(wave, Lc, dAl, lane, dK[0], dK[1]);
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int rt = h == 0 ? pA : pB;
#pragma unroll
        for (int ct = 0; ct < 2; ++ct) {
          const float* za = zs + (16 * rt + c) * DS + g;
          const float* xb = xs + (16 * ct + c) * DS + g;
          f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
          for (int k = 0; k < DQ / 4; ++k) acc = mfma32(za[4 * k], xb[4 * k], acc);
          const int col = 16 * ct + c;
          const float xnc = xn[col];
          f32x4 kv;
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int p = 16 * rt + 4 * g + r;
            float dist = zn[p] + xnc - 2.f * acc[r];
            dist = dist < 0.f ? 0.f : dist;
            kv[r] = (p < M && col < nvalid) ? s2 * __builtin_amdgcn_exp2f(kNHalfLog2e * dist) : 0.f;
            Qt[h][ct][r] = dK[h][ct][r] * kv[r];
          }
        }
      }
    }
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int rt = h == 0 ? pA : pB;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float v = row16_sum_f(Qt[h][0][r] + Qt[h][1][r]);
        if (c == 0) lds_acc(qrow + 16 * rt + 4 * g + r, v);
      }
    }
#pragma unroll
    for (int ct = 0; ct < 2; ++ct) {
      float v = 0.f;
#pragma unroll
      for (int h = 0; h < 2; ++h) v += (Qt[h][ct][0] + Qt[h][ct][1]) + (Qt[h][ct][2] + Qt[h][ct][3]);
      sumQ += v;
      v += __shfl_xor(v, 16, 64);
      v += __shfl_xor(v, 32, 64);
      if (g == 0) red[wave * LTW + 16 * ct + c] = v;
    }
    {
      f32x4 xz[2][NDT];
#pragma unroll
      for (int ct = 0; ct < 2; ++ct)
#pragma unroll
        for (int dt = 0; dt < NDT; ++dt) xz[ct][dt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int rt = h == 0 ? pA : pB;
#pragma unroll
        for (int r = 0; r < 4; ++r)
#pragma unroll
          for (int dt = 0; dt < NDT; ++dt) {
            const float zb = zs[(16 * rt + 4 * g + r) * DS + 16 * dt + c];
#pragma unroll
            for (int ct = 0; ct < 2; ++ct) xz[ct][dt] = mfma32(Qt[h][ct][r], zb, xz[ct][dt]);
          }
      }
#pragma unroll
      for (int ct = 0; ct < 2; ++ct)
#pragma unroll
        for (int dt = 0; dt < NDT; ++dt)
#pragma unroll
          for (int r = 0; r < 4; ++r)
            xzl[(wave * LTW + 16 * ct + 4 * g + r) * DQ + 16 * dt + c] = xz[ct][dt][r];
    }
#pragma unroll
    for (int h = 0; h < 2; ++h) {
#pragma unroll
      for (int ct = 0; ct < 2; ++ct) {
#pragma unroll
        for (int r = 0; r < 4; ++r) scr[lane * 5 + r] = Qt[h][ct][r];
        adj_lds_order();
        float aq[4];
#pragma unroll
        for (int s4 = 0; s4 < 4; ++s4) aq[s4] = scr[(16 * (c >> 2) + 4 * s4 + g) * 5 + (c & 3)];
        adj_lds_order();
#pragma unroll
        for (int dt = 0; dt < NDT; ++dt)
#pragma unroll
          for (int s4 = 0; s4 < 4; ++s4)
            qx[h][dt] = mfma32(aq[s4], xs[(16 * ct + 4 * s4 + g) * DS + 16 * dt + c], qx[h][dt]);
      }
    }
    lds_barrier();
    for (int e = tid; e < LTW * DQ; e += NT) {
      const int col = e / DQ;
      float v = 0.f, r = 0.f;
#pragma unroll
      for (int q = 0; q < NWV; ++q) {
        v += xzl[(q * LTW + col) * DQ + dd];
        r += red[q * LTW + col];
      }
      const float xv = xs[col * DS + dd];
      if (col < nvalid && dd < D) {
        dX[(col0 + col) * D + dd] = (v - xv * r) * il_dd + gmc[col] * w_dd;
        rx2 = __builtin_fmaf(r * xv, xv, rx2);
        gxa = __builtin_fmaf(gmc[col], xv, gxa);
      }
    }
  }
  lds_barrier();
  // partial fields: QX (M x D) | q (M) | dvm (M) | dsm (M) | rx2 (D) | sumQ | sumgv | gx (D) | sumgm
  const int P = M * D + 3 * M + 2 * D + 3;
  float* po = wspart + (size_t)blockIdx.x * P;
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int rt = h == 0 ? pA : pB;
#pragma unroll
    for (int dt = 0; dt < NDT; ++dt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int p = 16 * rt + 4 * g + r, d = 16 * dt + c;
        if (p < M && d < D) po[p * D + d] = qx[h][dt][r];
      }
  }
  for (int m = tid; m < M; m += NT) {
    po[M * D + m] = vsm[G::kQ + m];
    po[M * D + M + m] = vsm[oRows + m];
    po[M * D + 2 * M + m] = vsm[oRows + G::MP + m];
  }
  lds_barrier();
  float* misc = vsm + G::kMisc;
  misc[tid] = rx2;
  misc[NT + tid] = gxa;
  sumQ = wave_sum(sumQ);
  if (lane == 0) misc[2 * NT + wave] = sumQ;
  lds_barrier();
  for (int d = tid; d < D; d += NT) {
    float v = 0.f, u = 0.f;
    for (int q = d; q < NT; q += DQ) { v += misc[q]; u += misc[NT + q]; }
    po[M * D + 3 * M + d] = v;
    po[M * D + 3 * M + D + 2 + d] = u;
  }
  if (tid == 0) {
    float v = 0.f;
    for (int q = 0; q < NWV; ++q) v += misc[2 * NT + q];
    po[M * D + 3 * M + D] = v;
  }
  if (wave == 0) {
    const float u = wave_sum(sumgm), v = wave_sum(sumgv);
    if (lane == 0) {
      po[M * D + 3 * M + 2 * D + 2] = u;
      po[M * D + 3 * M + D + 1] = v;
    }
  }
}

// dL^{-1}[p][q] = m_p u_q + 2 (s_p^2 - 1) G'[p][q] for q <= p, 0 above (fp64), elementwise from
// the fixed-order totals gtot (G' lower tiles in acc layout | u).
GPK_DEVICE void var_gdl_elem(long long e, const double* __restrict__ gtot, const float* __restrict__ vmean,
                             const float* __restrict__ vstd, int M, int MB, double* __restrict__ dLinv) {
  if (e >= (long long)M * M) return;
  const int p = (int)(e / M), q = (int)(e - (long long)p * M);
  double v = 0.0;
  if (q <= p) {
    const int ti = p >> 4, tj = q >> 4, ra = p & 15, cb = q & 15;
    const double gp = gtot[(ti * (ti + 1) / 2 + tj) * 256 + ((ra >> 2) * 16 + cb) * 4 + (ra & 3)];
    const double u = gtot[(size_t)(MB * (MB + 1) / 2) * 256 + q];
    const double sd = (double)vstd[p];
    v = (double)vmean[p] * u + 2.0 * (sd * sd - 1.0) * gp;
  }
  dLinv[e] = v;
}

// ---------------------------------------------------------------------------
// dL^{-1} = sum_cols dA[:, col] K[:, col]^T (lower part): split-K fp64-MFMA GEMM.
// Workgroup = one 64 x 64 lower output tile (ti >= tj) x one split of the columns;
// 4 waves, each a 32 x 32 quadrant (2 x 2 MFMA tiles). fp32 operands are exact in fp64.
// Partials -> ws (split, tile, 64 x 64) doubles.
// ---------------------------------------------------------------------------
constexpr int DLKC = 32;   // columns staged per step
constexpr int DLST = 34;   // LDS row stride (floats): 2c + g spreads the MFMA operand reads

__global__ void __launch_bounds__(256)
gpk_dlinv_kernel(const float* __restrict__ dA, const float* __restrict__ Kz, int M, long long BN,
                 int ntiles, long long cols_per_split, double* __restrict__ part) {
  __shared__ float sa[64 * DLST];
  __shared__ float sb[64 * DLST];
  const int tid = threadIdx.x, lane = tid & 63, c = lane & 15, g = lane >> 4;
  const int wave = tid >> 6, qr = wave >> 1, qc = wave & 1;
  const int tile = blockIdx.x % ntiles, split = blockIdx.x / ntiles;
  int ti = 0;
  while ((ti + 1) * (ti + 2) / 2 <= tile) ++ti;
  const int tj = tile - ti * (ti + 1) / 2;
  const int m0 = 64 * ti, p0 = 64 * tj;
  const long long c0 = (long long)split * cols_per_split;
  long long c1 = c0 + cols_per_split;
  c1 = c1 < BN ? c1 : BN;
  const bool vec = (BN & 3) == 0;   // 16-B loads need 16-B aligned rows
  f64x4 acc[2][2];
#pragma unroll
  for (int u = 0; u < 2; ++u)
#pragma unroll
    for (int v = 0; v < 2; ++v) acc[u][v] = f64x4{0.0, 0.0, 0.0, 0.0};
  // each thread stages 2 x 4 consecutive columns of one row of each operand per step:
  // e = tid + 256 h (h = 0, 1) -> row e / 8, columns 4 (e % 8) .. +3
  float4 ra[2], rb[2];
  auto load = [&](long long cb, float4 (&xa)[2], float4 (&xb)[2]) {
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int e = tid + 256 * h, rr = e >> 3, k4 = 4 * (e & 7);
      const long long col = cb + k4;
      float4 va = {0.f, 0.f, 0.f, 0.f}, vb = {0.f, 0.f, 0.f, 0.f};
      if (vec && col + 3 < c1) {
        if (m0 + rr < M) va = *(const float4*)&dA[(size_t)(m0 + rr) * BN + col];
        if (p0 + rr < M) vb = *(const float4*)&Kz[(size_t)(p0 + rr) * BN + col];
      } else {
        float ta[4], tb[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const bool ok = col + u < c1;
          ta[u] = (ok && m0 + rr < M) ? dA[(size_t)(m0 + rr) * BN + col + u] : 0.f;
          tb[u] = (ok && p0 + rr < M) ? Kz[(size_t)(p0 + rr) * BN + col + u] : 0.f;
        }
        va = float4{ta[0], ta[1], ta[2], ta[3]};
        vb = float4{tb[0], tb[1], tb[2], tb[3]};
      }
      xa[h] = va;
      xb[h] = vb;
    }
  };
  load(c0, ra, rb);
  for (long long cb = c0; cb < c1; cb += DLKC) {
    lds_barrier();  // previous step's MFMA operand reads are done
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int e = tid + 256 * h, rr = e >> 3, k4 = 4 * (e & 7);
      *(float2*)&sa[rr * DLST + k4] = float2{ra[h].x, ra[h].y};
      *(float2*)&sa[rr * DLST + k4 + 2] = float2{ra[h].z, ra[h].w};
      *(float2*)&sb[rr * DLST + k4] = float2{rb[h].x, rb[h].y};
      *(float2*)&sb[rr * DLST + k4 + 2] = float2{rb[h].z, rb[h].w};
    }
    lds_barrier();
    if (cb + DLKC < c1) load(cb + DLKC, ra, rb);   // next step's loads overlap the MFMAs
#pragma unroll
    for (int k = 0; k < DLKC / 4; ++k) {
      double a[2], bb[2];
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        a[u] = (double)sa[(32 * qr + 16 * u + c) * DLST + 4 * k + g];
        bb[u] = (double)sb[(32 * qc + 16 * u + c) * DLST + 4 * k + g];
      }
#pragma unroll
      for (int u = 0; u < 2; ++u)
#pragma unroll
        for (int v = 0; v < 2; ++v) acc[u][v] = mfma64(a[u], bb[v], acc[u][v]);
    }
  }
  double* po = part + ((size_t)split * ntiles + tile) * 4096;
#pragma unroll
  for (int u = 0; u < 2; ++u)
#pragma unroll
    for (int v = 0; v < 2; ++v)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = 32 * qr + 16 * u + g + 4 * r, col = 32 * qc + 16 * v + c;
        po[row * 64 + col] = acc[u][v][r];
      }
}

// Fixed-order reductions, 32 outputs per workgroup, 8 lanes per output each summing
// every 8th partial, then the 8 lane sums in a fixed order (fp64):
//   (a) the per-workgroup adjoint partials -> tot (P doubles);
//   (b) the split-K dL^{-1} partials -> dLinv (M x M, upper zero).
__global__ void __launch_bounds__(256)
gpk_var_red_kernel(const float* __restrict__ wspart, int nwg, int P, double* __restrict__ tot,
                   const double* __restrict__ dlpart, int nsplit, int ntiles, int M,
                   double* __restrict__ dLinv, const float* __restrict__ wspart2, int P2,
                   double* __restrict__ tot2) {
  __shared__ double red[8][33];
  const int tid = threadIdx.x, o = tid & 31, q0 = tid >> 5;
  const int nblk_a = (P + 31) / 32;
  double s = 0.0;
  long long out;
  if ((int)blockIdx.x < nblk_a) {
    out = (long long)blockIdx.x * 32 + o;
    if (out < P) {
#pragma unroll 4
      for (int q = q0; q < nwg; q += 8) s += (double)wspart[(size_t)q * P + out];
    }
  } else if (wspart2 != nullptr) {
    // a second partial array with the same workgroup count (one launch for both sums)
    out = (long long)(blockIdx.x - nblk_a) * 32 + o;
    if (out < P2) {
#pragma unroll 4
      for (int q = q0; q < nwg; q += 8) s += (double)wspart2[(size_t)q * P2 + out];
    }
  } else {
    out = (long long)(blockIdx.x - nblk_a) * 32 + o;
    if (out < (long long)M * M) {
      const int m = (int)(out / M), p = (int)(out - (long long)m * M);
      if (p <= m) {
        const int ti = m >> 6, tj = p >> 6;
        const int tile = ti * (ti + 1) / 2 + tj;
        const int off = (m & 63) * 64 + (p & 63);
#pragma unroll 4
        for (int q = q0; q < nsplit; q += 8) s += dlpart[((size_t)q * ntiles + tile) * 4096 + off];
      }
    }
  }
  red[q0][o] = s;
  lds_barrier();
  if (q0 == 0) {
    double t = 0.0;
#pragma unroll
    for (int q = 0; q < 8; ++q) t += red[q][o];
    if ((int)blockIdx.x < nblk_a) {
      if (out < P) tot[out] = t;
    } else if (wspart2 != nullptr) {
      if (out < P2) tot2[out] = t;
    } else if (out < (long long)M * M) {
      dLinv[out] = t;
    }
  }
}

// Outputs from the reduced totals, ONE launch (gpk_var_fin_kernel):
//   blocks 0 .. nblk-1 (16 inducing points each):  dZ_p = (QX_p - zs_p q_p) / l
//   block nblk (the totals block, all M rows):
//       dl_d = (sum_p (q_p zs_pd^2 - 2 zs_pd QX_pd) + sum_i r_i xs_id^2) / l_d
//       ds2 = sum Q / s2 + sum gvar;    dvmean = sum gmean A;   dvstd = 2 s sum gvar A^2
//       dw_d = l_d (sum_i gmean_i xs_id + cm_d sum_i gmean_i);   db0 = sum_i gmean_i
//   block nblk + 1 (gd.gtot != nullptr, register path): dL^{-1} from the K-Gram totals
// dpar = [dvmean (M) | dvstd (M) | ds2 | dl (D) | dw (D) | db0]. zs = Z / l - cm with the centre
// cm from the adjoint kernel (cm_in: its stage_inducing) or, without it, recomputed by
// col_means -- the same fixed-order fp32 sums, so the identical centre. No block depends on
// another: the round-4 second launch (block partials of dl) is gone.
constexpr int kFinRows = 16;

GPK_DEVICE void var_gdl_block(const double* __restrict__ gtot, const double* __restrict__ Linv,
                              const float* __restrict__ vmean, const float* __restrict__ vstd, int M,
                              double* __restrict__ dLinv, double (*Gs)[65], double* us);

// gd.gtot != nullptr: dL^{-1} from the K-Gram totals in extra workgroups of the output launch
// instead of a launch of its own -- MB == 0 (register path, M <= 64): one workgroup
// (var_gdl_block, L^{-1} G on fp64 MFMA); MB > 0 (saved-state path): M^2 / 256 workgroups of
// the elementwise m u^T + 2 (s^2 - 1) G' (var_gdl_elem)
struct VarGdlArgs {
  const double* gtot;
  const double* Linv;
  const float* vmean;
  const float* vstd;
  double* dLinv;
  int MB;
};
GPK_DEVICE void var_gdl_elem(long long e, const double* __restrict__ gtot, const float* __restrict__ vmean,
                             const float* __restrict__ vstd, int M, int MB, double* __restrict__ dLinv);

__global__ void __launch_bounds__(256)
gpk_var_fin_kernel(const float* __restrict__ Z, const float* __restrict__ vstd,
                   const float* __restrict__ hyp, const double* __restrict__ tot, int M, int D,
                   float* __restrict__ dZ, float* __restrict__ dpar, const float* __restrict__ cm_in,
                   VarGdlArgs gd) {
  extern __shared__ __attribute__((aligned(16))) float fzs[];   // M x D zs (centred Z / l)
  __shared__ double red[256];
  __shared__ float cmf[64];
  __shared__ float cms[kCmParts * 64];
  const int tid = threadIdx.x;
  const int nblk = (M + kFinRows - 1) / kFinRows;
  if (gd.gtot != nullptr && (int)blockIdx.x > nblk) {
    if (gd.MB == 0) {
      double* gl = (double*)fzs;
      var_gdl_block(gd.gtot, gd.Linv, gd.vmean, gd.vstd, M, gd.dLinv, (double(*)[65])gl, gl + 64 * 65);
    } else {
      var_gdl_elem((long long)(blockIdx.x - nblk - 1) * 256 + tid, gd.gtot, gd.vmean, gd.vstd, M, gd.MB,
                   gd.dLinv);
    }
    return;
  }
  const bool totals = (int)blockIdx.x == nblk;
  const float* ls = hyp + 4 + D;
  const int p0 = totals ? 0 : blockIdx.x * kFinRows;
  const int np = totals ? M : (M - p0 < kFinRows ? M - p0 : kFinRows);
  if (cm_in != nullptr) {
    // the centre from the adjoint kernel, so only this block's rows of Z are staged
    if (tid < D) cmf[tid] = cm_in[tid];
    for (int base = 0; base < np * D; base += 8 * 256) {
      float zv[8], lv[8], cv[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int e = base + 256 * u + tid, ec = e < np * D ? e : 0, d = ec % D;
        zv[u] = Z[(size_t)p0 * D + ec];
        lv[u] = ls[d];
        cv[u] = cm_in[d];
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int e = base + 256 * u + tid;
        if (e < np * D) fzs[p0 * D + e] = zv[u] / lv[u] - cv[u];
      }
    }
  } else {
    for (int base = 0; base < M * D; base += 32 * 256) {
      float zv[32], lv[32];
#pragma unroll
      for (int u = 0; u < 32; ++u) {
        const int e = base + 256 * u + tid, ec = e < M * D ? e : 0;
        zv[u] = Z[ec];
        lv[u] = ls[ec % D];
      }
#pragma unroll
      for (int u = 0; u < 32; ++u) {
        const int e = base + 256 * u + tid;
        if (e < M * D) fzs[e] = zv[u] / lv[u];
      }
    }
    lds_barrier();
    col_means(fzs, M, D, D, D, cms, cmf);   // the same fp32 sums as stage_inducing: the identical centre
    for (int e = tid; e < np * D; e += 256) fzs[p0 * D + e] -= cmf[e % D];
  }
  lds_barrier();
  const double* QX = tot;
  const double* q = tot + (size_t)M * D;
  if (!totals) {
    const int e = tid;   // np * D <= 16 * 64 = 1024: up to 4 per thread, loads together
    double xv[4], qv[4];
    float lv[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int ee = e + 256 * u, ok = ee < np * D;
      const int p = p0 + (ok ? ee / D : 0), d = ok ? ee % D : 0;
      xv[u] = QX[(size_t)p * D + d];
      qv[u] = q[p];
      lv[u] = ls[d];
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int ee = e + 256 * u;
      if (ee < np * D) {
        const int p = p0 + ee / D, d = ee % D;
        const double zsv = (double)fzs[p * D + d];
        dZ[(size_t)p * D + d] = (float)((xv[u] - zsv * qv[u]) / (double)lv[u]);
      }
    }
    return;
  }
  // ---- the totals block: dl over all M rows, threads (d, k), k = tid / D, rows k, k + nk, ..
  // (16 rows' loads in flight per thread, fixed order)
  const double* dvm = tot + (size_t)M * D + M;
  const double* dsm = dvm + M;
  const double* rx2 = dsm + M;
  const double* gx = rx2 + D + 2;
  const int nk = 256 / D;
  double acc = 0.0;
  if (tid < nk * D) {
    const int d = tid % D, k = tid / D;
    for (int base = k; base < M; base += 16 * nk) {
      double qv[16], xv[16];
#pragma unroll
      for (int u = 0; u < 16; ++u) {
        const int pl = base + nk * u, pc = pl < M ? pl : 0;
        qv[u] = q[pc];
        xv[u] = QX[(size_t)pc * D + d];
      }
#pragma unroll
      for (int u = 0; u < 16; ++u) {
        const int pl = base + nk * u;
        if (pl < M) {
          const double zsv = (double)fzs[pl * D + d];
          acc += qv[u] * zsv * zsv - 2.0 * zsv * xv[u];
        }
      }
    }
  }
  red[tid] = acc;
  lds_barrier();
  const float s2 = hyp[0];
  if (tid < D) {
    double v = rx2[tid];
    for (int k = 0; k < nk; ++k) v += red[k * D + tid];
    const double sumgm = gx[D];
    dpar[2 * M + 1 + tid] = (float)(v / (double)ls[tid]);
    dpar[2 * M + 1 + D + tid] = (float)((double)ls[tid] * (gx[tid] + (double)cmf[tid] * sumgm));
  }
  for (int m = tid; m < M; m += 256) {
    dpar[m] = (float)dvm[m];
    dpar[M + m] = (float)(2.0 * (double)vstd[m] * dsm[m]);
  }
  if (tid == 0) {
    const double sumQ = rx2[D], sumgv = rx2[D + 1], sumgm = gx[D];
    dpar[2 * M] = (float)(sumQ / (double)s2 + sumgv);
    dpar[2 * M + 1 + 2 * D] = (float)sumgm;
  }
}

// the two output launches (ws: nblk x D doubles of dl partials, then D floats of the centre)
int launch_var_fin(const float* Z, const float* vstd, const float* hyp, const double* tot, int M, int D,
                   float* dZ, float* dpar, hipStream_t stream, const float* cm_in = nullptr,
                   const VarGdlArgs* gd = nullptr);

// ---------------------------------------------------------------------------
// Register-resident variants for M <= 64, D <= 32 (BASELINE cfg 5: M = 64, D = 32).
// With at most 4 row tiles every wave owns ALL rows of its points, so the waves of a
// workgroup never exchange data: each wave walks its own 32-point chunks (2 column
// tiles) and keeps K_ZX, A = L^{-1} K_ZX, dA, dK and Q in MFMA registers. The f32 Gram
// feeds the zs rows in the order pi(x) = (x >> 2) + 4 (x & 3), so its accumulator holds
// row g + 4r in register r -- the f64 MFMA layout -- and K_ZX tiles are directly the B
// operands of the f64 products. L^{-1} (fp64, row stride 66: conflict-free reads) and zs
// live in LDS, shared by the 4 waves; only the adjoint's Q^T needs a per-wave LDS
// transpose (one tile at a time).
// ---------------------------------------------------------------------------
#ifndef GPK_FWD_OCC
#define GPK_FWD_OCC 3   // waves per SIMD gpk_var_fwd_r_kernel's register budget is sized for (3: 161
                         // VGPRs, cfg 5 forward 55.7 vs 56.6 us unbounded; a next-chunk point
                         // prefetch measured slower at 3 (spills) and at 2 waves/SIMD)
#endif
constexpr int RLS = 66;        // L^{-1} row stride (doubles)
constexpr int kGTiles = 10;                  // lower 16 x 16 tiles of a 64 x 64 G
constexpr int kGPart = kGTiles * 256 + 64;   // floats per workgroup K-Gram partial

// NW waves per workgroup; FG: the adjoint also accumulates the K-Gram G / u per wave
// (gpk_var_adj_r_kernel with the K-Gram folded in, 8 waves: 154 KB at DQ = 32)
template <int DQ, int NW = 4, bool FG = false>
struct RegLds {
  static constexpr int ZS = DQ + 1;
  static constexpr int zs = 0;                      // 64 x ZS
  static constexpr int zn = zs + 64 * ZS;           // 64
  static constexpr int vm = zn + 64;                // 64
  static constexpr int sm1 = vm + 64;               // 64
  static constexpr int cm = sm1 + 64;               // DQ
  static constexpr int li = ((cm + DQ + 3) / 4) * 4;          // 64 x RLS doubles (16-B aligned)
  static constexpr int fwd_total = li + 2 * 64 * RLS;
  // adjoint only: per-wave transpose scratch, per-wave row accumulators, reductions
  static constexpr int scr = fwd_total;             // NW x 320
  static constexpr int rows = scr + NW * 320;       // NW waves x 4 x 64 (dvm, dsm, q, u)
  static constexpr int qxr = rows + NW * 4 * 64;    // 64 x DQ  (workgroup QX)
  static constexpr int misc = qxr + 64 * DQ;        // NW x (2 DQ + 3)
  static constexpr int gacc = ((misc + NW * (2 * DQ + 3) + 3) / 4) * 4;   // NW x 10 G tiles
  static constexpr int adj_total = gacc + (FG ? NW * kGTiles * 256 : 0);
};

// stage zs, norms, q(u) moments (stage_inducing) and L^{-1} (zero padded to 64 x 64)
template <int DQ>
GPK_DEVICE void stage_reg(const float* Z, const float* ls, const float* vmean, const float* vstd,
                          const double* Linv, int M, int D, float* sm) {
  using L = RegLds<DQ>;
  stage_inducing(Z, ls, vmean, vstd, M, D, 64, DQ, L::ZS, sm + L::zs, sm + L::zn, sm + L::cm,
                 sm + L::vm, sm + L::sm1, sm + L::li);   // (L^{-1} is staged afterwards)
  double* li = (double*)(sm + L::li);
  for (int base = 0; base < 64 * 64; base += 8 * (int)blockDim.x) {   // 8 loads in flight
    double v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int e = base + u * blockDim.x + threadIdx.x, r = e >> 6, c = e & 63;
      v[u] = Linv[(e < 64 * 64 && r < M && c < M) ? (size_t)r * M + c : 0];
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int e = base + u * blockDim.x + threadIdx.x, r = e >> 6, c = e & 63;
      if (e < 64 * 64) li[r * RLS + c] = (r < M && c < M) ? v[u] : 0.0;
    }
  }
  lds_barrier();
}

GPK_DEVICE int pi_row(int x) { return (x >> 2) + 4 * (x & 3); }


// Points i0 + 16q + c of window b: Gram B operands xb[q][s] = xs[i][4s + g], squared
// norms (full, every lane), and optionally x . w (full).
template <int DQ>
struct RegPoints {
  float xb[2][DQ / 4];
  float xn[2];
  float lin[2];
};

template <int DQ, bool LIN>
GPK_DEVICE void load_points(const float* X, int N, int D, int b, int i0, const float (&il)[DQ / 4],
                            const float (&cmv)[DQ / 4], const float (&wv)[DQ / 4], RegPoints<DQ>& P) {
  const int lane = threadIdx.x & 63, c = lane & 15, g = lane >> 4;
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    const int i = i0 + 16 * q + c;
    const bool ok = i < N;
    const float* xr = X + ((size_t)b * N + (ok ? i : 0)) * D;
    float nn = 0.f, lw = 0.f;
#pragma unroll
    for (int s = 0; s < DQ / 4; ++s) {
      const int d = 4 * s + g;
      const float raw = (ok && d < D) ? xr[d] : 0.f;
      const float v = (d < D) ? raw * il[s] - cmv[s] : 0.f;
      P.xb[q][s] = ok ? v : 0.f;
      nn = __builtin_fmaf(P.xb[q][s], P.xb[q][s], nn);
      if (LIN) lw = __builtin_fmaf(raw, wv[s], lw);
    }
    nn += __shfl_xor(nn, 16, 64);
    nn += __shfl_xor(nn, 32, 64);
    P.xn[q] = nn;
    if (LIN) {
      lw += __shfl_xor(lw, 16, 64);
      lw += __shfl_xor(lw, 32, 64);
      P.lin[q] = lw;
    }
  }
}

// K_ZX tiles (register r <-> row 16 rt + g + 4r, column 16q + c), zero outside M x N
template <int DQ>
GPK_DEVICE void build_k_reg(const float* sm, const RegPoints<DQ>& P, int M, int N, int i0, float s2,
                            f32x4 (&K)[4][2]) {
  using L = RegLds<DQ>;
  const int lane = threadIdx.x & 63, c = lane & 15, g = lane >> 4;
  const float* zs = sm + L::zs;
  const float* zn = sm + L::zn;
#pragma unroll
  for (int rt = 0; rt < 4; ++rt) {
    float za[DQ / 4];
#pragma unroll
    for (int s = 0; s < DQ / 4; ++s) za[s] = zs[(16 * rt + pi_row(c)) * L::ZS + 4 * s + g];
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = 0; s < DQ / 4; ++s) acc = mfma32(za[s], P.xb[q][s], acc);
      const bool ok = i0 + 16 * q + c < N;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int p = 16 * rt + g + 4 * r;
        const float d2 = __builtin_fmaxf(zn[p] + P.xn[q] - 2.f * acc[r], 0.f);
        K[rt][q][r] = (ok && p < M) ? s2 * __builtin_amdgcn_exp2f(kNHalfLog2e * d2) : 0.f;
      }
    }
  }
}

// A = L^{-1} K (fp64 MFMA, k-order m = 16 kb + g + 4u; L^{-1} lower: kb <= rt), one row
// tile at a time, cast to fp32 as the reference does (A.float()): the f64 accumulators of
// only one row tile are live at a time.
template <int DQ>
GPK_DEVICE void linv_times_k(const float* sm, const f32x4 (&K)[4][2], f32x4 (&A)[4][2]) {
  using L = RegLds<DQ>;
  const int lane = threadIdx.x & 63, c = lane & 15, g = lane >> 4;
  const double* li = (const double*)(sm + L::li);
#pragma unroll
  for (int rt = 0; rt < 4; ++rt) {
    f64x4 acc[2] = {f64x4{0.0, 0.0, 0.0, 0.0}, f64x4{0.0, 0.0, 0.0, 0.0}};
#pragma unroll
    for (int kb = 0; kb <= rt; ++kb)
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const double la = li[(16 * rt + c) * RLS + 16 * kb + g + 4 * u];
#pragma unroll
        for (int q = 0; q < 2; ++q) acc[q] = mfma64(la, (double)K[kb][q][u], acc[q]);
      }
#pragma unroll
    for (int q = 0; q < 2; ++q)
#pragma unroll
      for (int r = 0; r < 4; ++r) A[rt][q][r] = (float)acc[q][r];
  }
}

// per-lane constants of the dims this lane touches as a Gram operand: 4s + g
template <int DQ>
GPK_DEVICE void dim_consts(const float* sm, const float* ls, const float* w, int D, float (&il)[DQ / 4],
                           float (&cmv)[DQ / 4], float (&wv)[DQ / 4]) {
  using L = RegLds<DQ>;
  const int g = (threadIdx.x & 63) >> 4;
  // every load issued first (clamped in-bounds addresses), then masked
  float lv[DQ / 4], wl[DQ / 4];
#pragma unroll
  for (int s = 0; s < DQ / 4; ++s) {
    const int d = 4 * s + g, dc = d < D ? d : 0;
    lv[s] = ls[dc];
    wl[s] = w != nullptr ? w[dc] : 0.f;
  }
#pragma unroll
  for (int s = 0; s < DQ / 4; ++s) {
    const int d = 4 * s + g;
    il[s] = d < D ? 1.f / lv[s] : 0.f;
    cmv[s] = sm[L::cm + d];
    wv[s] = d < D ? wl[s] : 0.f;
  }
}

template <int DQ>
__global__ void __launch_bounds__(256, GPK_FWD_OCC)
gpk_var_fwd_r_kernel(const float* __restrict__ X, const float* __restrict__ Z,
                     const double* __restrict__ Linv, const float* __restrict__ vmean,
                     const float* __restrict__ vstd, const float* __restrict__ hyp, int B, int N,
                     int M, int D, float* __restrict__ mean_out, float* __restrict__ var_out,
                     int* __restrict__ flags) {
  using L = RegLds<DQ>;
  extern __shared__ __attribute__((aligned(16))) float vsm[];
  const float s2 = hyp[0], jit = hyp[2], b0 = hyp[3];
  const float* w = hyp + 4;
  const float* ls = hyp + 4 + D;
  stage_reg<DQ>(Z, ls, vmean, vstd, Linv, M, D, vsm);
  const int lane = threadIdx.x & 63, c = lane & 15, g = lane >> 4;
  const int wave = threadIdx.x >> 6;
  float il[DQ / 4], cmv[DQ / 4], wv[DQ / 4];
  dim_consts<DQ>(vsm, ls, w, D, il, cmv, wv);
  const int nch = (N + 31) / 32;
  const long long total = (long long)B * nch;
  int clamped = 0;
  for (long long t = (long long)blockIdx.x * 4 + wave; t < total; t += (long long)gridDim.x * 4) {
    const int b = (int)(t / nch), i0 = (int)(t - (long long)b * nch) * 32;
    const float* sm = fresh_lds(vsm);
    const float* vm = sm + L::vm;
    const float* sm1 = sm + L::sm1;
    RegPoints<DQ> P;
    load_points<DQ, true>(X, N, D, b, i0, il, cmv, wv, P);
    f32x4 K[4][2];
    build_k_reg<DQ>(sm, P, M, N, i0, s2, K);
    f32x4 A[4][2];
    linv_times_k<DQ>(sm, K, A);
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      float mp = 0.f, vp = 0.f;
#pragma unroll
      for (int rt = 0; rt < 4; ++rt)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int p = 16 * rt + g + 4 * r;
          const float a32 = A[rt][q][r];   // A is cast to fp32 (reference)
          mp = __builtin_fmaf(a32, vm[p], mp);
          vp = __builtin_fmaf(a32 * a32, sm1[p], vp);
        }
      mp += __shfl_xor(mp, 16, 64);
      mp += __shfl_xor(mp, 32, 64);
      vp += __shfl_xor(vp, 16, 64);
      vp += __shfl_xor(vp, 32, 64);
      const int i = i0 + 16 * q + c;
      if (g == q && i < N) {
        float var_i = s2 + jit + vp;
        if (var_i < 1e-6f) { var_i = 1e-6f; clamped = 1; }   // MVN.variance clamp (fp32)
        mean_out[(size_t)b * N + i] = mp + (P.lin[q] + b0);
        var_out[(size_t)b * N + i] = var_i;
      }
    }
  }
  if (flags != nullptr && clamped)
    (void)__hip_atomic_fetch_or(flags, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// FG (the K-Gram folded in, NW = 8): the same pass also accumulates the K-Gram partials of
// gpk_var_kgram_r_kernel -- G = K_ZX diag(gvar) K_ZX^T (10 lower tiles, per-wave fp32 in LDS)
// and u = sum gmean K_ZX -- from the K_ZX tiles it already holds, so X is read once per
// adjoint instead of twice and the clamp-masked gvar never goes to HBM. The K-Gram partial
// follows the adjoint partial in the workgroup's row (one reduction launch for both), and
// block 0 writes the centre cm for gpk_var_fin_kernel.

#ifndef GPK_ADJR_STAMPS
#define GPK_ADJR_STAMPS 0   // dev builds: per-phase s_memtime cycle totals per wave (gpk_dev_adjr_stamps)
#endif
#if GPK_ADJR_STAMPS
__device__ unsigned g_adjr_st[4096 * 16];
extern "C" int gpk_dev_adjr_stamps(unsigned* host, int n) {
  return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(g_adjr_st), (size_t)n * sizeof(unsigned), 0,
                                  hipMemcpyDeviceToHost);
}
#endif
#ifndef GPK_ADJR_SKIP
#define GPK_ADJR_SKIP 0   // timing-only ablations (wrong results): 1 G, 2 dK, 4 Q^T zs, 8 QX, 16 dX, 64 A
#endif
#ifndef GPK_ADJR_DK32
#define GPK_ADJR_DK32 1   // dK = L^{-T} dA on f32 MFMA (0: fp64, the round-5 form)
#endif
template <int DQ, int NW, bool FG>
__global__ void __launch_bounds__(64 * NW, 8 / NW)
gpk_var_adj_r_kernel(const float* __restrict__ X, const float* __restrict__ Z,
                     const double* __restrict__ Linv, const float* __restrict__ vmean,
                     const float* __restrict__ vstd, const float* __restrict__ hyp,
                     const float* __restrict__ gmean, const float* __restrict__ gvar, int B, int N,
                     int M, int D, long long BN, float* __restrict__ wsgv,
                     float* __restrict__ wspart, float* __restrict__ cm_out, float* __restrict__ dX) {
  using L = RegLds<DQ, NW, FG>;
  constexpr int NDT = DQ / 16;
  extern __shared__ __attribute__((aligned(16))) float vsm[];
  const float s2 = hyp[0], jit = hyp[2];
  const float* w = hyp + 4;
  const float* ls = hyp + 4 + D;
  const int tid = threadIdx.x, lane = tid & 63, c = lane & 15, g = lane >> 4;
  const int wave = tid >> 6;
  stage_reg<DQ>(Z, ls, vmean, vstd, Linv, M, D, vsm);
  float* rows = vsm + L::rows + wave * 4 * 64;    // this wave's dvm | dsm | q | u accumulators
  for (int e = lane; e < 4 * 64; e += 64) rows[e] = 0.f;
  float* scr = vsm + L::scr + wave * 320;
  float* ga = vsm + L::gacc + wave * (kGTiles * 256);   // FG: this wave's G tiles (acc order)
  if constexpr (FG)
    for (int e = lane; e < kGTiles * 64; e += 64) *(f32x4*)(ga + 4 * e) = f32x4{0.f, 0.f, 0.f, 0.f};
  float il[DQ / 4], cmv[DQ / 4], wv[DQ / 4];
  dim_consts<DQ>(vsm, ls, nullptr, D, il, cmv, wv);
  // constants of the dims 16 dt + c (QX / dX operands)
  float ilc[NDT], cmc[NDT], wc[NDT];
#pragma unroll
  for (int dt = 0; dt < NDT; ++dt) {
    const int d = 16 * dt + c;
    const float lsv = ls[d < D ? d : 0], wv_ = w[d < D ? d : 0];   // unconditional loads
    ilc[dt] = d < D ? 1.f / lsv : 0.f;
    cmc[dt] = vsm[L::cm + d];
    wc[dt] = d < D ? wv_ : 0.f;
  }
  f32x4 qx[4][NDT];
#pragma unroll
  for (int rt = 0; rt < 4; ++rt)
#pragma unroll
    for (int dt = 0; dt < NDT; ++dt) qx[rt][dt] = f32x4{0.f, 0.f, 0.f, 0.f};
  float rx2[NDT] = {}, gx[NDT] = {};
  float sumQ = 0.f, sumgv = 0.f, sumgm = 0.f;

  const int nch = (N + 31) / 32;
  const long long total = (long long)B * nch;
#if GPK_ADJR_STAMPS
  unsigned long long st_acc[10] = {}, st_last = __builtin_amdgcn_s_memtime();
#define GPK_ADJR_ST(k)                                          \
  {                                                             \
    __builtin_amdgcn_sched_barrier(0);                          \
    const unsigned long long _n = __builtin_amdgcn_s_memtime(); \
    st_acc[k] += _n - st_last;                                  \
    st_last = _n;                                               \
    __builtin_amdgcn_sched_barrier(0);                          \
  }
#else
#define GPK_ADJR_ST(k)
#endif
  for (long long t = (long long)blockIdx.x * NW + wave; t < total; t += (long long)gridDim.x * NW) {
    GPK_ADJR_ST(0)
    const int b = (int)(t / nch), i0 = (int)(t - (long long)b * nch) * 32;
    const size_t col0 = (size_t)b * N;
    const float* sm = fresh_lds(vsm);
    const float* zs = sm + L::zs;
    const float* vm = sm + L::vm;
    const float* sm1 = sm + L::sm1;
    const double* li = (const double*)(sm + L::li);
    RegPoints<DQ> P;
    load_points<DQ, false>(X, N, D, b, i0, il, cmv, wv, P);
    f32x4 K[4][2];
    build_k_reg<DQ>(sm, P, M, N, i0, s2, K);
    GPK_ADJR_ST(1)
    f32x4 A[4][2];
    if (GPK_ADJR_SKIP & 64) {
#pragma unroll
      for (int rt = 0; rt < 4; ++rt)
#pragma unroll
        for (int q = 0; q < 2; ++q) A[rt][q] = K[rt][q];
    } else {
      linv_times_k<DQ>(sm, K, A);
    }
    GPK_ADJR_ST(2)
    // variance -> clamp mask; point gradients
    float gmq[2], gvq[2];
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      float vp = 0.f;
#pragma unroll
      for (int rt = 0; rt < 4; ++rt)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float a32 = A[rt][q][r];
          vp = __builtin_fmaf(a32 * a32, sm1[16 * rt + g + 4 * r], vp);
        }
      vp += __shfl_xor(vp, 16, 64);
      vp += __shfl_xor(vp, 32, 64);
      const int i = i0 + 16 * q + c;
      const bool ok = i < N;
      const float gml = gmean[col0 + (ok ? i : 0)], gvl = gvar[col0 + (ok ? i : 0)];   // clamped
      gmq[q] = ok ? gml : 0.f;
      gvq[q] = ok ? gvl : 0.f;
      if (s2 + jit + vp < 1e-6f) gvq[q] = 0.f;   // clamp_min(1e-6): gradient masked
      if (g == 0) {
        sumgv += gvq[q];
        sumgm += gmq[q];
      }
    }
    // dA (fp32, in A's registers) and the dvmean / dvstd row partials
    f32x4 (&dA)[4][2] = A;
#pragma unroll
    for (int rt = 0; rt < 4; ++rt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int p = 16 * rt + g + 4 * r;
        const float vmp = vm[p], smp = sm1[p];
        float pm = 0.f, ps = 0.f;
#pragma unroll
        for (int q = 0; q < 2; ++q) {
          const float a32 = A[rt][q][r];
          dA[rt][q][r] = gmq[q] * vmp + 2.f * gvq[q] * smp * a32;
          pm = __builtin_fmaf(gmq[q], a32, pm);
          ps = __builtin_fmaf(gvq[q], a32 * a32, ps);
        }
        pm = row16_sum_f(pm);
        ps = row16_sum_f(ps);
        float pu = 0.f;
        if constexpr (FG) pu = row16_sum_f(__builtin_fmaf(gmq[1], K[rt][1][r], gmq[0] * K[rt][0][r]));
        if (c == 0) {
          lds_acc(rows + p, pm);
          lds_acc(rows + 64 + p, ps);
          if constexpr (FG) lds_acc(rows + 192 + p, pu);
        }
      }
    GPK_ADJR_ST(3)
    // dL^{-1} = vm u^T + 2 (s^2 - 1) o L^{-1} G with u = sum gmean K_ZX and
    // G = K_ZX diag(gvar) K_ZX^T, so neither dA nor K_ZX makes an HBM round trip
    if constexpr (FG && !(GPK_ADJR_SKIP & 1)) {
      // G(rt, rp) += sum_points K_rt diag(gv) K_rp^T: each K tile transposed through the
      // wave's scratch (points -> k), then sum_s mfma(K^T.reg[s], (gv K)^T.reg[s]) as in
      // gpk_var_kgram_r_kernel (same acc layout); the tiles live in LDS between chunks
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        float aK[4][4], aW[4][4];
#pragma unroll
        for (int rt = 0; rt < 4; ++rt) {
#pragma unroll
          for (int r = 0; r < 4; ++r) scr[lane * 5 + r] = K[rt][q][r];
          adj_lds_order();
#pragma unroll
          for (int s = 0; s < 4; ++s) aK[rt][s] = scr[((c & 3) * 16 + 4 * s + g) * 5 + (c >> 2)];
          adj_lds_order();
        }
#pragma unroll
        for (int s = 0; s < 4; ++s) {
          const float gvp = __shfl(gvq[q], 4 * s + g, 64);   // gvar of point 16 q + 4 s + g
#pragma unroll
          for (int rt = 0; rt < 4; ++rt) aW[rt][s] = aK[rt][s] * gvp;
        }
#pragma unroll
        for (int rt = 0; rt < 4; ++rt)
#pragma unroll
          for (int rp = 0; rp <= rt; ++rp) {
            f32x4* gp = (f32x4*)(ga + 4 * ((rt * (rt + 1) / 2 + rp) * 64 + lane));
            f32x4 acc = *gp;
#pragma unroll
            for (int s = 0; s < 4; ++s) acc = mfma32(aK[rt][s], aW[rp][s], acc);
            *gp = acc;
          }
      }
    } else if constexpr (!FG) {
      // the clamp-masked gvar -> workspace for gpk_var_kgram_r_kernel
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        const int i = i0 + 16 * q + c;
        if (i < N && g == 0) wsgv[col0 + i] = gvq[q];
      }
    }
    GPK_ADJR_ST(4)
    // dK = L^{-T} dA (L^{-T} upper: kb >= rt), then Q = dK o K_ZX (in K's registers). Round 6:
    // on f32 MFMA (GPK_ADJR_DK32; the reference's dK is fp64, the gradients stay ~1e-6 from the
    // fp64 oracle) with the L^{-1} columns fed in pi order, so the f32 C layout of the result
    // (row 4 g + r) holds dK row g + 4 r -- K's layout -- in register r.
#pragma unroll
    for (int rt = 0; rt < 4 && !(GPK_ADJR_SKIP & 2); ++rt) {
      if constexpr (GPK_ADJR_DK32) {
        f32x4 acc[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
        const int cp = pi16(c);
#pragma unroll
        for (int kb = rt; kb < 4; ++kb)
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            const float la = (float)li[(16 * kb + g + 4 * u) * RLS + 16 * rt + cp];
#pragma unroll
            for (int q = 0; q < 2; ++q) acc[q] = mfma32(la, dA[kb][q][u], acc[q]);
          }
#pragma unroll
        for (int q = 0; q < 2; ++q)
#pragma unroll
          for (int r = 0; r < 4; ++r) K[rt][q][r] = acc[q][r] * K[rt][q][r];
      } else {
        f64x4 acc[2] = {f64x4{0.0, 0.0, 0.0, 0.0}, f64x4{0.0, 0.0, 0.0, 0.0}};
#pragma unroll
        for (int kb = rt; kb < 4; ++kb)
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            const double la = li[(16 * kb + g + 4 * u) * RLS + 16 * rt + c];
#pragma unroll
            for (int q = 0; q < 2; ++q) acc[q] = mfma64(la, (double)dA[kb][q][u], acc[q]);
          }
#pragma unroll
        for (int q = 0; q < 2; ++q)
#pragma unroll
          for (int r = 0; r < 4; ++r) K[rt][q][r] = (float)acc[q][r] * K[rt][q][r];
      }
    }
    GPK_ADJR_ST(5)
    // r_i = sum_p Q_pi (every lane c of a column), q_p row partials, sum Q
    float rq[2];
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      float v = 0.f;
#pragma unroll
      for (int rt = 0; rt < 4; ++rt) v += (K[rt][q][0] + K[rt][q][1]) + (K[rt][q][2] + K[rt][q][3]);
      sumQ += v;
      v += __shfl_xor(v, 16, 64);
      v += __shfl_xor(v, 32, 64);
      rq[q] = v;
    }
#pragma unroll
    for (int rt = 0; rt < 4; ++rt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float v = row16_sum_f(K[rt][0][r] + K[rt][1][r]);
        if (c == 0) lds_acc(rows + 128 + 16 * rt + g + 4 * r, v);
      }
    GPK_ADJR_ST(6)
    // (Q^T zs)_i: f32 MFMA with k = p (rows g + 4r of each row tile)
    f32x4 xz[2][NDT];
#pragma unroll
    for (int q = 0; q < 2; ++q)
#pragma unroll
      for (int dt = 0; dt < NDT; ++dt) xz[q][dt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int rt = 0; rt < 4; ++rt)
#pragma unroll
      for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int dt = 0; dt < NDT; ++dt) {
          const float zb = zs[(16 * rt + g + 4 * r) * L::ZS + 16 * dt + c];
#pragma unroll
          for (int q = 0; q < 2; ++q)
            if (!(GPK_ADJR_SKIP & 4)) xz[q][dt] = mfma32(K[rt][q][r], zb, xz[q][dt]);
        }
    GPK_ADJR_ST(7)
    // QX_p += sum_i Q_pi xs_i: Q tiles transposed through LDS (k = point 4s + g)
#pragma unroll
    for (int q = 0; q < 2 && !(GPK_ADJR_SKIP & 8); ++q) {
      float xb2[4][NDT];
#pragma unroll
      for (int s = 0; s < 4; ++s)     // unconditional (clamped) loads: all in flight together
#pragma unroll
        for (int dt = 0; dt < NDT; ++dt) {
          const int i = i0 + 16 * q + 4 * s + g, d = 16 * dt + c;
          xb2[s][dt] = X[(i < N && d < D) ? (col0 + i) * D + d : 0];
        }
#pragma unroll
      for (int s = 0; s < 4; ++s)
#pragma unroll
        for (int dt = 0; dt < NDT; ++dt) {
          const int i = i0 + 16 * q + 4 * s + g, d = 16 * dt + c;
          xb2[s][dt] = (i < N && d < D) ? xb2[s][dt] * ilc[dt] - cmc[dt] : 0.f;
        }
#pragma unroll
      for (int rt = 0; rt < 4; ++rt) {
#pragma unroll
        for (int r = 0; r < 4; ++r) scr[lane * 5 + r] = K[rt][q][r];
        adj_lds_order();
        float aq[4];
#pragma unroll
        for (int s = 0; s < 4; ++s) aq[s] = scr[((c & 3) * 16 + 4 * s + g) * 5 + (c >> 2)];
        adj_lds_order();   // the next tile overwrites scr
#pragma unroll
        for (int dt = 0; dt < NDT; ++dt)
#pragma unroll
          for (int s = 0; s < 4; ++s) qx[rt][dt] = mfma32(aq[s], xb2[s][dt], qx[rt][dt]);
      }
    }
    GPK_ADJR_ST(8)
    // dX_i = ((Q^T zs)_i - xs_i r_i) / l + gmean_i w; sum_i r_i xs_i^2, sum_i gmean_i xs_i
    // (the point values are requested up front, unconditionally: clamped addresses)
    float xo[2][4][NDT];
#pragma unroll
    for (int q = 0; q < 2; ++q)
#pragma unroll
      for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int dt = 0; dt < NDT; ++dt) {
          const int i = i0 + 16 * q + 4 * g + r, d = 16 * dt + c;
          xo[q][r][dt] = X[(i < N && d < D) ? (col0 + i) * D + d : 0];
        }
    // (branch-free but for the stores: a load whose only use sits under the point / dim
    // guard is sunk into it by the compiler and waited for one point at a time)
#pragma unroll
    for (int q = 0; q < 2 && !(GPK_ADJR_SKIP & 16); ++q)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int pc = 4 * g + r;                  // point (within the tile) of register r
        const float rr = __shfl(rq[q], pc, 64);
        const float gm = __shfl(gmq[q], pc, 64);
        const int i = i0 + 16 * q + pc;
#pragma unroll
        for (int dt = 0; dt < NDT; ++dt) {
          const int d = 16 * dt + c;
          const bool ok = i < N && d < D;
          const float xv = ok ? xo[q][r][dt] * ilc[dt] - cmc[dt] : 0.f;
          const float dxv = (xz[q][dt][r] - xv * rr) * ilc[dt] + gm * wc[dt];
          if (ok) dX[(col0 + i) * D + d] = dxv;
          rx2[dt] = __builtin_fmaf(rr * xv, xv, rx2[dt]);
          gx[dt] = __builtin_fmaf(gm, xv, gx[dt]);
        }
      }
    GPK_ADJR_ST(9)
  }
#if GPK_ADJR_STAMPS
  if (lane == 0) {
#pragma unroll
    for (int k2 = 0; k2 < 10; ++k2) g_adjr_st[(blockIdx.x * NW + wave) * 16 + k2] = (unsigned)st_acc[k2];
  }
#endif
#undef GPK_ADJR_ST


  // ---- workgroup partials, summed over the waves in a fixed order:
  //   [QX (M x D) | q (M) | dvm (M) | dsm (M) | rx2 (D) | sumQ | sumgv | gx (D) | sumgm]
  float* qxr = vsm + L::qxr;
  float* misc = vsm + L::misc + wave * (2 * DQ + 3);
#pragma unroll
  for (int dt = 0; dt < NDT; ++dt) {
    float v = rx2[dt], u = gx[dt];
    v += __shfl_xor(v, 16, 64);
    v += __shfl_xor(v, 32, 64);
    u += __shfl_xor(u, 16, 64);
    u += __shfl_xor(u, 32, 64);
    if (g == 0) {
      misc[16 * dt + c] = v;
      misc[DQ + 16 * dt + c] = u;
    }
  }
  sumQ = wave_sum(sumQ);
  sumgv = wave_sum(sumgv);
  sumgm = wave_sum(sumgm);
  if (lane == 0) {
    misc[2 * DQ] = sumQ;
    misc[2 * DQ + 1] = sumgv;
    misc[2 * DQ + 2] = sumgm;
  }
  for (int wv2 = 0; wv2 < NW; ++wv2) {
    lds_barrier();
    if (wave == wv2) {
#pragma unroll
      for (int rt = 0; rt < 4; ++rt)
#pragma unroll
        for (int dt = 0; dt < NDT; ++dt)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int e = (16 * rt + 4 * g + r) * DQ + 16 * dt + c;
            qxr[e] = (wv2 == 0 ? 0.f : qxr[e]) + qx[rt][dt][r];
          }
    }
  }
  lds_barrier();
  const int P = M * D + 3 * M + 2 * D + 3;
  float* po = wspart + (size_t)blockIdx.x * (P + (FG ? kGPart : 0));
  if (FG && blockIdx.x == 0 && tid < D) cm_out[tid] = vsm[L::cm + tid];
  for (int e = tid; e < M * D; e += blockDim.x) {
    const int p = e / D, d = e - p * D;
    po[e] = qxr[p * DQ + d];
  }
  const float* rw = vsm + L::rows;
  for (int m = tid; m < M; m += blockDim.x) {
    float a = 0.f, s = 0.f, qq = 0.f;
    for (int u = 0; u < NW; ++u) {
      a += rw[u * 256 + m];
      s += rw[u * 256 + 64 + m];
      qq += rw[u * 256 + 128 + m];
    }
    po[M * D + m] = qq;
    po[M * D + M + m] = a;
    po[M * D + 2 * M + m] = s;
  }
  const float* ms = vsm + L::misc;
  for (int d = tid; d < D; d += blockDim.x) {
    float v = 0.f, u = 0.f;
    for (int k = 0; k < NW; ++k) {
      v += ms[k * (2 * DQ + 3) + d];
      u += ms[k * (2 * DQ + 3) + DQ + d];
    }
    po[M * D + 3 * M + d] = v;
    po[M * D + 3 * M + D + 2 + d] = u;
  }
  if (tid == 0) {
    float a = 0.f, v = 0.f, u = 0.f;
    for (int k = 0; k < NW; ++k) {
      a += ms[k * (2 * DQ + 3) + 2 * DQ];
      v += ms[k * (2 * DQ + 3) + 2 * DQ + 1];
      u += ms[k * (2 * DQ + 3) + 2 * DQ + 2];
    }
    po[M * D + 3 * M + D] = a;
    po[M * D + 3 * M + D + 1] = v;
    po[M * D + 3 * M + 2 * D + 2] = u;
  }
  if constexpr (FG) {
    // K-Gram partial [G lower tiles (10 x 256, acc order) | u (64)], waves in a fixed order
    const float* gw = vsm + L::gacc;
    float* pg = po + P;
    for (int e = tid; e < kGTiles * 256; e += blockDim.x) {
      const int t2 = e >> 8, r = (e >> 6) & 3, ln = e & 63;
      float v = 0.f;
#pragma unroll
      for (int k = 0; k < NW; ++k) v += gw[k * (kGTiles * 256) + 4 * (t2 * 64 + ln) + r];
      pg[e] = v;
    }
    for (int m = tid; m < 64; m += blockDim.x) {
      float v = 0.f;
#pragma unroll
      for (int k = 0; k < NW; ++k) v += rw[k * 256 + 192 + m];
      pg[kGTiles * 256 + m] = v;
    }
  }
}

// dL^{-1}[p][k] = vm_p u_k + 2 (s_p^2 - 1) (L^{-1} G)[p][k]  (k <= p < M; upper zero) from the
// reduced totals (fp64). One workgroup: G (symmetric, from its lower tiles) in LDS, wave w
// forms the 16-row block w of L^{-1} G on fp64 MFMA with its L^{-1} operands requested up
// front (the triangular k-range: jb <= w).
// (256 threads; Gs: 64 x 65 doubles, us: 64 doubles of LDS)
GPK_DEVICE void var_gdl_block(const double* __restrict__ gtot, const double* __restrict__ Linv,
                              const float* __restrict__ vmean, const float* __restrict__ vstd, int M,
                              double* __restrict__ dLinv, double (*Gs)[65], double* us) {
  const int tid = threadIdx.x, lane = tid & 63, c = lane & 15, g = lane >> 4;
  const int w = tid >> 6;
  // the 10 tile elements of this thread requested together (acc order: tile, reg r, lane)
  double gv[kGTiles];
#pragma unroll
  for (int t2 = 0; t2 < kGTiles; ++t2) gv[t2] = gtot[t2 * 256 + tid];
  const double uv = gtot[kGTiles * 256 + (tid & 63)];
#pragma unroll
  for (int t2 = 0; t2 < kGTiles; ++t2) {
    constexpr int kRt[kGTiles] = {0, 1, 1, 2, 2, 2, 3, 3, 3, 3};
    const int rt = kRt[t2], rp = t2 - rt * (rt + 1) / 2;
    const int r = tid >> 6, ln = tid & 63;
    const int row = 16 * rt + 4 * (ln >> 4) + r, col = 16 * rp + (ln & 15);   // f32 acc: row 4g + r
    if (rt == rp && row < col) continue;   // one writer per element: deterministic
    Gs[row][col] = gv[t2];
    Gs[col][row] = gv[t2];
  }
  if (tid < 64) us[tid] = uv;
  // A operands L^{-1}[16 w + c][16 jb + 4 s + g] for jb <= w, requested before the barrier
  double la[4][4];
#pragma unroll
  for (int jb = 0; jb < 4; ++jb)
#pragma unroll
    for (int s4 = 0; s4 < 4; ++s4) {
      const int p = 16 * w + c, j = 16 * jb + 4 * s4 + g;
      const bool ok = jb <= w && p < M && j < M;
      const double v = Linv[ok ? (size_t)p * M + j : 0];
      la[jb][s4] = ok ? v : 0.0;
    }
  lds_barrier();
#pragma unroll
  for (int kb = 0; kb < 4; ++kb) {
    f64x4 acc = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int jb = 0; jb < 4; ++jb)
#pragma unroll
      for (int s4 = 0; s4 < 4; ++s4) acc = mfma64(la[jb][s4], Gs[16 * jb + 4 * s4 + g][16 * kb + c], acc);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int p = 16 * w + g + 4 * r, k = 16 * kb + c;
      if (p < M && k < M) {
        const double sd = (double)vstd[p];
        dLinv[(size_t)p * M + k] = k <= p ? (double)vmean[p] * us[k] + 2.0 * (sd * sd - 1.0) * acc[r] : 0.0;
      }
    }
  }
}


// ---------------------------------------------------------------------------
// launchers
// ---------------------------------------------------------------------------
template <int MB>
size_t var_fwd_lds(int D) {
  using G = VarGeo<MB>;
  const int Dq = dq_of(D), ds = Dq + 2;
  return (size_t)(G::MP * ds + G::TW * ds + G::MP + G::TW + 2 * G::MP + Dq + G::MP * G::TW +
                  2 * G::WR * G::TW) * sizeof(float);
}

template <int MB, int DQ>
size_t var_adj_lds() {
  using G = VarGeo<MB>;
  const int Dq = DQ, ds = Dq + 2;
  const size_t kl = (size_t)G::MP * G::TW > (size_t)G::WR * G::TW * Dq ? (size_t)G::MP * G::TW
                                                                       : (size_t)G::WR * G::TW * Dq;
  const size_t da = (size_t)G::MP * G::TW > (size_t)G::TW * G::QST ? (size_t)G::MP * G::TW
                                                                   : (size_t)G::TW * G::QST;
  return ((size_t)G::MP * ds + G::TW * ds + G::MP + G::TW + 2 * G::MP + Dq + 3 * G::TW + G::MP +
          2 * G::WC * G::MP + 2 * 256 + 2 * G::WR * G::TW + kl + da) * sizeof(float);
}

// hipFuncSetAttribute once per kernel instantiation (thread-safe; the C ABI has no
// mutable global state beyond this idempotent one-time setup).
template <auto Kernel, int Bytes = 160 * 1024>
void set_lds_once() {
  static std::once_flag once;  // one flag per kernel instantiation
  std::call_once(once, [] {
    (void)hipFuncSetAttribute((const void*)Kernel, hipFuncAttributeMaxDynamicSharedMemorySize, Bytes);
    (void)hipGetLastError();   // never leave a sticky error for the launch check to pick up
  });
}

// Workgroups for a chunk list: every chunk once, at most ~4 per CU so the inducing-point
// staging of a workgroup is amortised over several chunks.
int chunk_grid(long long nchunks, int per_cu) {
  const long long cap = 256LL * per_cu;
  return (int)(nchunks < cap ? nchunks : cap);
}

template <int MB>
int launch_var_fwd(const GpkVarArgs& a, int* flags, hipStream_t stream) {
  using G = VarGeo<MB>;
  const size_t lds = var_fwd_lds<MB>(a.D);
  if (lds > 160 * 1024) return -11;
  set_lds_once<gpk_var_fwd_kernel<MB>>();
  const long long nch = (long long)a.B * ((a.N + G::TW - 1) / G::TW);
  if (nch > 0x7fffffffLL) return -8;
  hipLaunchKernelGGL((gpk_var_fwd_kernel<MB>), dim3(chunk_grid(nch, 4)), dim3(256), lds, stream,
                     a.X, a.Z, a.Linv, a.vmean, a.vstd, a.hyp, a.N, a.M, a.D, (int)nch, a.mean,
                     a.var, flags);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return (int)e;
  if (a.ell != nullptr) {
    hipLaunchKernelGGL(gpk_var_ell_kernel, dim3(a.B), dim3(256), 0, stream, a.mean, a.var, a.y,
                       a.hyp, a.N, a.ell);
    e = hipGetLastError();
  }
  return e == hipSuccess ? 0 : (int)e;
}

// The saved-state adjoint (gpk_var_adjs_l_kernel + K-Gram) serves M > 64 when its LDS plan fits
// (D <= 32 at M = 256); the training forward then keeps A for it.
// 0: A/B builds with the LDS-tiled forward for M > 64 (that forward keeps no state, so the
// saved-state training pair is off too: var_saved_path is false and saved_bytes 0)
#ifndef GPK_VAR_LREG
#define GPK_VAR_LREG 1
#endif
template <int MB, int DQ>
constexpr bool var_saved_fits() {
  if constexpr (MB >= 5) return LAdjGeo<MB, DQ>::fits && (size_t)LGramGeo<MB, DQ>::total * 4 <= 160 * 1024;
  return false;
}
template <int MB, int DQ>
bool var_saved_path(int M) { return GPK_VAR_LREG && var_saved_fits<MB, DQ>() && M > 64; }

template <int MB, int DQ>
int launch_var_fwd_l(const GpkVarArgs& a, int* flags, hipStream_t stream) {
  using G = LGeo<MB, DQ>;
  const size_t lds = (size_t)G::total * sizeof(float);
  if (lds > 160 * 1024) return -11;
  set_lds_once<gpk_var_fwd_l_kernel<MB, DQ>>();
  const long long nch = (long long)a.B * ((a.N + LTW - 1) / LTW);
  if (nch > 0x7fffffffLL) return -8;
  const int per_cu = G::NWV <= 4 ? 2 : 1;   // <= 2 waves per SIMD (256 VGPRs: L^{-1} resident)
  // the training forward keeps A for the adjoint when the saved-state adjoint serves this shape
  float* saved = (a.saved != nullptr && var_saved_path<MB, DQ>(a.M)) ? a.saved : nullptr;
  hipLaunchKernelGGL((gpk_var_fwd_l_kernel<MB, DQ>), dim3(chunk_grid(nch, per_cu)), dim3(G::NT), lds,
                     stream, a.X, a.Z, a.Linv, a.vmean, a.vstd, a.hyp, a.N, a.M, a.D, (int)nch,
                     a.mean, a.var, flags, saved);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return (int)e;
  if (a.ell != nullptr) {
    hipLaunchKernelGGL(gpk_var_ell_kernel, dim3(a.B), dim3(256), 0, stream, a.mean, a.var, a.y,
                       a.hyp, a.N, a.ell);
    e = hipGetLastError();
  }
  return e == hipSuccess ? 0 : (int)e;
}


struct AdjPlan {
  int nchunks, nwg, P, ntiles, nsplit;
  long long BN, cols_per_split;
  size_t off_dA, off_K, off_part, off_tot, off_dl, total;  // byte offsets
  size_t fin_lds;
};

// register-resident path (M <= 64, D <= 32): 32-point chunks, one per wave, 4 waves per
// workgroup, 2 workgroups per CU
#ifndef GPK_VAR_REG
#define GPK_VAR_REG 1   // 0: A/B builds without the register-resident path
#endif
GPK_HOST_DEVICE_INLINE bool var_reg_path(int M, int D) { return GPK_VAR_REG && M <= 64 && D <= 32; }
constexpr int kAdjRWaves = 8;   // waves per register-path adjoint workgroup (K-Gram folded in)

AdjPlan adj_plan_common(AdjPlan p, int B, int N, int M, int D);

template <int MB, int DQ>
constexpr bool var_adj_lreg_fits() {
  if constexpr (MB >= 5) return LAdjGeo<MB, DQ>::fits;
  return false;
}
GPK_HOST_DEVICE_INLINE int adj_dq(int D) { return D <= 32 ? 32 : 64; }

template <int MB>
AdjPlan adj_plan(int B, int N, int M, int D) {
  using G = VarGeo<MB>;
  AdjPlan p{};
  if constexpr (MB >= 5) {
    const bool fits = adj_dq(D) == 32 ? var_adj_lreg_fits<MB, 32>() : var_adj_lreg_fits<MB, 64>();
    const bool small_ws = (long long)M * B * N * 4 < (1LL << 31);   // 32-bit buffer offsets
    if (GPK_VAR_LREG && M > 64 && fits && small_ws) {   // persistent, <= 2 waves / SIMD
      const long long nch = (long long)B * ((N + LTW - 1) / LTW);
      p.nchunks = (int)nch;
      p.nwg = chunk_grid(nch, LAdjGeo<MB, 32>::NWV <= 4 ? 2 : 1);
      return adj_plan_common(p, B, N, M, D);
    }
  }
  if (var_reg_path(M, D)) {
    // workspace (the K-Gram folded into the adjoint): the centre (64) | rows of
    // [adjoint | K-Gram] partials | their fp64 totals (the K-Gram totals at + P)
    const long long nch = (long long)B * ((N + 31) / 32);
    p.nchunks = (int)nch;
    // one workgroup per CU (8 waves, K-Gram folded in)
    const long long nwg_max = 2048 / kAdjRWaves;
    p.nwg = (int)((nch + kAdjRWaves - 1) / kAdjRWaves < nwg_max ? (nch + kAdjRWaves - 1) / kAdjRWaves : nwg_max);
    p = adj_plan_common(p, B, N, M, D);
    auto al = [](size_t x) { return (x + 255) & ~(size_t)255; };
    size_t o = 0;
    p.off_dA = o; o = al(o + 64 * sizeof(float));
    p.off_K = o;
    p.off_part = o; o = al(o + (size_t)p.nwg * (p.P + kGPart) * sizeof(float));
    p.off_tot = o; o = al(o + (size_t)(p.P + kGPart) * sizeof(double));
    p.off_dl = o;
    p.total = o;
    return p;
  }
  p.nchunks = B * ((N + G::TW - 1) / G::TW);
  p.nwg = chunk_grid(p.nchunks, 2);
  return adj_plan_common(p, B, N, M, D);
}

AdjPlan adj_plan_common(AdjPlan p, int B, int N, int M, int D) {
  p.P = M * D + 3 * M + 2 * D + 3;
  p.fin_lds = (size_t)M * D * sizeof(float);
  p.BN = (long long)B * N;
  const int MT = (M + 63) / 64;
  p.ntiles = MT * (MT + 1) / 2;
  long long want = 512 / p.ntiles;
  if (want < 1) want = 1;
  long long cps = (p.BN + want - 1) / want;
  cps = ((cps + DLKC - 1) / DLKC) * DLKC;
  if (cps < DLKC) cps = DLKC;
  p.cols_per_split = cps;
  p.nsplit = (int)((p.BN + cps - 1) / cps);
  auto al = [](size_t x) { return (x + 255) & ~(size_t)255; };
  size_t o = 0;
  p.off_dA = o; o = al(o + (size_t)M * p.BN * sizeof(float));
  p.off_K = o; o = al(o + (size_t)M * p.BN * sizeof(float));
  p.off_part = o; o = al(o + (size_t)p.nwg * p.P * sizeof(float));
  p.off_tot = o; o = al(o + (size_t)p.P * sizeof(double));
  p.off_dl = o; o = al(o + (size_t)p.nsplit * p.ntiles * 4096 * sizeof(double));
  p.total = o;
  return p;
}

template <int DQ>
int launch_var_fwd_r(const GpkVarArgs& a, int* flags, hipStream_t stream) {
  const size_t lds = (size_t)RegLds<DQ>::fwd_total * sizeof(float);
  set_lds_once<gpk_var_fwd_r_kernel<DQ>>();
  const long long nch = (long long)a.B * ((a.N + 31) / 32);
  const long long nwg = (nch + 3) / 4 < 768 ? (nch + 3) / 4 : 768;
  hipLaunchKernelGGL((gpk_var_fwd_r_kernel<DQ>), dim3((unsigned)nwg), dim3(256), lds, stream, a.X, a.Z,
                     a.Linv, a.vmean, a.vstd, a.hyp, a.B, a.N, a.M, a.D, a.mean, a.var, flags);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return (int)e;
  if (a.ell != nullptr) {
    hipLaunchKernelGGL(gpk_var_ell_kernel, dim3(a.B), dim3(256), 0, stream, a.mean, a.var, a.y,
                       a.hyp, a.N, a.ell);
    e = hipGetLastError();
  }
  return e == hipSuccess ? 0 : (int)e;
}

int launch_var_adj_tail(const GpkVarAdjArgs& a, const AdjPlan& p, hipStream_t stream);

template <int MB, int DQ>
int launch_var_adj_saved(const GpkVarAdjArgs& a, hipStream_t stream);

template <int MB, int DQ>
int launch_var_adj(const GpkVarAdjArgs& a, hipStream_t stream) {
  if (a.saved != nullptr) {
    if (!var_saved_path<MB, DQ>(a.M)) return -13;
    return launch_var_adj_saved<MB, DQ>(a, stream);
  }
  const AdjPlan p = adj_plan<MB>(a.B, a.N, a.M, a.D);
  char* ws = (char*)a.ws;
  float* wsdA = (float*)(ws + p.off_dA);
  float* wsK = (float*)(ws + p.off_K);
  float* wspart = (float*)(ws + p.off_part);
  if (var_reg_path(a.M, a.D)) {
    constexpr int RQ = DQ <= 16 ? 16 : 32;
    float* wsgv = wsdA;   // FG: the centre cm (D floats)
    double* tot = (double*)(ws + p.off_tot);
    constexpr int NW = kAdjRWaves;
    constexpr bool FG = true;   // the K-Gram folded into the adjoint (round 5)
    double* gtot = tot + p.P;   // the K-Gram totals after the adjoint totals
    static_assert(RegLds<RQ, NW, FG>::adj_total * sizeof(float) <= 160 * 1024, "LDS per workgroup");
    const size_t lds = (size_t)RegLds<RQ, NW, FG>::adj_total * sizeof(float);
    set_lds_once<gpk_var_adj_r_kernel<RQ, NW, FG>>();
    hipLaunchKernelGGL((gpk_var_adj_r_kernel<RQ, NW, FG>), dim3(p.nwg), dim3(64 * NW), lds, stream, a.X,
                       a.Z, a.Linv, a.vmean, a.vstd, a.hyp, a.gmean, a.gvar, a.B, a.N, a.M, a.D, p.BN,
                       wsgv, wspart, wsgv, a.dX);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return (int)e;
    // one fixed-order reduction of the [adjoint | K-Gram] rows; dL^{-1} in the output launch
    const int PR = p.P + kGPart;
    hipLaunchKernelGGL(gpk_var_red_kernel, dim3((PR + 31) / 32), dim3(256), 0, stream, wspart, p.nwg, PR,
                       tot, nullptr, 0, 0, 0, nullptr, nullptr, 0, nullptr);
    if ((e = hipGetLastError()) != hipSuccess) return (int)e;
    const VarGdlArgs gd{gtot, a.Linv, a.vmean, a.vstd, a.dLinv, 0};
    return launch_var_fin(a.Z, a.vstd, a.hyp, tot, a.M, a.D, a.dZ, a.dpar, stream, wsgv, &gd);
  }
  if constexpr (var_adj_lreg_fits<MB, DQ>()) {
    if (GPK_VAR_LREG && a.M > 64 && (long long)a.M * p.BN * 4 < (1LL << 31)) {
      using LG = LAdjGeo<MB, DQ>;
      set_lds_once<gpk_var_adja_l_kernel<MB, DQ>>();
      set_lds_once<gpk_var_adjk_l_kernel<MB, DQ>>();
      hipLaunchKernelGGL((gpk_var_adja_l_kernel<MB, DQ>), dim3(p.nwg), dim3(LG::NT),
                         (size_t)LG::a_total * sizeof(float), stream, a.X, a.Z, a.Linv, a.vmean,
                         a.vstd, a.hyp, a.gmean, a.gvar, a.N, a.M, a.D, p.nchunks, p.BN, wsdA, wsK,
                         wspart);
      hipError_t e = hipGetLastError();
      if (e != hipSuccess) return (int)e;
      hipLaunchKernelGGL((gpk_var_adjk_l_kernel<MB, DQ>), dim3(p.nwg), dim3(LG::NT),
                         (size_t)LG::k_total * sizeof(float), stream, a.X, a.Z, a.Linv, a.vmean,
                         a.vstd, a.hyp, a.gmean, a.N, a.M, a.D, p.nchunks, p.BN, wsdA, wsK, wspart,
                         a.dX);
      e = hipGetLastError();
      if (e != hipSuccess) return (int)e;
      return launch_var_adj_tail(a, p, stream);
    }
  }
  const size_t lds = var_adj_lds<MB, DQ>();
  if (lds > 160 * 1024) return -12;
  set_lds_once<gpk_var_adj_kernel<MB, DQ>>();
  hipLaunchKernelGGL((gpk_var_adj_kernel<MB, DQ>), dim3(p.nwg), dim3(256), lds, stream, a.X, a.Z,
                     a.Linv, a.vmean, a.vstd, a.hyp, a.gmean, a.gvar, a.N, a.M, a.D, p.nchunks,
                     p.BN, wsdA, wsK, wspart, a.dX);
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) return (int)e;
  return launch_var_adj_tail(a, p, stream);
}

int launch_var_fin(const float* Z, const float* vstd, const float* hyp, const double* tot, int M, int D,
                   float* dZ, float* dpar, hipStream_t stream, const float* cm_in,
                   const VarGdlArgs* gd) {
  const int nblk = (M + kFinRows - 1) / kFinRows;
  set_lds_once<gpk_var_fin_kernel, 64 * 1024>();   // + ~3.3 KB static
  size_t lds = (size_t)M * D * sizeof(float);
  VarGdlArgs g{};
  int ngd = 0;
  if (gd != nullptr) {
    g = *gd;
    if (g.MB == 0) {
      ngd = 1;
      const size_t gl = (64 * 65 + 64) * sizeof(double);
      if (lds < gl) lds = gl;
    } else {
      ngd = (int)(((long long)M * M + 255) / 256);
    }
  }
  hipLaunchKernelGGL(gpk_var_fin_kernel, dim3(nblk + 1 + ngd), dim3(256), lds, stream, Z,
                     vstd, hyp, tot, M, D, dZ, dpar, cm_in, g);
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? 0 : (int)e;
}

// dL^{-1} GEMM, the fixed-order reductions and the outputs (both adjoint paths)
int launch_var_adj_tail(const GpkVarAdjArgs& a, const AdjPlan& p, hipStream_t stream) {
  char* ws = (char*)a.ws;
  float* wsdA = (float*)(ws + p.off_dA);
  float* wsK = (float*)(ws + p.off_K);
  float* wspart = (float*)(ws + p.off_part);
  double* tot = (double*)(ws + p.off_tot);
  double* dl = (double*)(ws + p.off_dl);
  hipLaunchKernelGGL(gpk_dlinv_kernel, dim3(p.ntiles * p.nsplit), dim3(256), 0, stream, wsdA, wsK,
                     a.M, p.BN, p.ntiles, p.cols_per_split, dl);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return (int)e;
  const long long nred = (p.P + 31) / 32 + ((long long)a.M * a.M + 31) / 32;
  hipLaunchKernelGGL(gpk_var_red_kernel, dim3((unsigned)nred), dim3(256), 0, stream,
                     wspart, p.nwg, p.P, tot, dl, p.nsplit, p.ntiles, a.M, a.dLinv, nullptr, 0, nullptr);
  e = hipGetLastError();
  if (e != hipSuccess) return (int)e;
  return launch_var_fin(a.Z, a.vstd, a.hyp, tot, a.M, a.D, a.dZ, a.dpar, stream);
}

// ---- the saved-state adjoint (M > 64): workspace G' partials | adjoint partials | their fp64 totals
// | the finalisation partials
struct AdjSavedPlan {
  int nchunks, nwg, nwg_g, P, PG;
  long long BN;
  size_t off_gpart, off_part, off_tot, off_gtot, off_cm, total, fin_lds;
};

template <int MB, int DQ>
AdjSavedPlan adj_saved_plan(int B, int N, int M, int D) {
  using LG = LGramGeo<MB, DQ>;
  AdjSavedPlan p{};
  const long long nch = (long long)B * ((N + LTW - 1) / LTW);
  p.nchunks = (int)nch;
  p.nwg = chunk_grid(nch, 1);      // 256 VGPRs: one 8-wave workgroup per CU
  p.nwg_g = chunk_grid(nch, 1);
  p.P = M * D + 3 * M + 2 * D + 3;
  p.PG = LG::PG;
  p.BN = (long long)B * N;
  p.fin_lds = (size_t)M * D * sizeof(float);
  auto al = [](size_t x) { return (x + 255) & ~(size_t)255; };
  size_t o = 0;
  p.off_gpart = o; o = al(o + (size_t)p.nwg_g * p.PG * sizeof(float));
  p.off_part = o; o = al(o + (size_t)p.nwg * p.P * sizeof(float));
  p.off_tot = o; o = al(o + (size_t)p.P * sizeof(double));
  p.off_gtot = o; o = al(o + (size_t)p.PG * sizeof(double));
  p.off_cm = o; o = al(o + 64 * sizeof(float));
  p.total = o;
  return p;
}

template <int MB, int DQ>
int launch_var_adj_saved(const GpkVarAdjArgs& a, hipStream_t stream) {
  if constexpr (var_saved_fits<MB, DQ>()) {
    using LA = LAdjGeo<MB, DQ>;
    using LG = LGramGeo<MB, DQ>;
    const AdjSavedPlan p = adj_saved_plan<MB, DQ>(a.B, a.N, a.M, a.D);
    char* ws = (char*)a.ws;
    float* gpart = (float*)(ws + p.off_gpart);
    float* wspart = (float*)(ws + p.off_part);
    double* tot = (double*)(ws + p.off_tot);
    double* gtot = (double*)(ws + p.off_gtot);
    set_lds_once<gpk_var_adjs_l_kernel<MB, DQ>>();
    hipLaunchKernelGGL((gpk_var_adjs_l_kernel<MB, DQ>), dim3(p.nwg), dim3(LA::NT), (size_t)LA::k_total * sizeof(float),
                       stream, a.X, a.Z, a.Linv, a.vmean, a.vstd, a.hyp, a.gmean, a.gvar, a.saved, a.N, a.M,
                       a.D, p.nchunks, wspart, a.dX, (float*)(ws + p.off_cm));
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return (int)e;
    set_lds_once<gpk_var_kgram_l_kernel<MB, DQ>>();
    hipLaunchKernelGGL((gpk_var_kgram_l_kernel<MB, DQ>), dim3(p.nwg_g), dim3(LG::NT), (size_t)LG::total * sizeof(float),
                       stream, a.X, a.Z, a.vmean, a.vstd, a.hyp, a.gmean, a.gvar, a.saved, a.N, a.M, a.D,
                       p.nchunks, gpart);
    if ((e = hipGetLastError()) != hipSuccess) return (int)e;
    // one fixed-order reduction launch for both partial arrays (same workgroup count), then
    // the output launch with dL^{-1} in extra workgroups
    if (p.nwg == p.nwg_g) {
      hipLaunchKernelGGL(gpk_var_red_kernel, dim3((p.P + 31) / 32 + (p.PG + 31) / 32), dim3(256), 0, stream,
                         wspart, p.nwg, p.P, tot, nullptr, 0, 0, 0, nullptr, gpart, p.PG, gtot);
      if ((e = hipGetLastError()) != hipSuccess) return (int)e;
    } else {
      hipLaunchKernelGGL(gpk_var_red_kernel, dim3((p.PG + 31) / 32), dim3(256), 0, stream, gpart, p.nwg_g,
                         p.PG, gtot, nullptr, 0, 0, 0, nullptr, nullptr, 0, nullptr);
      if ((e = hipGetLastError()) != hipSuccess) return (int)e;
      hipLaunchKernelGGL(gpk_var_red_kernel, dim3((p.P + 31) / 32), dim3(256), 0, stream, wspart, p.nwg, p.P,
                         tot, nullptr, 0, 0, 0, nullptr, nullptr, 0, nullptr);
      if ((e = hipGetLastError()) != hipSuccess) return (int)e;
    }
    const VarGdlArgs gd{gtot, a.Linv, a.vmean, a.vstd, a.dLinv, MB};
    return launch_var_fin(a.Z, a.vstd, a.hyp, tot, a.M, a.D, a.dZ, a.dpar, stream,
                          (const float*)(ws + p.off_cm), &gd);
  } else {
    return -13;
  }
}

// Instantiated row-block counts; M is padded up to the next one (zero rows).
#define GPK_MB_SWITCH(MBV, CALL)                                                   \
  {                                                                                \
    const int mbv_ = (MBV);                                                        \
    if (mbv_ <= 1) { CALL(1) } else if (mbv_ <= 2) { CALL(2) }                     \
    else if (mbv_ <= 3) { CALL(3) } else if (mbv_ <= 4) { CALL(4) }                \
    else if (mbv_ <= 6) { CALL(6) } else if (mbv_ <= 8) { CALL(8) }                \
    else if (mbv_ <= 12) { CALL(12) } else if (mbv_ <= 16) { CALL(16) }            \
  }

}  // namespace

int gpk_launch_var(const GpkVarArgs& a, int* flags, hipStream_t stream) {
  if (flags != nullptr) {
    const hipError_t e = hipMemsetAsync(flags, 0, sizeof(int), stream);
    if (e != hipSuccess) return (int)e;
  }
  if (var_reg_path(a.M, a.D)) return a.D <= 16 ? launch_var_fwd_r<16>(a, flags, stream)
                                               : launch_var_fwd_r<32>(a, flags, stream);
  if (GPK_VAR_LREG && a.M > 64) {
#define GPK_CALL_FWDL(mb)                                                     \
  if (a.D <= 16) return launch_var_fwd_l<mb, 16>(a, flags, stream);           \
  if (a.D <= 32) return launch_var_fwd_l<mb, 32>(a, flags, stream);           \
  return launch_var_fwd_l<mb, 64>(a, flags, stream);
    const int mb = (a.M + 15) / 16;
    if (mb <= 6) { GPK_CALL_FWDL(6) }
    if (mb <= 8) { GPK_CALL_FWDL(8) }
    if (mb <= 12) { GPK_CALL_FWDL(12) }
    if (mb <= 16) { GPK_CALL_FWDL(16) }
#undef GPK_CALL_FWDL
    return -10;
  }
#define GPK_CALL_FWD(mb) return launch_var_fwd<mb>(a, flags, stream);
  GPK_MB_SWITCH((a.M + 15) / 16, GPK_CALL_FWD)
#undef GPK_CALL_FWD
  return -10;
}

size_t gpk_var_adjoint_ws_bytes(int B, int N, int M, int D) {
#define GPK_CALL_WS(mb) return adj_plan<mb>(B, N, M, D).total;
  GPK_MB_SWITCH((M + 15) / 16, GPK_CALL_WS)
#undef GPK_CALL_WS
  return 0;
}

// the saved-state path (training forward keeps A; M > 64, its LDS plan fits): bytes of the saved
// state and of the adjoint's workspace, 0 when the path does not serve the shape
size_t gpk_var_saved_bytes(int B, int N, int M, int D) {
#define GPK_CALL_SV(mb)                                                                        \
  if (adj_dq(D) == 32) return var_saved_path<mb, 32>(M) ? (size_t)B * ((N + LTW - 1) / LTW) *  \
                                  LSaved<mb>::blk * sizeof(float) : 0;                        \
  return var_saved_path<mb, 64>(M) ? (size_t)B * ((N + LTW - 1) / LTW) * LSaved<mb>::blk * sizeof(float) : 0;
  GPK_MB_SWITCH((M + 15) / 16, GPK_CALL_SV)
#undef GPK_CALL_SV
  return 0;
}
size_t gpk_var_adjoint_saved_ws_bytes(int B, int N, int M, int D) {
  if (gpk_var_saved_bytes(B, N, M, D) == 0) return 0;
#define GPK_CALL_SW(mb)                                                        \
  if (adj_dq(D) == 32) return adj_saved_plan<mb, 32>(B, N, M, D).total;        \
  return adj_saved_plan<mb, 64>(B, N, M, D).total;
  GPK_MB_SWITCH((M + 15) / 16, GPK_CALL_SW)
#undef GPK_CALL_SW
  return 0;
}

int gpk_launch_var_adjoint(const GpkVarAdjArgs& a, hipStream_t stream) {
#define GPK_CALL_ADJ(mb)                                         \
  if (a.D <= 32) return launch_var_adj<mb, 32>(a, stream);       \
  return launch_var_adj<mb, 64>(a, stream);
  GPK_MB_SWITCH((a.M + 15) / 16, GPK_CALL_ADJ)
#undef GPK_CALL_ADJ
  return -11;
}
