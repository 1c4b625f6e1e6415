// Shared inducing-point factorisation K_ZZ + jitter = L L^T (fp64) and L^{-1}, once per
// optimizer step (include/gpk.h::gpk_kzz_chol_f64).
//
// Reference: VariationalStrategy._cholesky_factor -> psd_safe_cholesky (fp64 ladder 1e-8 x10^t)
// for ToyDeepGPHiddenLayer (denoising_model/DeepGP.py:33-38 via upstream
// variational_strategy.py); the reference runs it b times per GP call (Z expanded over the
// batch). oracle/gp_oracle.py::kzz_factor restates it.
//
// gpk_kzz16_kernel<NS>: ONE workgroup of 16 waves; the UPPER triangle of K_ZZ (padded to
// T 16-blocks, identity padding) is held as 16 x 16 fp64 tiles in v_mfma_f64_16x16x4f64
// accumulators (acc layout: lane (c, g), reg r <-> row g + 4r, column c) for the whole
// factorisation by 15 WORKER waves (tiles dealt round-robin in column-major order, NS per
// wave); wave 15 is the DIAGONAL wave and holds no tile. Blocked right-looking Cholesky of
// R = L^T in 16-column steps:
//   diag   the diagonal wave factors T'_kk in ONE sweep of the augmented [T_kk | I] (lanes
//          0-15: columns of T_kk -> rows of L_kk, lanes 16-31: identity columns -> columns of
//          L_kk^{-1}), broadcasts by 64-bit DPP (diag_col64) -- LOOK-AHEAD: the owners of
//          (k+1, k+1) and (k, k+1) update and hand them over first in step k-1's update; the
//          diagonal wave forms R_{k,k+1} and T''_{k+1,k+1} itself beside step k's TRSM, so
//          the sweep of (k+1, k+1) overlaps the workers' trailing update of step k;
//   TRSM   owners of block row k: R_kj = L_kk^{-1} T'_kj (4 f64 MFMAs, the register tile is
//          the B operand) -> LDS panel + L's block (j, k);
//   update every tile (i, j), k < i <= j: T'_ij -= R_ki^T R_kj (4 f64 MFMAs, both operands
//          read from the LDS panel in acc layout: conflict-free; R_kj once per column).
// Two workgroup barriers per step. GPyTorch's fp64 ladder restarts in-kernel (info = -t).
// gpk_kzz_inv_kernel: L^{-1}, one workgroup of 16 waves per 16-column block column (block
// forward substitution on fp64 MFMA, one S tile per wave; the diagonal-block inverses come
// from the factor kernel, which forms each L_kk^{-1} anyway), the block columns on
// different CUs.
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

#ifndef GPK_KZZ_WAVES
#define GPK_KZZ_WAVES 16   // 15 workers + the diagonal wave (4 waves / SIMD, 128 VGPRs each)
#endif
#ifndef GPK_KZZ_STAMPS
#define GPK_KZZ_STAMPS 0   // debug: per-step phase clocks into info[1..] (results still valid)
#endif
constexpr int KW = GPK_KZZ_WAVES;
constexpr int KT = 64 * KW;
// (Measured and dropped, scripts/r05/gpu_kzz_ab.sh: keeping the diagonal wave's SIMD free of
// worker tiles: the sweep then runs at its 4.7 K-cycle floor instead of 8-11 K in the early
// steps, but 3 SIMDs make those steps update-bound (121 -> 123 us per factor + inverse), and
// with 12 tiles per worker the kernel spills (118 -> 191 us); prefetching the inverse's L
// operands two steps ahead: no change.)
constexpr int kKzzWorkers = KW - 1;
__host__ __device__ inline int kzz_zstride(int D) { return ((D + 15) & ~15) + 4; }
constexpr int kLinvStride = 17;   // L_kk^{-1} rows in LDS (odd: conflict-free column reads)

#ifndef GPK_KZZ_FUSED_DPP
#define GPK_KZZ_FUSED_DPP 1   // 1: the sweep's broadcast FMAs as single v_fmac_f64_dpp (inline asm)
#endif
#ifndef GPK_KZZ_DPP
#define GPK_KZZ_DPP 1   // 1: the diagonal sweep broadcasts by 64-bit DPP (row_newbcast); 0: readlanes
#endif

// x of lane 16 r' + i for every lane of row r' (64-bit row_newbcast:i; bound_ctrl: every lane
// has a source, and the destination needs no zero-initialisation)
template <int I>
GPK_DEVICE double nbc(double x) {
  return __builtin_amdgcn_update_dpp(0.0, x, 0x150 + I, 0xf, 0xf, true);
}
// acc += (nr of lane i of the row) * vq as ONE v_fmac_f64_dpp (the compiler emits a separate
// v_mov_b64_dpp + v_fmac_f64). NOP: the 2 wait states a DPP read of nr needs after the VALU
// write of nr (the hazard recognizer does not look inside asm); the first use per column.
#define GPK_FMAC_BC(I)                                                                       \
  template <bool NOP>                                                                        \
  GPK_DEVICE void fmac_bc##I(double& acc, double nr, double vq) {                            \
    if constexpr (NOP)                                                                       \
      asm volatile("s_nop 1\n\tv_fmac_f64_dpp %0, %1, %2 row_newbcast:" #I                    \
                   " row_mask:0xf bank_mask:0xf" : "+v"(acc) : "v"(nr), "v"(vq));            \
    else                                                                                     \
      asm volatile("v_fmac_f64_dpp %0, %1, %2 row_newbcast:" #I " row_mask:0xf bank_mask:0xf" \
                   : "+v"(acc) : "v"(nr), "v"(vq));                                         \
  }
GPK_FMAC_BC(1) GPK_FMAC_BC(2) GPK_FMAC_BC(3) GPK_FMAC_BC(4) GPK_FMAC_BC(5)
GPK_FMAC_BC(6) GPK_FMAC_BC(7) GPK_FMAC_BC(8) GPK_FMAC_BC(9) GPK_FMAC_BC(10)
GPK_FMAC_BC(11) GPK_FMAC_BC(12) GPK_FMAC_BC(13) GPK_FMAC_BC(14) GPK_FMAC_BC(15)
#undef GPK_FMAC_BC
// row 0's value in rows 0 and 1 (and row 2's in rows 2 and 3): permlane16_swap per half
GPK_DEVICE double row_even_both(double x) {
  const unsigned long long u = __builtin_bit_cast(unsigned long long, x);
  const unsigned lo = (unsigned)u, hi = (unsigned)(u >> 32);
  const unsigned nl = __builtin_amdgcn_permlane16_swap(lo, lo, false, false)[0];
  const unsigned nh = __builtin_amdgcn_permlane16_swap(hi, hi, false, false)[0];
  return __builtin_bit_cast(double, ((unsigned long long)nh << 32) | nl);
}

// Column Q of the fused sweep (layout of factor_diag): every lane gets -R[Q][c] of its row's
// R lane (row 0), the pivot by DPP, then v[i] += (-R[Q][i]) v[Q] for i > Q with -R[Q][i]
// broadcast from lane i of the row. No readlanes: the sweep keeps issuing beside the
// workers' MFMA and LDS waves (the readlane form starves there, scripts/microbench).
template <int Q>
GPK_DEVICE void diag_col64(double (&v)[16]) {
  const double ta = row_even_both(v[Q]);
  const double p = nbc<Q>(ta);
  const double s = rsq64(p);
  const double nr = -(ta * s);
  v[Q] = v[Q] * s;
  if constexpr (Q < 15) {
#pragma unroll
    for (int i = Q + 1; i < 16; ++i) {
#if GPK_KZZ_FUSED_DPP
      const bool first = i == Q + 1;
      switch (i) {   // (compile-time after unrolling)
#define GPK_FMAC_CASE(I) \
        case I: if (first) fmac_bc##I<true>(v[i], nr, v[Q]); else fmac_bc##I<false>(v[i], nr, v[Q]); break;
        GPK_FMAC_CASE(1) GPK_FMAC_CASE(2) GPK_FMAC_CASE(3) GPK_FMAC_CASE(4) GPK_FMAC_CASE(5)
        GPK_FMAC_CASE(6) GPK_FMAC_CASE(7) GPK_FMAC_CASE(8) GPK_FMAC_CASE(9) GPK_FMAC_CASE(10)
        GPK_FMAC_CASE(11) GPK_FMAC_CASE(12) GPK_FMAC_CASE(13) GPK_FMAC_CASE(14)
        default: if (first) fmac_bc15<true>(v[i], nr, v[Q]); else fmac_bc15<false>(v[i], nr, v[Q]); break;
#undef GPK_FMAC_CASE
      }
#else
      double b;
      switch (i) {   // (compile-time after unrolling)
        case 1: b = nbc<1>(nr); break;   case 2: b = nbc<2>(nr); break;
        case 3: b = nbc<3>(nr); break;   case 4: b = nbc<4>(nr); break;
        case 5: b = nbc<5>(nr); break;   case 6: b = nbc<6>(nr); break;
        case 7: b = nbc<7>(nr); break;   case 8: b = nbc<8>(nr); break;
        case 9: b = nbc<9>(nr); break;   case 10: b = nbc<10>(nr); break;
        case 11: b = nbc<11>(nr); break; case 12: b = nbc<12>(nr); break;
        case 13: b = nbc<13>(nr); break; case 14: b = nbc<14>(nr); break;
        default: b = nbc<15>(nr); break;
      }
      v[i] = __builtin_fma(b, v[Q], v[i]);
#endif
    }
    diag_col64<Q + 1>(v);
  }
}

// x of the odd row (1 -> 0, 3 -> 2) in the even rows' lanes (permlane16_swap, new src0)
GPK_DEVICE double from_odd_row(double x) {
  const unsigned long long u = __builtin_bit_cast(unsigned long long, x);
  const unsigned lo = (unsigned)u, hi = (unsigned)(u >> 32);
  const unsigned nl = __builtin_amdgcn_permlane16_swap(lo, lo, false, false)[1];
  const unsigned nh = __builtin_amdgcn_permlane16_swap(hi, hi, false, false)[1];
  return __builtin_bit_cast(double, ((unsigned long long)nh << 32) | nl);
}
// x of rows 2, 3 in rows 0, 1 (permlane32_swap, new src0)
GPK_DEVICE double from_upper_half(double x) {
  const unsigned long long u = __builtin_bit_cast(unsigned long long, x);
  const unsigned lo = (unsigned)u, hi = (unsigned)(u >> 32);
  const unsigned nl = __builtin_amdgcn_permlane32_swap(lo, lo, false, false)[1];
  const unsigned nh = __builtin_amdgcn_permlane32_swap(hi, hi, false, false)[1];
  return __builtin_bit_cast(double, ((unsigned long long)nh << 32) | nl);
}
// The sweep's operand from an acc-layout tile in registers: lanes 0-15 get column c
// (v[g' + 4r] = reg r of lane c + 16 g'), lanes 16-31 the identity column c - 16.
GPK_DEVICE void acc_to_sweep(const f64x4 t, double (&v)[16]) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const double up = from_upper_half(t[r]);
    v[4 * r] = t[r];
    v[4 * r + 1] = from_odd_row(t[r]);
    v[4 * r + 2] = up;
    v[4 * r + 3] = from_odd_row(up);
  }
#pragma unroll
  for (int i = 0; i < 16; ++i) v[i] = lane < 16 ? v[i] : ((lane - 16 == i) ? 1.0 : 0.0);
}

// The diagonal wave factors the (updated, handed-over) diagonal tile t = T'_kk:
// one broadcast sweep (diag_col64) of the augmented [T_kk | I] (lanes 0-15: columns of T_kk
// -> rows of L_kk, lanes 16-31: identity columns -> columns of L_kk^{-1}). Results: lkk
// (16 x 17, row-major L_kk), linv (16 x 17, L_kk^{-1}) in LDS; status = failed column + 1.
GPK_DEVICE void sweep_diag(int k, double (&v)[16], double* lkk, double* linv, int* status, int* stamp) {
  const int lane = threadIdx.x & 63, c = lane & 15;
  const bool left = lane < 16;
  int bad = 0;
#if GPK_KZZ_STAMPS
  if (stamp != nullptr) {
    asm volatile("" ::"v"(v[15]));   // the operand is in registers
    if (lane == 0) stamp[1] = (int)__builtin_amdgcn_s_memtime();
  }
#endif
#if GPK_KZZ_DPP
  diag_col64<0>(v);
  {
    // first column whose R[c][c] is not positive-finite (a non-positive pivot makes it NaN
    // through the rsqrt; the columns before it are untouched by that)
    double dg = v[0];
#pragma unroll
    for (int i = 1; i < 16; ++i) dg = (c == i) ? v[i] : dg;
    const bool okd = (dg > 0.0) && (dg < __builtin_huge_val());
    const unsigned long long badm = __ballot(lane < 16 && !okd);
    bad = badm ? __builtin_ctzll(badm) + 1 : 0;
  }
#else
#pragma unroll
  for (int q = 0; q < 16; ++q) {
    const double p = readlane_d(v[q], q);
    if (!(p > 0.0) && bad == 0) bad = q + 1;
    const double s = rsq64(p > 0.0 ? p : 1.0);
    const double vq = v[q];
    const double t = (s * s) * vq;   // row q's multiple: the multipliers stay SGPR operands
    v[q] = vq * s;
#pragma unroll
    for (int i = q + 1; i < 16; ++i) v[i] = __builtin_fma(-readlane_d(v[i], q), t, v[i]);
  }
#endif
  // lanes 0-15: v[i] = L_kk[c][i] (i <= c); lanes 16-31: v[i] = L_kk^{-1}[i][c - 16]
  if (left) {
#pragma unroll
    for (int i = 0; i < 16; ++i) lkk[c * kLinvStride + i] = i <= c ? v[i] : 0.0;
  } else if (lane < 32) {
#pragma unroll
    for (int i = 0; i < 16; ++i) linv[i * kLinvStride + c] = v[i];
  }
  if (lane == 0) status[0] = bad == 0 ? 0 : 16 * k + bad;
#if GPK_KZZ_STAMPS
  if (stamp != nullptr && lane == 0) stamp[2] = (int)__builtin_amdgcn_s_memtime();
#endif
}

// Tile (0, 0), handed over raw in acc layout through LDS (dbuf).
GPK_DEVICE void factor_diag0(const double* dbuf, double* lkk, double* linv, int* status, int* stamp) {
  const int lane = threadIdx.x & 63;
  f64x4 t;
#pragma unroll
  for (int r = 0; r < 4; ++r) t[r] = dbuf[r * 64 + lane];
  double v[16];
  acc_to_sweep(t, v);
  sweep_diag(0, v, lkk, linv, status, stamp);
}

// LDS flag words of the factor kernel (volatile, LDS address space: ds_read / ds_write only)
// kKfTile: epoch of the raw (0, 0) hand-over of the tile formation (every later hand-over is
// ordered by the step barriers)
// kKfSync: the workers' step barrier [B] (monotone count: one add per worker wave per step)
enum KzzFlag { kKfTile = 0, kKfTmo = 1, kKfStatus = 2, kKfSync = 3, kKfWords = 8 };
constexpr int kKzzTimeout = 1 << 20;   // info code of an expired spin-wait (never NotPSD)

GPK_DEVICE void kzz_spin_ge(lds_vint* f, int word, int target) {
  int n = 0;
  while (f[word] < target) {
    if (++n > (1 << 20)) {
      f[kKfTmo] = 1;
      break;
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

GPK_DEVICE void kzz_spin_until(lds_vint* f, int word, int target) {
  int n = 0;
  while (f[word] != target) {
    if (++n > (1 << 20)) {   // bounded: a logic error ends as info = 1 << 20, never a hang
      f[kKfTmo] = 1;
      break;
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

// K_ZZ tile (it, jt) of the padded matrix + jitter (+ ladder) into an fp64 acc tile: fp32 Gram
// on MFMA (A rows fed in the order pi(x) = (x >> 2) + 4 (x & 3) so the fp32 accumulator lands
// in the fp64 acc layout), the fp32 kernel and jitter as the reference, then fp64.
GPK_DEVICE f64x4 kzz_tile(const float* zt, const float* zn, int ZS, int D16, int M, int T, int it,
                          int jt, float s2, float jitter_var, double ladder) {
  const int lane = threadIdx.x & 63, c = lane & 15, g = lane >> 4;
  const int j = 16 * jt + c;
  f32x4 gram = {0.f, 0.f, 0.f, 0.f};
  const int ia = 16 * it + (c >> 2) + 4 * (c & 3);
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
  f64x4 t;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int i = 16 * it + g + 4 * r;
    double v = (i == j) ? 1.0 : 0.0;
    if (i < M && j < M) {
      float dist = zn[i] + zn[j] - 2.f * gram[r];
      dist = dist < 0.f ? 0.f : dist;
      float kv = s2 * __expf(-0.5f * dist);
      if (i == j) kv = kv + jitter_var;
      v = (double)kv;
      if (i == j) v += ladder;
    }
    t[r] = v;
  }
  return t;
}

GPK_DEVICE double ladder_of(int attempt, double jitter_chol) {   // GPyTorch: cumulative increments
  double ladder = 0.0, prev = 0.0, p10 = 1.0;
  for (int q = 0; q < attempt; ++q) {
    const double jn = jitter_chol * p10;
    ladder += jn - prev;
    prev = jn;
    p10 *= 10.0;
  }
  return ladder;
}

// Waves 0 .. KW-2 are WORKERS holding the upper triangle's tiles (dealt round-robin in
// column-major order); wave KW-1 is the DIAGONAL wave and holds no tile. Per step k:
//   [A] workgroup barrier: L_kk, L_kk^{-1} (LDS, parity k & 1) and the step's status are out;
//   [B] workers: TRSM of block row k -> LDS panel + L, then a WORKER-ONLY barrier (LDS
//       counter, kKfSync); the diagonal wave does not join it: it forms R_{k,k+1} =
//       L_kk^{-1} T'_{k,k+1} and T''_{k+1,k+1} = T'_{k+1,k+1} - R^T R from the two hand-over
//       tiles itself (the same MFMAs as the owners'), writes the diagonal blocks of L and
//       L^{-1} to HBM and starts the sweep of (k+1, k+1) at once;
//   [C] the owners of (k+2, k+2) and (k+1, k+2) update them FIRST and hand them over (LDS,
//       read by the diagonal wave after the next [A]), then their other tiles, while the
//       diagonal wave sweeps: the 16-column sweeps are the only sequential chain.
// The diagonal wave's registers are disjoint from the workers' (separate loops), so the
// tiles (NS per worker) and the sweep do not compete for the 256-VGPR budget.
template <int NS>
__global__ void __launch_bounds__(KT, 1)
gpk_kzz16_kernel(const float* __restrict__ Z, const float* __restrict__ hyp, int M, int D,
                 float jitter_var, double jitter_chol, int max_tries, double* __restrict__ L,
                 double* __restrict__ Linv, int* __restrict__ info) {
  extern __shared__ __attribute__((aligned(16))) double dsm[];
  const int T = (M + 15) >> 4;
  double* panel = dsm;                 // (T - 1) tiles x 256, [slot][reg][lane]
  double* dbuf = panel + (size_t)(T > 1 ? T - 1 : 1) * 256;   // 2 x 256: hand-over tiles (t, t)
  double* obuf = dbuf + 512;           // 2 x 256: hand-over tiles (t - 1, t), parity t & 1
  double* linvb = obuf + 512;          // 2 x 16 x 17: L_kk^{-1}, parity k & 1
  double* lkkb = linvb + 2 * 16 * kLinvStride;                // 2 x 16 x 17: L_kk, parity k & 1
  int* flagw = (int*)(lkkb + 2 * 16 * kLinvStride);           // KzzFlag words
  lds_vint* fl = as_lds_flags(flagw);
  float* zt = (float*)(flagw + kKfWords);   // M x ZS  Z / l, centred (zero padded)
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
  if (tid < kKfWords) flagw[tid] = tid == kKfTile ? -1 : 0;
  lds_barrier();
  for (int d = wave; d < D; d += KT / 64) {   // column means: one wave per column
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

  constexpr int NWK = KW - 1;          // workers
  int result = 0;
  if (wave == NWK) {
    // ================= diagonal wave =================
    // critical path: win issue arbitration against the workers' MFMA / LDS streams (the
    // stamps show the step-k+1 sweep taking 13 K cycles beside step k's update at M = 256
    // vs 6 K alone)
    __builtin_amdgcn_s_setprio(3);
    for (int attempt = 0; attempt <= max_tries; ++attempt) {
      int failed = 0;
      // tile (0, 0): handed over raw by the tile formation
      kzz_spin_until(fl, kKfTile, attempt * (T + 1));
#if GPK_KZZ_STAMPS
      if (attempt == 0 && lane == 0) info[1 + 3 * T] = (int)__builtin_amdgcn_s_memtime();
#endif
      factor_diag0(dbuf, lkkb, linvb, flagw + kKfStatus, attempt == 0 ? info + 1 + 3 * T : nullptr);
      for (int k = 0; k < T; ++k) {
        const int tk = k + 1;
        int* stamp = nullptr;
#if GPK_KZZ_STAMPS
        if (attempt == 0 && tk < T) stamp = info + 1 + 3 * T + 3 * tk;
#endif
        // L_kk^{-1} (this wave's own sweep output): A operands of R_{k,k+1}, read before [A]
        double la[4];
        wave_lds_sync();
#pragma unroll
        for (int kk = 0; kk < 4; ++kk) la[kk] = linvb[(k & 1) * 16 * kLinvStride + c * kLinvStride + g + 4 * kk];
        lds_barrier();   // [A]
        failed = fl[kKfStatus];
        if (fl[kKfTmo]) failed = kKzzTimeout;
        if (failed) break;
        if (tk < T) {
          // LOOK-AHEAD beside the workers' TRSM of block row k: R_{k,k+1} = L_kk^{-1} T'_{k,k+1}
          // and T''_{k+1,k+1} = T'_{k+1,k+1} - R^T R from the two tiles handed over in step
          // k-1's [C] (panels < k applied) -- the same MFMAs as the owners' TRSM and update --
          // then straight into the sweep of (k+1, k+1), operands moved by permlanes
#if GPK_KZZ_STAMPS
          if (stamp != nullptr && lane == 0) stamp[0] = (int)__builtin_amdgcn_s_memtime();
#endif
          const double* ob = obuf + (tk & 1) * 256;
          const double* db = dbuf + (tk & 1) * 256;
          f64x4 o, t;
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            o[r] = ob[r * 64 + lane];
            t[r] = db[r * 64 + lane];
          }
#if GPK_KZZ_STAMPS
          int* s2p = stamp != nullptr ? info + 1 + 8 * T + 4 * tk : nullptr;
          if (s2p != nullptr) {
            __builtin_amdgcn_s_waitcnt(0xc07f);
            if (lane == 0) s2p[0] = (int)__builtin_amdgcn_s_memtime();
          }
#endif
          f64x4 x = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
          for (int kk = 0; kk < 4; ++kk) x = mfma64(la[kk], o[kk], x);
#if GPK_KZZ_STAMPS
          if (s2p != nullptr) {
            asm volatile("" ::"v"(x[3]));   // the MFMA chain's result is in
            if (lane == 0) s2p[1] = (int)__builtin_amdgcn_s_memtime();
          }
#endif
#pragma unroll
          for (int kk = 0; kk < 4; ++kk) t = mfma64(-x[kk], x[kk], t);
#if GPK_KZZ_STAMPS
          if (s2p != nullptr) {
            asm volatile("" ::"v"(t[3]));
            if (lane == 0) s2p[2] = s2p[3] = (int)__builtin_amdgcn_s_memtime();
          }
#endif
          // [C] the sweep of (k+1, k+1) overlaps the workers' trailing update of step k; it
          // writes the other parity of L_kk / L_kk^{-1} (the workers read parity k & 1)
          double v[16];
          acc_to_sweep(t, v);
          sweep_diag(tk, v, lkkb + (tk & 1) * 16 * kLinvStride, linvb + (tk & 1) * 16 * kLinvStride,
                     flagw + kKfStatus, stamp);
        }
      }
      if (!failed) {
        result = attempt > 0 ? -attempt : 0;
        break;
      }
      result = failed;
      lds_barrier();
      if (failed == kKzzTimeout) break;
      if (lane == 0) fl[kKfStatus] = 0;
      lds_barrier();
    }
    __builtin_amdgcn_s_setprio(0);
  } else {
    // ================= workers =================
    // upper tiles in column-major order t = j (j + 1) / 2 + i, dealt round-robin to the workers
    int its[NS], jts[NS];
    {
      const int ntile = T * (T + 1) / 2;
#pragma unroll
      for (int q = 0; q < NS; ++q) {
        const int t = wave + kKzzWorkers * q;
        int it = T, jt = T;   // no tile: coordinates past the end (skipped everywhere)
        if (t < ntile) tile_of(t, T, it, jt);
        its[q] = __builtin_amdgcn_readfirstlane(it);
        jts[q] = __builtin_amdgcn_readfirstlane(jt);
      }
    }
    f64x4 acc[NS];
    int nsync = 0;   // worker barriers passed
    for (int attempt = 0; attempt <= max_tries; ++attempt) {
      const double ladder = ladder_of(attempt, jitter_chol);
#pragma unroll
      for (int q = 0; q < NS; ++q) {
        asm volatile("" : "+s"(its[q]), "+s"(jts[q]));
        if (its[q] < T) acc[q] = kzz_tile(zt, zn, ZS, D16, M, T, its[q], jts[q], s2, jitter_var, ladder);
        if (its[q] == 0 && jts[q] == 0) {   // hand (0, 0) over raw: the sweep starts at once
#pragma unroll
          for (int r = 0; r < 4; ++r) dbuf[r * 64 + lane] = acc[q][r];
          __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
          if (lane == 0) fl[kKfTile] = attempt * (T + 1);
        }
        if (jts[q] == 1 && T > 1) {   // (0, 1), (1, 1) raw: read after barrier [A] of step 0
#pragma unroll
          for (int r = 0; r < 4; ++r) (its[q] == 1 ? dbuf : obuf)[256 + r * 64 + lane] = acc[q][r];
        }
      }
      int failed = 0;
      for (int k = 0; k < T; ++k) {
#pragma unroll
        for (int q = 0; q < NS; ++q) asm volatile("" : "+s"(its[q]), "+s"(jts[q]));
#if GPK_KZZ_STAMPS
        if (tid == 0 && attempt == 0) info[1 + 3 * k] = (int)__builtin_amdgcn_s_memtime();
#endif
        lds_barrier();   // [A]
#if GPK_KZZ_STAMPS
        if (tid == 0 && attempt == 0) info[2 + 3 * k] = (int)__builtin_amdgcn_s_memtime();
#endif
        failed = fl[kKfStatus];
        if (fl[kKfTmo]) failed = kKzzTimeout;
        if (failed) break;
        // [B] TRSM of block row k: R_kj = L_kk^{-1} T'_kj -> registers, LDS panel, L
        double la[4];
#pragma unroll
        for (int kk = 0; kk < 4; ++kk) la[kk] = linvb[(k & 1) * 16 * kLinvStride + c * kLinvStride + g + 4 * kk];
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
            const int row = 16 * jts[q] + c;   // L block (j, k) = R_kj^T
            if (row < M) {
#pragma unroll
              for (int r = 0; r < 4; ++r) L[(size_t)row * M + 16 * k + g + 4 * r] = x[r];
            }
          }
        }
        // worker-only barrier (LDS counter; the diagonal wave is sweeping tile k+1 meanwhile):
        // panel k is complete. Every worker leaves a failed attempt at the same [A], so the
        // counts stay in step across attempts.
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
        ++nsync;
        if (lane == 0)
          (void)__atomic_fetch_add((__attribute__((address_space(3))) int*)&flagw[kKfSync], 1, __ATOMIC_RELAXED);
        kzz_spin_ge(fl, kKfSync, kKzzWorkers * nsync);
#if GPK_KZZ_STAMPS
        if (tid == 0 && attempt == 0) info[3 + 3 * k] = (int)__builtin_amdgcn_s_memtime();
#endif
        // [C] hand over (k+2, k+2) and (k+1, k+2) through panel k first (the diagonal wave
        // applies panel k+1 to them itself in step k+1's [B']; it reads them after barrier
        // [A] of step k+1); (k+1, k+1) is the diagonal wave's from here on
#pragma unroll
        for (int q = 0; q < NS; ++q) {
          if (jts[q] == k + 2 && its[q] >= k + 1 && k + 2 < T) {
            const int tk = k + 2;
            const double* pa = panel + (size_t)(its[q] - k - 1) * 256;
#pragma unroll
            for (int kk = 0; kk < 4; ++kk)
              acc[q] = mfma64(-pa[kk * 64 + lane], panel[256 + kk * 64 + lane], acc[q]);
            double* hb = (its[q] == tk ? dbuf : obuf) + (tk & 1) * 256;
#pragma unroll
            for (int r = 0; r < 4; ++r) hb[r * 64 + lane] = acc[q][r];
          }
        }
        // (a program-order software pipeline of the operand reads -- tile q+1's requested
        // before tile q's MFMAs -- measured slower: 155 vs 148 us at M = 256)
#pragma unroll
        for (int q = 0; q < NS; ++q) {
          if (its[q] > k && its[q] < T && !(its[q] == jts[q] && its[q] <= k + 2) &&
              !(its[q] == k + 1 && jts[q] == k + 2)) {
            const double* pa = panel + (size_t)(its[q] - k - 1) * 256;
            const double* pb = panel + (size_t)(jts[q] - k - 1) * 256;
#pragma unroll
            for (int kk = 0; kk < 4; ++kk) acc[q] = mfma64(-pa[kk * 64 + lane], pb[kk * 64 + lane], acc[q]);
          }
        }
        // the diagonal blocks of L and L^{-1} of step k (LDS parity k & 1, overwritten by the
        // sweep of tile k+2 only after the next [A]): one 64-element slice per wave 0..7
        if (wave < 8) {
          const int e = lane + 64 * wave, r = (e >> 4) & 15, cc = e & 15;
          const int row = 16 * k + r, col = 16 * k + cc;
          const int o = (k & 1) * 16 * kLinvStride + r * kLinvStride + cc;
          if (row < M && col < M) {
            if (e < 256) L[(size_t)row * M + col] = lkkb[o];
            else Linv[(size_t)row * M + col] = linvb[o];
          }
        }
      }
      if (!failed) {
        result = attempt > 0 ? -attempt : 0;
        break;
      }
      result = failed;
      lds_barrier();
      if (failed == kKzzTimeout) break;
      lds_barrier();   // (the diagonal wave resets the status between these two)
    }
  }
  for (int i = wave; i < M; i += KT / 64) {   // strict upper triangle of L: one row per wave
    for (int j = i + 1 + lane; j < M; j += 64) L[(size_t)i * M + j] = 0.0;
  }
  if (tid == 0) info[0] = result;
}

// L^{-1} of the K_ZZ factor: one workgroup per 16-column block column jb (grid T16), so
// the block columns run concurrently on different CUs. Block forward substitution,
// right-looking, on fp64 MFMA:
//   T_u = L_uu^{-1} (the diagonal blocks of Linv, written by gpk_kzz16_kernel),
//   X_jb = T_jb;  for k = jb ..: S_u += -L_uk X_k (u > k), X_{k+1} = T_{k+1} S_{k+1}.
// k-order of every MFMA: q = g + 4 kk, so a tile held in acc layout (reg r <-> row g + 4r)
// is the B operand of k-step kk straight from register kk. S tiles dealt over 16 waves
// (u = wave: one tile per wave, M <= 256). Each step's L block column is STAGED in LDS by
// the whole workgroup from loads along the rows of L, issued two steps ahead (register sets
// by step parity) and stored into a double-buffered LDS block after the MFMAs of the step
// before its use: the round-4 per-lane operand gather (16 rows per load instruction) waited
// for every load right where it was issued (a load under a branch merged into a value makes
// the compiler wait at the join), ~3-5 K cycles per step against ~1 K of MFMA chain.
constexpr int KIT = 1024, KIW = KIT / 64;
constexpr int kInvLS = 17;                 // row stride (doubles) of a staged L tile: conflict-free
constexpr int kInvTile = 16 * kInvLS;
__host__ __device__ inline size_t kzz_inv_lds_bytes(int T16) {
  return ((size_t)T16 * kInvTile + (size_t)T16 * 256 + (size_t)2 * 16 * kInvTile) * sizeof(double);
}
__global__ void __launch_bounds__(KIT)
gpk_kzz_inv_kernel(const double* __restrict__ L, int M, const int* __restrict__ info,
                   double* __restrict__ Linv) {
  extern __shared__ __attribute__((aligned(16))) double dsm[];
  const int Mp = (M + 15) & ~15, T16 = Mp >> 4;
  const int jb = blockIdx.x;
  const int nb = T16 - jb;            // block rows jb .. T16-1 of this block column
  double* Tv = dsm;                   // nb tiles: T_{jb+u}, row-major [row][col], row stride 17
  double* Xs = Tv + T16 * kInvTile;   // nb x 256: X_{jb+u}, row-major
  double* Lb = Xs + T16 * 256;        // 2 x 16 tiles: L_{jb+u, jb+k} of step k, parity k & 1
  const int tid = threadIdx.x, lane = tid & 63, c = lane & 15, g = lane >> 4;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  if (info[0] > 0) return;           // no factor (the op raises NotPSDError)
#if GPK_KZZ_STAMPS
  // block column 0's clock: start, after the prologue, after each step's barrier
  int* ist = (jb == 0 && tid == 0) ? const_cast<int*>(info) + 1 + 6 * T16 : nullptr;
  if (ist) ist[0] = (int)__builtin_amdgcn_s_memtime();
#endif
  for (int e = tid; e < 16 * jb * 16; e += KIT) {   // block rows above the diagonal: zero
    const int i = e >> 4, j = 16 * jb + (e & 15);
    if (i < M && j < M) Linv[(size_t)i * M + j] = 0.0;
  }
  // staging of step s's L tiles u = s+1 .. nb-1 (block column jb + s): piece p = 2 doubles of
  // one tile row, two pieces per thread (15 tiles x 128 pieces <= 2 x 1024). Two register sets
  // (step parity): step s+2's loads are issued in step s and land in LDS at the end of step
  // s+1, two steps of compute behind the load latency.
  double st[2][2][2];
  auto stage_load = [&](int s, double (&st)[2][2]) {
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int p = tid + KIT * h, tt = p >> 7, row = (p >> 3) & 15, pc = p & 7;
      const int i = 16 * (jb + s + 1 + tt) + row, j = 16 * (jb + s) + 2 * pc;
      const int ic = i < M ? i : M - 1;      // unconditional loads (clamped): no wait at a join
      const size_t o = (size_t)ic * M;
      st[h][0] = L[o + (j < M ? j : M - 1)];
      st[h][1] = L[o + (j + 1 < M ? j + 1 : M - 1)];
    }
  };
  auto stage_store = [&](int s, const double (&st)[2][2]) {
    double* dst = Lb + (s & 1) * 16 * kInvTile;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int p = tid + KIT * h, tt = p >> 7, row = (p >> 3) & 15, pc = p & 7;
      if (s + 1 + tt < nb) {
        const int i = 16 * (jb + s + 1 + tt) + row, j = 16 * (jb + s) + 2 * pc;
#pragma unroll
        for (int q = 0; q < 2; ++q)
          dst[tt * kInvTile + row * kInvLS + 2 * pc + q] =
              (i < M && j + q < M) ? st[h][q] : (i == j + q ? 1.0 : 0.0);
      }
    }
  };
  stage_load(0, st[0]);
  stage_load(1, st[1]);
  // diagonal-block inverses T_u = L_uu^{-1}: the factor kernel stored them as the diagonal
  // blocks of Linv (identity padding beyond M)
  for (int e = tid; e < nb * 256; e += KIT) {
    const int u = e >> 8, r = (e >> 4) & 15, q = e & 15;
    const int i = 16 * (jb + u) + r, j = 16 * (jb + u) + q;
    Tv[u * kInvTile + r * kInvLS + q] = (i < M && j < M) ? Linv[(size_t)i * M + j] : (i == j ? 1.0 : 0.0);
  }
  if (nb > 1) stage_store(0, st[0]);
  lds_barrier();
  for (int e = tid; e < 256; e += KIT) {      // X_jb = T_jb
    const double tv = Tv[(e >> 4) * kInvLS + (e & 15)];
    Xs[e] = tv;
    const int i = 16 * jb + (e >> 4), j = 16 * jb + (e & 15);
    if (i < M && j < M) Linv[(size_t)i * M + j] = tv;
  }
  lds_barrier();
#if GPK_KZZ_STAMPS
  if (ist) ist[1] = (int)__builtin_amdgcn_s_memtime();
#endif
  f64x4 S = {0.0, 0.0, 0.0, 0.0};
  const int u = wave;                          // this wave's S tile (block row jb + u)
  // step k: loads of step k+2 into `ld` (unconditional, clamped: no wait at a branch join),
  // the MFMAs, then step k+1's staged tiles (`sv`, loaded in step k-1) into LDS
  auto step = [&](int k, double (&ld)[2][2], const double (&sv)[2][2]) {
    stage_load(k + 2, ld);
    // the next owner's chain (S_{k+1} -> X_{k+1}) is the step's critical path: it wins the
    // MFMA issue arbitration against the 14 other waves' S updates on its SIMD
    const bool owner = wave == k + 1;
    if (owner) __builtin_amdgcn_s_setprio(3);
    double tq[4];                              // the owner's T_{k+1} operands, read up front
#pragma unroll
    for (int kk = 0; kk < 4; ++kk) tq[kk] = Tv[(owner ? k + 1 : 0) * kInvTile + c * kInvLS + g + 4 * kk];
    const bool act = u > k && u < nb;
    const double* lt = Lb + (k & 1) * 16 * kInvTile + (act ? u - k - 1 : 0) * kInvTile;
    double a[4], xb[4];
#pragma unroll
    for (int kk = 0; kk < 4; ++kk) {
      a[kk] = act ? -lt[c * kInvLS + g + 4 * kk] : 0.0;
      xb[kk] = Xs[k * 256 + (g + 4 * kk) * 16 + c];
    }
    if (act) {
#pragma unroll
      for (int kk = 0; kk < 4; ++kk) S = mfma64(a[kk], xb[kk], S);
    }
#if GPK_KZZ_STAMPS
    int* ost = (jb == 0 && owner && lane == 0) ? const_cast<int*>(info) + 1 + 12 * T16 + 4 * k : nullptr;
    if (ost) {
      asm volatile("" ::"v"(S[3]));
      ost[0] = (int)__builtin_amdgcn_s_memtime();
    }
#endif
    if (owner) {                               // X_{k+1} = T_{k+1} S_{k+1}
      f64x4 xv = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
      for (int kk = 0; kk < 4; ++kk) xv = mfma64(tq[kk], S[kk], xv);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        Xs[(k + 1) * 256 + (g + 4 * r) * 16 + c] = xv[r];
        const int i = 16 * (jb + k + 1) + g + 4 * r, j = 16 * jb + c;
        if (i < M && j < M) Linv[(size_t)i * M + j] = xv[r];
      }
      __builtin_amdgcn_s_setprio(0);
    }
#if GPK_KZZ_STAMPS
    if (ost) ost[1] = (int)__builtin_amdgcn_s_memtime();
#endif
    if (k + 2 < nb) stage_store(k + 1, sv);
#if GPK_KZZ_STAMPS
    if (ost) {
      __builtin_amdgcn_s_waitcnt(0);
      ost[2] = (int)__builtin_amdgcn_s_memtime();
    }
#endif
    lds_barrier();
#if GPK_KZZ_STAMPS
    if (ost) ost[3] = (int)__builtin_amdgcn_s_memtime();
#endif
#if GPK_KZZ_STAMPS
    if (ist) ist[2 + k] = (int)__builtin_amdgcn_s_memtime();
#endif
  };
  for (int k = 0; k + 1 < nb; k += 2) {        // unrolled by two: static register sets
    step(k, st[0], st[1]);
    if (k + 2 < nb) step(k + 1, st[1], st[0]);
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
  const size_t lds = (size_t)((T > 1 ? T - 1 : 1) * 256 + 1024 + 4 * 16 * kLinvStride) * sizeof(double) +
                     kKfWords * sizeof(int) + (size_t)(a.M * kzz_zstride(a.D) + a.M + a.D) * sizeof(float);
  if (lds > 160 * 1024) return -4;
  set_lds_once<gpk_kzz16_kernel<NS>>();
  hipLaunchKernelGGL((gpk_kzz16_kernel<NS>), dim3(1), dim3(KT), lds, stream, a.Z, a.hyp, a.M, a.D,
                     a.jitter_var, a.jitter_chol, a.max_tries, a.L, a.Linv, a.info);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return (int)e;
  set_lds_once<gpk_kzz_inv_kernel>();
  hipLaunchKernelGGL(gpk_kzz_inv_kernel, dim3(T), dim3(KIT), kzz_inv_lds_bytes(T), stream, a.L, a.M,
                     a.info, a.Linv);
  e = hipGetLastError();
  return e == hipSuccess ? 0 : (int)e;
}

}  // namespace

int gpk_launch_kzz16(const GpkKzzArgs& a, hipStream_t stream) {
  const int T = (a.M + 15) >> 4;
  const int ns = (T * (T + 1) / 2 + kKzzWorkers - 1) / kKzzWorkers;   // tiles per worker (round-robin)
  if (ns <= 2) return launch_kzz16<2>(a, stream);
  if (ns <= 4) return launch_kzz16<4>(a, stream);
  if (ns <= 7) return launch_kzz16<7>(a, stream);
  if (ns <= 10) return launch_kzz16<10>(a, stream);
  if (ns <= 17) return launch_kzz16<17>(a, stream);
  if (ns <= 21) return launch_kzz16<21>(a, stream);
  return -3;
}
