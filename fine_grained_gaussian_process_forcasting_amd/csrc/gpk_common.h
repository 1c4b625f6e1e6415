// Shared device helpers for the gfx950 GP kernels.
//
// Tile convention used by every kernel in this library ("acc layout"):
// a 16x16 fp32 tile P is held by one wave, 4 registers per lane, exactly as
// the accumulator of v_mfma_f32_16x16x4_f32 lays it out:
//     lane l = 16*g + c  (g = l >> 4, c = l & 15),  reg r  <->  P[4g + r][c].
// With the k-order pi(s, g) = 4g + s, a tile held in acc layout is directly a
// legal A or B operand of the same MFMA (reg s in MFMA step s):
//     sum_s mfma(Q.reg[s], P.reg[s])  ==  Q^T * P
// so Cholesky panels, trailing updates, TRSMs and the RBF Gram all run on
// register tiles with no transposes.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef double f64x4 __attribute__((ext_vector_type(4)));
typedef _Float16 half4_t __attribute__((ext_vector_type(4)));
typedef _Float16 half8_t __attribute__((ext_vector_type(8)));

#define GPK_DEVICE __device__ __forceinline__

// D += Q^T P for 16x16 tiles given in acc layout (4 MFMAs, K = 16).
GPK_DEVICE f32x4 mma_tn(const f32x4 q, const f32x4 p, f32x4 d) {
  d = __builtin_amdgcn_mfma_f32_16x16x4f32(q[0], p[0], d, 0, 0, 0);
  d = __builtin_amdgcn_mfma_f32_16x16x4f32(q[1], p[1], d, 0, 0, 0);
  d = __builtin_amdgcn_mfma_f32_16x16x4f32(q[2], p[2], d, 0, 0, 0);
  d = __builtin_amdgcn_mfma_f32_16x16x4f32(q[3], p[3], d, 0, 0, 0);
  return d;
}

// Split-f16 tiles. A factor tile R is ROUNDED to R^ = hi + lo (hi = f16(R),
// lo = f16(R - hi): 22 significant bits, relative rounding <= 2^-22 for
// |R| >= 2^-2; absolute <= 2^-25 below) and R^ is used everywhere the factor is
// used -- written to L, and stored as two f16 planes (hi, lo: 64 lanes x half4
// = 512 B each) for the trailing updates. The products hi.hi, hi.lo, lo.hi,
// lo.lo are exact in the f16 MFMAs, so the update R^T R^ is accumulated like an
// fp32 MFMA would with R^ as input: the factorisation stays self-consistent and
// only the 22-bit storage of the factor costs accuracy (vs 24 bits in fp32).
GPK_DEVICE f32x4 round_split_f16(const f32x4 v, half4_t& h, half4_t& l) {
  f32x4 o;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    h[r] = (_Float16)v[r];
    l[r] = (_Float16)(v[r] - (float)h[r]);
    o[r] = (float)h[r] + (float)l[r];
  }
  return o;
}
GPK_DEVICE void store_split_planes(float* tile, int lane, const half4_t h, const half4_t l) {
  *(half4_t*)&tile[2 * lane] = h;
  *(half4_t*)&tile[128 + 2 * lane] = l;
}

// D += Q^T P for tiles stored as split planes (R^ = hi + lo exactly):
//   K=32 MFMA with A = {Q.hi, Q.lo}, B = {P.hi, P.lo}:  Q.hi P.hi + Q.lo P.lo
//   K=32 MFMA with A = {Q.hi, Q.lo}, B = {P.lo, P.hi}:  Q.hi P.lo + Q.lo P.hi
// (k-order {4g+r | first half} ++ {second half}; every product is exact).
GPK_DEVICE half8_t load_split_hl(const float* tile, int lane) {
  const half4_t h = *(const half4_t*)&tile[2 * lane];
  const half4_t l = *(const half4_t*)&tile[128 + 2 * lane];
  return half8_t{h[0], h[1], h[2], h[3], l[0], l[1], l[2], l[3]};
}
GPK_DEVICE f32x4 mma_tn_split(const half8_t q_hl, const float* ptile, int lane, f32x4 d) {
  const half4_t h = *(const half4_t*)&ptile[2 * lane];
  const half4_t l = *(const half4_t*)&ptile[128 + 2 * lane];
  const half8_t p_hl = {h[0], h[1], h[2], h[3], l[0], l[1], l[2], l[3]};
  const half8_t p_lh = {l[0], l[1], l[2], l[3], h[0], h[1], h[2], h[3]};
  d = __builtin_amdgcn_mfma_f32_16x16x32_f16(q_hl, p_hl, d, 0, 0, 0);
  d = __builtin_amdgcn_mfma_f32_16x16x32_f16(q_hl, p_lh, d, 0, 0, 0);
  return d;
}

// Volatile LDS words used as intra-workgroup flags. Typed in the LDS address
// space so every access is a ds_read / ds_write (lgkmcnt only): through a generic
// pointer a volatile access stays a FLAT op, whose s_waitcnt vmcnt(0) would also
// drain every outstanding global store of the wave.
typedef __attribute__((address_space(3))) volatile int lds_vint;
GPK_DEVICE lds_vint* as_lds_flags(int* p) { return (lds_vint*)p; }

// Make this wave's LDS writes visible to its own other lanes before reading.
GPK_DEVICE void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Workgroup barrier ordering LDS only: unlike __syncthreads() it does not wait for the
// wave's outstanding global stores (s_waitcnt vmcnt(0)), so result stores and spills
// stay in flight across the barrier. Only for kernels whose threads never read global
// data another thread of the same launch wrote.
GPK_DEVICE void lds_barrier() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

GPK_DEVICE float readlane_f(float v, int lane) {
  return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), lane));
}

GPK_DEVICE int wave_id_uniform() {
  return __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
}

GPK_DEVICE float wave_sum(float v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}

// Max over the wave, result uniform. ds_swizzle (immediate xor pattern) needs
// no lane-address registers, unlike __shfl_xor.
GPK_DEVICE float wave_max(float v) {
#define GPK_SWZ_MAX(k) \
  v = __builtin_fmaxf(v, __builtin_bit_cast(float, __builtin_amdgcn_ds_swizzle(__builtin_bit_cast(int, v), ((k) << 10) | 0x1f)));
  GPK_SWZ_MAX(1) GPK_SWZ_MAX(2) GPK_SWZ_MAX(4) GPK_SWZ_MAX(8) GPK_SWZ_MAX(16)
#undef GPK_SWZ_MAX
  return __builtin_fmaxf(readlane_f(v, 0), readlane_f(v, 32));
}

// Max over the wave with DPP row permutes (pure VALU: no LDS-unit round trips,
// which queue behind other waves' LDS traffic) and four readlanes.
#define GPK_DPP_MAX(ctrl) \
  v = __builtin_fmaxf(v, __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), ctrl, 0xf, 0xf, false)));
GPK_DEVICE float wave_max_dpp(float v) {
  GPK_DPP_MAX(0xB1)   // quad_perm [1,0,3,2]
  GPK_DPP_MAX(0x4E)   // quad_perm [2,3,0,1]
  GPK_DPP_MAX(0x141)  // row_half_mirror
  GPK_DPP_MAX(0x140)  // row_mirror
  return __builtin_fmaxf(__builtin_fmaxf(readlane_f(v, 0), readlane_f(v, 16)),
                         __builtin_fmaxf(readlane_f(v, 32), readlane_f(v, 48)));
}
#undef GPK_DPP_MAX

GPK_DEVICE double wave_sum_d(double v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}

// Select element 4*g + r of a 16-entry register array with a per-lane g (0..3)
// without dynamic register indexing (which would go to scratch).
GPK_DEVICE f32x4 pick_group4(const float (&v)[16], int g) {
  f32x4 o;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    float a = v[r], b = v[4 + r], c = v[8 + r], d = v[12 + r];
    o[r] = g == 0 ? a : (g == 1 ? b : (g == 2 ? c : d));
  }
  return o;
}

// Tile enumeration for an upper-triangular tile set of NB block rows/cols plus
// an optional right-hand-side block column (index NB):
//   t <  NB(NB+1)/2 : (i, j) with i <= j < NB, column-major  t = j(j+1)/2 + i
//   t >= NB(NB+1)/2 : (t - NB(NB+1)/2, NB)
GPK_DEVICE void tile_of(int t, int NB, int& i, int& j) {
  const int tu = NB * (NB + 1) / 2;
  if (t >= tu) { i = t - tu; j = NB; return; }
  int jj = (int)((__builtin_sqrtf(8.0f * (float)t + 1.0f) - 1.0f) * 0.5f);
  while ((jj + 1) * (jj + 2) / 2 <= t) ++jj;
  while (jj * (jj + 1) / 2 > t) --jj;
  j = jj;
  i = t - jj * (jj + 1) / 2;
}
