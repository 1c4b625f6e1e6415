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
// Two phases (three launches in the fp32 form; ONE launch, gpk_grad_fused_kernel,
// for NB = 16), inputs are the forward's L and z (nothing is refactored):
//   gpk_grad_solve_kernel  one workgroup (16 waves) per window: alpha = L^-T z, dy, and the
//       lower block tiles of K^-1: wave J solves block column J with its tiles in registers
//         forward   V_I = -Linv_II sum_{K=J}^{I-1} L_IK V_K       (I > J, V_J = Linv_JJ)
//                   alpha_J += V_IJ^T z_I                          (alpha = V^T z, block J)
//         backward  U_I =  Linv_II^T (V_I - sum_{K>I} L_KI^T U_K)  (I = NB-1 .. J)
//       split-f16 MFMA (GPK_GRAD_SPLIT); all waves step together and each step's block row /
//       column of L is staged once in LDS (as split planes) by the workgroup, fetched two
//       steps ahead (double buffer); the diagonal-block inverses Linv_II live in LDS.
//       U_I = K^-1_IJ -> workspace.
//   gpk_grad_gram_split_kernel (gpk_grad_gram_kernel: the fp32 form) one wave per (window,
//       block row I), no atomics: for every J the tile K^-1_JI (stored, or the transpose of
//       the stored K^-1_IJ), the RBF tile recomputed from xs (split-f16 MFMA Gram), G, W and
//       Wx_I += W_JI^T xs_J (split-f16 MFMA, W scaled by a power of two), w1_I; then dX of
//       rows I and the block row's partials of ds2, dnoise, dl, summed in a fixed order by
//       the same workgroup -> dhyp (deterministic; gpk_grad_fin_kernel in the fp32 form).
#include "gpk_common.h"
#include "gpk_internal.h"

#include <mutex>
#include <type_traits>

// Timing experiments only (A/B builds of the solve kernel; results are wrong when set):
// bit 1 skips the phase-1 tile math, 2 the phase-2 tile math, 4 the L staging, 8 the
// K^-1 tile stores, 16 the alpha products, 32 the phase-2 staging stores, 64 the split gram
// kernel's J loop.
#ifndef GPK_GRAD_SKIP
#define GPK_GRAD_SKIP 0
#endif
// 1: the solve's tile products on split-f16 MFMA (operands rounded to hi + lo f16, 22
// significant bits; every product exact, fp32 accumulation -- the forward's trailing-update
// scheme); 0: fp32 MFMA (mfma_f32_16x16x4f32). B=512 N=256 D=32 backward:
// 0.153 ms split vs 0.184 ms fp32 (scripts/ab/gpu_grad_abt.sh), same accuracy vs the oracle.
#ifndef GPK_GRAD_SPLIT
#define GPK_GRAD_SPLIT 1
#endif
// Timeline builds (GPK_GRAD_STAMPS=1, timing only): the solve kernel writes s_memtime
// stamps into dX (which the gram kernel then leaves alone): per window, per step s (0..2NB-1),
// per wave, 4 events (step start, math done, barrier passed, staging stored).
#ifndef GPK_GRAM_WPE
#define GPK_GRAM_WPE 4   // split gram kernel, D <= 32: waves per SIMD it is compiled for (8: spills,
                         // 0.167 vs 0.139 ms for the whole backward)
#endif
#ifndef GPK_GRAD_STAMPS
#define GPK_GRAD_STAMPS 0
#endif
// 1: NB = 16 windows (N in 241..256) run the solve and the gram as one launch
// (gpk_grad_fused_kernel); 0: two launches.
#ifndef GPK_GRAD_FUSED
#define GPK_GRAD_FUSED 1
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

// D += Q^T P with Q, P split-f16 operands in registers ({hi, lo} per lane, acc layout):
// hi.hi + lo.lo, then lo.hi + hi.lo -- two K=32 f16 MFMAs, every product exact.
GPK_DEVICE f32x4 mma_split(const half8_t q, const half8_t p, f32x4 d) {
  const half8_t q_lh = {q[4], q[5], q[6], q[7], q[0], q[1], q[2], q[3]};
  d = __builtin_amdgcn_mfma_f32_16x16x32_f16(q, p, d, 0, 0, 0);
  d = __builtin_amdgcn_mfma_f32_16x16x32_f16(q_lh, p, d, 0, 0, 0);
  return d;
}
GPK_DEVICE half8_t to_split(const f32x4 v) {
  half4_t h, l;
  (void)round_split_f16(v, h, l);
  return half8_t{h[0], h[1], h[2], h[3], l[0], l[1], l[2], l[3]};
}
GPK_DEVICE f32x4 from_split(const half8_t v) {
  return f32x4{(float)v[0] + (float)v[4], (float)v[1] + (float)v[5], (float)v[2] + (float)v[6],
               (float)v[3] + (float)v[7]};
}
// Operand tile -> LDS split planes: the value of (lane l, reg r) of the acc layout.
GPK_DEVICE void put_split_elem(float* tile, int l, int r, float v) {
  const _Float16 h = (_Float16)v;
  ((_Float16*)tile)[4 * l + r] = h;
  ((_Float16*)(tile + 128))[4 * l + r] = (_Float16)(v - (float)h);
}

GPK_DEVICE f32x4 mfma4(const f32x4 a, const f32x4 b, f32x4 d) {
  d = __builtin_amdgcn_mfma_f32_16x16x4f32(a[0], b[0], d, 0, 0, 0);
  d = __builtin_amdgcn_mfma_f32_16x16x4f32(a[1], b[1], d, 0, 0, 0);
  d = __builtin_amdgcn_mfma_f32_16x16x4f32(a[2], b[2], d, 0, 0, 0);
  d = __builtin_amdgcn_mfma_f32_16x16x4f32(a[3], b[3], d, 0, 0, 0);
  return d;
}

// Compile-time loop A..B inclusive (register-array indices stay constants: a rolled loop
// would index X[] dynamically and move it to scratch)
template <int V>
struct IdxC { static constexpr int value = V; };
template <int A, int B, typename F>
GPK_DEVICE void sfor(F&& f) {
  if constexpr (A <= B) {
    f(IdxC<A>{});
    sfor<A + 1, B>(f);
  }
}

// Uniform value the compiler must treat as unknown at this point: keeps per-tile
// addresses from being hoisted out of their step (live addresses would spill).
GPK_DEVICE int opaque_s(int v) {
  asm volatile("" : "+s"(v));
  return v;
}

// Per-lane value the compiler must treat as unknown here (keeps a per-lane address from
// being hoisted out of its step and kept live -- or spilled -- across the whole kernel).
GPK_DEVICE int opaque_v(int v) {
  asm volatile("" : "+v"(v));
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
  int dinv, dsa, dsb, stg, sv, alpha, red, total;
};
__host__ __device__ inline SolveLds solve_lds(int NB) {
  SolveLds o;
  const int TS = (NB > 1 ? NB - 1 : 1) * 256;
  const int stg = 2 * TS > NB * 256 ? 2 * TS : NB * 256;   // (prologue: diagonal blocks of L)
  o.dinv = 0;                     // NB x 16 x 16 row-major Linv_II
  o.dsa = o.dinv + NB * 256;      // GPK_GRAD_SPLIT: Linv_II^T as split planes (phase-1 operand)
  o.dsb = o.dsa + (GPK_GRAD_SPLIT ? NB * 256 : 0);   // Linv_II as split planes (phase 2)
  o.stg = o.dsb + (GPK_GRAD_SPLIT ? NB * 256 : 0);
  o.sv = o.stg + stg;             // NP
  o.alpha = o.sv + 16 * NB;       // NP
  o.red = o.alpha + 16 * NB;      // kST column-sum partials + 64
  o.total = o.red + kST + 64;
  return o;
}

template <int NB, bool FULL>
GPK_DEVICE void grad_solve_body(const GpkExactGradArgs& a, float* smem) {
  constexpr bool SPLIT = GPK_GRAD_SPLIT && NB > 0;   // (dependent: the other branch is discarded)
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
      if constexpr (SPLIT) {
#pragma unroll
        for (int m = 0; m < 16; ++m) {
          put_split_elem(smem + lay.dsa + bi * 256, 16 * (cc >> 2) + m, cc & 3, x[m]);   // Linv^T
          put_split_elem(smem + lay.dsb + bi * 256, 16 * (m >> 2) + cc, m & 3, x[m]);    // Linv
        }
      }
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
  const float gw = a.gout[b];
  const float invN = 1.f / (float)N;
  const f32x4 z4 = {0.f, 0.f, 0.f, 0.f};
  // The staging prefetch of a step is issued and consumed under wave-uniform branches; at the
  // join the compiler cannot tell that the load was consumed, and waits for vmcnt(0) (this
  // step's fresh prefetch included) the first time it reuses the old destination registers --
  // at the start of the step's math, exposing the whole global latency every step. An
  // unconditional vmcnt(0) right after the staging store (where the wave waits anyway)
  // retires the old load on every path.
  // window's L as a buffer resource (FULL: N*N*4 bytes < 2^31)
  const __amdgpu_buffer_rsrc_t lrsrc =
      __builtin_amdgcn_make_buffer_rsrc((void*)Lb, 0, 0x7fffffff, 0x00020000);
  auto lbuf_load = [&](int off) -> f32x4 {
    return __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(lrsrc, 4 * off, 0, 0));
  };
  auto vm_drain = [&]() { __builtin_amdgcn_s_waitcnt(0x0F70); };   // vmcnt(0) only
  auto fetch_row = [&](const int I) -> f32x4 {    // tiles (I, K < I), row-major
    if (tid >= I * 64 || (GPK_GRAD_SKIP & 4)) return z4;
    const int K = tid >> 6, q = tid & 63, m = q >> 2, cg = (q & 3) * 4;
    const int row = 16 * I + m, col0 = 16 * K + cg;
    if (FULL) return lbuf_load(row * N + col0);
    f32x4 v;
#pragma unroll
    for (int j = 0; j < 4; ++j) v[j] = (row < N && col0 + j < N) ? Lb[(size_t)row * N + col0 + j] : 0.f;
    return v;
  };
  auto put_row = [&](float* buf, const int I, const f32x4 v) {
    if (tid >= I * 64) return;
    const int K = tid >> 6, q = tid & 63, m = q >> 2, cg = (q & 3) * 4;
    if constexpr (SPLIT) {   // reader lane (g, c) = (q & 3, m) takes row m, columns 4g..4g+3
      half4_t h, l;
      (void)round_split_f16(v, h, l);
      store_split_planes(buf + K * 256, 16 * (q & 3) + m, h, l);
    } else {
      *(f32x4*)&buf[K * 256 + m * 16 + cg] = v;
    }
  };
  auto fetch_col = [&](const int I) -> f32x4 {    // tiles (K > I, I)
    if (tid >= (NB - 1 - I) * 64 || (GPK_GRAD_SKIP & 4)) return z4;
    const int sl = tid >> 6, q = tid & 63;
    if constexpr (SPLIT) {
      // lane (g, c) = (q >> 4, q & 15) loads the column segment L_KI[4g .. 4g+3][c] (rows of
      // the acc layout): 4 dword loads, each 16 lanes reading 64 contiguous bytes, so the
      // staging store is two 8-byte split-plane writes instead of eight 2-byte scatters
      const int g4 = 4 * (q >> 4), cc = q & 15;
      const int row0 = 16 * (I + 1 + sl) + g4, col = 16 * I + cc;
      f32x4 v;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        if (FULL) {
          v[r] = Lb[opaque_v((row0 + r) * N + col)];
        } else {
          v[r] = (row0 + r < N && col < N) ? Lb[(size_t)(row0 + r) * N + col] : 0.f;
        }
      }
      return v;
    } else {
      const int k = q >> 2, cg = (q & 3) * 4;
      const int row = 16 * (I + 1 + sl) + k, col0 = 16 * I + cg;
      if (FULL) return lbuf_load(row * N + col0);
      f32x4 v;
#pragma unroll
      for (int j = 0; j < 4; ++j) v[j] = (row < N && col0 + j < N) ? Lb[(size_t)row * N + col0 + j] : 0.f;
      return v;
    }
  };
  auto put_col = [&](float* buf, const int I, const f32x4 v) {   // stored transposed
    if (tid >= (NB - 1 - I) * 64) return;
    const int sl = tid >> 6, q = tid & 63;
    if constexpr (SPLIT) {   // v is already the acc-layout column segment of lane q
      half4_t h, l;
      (void)round_split_f16(v, h, l);
      store_split_planes(buf + sl * 256, q, h, l);
    } else {
      const int k = q >> 2, cg = (q & 3) * 4;
#pragma unroll
      for (int j = 0; j < 4; ++j) buf[sl * 256 + (cg + j) * 16 + k] = v[j];
    }
  };
  // X[K]: the wave's tile of block row K (V, then U = K^-1), an MFMA B operand: fp32 acc
  // layout, or split-f16 {hi, lo} (GPK_GRAD_SPLIT)
  using XT = typename std::conditional<SPLIT, half8_t, f32x4>::type;
  // independent MFMA accumulator chains (split: 2; 4 measured 1.7 µs slower per launch)
  constexpr int NCH = SPLIT ? 2 : 4;
  // X[K < J] stay zero: a wave may run the products of a whole group of 4 tiles (below)
  XT X[NB];
  sfor<0, NB - 1>([&](auto Kc) { X[decltype(Kc)::value] = XT{}; });
  const float* dsa = smem + lay.dsa;
  const float* dsb = smem + lay.dsb;
  // s[K % NCH] += Q_K^T X[K] for K in [KLO, KHI], Q_K the staged tile at base + (K - KOFS)
  // tiles, in groups of 4 tiles (one wave-uniform branch per group, kmin <= the group's last
  // K): the group's LDS operands are all loaded before its MFMAs, so the LDS latency is paid
  // once per group, not once per product
  auto prod_range = [&](f32x4* s, const float* base, auto KLOc, auto KHIc, auto KOFSc, int kmin) {
    constexpr int KLO = decltype(KLOc)::value, KHI = decltype(KHIc)::value;
    constexpr int KOFS = decltype(KOFSc)::value;
    constexpr int GS = 4;   // (groups of 2 or 8: 1-2 µs slower per launch)
    sfor<0, (KHI - KLO + GS) / GS - 1>([&](auto Qc) {
      constexpr int K0 = KLO + GS * decltype(Qc)::value;
      constexpr int K1 = (K0 + GS - 1 < KHI) ? K0 + GS - 1 : KHI;
      if (kmin <= K1) {
        XT op[GS];
        sfor<K0, K1>([&](auto Kc) {
          constexpr int K = decltype(Kc)::value;
          const float* tile = base + (K - KOFS) * 256;
          if constexpr (SPLIT) op[K - K0] = load_split_hl(tile, lane);
          else op[K - K0] = *(const f32x4*)&tile[c * 16 + 4 * g];
        });
        sfor<K0, K1>([&](auto Kc) {
          constexpr int K = decltype(Kc)::value;
          if constexpr (SPLIT) s[K % NCH] = mma_split(op[K - K0], X[K], s[K % NCH]);
          else s[K % NCH] = mfma4(op[K - K0], X[K], s[K % NCH]);
        });
      }
    });
  };
  // Step s reads buffer s & 1: phase 1 step I (s = I) block row I, phase 2 step I
  // (s = 2NB-1-I) block column I. The tiles of step s+2 are fetched during step s and
  // written into buffer s & 1 after the step's barrier (everyone is done reading it).
  unsigned long long* stamps = (unsigned long long*)(a.dX + (size_t)b * N * D);
  auto stamp = [&](int st, int ev) {
    if constexpr (GPK_GRAD_STAMPS) {
      if (lane == 0) stamps[(st * kSW + wave) * 4 + ev] = __builtin_amdgcn_s_memtime();
    }
  };
  f32x4 al = z4;   // alpha block J (column 0 of the acc tile)
  if (NB > 1) put_row(stg + TS, 1, fetch_row(1));
  lds_barrier();
  sfor<0, NB - 1>([&](auto Ic) {
    constexpr int I = decltype(Ic)::value;
    stamp(I, 0);
    const f32x4 nxt = (I + 2 < NB) ? fetch_row(I + 2) : ((I + 2 == NB + 1 && NB >= 2) ? fetch_col(NB - 2) : z4);
    const float* buf = stg + (I & 1) * TS;
    const int I16 = opaque_s(16 * I);
    if (live && !(GPK_GRAD_SKIP & 1)) {
      if (I == J) {
        if constexpr (SPLIT) {
          X[I] = load_split_hl(dsb + I16 * 16, lane);
        } else {
#pragma unroll
          for (int r = 0; r < 4; ++r) X[I][r] = dinv[I16 * 16 + (4 * g + r) * 16 + c];
        }
      } else if (I > J) {
        f32x4 s[4] = {z4, z4, z4, z4};   // 4 independent MFMA chains
        prod_range(s, buf, IdxC<0>{}, IdxC<I - 1>{}, IdxC<0>{}, J);
        const f32x4 t = (NCH == 4 ? (s[0] + s[1]) + (s[2] + s[3]) : (NCH == 2 ? s[0] + s[1] : s[0]));
        if constexpr (SPLIT) {
          X[I] = to_split(-mma_split(load_split_hl(dsa + I16 * 16, lane), to_split(t), z4));
        } else {
          const f32x4 di = *(const f32x4*)&dinv[I16 * 16 + c * 16 + 4 * g];
          X[I] = -mfma4(di, t, z4);
        }
      }
      // alpha_J += V_IJ^T z_I  (alpha = L^-T z = V^T z, block J; z_I in column 0 of a tile)
      if (I >= J && !(GPK_GRAD_SKIP & 16)) {
        f32x4 zt;
#pragma unroll
        for (int r = 0; r < 4; ++r) zt[r] = c == 0 ? sv[16 * I + 4 * g + r] : 0.f;
        if constexpr (SPLIT) al = mma_split(X[I], to_split(zt), al);
        else al = mfma4(X[I], zt, al);
      }
    }
    stamp(I, 1);
    lds_barrier();
    stamp(I, 2);
    if (I + 2 < NB) put_row(stg + (I & 1) * TS, I + 2, nxt);
    else if (I + 2 == NB + 1 && NB >= 2) put_col(stg + (I & 1) * TS, NB - 2, nxt);   // step 2NB-1-(NB-2)
    vm_drain();
    stamp(I, 3);
  });
  // alpha block J -> workspace, dy; per-wave partial of sum(alpha) (summed after phase 2)
  if (live) {
    float asp = 0.f;
    if (c == 0) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int n = 16 * J + 4 * g + r;
        const float an = al[r];
        wsb[ws.alpha + n] = an;
        if (FULL || n < N) {
          asp += an;
          if (a.dy != nullptr) a.dy[(size_t)b * N + n] = -gw * an * invN;
        }
      }
    }
    asp = wave_sum(asp);
    if (lane == 0) red[J] = asp;
  }
  lds_barrier();
  // U_I = Linv_II^T t  (Q = Linv_II)
  auto back_tile = [&](const int I16, const f32x4 t) -> f32x4 {
    if constexpr (SPLIT) {
      return mma_split(load_split_hl(dsb + I16 * 16, lane), to_split(t), z4);
    } else {
      f32x4 dt;
#pragma unroll
      for (int r = 0; r < 4; ++r) dt[r] = dinv[I16 * 16 + (4 * g + r) * 16 + c];
      return mfma4(dt, t, z4);
    }
  };
  auto as_f32 = [&](const XT& x) -> f32x4 {
    if constexpr (SPLIT) return from_split(x); else return x;
  };
  auto as_x = [&](const f32x4 v) -> XT {
    if constexpr (SPLIT) return to_split(v); else return v;
  };
  sfor<0, NB - 1>([&](auto Tc) {
    constexpr int I = NB - 1 - decltype(Tc)::value;
    const int st = 2 * NB - 1 - I;
    stamp(st, 0);
    const f32x4 nxt = (I > 1) ? fetch_col(I - 2) : z4;
    const float* buf = stg + (st & 1) * TS;
    const int I16 = opaque_s(16 * I);
    if (live && I >= J && !(GPK_GRAD_SKIP & 2)) {
      f32x4 s[4] = {z4, z4, z4, z4};   // 4 independent MFMA chains
      prod_range(s, buf, IdxC<I + 1>{}, IdxC<NB - 1>{}, IdxC<I + 1>{}, 0);
      const f32x4 U = back_tile(I16, as_f32(X[I]) - ((NCH == 4 ? (s[0] + s[1]) + (s[2] + s[3]) : (NCH == 2 ? s[0] + s[1] : s[0]))));
      X[I] = as_x(U);
      if (!(GPK_GRAD_SKIP & 8)) *(f32x4*)&wsb[ws.kinv + (size_t)tile_index(I, J) * 256 + lane * 4] = U;
    }
    stamp(st, 1);
    lds_barrier();
    stamp(st, 2);
    if (I > 1 && !(GPK_GRAD_SKIP & 32)) put_col(stg + (st & 1) * TS, I - 2, nxt);
    vm_drain();
    stamp(st, 3);
  });
  if (tid == 0) {   // fixed-order sum of the per-block partials (deterministic)
    float asum = 0.f;
    for (int j = 0; j < NB; ++j) asum += red[j];
    wsb[ws.asum] = asum;
  }
}

template <int NB, bool FULL>
__global__ void __launch_bounds__(kST, 1) gpk_grad_solve_kernel(GpkExactGradArgs a) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  grad_solve_body<NB, FULL>(a, smem);
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
        if (a.dX != nullptr && !GPK_GRAD_STAMPS) a.dX[((size_t)b * N + row) * D + d] = -2.f * e * ilq;
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

// Split-f16 form of the same contractions (GPK_GRAD_SPLIT): xs is staged ONCE as hi + lo f16
// planes in two layouts -- rows (the Gram operands: lane (g, c) takes dims 8g..8g+7 of a row)
// and columns (the Wx operand: lane (g, c) takes rows 4g..4g+3 of a dim) -- so the RBF Gram
// is 3 K=32 f16 MFMAs per 32 dims (hi.hi + hi.lo + lo.hi, as the forward builds K) and
// Wx_I += W_JI^T xs_J is 2 per 16 dims (exact products of the split W and xs), against 8 + 8
// fp32 MFMAs. Norms and the dX epilogue use the rounded xs^ = hi + lo (22 bits).
struct GramLds {
  int RS, TSd, xh, xl, th, tl, nrm, al, bmax, part, total_bytes;
};
__host__ __device__ inline GramLds gram_lds(int NP, int DQ) {
  GramLds o;
  const int DP = 16 * DQ, DW = DP < 32 ? 32 : DP;
  o.RS = DW + 8;          // row-plane stride (halves): 16-B reads of 8 rows conflict-free
  o.TSd = NP + 16;        // column-plane stride (halves): 8-B reads of 32 lanes conflict-free
  o.xh = 0;               // offsets in halves
  o.xl = o.xh + NP * o.RS;
  o.th = o.xl + NP * o.RS;
  o.tl = o.th + DP * o.TSd;
  const int fl = ((o.tl + DP * o.TSd) * 2 + 15) / 16 * 4;   // float offset, 16-B aligned
  o.nrm = fl;
  o.al = o.nrm + NP;
  o.bmax = o.al + NP;          // 2 x 16 block-max slots
  o.part = o.bmax + 32;        // NB x (2 + DP) block-row partials (ds2, dnoise, dl[d])
  o.total_bytes = (o.part + (NP / 16) * (2 + DP)) * 4;
  return o;
}

template <int DQ, bool FULL>
GPK_DEVICE void grad_gram_split_body(const GpkExactGradArgs& a, float* smem) {
  constexpr int DP = 16 * DQ, DW = DP < 32 ? 32 : DP, KC = DW / 32;
  const int N = a.N, D = a.D;
  const GradWs ws = grad_ws(N);
  const int NB = ws.NB, NP = 16 * NB;
  const GramLds lay = gram_lds(NP, DQ);
  const int RS = lay.RS, TSd = lay.TSd;
  _Float16* hs = (_Float16*)smem;
  _Float16* xh = hs + lay.xh;
  _Float16* xl = hs + lay.xl;
  _Float16* th = hs + lay.th;
  _Float16* tl = hs + lay.tl;
  float* nrm = smem + lay.nrm;
  float* al = smem + lay.al;
  const int tid = threadIdx.x, lane = tid & 63, I = tid >> 6;
  const int c = lane & 15, g = lane >> 4;
  const int b = blockIdx.x;
  const float* Xb = a.X + (size_t)b * N * D;
  const float* wsb = a.ws + (size_t)b * ws.per;
  const float* hyp = a.hyp;
  const bool ard = a.n_ls > 1;
  // xs = x / l - mean -> split planes (rows: dims 0..DW-1, zero padded; columns: dims < DP)
  for (int base = 0; base < NP * DW; base += 4 * 64 * kGW) {
    float v[4], l[4], mu[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int e = base + u * 64 * kGW + tid, n = e / DW, d = e - n * DW;
      const bool ok = e < NP * DW && (FULL || n < N) && d < D;
      v[u] = Xb[ok ? (size_t)n * D + d : 0];
      l[u] = hyp[3 + ((ok && ard) ? d : 0)];
      mu[u] = wsb[ws.mean + (ok ? d : 0)];
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int e = base + u * 64 * kGW + tid, n = e / DW, d = e - n * DW;
      if (e < NP * DW) {
        const float x = ((FULL || n < N) && d < D) ? v[u] / l[u] - mu[u] : 0.f;
        const _Float16 h = (_Float16)x, lo = (_Float16)(x - (float)h);
        xh[n * RS + d] = h;
        xl[n * RS + d] = lo;
        if (d < DP) {
          th[d * TSd + n] = h;
          tl[d * TSd + n] = lo;
        }
      }
    }
  }
  // W = G s2 E is scaled by a power of two S before its hi + lo split, so that its largest
  // entries sit near 2^10 (f16 keeps their lo part normal; W itself is ~1/N-sized and its lo
  // part would underflow): |W_ij| <= |gs| s2 (max|alpha|^2 + max_j K^-1_jj)
  float* bmax = smem + lay.bmax;
  float* pl = smem + lay.part;
  float am = 0.f, tm = 0.f;
  for (int n = tid; n < NP; n += 64 * kGW) {
    const float an = wsb[ws.alpha + n];
    al[n] = an;
    am = __builtin_fmaxf(am, __builtin_fabsf(an));
    const int Jn = n >> 4, m = n & 15;
    tm = __builtin_fmaxf(tm, __builtin_fabsf(wsb[ws.kinv + (size_t)tile_index(Jn, Jn) * 256 +
                                                 (16 * (m >> 2) + m) * 4 + (m & 3)]));
  }
  am = wave_max(am);
  tm = wave_max(tm);
  if (lane == 0) {
    bmax[I] = am;
    bmax[16 + I] = tm;
  }
  lds_barrier();
  for (int n = tid; n < NP; n += 64 * kGW) {
    // |xs_n|^2 from the planes, 16-byte reads (the same dims in the same order as 2-byte reads)
    float t = 0.f;
#pragma unroll
    for (int d0 = 0; d0 < DW; d0 += 8) {
      const half8_t h8 = *(const half8_t*)&xh[n * RS + d0];
      const half8_t l8 = *(const half8_t*)&xl[n * RS + d0];
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const float x = (float)h8[q] + (float)l8[q];
        t = __builtin_fmaf(x, x, t);
      }
    }
    nrm[n] = t;
  }
  lds_barrier();
  const float s2 = hyp[0];
  const float gw = a.gout[b];
  const float gs = gw / (2.f * (float)N);
  float wscale = 1.f;
  {
    float amax = 0.f, tmax = 0.f;
    for (int w = 0; w < kGW; ++w) {
      amax = __builtin_fmaxf(amax, bmax[w]);
      tmax = __builtin_fmaxf(tmax, bmax[16 + w]);
    }
    const float bound = __builtin_fabsf(gs) * __builtin_fabsf(s2) * (amax * amax + tmax);
    if (bound > 0.f && bound < 3.0e38f)
      wscale = __builtin_ldexpf(1.f, 10 - (int)__builtin_ceilf(__builtin_log2f(bound)));
  }
  constexpr float nhalf_log2e = -0.72134752044448170f;
  if (I < NB) {   // wave-uniform (the waves of a short window still meet the final barrier)
  // Gram B operand for the columns i = 16I + c: dims 32kc + 8g .. +7 of row i
  half8_t bh[KC], bl[KC];
#pragma unroll
  for (int kc = 0; kc < KC; ++kc) {
    bh[kc] = *(const half8_t*)&xh[(16 * I + c) * RS + 32 * kc + 8 * g];
    bl[kc] = *(const half8_t*)&xl[(16 * I + c) * RS + 32 * kc + 8 * g];
  }
  const int col = 16 * I + c;
  const float ni = nrm[col], ai = al[col];
  f32x4 wx[DQ];
#pragma unroll
  for (int q = 0; q < DQ; ++q) wx[q] = f32x4{0.f, 0.f, 0.f, 0.f};
  float w1p = 0.f, ds2 = 0.f, dnz = 0.f;
  auto load_T = [&](int J) -> f32x4 {   // K^-1_JI in acc layout (rows j, cols i)
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
  for (int J = 0; J < ((GPK_GRAD_SKIP & 64) ? 0 : NB); ++J) {
    const f32x4 T = Tn;
    if (J + 1 < NB) Tn = load_T(J + 1);
    const int j0 = 16 * J;
    f32x4 gr = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kc = 0; kc < KC; ++kc) {
      const half8_t ah = *(const half8_t*)&xh[(j0 + c) * RS + 32 * kc + 8 * g];
      const half8_t alo = *(const half8_t*)&xl[(j0 + c) * RS + 32 * kc + 8 * g];
      gr = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, bh[kc], gr, 0, 0, 0);
      gr = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, bl[kc], gr, 0, 0, 0);
      gr = __builtin_amdgcn_mfma_f32_16x16x32_f16(alo, bh[kc], gr, 0, 0, 0);
    }
    half8_t pj[DQ];   // xs_J columns 16q + c, rows j0 + 4g .. +3 (hi | lo)
#pragma unroll
    for (int q = 0; q < DQ; ++q) {
      const half4_t h4 = *(const half4_t*)&th[(16 * q + c) * TSd + j0 + 4 * g];
      const half4_t l4 = *(const half4_t*)&tl[(16 * q + c) * TSd + j0 + 4 * g];
      pj[q] = half8_t{h4[0], h4[1], h4[2], h4[3], l4[0], l4[1], l4[2], l4[3]};
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
    // Wx_I += W_JI^T xs_J  (rows i, dims): split W times split xs, exact products
    const half8_t ws8 = to_split(W * wscale);
#pragma unroll
    for (int q = 0; q < DQ; ++q) wx[q] = mma_split(ws8, pj[q], wx[q]);
  }
#pragma unroll
  for (int q = 0; q < DQ; ++q) wx[q] = wx[q] * (1.f / wscale);   // (exact: a power of two)
  w1p += __shfl_xor(w1p, 16, 64);
  w1p += __shfl_xor(w1p, 32, 64);
  float w1r[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) w1r[r] = __shfl(w1p, 4 * g + r, 64);
  float* part = pl + I * (2 + DP);
#pragma unroll
  for (int q = 0; q < DQ; ++q) {
    const int d = 16 * q + c;
    const float ilq = d < D ? 1.f / hyp[3 + (ard ? d : 0)] : 0.f;
    float lp = 0.f;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int row = 16 * I + 4 * g + r;
      const float x = (float)xh[row * RS + d] + (float)xl[row * RS + d];
      const float e = x * w1r[r] - wx[q][r];   // = -dxs / 2
      if ((FULL || row < N) && d < D) {
        if (a.dX != nullptr && !GPK_GRAD_STAMPS) a.dX[((size_t)b * N + row) * D + d] = -2.f * e * ilq;
        lp = __builtin_fmaf(x, e, lp);
      }
    }
    lp += __shfl_xor(lp, 16, 64);
    lp += __shfl_xor(lp, 32, 64);
    if (g == 0) part[2 + d] = lp;
  }
  ds2 = wave_sum(ds2);
  dnz = wave_sum(dnz);
  if (lane == 0) {
    part[0] = ds2;
    part[1] = dnz;
  }
  }
  // fixed-order sums of the block-row partials -> dhyp (gpk_grad_fin_kernel, fused)
  lds_barrier();
  if (tid < 128) {
    float* o = a.dhyp + (size_t)b * (3 + a.n_ls);
    const int t = tid;
    const int f = t < 64 ? (t < D ? 2 + t : -1) : (t == 64 ? 0 : (t == 65 ? 1 : -1));
    float sacc = 0.f;
    if (f >= 0)
      for (int I2 = 0; I2 < NB; ++I2) sacc += pl[I2 * (2 + DP) + f];
    if (t == 64) o[0] = sacc;
    if (t == 65) o[1] = sacc;
    if (t == 66) o[2] = gw * wsb[ws.asum] / (float)N;
    if (t < 64) {
      if (a.n_ls == 1) {
        const float tot = wave_sum(sacc);
        if (t == 0) o[3] = 2.f * tot / hyp[3];
      } else if (t < D) {
        o[3 + t] = 2.f * sacc / hyp[3 + t];
      }
    }
  }
}

template <int DQ, bool FULL>
__global__ void __launch_bounds__(64 * kGW, DQ == 4 ? 4 : GPK_GRAM_WPE) gpk_grad_gram_split_kernel(GpkExactGradArgs a) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  grad_gram_split_body<DQ, FULL>(a, smem);
}

// The solve and the gram in ONE launch (NB = 16, split form): the same 16-wave workgroup runs
// the gram after the solve, so the K^-1 tiles the solve's waves store are read back by the
// other waves of the same workgroup (L2-resident) instead of by a second launch from HBM; the
// gram re-stages its LDS from offset 0 once the solve is done with it.
template <int DQ, bool FULL>
__global__ void __launch_bounds__(kST, 1) gpk_grad_fused_kernel(GpkExactGradArgs a) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  grad_solve_body<16, FULL>(a, smem);
  __syncthreads();   // every wave's workspace stores visible (workgroup scope); LDS reusable
  grad_gram_split_body<DQ, FULL>(a, smem);
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
  if (GPK_GRAD_SPLIT) {
    const size_t lds = (size_t)gram_lds(16 * NB, DQ).total_bytes;
    if (lds > 160 * 1024) return -7;
    static std::once_flag once_s;
    std::call_once(once_s, [&] {
      (void)hipFuncSetAttribute((const void*)gpk_grad_gram_split_kernel<DQ, true>,
                                hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
      (void)hipFuncSetAttribute((const void*)gpk_grad_gram_split_kernel<DQ, false>,
                                hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
      (void)hipGetLastError();
    });
    if (a.N == 16 * NB)
      hipLaunchKernelGGL((gpk_grad_gram_split_kernel<DQ, true>), dim3(a.B), dim3(64 * kGW), lds, stream, a);
    else
      hipLaunchKernelGGL((gpk_grad_gram_split_kernel<DQ, false>), dim3(a.B), dim3(64 * kGW), lds, stream, a);
    return (int)hipGetLastError();
  }
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

template <int DQ>
int launch_fused(const GpkExactGradArgs& a, hipStream_t stream) {
  const size_t l1 = (size_t)solve_lds(16).total * sizeof(float);
  const size_t l2 = (size_t)gram_lds(256, DQ).total_bytes;
  const size_t lds = l1 > l2 ? l1 : l2;
  if (lds > 160 * 1024) return -7;
  static std::once_flag once;
  std::call_once(once, [&] {
    (void)hipFuncSetAttribute((const void*)gpk_grad_fused_kernel<DQ, true>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    (void)hipFuncSetAttribute((const void*)gpk_grad_fused_kernel<DQ, false>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    (void)hipGetLastError();
  });
  if (a.N == 256)
    hipLaunchKernelGGL((gpk_grad_fused_kernel<DQ, true>), dim3(a.B), dim3(kST), lds, stream, a);
  else
    hipLaunchKernelGGL((gpk_grad_fused_kernel<DQ, false>), dim3(a.B), dim3(kST), lds, stream, a);
  return (int)hipGetLastError();
}

int gpk_launch_exact_grad(const GpkExactGradArgs& a, hipStream_t stream) {
  if (GPK_GRAD_FUSED && GPK_GRAD_SPLIT && !GPK_GRAD_STAMPS && (a.N + 15) / 16 == 16)
    return a.D <= 16 ? launch_fused<1>(a, stream) : (a.D <= 32 ? launch_fused<2>(a, stream) : launch_fused<4>(a, stream));
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
  if (!GPK_GRAD_SPLIT)   // (the split gram kernel sums its partials itself)
    hipLaunchKernelGGL(gpk_grad_fin_kernel, dim3(a.B), dim3(128), 0, stream, a, 0);
  return (int)hipGetLastError();
}
