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
// Design: one workgroup of W waves per window, two workgroups
// per CU. The padded K_hat (NB x NB tiles of 16x16, upper triangle) lives in
// REGISTERS as MFMA accumulators (acc layout, see gpk_common.h) of the W-1
// worker waves; the right-hand side y - c is a block column in LDS. Tiles are
// dealt to workers in row-descending order (plan_tile), so at step k the tiles
// a wave still has to update are a PREFIX of its slots. The blocked
// right-looking Cholesky works on R = L^T (accumulators hold -T, so every
// update is a plain MFMA accumulate).
// The last wave is the DIAGONAL wave and owns the critical path alone:
//   factor (k,k) -> publish R_kk^{-T} -> R_{k,k+1} = R_kk^{-T} T'_{k,k+1} ->
//   T''_{k+1,k+1} = T'_{k+1,k+1} - R_{k,k+1}^T R_{k,k+1} -> factor (k+1,k+1)
// (look-ahead), fed by the workers with (k,k+1) and (k+1,k+1) updated through
// panel k-1. It never joins a barrier: the workers synchronise among
// themselves (LDS counter) and every hand-off is an LDS flag holding a
// monotone epoch. The workers per step: trailing update from panel k-1 (the
// two hand-over tiles first), upper-L zeroing, right-hand side, the deferred
// RBF of block row k+2 (the Gram is additive, so it may land after earlier
// updates), then the TRSM of block row k into panel k once R_kk^{-T} is out.
// Diagonal tiles are factored by one wave in one sweep: lanes 0-15 hold columns
// of R, lanes 16-31 columns of R^{-T}, and both are produced by the SAME
// readlane-broadcast instruction stream.
// Flag waits read LDS only (ds_read + lgkmcnt): the L stores stream out behind
// the factorisation instead of being drained at each step.
#include "gpk_common.h"
#include "gpk_internal.h"

#include "gpk_exact_dev.h"

namespace {

constexpr float kLog2Pi = 1.8378770664093453f;

// Static tile -> (wave, slot) plan (host-evaluable reference; the device uses the
// closed form plan_tile). Tiles are listed row-descending (i = NB-1
// .. 0), j = i..NB-1 inside a row, and dealt cyclically: tile t -> worker
// wave t % WK, slot t / WK. Then
//   tiles with i > k            = { t < P(k) },  P(k) = (NB-k)(NB-k-1)/2
//   diagonal tile (k,k)         = t = P(k)
//   off-diagonal row-k tiles    = P(k) < t <= P(k) + NB - k - 1
// The right-hand-side block column (y - c) is NOT in the plan: it has one live
// column, so it is kept in LDS (rw) instead of 16 register tiles; block row i
// of it belongs to worker i % WK.
template <int NB>
struct ExactPlan {
  static constexpr int NT = NB * (NB + 1) / 2;
  int ij[NT];   // i | j << 8
  constexpr ExactPlan() : ij() {
    int t = 0;
    for (int i = NB - 1; i >= 0; --i)
      for (int j = i; j < NB; ++j) ij[t++] = i | (j << 8);
  }
};

template <int NB>
GPK_DEVICE constexpr int plan_P(int k) {
  return (NB - k) * (NB - k - 1) / 2;
}

// Row-descending plan in closed form: tile t lies in block row i = NB - m where
// m(m-1)/2 <= t < m(m+1)/2, at column j = i + t - m(m-1)/2.
constexpr int plan_m(int t) {
  int m = 1;
  while ((m + 1) * m / 2 <= t) ++m;
  return m;
}

// Tile (i | j << 8) of plan index t, for t known to lie in [LO, HI] at compile
// time (t = wave + WK * slot): a short chain of scalar compares instead of a
// constant-memory lookup (which costs two dependent SMEM round trips per tile).
template <int M0, int HI, int Q>
GPK_DEVICE int plan_m_tail(int t) {
  constexpr int bq = (M0 + 1 + Q) * (M0 + Q) / 2;  // first tile of the row with m = M0 + 1 + Q
  if constexpr (bq > HI) {
    return M0 + Q;
  } else {
    return t >= bq ? plan_m_tail<M0, HI, Q + 1>(t) : M0 + Q;
  }
}

template <int NB, int LO, int HI>
GPK_DEVICE int plan_tile(int t) {
  const int m = plan_m_tail<plan_m(LO), HI, 0>(t);
  const int i = NB - m;
  const int j = i + t - m * (m - 1) / 2;
  return i | (j << 8);
}

// R_kk^{-T} in LDS: 16 rows of stride kWS floats (20: the diagonal wave's 16-B row writes and
// the workers' column reads are both conflict-free; 16 was 4-way on both)
constexpr int kWS = 20, kWBuf = 16 * kWS;

struct ExactLds {
  // offsets in floats
  int xf, xh, xl, nrm, rv, rw, panel, wbuf, dsc, hbuf, cpart, rbfc, red, total;
};

__host__ __device__ inline ExactLds exact_lds_layout(int NB, int DC, int W) {
  const int DC32 = (DC + 1) / 2;
  ExactLds o;
  o.xf = 0;                              // fp32 staging, later f16 hi/lo images (aliased)
  o.xh = 0;
  o.xl = 0;
  o.nrm = o.xf + NB * (2 * DC32) * 256;
  o.rv = o.nrm + NB * 16;
  o.rw = o.rv + NB * 16;                 // working copy of -(y - c) (the RHS column)
  o.panel = o.rw + NB * 16;
  o.wbuf = o.panel + 2 * (NB + 1) * 256;  // (panel: double-buffered R rows)
  o.dsc = o.wbuf + 3 * kWBuf;            // (wbuf: R_kk^{-T}, triple-buffered by step mod 3)
  o.hbuf = o.dsc + 256;                  // (dsc: the diagonal wave's working tile)
  // (hbuf: look-ahead hand-off {(k,k+1), (k+1,k+1)} x parity). The prologue's column
  // partials and means (64 W + 256 <= 1280 floats for W <= 16) alias dsc + hbuf: both are
  // first written after the prologue's closing barrier.
  o.cpart = o.dsc;
  o.rbfc = o.hbuf + 2 * 512;             // RbfK (16-byte aligned)
  o.red = o.rbfc + 4;
  o.total = o.red + 4 * W + 96;          // flag words (see the kFlag enum)
  if (kEpochCheck) o.total += 48;        // (check builds: epoch shadows, kShadowPan..)
  return o;
}

// fp32 staging of X (16x16x4 fragment layout, CHUNK-major so that 16-column
// chunks 2q and 2q+1 occupy exactly the bytes of the f16 hi / lo images of
// 32-column chunk q, which overwrite them in place).
GPK_DEVICE int frag_index(int n, int d, int NB) {
  const int blk = n >> 4, c = n & 15, dd = d >> 4, g = (d >> 2) & 3, r = d & 3;
  return ((dd * NB + blk) * 64 + 16 * g + c) * 4 + r;
}

// f16 hi (part 0) / lo (part 1) images of 32-column chunk q, 16x16x32 fragment
// layout: lane 16g + c of block b holds x[16b + c][32q + 8g + j], j = 0..7.
// Returned as a half index from the start of the staging area.
GPK_DEVICE int hfrag_index(int n, int d, int NB, int part) {
  const int blk = n >> 4, c = n & 15, q = d >> 5, g = (d >> 3) & 3, j = d & 7;
  return (2 * q + part) * NB * 512 + ((blk * 64) + 16 * g + c) * 8 + j;
}

GPK_DEVICE int launder_s(int v) {
  asm volatile("" : "+s"(v));
  return v;
}

// Workgroup barrier that orders LDS only; outstanding global stores keep flowing.
GPK_DEVICE void barrier_lds() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

// One 16-byte store into a window's L (base = the window's L, wave-uniform).
GPK_DEVICE void lstore(float* base, int off, const f32x4 v) {
  if constexpr (GPK_LST_AUX < 0) {
    *(f32x4*)&base[off] = v;
  } else {
    typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
    const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(base, 0, 0x7fffffff, 0x00020000);
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), r, off * 4, 0, GPK_LST_AUX < 0 ? 0 : GPK_LST_AUX);
  }
}

// FULL: N == 16 * NB (no padding) -- every row and column of every tile is real.
template <bool FULL>
GPK_DEVICE void store4(float* p, int N, int row, int colg, const f32x4 v) {
  if constexpr (FULL) {
    lstore(p, row * N + colg, v);
    return;
  }
  if (row >= N) return;
  if (((N & 3) == 0) && colg + 3 < N) {
    *(f32x4*)&p[(size_t)row * N + colg] = v;
  } else {
#pragma unroll
    for (int r = 0; r < 4; ++r)
      if (colg + r < N) p[(size_t)row * N + colg + r] = v[r];
  }
}

// Zero L's strictly-upper part of block row KZ (rows 16 KZ .. +15, columns >= 16 (KZ + 1)):
// rows q = first, first + step, ... of the block by this wave, 16 B per lane.
template <bool FULL>
GPK_DEVICE void zero_l_block(float* Lb, int N, int KZ, int first, int step, int lane) {
  const int c0 = 16 * (KZ + 1);
  for (int q = first; q < 16; q += step) {
    const int row = 16 * KZ + q;
    if (row < N) {
      if ((N & 3) == 0) {
        for (int cc = c0 + 4 * lane; cc < N; cc += 256) lstore(Lb, row * N + cc, f32x4{0.f, 0.f, 0.f, 0.f});
      } else {
        for (int cc = c0 + lane; cc < N; cc += 64) Lb[(size_t)row * N + cc] = 0.f;
      }
    }
  }
}

template <int I>
GPK_DEVICE void pin_row(float (&sb)[16]);

// pin_row<I>: one asm statement consuming sb[I..15] as SGPR operands.
template <> GPK_DEVICE void pin_row<1>(float (&sb)[16]) { asm volatile("" : "+s"(sb[1]), "+s"(sb[2]), "+s"(sb[3]), "+s"(sb[4]), "+s"(sb[5]), "+s"(sb[6]), "+s"(sb[7]), "+s"(sb[8]), "+s"(sb[9]), "+s"(sb[10]), "+s"(sb[11]), "+s"(sb[12]), "+s"(sb[13]), "+s"(sb[14]), "+s"(sb[15])); }
template <> GPK_DEVICE void pin_row<2>(float (&sb)[16]) { asm volatile("" : "+s"(sb[2]), "+s"(sb[3]), "+s"(sb[4]), "+s"(sb[5]), "+s"(sb[6]), "+s"(sb[7]), "+s"(sb[8]), "+s"(sb[9]), "+s"(sb[10]), "+s"(sb[11]), "+s"(sb[12]), "+s"(sb[13]), "+s"(sb[14]), "+s"(sb[15])); }
template <> GPK_DEVICE void pin_row<3>(float (&sb)[16]) { asm volatile("" : "+s"(sb[3]), "+s"(sb[4]), "+s"(sb[5]), "+s"(sb[6]), "+s"(sb[7]), "+s"(sb[8]), "+s"(sb[9]), "+s"(sb[10]), "+s"(sb[11]), "+s"(sb[12]), "+s"(sb[13]), "+s"(sb[14]), "+s"(sb[15])); }
template <> GPK_DEVICE void pin_row<4>(float (&sb)[16]) { asm volatile("" : "+s"(sb[4]), "+s"(sb[5]), "+s"(sb[6]), "+s"(sb[7]), "+s"(sb[8]), "+s"(sb[9]), "+s"(sb[10]), "+s"(sb[11]), "+s"(sb[12]), "+s"(sb[13]), "+s"(sb[14]), "+s"(sb[15])); }
template <> GPK_DEVICE void pin_row<5>(float (&sb)[16]) { asm volatile("" : "+s"(sb[5]), "+s"(sb[6]), "+s"(sb[7]), "+s"(sb[8]), "+s"(sb[9]), "+s"(sb[10]), "+s"(sb[11]), "+s"(sb[12]), "+s"(sb[13]), "+s"(sb[14]), "+s"(sb[15])); }
template <> GPK_DEVICE void pin_row<6>(float (&sb)[16]) { asm volatile("" : "+s"(sb[6]), "+s"(sb[7]), "+s"(sb[8]), "+s"(sb[9]), "+s"(sb[10]), "+s"(sb[11]), "+s"(sb[12]), "+s"(sb[13]), "+s"(sb[14]), "+s"(sb[15])); }
template <> GPK_DEVICE void pin_row<7>(float (&sb)[16]) { asm volatile("" : "+s"(sb[7]), "+s"(sb[8]), "+s"(sb[9]), "+s"(sb[10]), "+s"(sb[11]), "+s"(sb[12]), "+s"(sb[13]), "+s"(sb[14]), "+s"(sb[15])); }
template <> GPK_DEVICE void pin_row<8>(float (&sb)[16]) { asm volatile("" : "+s"(sb[8]), "+s"(sb[9]), "+s"(sb[10]), "+s"(sb[11]), "+s"(sb[12]), "+s"(sb[13]), "+s"(sb[14]), "+s"(sb[15])); }
template <> GPK_DEVICE void pin_row<9>(float (&sb)[16]) { asm volatile("" : "+s"(sb[9]), "+s"(sb[10]), "+s"(sb[11]), "+s"(sb[12]), "+s"(sb[13]), "+s"(sb[14]), "+s"(sb[15])); }
template <> GPK_DEVICE void pin_row<10>(float (&sb)[16]) { asm volatile("" : "+s"(sb[10]), "+s"(sb[11]), "+s"(sb[12]), "+s"(sb[13]), "+s"(sb[14]), "+s"(sb[15])); }
template <> GPK_DEVICE void pin_row<11>(float (&sb)[16]) { asm volatile("" : "+s"(sb[11]), "+s"(sb[12]), "+s"(sb[13]), "+s"(sb[14]), "+s"(sb[15])); }
template <> GPK_DEVICE void pin_row<12>(float (&sb)[16]) { asm volatile("" : "+s"(sb[12]), "+s"(sb[13]), "+s"(sb[14]), "+s"(sb[15])); }
template <> GPK_DEVICE void pin_row<13>(float (&sb)[16]) { asm volatile("" : "+s"(sb[13]), "+s"(sb[14]), "+s"(sb[15])); }
template <> GPK_DEVICE void pin_row<14>(float (&sb)[16]) { asm volatile("" : "+s"(sb[14]), "+s"(sb[15])); }
template <> GPK_DEVICE void pin_row<15>(float (&sb)[16]) { asm volatile("" : "+s"(sb[15])); }

// Software-pipelined right-looking sweep of the fused R / R^{-T} factorisation
// (see diag_factor). Step m is split into
//   crit(m): pivot broadcast, scaling of row m, and the ONE update that the next
//            pivot depends on (v[m+1]);
//   rest(m): the other 14-m column updates of step m,
// emitted as crit(0) crit(1) rest(0) crit(2) rest(1) ... so the broadcast / FMA
// stream of rest(m-1) fills the rsq latency of crit(m). The readlanes of a group
// land in distinct SGPRs pinned by one asm statement, and the FMAs run as
// packed pairs (v_pk_fma_f32) on SGPR pairs.
template <int M>
GPK_DEVICE void diag_crit(float (&v)[16]) {
  const float piv = readlane_f(v[M], M);
  const float rs = __builtin_amdgcn_rsqf(piv);
  v[M] = v[M] * rs;
  if constexpr (M < 15) {
    float s1 = readlane_f(v[M], M + 1);
    asm volatile("" : "+s"(s1));
    v[M + 1] = __builtin_fmaf(-s1, v[M], v[M + 1]);
  }
}

typedef float f32x2 __attribute__((ext_vector_type(2)));

template <int M>
GPK_DEVICE void diag_rest(float (&v)[16]) {
  constexpr int I0 = M + 2;
  if constexpr (I0 < 16) {
    float sb[16];
#pragma unroll
    for (int i = I0; i < 16; ++i) sb[i] = readlane_f(v[M], i);
    pin_row<I0>(sb);
    const f32x2 vm = {v[M], v[M]};
    int i = I0;
    if constexpr ((16 - I0) & 1) {
      v[i] = __builtin_fmaf(-sb[i], v[M], v[i]);
      ++i;
    }
#pragma unroll
    for (; i < 16; i += 2) {
      f32x2 a = {v[i], v[i + 1]};
      const f32x2 sv = {-sb[i], -sb[i + 1]};
      a = __builtin_elementwise_fma(sv, vm, a);
      v[i] = a[0];
      v[i + 1] = a[1];
    }
  }
}

template <int M>
GPK_DEVICE void diag_sweep(float (&v)[16]) {
  __builtin_amdgcn_sched_barrier(0);
  diag_crit<M>(v);
  if constexpr (M > 0) diag_rest<M - 1>(v);
#pragma unroll
  for (int i = M; i < 16; ++i) asm volatile("" : "+v"(v[i]));
  if constexpr (M < 15) diag_sweep<M + 1>(v);
}

#include "gpk_diag_dpp.inc"

// Flag words (ints in LDS). The epoch flags are monotone within a launch (epoch =
// 32 * attempt + k); the per-attempt counters kFlagSync / kFlagTrsm / kFlagBulk restart
// from 0 between the two restart barriers of a failed attempt (kFlagRst is never reset):
enum : int {
  kFlagT00 = 1,     // tile (0,0) of this attempt is in dsc                (32 * attempt)
  kFlagFact = 2,    // R_kk^{-T} of step k is in wbuf[k % 3]                (epoch)
  kFlagFail = 3,    // [3 + attempt]: failure verdict of the attempt: provisional 16 k + 1 at
                    // the failing step k, then 16 k + the failing column; workers decode the
                    // step as (word - 1) >> 4
  // look-ahead hand-over (k, k+1) -> hbuf[k & 1], (k+1, k+1) -> hbuf[k & 1] + 256: ONE FLAG WORD
  // PER PARITY (kFlagHA + (k & 1), kFlagHB + (k & 1); epoch). In the column plan consecutive
  // hand-overs come from different waves, so with one shared word the owner of step k+1 could
  // raise it before the owner of step k had written its tile, and the diagonal wave would read
  // a stale hbuf[k & 1] (seen: 2 of 512 windows with a wrong (8,8) block).
  kFlagHA = 40,     // [40 + (k & 1)]
  kFlagHB = 42,     // [42 + (k & 1)]
  kFlagSync = 20,   // worker-only barrier counter
  kFlagTmo = 21,    // a spin wait ran out (safety net: the launch still drains)
  kFlagInvSigma = 30,
  kFlagGm2 = 31,
  // column-ownership worker path (GPK_EXACT_COL): words 64.. (STAMPS builds use 24..39)
  kFlagPan = 64,    // [64 + j]: panel tile R_{k,j} of the latest step k is out      (epoch)
  kFlagZ = 80,      // z_k of the latest step k is out                               (epoch)
  kFlagTrsm = 81,   // worker TRSM phases completed in this attempt (one add per wave per step)
  kFlagBulk = 82,   // worker steps whose panel reads are all done (one add per wave per step)
  kFlagRst = 83,    // restart barrier (two adds per wave per failed attempt, never reset)
};

// Poll an LDS flag until it reaches `target`. Every wait is bounded: after
// 2^18 polls (milliseconds) the wave gives up, records it in kFlagTmo and
// carries on, so a logic error can never leave waves spinning on the GPU
// (the window then reports info = kInfoTimeout).
constexpr int kInfoTimeout = 1 << 20;
GPK_DEVICE void spin_until(lds_vint* flags, int idx, int target) {
  int n = 0;
  while (flags[idx] < target) {
    if ((n & 255) == 255 && flags[kFlagTmo] != 0) break;  // (checked rarely: one LDS read per poll)
    // tight poll (no s_sleep): measured 3 % faster per launch than sleeping 64
    // clocks between polls -- the wake-up latency sits on every hand-off
    if (++n > (1 << 18)) {
      flags[kFlagTmo] = 1;
      if (GPK_TMO_DEBUG) flags[kFlagTmo + 1] = idx | (target << 8);   // which wait expired
      break;
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

// A worker wait inside a factorisation step. It does NOT watch the failure word: the restart
// is correct because every wait a worker makes in step K is satisfied by work that its
// producers do BEFORE they reach their own R_{K+1,K+1}^{-T} check: panel / z / counter flags of
// step K-1 or earlier, and -- phase 4b of the column plan -- tiles of panel K itself, which
// their owners write right after passing the step-K check. The diagonal wave reports a
// failure no earlier than at the step F it fails at, and a worker leaves the attempt only at
// the R_KK^{-T} check of a step K >= F ((fail - 1) >> 4 <= K). So for K < F every producer
// passes its step-K check and does the awaited work before its step-(K+1) check <= F; at
// K = F nobody gets past the check to wait for step-F work; all workers leave at the same
// check, and none waits for work that never comes. A new wait must keep this invariant: wait
// only for work of steps <= K that precedes the producer's next check (else it spins until
// the 2^18-poll bound).
#define GPK_WAITF(idx, target)                                                  \
  {                                                                             \
    unsigned long long _w0 = 0;                                                 \
    if constexpr (ST) _w0 = __builtin_amdgcn_s_memtime();                       \
    spin_until(x.vflag, (idx), (target));                                       \
    if constexpr (ST) x.st[9] += __builtin_amdgcn_s_memtime() - _w0;            \
  }


// Epoch shadows (GPK_EPOCH_CHECK builds only; gpk_exact_dev.h; every use is inside GPK_EP(...),
// which expands to nothing in product builds, so their device code is unchanged). Flag words past the product
// layout: panel tile j of step k at kShadowPan + (k & 1) (NB + 1) + j, the hand-over tiles of step
// k at kShadowHo + 2 (k & 1) + {0: (k, k+1), 1: (k+1, k+1)}, R_kk^{-T} at kShadowW + k % 3. The
// producer writes the epoch of the tile after the tile and before its flag release; the
// consumer compares it after the acquire.
constexpr int kFlagEpochBad = 84;   // site | slot << 8 of the first mismatch (check builds)
constexpr int kShadowPan = 96, kShadowHo = 130, kShadowW = 134;
GPK_DEVICE void epoch_mark(lds_vint* flags, int idx, int epoch, int lane) {
  if (lane == 0) flags[idx] = epoch;
}
GPK_DEVICE void epoch_expect(lds_vint* flags, int idx, int epoch, int site) {
  if (flags[idx] != epoch) {
    flags[kFlagEpochBad] = site | (idx << 8);
    flags[kFlagTmo] = 1;   // the window ends with info = kInfoTimeout; the launch still drains
  }
}

GPK_DEVICE void publish_tile(float* dst, int lane, const f32x4 v, lds_vint* flags, int idx, int value) {
  *(f32x4*)&dst[lane * 4] = v;
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
  if (lane == 0) flags[idx] = value;
}

// R_kj = R_kk^{-T} T_kj for one tile: q = -W^T (from wbuf, acc layout), t = -T_kj.
// Two independent 2-MFMA chains (80 cycles of dependent latency instead of 160).
// Used by the worker TRSM and by the diagonal wave's look-ahead alike, so both
// produce bit-identical panels.
GPK_DEVICE f32x4 trsm_tile_f32(const f32x4 q, const f32x4 t) {
  const f32x4 z = {0.f, 0.f, 0.f, 0.f};
  f32x4 d0 = __builtin_amdgcn_mfma_f32_16x16x4f32(q[0], t[0], z, 0, 0, 0);
  f32x4 d1 = __builtin_amdgcn_mfma_f32_16x16x4f32(q[2], t[2], z, 0, 0, 0);
  d0 = __builtin_amdgcn_mfma_f32_16x16x4f32(q[1], t[1], d0, 0, 0, 0);
  d1 = __builtin_amdgcn_mfma_f32_16x16x4f32(q[3], t[3], d1, 0, 0, 0);
  return d0 + d1;
}

typedef f32x4 WOp;
GPK_DEVICE WOp w_split(const f32x4 q) { return q; }
GPK_DEVICE f32x4 trsm_tile(const WOp& w, const f32x4 t) { return trsm_tile_f32(w, t); }

GPK_DEVICE f32x4 load_w(const float* wb, int c, int grp) {
  f32x4 q;
#pragma unroll
  for (int r = 0; r < 4; ++r) q[r] = wb[(4 * grp + r) * kWS + c];
  return q;
}
// The same through volatile LDS reads (ordered after a flag read, see worker_step).
GPK_DEVICE f32x4 load_w_v(const float* wb, int c, int grp) {
  typedef __attribute__((address_space(3))) volatile float lds_vfloat;
  const lds_vfloat* w = (const lds_vfloat*)wb;
  f32x4 q;
#pragma unroll
  for (int r = 0; r < 4; ++r) q[r] = w[(4 * grp + r) * kWS + c];
  return q;
}

// d += R^T R for a rounded factor tile held as registers (hi, lo).
GPK_DEVICE f32x4 mma_tn_split_regs(const half4_t h, const half4_t l, f32x4 d) {
  const half8_t hl = {h[0], h[1], h[2], h[3], l[0], l[1], l[2], l[3]};
  const half8_t lh = {l[0], l[1], l[2], l[3], h[0], h[1], h[2], h[3]};
  d = __builtin_amdgcn_mfma_f32_16x16x32_f16(hl, hl, d, 0, 0, 0);
  d = __builtin_amdgcn_mfma_f32_16x16x32_f16(hl, lh, d, 0, 0, 0);
  return d;
}

// Panel operand of the trailing updates. GPK_SPLIT_UPDATE=1 (default): factor tiles
// are rounded to hi + lo f16 planes (22 significant bits) and the updates run on
// mfma_f32_16x16x32_f16 (2 MFMAs per K=16 tile product, every product exact);
// GPK_SPLIT_UPDATE=0: fp32 tiles (24 bits) and mfma_f32_16x16x4f32 (4 MFMAs per
// tile product). Same LDS footprint (16 B per lane per tile). DESIGN.md §4.1 states
// the measured speed / precision trade of the two.
#if GPK_SPLIT_UPDATE
typedef half8_t pan_op_t;
GPK_DEVICE pan_op_t pan_load(const float* tile, int lane) { return load_split_hl(tile, lane); }
GPK_DEVICE f32x4 pan_mma(const pan_op_t q, const float* ptile, int lane, f32x4 d) {
  return mma_tn_split(q, ptile, lane, d);
}
GPK_DEVICE f32x4 pan_mma_op(const pan_op_t q, const pan_op_t p_hl, f32x4 d) {   // d += Q^T P, both loaded
  const half8_t p_lh = {p_hl[4], p_hl[5], p_hl[6], p_hl[7], p_hl[0], p_hl[1], p_hl[2], p_hl[3]};
  d = __builtin_amdgcn_mfma_f32_16x16x32_f16(q, p_hl, d, 0, 0, 0);
  d = __builtin_amdgcn_mfma_f32_16x16x32_f16(q, p_lh, d, 0, 0, 0);
  return d;
}
GPK_DEVICE f32x4 pan_store(float* tile, int lane, const f32x4 v) {
  half4_t h, l;
  const f32x4 o = round_split_f16(v, h, l);
  store_split_planes(tile, lane, h, l);
  return o;
}
GPK_DEVICE f32x4 pan_self(const f32x4 v, f32x4 d) {   // d += V^T V of the rounded tile
  half4_t h, l;
  (void)round_split_f16(v, h, l);
  return mma_tn_split_regs(h, l, d);
}
#else
typedef f32x4 pan_op_t;
GPK_DEVICE pan_op_t pan_load(const float* tile, int lane) { return *(const f32x4*)&tile[4 * lane]; }
GPK_DEVICE f32x4 pan_mma(const pan_op_t q, const float* ptile, int lane, f32x4 d) {
  return mma_tn(q, *(const f32x4*)&ptile[4 * lane], d);
}
GPK_DEVICE f32x4 pan_store(float* tile, int lane, const f32x4 v) {
  *(f32x4*)&tile[4 * lane] = v;
  return v;
}
GPK_DEVICE f32x4 pan_self(const f32x4 v, f32x4 d) { return mma_tn(v, v, d); }
GPK_DEVICE f32x4 pan_mma_op(const pan_op_t q, const pan_op_t p, f32x4 d) { return mma_tn(q, p, d); }
#endif

// Lane moves of the sweep operand (one wave, no LDS round trip): x of the odd rows in the
// even rows' lanes (row 1 -> 0, 3 -> 2; permlane16_swap, new src0) and of rows 2, 3 in rows
// 0, 1 (permlane32_swap, new src0).
GPK_DEVICE float from_odd_row_f(float x) {
  const unsigned u = __builtin_bit_cast(unsigned, x);
  return __builtin_bit_cast(float, (unsigned)__builtin_amdgcn_permlane16_swap(u, u, false, false)[1]);
}
GPK_DEVICE float from_upper_half_f(float x) {
  const unsigned u = __builtin_bit_cast(unsigned, x);
  return __builtin_bit_cast(float, (unsigned)__builtin_amdgcn_permlane32_swap(u, u, false, false)[1]);
}

// Factor one 16x16 diagonal tile T in ONE wave (the diagonal wave).
//   lanes  0-15 (column c): v[m] <- R[m][c]             (R^T R = T, upper)
//   lanes 16-31 (column c): v[m] <- W[m][c], W = R^{-T}  (lower), started from I
// from one instruction stream: at step m every lane does
//   v[m] *= rsqrt(pivot);   v[i] -= R[m][i] * v[m]   (i > m)
// with R[m][i] broadcast from R-lane i by DPP. `t` holds -T in acc layout IN REGISTERS
// (lane 16 g + c: rows 4 g + r of column c); lane c gathers its column by permlane swaps.
// -W (transposed: wbuf[c*kWS+m] = -W[m][c]) is published FIRST together with the pass/fail
// verdict (every pivot checked positive-finite), then the factor-done flag is raised. The L
// diagonal block and log|T| come later, from `v` and `dg`, in diag_finish: the caller issues
// them under the next look-ahead's MFMAs instead of ahead of them.
template <bool ST, bool FULL>
GPK_DEVICE int diag_factor(const f32x4 t, float (&v)[16], float& dg, float* wbuf, lds_vint* flags,
                           lds_vint* fail_flag, int epoch, const float* tile, unsigned long long* dst = nullptr) {
  unsigned long long t0 = 0;
  if constexpr (ST) t0 = __builtin_amdgcn_s_memtime();
  int lane = threadIdx.x & 63;
  asm volatile("" : "+v"(lane));  // keep per-lane masks local to this call
  const int c = lane & 15, grp = lane >> 4;
  if (GPK_DIAG_PERMLANE) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float a2 = from_upper_half_f(t[r]);     // rows 2, 3 -> rows 0, 1
      v[r] = t[r];
      v[4 + r] = from_odd_row_f(t[r]);
      v[8 + r] = a2;
      v[12 + r] = from_odd_row_f(a2);
    }
  } else {   // (A/B: the same gather through the tile in LDS)
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const f32x4 u = *(const f32x4*)&tile[(16 * g + c) * 4];
#pragma unroll
      for (int r = 0; r < 4; ++r) v[4 * g + r] = u[r];
    }
  }
#pragma unroll
  for (int i = 0; i < 16; ++i) v[i] = (grp == 0) ? -v[i] : ((grp == 1 && i == c) ? 1.f : 0.f);
  if constexpr (ST) {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    if (lane == 0) dst[0] += t1 - t0;
    t0 = t1;
    __builtin_amdgcn_sched_barrier(0);
  }
#if GPK_DIAG_DPP
  if (!kKoDiagSweep) diag_sweep_dpp(v);
#else
  diag_sweep<0>(v);
#endif
  if constexpr (ST) {
    __builtin_amdgcn_sched_barrier(0);
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    if (lane == 0) dst[1] += t1 - t0;
    t0 = t1;
    __builtin_amdgcn_sched_barrier(0);
  }
  if (grp == 1) {
#pragma unroll
    for (int g = 0; g < 4; ++g)
      *(f32x4*)&wbuf[c * kWS + 4 * g] = f32x4{-v[4 * g], -v[4 * g + 1], -v[4 * g + 2], -v[4 * g + 3]};
  }
  // diagonal of R (lane c < 16 holds R[c][c] in v[c])
  dg = v[0];
#pragma unroll
  for (int i = 1; i < 16; ++i) dg = (c == i) ? v[i] : dg;
  const bool okd = (dg > 0.f) && (dg < __builtin_huge_valf());
  const unsigned long long badm = kKoAny ? 0ull : __ballot(lane < 16 && !okd);
  // provisional (the exact column follows): 16 k + 1 -- the failing STEP is readable from
  // either value as (word - 1) >> 4, so a worker that is still at an earlier step does not
  // leave the attempt before the others (they all leave at step k)
  if (badm != 0 && lane == 0) *fail_flag = 16 * (epoch & 31) + 1;
  GPK_EP(epoch_mark(flags, kShadowW + (epoch & 31) % 3, epoch, lane);)
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
  if (lane == 0) flags[kFlagFact] = epoch;
  if constexpr (ST) {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    if (lane == 0) dst[2] += t1 - t0;
    __builtin_amdgcn_sched_barrier(0);
  }
  return badm ? __builtin_ctzll(badm) + 1 : 0;
}

// The rest of a factored diagonal step, off the chain: per-lane partial log2|T| (lanes 0-15;
// reduced across lanes once, at the end -- a per-step shuffle reduction is 4 LDS round trips)
// and L's diagonal block from the R lanes.
template <bool FULL>
GPK_DEVICE void diag_finish(float (&v)[16], float dg, float* Lb, int N, int row0, float inv_sigma,
                            float& logdet) {
  int lane = threadIdx.x & 63;
  asm volatile("" : "+v"(lane));
  const int c = lane & 15, grp = lane >> 4;
  logdet += (lane < 16) ? __builtin_amdgcn_logf(dg * dg) : 0.f;
  if (grp == 0) {
    // R lanes: zero below-diagonal garbage, write L[row0 + c][row0 + m] = R[m][c]
#pragma unroll
    for (int i = 0; i < 16; ++i)
      if (i > c) v[i] = 0.f;
    if (Lb != nullptr) {
#pragma unroll
      for (int g = 0; g < 4; ++g)
        store4<FULL>(Lb, N, row0 + c, row0 + 4 * g,
               f32x4{v[4 * g], v[4 * g + 1], v[4 * g + 2], v[4 * g + 3]} * inv_sigma);
    }
  }
}

// ---------------------------------------------------------------------------
// RBF tile straight into accumulator form: returns -K_hat(tile i, j) in acc
// layout (three split-f16 MFMA passes for the Gram).
// ---------------------------------------------------------------------------
// Its scalars live in one 16-byte LDS word group (rbfc), read ONCE per batch
// of tiles (one ds_read_b128) so they do not pin SGPRs across the unrolled
// factorisation steps: {gm2 = -2 / 2^(2a) (undoes the f16 image scale on the
// Gram), s2 * sigma^2, (s2 + noise + jitter) * sigma^2, LDS float offset of the
// squared norms | (D chunks of 32) << 20}.
struct RbfK {
  float gm2, s2, diagval;
  int nrm_dc;
};
GPK_DEVICE RbfK read_rbfk(const float* rbfc) {
  // plain (non-volatile) 16-byte LDS load through a laundered address: one
  // ds_read_b128, never hoisted or merged across steps
  typedef int i32x4 __attribute__((ext_vector_type(4)));
  unsigned addr = (unsigned)(uintptr_t)(const __attribute__((address_space(3))) float*)rbfc;
  asm volatile("" : "+v"(addr));
  const i32x4 v = *(const __attribute__((address_space(3))) i32x4*)(uintptr_t)addr;
  RbfK k;
  k.gm2 = __builtin_bit_cast(float, __builtin_amdgcn_readfirstlane(v[0]));
  k.s2 = __builtin_bit_cast(float, __builtin_amdgcn_readfirstlane(v[1]));
  k.diagval = __builtin_bit_cast(float, __builtin_amdgcn_readfirstlane(v[2]));
  k.nrm_dc = __builtin_amdgcn_readfirstlane(v[3]);
  return k;
}

template <int NB, bool FULL>
GPK_DEVICE f32x4 rbf_tile(const float* smem, const RbfK& k, int i, int j, int lane, int N) {
  constexpr float nhalf_log2e = -0.72134752044448170f;  // -0.5 * log2(e)
  const int c = lane & 15, grp = lane >> 4;
  const int DC32 = k.nrm_dc >> 20;
  const float* nrm = smem + (k.nrm_dc & 0xfffff);
  const half8_t* x8 = (const half8_t*)smem;  // f16 hi / lo images (hfrag layout) at offset 0
  // every LDS operand of the tile is requested before the first MFMA (one
  // round trip instead of a load -> wait -> MFMA chain)
  const f32x4 nr = *(const f32x4*)&nrm[16 * i + 4 * grp];
  const int col = 16 * j + c;
  const float nc = nrm[col];
  // first 32-column chunk peeled (D <= 32 is the whole Gram): its four operand loads
  // go out together with the norms, one LDS round trip per tile
  const half8_t al = x8[NB * 64 + i * 64 + lane], ah = x8[i * 64 + lane];
  const half8_t bh = x8[j * 64 + lane], bl = x8[NB * 64 + j * 64 + lane];
  f32x4 g = {0.f, 0.f, 0.f, 0.f};
  g = __builtin_amdgcn_mfma_f32_16x16x32_f16(al, bh, g, 0, 0, 0);
  g = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, bh, g, 0, 0, 0);
  g = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, bl, g, 0, 0, 0);
  for (int dd = 1; dd < DC32; ++dd) {
    const half8_t* xhv = x8 + (2 * dd) * NB * 64;
    const half8_t* xlv = x8 + (2 * dd + 1) * NB * 64;
    const half8_t al2 = xlv[i * 64 + lane], bh2 = xhv[j * 64 + lane];
    const half8_t ah2 = xhv[i * 64 + lane], bl2 = xlv[j * 64 + lane];
    g = __builtin_amdgcn_mfma_f32_16x16x32_f16(al2, bh2, g, 0, 0, 0);
    g = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah2, bh2, g, 0, 0, 0);
    g = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah2, bl2, g, 0, 0, 0);
  }
  const float gm2 = k.gm2, ns2 = -k.s2, diagval = k.diagval;
  f32x4 o;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    float dist = __builtin_fmaf(gm2, g[q], nr[q] + nc);
    dist = dist < 0.f ? 0.f : dist;  // clamp_min(0), NaN-propagating like torch
    o[q] = ns2 * __builtin_amdgcn_exp2f(nhalf_log2e * dist);   // -K (accumulator sign)
  }
  if (i == j) {   // wave-uniform: only diagonal tiles pay for the diagonal / padding selects
#pragma unroll
    for (int q = 0; q < 4; ++q)
      if (16 * i + 4 * grp + q == col) o[q] = -diagval;
  }
  if constexpr (!FULL) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int row = 16 * i + 4 * grp + q;
      if (row >= N || col >= N) o[q] = (row == col) ? -1.f : 0.f;
    }
  }
  return o;
}

// ---------------------------------------------------------------------------
// Worker-wave factorisation steps, unrolled at compile time. Step K's active
// tile set is a slot PREFIX whose full part NALL(K) = P(K-1) / WK is a
// compile-time constant, so the bulk trailing update is straight-line MFMA
// code with in-place accumulators (no per-slot branches, no phi copies).
// ---------------------------------------------------------------------------
template <int I>
struct IC { static constexpr int value = I; };

template <int N, typename F>
GPK_DEVICE void static_for_desc(F&& f) {
  if constexpr (N > 0) {
    f(IC<N - 1>{});
    static_for_desc<N - 1>(f);
  }
}

template <int A, int B, typename F>
GPK_DEVICE void static_for_range(F&& f) {  // A..B inclusive, ascending
  if constexpr (A <= B) {
    f(IC<A>{});
    static_for_range<A + 1, B>(f);
  }
}

struct WorkerCtx {
  float* panel;
  float* wbuf;
  float* hbuf;
  lds_vint* vflag;
  float* Lb;
  float* zout;
  float* rw;
  const float* smem;
  int rbfc;    // LDS float offset of the RBF constants (RbfK)
  int N, b, lane, c, grp, wv;
  int epoch0;  // flag value of step 0 in this attempt (32 * attempt)
  int nsync;   // worker-only barriers passed by this wave
  float sumz2;
  unsigned long long* st;  // STAMPS builds only: [0..7] phase clocks, [8] last stamp
  unsigned long long* tl;  // STAMPS builds only: per-step timeline [(k * 8 + wave) * 8 + event]
};

// Check builds (GPK_EPOCH_CHECK): the panel tile at `tile` (either parity buffer) carries the
// epoch of the step that wrote it -- step K in the buffer of parity K & 1, else step K - 1.
template <int NB, int K>
GPK_DEVICE void epoch_pan(const WorkerCtx& x, const float* tile, int e0, int site) {
  GPK_EP(const int s = (int)(tile - x.panel) >> 8; epoch_expect(x.vflag, kShadowPan + s, e0 + (s / (NB + 1) == (K & 1) ? K : K - 1), site);)
}
GPK_DEVICE void epoch_pan_mark(const WorkerCtx& x, const float* tile, int epoch) {
  GPK_EP(epoch_mark(x.vflag, kShadowPan + ((int)(tile - x.panel) >> 8), epoch, x.lane);)
}

// Barrier among the WK worker waves only (the diagonal wave runs ahead of them
// and never joins): monotone LDS counter, one ds_add per wave.
// Split into arrive (publish this wave's LDS writes, count in) and wait, so
// independent work can run in between.
GPK_DEVICE void worker_arrive(WorkerCtx& x) {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
  x.nsync += 1;
  if (x.lane == 0)
    (void)__atomic_fetch_add((__attribute__((address_space(3))) int*)&x.vflag[kFlagSync], 1,
                             __ATOMIC_RELAXED);
}
template <int WK>
GPK_DEVICE bool worker_wait(WorkerCtx& x) {   // (always false: every worker leaves a failed
  spin_until(x.vflag, kFlagSync, WK * x.nsync);  // attempt at the same step, see diag_factor)
  return false;
}
// Restart barrier after a failed attempt (jitter ladder), on its own monotone counter: r-th
// barrier of the launch. Between its two uses the per-attempt counters are reset.
template <int WK>
GPK_DEVICE void restart_sync(WorkerCtx& x, int r) {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
  if (x.lane == 0)
    (void)__atomic_fetch_add((__attribute__((address_space(3))) int*)&x.vflag[kFlagRst], 1, __ATOMIC_RELAXED);
  spin_until(x.vflag, kFlagRst, WK * r);
}

// One right-looking step K for the worker waves. The diagonal wave owns the
// diagonal tiles from the moment they are handed over: at step K it factors
// (K,K), computes R_{K,K+1} itself and applies that last update to (K+1,K+1)
// (look-ahead), so the workers
//   1. apply panel K-1 to their tiles with i >= K except (K,K), updating and
//      handing over (K,K+1) and (K+1,K+1) FIRST (hbuf[K & 1], flags HA / HB);
//   2. zero L's upper part of block row K, update the right-hand side;
//   3. wait for R_KK^{-T}, TRSM block row K (+ z_K) into panel K;
//   4. ARRIVE at the worker-only step barrier (panel K is complete once every
//      worker has arrived), then build the RBF tiles of block row K+2
//      (deferred Gram: additive, so it can land after earlier trailing
//      updates; nothing depends on it before step K+1) while the slower
//      waves finish their TRSM;
//   5. WAIT at the barrier (split-phase: the RBF absorbs the step's load
//      imbalance; measured 5-7 % per launch over a plain barrier after 4.).
// Returns nonzero when the diagonal wave reported a failed factorisation.
template <int NB, int WK, int SLOTS, int K, bool ST, bool FULL>
GPK_DEVICE int worker_step_split(f32x4 (&acc)[SLOTS], WorkerCtx& x) {
  constexpr int Pk = plan_P<NB>(K);
  constexpr bool LAST = (K == NB - 1);
  constexpr int TD = Pk;                                  // (K, K): the diagonal wave's
  constexpr int TA = Pk + 1;                              // (K, K+1)
  constexpr int TB = LAST ? -1 : plan_P<NB>(K + 1);       // (K+1, K+1)
  // launder per step: keeps the per-slot plan loads / LDS addresses of this
  // step from being hoisted (and pinned in registers) across all NB steps
  const int wv = launder_s(x.wv);
  const int e0 = launder_s(x.epoch0);
  int lane = x.lane;
  asm volatile("" : "+v"(lane));
  const int c = lane & 15, grp = lane >> 4;
  const float* pprev = x.panel + ((K + 1) & 1) * (NB + 1) * 256;  // panel K-1
  float* pcur = x.panel + (K & 1) * (NB + 1) * 256;                // panel K
  float* hA = x.hbuf + (K & 1) * 512;
  if constexpr (ST) {
    if (x.lane == 0) x.tl[(K * 8 + x.wv) * 8] = __builtin_amdgcn_s_memtime();
  }
  // (the hand-over tiles have compile-time (i, j): no plan lookup, so nothing
  // wave-specialised gets hoisted out of the attempt loop)
  auto upd_ij = [&](f32x4& d, auto I, auto J) {
    constexpr int i = decltype(I)::value, j = decltype(J)::value;
    GPK_EP(epoch_pan<NB, K>(x, pprev + i * 256, e0, 1);)
    GPK_EP(epoch_pan<NB, K>(x, pprev + j * 256, e0, 1);)
    d = pan_mma(pan_load(pprev + i * 256, lane), pprev + j * 256, lane, d);
  };
  if constexpr (K > 0) {
    if constexpr (!LAST) {
      if constexpr (GPK_EXACT_PRIO) __builtin_amdgcn_s_setprio(GPK_EXACT_PRIO);   // hand-over: the diagonal wave waits
      if (wv == TA % WK) {
        upd_ij(acc[TA / WK], IC<K>{}, IC<K + 1>{});
        GPK_EP(epoch_mark(x.vflag, kShadowHo + 2 * (K & 1), e0 + K, lane);)
        publish_tile(hA, lane, acc[TA / WK], x.vflag, kFlagHA + (K & 1), e0 + K);
      }
      if (wv == TB % WK) {
        upd_ij(acc[TB / WK], IC<K + 1>{}, IC<K + 1>{});
        GPK_EP(epoch_mark(x.vflag, kShadowHo + 2 * (K & 1) + 1, e0 + K, lane);)
        publish_tile(hA + 256, lane, acc[TB / WK], x.vflag, kFlagHB + (K & 1), e0 + K);
      }
      if constexpr (GPK_EXACT_PRIO) __builtin_amdgcn_s_setprio(0);
    }
    // trailing update from panel K-1 over the other tiles with i >= K
    // (t < P(K-1)), highest slot first. Re-laundered: the hand-over branches
    // above pin wv to a constant, and code tail-duplicated into them would
    // turn plan lookups into constants hoisted out of the attempt loop.
    const int wv = launder_s(x.wv);
    auto upd = [&](f32x4& d, auto I) {
      constexpr int s = decltype(I)::value;
      const int p = plan_tile<NB, WK * s, WK * s + WK - 1>(wv + WK * s);
      GPK_EP(epoch_pan<NB, K>(x, pprev + (p & 255) * 256, e0, 2);)
      GPK_EP(epoch_pan<NB, K>(x, pprev + (p >> 8) * 256, e0, 2);)
      if constexpr (kKoOneOperand) {   // knockout: one LDS operand per tile update
        const pan_op_t q = pan_load(pprev + (p & 255) * 256, lane);
        d = pan_mma_op(q, q, d);
      } else {
        d = pan_mma(pan_load(pprev + (p & 255) * 256, lane), pprev + (p >> 8) * 256, lane, d);
      }
    };
    constexpr int Pkm1 = plan_P<NB>(K - 1);
    constexpr int NALL = Pkm1 / WK;
    auto bulk = [&](auto I) {
      constexpr int s = decltype(I)::value;
      bool sk = false;
      if constexpr (s == TD / WK) sk = sk || (wv == TD % WK);
      if constexpr (!LAST && s == TA / WK) sk = sk || (wv == TA % WK);
      if constexpr (!LAST && s == TB / WK) sk = sk || (wv == TB % WK);
      if (!sk && !kKoBulkUpdate) upd(acc[s], I);
    };
    if constexpr (NALL < SLOTS && (Pkm1 % WK) != 0) {
      if (wv < Pkm1 % WK) bulk(IC<NALL>{});
    }
    static_for_desc<NALL>(bulk);
  }
  GPK_WSTAMP(2, 1)  // trailing update (+ hand-over)
#if GPK_EXACT_PRIO_RHS
  __builtin_amdgcn_s_setprio(GPK_EXACT_PRIO);   // zero-L + right-hand side lead into the TRSM
#endif
  // zero L's strictly-upper part of block row K (streams out behind the MFMAs)
  if (!kKoZeroL && x.Lb != nullptr) zero_l_block<FULL>(x.Lb, FULL ? 16 * NB : x.N, K, wv, WK, lane);
  // right-hand side, block rows i >= K owned by this wave: rw_i += R_{K-1,i}^T z_{K-1}
  // (rw holds -(y - c); only column 0 of the tile is live, so it round-trips
  // through LDS on the c == 0 lanes)
  const int rfirst = K + (((wv - K) % WK) + WK) % WK;
  if constexpr (K > 0 && !kKoRhs) {
    for (int i = rfirst; i < NB; i += WK) {
      f32x4 d = *(const f32x4*)&x.rw[16 * i + 4 * grp];
      if (c != 0) d = f32x4{0.f, 0.f, 0.f, 0.f};
      GPK_EP(epoch_pan<NB, K>(x, pprev + i * 256, e0, 3);)
      GPK_EP(epoch_pan<NB, K>(x, pprev + NB * 256, e0, 3);)
      d = pan_mma(pan_load(pprev + i * 256, lane), pprev + NB * 256, lane, d);
      if (c == 0) *(f32x4*)&x.rw[16 * i + 4 * grp] = d;
    }
  }
  GPK_WSTAMP(6, 2)  // right-hand side
  // TRSM of the row-K off-diagonal tiles (P(K) < t <= P(K) + NB - K - 1) and,
  // by the owner of RHS block row K, of the right-hand side: z_K
  // One LDS round trip in the usual case (the diagonal wave is ahead): the epoch flag, the
  // failure word, R_KK^{-T} and 1/sigma are requested together. A wave's LDS reads are
  // served in order, and the diagonal wave completes its R_KK^{-T} and failure-word writes
  // before it releases the flag, so reads issued after a flag read that sees epoch K see
  // them too (all volatile: the compiler keeps the order). Otherwise: wait, re-read.
  const float* wbk = x.wbuf + (K % 3) * kWBuf;
  const int flag_now = x.vflag[kFlagFact];
  int fail = x.vflag[kFlagFail + e0 / 32];
  f32x4 q = load_w_v(wbk, c, grp);
  // the factor runs on sigma^2 K_hat (power of two): L = R'^T / sigma
  const float inv_sigma = __builtin_bit_cast(float, (int)x.vflag[kFlagInvSigma]);
  if (flag_now < e0 + K) {
    spin_until(x.vflag, kFlagFact, e0 + K);
    fail = x.vflag[kFlagFail + e0 / 32];
    q = load_w_v(wbk, c, grp);
  }
  GPK_WSTAMP(7, 4)  // wait for R_KK^{-T}
  GPK_EP(epoch_expect(x.vflag, kShadowW + K % 3, e0 + K, 4);)
  if (!kKoAny && fail != 0 && ((fail - 1) >> 4) <= K) {   // the attempt failed at step <= K
    __builtin_amdgcn_s_setprio(0);   // the jitter-ladder retry starts at the base priority
    return 1;
  }
  if constexpr (GPK_EXACT_PRIO) __builtin_amdgcn_s_setprio(GPK_EXACT_PRIO);   // TRSM: panel K gates step K+1
  const WOp wq = w_split(q);
  constexpr int TLO = Pk + 1, THI = Pk + NB - K - 1;
  constexpr int SLO = TLO >= WK ? (TLO - (WK - 1)) / WK : 0;
  constexpr int SHI = (THI / WK) < SLOTS - 1 ? (THI / WK) : SLOTS - 1;
  {
    if constexpr (THI >= TLO) {
      static_for_range<SLO, SHI>([&](auto I) {
        constexpr int s = decltype(I)::value;
        const int t = wv + WK * s;
        if (t >= TLO && t <= THI) {
          const int j = plan_tile<NB, WK * s, WK * s + WK - 1>(t) >> 8;
          const f32x4 rkj = pan_store(pcur + j * 256, lane, kKoTrsmMfma ? acc[s] : trsm_tile(wq, acc[s]));
          GPK_EP(epoch_pan_mark(x, pcur + j * 256, e0 + K);)
          // L[16j + c][16K + 4g + r] = R_Kj[4g + r][c] / sigma
          if (!kKoTrsmLStores && x.Lb != nullptr)
            store4<FULL>(x.Lb, x.N, 16 * j + c, 16 * K + 4 * grp, rkj * inv_sigma);
        }
      });
    }
    if (rfirst == K) {
      f32x4 d = *(const f32x4*)&x.rw[16 * K + 4 * grp];
      if (c != 0) d = f32x4{0.f, 0.f, 0.f, 0.f};
      const f32x4 zk = pan_store(pcur + NB * 256, lane, trsm_tile_f32(q, d));   // (y unbounded: fp32)
      GPK_EP(epoch_pan_mark(x, pcur + NB * 256, e0 + K);)
      if (c == 0) {
#pragma unroll
        for (int r = 0; r < 4; ++r) x.sumz2 = __builtin_fmaf(zk[r], zk[r], x.sumz2);
        if (x.zout != nullptr) {
          const int row = 16 * K + 4 * grp;
#pragma unroll
          for (int r = 0; r < 4; ++r)
            if (FULL || row + r < x.N) x.zout[(size_t)x.b * x.N + row + r] = zk[r];
        }
      }
    }
  }
  GPK_WSTAMP(4, 5)  // TRSM
  // panel K and z_K are out: count in at the step barrier, then do the work that
  // does not depend on the other waves (zero-L, deferred RBF) before waiting on it
  worker_arrive(x);
  if constexpr (GPK_EXACT_PRIO) __builtin_amdgcn_s_setprio(0);
  // deferred RBF of block row K+2 (its diagonal tile is handed over at step K+1)
  if constexpr (K + 2 < NB && !kKoDeferredRbf) {
    constexpr int RLO = plan_P<NB>(K + 2), RHI = plan_P<NB>(K + 1) - 1;
    constexpr int SLO = RLO / WK;
    constexpr int SHI = (RHI / WK) < SLOTS - 1 ? (RHI / WK) : SLOTS - 1;
    const RbfK rk = read_rbfk(x.smem + x.rbfc);
    static_for_range<SLO, SHI>([&](auto I) {
      constexpr int s = decltype(I)::value;
      const int t = wv + WK * s;
      if (t >= RLO && t <= RHI) {
        const int p = plan_tile<NB, WK * s, WK * s + WK - 1>(t);
        acc[s] += rbf_tile<NB, FULL>(x.smem, rk, p & 255, p >> 8, lane, x.N);
      }
    });
  }
  GPK_WSTAMP(3, 3)  // deferred RBF (after the arrive)
  if (worker_wait<WK>(x)) return 1;
  GPK_WSTAMP(5, 6)  // worker barrier
  return 0;
}

// ---------------------------------------------------------------------------
// Column-ownership worker plan (GPK_EXACT_COL: NB = 16 with 7 worker waves, the headline
// N = 256 shape). Worker w owns the block columns A = 15 - w and B = w + 1 of the upper
// triangle (16 - w + w + 2 = 18 tiles for every wave) plus rows {w, w + 7} <= 8 of the
// middle column 8. Slots: (i, A) -> i, (i, B) -> 17 - i, (w, 8) -> 18, (w + 7, 8) -> 19, so
// the tiles of one block row sit in COMPILE-TIME slots (guarded by wave-uniform compares)
// and a column's panel tile R_{k-1,j} -- the P operand of every update of column j -- is
// read from LDS once per step instead of once per tile. Per step the workers synchronise
// through per-column panel flags (kFlagPan + j), the z flag and two monotone counters
// (TRSM phases done / panel reads done) instead of a workgroup-wide step barrier:
//   2. the other tiles of block row K through panel K-1 (this step's TRSM inputs);
//   3. right-hand side row K (owner of column K);
//   4. TRSM of row K with R_KK^{-T} (+ z_K): panel K, flags; the panel buffer is reused
//      only once every wave has finished reading panel K-2 (kFlagBulk);
//   4b. the NEXT step's hand-over HO_{K+1} = (K+1, K+2), (K+2, K+2), by their owners: panel
//      K-1, (K+2, K+2)'s deferred RBF, then panel K as soon as R_{K,K+1}, R_{K,K+2} are out
//      (round 5; before, HO_K opened step K, i.e. it waited for the owners' whole step K-1);
//   5. the rest of the trailing update through panel K-1 once panel K-1 is complete
//      (kFlagTrsm), one P load per column;
//   6. right-hand side rows > K of the owned columns; count the panel reads done;
//   7. deferred RBF of block row K+2 (less (K+2, K+2): 4b), zero-L.
// ---------------------------------------------------------------------------
constexpr int kColSlots = 20;

template <int K>
struct ColOwners {
  // owner (wave) of block column j's HO / RHS duties
  static constexpr int col_owner(int j) { return j >= 9 ? 15 - j : (j >= 1 && j <= 7 ? j - 1 : (j == 8 ? 1 : 0)); }
};

GPK_DEVICE f32x4 pan_mma2(const pan_op_t q, const pan_op_t p_hl, const pan_op_t p_lh, f32x4 d) {
#if GPK_SPLIT_UPDATE
  d = __builtin_amdgcn_mfma_f32_16x16x32_f16(q, p_hl, d, 0, 0, 0);
  d = __builtin_amdgcn_mfma_f32_16x16x32_f16(q, p_lh, d, 0, 0, 0);
  return d;
#else
  (void)p_lh;
  return mma_tn(q, p_hl, d);
#endif
}
GPK_DEVICE pan_op_t pan_swap(const pan_op_t p) {
#if GPK_SPLIT_UPDATE
  return pan_op_t{p[4], p[5], p[6], p[7], p[0], p[1], p[2], p[3]};
#else
  return p;
#endif
}

GPK_DEVICE void count_in(WorkerCtx& x, int idx) {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
  if (x.lane == 0)
    (void)__atomic_fetch_add((__attribute__((address_space(3))) int*)&x.vflag[idx], 1, __ATOMIC_RELAXED);
}

template <int NB, int WK, int SLOTS, int K, bool ST, bool FULL>
GPK_DEVICE int worker_step_col(f32x4 (&acc)[SLOTS], WorkerCtx& x) {
  static_assert(NB == 16 && WK == 7 && SLOTS == kColSlots, "column plan: NB = 16, 7 workers");
  const int wv = launder_s(x.wv);
  const int e0 = launder_s(x.epoch0);
  int lane = x.lane;
  asm volatile("" : "+v"(lane));
  const int c = lane & 15, grp = lane >> 4;
  const int jA = 15 - wv, jB = wv + 1;
  const float* pprev = x.panel + ((K + 1) & 1) * (NB + 1) * 256;   // panel K-1
  float* pcur = x.panel + (K & 1) * (NB + 1) * 256;                // panel K
  constexpr int OWN_K = ColOwners<K>::col_owner(K);                 // RHS row K, column K
  if constexpr (ST) {
    if (x.lane == 0) x.tl[(K * 8 + x.wv) * 8] = __builtin_amdgcn_s_memtime();
  }
  auto upd = [&](f32x4& d, const float* qt, const pan_op_t p_hl, const pan_op_t p_lh) {
    GPK_EP(epoch_pan<NB, K>(x, qt, e0, 10);)
    d = pan_mma2(pan_load(qt, lane), p_hl, p_lh, d);
  };
  // (check builds) a column operand P of this step's updates
  GPK_EP(auto pck = [&](const float* t, int site) { epoch_pan<NB, K>(x, t, e0, site); };)
  // ---- 1. (the hand-over HO_K = (K, K+1), (K+1, K+1) was produced in step K-1: see 4b)
  // ---- 2. the other tiles of row K (K, j), j >= K+2, through panel K-1
  if constexpr (K > 0) {
    const bool a_row = (K + 2 <= jA);                 // (K, A), A >= K+2
    const bool b_row = (K + 2 <= jB);                 // (K, B)
    constexpr bool C8 = (K + 2 <= 8);                 // (K, 8): slot 18 of wave K (K <= 6)
    const bool c_row = C8 && (wv == K);
    if (a_row || b_row || c_row) {
      GPK_WAITF(kFlagPan + K, e0 + K - 1)
      if (c_row) { GPK_WAITF(kFlagPan + 8, e0 + K - 1) }
      const float* qt = pprev + K * 256;
      if (a_row) {
        GPK_EP(pck(pprev + jA * 256, 11);)
        const pan_op_t p = pan_load(pprev + jA * 256, lane);
        upd(acc[K], qt, p, pan_swap(p));
      }
      if constexpr (17 - K >= 0 && 17 - K < 18) {
        if (b_row) {
          GPK_EP(pck(pprev + jB * 256, 12);)
          const pan_op_t p = pan_load(pprev + jB * 256, lane);
          upd(acc[17 - K], qt, p, pan_swap(p));
        }
      }
      if constexpr (C8) {
        if (c_row) {
          GPK_EP(pck(pprev + 8 * 256, 13);)
          const pan_op_t p = pan_load(pprev + 8 * 256, lane);
          upd(acc[18], qt, p, pan_swap(p));
        }
      }
    }
  }
  // ---- 3. right-hand side row K: rw_K += R_{K-1,K}^T z_{K-1} (owner of column K)
  if constexpr (K > 0) {
    if (wv == OWN_K) {
      GPK_WAITF(kFlagZ, e0 + K - 1)
      if constexpr (K == 8) { GPK_WAITF(kFlagPan + 8, e0 + K - 1) }
      f32x4 d = *(const f32x4*)&x.rw[16 * K + 4 * grp];
      if (c != 0) d = f32x4{0.f, 0.f, 0.f, 0.f};
      GPK_EP(pck(pprev + K * 256, 14);)
      GPK_EP(pck(pprev + NB * 256, 14);)
      d = pan_mma(pan_load(pprev + K * 256, lane), pprev + NB * 256, lane, d);
      if (c == 0) *(f32x4*)&x.rw[16 * K + 4 * grp] = d;
    }
  }
  GPK_WSTAMP(6, 2)  // row K + RHS row K
  // ---- 4. TRSM of row K with R_KK^{-T} (panel K) and z_K
  const float* wbk = x.wbuf + (K % 3) * kWBuf;
  const int flag_now = x.vflag[kFlagFact];
  int fail = x.vflag[kFlagFail + e0 / 32];
  f32x4 q = load_w_v(wbk, c, grp);
  const float inv_sigma = __builtin_bit_cast(float, (int)x.vflag[kFlagInvSigma]);
  if (flag_now < e0 + K) {
    spin_until(x.vflag, kFlagFact, e0 + K);
    fail = x.vflag[kFlagFail + e0 / 32];
    q = load_w_v(wbk, c, grp);
  }
  GPK_WSTAMP(7, 4)  // wait for R_KK^{-T}
  GPK_EP(epoch_expect(x.vflag, kShadowW + K % 3, e0 + K, 15);)
  if (!kKoAny && fail != 0 && ((fail - 1) >> 4) <= K) return 1;
  if constexpr (GPK_EXACT_PRIO) __builtin_amdgcn_s_setprio(GPK_EXACT_PRIO);
  // panel buffer K & 1 held panel K-2 (read in step K-1): every wave must be past step K-1's
  // panel reads (one kFlagBulk add per wave per step)
  if constexpr (K >= 2) { GPK_WAITF(kFlagBulk, WK * K) }
  {
    const WOp wq = w_split(q);
    const bool a_t = (K + 1 <= jA), b_t = (K + 1 <= jB);
    if (a_t) {
      const f32x4 r = pan_store(pcur + jA * 256, lane, trsm_tile(wq, acc[K]));
      GPK_EP(epoch_pan_mark(x, pcur + jA * 256, e0 + K + ((kEpochSabotage && K == 3) ? 1 : 0));)
      if (x.Lb != nullptr) store4<FULL>(x.Lb, x.N, 16 * jA + c, 16 * K + 4 * grp, r * inv_sigma);
    }
    if constexpr (17 - K >= 0 && 17 - K < 18) {
      if (b_t) {
        const f32x4 r = pan_store(pcur + jB * 256, lane, trsm_tile(wq, acc[17 - K]));
        GPK_EP(epoch_pan_mark(x, pcur + jB * 256, e0 + K);)
        if (x.Lb != nullptr) store4<FULL>(x.Lb, x.N, 16 * jB + c, 16 * K + 4 * grp, r * inv_sigma);
      }
    }
    constexpr int C8S = K <= 6 ? 18 : (K == 7 ? 19 : -1);      // (K, 8): wave K slot 18, or wave 0 slot 19
    constexpr int C8W = K <= 6 ? K : 0;
    if constexpr (C8S >= 0) {
      if (wv == C8W) {
        const f32x4 r = pan_store(pcur + 8 * 256, lane, trsm_tile(wq, acc[C8S]));
        GPK_EP(epoch_pan_mark(x, pcur + 8 * 256, e0 + K);)
        if (x.Lb != nullptr) store4<FULL>(x.Lb, x.N, 16 * 8 + c, 16 * K + 4 * grp, r * inv_sigma);
      }
    }
    if (wv == OWN_K) {   // z_K = R_KK^{-T} rw_K
      f32x4 d = *(const f32x4*)&x.rw[16 * K + 4 * grp];
      if (c != 0) d = f32x4{0.f, 0.f, 0.f, 0.f};
      const f32x4 zk = pan_store(pcur + NB * 256, lane, trsm_tile_f32(q, d));   // (y unbounded: fp32)
      GPK_EP(epoch_pan_mark(x, pcur + NB * 256, e0 + K);)
      if (c == 0) {
#pragma unroll
        for (int r = 0; r < 4; ++r) x.sumz2 = __builtin_fmaf(zk[r], zk[r], x.sumz2);
        if (x.zout != nullptr) {
          const int row = 16 * K + 4 * grp;
#pragma unroll
          for (int r = 0; r < 4; ++r)
            if (FULL || row + r < x.N) x.zout[(size_t)x.b * x.N + row + r] = zk[r];
        }
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
    if (x.lane == 0) {
      if (a_t) x.vflag[kFlagPan + jA] = e0 + K;
      if (b_t) x.vflag[kFlagPan + jB] = e0 + K;
      if constexpr (C8S >= 0) {
        if (wv == C8W) x.vflag[kFlagPan + 8] = e0 + K;
      }
      if (wv == OWN_K) x.vflag[kFlagZ] = e0 + K;
    }
    count_in(x, kFlagTrsm);
  }
  // ---- 4b. hand-over HO_{K+1} = (K+1, K+2), (K+2, K+2) through panels K-1 AND K, right
  // after this step's TRSM instead of at the start of step K+1 (behind this step's bulk
  // update): the owners apply panel K-1, then (K+2, K+2)'s deferred RBF, then panel K as soon
  // as its two tiles are out -- the same updates in the same order as before, so the same
  // values -- and the diagonal wave's look-ahead stops waiting for the bulk update.
  if constexpr (K + 2 < NB) {
    constexpr int K1 = K + 1;
    constexpr int HAW = K1 <= 6 ? K1 : (K1 == 7 ? 0 : 14 - K1);   // owner of (K1, K1+1)
    constexpr int HBW = K1 <= 6 ? K1 : (K1 == 7 ? 1 : 14 - K1);   // owner of (K1+1, K1+1)
    constexpr int SA = K1 <= 6 ? 17 - K1 : (K1 == 7 ? 19 : K1);
    constexpr int SB = K1 <= 6 ? 16 - K1 : (K1 == 7 ? 19 : K1 + 1);
    if (wv == HAW || wv == HBW) {
      float* hN = x.hbuf + (K1 & 1) * 512;
      if constexpr (K > 0) {   // panel K-1
        GPK_WAITF(kFlagPan + K1 + 1, e0 + K - 1)
        GPK_EP(pck(pprev + (K1 + 1) * 256, 16);)
        const pan_op_t p = pan_load(pprev + (K1 + 1) * 256, lane);
        const pan_op_t pl = pan_swap(p);
        if (wv == HAW) {
          GPK_WAITF(kFlagPan + K1, e0 + K - 1)
          upd(acc[SA], pprev + K1 * 256, p, pl);
        }
        if (wv == HBW) acc[SB] = pan_mma2(p, p, pl, acc[SB]);
      }
      if (wv == HBW) {   // (K+2, K+2)'s deferred RBF (phase 7 skips it)
        const RbfK rk = read_rbfk(x.smem + x.rbfc);
        acc[SB] += rbf_tile<NB, FULL>(x.smem, rk, K1 + 1, K1 + 1, lane, x.N);
      }
      // panel K (this step's TRSM)
      GPK_WAITF(kFlagPan + K1 + 1, e0 + K)
      GPK_EP(pck(pcur + (K1 + 1) * 256, 17);)
      const pan_op_t p = pan_load(pcur + (K1 + 1) * 256, lane);
      const pan_op_t pl = pan_swap(p);
      if (wv == HAW) {
        GPK_WAITF(kFlagPan + K1, e0 + K)
        upd(acc[SA], pcur + K1 * 256, p, pl);
        GPK_EP(epoch_mark(x.vflag, kShadowHo + 2 * (K1 & 1), e0 + K1, lane);)
        publish_tile(hN, lane, acc[SA], x.vflag, kFlagHA + (K1 & 1), e0 + K1);
      }
      if (wv == HBW) {
        acc[SB] = pan_mma2(p, p, pl, acc[SB]);
        GPK_EP(epoch_mark(x.vflag, kShadowHo + 2 * (K1 & 1) + 1, e0 + K1, lane);)
        publish_tile(hN + 256, lane, acc[SB], x.vflag, kFlagHB + (K1 & 1), e0 + K1);
      }
    }
  }
  if constexpr (GPK_EXACT_PRIO) __builtin_amdgcn_s_setprio(0);
  GPK_WSTAMP(4, 5)  // TRSM + hand-over
  if constexpr (K + 1 == NB) return 0;
  // ---- 5. the rest of the trailing update through panel K-1: rows K+1 .. of the owned columns
  if constexpr (K > 0) {
    GPK_WAITF(kFlagTrsm, WK * K)   // panel K-1 complete
    // column A (rows K+1 .. jA; (K+1, K+1) is HB: done)
    if (K + 1 <= jA) {
      GPK_EP(pck(pprev + jA * 256, 18);)
      const pan_op_t p = pan_load(pprev + jA * 256, lane);
      const pan_op_t pl = pan_swap(p);
      static_for_range<K + 1, 15>([&](auto I) {
        constexpr int i = decltype(I)::value;
        constexpr bool ho = K + 2 < NB && (i == K + 1 || i == K + 2);   // HO_{K+1}: done in 4b
        if (i <= jA && !(i == K + 1 && jA == K + 1) && !(ho && jA == K + 2))
          upd(acc[i], pprev + i * 256, p, pl);
      });
    }
    // column B (rows K+1 .. jB <= 7)
    if constexpr (K + 1 <= 7) {
      if (K + 1 <= jB) {
        GPK_EP(pck(pprev + jB * 256, 19);)
        const pan_op_t p = pan_load(pprev + jB * 256, lane);
        const pan_op_t pl = pan_swap(p);
        static_for_range<K + 1, 7>([&](auto I) {
          constexpr int i = decltype(I)::value;
          constexpr bool ho = K + 2 < NB && (i == K + 1 || i == K + 2);
          if (i <= jB && !(i == K + 1 && jB == K + 1) && !(ho && jB == K + 2))
            upd(acc[17 - i], pprev + i * 256, p, pl);
        });
      }
    }
    // column 8: (w, 8) slot 18 and (w + 7, 8) slot 19
    if constexpr (K + 1 <= 8) {
      const bool s18 = (wv >= K + 1);                             // row w <= 6 < 8
      const bool s19 = (wv <= 1) && (wv + 7 >= K + 1) && !(wv + 7 == 8 && K + 1 == 8) &&
                       !(K + 2 == 8 && (wv + 7 == K + 1 || wv + 7 == K + 2));   // HO_7: 4b
      if (s18 || s19) {
        GPK_EP(pck(pprev + 8 * 256, 20);)
        const pan_op_t p = pan_load(pprev + 8 * 256, lane);
        const pan_op_t pl = pan_swap(p);
        if (s18) upd(acc[18], pprev + wv * 256, p, pl);
        if (s19) upd(acc[19], pprev + (wv + 7) * 256, p, pl);
      }
    }
    GPK_WSTAMP(2, 1)  // trailing update
    // ---- 6. right-hand side rows > K of the owned columns: rw_j += R_{K-1,j}^T z_{K-1}
    auto rhs = [&](int j) {
      f32x4 d = *(const f32x4*)&x.rw[16 * j + 4 * grp];
      if (c != 0) d = f32x4{0.f, 0.f, 0.f, 0.f};
      GPK_EP(pck(pprev + j * 256, 21);)
      GPK_EP(pck(pprev + NB * 256, 21);)
      d = pan_mma(pan_load(pprev + j * 256, lane), pprev + NB * 256, lane, d);
      if (c == 0) *(f32x4*)&x.rw[16 * j + 4 * grp] = d;
    };
    GPK_WAITF(kFlagZ, e0 + K - 1)
    if (K + 1 <= jA) rhs(jA);
    if (K + 1 <= jB) rhs(jB);
    if constexpr (K + 1 <= 8) {
      if (wv == 1) rhs(8);
    }
  }
  count_in(x, kFlagBulk);   // this wave is done reading panel K-1
  GPK_WSTAMP(5, 6)
  // ---- 7. deferred RBF of block row K+2 and L's upper zeros
  if constexpr (K + 2 < NB) {
    constexpr int R = K + 2;
    const RbfK rk = read_rbfk(x.smem + x.rbfc);
    // ((R, R) is HO_{K+1}'s tile: its RBF went in with the hand-over, 4b)
    if (R < jA) acc[R] += rbf_tile<NB, FULL>(x.smem, rk, R, jA, lane, x.N);
    if constexpr (17 - R >= 0 && R <= 7) {
      if (R < jB) acc[17 - R] += rbf_tile<NB, FULL>(x.smem, rk, R, jB, lane, x.N);
    }
    if constexpr (R <= 6) {
      if (wv == R) acc[18] += rbf_tile<NB, FULL>(x.smem, rk, R, 8, lane, x.N);
    }
    if constexpr (R == 7) {
      if (wv == 0) acc[19] += rbf_tile<NB, FULL>(x.smem, rk, R, 8, lane, x.N);
    }
  }
  if (x.Lb != nullptr) zero_l_block<FULL>(x.Lb, FULL ? 16 * NB : x.N, K, wv, WK, lane);
  GPK_WSTAMP(3, 3)  // RBF + zero-L
  if constexpr (ST) {
    if (x.lane == 0) x.tl[(K * 8 + x.wv) * 8 + 7] = x.st[9];   // cumulative flag-wait cycles
  }
  return 0;
}

template <int NB, int WK, int SLOTS, int K, bool ST, bool FULL, bool COL>
GPK_DEVICE int worker_steps(f32x4 (&acc)[SLOTS], WorkerCtx& x) {
  if constexpr (K < NB) {
    if constexpr (COL) {
      if (worker_step_col<NB, WK, SLOTS, K, ST, FULL>(acc, x)) return 1;
    } else {
      if (worker_step_split<NB, WK, SLOTS, K, ST, FULL>(acc, x)) return 1;
    }
    return worker_steps<NB, WK, SLOTS, K + 1, ST, FULL, COL>(acc, x);
  } else {
    return 0;
  }
}

// OCC = workgroups per CU the register budget is sized for: 2 (the B >= 2 x CUs
// layout, two windows per CU) or 1 (small batches: one window per CU with W = 16
// waves, twice the workers per window -- launch_exact_nb).
// Role of physical wave p in the DIAG_ALONE layout (a permutation of 0..15): the waves of
// SIMD 3 (p % 4 == 3) are the diagonal wave (p = 15 -> 12) and three idle waves (13..15);
// the 12 waves of SIMDs 0-2 are workers 0..11. Every wave still joins the prologue and the
// final reduction (the permutation keeps their per-wave LDS slots distinct).
GPK_DEVICE int exact_role(int p) {
  if (p == 15) return 12;
  if ((p & 3) == 3) return 13 + (p >> 2);
  return (p >> 2) * 3 + (p & 3);
}

template <int NB, int W, bool STAMPS, bool FULL, int OCC = 2>
__global__ void __launch_bounds__(64 * W, (OCC * W) / 4)
gpk_exact_kernel(const float* __restrict__ X, const float* __restrict__ y,
                 const float* __restrict__ hyp, int n_ls, int N_in, int D, int DC,
                 double jitter0, int max_tries, float* __restrict__ Lout,
                 float* __restrict__ zout, float* __restrict__ mll,
                 int* __restrict__ info, unsigned long long* __restrict__ stamps = nullptr) {
  constexpr int NT = ExactPlan<NB>::NT;
  const int N = FULL ? 16 * NB : N_in;  // FULL: no padded rows anywhere
  // DIAG_ALONE (small-batch layout, 16 waves, NB <= 8): the diagonal wave gets a SIMD to
  // itself -- waves are dealt to the 4 SIMDs round-robin, so the three other waves of its
  // SIMD idle and 12 workers remain (see exact_role). Measured (profiles/r06_exact_alone_ab.txt):
  // B=128 N=128 20.3 -> 19.2 us; at N=256 (136 tiles) the workers pace the steps and the same
  // layout is 2 % slower, so NB > 8 keeps 15 workers.
  constexpr bool ALONE = GPK_EXACT_DIAG_ALONE && OCC == 1 && W == 16 && NB <= 8;
  constexpr int WK = ALONE ? 12 : W - 1;     // worker waves; wave WK is the diagonal wave
  constexpr bool COL = GPK_EXACT_COL && NB == 16 && WK == 7;   // column-ownership worker plan
  constexpr int SLOTS = COL ? kColSlots : (NT + WK - 1) / WK;
  constexpr int T = 64 * W;
  // Diagnostic-only phase clocks (STAMPS build): wave 0 lane 0 of each workgroup.
  unsigned long long st_acc[14] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0}, st_last = 0, st_t0 = 0, st_rt0 = 0;
  if constexpr (STAMPS) {
    st_rt0 = __builtin_amdgcn_s_memrealtime();
    st_t0 = __builtin_amdgcn_s_memtime();
    st_last = st_t0;
  }
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const ExactLds lay = exact_lds_layout(NB, DC, W);
  float* xf = smem + lay.xf;
  float* nrm = smem + lay.nrm;
  float* rv = smem + lay.rv;
  float* rw = smem + lay.rw;
  float* panel = smem + lay.panel;
  float* wbuf = smem + lay.wbuf;
  float* dsc = smem + lay.dsc;
  float* hbuf = smem + lay.hbuf;
  float* cpart = smem + lay.cpart;
  float* red = smem + lay.red;
  int* flag = (int*)(red + 4 * W);

  const int tid = threadIdx.x;
  const int lane = tid & 63, c = lane & 15, grp = lane >> 4;
  const int wave = ALONE ? exact_role(wave_id_uniform()) : wave_id_uniform();
  const int b = blockIdx.x;
  const int DP = DC * 16;
  const int NP = NB * 16;

  const float s2u = hyp[0];
  const float noise = hyp[1];
  const float cmean = hyp[2];
  // Factor sigma^2 * K_hat with sigma = 2^sh chosen so the diagonal lands in
  // [2^13, 2^15): exact in binary (every fp32 result is the unscaled one times a
  // power of two) and it puts the split-f16 trailing-update operands (|R_ij| <=
  // sqrt(K_jj) <= 2^7.5) high in the f16 range, so lo parts stay normal down to
  // entries 2^-9 of the largest. Undone on output: L = R'^T / sigma,
  // log|K_hat| -= N log sigma^2, and z = L^{-1}(y - c) is unchanged when the
  // right-hand side is scaled by sigma.
  int sh = 0;
  {
    int e = 0;
    const float d0 = s2u + noise;
    if (d0 > 0.f && d0 < __builtin_huge_valf()) (void)__builtin_frexpf(d0, &e);
    sh = 7 - (e >> 1);  // d0 * 2^(2 sh) in [2^13, 2^15)
  }
  const float sigma = __builtin_ldexpf(1.f, sh), sigma2 = sigma * sigma;
  const float inv_sigma = __builtin_ldexpf(1.f, -sh);
  const float s2 = s2u * sigma2;
  const float* Xb = X + (size_t)b * N * D;
  float* Lb = Lout ? Lout + (size_t)b * N * N : nullptr;

  // Fast prologue (DC in {1, 2, 4} and one (row, 16-column chunk) item per thread, e.g.
  // N=256 D=32): X stays in registers from the load to the f16 images -- column sums by a
  // register butterfly (permlane32 / permlane16 swaps, DPP) and one LDS partial per wave,
  // the y load issued with the X loads. Otherwise the staged path below.
  const bool fast = (DC == 1 || DC == 2 || DC == 4) && NP * DC <= T;
  if (fast) {
    const int q = tid;
    const int n = q / DC, dd = q & (DC - 1), d0 = 16 * dd;
    const bool live = q < NP * DC;
    float v[16];
    float yv = 0.f;
    if (live && dd == 0 && n < N) yv = y[(size_t)b * N + n];
    if (live && n < N && (D & 3) == 0 && d0 + 16 <= D) {
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const f32x4 t = *(const f32x4*)&Xb[(size_t)n * D + d0 + 4 * u];
#pragma unroll
        for (int r = 0; r < 4; ++r) v[4 * u + r] = t[r];
      }
    } else {
#pragma unroll
      for (int e = 0; e < 16; ++e) v[e] = Xb[(live && n < N && d0 + e < D) ? (size_t)n * D + d0 + e : 0];
#pragma unroll
      for (int e = 0; e < 16; ++e)
        if (!(live && n < N && d0 + e < D)) v[e] = 0.f;
    }
    if (n_ls == 1) {
      const float inv_l0 = 1.f / hyp[3];
#pragma unroll
      for (int e = 0; e < 16; ++e) v[e] *= inv_l0;
    } else {
      float l[16];
#pragma unroll
      for (int e = 0; e < 16; ++e) l[e] = hyp[3 + (d0 + e < D ? d0 + e : 0)];
#pragma unroll
      for (int e = 0; e < 16; ++e)
        if (d0 + e < D) v[e] = v[e] / l[e];
    }
    float mx = 0.f;
#pragma unroll
    for (int e = 0; e < 16; ++e) mx = __builtin_fmaxf(mx, __builtin_fabsf(v[e]));
    mx = wave_max_dpp(mx);
    if (lane == 0) red[wave] = mx;
    // column sums of this wave's rows: reduce-scatter over lane bits 5, 4, 3, then plain
    // DPP adds over the lane bits that hold other rows of the same chunk
    float s8[8], t4[4], u2[2];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const auto r = __builtin_amdgcn_permlane32_swap(__builtin_bit_cast(int, v[i]), __builtin_bit_cast(int, v[i + 8]),
                                                      false, false);
      s8[i] = __builtin_bit_cast(float, (int)r[0]) + __builtin_bit_cast(float, (int)r[1]);  // col i + 8 b5
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const auto r = __builtin_amdgcn_permlane16_swap(__builtin_bit_cast(int, s8[i]), __builtin_bit_cast(int, s8[i + 4]),
                                                      false, false);
      t4[i] = __builtin_bit_cast(float, (int)r[0]) + __builtin_bit_cast(float, (int)r[1]);  // + 4 b4
    }
    const bool b3 = (lane >> 3) & 1;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const float keep = b3 ? t4[i + 2] : t4[i];
      const float send = b3 ? t4[i] : t4[i + 2];
      u2[i] = keep + __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, send), 0x128, 0xf, 0xf, false));
      if (DC == 1)
        u2[i] += __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, u2[i]), 0xB1, 0xf, 0xf, false));
      if (DC <= 2)
        u2[i] += __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, u2[i]), 0x4E, 0xf, 0xf, false));
    }
    // partials: xf[col * 2W + 2 * wave + bit2] (the image area is free until the barrier
    // after the mean)
    const bool writer = DC == 1 ? (lane & 3) == 0 : (DC == 2 ? (lane & 2) == 0 : true);
    if (writer) {
      const int cc = 2 * ((lane >> 3) & 1) + 4 * ((lane >> 4) & 1) + 8 * ((lane >> 5) & 1);
      const int col = 16 * (lane & (DC - 1)) + cc;
      const int slot = 2 * wave + ((lane >> 2) & 1);
      xf[col * 2 * W + slot] = u2[0];
      xf[(col + 1) * 2 * W + slot] = u2[1];
    }
    barrier_lds();
    GPK_STAMP(8)
    if (tid == 0) {
      flag[0] = 0;
      flag[kFlagT00] = -1;
      flag[kFlagFact] = -1;
      for (int qq = 3; qq < 16; ++qq) flag[qq] = 0;
      for (int qq = 0; qq < 2; ++qq) flag[kFlagHA + qq] = flag[kFlagHB + qq] = -1;
      flag[kFlagSync] = 0;
      flag[kFlagTmo] = 0;
      for (int qq = kFlagPan; qq <= kFlagZ; ++qq) flag[qq] = -1;
      flag[kFlagTrsm] = 0;
      flag[kFlagBulk] = 0;
      flag[kFlagRst] = 0;
      flag[kFlagInvSigma] = __builtin_bit_cast(int, inv_sigma);
      smem[lay.rbfc + 1] = s2;
      ((int*)smem)[lay.rbfc + 3] = lay.nrm | (((DC + 1) / 2) << 20);
      if constexpr (STAMPS) {
        ((unsigned long long*)(red + 4 * W + 24))[0] = 0;
        ((unsigned long long*)(red + 4 * W + 26))[0] = 0;
        ((unsigned long long*)(red + 4 * W + 28))[0] = 0;
        for (int qq = 0; qq < 3; ++qq) ((unsigned long long*)(red + 4 * W + 32))[qq] = 0;
      }
    }
    if (tid < DP) {
      float sum = 0.f;
      for (int w = 0; w < 2 * W; w += 4) {
        const f32x4 p4 = *(const f32x4*)&xf[tid * 2 * W + w];
        sum += (p4[0] + p4[1]) + (p4[2] + p4[3]);
      }
      cpart[64 * W + tid] = sum / (float)N;
    }
    int a_sc = 0;
    {
      float m = 0.f;
      for (int w = 0; w < W; ++w) m = __builtin_fmaxf(m, red[w]);
      int e = 0;
      if (m > 0.f && m < __builtin_huge_valf()) (void)__builtin_frexpf(m, &e);
      a_sc = 13 - e;
      a_sc = a_sc > 100 ? 100 : (a_sc < -100 ? -100 : a_sc);
    }
    const float xsc = __builtin_ldexpf(1.f, a_sc);
    if (tid == 0) smem[lay.rbfc] = __builtin_ldexpf(-2.f, -2 * a_sc);
    barrier_lds();
    GPK_STAMP(10)
    // centre, squared norms, split into f16 hi + lo images (hfrag layout)
    float sq = 0.f;
    if (live && n < N) {
      const float* cm = cpart + 64 * W + d0;
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const f32x4 m4 = *(const f32x4*)&cm[4 * u];
#pragma unroll
        for (int r = 0; r < 4; ++r) v[4 * u + r] = (d0 + 4 * u + r < D) ? v[4 * u + r] - m4[r] : 0.f;
      }
    }
#pragma unroll
    for (int e = 0; e < 16; ++e) sq = __builtin_fmaf(v[e], v[e], sq);
    if (DC >= 2)
      sq += __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, sq), 0xB1, 0xf, 0xf, false));
    if (DC >= 4)
      sq += __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, sq), 0x4E, 0xf, 0xf, false));
    if (live) {
      _Float16* xh16 = (_Float16*)(smem + lay.xf);
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        half8_t hi, lo;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float ts = v[8 * h + j] * xsc;
          hi[j] = (_Float16)ts;
          lo[j] = (_Float16)(ts - (float)hi[j]);
        }
        *(half8_t*)&xh16[hfrag_index(n, d0 + 8 * h, NB, 0)] = hi;
        *(half8_t*)&xh16[hfrag_index(n, d0 + 8 * h, NB, 1)] = lo;
        if (DC == 1) {   // columns 16-31 of the 32-column image chunk are padding
          const half8_t z = {};
          *(half8_t*)&xh16[hfrag_index(n, 16 + 8 * h, NB, 0)] = z;
          *(half8_t*)&xh16[hfrag_index(n, 16 + 8 * h, NB, 1)] = z;
        }
      }
      if (dd == 0) {
        nrm[n] = sq;
        rv[n] = (n < N) ? (yv - cmean) * sigma : 0.f;
      }
    }
  } else {
    // ---- 1. stage X / l into LDS in fragment layout (zero padded) ----------
    // Each thread owns 16-column chunks of rows; all of its global loads are
    // issued before any is consumed.
    {
      const int chunks = NP * DC;  // (row, 16-col chunk) pairs
      float mx = 0.f;              // max |x / l| (bounds the centred values for the f16 split)
      // x / l as x * (1 / l): one uniform division (GPyTorch divides; the <= 1 ulp
      // difference is far inside the 1e-4 parity bound)
      const float inv_l0 = 1.f / hyp[3];
      for (int base = 0; base < chunks; base += T) {
        const int q = base + tid;
        float v[16];
        const int n = q / DC, dd = q - n * DC;
        if (q < chunks) {
          const int d0 = dd * 16;
          if (n < N && (D & 3) == 0 && d0 + 16 <= D) {
  #pragma unroll
            for (int u = 0; u < 4; ++u) {
              const f32x4 t = *(const f32x4*)&Xb[(size_t)n * D + d0 + 4 * u];
  #pragma unroll
              for (int r = 0; r < 4; ++r) v[4 * u + r] = t[r];
            }
          } else {
            // ragged: clamped unconditional loads (all 16 in flight), masked afterwards
  #pragma unroll
            for (int e = 0; e < 16; ++e) v[e] = Xb[(n < N && d0 + e < D) ? (size_t)n * D + d0 + e : 0];
  #pragma unroll
            for (int e = 0; e < 16; ++e)
              if (!(n < N && d0 + e < D)) v[e] = 0.f;
          }
          if (n_ls == 1) {
  #pragma unroll
            for (int e = 0; e < 16; ++e) v[e] *= inv_l0;
          } else {
            float l[16];
  #pragma unroll
            for (int e = 0; e < 16; ++e) l[e] = hyp[3 + (d0 + e < D ? d0 + e : 0)];
  #pragma unroll
            for (int e = 0; e < 16; ++e)
              if (d0 + e < D) v[e] = v[e] / l[e];
          }
  #pragma unroll
          for (int e = 0; e < 16; ++e) mx = __builtin_fmaxf(mx, __builtin_fabsf(v[e]));
  #pragma unroll
          for (int u = 0; u < 4; ++u)
            *(f32x4*)&xf[frag_index(n, d0 + 4 * u, NB)] = f32x4{v[4 * u], v[4 * u + 1], v[4 * u + 2], v[4 * u + 3]};
        }
      }
      mx = wave_max_dpp(mx);
      if (lane == 0) red[wave] = mx;
    }
    barrier_lds();
    GPK_STAMP(8)  // X loads + fp32 staging + max
    if (tid == 0) {
      flag[0] = 0;
      flag[kFlagT00] = -1;
      flag[kFlagFact] = -1;
      for (int q = 3; q < 16; ++q) flag[q] = 0;
      for (int qq = 0; qq < 2; ++qq) flag[kFlagHA + qq] = flag[kFlagHB + qq] = -1;
      flag[kFlagSync] = 0;
      flag[kFlagTmo] = 0;
      for (int qq = kFlagPan; qq <= kFlagZ; ++qq) flag[qq] = -1;
      flag[kFlagTrsm] = 0;
      flag[kFlagBulk] = 0;
      flag[kFlagRst] = 0;
      flag[kFlagInvSigma] = __builtin_bit_cast(int, inv_sigma);  // read back per step (SGPR budget)
      smem[lay.rbfc + 1] = s2;
      ((int*)smem)[lay.rbfc + 3] = lay.nrm | (((DC + 1) / 2) << 20);
      if constexpr (STAMPS) {
        ((unsigned long long*)(red + 4 * W + 24))[0] = 0;
        ((unsigned long long*)(red + 4 * W + 26))[0] = 0;
        ((unsigned long long*)(red + 4 * W + 28))[0] = 0;
        for (int q = 0; q < 3; ++q) ((unsigned long long*)(red + 4 * W + 32))[q] = 0;
      }
    }
    // ---- 2. centre columns by the mean over the N real rows (GPyTorch _sq_dist)
    {
      const int parts = T / DP;
      const int part = tid / DP, d = tid - part * DP;
      if (part < parts) {
        float sacc[4] = {0.f, 0.f, 0.f, 0.f};
        int n = part;
        for (; n + 3 * parts < N; n += 4 * parts) {
  #pragma unroll
          for (int u = 0; u < 4; ++u) sacc[u] += xf[frag_index(n + u * parts, d, NB)];
        }
        for (; n < N; n += parts) sacc[0] += xf[frag_index(n, d, NB)];
        cpart[part * DP + d] = (sacc[0] + sacc[1]) + (sacc[2] + sacc[3]);
      }
      barrier_lds();
      GPK_STAMP(9)  // column partial sums
      if (tid < DP) {
        float s = 0.f;
        for (int p = 0; p < parts; ++p) s += cpart[p * DP + tid];
        cpart[64 * W + tid] = s / (float)N;
      }
      barrier_lds();
      GPK_STAMP(10)  // mean
    }
    // ---- 3. subtract the mean, squared norms, residual r = y - c -----------
    // The centred rows are split into f16 hi + lo parts (x = hi + lo + O(2^-22 x))
    // for the 3-pass f16 MFMA Gram; the images overwrite the
    // fp32 staging chunk pair they were read from (read all -> barrier -> write).
    {
      const float* cmean_d = cpart + 64 * W;
      _Float16* xh16 = (_Float16*)(smem + lay.xf);
      // power-of-two scale 2^a for the f16 images: |x - mean| <= 2 max|x| < 2^(e+1)
      // -> scaled magnitudes < 2^14 (f16 max 65504), lo parts normal down to 2^-2.
      // The Gram comes back times 2^(2a) and is rescaled exactly in the RBF.
      int a_sc = 0;
      {
        float m = 0.f;
        for (int w = 0; w < W; ++w) m = __builtin_fmaxf(m, red[w]);
        int e = 0;
        if (m > 0.f && m < __builtin_huge_valf()) (void)__builtin_frexpf(m, &e);
        a_sc = 13 - e;
        a_sc = a_sc > 100 ? 100 : (a_sc < -100 ? -100 : a_sc);
      }
      const float xsc = __builtin_ldexpf(1.f, a_sc);
      if (tid == 0) smem[lay.rbfc] = __builtin_ldexpf(-2.f, -2 * a_sc);
      const int DC32 = (DC + 1) / 2;
      const int n = tid;  // NP <= 256 <= T: one row per thread
      float s = 0.f;
      for (int q = 0; q < DC32; ++q) {
        float v[32];
  #pragma unroll
        for (int u = 0; u < 8; ++u) {
          const int d0 = 32 * q + 4 * u;
          f32x4 t = {0.f, 0.f, 0.f, 0.f};
          if (n < NP && d0 < 16 * DC) {
            t = *(const f32x4*)&xf[frag_index(n, d0, NB)];
            if (n < N) {
              const f32x4 m4 = *(const f32x4*)&cmean_d[d0];
  #pragma unroll
              for (int r = 0; r < 4; ++r) t[r] = (d0 + r < D) ? t[r] - m4[r] : 0.f;
            }
          }
  #pragma unroll
          for (int r = 0; r < 4; ++r) v[4 * u + r] = t[r];
        }
        barrier_lds();
        if (n < NP) {
  #pragma unroll
          for (int u = 0; u < 8; ++u) {
            half4_t hi, lo;
  #pragma unroll
            for (int r = 0; r < 4; ++r) {
              const float t = v[4 * u + r];
              s = __builtin_fmaf(t, t, s);
              const float ts = t * xsc;
              hi[r] = (_Float16)ts;
              lo[r] = (_Float16)(ts - (float)hi[r]);
            }
            *(half4_t*)&xh16[hfrag_index(n, 32 * q + 4 * u, NB, 0)] = hi;
            *(half4_t*)&xh16[hfrag_index(n, 32 * q + 4 * u, NB, 1)] = lo;
          }
        }
        barrier_lds();
        GPK_STAMP(11)  // centre + f16 split (per 32-col chunk)
      }
      if (n < NP) {
        nrm[n] = s;
        rv[n] = (n < N) ? (y[(size_t)b * N + n] - cmean) * sigma : 0.f;
      }
    }
  }
  barrier_lds();
  GPK_STAMP(0)

  int info_w = 0, failed = 0, att_end = 0;
  float logdet = 0.f, sumz2 = 0.f;
  lds_vint* vflag = as_lds_flags(flag);
  // The diagonal wave and the worker waves run separate programs and meet at
  // no barrier until the end: within an attempt every hand-off goes through
  // LDS flags holding monotone epochs, and the workers synchronise among
  // themselves (worker_sync). The diagonal wave runs AHEAD of the workers: its
  // per-step chain is factor (k,k) -> R_{k,k+1} -> last update of (k+1,k+1) ->
  // factor (k+1,k+1), with the inputs of the look-ahead handed over early.
  if (wave == WK) {
    // ================================================= diagonal wave program
    __builtin_amdgcn_s_setprio(3);  // critical path: win issue arbitration
    for (int attempt = 0; attempt <= max_tries; ++attempt) {
      att_end = attempt;
      logdet = 0.f;
      failed = 0;
      spin_until(vflag, kFlagT00, 32 * attempt);
      // the tile being factored, acc layout in registers: (0,0) from the worker that built it,
      // then each look-ahead's (k+1,k+1) straight from its MFMAs
      f32x4 tcur = *(const f32x4*)&dsc[lane * 4];
      for (int k = 0; k < NB; ++k) {
        const int epoch = 32 * attempt + k;
        float* wb = wbuf + (k % 3) * kWBuf;
        unsigned long long dt0 = 0;
        if constexpr (STAMPS) {
          dt0 = __builtin_amdgcn_s_memtime();
          if (lane == 0 && k == 0) {
            flag[16] = __builtin_amdgcn_s_getreg(4 | (31 << 11));   // HW_ID
            flag[17] = __builtin_amdgcn_s_getreg(20 | (31 << 11));  // XCC_ID
          }
        }
        float dv[16], dg;
        const int f = diag_factor<STAMPS, FULL>(tcur, dv, dg, wb, vflag, vflag + kFlagFail + attempt, epoch, dsc,
                                                (unsigned long long*)(red + 4 * W + 32));
        if constexpr (STAMPS) {
          const unsigned long long dt1 = __builtin_amdgcn_s_memtime();
          if (lane == 0) {
            ((unsigned long long*)(red + 4 * W + 24))[0] += dt1 - dt0;
            unsigned long long* tl = stamps + (size_t)b * kStampStride + 32 + (k * 8 + 7) * 8;
            tl[0] = dt0;
            tl[1] = dt1;
          }
        }
        if (f != 0) {
          failed = 16 * k + f;
          if (lane == 0) vflag[kFlagFail + attempt] = failed;
          break;
        }
        if (k == NB - 1) {
          diag_finish<FULL>(dv, dg, Lb, N, 16 * k, inv_sigma, logdet);
          break;
        }
        // look-ahead: R_{k,k+1} = R_kk^{-T} T'_{k,k+1}, then the last update of
        // (k+1,k+1); both tiles arrive (updated through panel k-1) in hbuf[k & 1]
        const float* hk = hbuf + (k & 1) * 512;
        // R_kk^{-T} back in the MFMA A layout (this wave's own LDS writes: no flag needed, and
        // the read is in flight while the wave waits for the hand-over)
        const f32x4 q = load_w(wb, c, grp);
        // step k's L block and log|T|: ahead of the wait (in the in-order wave, work after the
        // wait sits on the chain)
        if (!GPK_DIAG_FINISH_LATE) diag_finish<FULL>(dv, dg, Lb, N, 16 * k, inv_sigma, logdet);
        unsigned long long hw0 = 0;
        if constexpr (STAMPS) hw0 = __builtin_amdgcn_s_memtime();
        spin_until(vflag, kFlagHA + (k & 1), epoch);
        spin_until(vflag, kFlagHB + (k & 1), epoch);
        if constexpr (STAMPS) {
          const unsigned long long hw1 = __builtin_amdgcn_s_memtime();
          if (lane == 0) {
            ((unsigned long long*)(red + 4 * W + 26))[0] += hw1 - hw0;
            stamps[(size_t)b * kStampStride + 32 + (k * 8 + 7) * 8 + 2] = hw1;
          }
          hw0 = hw1;
        }
        GPK_EP(epoch_expect(vflag, kShadowHo + 2 * (k & 1), epoch, 30); epoch_expect(vflag, kShadowHo + 2 * (k & 1) + 1, epoch, 31);)
        const f32x4 ta = *(const f32x4*)&hk[lane * 4];
        f32x4 tb = *(const f32x4*)&hk[256 + lane * 4];
        tb = pan_self(trsm_tile(w_split(q), ta), tb);
        if (GPK_DIAG_FINISH_LATE) diag_finish<FULL>(dv, dg, Lb, N, 16 * k, inv_sigma, logdet);
        tcur = tb;
        if (!GPK_DIAG_PERMLANE) *(f32x4*)&dsc[lane * 4] = tb;
        if constexpr (STAMPS) {
          const unsigned long long hw2 = __builtin_amdgcn_s_memtime();
          if (lane == 0) {
            ((unsigned long long*)(red + 4 * W + 28))[0] += hw2 - hw0;
            stamps[(size_t)b * kStampStride + 32 + (k * 8 + 7) * 8 + 3] = hw2;
          }
        }
      }
      if (!failed) { info_w = attempt > 0 ? -attempt : 0; break; }
      info_w = failed;
    }
    if (GPK_TMO_DEBUG && lane == 0) vflag[24] = att_end;
    __builtin_amdgcn_s_setprio(0);
  } else if (!ALONE || wave < WK) {
    // ================================================= worker program
    float diagval = (s2u + noise) * sigma2;
    double jit_prev = 0.0;
    f32x4 acc[SLOTS];
    unsigned long long wst[10] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
    WorkerCtx wx{panel, wbuf, hbuf, vflag, Lb, zout, rw, smem, lay.rbfc, N, b, lane, c, grp,
                 launder_s(wave), 0, 0, 0.f, nullptr,
                 STAMPS ? stamps + (size_t)b * kStampStride + 32 : nullptr};
    for (int attempt = 0; attempt <= max_tries; ++attempt) {
      att_end = attempt;
      if (attempt > 0) {
        double p10 = 1.0;
        for (int q = 1; q < attempt; ++q) p10 *= 10.0;
        const double jn = jitter0 * p10;
        diagval = diagval + (float)(jn - jit_prev) * sigma2;
        jit_prev = jn;
      }
      // right-hand side: this wave's block rows of rw <- -(y - c) (fresh per attempt); in the
      // column plan each row is initialised by the wave that owns it (columns A, B; 8: wave 1)
      if constexpr (COL) {
        const int wv = launder_s(wave);
        if (lane < 16) {
          rw[16 * (15 - wv) + lane] = -rv[16 * (15 - wv) + lane];
          rw[16 * (wv + 1) + lane] = -rv[16 * (wv + 1) + lane];
          if (wv == 1) rw[16 * 8 + lane] = -rv[16 * 8 + lane];
          if (wv == 0) rw[lane] = -rv[lane];
        }
      } else {
        for (int i = wave; i < NB; i += WK)
          if (lane < 16) rw[16 * i + lane] = -rv[16 * i + lane];
      }
      // ---- 4. RBF of block rows 0-2 (the rest is deferred into the
      // factorisation steps); the owners of (0,0), (0,1), (1,1) build and hand
      // those over first, so the diagonal wave starts right away.
      {
        const int wv = launder_s(wave);
        // every worker writes the same value; nobody reads it before this
        // attempt's first RBF tile (the failed attempt ended at a worker_sync)
        if (lane == 0) *(__attribute__((address_space(3))) volatile float*)&smem[lay.rbfc + 2] = diagval;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
        const RbfK rk = read_rbfk(smem + lay.rbfc);
        if constexpr (COL) {
          // (0,0) is built by wave 6 and handed over (column 0 has no worker); (0,1), (1,1) --
          // column 1 = B of wave 0 -- first, then rows 0-1 of every owned column
          const int e0 = 32 * attempt;
          const int jA = 15 - wv, jB = wv + 1;
          if (wv == 6) {
            const f32x4 t00 = rbf_tile<NB, FULL>(smem, rk, 0, 0, lane, N);
            publish_tile(dsc, lane, t00, vflag, kFlagT00, e0);
          }
          acc[17] = rbf_tile<NB, FULL>(smem, rk, 0, jB, lane, N);
          acc[16] = rbf_tile<NB, FULL>(smem, rk, 1, jB, lane, N);
          if (wv == 0) {
            GPK_EP(epoch_mark(vflag, kShadowHo, e0, lane); epoch_mark(vflag, kShadowHo + 1, e0, lane);)
            publish_tile(hbuf, lane, acc[17], vflag, kFlagHA + 0, e0);
            publish_tile(hbuf + 256, lane, acc[16], vflag, kFlagHB + 0, e0);
          }
          acc[0] = rbf_tile<NB, FULL>(smem, rk, 0, jA, lane, N);
          acc[1] = rbf_tile<NB, FULL>(smem, rk, 1, jA, lane, N);
          acc[18] = wv <= 1 ? rbf_tile<NB, FULL>(smem, rk, wv, 8, lane, N) : f32x4{0.f, 0.f, 0.f, 0.f};
          static_for_range<2, 15>([&](auto I) { acc[decltype(I)::value] = f32x4{0.f, 0.f, 0.f, 0.f}; });
          acc[19] = f32x4{0.f, 0.f, 0.f, 0.f};
        } else {
        constexpr int P0 = plan_P<NB>(0);
        constexpr int P1 = NB > 1 ? plan_P<NB>(1) : 0;
        constexpr int P2 = P1;   // rows 0-1 now, row k+2 at step k
        constexpr int T01 = P0 + 1;
        const int e0 = 32 * attempt;
        if (wv == P0 % WK) {
          acc[P0 / WK] = rbf_tile<NB, FULL>(smem, rk, 0, 0, lane, N);
          publish_tile(dsc, lane, acc[P0 / WK], vflag, kFlagT00, e0);
        }
        if constexpr (NB > 1) {
          if (wv == T01 % WK) {
            acc[T01 / WK] = rbf_tile<NB, FULL>(smem, rk, 0, 1, lane, N);
            GPK_EP(epoch_mark(vflag, kShadowHo, e0, lane);)
            publish_tile(hbuf, lane, acc[T01 / WK], vflag, kFlagHA + 0, e0);
          }
          if (wv == P1 % WK) {
            acc[P1 / WK] = rbf_tile<NB, FULL>(smem, rk, 1, 1, lane, N);
            GPK_EP(epoch_mark(vflag, kShadowHo + 1, e0, lane);)
            publish_tile(hbuf + 256, lane, acc[P1 / WK], vflag, kFlagHB + 0, e0);
          }
        }
        static_for_desc<SLOTS>([&](auto I) {
          constexpr int s = decltype(I)::value;
          const int t = wv + WK * s;
          if (t < NT) {
            bool sk = false;
            if constexpr (s == P0 / WK) sk = sk || (wv == P0 % WK);
            if constexpr (NB > 1 && s == T01 / WK) sk = sk || (wv == T01 % WK);
            if constexpr (NB > 1 && s == P1 / WK) sk = sk || (wv == P1 % WK);
            if (!sk) {
              if (t >= P2) {
                const int pk = plan_tile<NB, WK * s, WK * s + WK - 1>(t);
                acc[s] = rbf_tile<NB, FULL>(smem, rk, pk & 255, pk >> 8, lane, N);
              } else {
                acc[s] = f32x4{0.f, 0.f, 0.f, 0.f};
              }
            }
          }
        });
        }
      }
      GPK_STAMP(1)
      wx.epoch0 = 32 * attempt;
      wx.sumz2 = 0.f;
      if constexpr (STAMPS) {
        wx.st = wst;
        wst[8] = st_last;
      }
      failed = worker_steps<NB, WK, SLOTS, 0, STAMPS, FULL, COL>(acc, wx);
      if constexpr (STAMPS) st_last = wst[8];
      sumz2 = wx.sumz2;
      if (!failed) { info_w = attempt > 0 ? -attempt : 0; break; }
      // every worker has left the failed attempt before anyone rebuilds; the per-attempt
      // counters restart from 0 between the two restart barriers
      restart_sync<WK>(wx, 2 * attempt + 1);
      if (wave == 0 && lane == 0) {
        vflag[kFlagSync] = 0;
        vflag[kFlagTrsm] = 0;
        vflag[kFlagBulk] = 0;
      }
      wx.nsync = 0;
      restart_sync<WK>(wx, 2 * attempt + 2);
    }
    if (GPK_TMO_DEBUG && wave == 0 && lane == 0) vflag[23] = att_end;
    if constexpr (STAMPS) {
      for (int q = 2; q < 8; ++q) st_acc[q] += wst[q];
    }
  }
  // ---- 5. reduce logdet / |z|^2 over waves, write the MLL ---------------
  const float ld_wave = wave_sum(logdet) * 0.69314718055994531f;  // v_log_f32 is log2
  if (lane == 0) red[wave] = ld_wave;
  const float z2 = wave_sum(sumz2);
  if (lane == 0) red[W + wave] = z2;
  barrier_lds();
  if (tid == 0) {
    const int fcol = vflag[kFlagFail + att_end];
    if (vflag[kFlagTmo] != 0) {
      info[b] = GPK_TMO_DEBUG ? ((1 << 30) | ((int)vflag[23] << 26) | ((int)vflag[24] << 22) |
                                 (((int)vflag[kFlagSync] & 0x3f) << 16) | ((int)vflag[kFlagTmo + 1] & 0xffff))
                              : kInfoTimeout;
      mll[b] = __builtin_nanf("");
    } else if (fcol != 0) {
      info[b] = fcol;
      mll[b] = __builtin_nanf("");
    } else {
      float ld = 0.f, zz = 0.f;
      for (int w = 0; w < W; ++w) { ld += red[w]; zz += red[W + w]; }
      ld -= (float)(2 * sh) * (float)N * 0.69314718055994531f;  // - N log sigma^2
      mll[b] = -0.5f * (zz + ld + (float)N * kLog2Pi) / (float)N;
      info[b] = info_w;
    }
  }
  if constexpr (STAMPS) {
    if (tid == 0) {
      unsigned long long* o = stamps + (size_t)b * kStampStride;
      for (int q = 0; q < 8; ++q) o[q] = q < 2 ? st_acc[q] : 0;
      for (int q = 2; q < 8; ++q) o[16 + q] = st_acc[q];
      for (int q = 8; q < 12; ++q) o[16 + q] = st_acc[q];
      o[13] = ((unsigned long long*)(red + 4 * W + 24))[0];
      o[14] = ((unsigned long long*)(red + 4 * W + 26))[0];
      o[15] = ((unsigned long long*)(red + 4 * W + 28))[0];
      for (int q = 0; q < 3; ++q) o[2 + q] = ((unsigned long long*)(red + 4 * W + 32))[q];
      o[10] = (unsigned)flag[16];
      o[11] = __builtin_amdgcn_s_getreg(4 | (31 << 11));
      o[12] = (unsigned)flag[17];
      o[8] = __builtin_amdgcn_s_memtime() - st_t0;
      o[9] = __builtin_amdgcn_s_memrealtime() - st_rt0;
    }
  }
}

template <int NB, int W, bool STAMPS, bool FULL, int OCC>
int launch_exact_w(const GpkExactArgs& a, unsigned long long* stamps, hipStream_t stream) {
  const int DC = (a.D + 15) / 16;
  const ExactLds lay = exact_lds_layout(NB, DC, W);
  const size_t lds = (size_t)lay.total * sizeof(float);
  if (DC * 16 > 64 * W || DC * 16 > 256) return -7;
  if (lds > 160 * 1024) return -7;
  if (lds > 64 * 1024)
    (void)hipFuncSetAttribute((const void*)gpk_exact_kernel<NB, W, STAMPS, FULL, OCC>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  hipLaunchKernelGGL((gpk_exact_kernel<NB, W, STAMPS, FULL, OCC>), dim3(a.B), dim3(64 * W), lds, stream,
                     a.X, a.y, a.hyp, a.n_ls, a.N, a.D, DC, a.jitter, a.max_tries,
                     a.L, a.z, a.mll, a.info, stamps);
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? 0 : (int)e;
}

// Compute units of the current device (for the small-batch layout choice).
int device_cus() {
  int dev = 0, n = 0;
  if (hipGetDevice(&dev) != hipSuccess) return 256;
  if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) return 256;
  return n;
}

template <int NB, bool STAMPS, bool FULL>
int launch_exact_nb(const GpkExactArgs& a, unsigned long long* stamps, hipStream_t stream) {
  constexpr int W = NB >= 12 ? GPK_EXACT_WBIG : (NB >= 6 ? 8 : 4);
#if GPK_EXACT_SMALLB
  // Small batches (B <= CUs: BASELINE configs[1], the strong-scaled per-GPU share of
  // configs[3]): a window's latency IS the launch time, and half the CUs would idle at
  // two windows per CU; one window per CU with 16 waves gives each window 15 workers.
  if constexpr (!STAMPS && NB >= 6) {
    if (a.B <= device_cus()) return launch_exact_w<NB, 16, STAMPS, FULL, 1>(a, stamps, stream);
  }
#endif
  return launch_exact_w<NB, W, STAMPS, FULL, 2>(a, stamps, stream);
}

template <int NB>
int launch_exact_any(const GpkExactArgs& a, hipStream_t stream) {
  return (a.N == 16 * NB) ? launch_exact_nb<NB, false, true>(a, nullptr, stream)
                          : launch_exact_nb<NB, false, false>(a, nullptr, stream);
}

}  // namespace

int gpk_launch_exact_stamps(const GpkExactArgs& a, unsigned long long* stamps, hipStream_t stream) {
  if (a.N != 256) return -6;
  return launch_exact_nb<16, true, true>(a, stamps, stream);
}

int gpk_launch_exact(const GpkExactArgs& a, hipStream_t stream) {
  const int NB = (a.N + 15) / 16;
  switch (NB) {
#define GPK_CASE(nb) case nb: return launch_exact_any<nb>(a, stream);
#if GPK_EXACT_DEV  // development A/B builds: the N=128 / N=256 instantiations only (fast compile)
    GPK_CASE(8) GPK_CASE(16)
#else
    GPK_CASE(1) GPK_CASE(2) GPK_CASE(3) GPK_CASE(4) GPK_CASE(5) GPK_CASE(6)
    GPK_CASE(7) GPK_CASE(8) GPK_CASE(9) GPK_CASE(10) GPK_CASE(11) GPK_CASE(12)
    GPK_CASE(13) GPK_CASE(14) GPK_CASE(15) GPK_CASE(16)
#endif
#undef GPK_CASE
    default: return -6;
  }
}
