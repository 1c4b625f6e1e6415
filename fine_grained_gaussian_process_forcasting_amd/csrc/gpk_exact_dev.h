// Build switches and development-only instrumentation of the exact kernel (gpk_exact.hip).
//
// Product builds (build_native.py) define none of these macros: every switch below defaults
// to the shipped, measured setting; the knockouts compile to `false`; the stamp macros only
// expand inside kernels instantiated with STAMPS = true (the gpk_debug_exact_stamps entry,
// scripts/r05/stamps_col.py). A/B builds: scripts/ab_build_one.sh <name> gpk_exact.hip -DNAME=v.
#pragma once

// ---- design switches: the defaults are the measured winners ----
#ifndef GPK_EXACT_WBIG
#define GPK_EXACT_WBIG 8
#endif
#ifndef GPK_SPLIT_UPDATE
#define GPK_SPLIT_UPDATE 1
#endif
#ifndef GPK_EXACT_SMALLB
#define GPK_EXACT_SMALLB 1   // B <= CUs: one window per CU with 16 waves (launch_exact_nb)
#endif
#ifndef GPK_EXACT_DIAG_ALONE
#define GPK_EXACT_DIAG_ALONE 1   // 1: small-batch layout (NB <= 8) with the diagonal wave alone on its SIMD
                                 // (12 workers; 0: 15 workers, the round-5 layout)
#endif
#ifndef GPK_EXACT_PRIO_RHS
#define GPK_EXACT_PRIO_RHS 1   // raise the worker priority already at the right-hand side (0: at the TRSM)
#endif
#ifndef GPK_EXACT_PRIO
#define GPK_EXACT_PRIO 1   // workers raise their issue priority to this for the hand-over and the TRSM
                           // (0: off; 1 measured 2.5 % faster per launch, scripts/gpu_ab_prio.sh)
#endif
#ifndef GPK_DIAG_DPP
#define GPK_DIAG_DPP 1   // diagonal sweep as DPP-broadcast FMAs (gpk_diag_dpp.inc); 0 = readlane form
#endif
#ifndef GPK_DIAG_PERMLANE
#define GPK_DIAG_PERMLANE 0   // 1: the diagonal wave gathers its sweep operand by permlane swaps from the
                              // look-ahead's registers (measured 0.6-0.8 us SLOWER per launch at B = 64 / 128);
                              // 0: through its LDS tile
#endif
#ifndef GPK_DIAG_FINISH_LATE
#define GPK_DIAG_FINISH_LATE 0   // 1: step k's L block + log|T| after the look-ahead MFMAs (measured
                                 // slower: the in-order wave puts them on the chain); 0: before the wait
#endif
#ifndef GPK_EXACT_COL
#define GPK_EXACT_COL 1   // 1: column-ownership worker plan for N = 256 at 8 waves (worker_step_col)
#endif
#ifndef GPK_LST_AUX
#define GPK_LST_AUX 17   // L stores: -1 plain global stores; >= 0 buffer stores with this cache-policy aux
                         // (17 = sc0 sc1: write-through, the lines leave L2 -- 64.5 -> 59.2 us per B=512 launch)
#endif

// ---- development only ----
#ifndef GPK_EXACT_DEV
#define GPK_EXACT_DEV 0   // 1: only the N = 128 / 256 instantiations (fast A/B compiles)
#endif
#ifndef GPK_TMO_DEBUG
#define GPK_TMO_DEBUG 0   // 1 (debug builds): a timed-out window's info = flag index | target << 8
#endif
#ifndef GPK_EPOCH_CHECK
#define GPK_EPOCH_CHECK 0   // 1 (check builds): every consumed panel / hand-over / R_kk^{-T} tile is checked
                            // against the epoch its consumer expects (epoch shadows in LDS, written by the
                            // producer before its flag release); a mismatch ends the window with
                            // info = 1<<20 and the site in flag word kFlagEpochBad. 2: the same plus a
                            // deliberate wrong mark (the check's own negative control).
#endif
constexpr bool kEpochCheck = GPK_EPOCH_CHECK != 0;
#if GPK_EPOCH_CHECK
#define GPK_EP(...) __VA_ARGS__
#else
#define GPK_EP(...)
#endif
constexpr bool kEpochSabotage = GPK_EPOCH_CHECK == 2;
#ifndef GPK_KO
#define GPK_KO 0   // knockout bits (timing only, results WRONG): see the constants below
#endif
constexpr bool kKoTrsmMfma = (GPK_KO & 1) != 0;       // TRSM MFMAs
constexpr bool kKoRhs = (GPK_KO & 2) != 0;            // right-hand side
constexpr bool kKoZeroL = (GPK_KO & 4) != 0;          // upper-L zeroing
constexpr bool kKoDeferredRbf = (GPK_KO & 8) != 0;    // deferred RBF of block row k + 2
constexpr bool kKoBulkUpdate = (GPK_KO & 16) != 0;    // bulk trailing update
constexpr bool kKoTrsmLStores = (GPK_KO & 32) != 0;   // TRSM L stores
constexpr bool kKoDiagSweep = (GPK_KO & 64) != 0;     // diagonal sweep
constexpr bool kKoOneOperand = (GPK_KO & 128) != 0;   // one LDS operand per tile update
constexpr bool kKoAny = GPK_KO != 0;                  // (disables the failure checks too)

// ---- stamp builds (STAMPS = true instantiations only) ----
constexpr int kStampStride = 32 + 16 * 8 * 8;  // phase clocks + per-step timeline

// Diagnostic phase clock inside the worker steps (STAMPS builds only).
#define GPK_WSTAMP(slot, ev)                                      \
  if constexpr (ST) {                                             \
    __builtin_amdgcn_sched_barrier(0);                            \
    const unsigned long long _n = __builtin_amdgcn_s_memtime();   \
    x.st[slot] += _n - x.st[8];                                   \
    x.st[8] = _n;                                                 \
    if (x.lane == 0) x.tl[(K * 8 + x.wv) * 8 + (ev)] = _n;        \
    __builtin_amdgcn_sched_barrier(0);                            \
  }

// Phase clock of the kernel body (wave 0 lane 0 of each workgroup).
#define GPK_STAMP(slot)                                           \
  if constexpr (STAMPS) {                                         \
    __builtin_amdgcn_sched_barrier(0);                            \
    const unsigned long long _n = __builtin_amdgcn_s_memtime();   \
    st_acc[slot] += _n - st_last;                                 \
    st_last = _n;                                                 \
    __builtin_amdgcn_sched_barrier(0);                            \
  }
