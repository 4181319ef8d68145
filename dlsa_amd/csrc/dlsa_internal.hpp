// Internal declarations shared by the HIP translation units of libdlsa_hip.so.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <string>

#include "../../include/dlsa_hip.h"

namespace dlsa {

// Per-partition Newton phase.  MIXED fits start in PHASE_F32 (approximate
// Hessian at the fit's approximate precision: bf16 MFMA in MIXED, fp32 in
// MIXED_F32; fp64 gradient) and switch to PHASE_F64 for the pass whose
// Hessian is returned as Sig_inv; FP64 fits start in PHASE_F64.  A partition
// whose bf16-steered Newton stalls (or whose bf16 Hessian is not positive
// definite) escalates to PHASE_F32X (fp32-MFMA Hessian), then to PHASE_F64.
// PHASE_LEVEL_DONE: finished the current warm-start subsample level.
// counters[PHASE_F32 .. PHASE_F32X] count the partitions running per phase.
enum : int32_t {
  PHASE_F32 = 0,
  PHASE_F64 = 1,
  PHASE_F32X = 2,
  PHASE_DONE = 3,
  PHASE_LEVEL_DONE = 4,
  // host-set for one launch only: a PHASE_F64 partition whose max |z| record
  // is stale, routed to the fp64-MFMA exact pass beside an int8 pass of the
  // fresh ones (capi.hip fused_pass); restored to PHASE_F64 before the solve
  PHASE_F64_STALE = 5
};
constexpr int kRunPhases = 3;
enum : int32_t { STATUS_RUNNING = -1 };
enum : int32_t { FAMILY_LOGISTIC = 0, FAMILY_GAUSSIAN = 1 };

// Cache policy of the LDS-DMA loads that stream X (the aux / cpol operand of
// buffer_load ... lds; profiling builds override it, tools/build_variants.sh).
// The cooperative and per-wave passes keep the default policy: with nt (2)
// the lines their consecutive blocks share are fetched twice (PMC, run r04g:
// 842.6 vs 812.4 B/row for the config-2 bf16 pass, 624 vs 523 B/row for the
// config-4 OLS pass, whose blocks are 8 rows); the Ozaki exact pass streams
// non-temporally (813.6 vs 812.4 B/row, 17.6-18.0 vs 17.9-18.1 ms at config
// 2 in two A/B runs, profiles/r04g_dma_policy_ab.txt).
#ifndef DLSA_X_DMA_AUX
#define DLSA_X_DMA_AUX 0
#endif
#ifndef DLSA_OZ_DMA_AUX
#define DLSA_OZ_DMA_AUX 2
#endif
// Cooperative pass: 4 (8) waves per workgroup, 32-row blocks.
constexpr int kCoopRows = 32;
// MFMA arithmetic of a pass's Hessian.
enum : int32_t { PREC_BF16 = 0, PREC_F32 = 1, PREC_F64 = 2 };

// Arguments of the fused IRLS pass (one workgroup = one chunk of one partition).
struct PassArgs {
  const double* X;            // [n_total, p]
  const double* y;            // [n_total]
  const int64_t* chunk_row0;  // [n_chunks] first global row of the chunk
  const int32_t* chunk_rows;  // [n_chunks]
  const int32_t* chunk_part;  // [n_chunks]
  const int32_t* phase;       // [K]
  const double* theta;        // [K, P] current iterate
  const double* center;       // [p] or null
  const double* scale;        // [p] or null
  double* slab_H;             // [n_chunks, T, 16, 16] partial X^T W X tiles
  double* slab_g;             // [n_chunks, 16*NT] partial X^T (y - mu)
  double* slab_ll;            // [n_chunks] partial log-likelihood
  uintptr_t x_last16;         // last 16-B aligned address whose 16 B are readable
  uintptr_t y_last4;          // last 4-B address inside y
  int32_t p;                  // columns of X
  int32_t P;                  // p + intercept
  int32_t intercept;
  int32_t want_phase;
  int32_t nslot;              // cooperative pass: LDS ring depth (32-row slots)
  int32_t slot_bytes;
  // Digit scales of the Ozaki exact pass (irls_oz_impl.hpp), written by the
  // bf16 passes of the final level when set:
  //   colmax  [n_chunks, 16*NT] per chunk and feature max |x| (the fp64 high
  //           dword, after standardisation)
  //   zcolmax [n_chunks, 16*NT] max |z|, z = sqrt(w) x at the pass's theta
  //           (fp32 bits)
  //   theta_rec [K, P] the theta of the partition's last recording pass
  uint32_t* colmax;
  uint32_t* zcolmax;
  const double* theta_rec;
  // null, or zcolmax is written only if zrec_gate[0] > 0: the near-switch
  // count of the solve before, for a pass enqueued before the host read it
  const int32_t* zrec_gate;
  int32_t waves;  // fp64 per-wave pass geometry (dlsa_fit_options.exact_waves; 0 = auto)
};

// A/B knobs of profiling builds.  The product library reads no environment
// variable that changes a result (include/dlsa_hip.h): env_knob() is getenv
// only in builds compiled with -DDLSA_ENV_KNOBS=1 (tools/build_variants.sh).
#ifndef DLSA_ENV_KNOBS
#define DLSA_ENV_KNOBS 0
#endif
inline const char* env_knob(const char* name) {
#if DLSA_ENV_KNOBS
  return getenv(name);
#else
  (void)name;
  return nullptr;
#endif
}

// Arguments of the per-partition Newton update.
struct SolveArgs {
  const int32_t* part_chunk_begin;  // [K+1]
  const double* slab_H;
  const double* slab_g;
  const double* slab_ll;
  double* theta;        // [K, P] (in/out: the iterate, returned as coef)
  double* theta_prev;   // [K, P]
  double* delta_prev;   // [K, P]
  double* ll_prev;      // [K]
  int32_t* phase;       // [K]
  int32_t* backtracks;  // [K]
  int32_t* iters;       // [K]
  int32_t* status;      // [K]
  int32_t* counters;    // [4]: [kRunPhases] partitions still running per phase, [3] of the
                        // PHASE_F32 ones, those whose step was <= kOzNearTol (1 + max|theta|)
  double* dm_prev;      // [K] max |step| of the last approximate iteration (0: none)
  int32_t* stall;       // [K] consecutive stalled approximate iterations
  double* sig_inv;      // [K, P, P] out
  double* loglik;       // [K] out
  int32_t P;
  int32_t NT;
  int32_t family;  // FAMILY_LOGISTIC: Newton to tol; FAMILY_GAUSSIAN: one exact step
  int32_t subsample;  // 1 on a warm-start level (row prefix of each partition)
  double tol;
  double switch_tol;
  double level_tol;   // warm-start level: stop when max|step| <= level_tol (1+max|theta|)
  int32_t escalate_to;  // next phase of a stalled PHASE_F32 partition (PHASE_F32X / PHASE_F64)
  int32_t eval_only;    // polish: publish Sig_inv / loglik at the current theta, no step
};

// Stall detection of the approximate phases (newton_solve.hip,
// wide_pass.hip).  With an approximate Hessian H~ and the exact gradient,
// Newton contracts at rate ~ ||I - H~^-1 H|| (about kappa 2^-8 for bf16): on
// an ill-conditioned design that rate nears 1 and the fit would crawl to
// max_iter.  Far from the MLE (Newton's damped phase) steps of similar size
// are normal whatever the Hessian precision, so evidence is only taken once
// the log-likelihood has gone quiet (the last step gained at most
// kStallDll (1 + |ll|)): there an approximate iteration "stalls" when its max
// |step| did not at least halve against the previous one, or when it
// backtracks; two stalls in a row move the partition one precision up
// (F32 -> escalate_to, F32X -> F64).  Returns the phase to continue in.
constexpr double kStallDll = 1e-5;
// An approximate iteration whose max |step| is below kOzNearTol (1 + max|theta|)
// is one or two iterations from the exact pass: the next bf16 pass records
// max |sqrt(w) x| for the Ozaki digit scales (capi.hip, irls_oz_impl.hpp)
constexpr double kOzNearTol = 1e-2;
__device__ __forceinline__ int32_t escalate_phase(const SolveArgs& a, int32_t ph) {
  return ph == PHASE_F32 ? a.escalate_to : PHASE_F64;
}
__device__ __forceinline__ int32_t approx_stall_step(const SolveArgs& a, int k, int32_t ph,
                                                     bool stalled) {
  const int st = stalled ? a.stall[k] + 1 : 0;
  if (st >= 2) {
    a.stall[k] = 0;
    a.dm_prev[k] = 0.0;
    return escalate_phase(a, ph);
  }
  a.stall[k] = st;
  return ph;
}
// Approximate-phase iteration with a step of max |d| = dm (not yet below
// switch_tol): log-likelihood ll at the pass's point, llp at the previous one.
__device__ __forceinline__ int32_t approx_next_phase(const SolveArgs& a, int k, int32_t ph,
                                                     double dm, double ll, double llp) {
  if (!(ll - llp <= kStallDll * (1.0 + fabs(ll)))) {  // damped phase (or first iteration)
    a.stall[k] = 0;
    a.dm_prev[k] = 0.0;
    return ph;
  }
  const double dp = a.dm_prev[k];
  const int32_t nph = approx_stall_step(a, k, ph, dp > 0.0 && dm > 0.5 * dp);
  if (nph == ph) a.dm_prev[k] = dm;
  return nph;
}
// A backtracking approximate iteration: a stall only once the fit was quiet.
__device__ __forceinline__ int32_t approx_backtrack_phase(const SolveArgs& a, int k, int32_t ph) {
  return a.dm_prev[k] > 0.0 ? approx_stall_step(a, k, ph, true) : ph;
}

// Arguments of the log-likelihood evaluation pass.
struct EvalArgs {
  const double* X;
  const double* y;
  const int64_t* chunk_row0;
  const int32_t* chunk_rows;
  const int32_t* chunk_part;
  const double* center;  // [p] or null
  const double* scale;
  const double* betas;   // [nbeta, P]
  double* partial;       // [n_chunks, nbeta]
  uintptr_t x_last16;
  uintptr_t y_last4;
  int32_t p, P, intercept, nbeta;
  int32_t nslot, slot_bytes;
};

// Wide-P path (DLSA_MAX_P_FUSED < P <= DLSA_MAX_P, wide_pass.hip): a row
// pass (eta, weights, gradient, log-lik) and a separate Gram pass over
// 128x128 output tiles of the padded PP = 128 * NB Hessian.
constexpr int kWideTile = 128;
struct WideArgs {
  const double* X;
  const double* y;
  const int64_t* rc_row0;  // row-pass chunks
  const int32_t* rc_rows;
  const int32_t* rc_part;
  const int64_t* gc_row0;  // Gram-pass row groups
  const int32_t* gc_rows;
  const int32_t* gc_part;
  const int32_t* phase;    // [K]
  const double* theta;     // [K, P]
  const double* center;    // [p] or null
  const double* scale;
  double* w;               // [n_total] IRLS weight of each row (row pass -> Gram pass)
  double* slab_g;          // [n_rchunks, PP] partial gradients
  double* slab_ll;         // [n_rchunks] partial log-likelihoods
  double* slab_G;          // [n_gchunks, TB, 128 * 128] partial Gram tiles
  double* slab_gz;         // [n_gchunks, PP] fused pass: partial gradients
  double* slab_llz;        // [n_gchunks] fused pass: partial log-likelihoods
  int32_t p, P, intercept;
  int32_t NB;              // 128-wide column blocks, PP = 128 NB
  int32_t n_gchunks;
  // int8 exact Gram (wide_oz.hip): the row pass's per-chunk max |sqrt(w) x|
  // (high dwords, [n_rchunks, PP]) when set
  uint32_t* slab_zmax;
};

// int8 exact Gram of the wide path (wide_oz.hip)
struct WideOzArgs {
  const int32_t* rcb;      // [K+1] row-pass chunks of each partition
  const uint32_t* zmax;    // [n_rchunks, PP] the row pass's max |sqrt(w) x| high dwords
  int32_t* E;              // [n_gchunks, PP] digit exponents of each Gram row group
  // digit records, part of the fit's workspace (WideLayout::off_digits):
  // [n_gchunks][maxblk][4 rowblocks][slice 0: PP x 16 B | slice 1: PP x 16 B |
  // slice 2: PP x 8 B] -- kWideOzRec bytes per (8 rows, feature)
  int8_t* D;
  int32_t maxblk;          // 32-row blocks of the largest Gram row group
};
hipError_t launch_wide_oz_scale(const WideArgs& a, const WideOzArgs& o, hipStream_t s);
hipError_t launch_wide_oz_digits(const WideArgs& a, const WideOzArgs& o, bool standardize,
                                 hipStream_t s);
hipError_t launch_wide_oz_gram(const WideArgs& a, const WideOzArgs& o, hipStream_t s);
constexpr int kWideOzMaxRows = 32767;  // int32 level sums of one row group
constexpr int kWideOzRec = 40;         // digit bytes per (8 rows, feature): 5 planes
// bytes of the digit records of a Gram plan with n_gchunks row groups of at
// most max_rows rows and PP padded features
inline int64_t wide_oz_digit_bytes(int n_gchunks, int max_rows, int PP) {
  const int64_t maxblk = (max_rows + 31) / 32;
  return (int64_t)(n_gchunks > 1 ? n_gchunks : 1) * maxblk * 4 * PP * kWideOzRec;
}

// Categorical-code pass (cat_pass.hip): q numeric fp64 columns + F uint8
// level codes per row; the one-hot blocks of X^T W X are LDS histograms.
constexpr int kCatMaxFactors = 16;
constexpr int kCatMaxPairs = kCatMaxFactors * (kCatMaxFactors - 1) / 2;
constexpr int kCatPMax = 192;  // P <= DLSA_MAX_P_FUSED (the Newton solve's limit)
constexpr int kCatQMax = 16;   // intercept + numeric columns
struct CatArgs {
  const double* Xn;           // [n_total, q] numeric columns
  const uint8_t* codes;       // [n_total, F] level codes (0 = baseline: no column)
  const double* y;            // [n_total]
  const int64_t* chunk_row0;
  const int32_t* chunk_rows;
  const int32_t* chunk_part;
  const int32_t* phase;
  const double* theta;        // [K, P]
  const double* center;       // [q] or null
  const double* scale;
  double* slab_H;             // same partial slab layout as PassArgs
  double* slab_g;
  double* slab_ll;
  int32_t q, F, P, intercept, NT, want_phase;
  int32_t hist_doubles;       // LDS histogram doubles
  int32_t nd_stride;          // 8-byte words per (replica, level) row of an nd histogram: q + 1
                              // rounded up to odd (the lanes' rows then fall on distinct banks)
  int32_t nlev[kCatMaxFactors];    // dummy columns of factor f (L_f - 1)
  int32_t nd_lev[kCatMaxFactors];  // level slots per replica of f's nd / gradient histograms:
                                   // nlev, + 1 for the fold factor (its baseline level)
  int32_t fold;                    // the exact-bucket kernel's fold factor, else -1: its
                                   // histograms also take the baseline level, so the
                                   // intercept row of X^T W X and gradient are the sums of
                                   // its levels (no register accumulators for them)
  int32_t doff[kCatMaxFactors];    // parameter index of factor f's first dummy
  int32_t nd_off[kCatMaxFactors];  // LDS: [rep][level slot][q + 1] (w, w x_0 ..; cat_slot)
  int32_t nd_rep[kCatMaxFactors];  // replicas (power of two)
  int32_t g_off[kCatMaxFactors];   // LDS: [rep][level slot] gradient
  int32_t pr_off[kCatMaxPairs];    // LDS: pair (f < g) [rep][nlev_f][nlev_g]
  int32_t pr_rep[kCatMaxPairs];
  // fixed-point scales of the int64 histograms per partition, device
  // [K][kCatQMax + 2] (powers of two: [0] w and the pair cells, [1] the
  // gradient residuals, [2 + i] w x_i of numeric column i)
  const double* hscale;
};

// Row repartitioning (partition_rows.hip): stable counting sort by partition id.
constexpr int kPartMaxArrays = 4;
constexpr int kPartMaxK = 16000;    // LDS histogram / cursors
constexpr int kPartSubRows = 4096;  // rows ranked per scatter sub-block
hipError_t launch_partition_rows(const int32_t* pid, int64_t n, int K, int64_t rows_per_block,
                                 int nb, int32_t* counts, int32_t* bad, int64_t* totals,
                                 int64_t* offsets_dev, hipStream_t s);
hipError_t launch_partition_scatter(const int32_t* pid, int64_t n, int K, int64_t rows_per_block,
                                    int nb, const int32_t* base, const int64_t* offsets_dev,
                                    const void* const* src, void* const* dst,
                                    const int64_t* row_bytes, int n_arrays, int64_t* order,
                                    hipStream_t s);

// Launchers (defined in the .hip files).
hipError_t launch_cat_pass(const CatArgs& a, bool standardize, int n_chunks, hipStream_t s);
size_t cat_lds_bytes(const CatArgs& a);  // dynamic LDS of the pass
bool cat_exact_bucket(const CatArgs& a);  // the pass's exact-bucket kernel applies (fold factor)
constexpr int kCatStaticLds =  // its tables: factor and pair records, dummy offsets
    16 * (kCatMaxFactors + 1) + 16 * (kCatMaxPairs + 1) + 4 * kCatMaxFactors;
hipError_t launch_cat_presence(const CatArgs& a, int n_chunks, int32_t* counts, int32_t* bad,
                               double* colmax,
                               hipStream_t s);
hipError_t launch_cat_mark(const CatArgs& a, const int32_t* pcb, const int32_t* counts,
                           const int32_t* bad, int K, int32_t* phase, int32_t* status,
                           int32_t* bad_part, hipStream_t s);
hipError_t launch_wide_row(const WideArgs& a, bool standardize, int family, int n_chunks,
                           hipStream_t s);
hipError_t launch_wide_gram(const WideArgs& a, bool standardize, hipStream_t s);
hipError_t launch_wide_fused(const WideArgs& a, bool standardize, hipStream_t s);
hipError_t launch_wide_assemble(const WideArgs& a, const int32_t* gcb, double* Hfull, int K,
                                hipStream_t s);
hipError_t launch_wide_newton(const SolveArgs& sa, const WideArgs& wa, const int32_t* rcb,
                              const int32_t* gcb, double* Hfull, int K, hipStream_t s);
int wide_newton_lds_bytes(int NB);
hipError_t launch_loglik_eval(const EvalArgs& a, int n_chunks, hipStream_t s);
hipError_t launch_loglik_reduce(const double* partial, const int32_t* pcb, int K, int B,
                                double* out, hipStream_t s);
int eval_slot_bytes(int p);
// per-wave fp64 pass (irls_wave_impl.hpp): P <= 128
hipError_t launch_irls_wave(const PassArgs& a, int NT, bool standardize, int family, int n_chunks,
                            hipStream_t s);
int wave_lds_bytes(int NT, int p);
constexpr int kWaveMaxNT = 8;
// Ozaki-scheme exact pass (irls_oz_impl.hpp): NT <= kOzMaxNT, chunks <= kOzMaxRows rows;
// a.nslot = oz_nslot(NT, p) ring slots
hipError_t launch_irls_oz(const PassArgs& a, int NT, bool standardize, int family, int n_chunks,
                          hipStream_t s);
bool oz_applies(int NT, int p);  // NT <= kOzMaxNT, image and 6-slot ring fit
constexpr int kOzMaxRows = 32767;
constexpr int kOzMaxNT = 7;
// OLS pass at theta = 0 streaming X into the MFMA operand registers
// (ols_stream.hip), P <= 64
bool ols_stream_applies(int NT);
hipError_t launch_ols_stream(const PassArgs& a, int NT, bool standardize, int n_chunks,
                             hipStream_t s);
hipError_t launch_irls_coop(const PassArgs& a, int NT, int prec, bool standardize, int family,
                            int n_chunks, hipStream_t s);
int coop_slot_bytes(int NT, int p);
int coop_extra_bytes(int NT);  // LDS beyond the ring
hipError_t launch_newton_solve(const SolveArgs& a, int K, hipStream_t s);
hipError_t launch_fit_init(const int64_t* offsets_dev, int K, int P, int start_phase,
                           double* theta, int32_t* phase, int32_t* backtracks,
                           int32_t* iters, int32_t* status, double* ll_prev,
                           double* sig_inv, double* loglik, hipStream_t s);
hipError_t launch_level_reset(int K, int P, int start_phase, int32_t* phase, int32_t* status,
                              double* ll_prev, int32_t* backtracks, double* theta,
                              int32_t* counters, hipStream_t s);
hipError_t launch_polish_mark(int K, int32_t* phase, const int32_t* status, int32_t* counters,
                              hipStream_t s);
// theta_rec[k] = theta[k] for the partitions in phase `ph` (before a pass
// that records the Ozaki digit scales)
hipError_t launch_theta_snapshot(int K, int P, const int32_t* phase, int ph, const double* theta,
                                 double* theta_rec, hipStream_t s, const int32_t* gate = nullptr);
hipError_t launch_fit_finalize(int K, int P, const double* theta, const double* sig_inv,
                               double* sig_inv_theta, int32_t* status, hipStream_t s);
hipError_t launch_reduce_partitions(const double* sig_inv, const double* sig_inv_theta,
                                    const double* theta, int K, int P, double* out,
                                    hipStream_t s);
hipError_t launch_simulate(double* X, double* y, int64_t n, int p, uint64_t seed,
                           int64_t row0, hipStream_t s);

// Column moments (moments.hip): out [5, p] = count, mean, M2, min, max; ws
// holds (5 G + 5) p doubles.
hipError_t launch_column_moments(const double* X, int64_t n, int p, double* out, double* ws,
                                 int G, int64_t rows_per_range, hipStream_t s);
void column_moments_plan(int64_t n, int p, int* G, int64_t* rows_per_range);

void set_error(const std::string& msg);

// Raise a kernel's dynamic-LDS limit to `bytes` once per (kernel, device):
// thread-safe (one process may drive several GPUs from several threads).
hipError_t ensure_max_lds(const void* kernel, int bytes);

}  // namespace dlsa
