/*
 * dlsa_hip.h -- C-ABI of libdlsa_hip.so, the MI355X (gfx950) DLSA estimator.
 *
 * This is the drop-in boundary for the reference's map/combine/select path
 * (Vicky-Lamperouge/dlsa).  The reference has no FFI: its map stage is a
 * Spark GROUPED_MAP pandas_udf around dlsa/models.py:logistic_model, its
 * combine is dlsa/dlsa.py:dlsa_mapred and its selection step is
 * dlsa/lsa.py:lars_lsa (or R lars.lsa via rpy2, dlsa/dlsa.py:64-81).  Each
 * entry point below names the reference interface it replaces.  The Python
 * binding (ctypes) lives in dlsa_amd/_hip.py; INTEGRATION.md shows the stub a
 * maintainer would add on the reference side.
 *
 * Conventions
 *   - Plain C types only.  Pointers named X/y/theta/... are DEVICE pointers
 *     (hipMalloc'd or torch tensor data_ptr()), except where "host" is noted.
 *   - The caller owns every buffer.  Scratch comes from the caller's
 *     workspace (dlsa_fit_options.workspace) or, when that is NULL, is
 *     hipMallocAsync'd on the stream and freed before return.
 *   - Work is enqueued on the caller's hipStream_t (`stream`, NULL = default
 *     stream).  dlsa_logistic_fit_batched* reads a 16-byte device counter
 *     back once per Newton iteration (a stream synchronisation); the other
 *     device entry points are fully asynchronous.
 *   - Return 0 on success, a negative DLSA_E_* code on failure; the message
 *     is in dlsa_last_error() (thread-local).
 *   - Row-major fp64.  Partition k owns rows offsets[k] .. offsets[k+1]-1 of X
 *     (partitions contiguous: the layout Spark's repartition(K,
 *     "partition_id") + groupby produce per task, projects/logistic_dlsa.py:
 *     303-325).  X must be readable up to the next 16-byte boundary past its
 *     last element (true for any torch/hipMalloc allocation that starts at
 *     the tensor).
 *   - P = p + fit_intercept is the parameter count; with an intercept the
 *     intercept is parameter 0 (dlsa/models.py:116-122).
 */
#ifndef DLSA_HIP_H
#define DLSA_HIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* error codes */
#define DLSA_OK 0
#define DLSA_E_INVALID (-1)
#define DLSA_E_HIP (-2)
#define DLSA_E_UNSUPPORTED (-3)
#define DLSA_E_WORKSPACE (-4)

/* per-partition status (status[] output) -- SURVEY.md section 5: the
 * reference only warns (models.py:84-91,144-145); here every partition
 * reports what happened. */
#define DLSA_STATUS_OK 0          /* converged */
#define DLSA_STATUS_MAXITER 1     /* max_iter reached; the last iterate is returned
                                     with Sig_inv = X^T W X evaluated at it (one
                                     extra exact pass, as sklearn's model is used at
                                     whatever coef it stopped at, models.py:114-130) */
#define DLSA_STATUS_SINGULAR 2    /* X^T W X not positive definite */
#define DLSA_STATUS_EMPTY 3       /* no rows: zero block, like models.py:84-91 */
#define DLSA_STATUS_NONFINITE 4   /* NaN/Inf in the data or the iterates */
#define DLSA_STATUS_MISSING_LEVEL 5  /* categorical fit: a selected dummy level has no
                                        rows in the partition -> the reference's
                                        all-zero frame (models.py:84-91) */

/* Hessian arithmetic of the Newton passes.  The gradient, eta, the weights
 * and the returned log-likelihood are fp64 in every mode; the approximate
 * Hessians only steer Newton (the fp64 gradient fixes the solution).  The
 * Hessian returned as Sig_inv comes from the EXACT pass(es) that end the fit,
 * whose arithmetic dlsa_fit_options.exact_pass selects (DLSA_EXACT_*). */
#define DLSA_HESSIAN_MIXED 0      /* bf16 MFMA Hessian until the step is below
                                     switch_tol, then exact pass(es); a partition
                                     whose step stops shrinking (two iterations
                                     in a row without halving, or backtracking)
                                     moves to fp32 MFMA, then to exact passes */
#define DLSA_HESSIAN_FP64 1       /* fp64 MFMA Hessian on every pass (exact_pass is
                                     ignored) */
#define DLSA_HESSIAN_MIXED_F32 2  /* as MIXED with fp32 MFMA approximate passes
                                     (for ill-conditioned designs) */

/* Arithmetic of the exact pass in the MIXED modes.
 * DLSA_EXACT_AUTO: X^T W X from int8 digit slices on the int8 matrix cores
 *   (the Ozaki scheme) wherever it applies -- P <= 112 with chunks of at most
 *   32767 rows, every partition of the pass carrying a max |z| record from
 *   its last approximate pass (a partition stopped by max_iter in an
 *   approximate phase does not), and P > DLSA_MAX_P_FUSED when the workspace
 *   holds the digit records -- otherwise fp64 MFMA.  A chunk whose bound on
 *   |z| passes 2^1009 fails its partition (non-finite) instead of wrapping
 *   its digits.  z = sqrt(w) x is rounded to a 38-bit
 *   fixed-point grid below 2^E_f per chunk (or row group) and feature, the
 *   digit products are summed exactly in int32 and the levels below 2^-40 of
 *   the leading product are dropped: every entry of Sig_inv is within about
 *   1e-12 sqrt(H_ii H_jj) of the fp64 sum (tests/test_gpu_ozaki.py pins
 *   < 1e-10 on heavy-tailed designs), and the result is bit-identical run to
 *   run.  The logistic weights, gradient, log-likelihood and theta stay fp64.
 * DLSA_EXACT_FP64: every exact pass on the fp64 MFMA (v_mfma_f64_16x16x4). */
#define DLSA_EXACT_AUTO 0
#define DLSA_EXACT_FP64 1

#define DLSA_MAX_P_FUSED 192  /* largest P handled by the fused pass + LDS Newton solve */
#define DLSA_MAX_P 512        /* largest P overall: above DLSA_MAX_P_FUSED a row pass, a
                                 128x128-tiled Gram pass and a blocked Cholesky in HBM
                                 take over (BASELINE config 5, p = 500) */

typedef struct dlsa_fit_options {
  int32_t hessian_mode;     /* DLSA_HESSIAN_MIXED (default) or _FP64 */
  int32_t record_timing;    /* 1: time every launch with hipEvents, see
                               dlsa_last_fit_stats() */
  double switch_tol;        /* MIXED: relative step size that triggers the fp64
                               pass (<= 0: default 1e-6) */
  void* workspace;          /* device scratch, NULL: allocate per call */
  int64_t workspace_bytes;  /* size of `workspace` */
  int32_t rows_per_chunk;   /* <= 0: automatic (rows one workgroup streams) */
  int32_t warm_start;       /* 1 (default): the first Newton iterations run on
                               row prefixes of each partition (1/16, then 1/4
                               of the rows, never fewer than max(2048, 64 P))
                               to a 0.1-relative step, then on all rows to tol -- the
                               fixed point is unchanged; 0: all rows from the
                               start.  Prefix iterations count against max_iter
                               (a level takes at most half of what is left), so
                               iters[k] <= max_iter and max_iter = 1 is one
                               full-data Newton step from 0 */
  int32_t exact_pass;       /* DLSA_EXACT_AUTO (default) or DLSA_EXACT_FP64 */
  int32_t exact_waves;      /* geometry of the fp64 exact pass for P <= 128: 0 =
                               automatic, 1 = all tiles in one wave, 2 = two waves
                               (P 17..112); the result does not depend on it */
  int64_t oz_max_bytes;     /* P > DLSA_MAX_P_FUSED, mixed mode: at most this many
                               bytes of int8 digit records (<= 0: no cap); more
                               runs the fp64 Gram (dlsa_fit_stats.oz_fallbacks) */
  int32_t reserved[2];
} dlsa_fit_options;
/* The library reads no environment variable that changes a result: the
 * output of every entry point depends only on its arguments.  (DLSA_TRACE
 * prints per-iteration steps to stderr; profiling builds compiled with
 * -DDLSA_ENV_KNOBS=1 also read the A/B knobs named in capi.hip.) */

typedef struct dlsa_fit_stats {
  int32_t iterations;       /* Newton iterations run (max over partitions) */
  int32_t passes_fp32;      /* approximate-Hessian (bf16/fp32 MFMA) pass launches */
  int32_t passes_fp64;      /* fp64-Hessian pass launches */
  int32_t n_chunks;         /* waves per pass launch */
  double ms_pass_fp32;      /* summed kernel time (record_timing only) */
  double ms_pass_fp64;
  double ms_solve;          /* per-partition Cholesky/Newton update kernels */
  double ms_total;          /* whole call, host wall clock */
  int64_t rows_fp32;        /* rows streamed by approximate-Hessian passes (sum
                               over launches, warm-start levels included) */
  int64_t rows_fp64;        /* rows streamed by fp64 passes (sum) */
  double ms_wide_row;       /* P > DLSA_MAX_P_FUSED: row-pass kernel time (there
                               ms_pass_fp32/fp64 hold the bf16 / fp64 Gram-pass time) */
  double ms_wide_gram;      /* P > DLSA_MAX_P_FUSED: Gram-pass kernel time */
  double ms_wide_assemble;  /* P > DLSA_MAX_P_FUSED: partial-tile assembly time */
  int32_t passes_f32x;      /* of passes_fp32: fp32-MFMA passes of partitions that
                               escalated from bf16 (stall / lost definiteness) */
  int32_t polish_partitions; /* partitions left running by max_iter that got the
                               exact pass publishing Sig_inv at their theta */
  int32_t passes_oz;        /* of passes_fp64: on the int8 matrix cores (Ozaki
                               digit slices) */
  int32_t oz_fallbacks;     /* P > DLSA_MAX_P_FUSED, mixed mode: fits whose exact
                               Gram took the fp64 MFMA path because the int8
                               digit records had no room (a workspace of at least
                               the size without them but smaller than
                               dlsa_logistic_workspace_bytes, a failed
                               allocation, or dlsa_fit_options.oz_max_bytes) */
  int32_t oz_stale_partitions; /* P <= 112, mixed mode: partition passes of an
                               exact pass that ran on the fp64 MFMA beside the
                               int8 launch of the others, for lack of a fresh
                               max |sqrt(w) x| record */
} dlsa_fit_stats;

/* Default options (mixed Hessian, automatic chunking, no timing). */
void dlsa_fit_options_default(dlsa_fit_options* opt);

/* Device scratch needed by a fit with these partitions (offsets: HOST array of
 * K+1 int64).  Pass at least this many bytes in dlsa_fit_options.workspace.
 * For P > DLSA_MAX_P_FUSED this includes the int8 digit records of the
 * mixed-mode exact Gram (n * PP * 5 bytes, PP = P rounded up to 128; DESIGN.md
 * 4.4b): a smaller workspace that still holds everything else runs the fp64
 * Gram instead (dlsa_fit_stats.oz_fallbacks).  The library keeps no device
 * memory between calls: a NULL workspace is allocated on the stream and
 * freed before return. */
int64_t dlsa_logistic_workspace_bytes(const int64_t* offsets, int32_t K,
                                      int32_t p, int32_t fit_intercept,
                                      int32_t rows_per_chunk);

/*
 * Batched local logistic fit -- replaces the body of the map-stage UDF,
 * dlsa/models.py:42-147 logistic_model(), for K partitions at once:
 *   standardise (models.py:99-101; center/scale may be NULL),
 *   unpenalised logistic MLE (sklearn newton-cg, models.py:110-113),
 *   theta = [b0, b] with the intercept first (models.py:116-122),
 *   Sig_inv = X^T diag(p(1-p)) X at theta (models.py:130),
 *   Sig_invMcoef = Sig_inv theta (models.py:131).
 * Newton/IRLS from theta = 0; converged when max|step| <= tol*(1+max|theta|).
 *
 *  X        [n_total, p] fp64 row-major, device
 *  y        [n_total] fp64 0/1 labels, device
 *  offsets  [K+1] int64, HOST, offsets[0] = 0, non-decreasing
 *  center, scale  [p] fp64 device or NULL (both or neither)
 *  theta          [K, P] out     sig_inv       [K, P, P] out
 *  sig_inv_theta  [K, P] out     loglik        [K] out (at theta)
 *  iters          [K] int32 out  status        [K] int32 out (DLSA_STATUS_*)
 * 1 <= P <= DLSA_MAX_P.
 */
int dlsa_logistic_fit_batched(const double* X, const double* y,
                              const int64_t* offsets, int32_t K, int32_t p,
                              int32_t fit_intercept, const double* center,
                              const double* scale, int32_t max_iter,
                              double tol, double* theta, double* sig_inv,
                              double* sig_inv_theta, double* loglik,
                              int32_t* iters, int32_t* status, void* stream);

/* Same, with options (Hessian mode, caller workspace, timing). */
int dlsa_logistic_fit_batched_ex(const double* X, const double* y,
                                 const int64_t* offsets, int32_t K, int32_t p,
                                 int32_t fit_intercept, const double* center,
                                 const double* scale, int32_t max_iter,
                                 double tol, double* theta, double* sig_inv,
                                 double* sig_inv_theta, double* loglik,
                                 int32_t* iters, int32_t* status,
                                 const dlsa_fit_options* opt, void* stream);

/*
 * Batched local OLS fit (the linear DLSA path; the
 * reference only has a statsmodels per-group demo,
 * projects/results/linear_regression_dc.py:27-37):
 *   theta_k = (X_k^T X_k)^-1 X_k^T y_k,  Sig_inv_k = X_k^T X_k,
 *   sig_inv_theta_k = Sig_inv_k theta_k (= X_k^T y_k),
 *   rss_k = sum (y - X theta_k)^2.
 * One fp64 pass over X at theta = 0 (w = 1; P <= 64: X streamed straight
 * into the fp64-MFMA operands, ols_stream.hip; larger P: the logistic pass's
 * kernels with w = 1) plus one per-partition Cholesky solve.  opt may be
 * NULL; its hessian_mode is ignored (always fp64).
 */
int dlsa_ols_fit_batched(const double* X, const double* y, const int64_t* offsets,
                         int32_t K, int32_t p, int32_t fit_intercept,
                         const double* center, const double* scale, double* theta,
                         double* sig_inv, double* sig_inv_theta, double* rss,
                         int32_t* status, const dlsa_fit_options* opt,
                         void* stream);

/*
 * Log-likelihood evaluation pass -- replaces the per-partition body of
 * dlsa/models.py:151-225 logistic_model_eval (driven by dlsa/model_eval.py:
 * 10-42): for every partition k and candidate vector b (intercept first when
 * fit_intercept, standardised like the fit),
 *   loglik[k * n_beta + b] = sum_i y_i x_i.beta_b - log(1 + exp(x_i.beta_b)).
 * betas [n_beta, P] device, 1 <= n_beta <= 16, P <= 512; loglik [K, n_beta]
 * device.  One pass over X for all candidates; synchronises the stream.
 */
int dlsa_logistic_loglik_batched(const double* X, const double* y,
                                 const int64_t* offsets, int32_t K, int32_t p,
                                 int32_t fit_intercept, const double* center,
                                 const double* scale, const double* betas,
                                 int32_t n_beta, double* loglik, void* stream);

/*
 * Batched local logistic fit on a categorical-code layout -- the dummy branch
 * of dlsa/models.py:56-91 logistic_model() (airline design, BASELINE config
 * 3) without materialising the dummy matrix.  Row i of partition k holds
 *   Xn[i, 0:q]     q numeric columns (fp64, standardised by center/scale
 *                  [q] like models.py:99-101 -- dummies are never standardised)
 *   codes[i, 0:F]  one uint8 level code per factor f: 0 = the baseline level
 *                  (dropped, models.py:67/77), c in 1..levels[f]-1 = dummy
 *                  column c of factor f
 *   y[i]           0/1 label.
 * Parameters (P = fit_intercept + q + sum_f (levels[f] - 1) <= DLSA_MAX_P_FUSED):
 *   [intercept] [numeric 0..q-1] [factor 0 dummies 1..L0-1] [factor 1 ...] ...
 * The one-hot blocks of X^T W X are computed as weighted histograms in LDS
 * with int64 fixed-point bins: each term w, w x_i, y - mu is rounded once to
 * a power-of-two grid chosen per partition and column from the partition's
 * own max |x_i| (so that no bin can overflow), then summed exactly --
 * bit-identical run to run and within ~1e-13 of an fp64 sum relative to the
 * column's scale; the numeric x numeric block is fp64.  Outputs are as in
 * dlsa_logistic_fit_batched (theta,
 * Sig_inv = X^T W X of the dummy-expanded design at theta, ...).  A partition
 * in which some dummy column has no rows gets DLSA_STATUS_MISSING_LEVEL and
 * all-zero outputs, the reference's "fake zero matrix".  Codes >= levels[f]
 * fail the call with DLSA_E_INVALID.  Limits: F <= 16, levels[f] in 1..256,
 * fit_intercept + q <= 16.  levels is a HOST array [F]; opt may be NULL
 * (hessian_mode is ignored: every pass is exact; warm_start runs a 1/16-prefix
 * level first only when the partitions average >= 2^19 rows).
 */
int dlsa_logistic_fit_categorical(const double* Xn, const uint8_t* codes, const double* y,
                                  const int64_t* offsets, int32_t K, int32_t q, int32_t F,
                                  const int32_t* levels, int32_t fit_intercept,
                                  const double* center, const double* scale,
                                  int32_t max_iter, double tol, double* theta,
                                  double* sig_inv, double* sig_inv_theta, double* loglik,
                                  int32_t* iters, int32_t* status,
                                  const dlsa_fit_options* opt, void* stream);

/* Timing/iteration record of the calling thread's last fit. */
int dlsa_last_fit_stats(dlsa_fit_stats* out);

/*
 * Local pre-reduction of this device's partitions -- the group-sum of
 * dlsa/dlsa.py:30-34 (groupby('par_id').sum), done in HBM before the one
 * RCCL all-reduce that replaces the Spark shuffle + collect:
 *   out[0 : P*P]          = sum_k sig_inv[k]
 *   out[P*P : P*P+P]      = sum_k sig_inv_theta[k]
 *   out[P*P+P : P*P+2P]   = sum_k theta[k]
 *   out[P*P+2P]           = K   (partition count, for ONESHOT, dlsa.py:51-52)
 * Deterministic (fixed summation order over k).
 */
int dlsa_reduce_partitions(const double* sig_inv, const double* sig_inv_theta,
                           const double* theta, int32_t K, int32_t p,
                           double* out, void* stream);

/*
 * Row repartitioning in HBM -- replaces the Spark shuffle that groups rows by
 * partition before the map stage: `repartition(K, "partition_id")` + the
 * `groupby("partition_id").apply(udf)` of projects/logistic_dlsa.py:303-325,
 * with ids from monotonically_increasing_id() % K (:243-245) or a column.
 * A stable counting sort: rows of partition k land in output rows
 * offsets[k] .. offsets[k+1]-1 in their input order.
 *  part_id   [n] int32 device, every id in [0, K) (else DLSA_E_INVALID)
 *  src, dst, row_bytes  HOST arrays of n_arrays (<= 4) entries: device
 *            pointers of row-major arrays with row_bytes bytes per row (e.g.
 *            X [n, p] fp64 -> 8p, y -> 8, uint8 codes [n, F] -> F); dst must
 *            not overlap src
 *  offsets   [K+1] int64 HOST out (the layout every fit entry point takes)
 *  order     [n] int64 device out or NULL: input row of each output row
 * 1 <= K <= 16000.  Synchronises the stream (offsets are read back).
 */
int dlsa_partition_rows(const int32_t* part_id, int64_t n, int32_t K, int32_t n_arrays,
                        const void* const* src, void* const* dst, const int64_t* row_bytes,
                        int64_t* offsets, int64_t* order, void* stream);

/*
 * Column moments in HBM -- the device half of Spark's describe(), which the
 * reference runs over the whole data set to standardise every partition
 * with the global mean and stddev (projects/logistic_dlsa.py:287-298, read
 * by dlsa/models.py:99-101):
 *   out[0 p + j] = count, out[1 p + j] = mean, out[2 p + j] = M2 = sum (x - mean)^2,
 *   out[3 p + j] = min,   out[4 p + j] = max    of column j of X [n, p] (fp64,
 * row-major, device; out device [5 p]).  NaN entries are skipped (describe
 * ignores nulls); a column without values gets count 0 and NaN elsewhere.
 * Two passes over X (mean, then the squared deviations, compensated sums in
 * a fixed order: bit-identical run to run); stddev = sqrt(M2 / (count - 1)).
 * Partial moments of several shards combine exactly by Chan's formula
 * (dlsa_amd.ingest.merge_moments).  Scratch is allocated on the stream and
 * freed before return.
 */
int dlsa_column_moments(const double* X, int64_t n, int32_t p, double* out, void* stream);

/*
 * Synthetic logistic data in HBM (the input generator of SURVEY 8(d) for
 * configs too large for the host): X[i, j] = u(seed, row0 + i, j) - 0.5 with
 * u a counter-based (splitmix64) U[0,1) double; beta* = 1 on the first
 * floor(0.4 p) columns (dlsa/models.py:12-19); y ~ Bernoulli(sigmoid(X beta*))
 * drawn from an independent counter stream (models.py:23-30).  Rows are
 * written partition-contiguous; row0 offsets the counter so shards on
 * different GPUs draw disjoint rows.  Bit-exact with the numpy restatement
 * in oracle/ (simulate_counter).
 */
int dlsa_simulate_logistic(double* X, double* y, int64_t n, int32_t p,
                           uint64_t seed, int64_t row0, void* stream);

/*
 * LARS / adaptive-lasso path on the LSA quadratic form, HOST code --
 * replaces dlsa/lsa.py:90-212 lars_lsa (and R lars.lsa called from
 * dlsa/dlsa.py:77-80).  Sigma0 [P*P] row-major and b0 [P] are HOST arrays.
 * type: 0 = "lar", 1 = "lasso".  max_steps <= 0 means 8*m (lsa.py:116-117)
 * with m = P - intercept.  Outputs (HOST, caller-allocated for
 * max_steps+1 rows): beta [(max_steps+1) * m] row-major, beta0, aic, bic
 * [max_steps+1]; *n_steps = number of rows written (k+1).
 * Reference defects fixed: lsa.py:100 (intercept indexes range(1, n) with the
 * sample size), lsa.py:141-142 (singular back-out).
 */
int dlsa_lars_lsa(const double* Sigma0, const double* b0, int32_t P,
                  int32_t intercept, double n, int32_t type, double eps,
                  int32_t max_steps, double* beta, double* beta0, double* aic,
                  double* bic, int32_t* n_steps);

/* Thread-local message of the last failing call ("" if none). */
const char* dlsa_last_error(void);

/* Library build identification (gfx target, git-independent version). */
const char* dlsa_build_info(void);

#ifdef __cplusplus
}
#endif

#endif /* DLSA_HIP_H */
