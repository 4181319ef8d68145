// Per-partition Newton update (one 1024-thread workgroup per partition).
//
// Replaces the outer Newton step of sklearn's newton-cg solve inside
// dlsa/models.py:110-113 (the reference solves H d = g iteratively by CG with
// 2 passes over X per CG step; here H is assembled once per pass and factored
// in LDS):
//   1. sum the chunk partials of the pass (fixed order -> deterministic),
//      keep the lower triangle packed in LDS (P <= 192: <= 152 KB);
//   2. step control: if the log-likelihood fell, halve the previous step
//      (the role of sklearn's line search);
//   3. publish H as Sig_inv (models.py:130: the information at the point the
//      pass was evaluated) and the log-likelihood;
//   4. Cholesky H = L L^T in LDS, solve L L^T d = g, theta += d;
//   5. convergence / phase switch (approximate Hessian -> fp64 pass), stall
//      escalation (bf16 -> fp32 -> fp64, dlsa_internal.hpp).
// eval_only (the polish pass after a budget ran out): steps 1 and 3 only.
#include <math.h>

#include "dlsa_internal.hpp"

// Newton steps refining v_rsq_f64 in the diagonal-block factor (A/B builds)
#ifndef DLSA_SOLVE_RSQ_STEPS
#define DLSA_SOLVE_RSQ_STEPS 2
#endif

// Profiling-only phase timestamps of partition 0 (tools/build_variants.sh
// solveprof; product build 0): printf of shader-clock deltas per phase.
#ifndef DLSA_SOLVE_PROFILE
#define DLSA_SOLVE_PROFILE 0
#endif
#if DLSA_SOLVE_PROFILE
#define SOLVE_MARK(i) \
  if (k == 0 && tid == 0) tmark[i] = clock64();
#else
#define SOLVE_MARK(i)
#endif

namespace dlsa {

// Threads per partition (NTHR): 1024 when K <= 256 -- one partition per CU,
// so the trailing updates (the bulk of the Cholesky at P >= 100) spread over
// 16 waves instead of 4 and the assembly holds T / 4 tiles per thread (configs
// 3, 5-share and the N = 8 share of config 2: K = 120-128); 256 above, where
// three partitions share a CU (config 2, K = 1024: the LDS of the packed
// triangle allows 3).  The diagonal blocks and triangular solves stay on wave 0.
constexpr int kMaxSolveWaves = 16;
constexpr int kRedFlag = kMaxSolveWaves, kRedSink = kMaxSolveWaves + 1,
              kRedLL = kMaxSolveWaves + 2, kRedZero = kMaxSolveWaves + 3;
constexpr int kRedSize = kMaxSolveWaves + 4;

__device__ __forceinline__ double block_max(double v, double* red) {
  for (int o = 32; o > 0; o >>= 1) v = fmax(v, __shfl_xor(v, o));
  const int w = threadIdx.x >> 6;
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[w] = v;
  __syncthreads();
  double r = red[0];
  for (int i = 1; i < (int)(blockDim.x >> 6); ++i) r = fmax(r, red[i]);
  return r;
}

// Sum of 64 lanes, result in every lane.
__device__ __forceinline__ double wave_sum(double v) {
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

typedef double d4s __attribute__((ext_vector_type(4)));

// v_readlane of a double (lane index wave-uniform)
__device__ __forceinline__ double readlane_f64(double v, int l) {
  const int lo = __builtin_amdgcn_readlane(__double2loint(v), l);
  const int hi = __builtin_amdgcn_readlane(__double2hiint(v), l);
  return __hiloint2double(hi, lo);
}

// Packed lower triangle: element (i, j), i >= j, at i (i + 1) / 2 + j.
__device__ __forceinline__ int tri(int i, int j) { return i * (i + 1) / 2 + j; }

template <int NT, int NTHR>
__global__ __launch_bounds__(NTHR) void newton_solve_kernel(const SolveArgs a) {
  constexpr int kSolveThreads = NTHR, kSolveWaves = NTHR / 64;
  extern __shared__ __attribute__((aligned(16))) double sm[];
  constexpr int T = NT * (NT + 1) / 2;
  constexpr int PP = 16 * NT;
  const int k = blockIdx.x;
  const int tid = threadIdx.x;
  const int lane = tid & 63, wid = tid >> 6;
  if (a.status[k] != STATUS_RUNNING) return;  // block-uniform
  const int P = a.P;
  double* dblk = sm;                 // [16][16]: the panel's L_bb (strict lower), 1 / L_kk
                                     // on the diagonal, at LDS offset 0: compile-time
                                     // addresses in the panel solve (packed-triangle
                                     // addresses of a moving panel, or a P-dependent base,
                                     // cost ~140 spilled SGPRs)
  double* H = sm + 256;              // packed lower triangle, P (P + 1) / 2
  double* g = H + P * (P + 1) / 2;   // PP
  double* z = g + PP;                // PP
  double* invd = z + PP;             // PP: 1 / L_jj
  double* red = invd + PP;           // kRedSize: [0, kSolveWaves) per-wave values, flag, sink, ll

  // chunk partials were summed into the partition's first chunk by
  // partials_sum_kernel (fixed chunk order)
  const int cb = a.part_chunk_begin[k], ce = min(a.part_chunk_begin[k + 1], cb + 1);
  const int phase = a.phase[k];
#if DLSA_SOLVE_PROFILE
  long long tmark[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  long long tpan[3] = {0, 0, 0}, tp0 = 0;  // Cholesky: diagonal block, panel rows, trailing
#define SOLVE_PAN(i)                             \
  if (k == 0 && tid == 0) {                      \
    const long long tn = clock64();              \
    if (i > 0) tpan[i - 1] += tn - tp0;          \
    tp0 = tn;                                    \
  }
#else
#define SOLVE_PAN(i)
#endif
  SOLVE_MARK(0)

  // 1. assemble: thread tid owns position tid % 256 of the tiles
  //    t = tid / 256 + 4 u (the partition's partials were summed into its first
  //    chunk by partials_sum_kernel).  Only the lower triangle is kept
  //    (diagonal tiles hold (w x_i) x_j and (w x_j) x_i, equal up to the last
  //    bit): Sig_inv comes out exactly symmetric.
  {
    constexpr int G = kSolveThreads / 256;
    constexpr int TG = (T + G - 1) / G;
    const int pos = tid & 255, grp = tid >> 8;
    const int r = pos >> 4, q = pos & 15;
    for (int c = cb; c < ce; ++c) {
      const double* src = a.slab_H + (int64_t)c * T * 256 + pos;
      constexpr int UB = TG < 8 ? TG : 8;  // tiles loaded together (unconditional loads)
#pragma unroll
      for (int u0 = 0; u0 < TG; u0 += UB) {
        double v[UB];
#pragma unroll
        for (int u = 0; u < UB; ++u) v[u] = src[min(grp + G * (u0 + u), T - 1) * 256];
#pragma unroll
        for (int u = 0; u < UB; ++u) {
          const int t = grp + G * (u0 + u);
          if (u0 + u < TG && t < T) {
            int I = 0;
            while ((I + 1) * (I + 2) / 2 <= t) ++I;
            const int gi = 16 * I + r, gj = 16 * (t - I * (I + 1) / 2) + q;
            if (gi < P && gi >= gj) H[tri(gi, gj)] = v[u];
          }
        }
      }
    }
  }
  if (tid < PP) {
    double s = 0.0;
    for (int c = cb; c < ce; ++c) s += a.slab_g[(int64_t)c * PP + tid];
    g[tid] = s;
    z[tid] = s;  // the augmented row of the factorisation: becomes L^-1 g (step 4)
  }
  if (wid == 0) {
    double s = 0.0;
    for (int c = cb + lane; c < ce; c += 64) s += a.slab_ll[c];
    s = wave_sum(s);
    if (lane == 0) red[kRedLL] = s;
  }
  __syncthreads();
  const double ll = red[kRedLL];
  const int it = a.iters[k];
  double* th = a.theta + (int64_t)k * P;

  // a warm-start level that fails (separation, too few rows) only restarts
  // the partition from theta = 0 on the next level
  auto level_fail = [&]() {
    for (int f = tid; f < P; f += kSolveThreads) th[f] = 0.0;
    if (tid == 0) {
      a.phase[k] = PHASE_LEVEL_DONE;
      a.iters[k] = it + 1;
    }
  };
  if (!isfinite(ll)) {
    if (a.subsample)
      level_fail();
    else if (tid == 0)
      a.status[k] = DLSA_STATUS_NONFINITE;
    return;
  }

  // 2. step halving on a log-likelihood decrease ---------------------------
  //    threshold above the fp32-log noise of mixed-mode log-likelihoods; real
  //    overshoots of a Newton step lose far more than 1e-6 relative
  const double llp = a.ll_prev[k];
  if (!a.eval_only && a.family == FAMILY_LOGISTIC && it > 0 &&
      ll < llp - 1e-6 * (1.0 + fabs(llp)) && a.backtracks[k] < 40) {
    const int bt = a.backtracks[k] + 1;
    const double sc = ldexp(1.0, -bt);
    const double* tp = a.theta_prev + (int64_t)k * P;
    const double* dp = a.delta_prev + (int64_t)k * P;
    for (int f = tid; f < P; f += kSolveThreads) th[f] = tp[f] + sc * dp[f];
    if (tid == 0) {
      a.backtracks[k] = bt;
      a.iters[k] = it + 1;
      int ph = phase;
      if (!a.subsample && ph != PHASE_F64) {  // an approximate step that overshot
        ph = approx_backtrack_phase(a, k, ph);
        a.phase[k] = ph;
      }
      atomicAdd(&a.counters[ph], 1);
    }
    return;
  }

  SOLVE_MARK(1)
  // 3. publish the information matrix at the evaluation point --------------
  if (!a.subsample) {
    double* S = a.sig_inv + (int64_t)k * P * P;
    for (int e = tid; e < P * P; e += kSolveThreads) {
      const int i = e / P, j = e - i * P;
      S[e] = H[i >= j ? tri(i, j) : tri(j, i)];
    }
    if (tid == 0) a.loglik[k] = ll;
  }
  if (a.eval_only) return;  // polish: Sig_inv at the returned theta, no step
  __syncthreads();

  // 4. Cholesky, blocked (16-column panels), lower, in place in the packed
  //    triangle.  Per panel b (columns c0 .. c0 + 15):
  //    (a) wave 0 factors the diagonal block in registers (lane i = row i,
  //        column values broadcast with v_readlane) and records 1 / L_jj;
  //    (b) every thread solves one row i of the panel below:
  //        L_ib = A_ib L_bb^-T (forward substitution against L_bb);
  //    (c) the trailing lower triangle is updated tile by tile on fp64 MFMA,
  //        A_IJ -= L_Ib L_Jb^T (16x16 tiles, 4 k-steps of 4 columns).
  //    Three barriers per 16 columns (was one per column with a serial
  //    per-thread row update).
  SOLVE_MARK(2)
  if (tid == 0) {
    red[kRedFlag] = 0.0;
    red[kRedZero] = 0.0;  // read by the triangular solves off the triangle
  }
  __syncthreads();
  bool ok = true;
  for (int b = 0; b < NT; ++b) {
    const int c0 = 16 * b;
    if (c0 >= P) break;
    const int nb = min(16, P - c0);
    SOLVE_PAN(0)
    // the lane index re-defined opaquely per panel: otherwise the compiler
    // hoists the ~40 lane-compare masks of the loop body out of the panel
    // loop and spills them (~140 SGPRs, a v_readlane per reload)
    int lv = lane;
    asm volatile("" : "+v"(lv));
    if (wid == 0) {
      const int i = lv & 15;
      const bool act = lv < nb;
      // branch-free: every lane loads an in-triangle address (clamped) and
      // selects; lanes / entries outside the block store to a dummy slot
      const int ri = min(c0 + i, P - 1);
      double av[16];
#pragma unroll
      for (int j = 0; j < 16; ++j) {
        const double hv = H[tri(ri, min(c0 + j, ri))];
        av[j] = (act && j <= i) ? hv : 0.0;
      }
      bool good = true;
      double ild = 0.0;  // lane kk: 1 / L_kk
#pragma unroll
      for (int kk = 0; kk < 16; ++kk) {
        if (kk < nb) {  // wave-uniform
          const double dkk = readlane_f64(av[kk], kk);
          good = good && dkk > 0.0 && isfinite(dkk);
          // 1 / sqrt(d) by v_rsq_f64 + two Newton steps (~1 ulp), L_kk = d / sqrt(d):
          // the serial chain of the block is 16 of these (IEEE sqrt + division:
          // ~2x the dependent latency)
          double il = __builtin_amdgcn_rsq(dkk);
#pragma unroll
          for (int nr = 0; nr < DLSA_SOLVE_RSQ_STEPS; ++nr) il = fma(il, fma(-0.5 * dkk * il, il, 0.5), il);
          const double lkk = dkk * il;
          if (lv == kk) ild = il;
          av[kk] = (i > kk) ? av[kk] * il : (i == kk ? lkk : av[kk]);
#pragma unroll
          for (int j = kk + 1; j < 16; ++j) {
            const double ljk = readlane_f64(av[kk], j);  // L[j][kk], row j's lane
            if (j <= i) av[j] = fma(-av[kk], ljk, av[j]);
          }
          if (lv == 0) invd[c0 + kk] = il;
        }
      }
#pragma unroll
      for (int j = 0; j < 16; ++j) *((act && j <= i) ? H + tri(ri, c0 + j) : red + kRedSink) = av[j];
      if (lv < 16) {
#pragma unroll
        for (int j = 0; j < 16; ++j) dblk[16 * lv + j] = j < i ? av[j] : (j == i ? ild : 0.0);
      }
      if (lv == 0 && !good) red[kRedFlag] = 1.0;
    }
    __syncthreads();
    SOLVE_PAN(1)
    if (red[kRedFlag] != 0.0) {  // block-uniform
      ok = false;
      break;
    }
    // (b) panel rows below the block, and the augmented row z (thread
    //     nbelow): its block entries become z_b = L_bb^-1 (g_b - sum_c L_bc z_c),
    //     the forward substitution L z = g folded into the factorisation (the
    //     serial per-column forward loop of step 5 is gone)
    const int nbelow = max(0, P - (c0 + 16));
    if (tid <= nbelow) {
      {
        double* hr = tid < nbelow ? H + tri(c0 + 16 + tid, c0) : z + c0;
        double x[16];
#pragma unroll
        for (int kk = 0; kk < 16; ++kk) x[kk] = hr[kk];
#pragma unroll
        for (int kk = 0; kk < 16; ++kk) {
          x[kk] *= dblk[17 * kk];
#pragma unroll
          for (int m = kk + 1; m < 16; ++m) x[m] = fma(-x[kk], dblk[16 * m + kk], x[m]);
        }
#pragma unroll
        for (int kk = 0; kk < 16; ++kk) hr[kk] = x[kk];
      }
    }
    __syncthreads();
    SOLVE_PAN(2)
    if (c0 + 16 < P) {
      // (c0) the augmented row's trailing update: z_j -= L_jb z_b, j below
      for (int jj = tid; jj < nbelow; jj += kSolveThreads) {
        const double* lr = H + tri(c0 + 16 + jj, c0);
        double acc = 0.0;
#pragma unroll
        for (int kk = 0; kk < 16; ++kk) acc = fma(lr[kk], z[c0 + kk], acc);
        z[c0 + 16 + jj] -= acc;
      }
      const int m = NT - b - 1;  // tile rows below the panel
      const int ntile = m * (m + 1) / 2;
      const int fl = lv & 15, q = lv >> 4;
      for (int t = wid; t < ntile; t += kSolveWaves) {  // wave-uniform
        int I = 0;
        while ((I + 1) * (I + 2) / 2 <= t) ++I;
        const int J = t - I * (I + 1) / 2;
        const int gI = c0 + 16 * (I + 1), gJ = c0 + 16 * (J + 1);
        // branch-free as above (clamped in-triangle loads, dummy-slot stores)
        d4s acc;
        int adr[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int row = gI + q + 4 * r, col = gJ + fl;
          const bool in = row < P && col <= row;
          const int rc = min(row, P - 1);
          const double hv = H[tri(rc, min(col, rc))];
          acc[r] = in ? hv : 0.0;
          adr[r] = in ? tri(row, col) : -1;
        }
        const int ra = min(gI + fl, P - 1), rb = min(gJ + fl, P - 1);
        const bool ina = gI + fl < P, inb = gJ + fl < P;
#pragma unroll
        for (int st = 0; st < 4; ++st) {
          const int kc = c0 + 4 * st + q;
          const double ha = H[tri(ra, kc)], hb = H[tri(rb, kc)];
          const double x_a = ina ? ha : 0.0;
          const double x_b = inb ? hb : 0.0;
          acc = __builtin_amdgcn_mfma_f64_16x16x4f64(-x_a, x_b, acc, 0, 0, 0);
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) *(adr[r] >= 0 ? H + adr[r] : red + kRedSink) = acc[r];
      }
    }
    __syncthreads();
    SOLVE_PAN(3)
  }
  if (!ok) {
    if (a.subsample) {
      level_fail();
      return;
    }
    if (tid == 0) {
      if (phase != PHASE_F64 && a.family == FAMILY_LOGISTIC) {
        // low-precision Hessian lost definiteness: redo this point one
        // precision up (bf16 -> fp32 -> fp64)
        const int32_t ph = escalate_phase(a, phase);
        a.phase[k] = ph;
        a.iters[k] = it + 1;
        a.stall[k] = 0;
        a.dm_prev[k] = 0.0;
        atomicAdd(&a.counters[ph], 1);
      } else {
        a.status[k] = DLSA_STATUS_SINGULAR;
      }
    }
    return;
  }

  SOLVE_MARK(3)
  // 5. back substitution L^T d = z (L z = g came out of step 4 as the
  //    augmented row), blocked by the 16-column panels from the last: wave 0
  //    solves the block's L_bb^T d_b = z_b in registers (lane i = row i, the
  //    pivot broadcast by v_readlane, 1 / L_kk from invd), then every thread j
  //    of the columns left of the block takes z_j -= sum_k L[c0 + k][j] d_k.
  //    Two barriers per 16 columns instead of a serial chain of P steps.
  for (int b = (P - 1) >> 4; b >= 0; --b) {
    const int c0 = 16 * b;
    const int nb = min(16, P - c0);
    int lv = lane;
    asm volatile("" : "+v"(lv));
    if (wid == 0) {
      const int i = lv & 15;
      const bool act = lv < nb;
      // L[c0 + m][c0 + i] for m > i (the block's column i), zero elsewhere
      double lc[16];
#pragma unroll
      for (int m = 0; m < 16; ++m)
        lc[m] = *((act && m > i && m < nb) ? H + tri(c0 + m, c0 + i) : red + kRedZero);
      double zi = act ? z[c0 + i] : 0.0;
      const double il = act ? invd[c0 + i] : 0.0;
#pragma unroll
      for (int kk = 15; kk >= 0; --kk) {
        if (kk < nb) {  // wave-uniform
          const double dk = readlane_f64(zi * il, kk);
          zi = (i == kk) ? dk : fma(-lc[kk], dk, zi);
        }
      }
      if (act && lv < 16) z[c0 + i] = zi;
    }
    __syncthreads();
    for (int j = tid; j < c0; j += kSolveThreads) {
      double acc = 0.0;
#pragma unroll
      for (int k2 = 0; k2 < 16; ++k2)
        if (k2 < nb) acc = fma(H[tri(c0 + k2, j)], z[c0 + k2], acc);
      z[j] -= acc;
    }
    __syncthreads();
  }

  SOLVE_MARK(4)
#if DLSA_SOLVE_PROFILE
  if (k == 0 && tid == 0)
    printf("[solve-profile] P=%d assemble %lld publish %lld cholesky %lld (diag %lld panel %lld "
           "trailing %lld) trisolve %lld\n", P, tmark[1] - tmark[0], tmark[2] - tmark[1],
           tmark[3] - tmark[2], tpan[0], tpan[1], tpan[2], tmark[4] - tmark[3]);
#endif
  // 6. update + convergence ------------------------------------------------
  double dm = 0.0, tm = 0.0, tg = 0.0;
  double* tp = a.theta_prev + (int64_t)k * P;
  double* dp = a.delta_prev + (int64_t)k * P;
  for (int f = tid; f < P; f += kSolveThreads) {
    const double d = z[f];
    const double t0 = th[f];
    const double t1 = t0 + d;
    tp[f] = t0;
    dp[f] = d;
    th[f] = t1;
    dm = fmax(dm, fabs(d));
    tm = fmax(tm, fabs(t1));
    tg += t1 * g[f];
  }
  dm = block_max(dm, red);
  tm = block_max(tm, red);
  if (!isfinite(dm) && !a.subsample) {
    // keep the last finite iterate (each thread restores the entries it
    // wrote): the status reports the failure and the combine step excludes
    // the partition
    for (int f = tid; f < P; f += kSolveThreads) th[f] = tp[f];
  }
  if (a.family == FAMILY_GAUSSIAN) {
    // OLS: theta was 0, one Newton step is the closed form (X^T X)^-1 X^T y;
    // residual sum of squares = y^T y - theta^T X^T y = -2 ll(0) - theta . g
    tg = wave_sum(tg);
    __syncthreads();
    if (lane == 0) red[wid] = tg;
    __syncthreads();
    if (tid == 0) {
      double tgs = 0.0;
#pragma unroll
      for (int w = 0; w < kSolveWaves; ++w) tgs += red[w];
      a.loglik[k] = -2.0 * ll - tgs;
      a.iters[k] = it + 1;
      a.status[k] = isfinite(dm) ? DLSA_STATUS_OK : DLSA_STATUS_NONFINITE;
      a.phase[k] = PHASE_DONE;
    }
    return;
  }
  if (a.subsample) {
    if (!isfinite(dm)) {
      level_fail();
      return;
    }
    if (tid == 0) {
      a.ll_prev[k] = ll;
      a.backtracks[k] = 0;
      a.iters[k] = it + 1;
      if (dm <= a.level_tol * (1.0 + tm)) {
        a.phase[k] = PHASE_LEVEL_DONE;
      } else {
        atomicAdd(&a.counters[phase], 1);
      }
    }
    return;
  }
  if (tid == 0) {
    a.ll_prev[k] = ll;
    a.backtracks[k] = 0;
    a.iters[k] = it + 1;
    int ph = phase;
    if (!isfinite(dm)) {
      a.status[k] = DLSA_STATUS_NONFINITE;
      return;
    }
    if (ph != PHASE_F64) {
      if (dm <= a.switch_tol * (1.0 + tm)) {
        ph = PHASE_F64;
      } else {
        ph = approx_next_phase(a, k, ph, dm, ll, llp);
        // near the switch: the next bf16 pass records the Ozaki digit scales
        if (ph == PHASE_F32 && dm <= kOzNearTol * (1.0 + tm)) atomicAdd(&a.counters[3], 1);
      }
    } else if (dm <= a.tol * (1.0 + tm)) {
      a.status[k] = DLSA_STATUS_OK;
      a.phase[k] = PHASE_DONE;
      return;
    }
    a.phase[k] = ph;
    atomicAdd(&a.counters[ph], 1);
  }
}


// Sum the per-chunk partials (Hessian tiles, gradient, log-likelihood) of
// every running partition into its first chunk's slab, in chunk order
// (deterministic).  Grid (ceil((T + 1) / 4), K): wave w of workgroup x owns
// tile 4x + w (tile T = the gradient and log-likelihood), so a partition's
// partials are read by many waves at once instead of by its single solve
// workgroup (config 3: 65 chunks x 78 tiles per partition).
__global__ __launch_bounds__(256) void partials_sum_kernel(const SolveArgs a, int T, int PP) {
  const int k = blockIdx.y;
  if (a.status[k] != STATUS_RUNNING) return;
  const int cb = a.part_chunk_begin[k], n = a.part_chunk_begin[k + 1] - cb;
  if (n <= 1) return;
  const int lane = threadIdx.x & 63;
  const int t = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (t < T) {
    const int64_t stride = (int64_t)T * 256;
    double* dst = const_cast<double*>(a.slab_H) + cb * stride + t * 256 + lane;
    const double* src = dst;
    double s0 = 0.0, s1 = 0.0, s2 = 0.0, s3 = 0.0;
#pragma unroll 8
    for (int c = 0; c < n; ++c) {
      const double* p = src + c * stride;
      s0 += p[0];
      s1 += p[64];
      s2 += p[128];
      s3 += p[192];
    }
    dst[0] = s0;
    dst[64] = s1;
    dst[128] = s2;
    dst[192] = s3;
  } else if (t == T) {
    double* g = const_cast<double*>(a.slab_g) + (int64_t)cb * PP;
    for (int e = lane; e < PP; e += 64) {
      double s = 0.0;
#pragma unroll 8
      for (int c = 0; c < n; ++c) s += g[(int64_t)c * PP + e];
      g[e] = s;
    }
    double* ll = const_cast<double*>(a.slab_ll) + cb;
    double s = 0.0;
    for (int c = lane; c < n; c += 64) s += ll[c];
    s = wave_sum(s);
    if (lane == 0) ll[0] = s;
  }
}

template <int NT>
static hipError_t launch_solve_t(const SolveArgs& a, int K, size_t lds, hipStream_t s) {
  const bool wide = K <= 256;
  auto kern = wide ? newton_solve_kernel<NT, 1024> : newton_solve_kernel<NT, 256>;
  {
    hipError_t e = ensure_max_lds((const void*)kern, 160 * 1024);
    if (e != hipSuccess) return e;
  }
  constexpr int T = NT * (NT + 1) / 2;
  hipLaunchKernelGGL(partials_sum_kernel, dim3((T + 1 + 3) / 4, K), dim3(256), 0, s, a, T, 16 * NT);
  hipLaunchKernelGGL(kern, dim3(K), dim3(wide ? 1024 : 256), lds, s, a);
  return hipGetLastError();
}

hipError_t launch_newton_solve(const SolveArgs& a, int K, hipStream_t s) {
  const int PP = 16 * a.NT;
  const size_t lds = ((size_t)a.P * (a.P + 1) / 2 + 3 * PP + kRedSize + 256) * sizeof(double);
  switch (a.NT) {
    case 1: return launch_solve_t<1>(a, K, lds, s);
    case 2: return launch_solve_t<2>(a, K, lds, s);
    case 3: return launch_solve_t<3>(a, K, lds, s);
    case 4: return launch_solve_t<4>(a, K, lds, s);
    case 5: return launch_solve_t<5>(a, K, lds, s);
    case 6: return launch_solve_t<6>(a, K, lds, s);
    case 7: return launch_solve_t<7>(a, K, lds, s);
    case 8: return launch_solve_t<8>(a, K, lds, s);
    case 9: return launch_solve_t<9>(a, K, lds, s);
    case 10: return launch_solve_t<10>(a, K, lds, s);
    case 11: return launch_solve_t<11>(a, K, lds, s);
    case 12: return launch_solve_t<12>(a, K, lds, s);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace dlsa
