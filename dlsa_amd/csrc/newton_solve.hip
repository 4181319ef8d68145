// Per-partition Newton update (one 256-thread workgroup per partition).
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
//   5. convergence / phase switch (fp32-MFMA Hessian -> fp64 pass).
#include <math.h>

#include "dlsa_internal.hpp"

namespace dlsa {

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

// Packed lower triangle: element (i, j), i >= j, at i (i + 1) / 2 + j.
__device__ __forceinline__ int tri(int i, int j) { return i * (i + 1) / 2 + j; }

template <int NT>
__global__ __launch_bounds__(256) void newton_solve_kernel(const SolveArgs a) {
  extern __shared__ __attribute__((aligned(16))) double sm[];
  constexpr int T = NT * (NT + 1) / 2;
  constexpr int PP = 16 * NT;
  constexpr int R = (PP + 63) / 64;  // solve registers per lane (rows lane + 64 r)
  const int k = blockIdx.x;
  const int tid = threadIdx.x;
  const int lane = tid & 63, wid = tid >> 6;
  if (a.status[k] != STATUS_RUNNING) return;  // block-uniform
  const int P = a.P;
  double* H = sm;                    // packed lower triangle, P (P + 1) / 2
  double* g = H + P * (P + 1) / 2;   // PP
  double* z = g + PP;                // PP
  double* red = z + PP;              // 8: [0..3] block reductions, [6] flag, [7] ll

  const int cb = a.part_chunk_begin[k], ce = a.part_chunk_begin[k + 1];
  const int phase = a.phase[k];

  // 1. assemble: thread tid owns element (tile t, position tid) of every
  //    tile; the chunk loop issues T independent loads per step.  Only the
  //    lower triangle is kept (diagonal tiles hold (w x_i) x_j and (w x_j) x_i,
  //    equal up to the last bit): Sig_inv comes out exactly symmetric.
  {
    double acc[T];
#pragma unroll
    for (int t = 0; t < T; ++t) acc[t] = 0.0;
    for (int c = cb; c < ce; ++c) {
      const double* src = a.slab_H + (int64_t)c * T * 256 + tid;
#pragma unroll
      for (int t = 0; t < T; ++t) acc[t] += src[t * 256];
    }
    const int r = tid >> 4, q = tid & 15;
#pragma unroll
    for (int I = 0; I < NT; ++I)
#pragma unroll
      for (int J = 0; J <= I; ++J) {
        const int t = I * (I + 1) / 2 + J;
        const int gi = 16 * I + r, gj = 16 * J + q;
        if (gi < P && gi >= gj) H[tri(gi, gj)] = acc[t];
      }
  }
  if (tid < PP) {
    double s = 0.0;
    for (int c = cb; c < ce; ++c) s += a.slab_g[(int64_t)c * PP + tid];
    g[tid] = s;
  }
  if (wid == 0) {
    double s = 0.0;
    for (int c = cb + lane; c < ce; c += 64) s += a.slab_ll[c];
    s = wave_sum(s);
    if (lane == 0) red[7] = s;
  }
  __syncthreads();
  const double ll = red[7];
  const int it = a.iters[k];
  double* th = a.theta + (int64_t)k * P;

  // a warm-start level that fails (separation, too few rows) only restarts
  // the partition from theta = 0 on the next level
  auto level_fail = [&]() {
    for (int f = tid; f < P; f += 256) th[f] = 0.0;
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
  if (a.family == FAMILY_LOGISTIC && it > 0 && ll < llp - 1e-6 * (1.0 + fabs(llp)) &&
      a.backtracks[k] < 40) {
    const int bt = a.backtracks[k] + 1;
    const double sc = ldexp(1.0, -bt);
    const double* tp = a.theta_prev + (int64_t)k * P;
    const double* dp = a.delta_prev + (int64_t)k * P;
    for (int f = tid; f < P; f += 256) th[f] = tp[f] + sc * dp[f];
    if (tid == 0) {
      a.backtracks[k] = bt;
      a.iters[k] = it + 1;
      atomicAdd(&a.counters[phase], 1);
    }
    return;
  }

  // 3. publish the information matrix at the evaluation point --------------
  if (!a.subsample) {
    double* S = a.sig_inv + (int64_t)k * P * P;
    for (int e = tid; e < P * P; e += 256) {
      const int i = e / P, j = e - i * P;
      S[e] = H[i >= j ? tri(i, j) : tri(j, i)];
    }
    if (tid == 0) a.loglik[k] = ll;
  }
  __syncthreads();

  // 4. Cholesky, right-looking, lower, in place.  Thread (tid/2, tid%2) owns
  //    the even/odd columns of rows tid/2, tid/2 + 128.  Column j is only READ
  //    during step j (l_xj = H[x][j] / sqrt(H[j][j]) recomputed by every
  //    reader); its scaled values are written back at step j+1, so one
  //    barrier per column suffices.
  const int row0 = tid >> 1, par = tid & 1;
  bool ok = true;
  double inv_prev = 0.0;
  for (int j = 0; j < P; ++j) {
    const double d = H[tri(j, j)];
    if (!(d > 0.0) || !isfinite(d)) {
      ok = false;  // uniform: every thread read the same d
      break;
    }
    const double inv = 1.0 / sqrt(d);
    const double* colj = H + j;  // H[tri(c, j)] = colj[c (c + 1) / 2]
    for (int row = row0; row < P; row += 128) {
      double* hr = H + tri(row, 0);
      if (par == 0 && j > 0 && row >= j - 1) {
        // deferred write-back of column j-1 (scaled) for this row
        hr[j - 1] = (row == j - 1) ? sqrt(hr[row]) : hr[j - 1] * inv_prev;
      }
      if (row > j) {
        const double lij = hr[j] * inv;
        for (int c = j + 1 + par; c <= row; c += 2) hr[c] -= lij * (colj[tri(c, 0)] * inv);
      }
    }
    inv_prev = inv;
    __syncthreads();
  }
  if (ok && par == 0 && row0 == (P - 1) % 128 && row0 < P) {
    // last column: only the diagonal element
    H[tri(P - 1, P - 1)] = sqrt(H[tri(P - 1, P - 1)]);
  }
  __syncthreads();
  if (!ok) {
    if (a.subsample) {
      level_fail();
      return;
    }
    if (tid == 0) {
      if (phase == PHASE_F32 && a.family == FAMILY_LOGISTIC) {
        // low-precision Hessian lost definiteness: redo this point with fp64
        a.phase[k] = PHASE_F64;
        a.iters[k] = it + 1;
        atomicAdd(&a.counters[PHASE_F64], 1);
      } else {
        a.status[k] = DLSA_STATUS_SINGULAR;
      }
    }
    return;
  }

  // 5. triangular solves L z = g, L^T d = z by wave 0 (no barriers: lane l
  //    holds z[l + 64 r]; the pivot is broadcast by shuffle)
  if (wid == 0) {
    double zr[R];
#pragma unroll
    for (int r = 0; r < R; ++r) zr[r] = lane + 64 * r < P ? g[lane + 64 * r] : 0.0;
    for (int j = 0; j < P; ++j) {
      double piv = 0.0;
#pragma unroll
      for (int r = 0; r < R; ++r)
        if ((j >> 6) == r) piv = zr[r];
      const double zj = __shfl(piv, j & 63) / H[tri(j, j)];
#pragma unroll
      for (int r = 0; r < R; ++r) {
        const int i = lane + 64 * r;
        if (i == j)
          zr[r] = zj;
        else if (i > j && i < P)
          zr[r] -= H[tri(i, j)] * zj;
      }
    }
    for (int j = P - 1; j >= 0; --j) {
      double piv = 0.0;
#pragma unroll
      for (int r = 0; r < R; ++r)
        if ((j >> 6) == r) piv = zr[r];
      const double zj = __shfl(piv, j & 63) / H[tri(j, j)];
      const double* lj = H + tri(j, 0);
#pragma unroll
      for (int r = 0; r < R; ++r) {
        const int i = lane + 64 * r;
        if (i == j)
          zr[r] = zj;
        else if (i < j)
          zr[r] -= lj[i] * zj;
      }
    }
#pragma unroll
    for (int r = 0; r < R; ++r)
      if (lane + 64 * r < P) z[lane + 64 * r] = zr[r];
  }
  __syncthreads();

  // 6. update + convergence ------------------------------------------------
  double dm = 0.0, tm = 0.0, tg = 0.0;
  double* tp = a.theta_prev + (int64_t)k * P;
  double* dp = a.delta_prev + (int64_t)k * P;
  for (int f = tid; f < P; f += 256) {
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
  if (a.family == FAMILY_GAUSSIAN) {
    // OLS: theta was 0, one Newton step is the closed form (X^T X)^-1 X^T y;
    // residual sum of squares = y^T y - theta^T X^T y = -2 ll(0) - theta . g
    tg = wave_sum(tg);
    __syncthreads();
    if (lane == 0) red[wid] = tg;
    __syncthreads();
    if (tid == 0) {
      a.loglik[k] = -2.0 * ll - (red[0] + red[1] + red[2] + red[3]);
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
    if (ph == PHASE_F32) {
      if (dm <= a.switch_tol * (1.0 + tm)) ph = PHASE_F64;
    } else if (dm <= a.tol * (1.0 + tm)) {
      a.status[k] = DLSA_STATUS_OK;
      a.phase[k] = PHASE_DONE;
      return;
    }
    a.phase[k] = ph;
    atomicAdd(&a.counters[ph], 1);
  }
}

template <int NT>
static hipError_t launch_solve_t(const SolveArgs& a, int K, size_t lds, hipStream_t s) {
  static bool attr_set = false;
  if (!attr_set) {
    hipError_t e = hipFuncSetAttribute((const void*)newton_solve_kernel<NT>,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    if (e != hipSuccess) return e;
    attr_set = true;
  }
  hipLaunchKernelGGL(newton_solve_kernel<NT>, dim3(K), dim3(256), lds, s, a);
  return hipGetLastError();
}

hipError_t launch_newton_solve(const SolveArgs& a, int K, hipStream_t s) {
  const int PP = 16 * a.NT;
  const size_t lds = ((size_t)a.P * (a.P + 1) / 2 + 2 * PP + 8) * sizeof(double);
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
