// Per-partition Newton update (one 256-thread workgroup per partition).
//
// Replaces the outer Newton step of sklearn's newton-cg solve inside
// dlsa/models.py:110-113 (the reference solves H d = g iteratively by CG with
// 2 passes over X per CG step; here H is assembled once per pass and factored
// in LDS):
//   1. sum the chunk partials of the pass (fixed order -> deterministic),
//      mirror the lower tiles into a full P x P matrix in LDS;
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

__global__ __launch_bounds__(256) void newton_solve_kernel(const SolveArgs a) {
  extern __shared__ __attribute__((aligned(16))) double sm[];
  const int k = blockIdx.x;
  const int tid = threadIdx.x;
  if (a.status[k] != STATUS_RUNNING) return;  // block-uniform
  const int P = a.P, NT = a.NT, PP = 16 * NT;
  const int T = NT * (NT + 1) / 2;
  const int LD = P + 1;
  double* H = sm;            // P x LD
  double* g = H + P * LD;    // PP
  double* z = g + PP;        // PP
  double* red = z + PP;      // 8: [0..3] block reductions, [6] flag, [7] ll

  const int cb = a.part_chunk_begin[k], ce = a.part_chunk_begin[k + 1];
  const int phase = a.phase[k];

  // 1. assemble ------------------------------------------------------------
  for (int e = tid; e < T * 256; e += 256) {
    const int t = e >> 8, within = e & 255;
    int I = 0;
    while ((I + 1) * (I + 2) / 2 <= t) ++I;
    const int J = t - I * (I + 1) / 2;
    const int gi = 16 * I + (within >> 4), gj = 16 * J + (within & 15);
    double s = 0.0;
    for (int c = cb; c < ce; ++c) s += a.slab_H[((int64_t)c * T + t) * 256 + within];
    // lower triangle only (diagonal tiles hold (w x_i) x_j and (w x_j) x_i,
    // which differ in the last bit): mirroring makes Sig_inv exactly symmetric
    if (gi < P && gj < P && gi >= gj) {
      H[gi * LD + gj] = s;
      H[gj * LD + gi] = s;
    }
  }
  for (int f = tid; f < P; f += 256) {
    double s = 0.0;
    for (int c = cb; c < ce; ++c) s += a.slab_g[(int64_t)c * PP + f];
    g[f] = s;
  }
  if (tid == 0) {
    double s = 0.0;
    for (int c = cb; c < ce; ++c) s += a.slab_ll[c];
    red[7] = s;
  }
  __syncthreads();
  const double ll = red[7];
  const int it = a.iters[k];
  double* th = a.theta + (int64_t)k * P;

  if (!isfinite(ll)) {
    if (tid == 0) a.status[k] = DLSA_STATUS_NONFINITE;
    return;
  }

  // 2. step halving on a log-likelihood decrease ---------------------------
  const double llp = a.ll_prev[k];
  // threshold above the fp32-log noise of mixed-mode log-likelihoods; real
  // overshoots of a Newton step lose far more than 1e-6 relative
  if (it > 0 && ll < llp - 1e-6 * (1.0 + fabs(llp)) && a.backtracks[k] < 40) {
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
  double* S = a.sig_inv + (int64_t)k * P * P;
  for (int e = tid; e < P * P; e += 256) S[e] = H[(e / P) * LD + (e % P)];
  if (tid == 0) a.loglik[k] = ll;

  // 4. Cholesky (right-looking, lower, in place) ---------------------------
  if (tid == 0) red[6] = 1.0;
  __syncthreads();
  for (int j = 0; j < P; ++j) {
    if (tid == 0) {
      const double d = H[j * LD + j];
      if (!(d > 0.0) || !isfinite(d)) red[6] = 0.0;
      else H[j * LD + j] = sqrt(d);
    }
    __syncthreads();
    if (red[6] == 0.0) break;
    const double djj = H[j * LD + j];
    for (int i = j + 1 + tid; i < P; i += 256) H[i * LD + j] /= djj;
    __syncthreads();
    const int n = P - j - 1;
    for (int e = tid; e < n * n; e += 256) {
      const int i = j + 1 + e / n, c = j + 1 + e % n;
      if (c <= i) H[i * LD + c] -= H[i * LD + j] * H[c * LD + j];
    }
    __syncthreads();
  }
  if (red[6] == 0.0) {
    if (tid == 0) {
      if (phase == PHASE_F32) {  // fp32 Hessian lost definiteness: redo in fp64
        a.phase[k] = PHASE_F64;
        a.iters[k] = it + 1;
        atomicAdd(&a.counters[PHASE_F64], 1);
      } else {
        a.status[k] = DLSA_STATUS_SINGULAR;
      }
    }
    return;
  }

  // 5. solve L z = g, L^T d = z (d overwrites z) ---------------------------
  for (int f = tid; f < PP; f += 256) z[f] = f < P ? g[f] : 0.0;
  __syncthreads();
  for (int j = 0; j < P; ++j) {
    if (tid == 0) z[j] /= H[j * LD + j];
    __syncthreads();
    const double zj = z[j];
    for (int i = j + 1 + tid; i < P; i += 256) z[i] -= H[i * LD + j] * zj;
    __syncthreads();
  }
  for (int j = P - 1; j >= 0; --j) {
    if (tid == 0) z[j] /= H[j * LD + j];
    __syncthreads();
    const double zj = z[j];
    for (int i = tid; i < j; i += 256) z[i] -= H[j * LD + i] * zj;
    __syncthreads();
  }

  // 6. update + convergence ------------------------------------------------
  double dm = 0.0, tm = 0.0;
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
  }
  dm = block_max(dm, red);
  tm = block_max(tm, red);
  if (a.family == FAMILY_GAUSSIAN) {
    // OLS: theta was 0, one Newton step is the closed form (X^T X)^-1 X^T y;
    // residual sum of squares = y^T y - theta^T X^T y = -2 ll(0) - theta . g
    double tg = 0.0;
    for (int f = tid; f < P; f += 256) tg += th[f] * g[f];
    for (int o = 32; o > 0; o >>= 1) tg += __shfl_xor(tg, o);
    __syncthreads();
    if ((tid & 63) == 0) red[tid >> 6] = tg;
    __syncthreads();
    if (tid == 0) {
      const double s = red[0] + red[1] + red[2] + red[3];
      a.loglik[k] = -2.0 * ll - s;
      a.iters[k] = it + 1;
      a.status[k] = isfinite(dm) ? DLSA_STATUS_OK : DLSA_STATUS_NONFINITE;
      a.phase[k] = PHASE_DONE;
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

hipError_t launch_newton_solve(const SolveArgs& a, int K, hipStream_t s) {
  const int PP = 16 * a.NT;
  const size_t lds = ((size_t)a.P * (a.P + 1) + 2 * PP + 8) * sizeof(double);
  static bool attr_set = false;
  if (!attr_set) {
    hipError_t e = hipFuncSetAttribute((const void*)newton_solve_kernel,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    if (e != hipSuccess) return e;
    attr_set = true;
  }
  hipLaunchKernelGGL(newton_solve_kernel, dim3(K), dim3(256), lds, s, a);
  return hipGetLastError();
}

}  // namespace dlsa
