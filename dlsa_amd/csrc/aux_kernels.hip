// Small kernels around the fused pass: fit state init/finalise, the local
// partition reduction (dlsa/dlsa.py:30-34 group-sum, done in HBM before the
// RCCL all-reduce) and the synthetic data generator.
#include <math.h>

#include "dlsa_internal.hpp"

namespace dlsa {

__global__ void fit_init_kernel(const int64_t* offsets, int K, int P, int start_phase,
                                double* theta, int32_t* phase, int32_t* backtracks,
                                int32_t* iters, int32_t* status, double* ll_prev,
                                double* sig_inv, double* loglik) {
  const int k = blockIdx.x;
  const bool empty = offsets[k + 1] <= offsets[k];
  for (int f = threadIdx.x; f < P; f += blockDim.x) theta[(int64_t)k * P + f] = 0.0;
  for (int e = threadIdx.x; e < P * P; e += blockDim.x) sig_inv[(int64_t)k * P * P + e] = 0.0;
  if (threadIdx.x == 0) {
    phase[k] = empty ? PHASE_DONE : start_phase;
    backtracks[k] = 0;
    iters[k] = 0;
    status[k] = empty ? DLSA_STATUS_EMPTY : STATUS_RUNNING;
    ll_prev[k] = -INFINITY;
    loglik[k] = 0.0;
  }
}

hipError_t launch_fit_init(const int64_t* offsets_dev, int K, int P, int start_phase,
                           double* theta, int32_t* phase, int32_t* backtracks, int32_t* iters,
                           int32_t* status, double* ll_prev, double* sig_inv, double* loglik,
                           hipStream_t s) {
  hipLaunchKernelGGL(fit_init_kernel, dim3(K), dim3(256), 0, s, offsets_dev, K, P, start_phase,
                     theta, phase, backtracks, iters, status, ll_prev, sig_inv, loglik);
  return hipGetLastError();
}

// Start of a warm-start level: running partitions re-enter the Newton loop
// (the log-likelihood scale changes with the row count), non-finite iterates
// restart from 0; counters[phase] = partitions running.
__global__ void level_reset_kernel(int K, int P, int start_phase, int32_t* phase,
                                   int32_t* status, double* ll_prev, int32_t* backtracks,
                                   double* theta, int32_t* counters) {
  for (int k = blockIdx.x * blockDim.x + threadIdx.x; k < K; k += gridDim.x * blockDim.x) {
    if (status[k] != STATUS_RUNNING) continue;
    bool finite = true;
    for (int f = 0; f < P; ++f) finite &= (bool)isfinite(theta[(int64_t)k * P + f]);
    if (!finite)
      for (int f = 0; f < P; ++f) theta[(int64_t)k * P + f] = 0.0;
    phase[k] = start_phase;
    ll_prev[k] = -INFINITY;
    backtracks[k] = 0;
    atomicAdd(&counters[start_phase], 1);
  }
}

hipError_t launch_level_reset(int K, int P, int start_phase, int32_t* phase, int32_t* status,
                              double* ll_prev, int32_t* backtracks, double* theta,
                              int32_t* counters, hipStream_t s) {
  hipLaunchKernelGGL(level_reset_kernel, dim3((K + 255) / 256), dim3(256), 0, s, K, P,
                     start_phase, phase, status, ll_prev, backtracks, theta, counters);
  return hipGetLastError();
}

// Polish pass of a budget that ran out: every still-running partition gets
// one exact pass at the theta it returns, whose X^T W X is published as
// Sig_inv -- models.py:114,130 evaluate the weights at whatever coef sklearn
// stopped at.  counters[PHASE_F64] = partitions marked.
__global__ void polish_mark_kernel(int K, int32_t* phase, const int32_t* status,
                                   int32_t* counters) {
  for (int k = blockIdx.x * blockDim.x + threadIdx.x; k < K; k += gridDim.x * blockDim.x) {
    if (status[k] != STATUS_RUNNING) continue;
    phase[k] = PHASE_F64;
    atomicAdd(&counters[PHASE_F64], 1);
  }
}

hipError_t launch_polish_mark(int K, int32_t* phase, const int32_t* status, int32_t* counters,
                              hipStream_t s) {
  hipLaunchKernelGGL(polish_mark_kernel, dim3((K + 255) / 256), dim3(256), 0, s, K, phase, status,
                     counters);
  return hipGetLastError();
}

// sig_inv_theta = Sig_inv @ theta (models.py:131); still-running -> MAXITER.
// Sig_inv_theta[k] = Sig_inv[k] theta[k].  Grid (K, ceil(P / 16)): wave w of
// workgroup (k, y) takes rows 16 y + w + 4 r; a row is read coalesced (lane
// j + 64 m) against theta in LDS and summed by a fixed butterfly, so the
// result is the same run to run.  (One thread per row walked its row with a
// P-long dependent chain of strided loads: 0.27 ms per fit at P = 500, K = 32.)
__global__ __launch_bounds__(256) void fit_finalize_kernel(int K, int P, const double* theta,
                                                           const double* sig_inv,
                                                           double* sig_inv_theta, int32_t* status) {
  __shared__ double th[DLSA_MAX_P];
  const int k = blockIdx.x;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const double* S = sig_inv + (int64_t)k * P * P;
  for (int j = threadIdx.x; j < P; j += 256) th[j] = theta[(int64_t)k * P + j];
  __syncthreads();
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int i = 16 * blockIdx.y + wid + 4 * r;  // wave-uniform
    if (i >= P) break;
    const double* Si = S + (int64_t)i * P;
    double acc = 0.0;
    for (int j = lane; j < P; j += 64) acc = fma(Si[j], th[j], acc);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o);
    if (lane == 0) sig_inv_theta[(int64_t)k * P + i] = acc;
  }
  if (blockIdx.y == 0 && threadIdx.x == 0 && status[k] == STATUS_RUNNING)
    status[k] = DLSA_STATUS_MAXITER;
}

hipError_t launch_fit_finalize(int K, int P, const double* theta, const double* sig_inv,
                               double* sig_inv_theta, int32_t* status, hipStream_t s) {
  if (K <= 0 || P <= 0) return hipSuccess;
  if (P > DLSA_MAX_P) return hipErrorInvalidValue;
  hipLaunchKernelGGL(fit_finalize_kernel, dim3(K, (P + 15) / 16), dim3(256), 0, s, K, P, theta,
                     sig_inv, sig_inv_theta, status);
  return hipGetLastError();
}

// theta_rec[k] = theta[k] for the partitions whose phase is ph: the point at
// which the next bf16 pass records their Ozaki digit scales
// gate: null, or the snapshot is taken only if gate[0] > 0 (the pass it
// belongs to records max |z| under the same condition, PassArgs::zrec_gate)
__global__ void theta_snapshot_kernel(int K, int P, const int32_t* phase, int ph,
                                      const double* theta, double* theta_rec, const int32_t* gate) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (int64_t)K * P) return;
  if (gate && gate[0] <= 0) return;
  if (phase[i / P] == ph) theta_rec[i] = theta[i];
}

hipError_t launch_theta_snapshot(int K, int P, const int32_t* phase, int ph, const double* theta,
                                 double* theta_rec, hipStream_t s, const int32_t* gate) {
  const int64_t n = (int64_t)K * P;
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(theta_snapshot_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, K,
                     P, phase, ph, theta, theta_rec, gate);
  return hipGetLastError();
}

// out = [sum_k Sig_inv_k | sum_k Sig_inv_k theta_k | sum_k theta_k | K]
// One thread per output element, partitions summed in index order.  The
// loads run 16 partitions ahead of the (sequential, order-preserving) adds:
// one dependent HBM round trip per partition made this 0.47 ms at K = 1024,
// P = 100 (40 workgroups, latency-bound).
template <int U>
__device__ __forceinline__ double ordered_sum(const double* __restrict__ a, int64_t stride, int K) {
  double s = 0.0;
  int k = 0;
  for (; k + U <= K; k += U) {
    double v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = __builtin_nontemporal_load(a + (int64_t)(k + u) * stride);
#pragma unroll
    for (int u = 0; u < U; ++u) s += v[u];
  }
  for (; k < K; ++k) s += a[(int64_t)k * stride];
  return s;
}

__global__ void reduce_partitions_kernel(const double* sig_inv, const double* sig_inv_theta,
                                         const double* theta, int K, int P, double* out) {
  const int64_t PP2 = (int64_t)P * P;
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e < PP2) {
    out[e] = ordered_sum<16>(sig_inv + e, PP2, K);
  } else if (e < PP2 + P) {
    out[e] = ordered_sum<16>(sig_inv_theta + (e - PP2), P, K);
  } else if (e < PP2 + 2 * P) {
    out[e] = ordered_sum<16>(theta + (e - PP2 - P), P, K);
  } else if (e == PP2 + 2 * P) {
    out[e] = (double)K;
  }
}

hipError_t launch_reduce_partitions(const double* sig_inv, const double* sig_inv_theta,
                                    const double* theta, int K, int P, double* out,
                                    hipStream_t s) {
  const int64_t n = (int64_t)P * P + 2 * P + 1;
  const int threads = 64;  // P = 100: 158 one-wave workgroups instead of 40
  const int blocks = (int)((n + threads - 1) / threads);
  hipLaunchKernelGGL(reduce_partitions_kernel, dim3(blocks), dim3(threads), 0, s, sig_inv,
                     sig_inv_theta, theta, K, P, out);
  return hipGetLastError();
}

// ---- synthetic data: counter-based splitmix64 streams -----------------------
// X[i, j] = u(seed, (row0 + i) * p + j) - 0.5, y[i] = u(seed ^ kYSalt, row0 + i) <
// sigmoid(sum_{j < floor(0.4 p)} X[i, j]).  oracle/dlsa_oracle.py:simulate_counter
// restates it bit for bit.
__device__ __forceinline__ double u01(uint64_t seed, uint64_t ctr) {
  uint64_t z = seed + (ctr + 1) * 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  z ^= z >> 31;
  return (double)(z >> 11) * 0x1.0p-53;
}
constexpr uint64_t kYSalt = 0x5DEECE66Dull;

__global__ void simulate_x_kernel(double* X, int64_t n, int p, uint64_t seed, int64_t row0) {
  const int64_t total = n * p;
  const int64_t base = row0 * p;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total;
       e += (int64_t)gridDim.x * blockDim.x)
    X[e] = u01(seed, (uint64_t)(base + e)) - 0.5;
}

__global__ void simulate_y_kernel(const double* X, double* y, int64_t n, int p, uint64_t seed,
                                  int64_t row0) {
  const int p1 = (int)(p * 0.4);
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    double eta = 0.0;
    for (int j = 0; j < p1; ++j) eta = eta + X[i * p + j];
    const double prob = 1.0 / (1.0 + exp(-eta));
    y[i] = u01(seed ^ kYSalt, (uint64_t)(row0 + i)) < prob ? 1.0 : 0.0;
  }
}

hipError_t launch_simulate(double* X, double* y, int64_t n, int p, uint64_t seed, int64_t row0,
                           hipStream_t s) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(simulate_x_kernel, dim3(8192), dim3(256), 0, s, X, n, p, seed, row0);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(simulate_y_kernel, dim3(4096), dim3(256), 0, s, X, y, n, p, seed, row0);
  return hipGetLastError();
}

}  // namespace dlsa
