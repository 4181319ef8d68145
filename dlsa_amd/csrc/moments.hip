// Column moments of a row-major fp64 matrix in HBM: count, mean, M2 (the sum
// of squared deviations), min and max of every column -- the device half of
// Spark's describe(), which the reference computes over the whole data set to
// standardise every partition with the global mean and stddev
// (projects/logistic_dlsa.py:287-298; dlsa/models.py:99-101 reads rows 1
// and 2, mean and stddev with n - 1).
//
// Two passes over X (the two-pass variance numpy / pandas use):
//   1. per row range and column: count, Neumaier-compensated sum, min, max;
//      the ranges merged in index order -> mean = sum / count;
//   2. per row range and column: compensated sum of (x - mean)^2, merged in
//      index order -> M2.
// NaN values are skipped (Spark's describe ignores nulls).  Fixed summation
// order everywhere: the result is bit-identical run to run.  HBM-bound: 8 B
// per element per pass.
#include <math.h>

#include <algorithm>

#include "dlsa_internal.hpp"

namespace dlsa {

namespace {

constexpr int kMomCols = 64;   // columns per workgroup (one per lane)
constexpr int kMomWaves = 4;   // row-interleaved waves per workgroup
constexpr int kMomUnroll = 4;  // rows in flight per wave

// Neumaier: (s, c) += x
__device__ __forceinline__ void neu_add(double& s, double& c, double x) {
  const double t = s + x;
  c += fabs(s) >= fabs(x) ? (s - t) + x : (x - t) + s;
  s = t;
}

// pass 1 (pass2 = false): [count, sum, comp, min, max]; pass 2: [sum, comp] of
// (x - mean)^2.  Grid (row ranges, column blocks), 256 threads.
template <bool PASS2>
__global__ __launch_bounds__(256) void moments_kernel(const double* X, int64_t n, int p,
                                                      int64_t rows_per_range,
                                                      const double* mean, double* part) {
  __shared__ double red[kMomWaves][kMomCols][5];
  const int g = blockIdx.x;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int c = blockIdx.y * kMomCols + lane;
  const bool col = c < p;
  const int64_t r0 = (int64_t)g * rows_per_range;
  const int64_t r1 = min(n, r0 + rows_per_range);
  const double mu = (PASS2 && col) ? mean[c] : 0.0;
  double cnt = 0.0, s = 0.0, cp = 0.0, mn = INFINITY, mx = -INFINITY;
  if (col) {
    int64_t r = r0 + w;
    for (; r + (kMomUnroll - 1) * kMomWaves < r1; r += kMomUnroll * kMomWaves) {
      double v[kMomUnroll];
#pragma unroll
      for (int u = 0; u < kMomUnroll; ++u) v[u] = X[(r + (int64_t)u * kMomWaves) * p + c];
#pragma unroll
      for (int u = 0; u < kMomUnroll; ++u) {
        const double x = v[u];
        if (x == x) {  // not NaN
          if constexpr (PASS2) {
            const double d = x - mu;
            neu_add(s, cp, d * d);
          } else {
            cnt += 1.0;
            neu_add(s, cp, x);
            mn = fmin(mn, x);
            mx = fmax(mx, x);
          }
        }
      }
    }
    for (; r < r1; r += kMomWaves) {
      const double x = X[r * p + c];
      if (x == x) {
        if constexpr (PASS2) {
          const double d = x - mu;
          neu_add(s, cp, d * d);
        } else {
          cnt += 1.0;
          neu_add(s, cp, x);
          mn = fmin(mn, x);
          mx = fmax(mx, x);
        }
      }
    }
  }
  red[w][lane][0] = cnt;
  red[w][lane][1] = s;
  red[w][lane][2] = cp;
  red[w][lane][3] = mn;
  red[w][lane][4] = mx;
  __syncthreads();
  if (w == 0 && col) {  // waves merged in index order
    double tc = 0.0, ts = 0.0, tcp = 0.0, tmn = INFINITY, tmx = -INFINITY;
#pragma unroll
    for (int k = 0; k < kMomWaves; ++k) {
      tc += red[k][lane][0];
      neu_add(ts, tcp, red[k][lane][1]);
      tcp += red[k][lane][2];
      tmn = fmin(tmn, red[k][lane][3]);
      tmx = fmax(tmx, red[k][lane][4]);
    }
    double* o = part + ((int64_t)g * p + c) * 5;
    o[0] = tc;
    o[1] = ts;
    o[2] = tcp;
    o[3] = tmn;
    o[4] = tmx;
  }
}

// Merge the row ranges of every column in index order.  pass 1 -> stats
// [count, mean, min, max] (mean into `mean`); pass 2 -> out [5, p] =
// count, mean, M2, min, max.
template <bool PASS2>
__global__ void moments_merge_kernel(const double* part, int G, int p, double* mean,
                                     double* stats, double* out) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= p) return;
  double tc = 0.0, ts = 0.0, tcp = 0.0, tmn = INFINITY, tmx = -INFINITY;
  for (int g = 0; g < G; ++g) {
    const double* o = part + ((int64_t)g * p + c) * 5;
    tc += o[0];
    neu_add(ts, tcp, o[1]);
    tcp += o[2];
    tmn = fmin(tmn, o[3]);
    tmx = fmax(tmx, o[4]);
  }
  if constexpr (!PASS2) {
    const double m = tc > 0.0 ? (ts + tcp) / tc : NAN;
    mean[c] = m;
    stats[4 * c + 0] = tc;
    stats[4 * c + 1] = m;
    stats[4 * c + 2] = tc > 0.0 ? tmn : NAN;
    stats[4 * c + 3] = tc > 0.0 ? tmx : NAN;
  } else {
    out[0 * p + c] = stats[4 * c + 0];
    out[1 * p + c] = stats[4 * c + 1];
    out[2 * p + c] = stats[4 * c + 0] > 0.0 ? ts + tcp : NAN;
    out[3 * p + c] = stats[4 * c + 2];
    out[4 * p + c] = stats[4 * c + 3];
  }
}

}  // namespace

hipError_t launch_column_moments(const double* X, int64_t n, int p, double* out, double* ws,
                                 int G, int64_t rows_per_range, hipStream_t s) {
  double* part = ws;                        // [G][p][5]
  double* mean = part + (int64_t)G * p * 5;  // [p]
  double* stats = mean + p;                 // [p][4]
  const dim3 grid(G, (p + kMomCols - 1) / kMomCols);
  hipLaunchKernelGGL(moments_kernel<false>, grid, dim3(256), 0, s, X, n, p, rows_per_range,
                     (const double*)nullptr, part);
  hipLaunchKernelGGL(moments_merge_kernel<false>, dim3((p + 255) / 256), dim3(256), 0, s, part, G,
                     p, mean, stats, (double*)nullptr);
  hipLaunchKernelGGL(moments_kernel<true>, grid, dim3(256), 0, s, X, n, p, rows_per_range,
                     (const double*)mean, part);
  hipLaunchKernelGGL(moments_merge_kernel<true>, dim3((p + 255) / 256), dim3(256), 0, s, part, G,
                     p, mean, stats, out);
  return hipGetLastError();
}

// row ranges: enough workgroups to fill the chip (>= ~4096 with the column
// blocks), at least 1024 rows each
void column_moments_plan(int64_t n, int p, int* G, int64_t* rows_per_range) {
  const int cb = (p + kMomCols - 1) / kMomCols;
  int64_t g = std::max<int64_t>(1, 4096 / cb);
  g = std::min<int64_t>(g, std::max<int64_t>(1, (n + 1023) / 1024));
  const int64_t rpr = std::max<int64_t>(1, (n + g - 1) / g);
  *G = (int)std::max<int64_t>(1, (n + rpr - 1) / rpr);
  *rows_per_range = rpr;
}

}  // namespace dlsa
