// OLS pass (BASELINE config 4: the closed-form Gram + X^T y of the reference's
// linear-model path, projects/results/linear_regression_dc.py:27-37) streaming
// X straight from HBM into the MFMA operand registers.
//
// The OLS fit is one pass at theta = 0 (fit_impl: max_iter 1, no warm start):
// w = 1, r = y, so a row needs no eta, no exp / log and no weight -- only
// X^T X (fp64 MFMA), X^T y and -y^2 / 2.  The per-wave LDS-DMA kernel
// (irls_wave_impl.hpp) staged every 8-row block through an LDS ring, at a
// cost in DMA issues (~100 cycles each in a busy wave), barriers and LDS
// reads that no fp64-MFMA work hides (fp64 VALU never co-executes with it):
// 14.9-15.3 ms per 1.25e8 x 64 pass = 4.3 TB/s.  Here each wave owns one chunk
// and loads its rows directly in the 16x16x4 f64 MFMA operand layout -- lane
// (fl = l & 15, q = l >> 4) reads x[row q][16 c + fl] for every tile column c,
// four rows x 128 contiguous bytes per instruction -- KS k-steps (4 rows each)
// of loads issued together, every load unconditional (rows past the chunk
// re-read its last row and are selected away: a predicated load gets a
// branch region and a vmcnt(0) of its own).  No LDS, no barriers, no DMA
// issue; the waves of a workgroup are independent chunks.  The tiles, X^T y
// and the log-likelihood go to the chunk's slab exactly as the other passes
// write them (newton_solve.hip sums a partition's chunks in fixed order).
#include "dlsa_internal.hpp"

// OLS pass by this kernel (1) or by the per-wave LDS-DMA kernel (0, A/B)
#ifndef DLSA_OLS_STREAM
#define DLSA_OLS_STREAM 1
#endif

namespace dlsa {

namespace {

typedef double d4o __attribute__((ext_vector_type(4)));
constexpr int kOlsWaves = 4;  // independent waves (chunks) per workgroup

// FULL: no intercept and p = 16 NT (every lane's features are columns of X,
// config 4): full row groups take their operands as loaded, no selects
template <int NT, int KS, bool STD, bool FULL>
__global__ __launch_bounds__(64 * kOlsWaves) void ols_stream_kernel(const PassArgs a, int n_chunks) {
  constexpr int T = NT * (NT + 1) / 2, PMAX = 16 * NT;
  const int lane = threadIdx.x & 63;
  const int chunk = blockIdx.x * kOlsWaves + (int)(threadIdx.x >> 6);  // wave-uniform
  if (chunk >= n_chunks) return;
  const int part = a.chunk_part[chunk];
  if (a.phase[part] != a.want_phase) return;
  const int64_t row0 = a.chunk_row0[chunk];
  const int nrows = a.chunk_rows[chunk];
  if (nrows <= 0) return;
  const int p = a.p, ic = a.intercept;
  const int fl = lane & 15, q = lane >> 4;

  // this lane's feature of tile column c: f = 16 c + fl, column f - ic of X
  int col[NT];
  bool fin[NT];
  double cen[NT], isc[NT];
#pragma unroll
  for (int c = 0; c < NT; ++c) {
    const int j = 16 * c + fl - ic;
    fin[c] = j >= 0 && j < p;
    col[c] = fin[c] ? j : 0;
    cen[c] = 0.0;
    isc[c] = 1.0;
    if constexpr (STD) {
      if (fin[c]) {
        cen[c] = a.center[j];
        isc[c] = 1.0 / a.scale[j];
      }
    }
  }
  const bool icpt = ic && fl == 0;  // feature 0 (c = 0) is the intercept column

  d4o acc[T];
#pragma unroll
  for (int t = 0; t < T; ++t) acc[t] = d4o{0.0, 0.0, 0.0, 0.0};
  double gacc[NT];
#pragma unroll
  for (int c = 0; c < NT; ++c) gacc[c] = 0.0;
  double ll = 0.0;

  const double* X = a.X + row0 * p;
  const double* Y = a.y + row0;
  // one group of KS k-steps (4 rows each) from row r0.  The fp64 MFMAs bound
  // this pass (10 x ~70 cycles per 4 rows at P = 64) and fp64 VALU work never
  // overlaps them, so the per-value work is one select (FULL: every lane's
  // feature is a column of X; rows past the chunk -> 0).  (A separate
  // select-free body for whole groups made the compiler copy the T x 4
  // accumulators AGPR <-> VGPR every group.)
  for (int r0 = 0; r0 < nrows; r0 += 4 * KS) {
    double xv[KS][NT], yv[KS];
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      const int rr = min(r0 + 4 * s + q, nrows - 1);
      const double* xr = X + (int64_t)rr * p;
#pragma unroll
      for (int c = 0; c < NT; ++c) xv[s][c] = xr[col[c]];
      yv[s] = Y[rr];
    }
#pragma unroll
    for (int s = 0; s < KS; ++s) {
#pragma unroll
      for (int c = 0; c < NT; ++c) asm volatile("" : "+v"(xv[s][c]));
      asm volatile("" : "+v"(yv[s]));
    }
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      const bool valid = r0 + 4 * s + q < nrows;
      double v[NT];
#pragma unroll
      for (int c = 0; c < NT; ++c) {
        double x = xv[s][c];
        if constexpr (STD) x = (x - cen[c]) * isc[c];
        if constexpr (FULL) {
          v[c] = valid ? x : 0.0;
        } else {
          const bool one = c == 0 && icpt;
          v[c] = valid && (fin[c] || one) ? (one ? 1.0 : x) : 0.0;
        }
      }
      const double y = valid ? yv[s] : 0.0;
#pragma unroll
      for (int c = 0; c < NT; ++c) gacc[c] = fma(v[c], y, gacc[c]);
      if (fl == 0) ll = fma(-0.5 * y, y, ll);  // each row once (lane fl = 0 of its group)
#pragma unroll
      for (int I = 0; I < NT; ++I)
#pragma unroll
        for (int J = 0; J <= I; ++J)
          acc[I * (I + 1) / 2 + J] = __builtin_amdgcn_mfma_f64_16x16x4f64(
              v[I], v[J], acc[I * (I + 1) / 2 + J], 0, 0, 0);
    }
  }

  // ---- epilogue: the chunk's slab (f64 16x16x4 C/D map: row q + 4 r, column fl)
  double* sH = a.slab_H + (int64_t)chunk * T * 256;
#pragma unroll
  for (int t = 0; t < T; ++t)
#pragma unroll
    for (int r = 0; r < 4; ++r) sH[t * 256 + (q + 4 * r) * 16 + fl] = acc[t][r];
#pragma unroll
  for (int c = 0; c < NT; ++c) {
    double g = gacc[c];
    g += __shfl_xor(g, 16);
    g += __shfl_xor(g, 32);
    if (q == 0) a.slab_g[(int64_t)chunk * PMAX + 16 * c + fl] = g;
  }
#pragma unroll
  for (int o = 16; o < 64; o <<= 1) ll += __shfl_xor(ll, o);
  if (lane == 0) a.slab_ll[chunk] = ll;
}

template <int NT>
hipError_t launch_ols_nt(const PassArgs& a, bool standardize, int n_chunks, hipStream_t s) {
  constexpr int KS = NT <= 2 ? 8 : 4;
  const dim3 grid((n_chunks + kOlsWaves - 1) / kOlsWaves), block(64 * kOlsWaves);
  const bool full = a.intercept == 0 && a.p == 16 * NT;
  if (standardize) {
    if (full)
      hipLaunchKernelGGL((ols_stream_kernel<NT, KS, true, true>), grid, block, 0, s, a, n_chunks);
    else
      hipLaunchKernelGGL((ols_stream_kernel<NT, KS, true, false>), grid, block, 0, s, a, n_chunks);
  } else {
    if (full)
      hipLaunchKernelGGL((ols_stream_kernel<NT, KS, false, true>), grid, block, 0, s, a, n_chunks);
    else
      hipLaunchKernelGGL((ols_stream_kernel<NT, KS, false, false>), grid, block, 0, s, a, n_chunks);
  }
  return hipGetLastError();
}

}  // namespace

bool ols_stream_applies(int NT) { return DLSA_OLS_STREAM && NT >= 1 && NT <= 4; }

hipError_t launch_ols_stream(const PassArgs& a, int NT, bool standardize, int n_chunks,
                             hipStream_t s) {
  if (n_chunks <= 0) return hipSuccess;
  switch (NT) {
    case 1: return launch_ols_nt<1>(a, standardize, n_chunks, s);
    case 2: return launch_ols_nt<2>(a, standardize, n_chunks, s);
    case 3: return launch_ols_nt<3>(a, standardize, n_chunks, s);
    case 4: return launch_ols_nt<4>(a, standardize, n_chunks, s);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace dlsa
