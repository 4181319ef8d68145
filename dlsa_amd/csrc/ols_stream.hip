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
// each k-step group loaded then computed (0), or the next group's loads in
// flight under the current group's MFMAs in a second register set (1, A/B).
// Round 6, config 4, alternated: two sets measured 12.08-12.44 ms per pass at
// KS = 2 / 3 / 4 and 12.7 at 6, one set (KS = 8) 12.06-12.11
// (profiles/r06q_ols_prefetch_ab.txt): with 2-3 waves per SIMD the loads of
// one wave already run under the other waves' MFMAs
#ifndef DLSA_OLS_PF
#define DLSA_OLS_PF 0
#endif

namespace dlsa {

namespace {

typedef double d4o __attribute__((ext_vector_type(4)));
constexpr int kOlsWaves = 4;  // independent waves (chunks) per workgroup

// Buffer resource over [base, base + bytes) with every word wave-uniform
// (readfirstlane: the loads take it in SGPRs).  Loads past `bytes` return 0.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t ols_rsrc(const void* base, uint32_t bytes) {
  const uint64_t b = (uint64_t)(uintptr_t)base;
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)b);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(b >> 32));
  const uint32_t nr = __builtin_amdgcn_readfirstlane(bytes);
  return __builtin_amdgcn_make_buffer_rsrc((void*)(((uint64_t)hi << 32) | lo), (short)0, (int)nr,
                                           0x00020000);
}

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

  // the chunk's rows as bounds-checked buffers: rows past the chunk read 0, so
  // x, y (and with them the MFMA products, X^T y and y^2) vanish there without
  // a select; the lane's byte offset in a row group is a constant VGPR and the
  // group's row offset an SGPR -- no per-load address arithmetic
  const __amdgpu_buffer_rsrc_t xr = ols_rsrc(a.X + row0 * p, (uint32_t)nrows * p * 8);
  const __amdgpu_buffer_rsrc_t yr = ols_rsrc(a.y + row0, (uint32_t)nrows * 8);
  int voff[NT];
#pragma unroll
  for (int c = 0; c < NT; ++c) voff[c] = (q * p + col[c]) * 8;
  // one group of KS k-steps (4 rows each) from row r0.  The fp64 MFMAs bound
  // this pass (10 x ~70 cycles per 4 rows at P = 64) and fp64 VALU work never
  // overlaps them: FULL groups (every lane's feature a column of X) feed the
  // loaded values to the MFMAs as they are; otherwise one select per value
  // (padding features, the intercept column, rows past the chunk).
  auto load_group = [&](int r0, double (&xv)[KS][NT], double (&yv)[KS]) {
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      const int so = __builtin_amdgcn_readfirstlane((r0 + 4 * s) * p * 8);
#pragma unroll
      for (int c = 0; c < NT; ++c)
        xv[s][c] = __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(xr, voff[c], so, 0));
      yv[s] = __builtin_bit_cast(
          double, __builtin_amdgcn_raw_buffer_load_b64(yr, q * 8, __builtin_amdgcn_readfirstlane((r0 + 4 * s) * 8), 0));
    }
  };
  auto compute_group = [&](int r0, const double (&xv)[KS][NT], const double (&yv)[KS]) {
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      // (a row past the chunk loads 0, which standardisation would shift)
      const bool valid = (FULL && !STD) || r0 + 4 * s + q < nrows;
      double v[NT];
#pragma unroll
      for (int c = 0; c < NT; ++c) {
        double x = xv[s][c];
        if constexpr (STD) x = (x - cen[c]) * isc[c];
        if constexpr (FULL && !STD) {
          v[c] = x;
        } else {
          const bool one = c == 0 && icpt;
          v[c] = valid && (fin[c] || one) ? (one ? 1.0 : x) : 0.0;
        }
      }
      const double y = yv[s];  // 0 past the chunk
#pragma unroll
      for (int c = 0; c < NT; ++c) gacc[c] = fma(v[c], y, gacc[c]);
      ll = fma(-0.5 * y, y, ll);  // each row in its 16 lanes: the sum is scaled by 1/16
#pragma unroll
      for (int I = 0; I < NT; ++I)
#pragma unroll
        for (int J = 0; J <= I; ++J)
          acc[I * (I + 1) / 2 + J] = __builtin_amdgcn_mfma_f64_16x16x4f64(
              v[I], v[J], acc[I * (I + 1) / 2 + J], 0, 0, 0);
    }
  };
  constexpr int GR = 4 * KS;  // rows per group
#if DLSA_OLS_PF
  // two register sets: the next group's loads are in flight while the
  // current group's MFMAs run (the loop is unrolled by two, so no register
  // copies cross the back edge; no early exit, which made the compiler keep a
  // second set of accumulators).  A group past the chunk loads 0 from the
  // bounds-checked buffers and adds zeros (masked when not FULL), in the
  // single-set loop's accumulation order
  double xa[KS][NT], ya[KS], xb[KS][NT], yb[KS];
  load_group(0, xa, ya);
  for (int r0 = 0; r0 < nrows; r0 += 2 * GR) {
    load_group(r0 + GR, xb, yb);
    compute_group(r0, xa, ya);
    load_group(r0 + 2 * GR, xa, ya);
    compute_group(r0 + GR, xb, yb);
  }
#else
  for (int r0 = 0; r0 < nrows; r0 += GR) {
    double xv[KS][NT], yv[KS];
    load_group(r0, xv, yv);
    compute_group(r0, xv, yv);
  }
#endif

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
  for (int o = 1; o < 64; o <<= 1) ll += __shfl_xor(ll, o);
  if (lane == 0) a.slab_ll[chunk] = ll * 0.0625;  // 16 lanes per row (exact: a power of 2)
}

// k-steps (4 rows each) whose loads are issued together.  At NT = 4 (config
// 4), 8 (2 waves per SIMD, 32 rows of loads in flight per wave) measured
// 11.96-12.26 ms per pass against 12.18-12.34 for 4 (3 waves per SIMD),
// 12.25-12.31 for 12 and 12.3-12.6 for 2 (4 waves per SIMD); 16 measured
// 13.5 ms (profiles/r05ok_ols_ks_sweep.jsonl).  DLSA_OLS_KS: A/B builds.
#ifndef DLSA_OLS_KS
#define DLSA_OLS_KS 8
#endif
template <int NT>
hipError_t launch_ols_nt(const PassArgs& a, bool standardize, int n_chunks, hipStream_t s) {
  constexpr int KS = DLSA_OLS_KS;
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
