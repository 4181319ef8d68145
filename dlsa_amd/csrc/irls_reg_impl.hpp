// Register-streaming fused IRLS pass (gfx950 / CDNA4) -- kernel template,
// instantiated by irls_reg_g*.hip (one translation unit per group of NT).
//
// Replaces, per Newton iteration, the per-partition work of the reference map
// stage (sklearn newton-cg Hessian-vector passes, predict_proba and
// Sig_inv = X^T diag(p(1-p)) X, dlsa/models.py:110-131) with ONE pass over X.
//
// One wave = one chunk of consecutive rows of one partition; no LDS, no
// barriers.  For a k-step of 4 rows lane l loads X[row 4s + (l >> 4)]
// [feature 16c + (l & 15)] for every column tile c straight from HBM into
// registers (16 lanes = 128 contiguous bytes of one row): that IS the A/B
// operand map of the 16x16x4 MFMA with K = rows, so tile (I, J) of X^T W X
// is mfma(w x[I], x[J], acc) with no data movement.  U k-steps of loads are
// kept in flight (a ring of register slots), and the wave owns all
// NT (NT + 1) / 2 lower-triangle accumulators (fp64: 8 AGPRs per tile), so
// the logistic row work of k-step s+1 (eta = x.theta, a 16-lane DPP
// reduction, w, r, log-lik, gradient) can issue while the MFMAs of k-step s
// run.  Measured against the LDS-staged kernels this is the structure of
// the wide-path Gram kernel that reaches ~76 TFLOP/s fp64.
#pragma once

#include "dlsa_internal.hpp"

namespace dlsa {

typedef double d4r __attribute__((ext_vector_type(4)));
typedef float f4r __attribute__((ext_vector_type(4)));

namespace {

template <int CTRL>
__device__ __forceinline__ double dpp_f64r(double v) {
  const int lo = __builtin_amdgcn_mov_dpp(__double2loint(v), CTRL, 0xF, 0xF, false);
  const int hi = __builtin_amdgcn_mov_dpp(__double2hiint(v), CTRL, 0xF, 0xF, false);
  return __hiloint2double(hi, lo);
}

// Sum over the 16 lanes of a row (row_ror 8, 4, 2, 1); every lane of the row
// ends with the bitwise-identical total.
__device__ __forceinline__ double red16r(double v) {
  v += dpp_f64r<0x128>(v);
  v += dpp_f64r<0x124>(v);
  v += dpp_f64r<0x122>(v);
  v += dpp_f64r<0x121>(v);
  return v;
}

}  // namespace

template <int NT, bool F64, bool STD, int FAM>
__global__ __launch_bounds__(64) void irls_reg_kernel(const PassArgs a) {
  constexpr int T = NT * (NT + 1) / 2;
  constexpr int U = F64 ? 4 : 4;  // k-steps of loads in flight
  const int chunk = blockIdx.x;
  const int part = a.chunk_part[chunk];
  if (a.phase[part] != a.want_phase) return;  // wave-uniform

  const int lane = threadIdx.x;
  const int fl = lane & 15, q = lane >> 4;
  const int p = a.p, P = a.P, ic = a.intercept;
  const int64_t row0 = a.chunk_row0[chunk];
  const int nrows = a.chunk_rows[chunk];
  const int nsteps = (nrows + 3) >> 2;

  // per-lane feature constants: lane fl holds feature f = 16 c + fl of its row
  double beta[NT], cen[STD ? NT : 1], isd[STD ? NT : 1];
  int col[NT];
  bool inr[NT];
#pragma unroll
  for (int c = 0; c < NT; ++c) {
    const int f = 16 * c + fl;
    const int j = f - ic;
    inr[c] = j >= 0 && j < p;
    col[c] = inr[c] ? j : 0;
    beta[c] = (f < P) ? a.theta[(int64_t)part * P + f] : 0.0;
    if constexpr (STD) {
      cen[c] = inr[c] ? a.center[j] : 0.0;
      isd[c] = inr[c] ? 1.0 / a.scale[j] : 1.0;
    }
  }
  const bool icpt_lane = ic && fl == 0;

  d4r accd[F64 ? T : 1];
  f4r accf[F64 ? 1 : T];
#pragma unroll
  for (int t = 0; t < (F64 ? T : 1); ++t) accd[t] = d4r{0.0, 0.0, 0.0, 0.0};
#pragma unroll
  for (int t = 0; t < (F64 ? 1 : T); ++t) accf[t] = f4r{0.f, 0.f, 0.f, 0.f};
  double gacc[NT];
#pragma unroll
  for (int c = 0; c < NT; ++c) gacc[c] = 0.0;
  double llacc = 0.0;

  double xb[U][NT], yb[U];
  auto load = [&](int u, int s) {
    int r = 4 * s + q;
    r = r < nrows ? r : nrows - 1;  // in-chunk address; weight zeroed below
    const double* xr = a.X + (row0 + r) * (int64_t)p;
#pragma unroll
    for (int c = 0; c < NT; ++c) xb[u][c] = __builtin_nontemporal_load(xr + col[c]);
    yb[u] = __builtin_nontemporal_load(a.y + row0 + r);
  };

  auto compute = [&](int u, int s) {
    const bool valid = 4 * s + q < nrows;
    double xf[NT];
#pragma unroll
    for (int c = 0; c < NT; ++c) {
      double v = inr[c] ? xb[u][c] : 0.0;
      if constexpr (STD) v = (v - cen[c]) * isd[c];
      xf[c] = v;
    }
    if (icpt_lane) xf[0] = 1.0;
    double e = 0.0;
#pragma unroll
    for (int c = 0; c < NT; ++c) e = fma(xf[c], beta[c], e);
    e = red16r(e);
    const double yv = yb[u];
    double w, r;
    if constexpr (FAM == FAMILY_LOGISTIC) {
      const double ea = exp(-fabs(e));
      const double inv = 1.0 / (1.0 + ea);
      const double mu = e >= 0.0 ? inv : ea * inv;
      w = ea * inv * inv;  // mu (1 - mu), cancellation free
      r = yv - mu;
      if (valid && fl == 0) {
        // exact fp64 log-likelihood in the fp64 pass (its value is returned);
        // fp32 log in the approximate passes (only drives step halving)
        const double sp = F64 ? log1p(ea) : (double)__logf(1.0f + (float)ea);
        llacc += yv * e - (fmax(e, 0.0) + sp);
      }
    } else {  // gaussian (OLS): mu = eta, w = 1, ll = -rss/2
      w = 1.0;
      r = yv - e;
      if (valid && fl == 0) llacc -= 0.5 * r * r;
    }
    if (!valid) {
      w = 0.0;
      r = 0.0;
    }
#pragma unroll
    for (int c = 0; c < NT; ++c) gacc[c] = fma(xf[c], r, gacc[c]);
    if constexpr (F64) {
      double af[NT];
#pragma unroll
      for (int c = 0; c < NT; ++c) af[c] = xf[c] * w;
#pragma unroll
      for (int I = 0; I < NT; ++I)
#pragma unroll
        for (int J = 0; J <= I; ++J) {
          const int t = I * (I + 1) / 2 + J;
          accd[t] = __builtin_amdgcn_mfma_f64_16x16x4f64(af[I], xf[J], accd[t], 0, 0, 0);
        }
    } else {
      float af[NT], bf[NT];
#pragma unroll
      for (int c = 0; c < NT; ++c) {
        af[c] = (float)(xf[c] * w);
        bf[c] = (float)xf[c];
      }
#pragma unroll
      for (int I = 0; I < NT; ++I)
#pragma unroll
        for (int J = 0; J <= I; ++J) {
          const int t = I * (I + 1) / 2 + J;
          accf[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(af[I], bf[J], accf[t], 0, 0, 0);
        }
    }
  };

#pragma unroll
  for (int u = 0; u < U; ++u) load(u, u < nsteps ? u : nsteps - 1);
  for (int s0 = 0; s0 < nsteps; s0 += U) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int s = s0 + u;
      if (s < nsteps) {  // wave-uniform
        compute(u, s);
        const int sn = s + U;
        load(u, sn < nsteps ? sn : nsteps - 1);  // tail: harmless re-fetch
      }
    }
  }

  // ---- epilogue: partial sums of this chunk (newton_solve.hip layout) -------
  double* sH = a.slab_H + (int64_t)chunk * T * 256;
#pragma unroll
  for (int t = 0; t < T; ++t) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      // f64 16x16x4 C/D map: row = (l>>4) + 4 r; f32 16x16x4: row = 4 (l>>4) + r
      const int row = F64 ? (q + 4 * r) : (4 * q + r);
      const double v = F64 ? accd[t][r] : (double)accf[t][r];
      sH[t * 256 + row * 16 + fl] = v;
    }
  }
#pragma unroll
  for (int c = 0; c < NT; ++c) {
    double v = gacc[c];
    v += __shfl_xor(v, 16);
    v += __shfl_xor(v, 32);
    if (q == 0) a.slab_g[(int64_t)chunk * (16 * NT) + 16 * c + fl] = v;
  }
  llacc += __shfl_xor(llacc, 16);
  llacc += __shfl_xor(llacc, 32);
  if (lane == 0) a.slab_ll[chunk] = llacc;
}

template <int NT, bool F64, bool STD, int FAM>
static hipError_t launch_reg_t(const PassArgs& a, int n_chunks, hipStream_t s) {
  hipLaunchKernelGGL((irls_reg_kernel<NT, F64, STD, FAM>), dim3(n_chunks), dim3(64), 0, s, a);
  return hipGetLastError();
}

template <int NT>
static hipError_t launch_reg_nt(const PassArgs& a, bool f64, bool std_, int family, int n_chunks,
                                hipStream_t s) {
  if (family == FAMILY_GAUSSIAN) {  // OLS: a single exact pass, fp64 only
    if (!f64) return hipErrorInvalidValue;
    return std_ ? launch_reg_t<NT, true, true, FAMILY_GAUSSIAN>(a, n_chunks, s)
                : launch_reg_t<NT, true, false, FAMILY_GAUSSIAN>(a, n_chunks, s);
  }
  if (f64)
    return std_ ? launch_reg_t<NT, true, true, FAMILY_LOGISTIC>(a, n_chunks, s)
                : launch_reg_t<NT, true, false, FAMILY_LOGISTIC>(a, n_chunks, s);
  return std_ ? launch_reg_t<NT, false, true, FAMILY_LOGISTIC>(a, n_chunks, s)
              : launch_reg_t<NT, false, false, FAMILY_LOGISTIC>(a, n_chunks, s);
}

}  // namespace dlsa
