// Categorical-code IRLS pass (BASELINE config 3).
//
// The reference dummy-encodes every factor on the host (dlsa/models.py:56-91:
// pd.get_dummies, baseline levels dropped, a chunk missing a selected level
// -> an all-zero frame) and then fits a dense n_k x p design.  Here a row is
// stored as q fp64 numeric columns + F one-byte level codes + y
// (8q + F + 8 bytes: 85 B at the airline shape instead of 1464 B dense), and
// the one-hot blocks of X^T W X are weighted histograms:
//
//   numeric x numeric            dense, per-thread registers (QN <= 16)
//   dummy (f,l) x numeric i      sum_{code_f = l} w x_i        LDS histogram
//   dummy (f,l) x dummy (f,l)    sum_{code_f = l} w            (same, x = 1)
//   dummy (f,l) x dummy (f,l')   0 (one-hot within a factor)
//   dummy (f,l) x dummy (g,m)    sum_{code_f = l, code_g = m} w   2-D histogram
//   gradient dummy (f,l)         sum_{code_f = l} (y - mu)
//
// The histogram bins are 64-bit FIXED-POINT integers (ds_add_u64): each term
// is rounded once to a power-of-two grid chosen per partition and column from
// the partition's own range (scale 2^E with 0.25 max|x| 2^E x rows-per-chunk
// <= 2^61, so no bin can overflow; for config 3 the grid step is ~1e-14 of the
// column's range; an outlier row coarsens only its own partition's grid),
// then integer addition is exact and order-free -- the result is bit-identical
// run to run whatever order the hardware applies the atomics in, and within
// ~1e-13 relative of an fp64 sum.  The dense blocks (numeric x numeric,
// gradient, log-lik) stay fp64 in registers with fixed-order reductions.  So
// every pass is an exact Newton pass (its H is Sig_inv) and the whole fit is
// deterministic.  Low-cardinality factors and pairs keep several histogram
// replicas (lane & (R-1)) so the lanes of a wave that share a frequent level
// do not serialise on one LDS address.
//
// Parameter order: [intercept] [q numeric] [factor 0: levels 1..L_0-1] ...
// -- the reference's column order (sorted numeric names, then each factor's
// sorted dummy names, models.py:70-79) when the host encodes codes in sorted
// dummy-name order (dlsa_amd.models.encode_categorical).
//
// The pass writes the same per-chunk partial slab (lower-triangle 16x16
// tiles, gradient, log-likelihood) as the dense fused pass, so the Newton
// solve, warm-start levels and phases are shared (capi.hip).
#include <math.h>

#include "dlsa_internal.hpp"

// Profiling-only ablation bits (tools/build_variants.sh cat*; product build 0):
// 1 no numeric x dummy histogram adds, 2 no pair adds, 4 no gradient adds,
// 8 no numeric register block, 16 no slab-epilogue lookups, 32 every row's
// loads from the chunk's first 1024 rows (cache-resident: the HBM latency
// and bytes removed).
#ifndef DLSA_CAT_ABLATE
#define DLSA_CAT_ABLATE 0
#endif
// Next row's loads issued under the current row's atomics (1) or at the end
// of the iteration (0, A/B)
#ifndef DLSA_CAT_PF
#define DLSA_CAT_PF 1
#endif
// Histogram slot order: replica outermost (0: slot = replica * levels + level)
// or innermost (1, A/B: slot = level * R + replica).  Innermost was meant to put
// the 16 lanes of an 8-byte LDS atomic group on 16 different bank pairs for
// the R = 16 factors; it measured slower: 5.71-5.72 vs 5.43-5.47 ms per full
// config-3 pass, alternated on one box (profiles/r06p_cat_slot_order_ab.txt)
#ifndef DLSA_CAT_RINNER
#define DLSA_CAT_RINNER 0
#endif

namespace dlsa {

// fixed-point term: v * scale rounded to the nearest integer, added as a
// two's-complement int64.  The rounding is the 1.5 * 2^52 trick: for
// |x| < 2^51, x + 1.5 * 2^52 has ulp 1, so one FMA rounds v * scale (exactly,
// once) and the low bits of the sum minus those of 1.5 * 2^52 are the
// integer -- an FMA and a 64-bit integer subtraction instead of the emulated
// f64 -> i64 conversion (7 VALU ops, 5 of them fp64).  The grids (capi.hip
// fit_categorical) bound every term by 2^50.
__device__ __forceinline__ unsigned long long fx_term(double v, double scale) {
  const double t = fma(v, scale, 6755399441055744.0);  // 1.5 * 2^52
  return (unsigned long long)__double_as_longlong(t) - 0x4338000000000000ull;
}
__device__ __forceinline__ void lds_add_u(unsigned long long* p, unsigned long long u) {
  __hip_atomic_fetch_add(p, u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ long long hist_at(const unsigned long long* h, int i) {
  return (long long)h[i];
}

// histogram slot of level slot lev, replica rp of a factor record
// {R - 1, level slots, ...}
__device__ __forceinline__ int cat_slot(const int4 r, int lev, int rp) {
  return DLSA_CAT_RINNER ? lev * (r.x + 1) + rp : rp * r.y + lev;
}

// pair index of factors f < g among F
__host__ __device__ __forceinline__ int cat_pair(int f, int g, int F) {
  return f * F - f * (f + 1) / 2 + (g - f - 1);
}

// EX: intercept fitted and QN = 1 + q exactly (the column bucket has no
// padding), so the per-column conditions and the row stride are compile-time:
// at the airline shape that removes a third of the row loop's instructions
// (1858 -> 1215; SGPR spills 124 -> 4)
template <int QN, int FM, int NTHR, bool STD, bool EX>
__global__ __launch_bounds__(NTHR) void cat_pass_kernel(const CatArgs a) {
  extern __shared__ __attribute__((aligned(16))) double sm[];
  constexpr int NW = NTHR / 64;
  // EX: the intercept row of the dense block (sum w, sum w x_i) and the
  // intercept gradient (sum r) come from the fold factor's histograms, which
  // also take its baseline level -- every row lands in exactly one of its
  // levels -- so the register block holds the numeric columns only (-22 VGPRs:
  // room for the next row's loads in flight)
  constexpr int Q0 = EX ? 1 : 0;     // first register-block column
  constexpr int NQ = QN - Q0;
  constexpr int NTRI = NQ * (NQ + 1) / 2;
  constexpr int NR = NTRI + NQ + 1;  // reduced register values: H block, gradient, ll
  const int chunk = blockIdx.x;
  const int part = a.chunk_part[chunk];
  if (a.phase[part] != a.want_phase) return;  // workgroup-uniform

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int q = EX ? QN - 1 : a.q, F = a.F, P = a.P, ic = EX ? 1 : a.intercept;
  const int Qn = ic + q;
  unsigned long long* hist = (unsigned long long*)sm;  // a.hist_doubles int64 bins
  double* th = sm + a.hist_doubles;        // kCatPMax: theta of this partition
  double* stdv = th + kCatPMax;            // 2 x kCatQMax: center, 1 / scale
  double* red = stdv + 2 * kCatQMax;       // NW x NR, then NR final sums

  // factor / pair tables in LDS, re-read (broadcast) every row instead of
  // pinning ~100 loop-invariant values in registers: one 16-byte record per
  // factor {replica mask, levels, nd offset, gradient offset} and per pair in
  // the row loop's (f, g) order for FM {offset, replica mask, L_f, L_g}, at
  // compile-time positions; records past F are zero
  constexpr int NPM = FM * (FM - 1) / 2;
  __shared__ int4 ftab[kCatMaxFactors + 1];
  __shared__ int4 ptab[kCatMaxPairs + 1];
  __shared__ int4 dtab[kCatMaxFactors / 4];  // first dummy parameter of each factor
  int32_t* t_doff = (int32_t*)dtab;
  for (int i = tid; i <= FM; i += NTHR)
    ftab[i] = i < F ? make_int4(a.nd_rep[i] - 1, a.nd_lev[i], a.nd_off[i], a.g_off[i])
                    : make_int4(0, 0, 0, 0);
  for (int i = tid; i <= NPM; i += NTHR) {
    int f = 0, g = i;  // position i = cat_pair(f, g, FM)
    while (f < FM - 1 && g >= FM - 1 - f) g -= FM - 1 - f, ++f;
    g += f + 1;
    int4 v = make_int4(0, 0, 0, 0);
    if (i < NPM && g < F) {
      const int pi = cat_pair(f, g, F);
      v = make_int4(a.pr_off[pi], a.pr_rep[pi] - 1, a.nlev[f], a.nlev[g]);
    }
    ptab[i] = v;
  }
  for (int i = tid; i < kCatMaxFactors; i += NTHR) t_doff[i] = a.doff[i];
  for (int i = tid; i < a.hist_doubles; i += NTHR) hist[i] = 0ull;
  for (int i = tid; i < kCatPMax; i += NTHR) th[i] = i < P ? a.theta[(int64_t)part * P + i] : 0.0;
  if (STD && tid < kCatQMax) {
    stdv[tid] = tid < q ? a.center[tid] : 0.0;
    stdv[kCatQMax + tid] = tid < q ? 1.0 / a.scale[tid] : 1.0;
  }
  __syncthreads();

  const int64_t row0 = a.chunk_row0[chunk];
  const int nrows = a.chunk_rows[chunk];
  // fixed-point scales in registers (not re-read from the kernel arguments
  // inside the row loop): [0] w, [1] residual, [2 + i - ic] w x_i
  double hsc[QN + 2];
#pragma unroll
  for (int i = 0; i < QN + 2; ++i)
    hsc[i] = (i < 2 + q && i < kCatQMax + 2) ? a.hscale[(int64_t)part * (kCatQMax + 2) + i] : 0.0;
  const double* hs = a.hscale + (int64_t)part * (kCatQMax + 2);  // the epilogue's
  double hacc[NTRI], gacc[NQ], llacc = 0.0;
#pragma unroll
  for (int i = 0; i < NTRI; ++i) hacc[i] = 0.0;
#pragma unroll
  for (int i = 0; i < NQ; ++i) gacc[i] = 0.0;
  const int fold = EX ? __builtin_amdgcn_readfirstlane(a.fold) : -1;

  // Software-pipelined row loop (DLSA_CAT_PF, default): the next row's x,
  // codes and y are loaded once the current row's triangle, gradient and
  // fixed-point terms are formed -- its x registers are dead by then -- so the
  // load latency runs under the current row's ~65 LDS atomics instead of
  // stalling the top of the next iteration (2 waves per SIMD: one workgroup's
  // histograms fill the CU's LDS).  Rows past the chunk load the chunk's last
  // row (a valid address, never used).
  double xl[QN];
  int cl[FM];
  double yl;
  auto load_row = [&](int rr) {
    const int64_t rw = row0 + rr;
    const int64_t rl = (DLSA_CAT_ABLATE & 32) ? row0 + (rr & 1023) % nrows : rw;
    const double* xr = a.Xn + rl * q;
    const uint8_t* cr = a.codes + rl * F;
#pragma unroll
    for (int i = 0; i < QN; ++i) {
      const int j = i - ic;
      xl[i] = (i < Qn && j >= 0) ? xr[j] : 0.0;
    }
    // unconditional byte loads (a factor past F re-reads the row's last code;
    // its uses are masked by f < F): a load under f < F would be sunk into a
    // branch region of its own, next to its first use.  F = 0 (no factors: the
    // codes may be a null pointer) skips them all, a uniform branch
    if (F > 0) {
#pragma unroll
      for (int f = 0; f < FM; ++f) cl[f] = (int)cr[f < F ? f : F - 1];
    } else {
#pragma unroll
      for (int f = 0; f < FM; ++f) cl[f] = 0;
    }
    yl = a.y[rl];
  };
  if (tid < nrows) load_row(tid);
  for (int r = tid; r < nrows; r += NTHR) {
    // parameter-order numeric vector: [1 if intercept] x_0 .. x_{q-1} (standardised)
    double xv[QN];
#pragma unroll
    for (int i = 0; i < QN; ++i) {
      const int j = i - ic;
      double v = 0.0;
      if (i < Qn) {
        if (j < 0) {
          v = 1.0;
        } else {
          v = xl[i];
          if constexpr (STD) v = (v - stdv[j]) * stdv[kCatQMax + j];
        }
      }
      xv[i] = v;
    }
    int cv[FM];
#pragma unroll
    for (int f = 0; f < FM; ++f) cv[f] = cl[f];
    const double yv = yl;

    double e0 = 0.0, e1 = 0.0;
#pragma unroll
    for (int i = 0; i < QN; ++i) {
      if (i & 1)
        e1 = fma(xv[i], th[i], e1);
      else
        e0 = fma(xv[i], th[i], e0);
    }
    // dummy effects: the gathers are unconditional (a baseline code reads a
    // valid slot and adds +0), so they issue back to back and one wait covers
    // them instead of one per factor
    // (the offsets are read as 16-byte records, FM / 4 reads and one wait)
    int4 dof[FM / 4];
#pragma unroll
    for (int k = 0; k < FM / 4; ++k) dof[k] = dtab[k];
    double de[FM];
#pragma unroll
    for (int f = 0; f < FM; ++f) {
      const int4 d4 = dof[f / 4];
      const int d = (f & 3) == 0 ? d4.x : (f & 3) == 1 ? d4.y : (f & 3) == 2 ? d4.z : d4.w;
      const bool on = f < F && cv[f] > 0;
      const double t = th[f < F ? d + (on ? cv[f] - 1 : 0) : 0];
      de[f] = on ? t : 0.0;
    }
#pragma unroll
    for (int f = 0; f < FM; ++f) e0 += de[f];
    const double e = e0 + e1;
    const double ea = exp(-fabs(e));
    const double inv = 1.0 / (1.0 + ea);
    const double mu = e >= 0.0 ? inv : ea * inv;
    const double w = ea * inv * inv;  // mu (1 - mu), cancellation free
    const double res = yv - mu;
    llacc += yv * e - (fmax(e, 0.0) + log1p(ea));

#pragma unroll
    for (int i = Q0; i < QN && !(DLSA_CAT_ABLATE & 8); ++i) {
      const int ii = i - Q0;
      gacc[ii] = fma(res, xv[i], gacc[ii]);
      const double wxi = w * xv[i];
#pragma unroll
      for (int j = Q0; j <= i; ++j)
        hacc[ii * (ii + 1) / 2 + j - Q0] = fma(wxi, xv[j], hacc[ii * (ii + 1) / 2 + j - Q0]);
    }
    // the row's fixed-point terms, formed once for all factors: [0] w,
    // [1] residual, [2 + i - ic] w x_i
    unsigned long long ut[QN + 2];
    ut[0] = fx_term(w, hsc[0]);
    ut[1] = fx_term(res, hsc[1]);
#pragma unroll
    for (int i = 0; i < QN; ++i)  // parameter i is numeric column i - ic: scale hsc[2 + i - ic]
      if (i >= ic) ut[2 + i - ic] = fx_term(w * xv[i], ic ? hsc[i + 1] : hsc[i + 2]);
#if DLSA_CAT_PF
    __builtin_amdgcn_sched_barrier(0);
    load_row(min(r + NTHR, nrows - 1));  // the next row, in flight under the atomics
    __builtin_amdgcn_sched_barrier(0);
#endif

    // one-hot blocks: fixed-point histograms in LDS
    // The record of factor f + 1 (pair p + 1) is read before factor f's (pair
    // p's) adds are issued: LDS operations complete in order, so a record read
    // after the adds would wait for every one of them (an s_waitcnt
    // lgkmcnt(0), a drain of the LDS queue, per factor and pair); read ahead,
    // the wait covers the read alone.
    int4 tf = ftab[0];
#pragma unroll
    for (int f = 0; f < FM; ++f) {
      const int4 tn = ftab[f + 1];
      if (f < F && (cv[f] > 0 || (EX && f == fold))) {
        // a baseline row of the fold factor goes to its extra slot (the last)
        const int slot = cat_slot(tf, cv[f] > 0 ? cv[f] - 1 : tf.y - 1, lane & tf.x);
        unsigned long long* h = hist + tf.z + slot * a.nd_stride;
        if constexpr (!(DLSA_CAT_ABLATE & 1)) {
          lds_add_u(h, ut[0]);
#pragma unroll
          for (int i = 0; i < QN; ++i)  // numeric columns (register index compile-time)
            if (i >= ic && i < Qn) lds_add_u(h + 1 + (i - ic), ut[2 + i - ic]);
        }
        if constexpr (!(DLSA_CAT_ABLATE & 4)) lds_add_u(hist + tf.w + slot, ut[1]);
      }
      tf = tn;
    }
    // pairs: one add each, so the records are read two ahead (one ahead,
    // every wait would drain all but the last add)
    int4 tp = ptab[0], tp1 = ptab[1];
#pragma unroll
    for (int f = 0; f < FM; ++f)
#pragma unroll
      for (int g = f + 1; g < FM; ++g) {
        const int pn = cat_pair(f, g, FM) + 2;
        const int4 tn = ptab[pn <= kCatMaxPairs ? pn : kCatMaxPairs];
        if (!(DLSA_CAT_ABLATE & 2) && g < F && cv[f] > 0 && cv[g] > 0)
          lds_add_u(hist + tp.x +
                        (DLSA_CAT_RINNER ? ((cv[f] - 1) * tp.w + cv[g] - 1) * (tp.y + 1) + (lane & tp.y)
                                         : ((lane & tp.y) * tp.z + cv[f] - 1) * tp.w + cv[g] - 1),
                    ut[0]);
        tp = tp1;
        tp1 = tn;
      }
#if !DLSA_CAT_PF
    if (r + NTHR < nrows) load_row(r + NTHR);
#endif
  }

  // ---- reduce the register blocks over the workgroup (fixed order) --------
  auto wave_red = [&](double v) {
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) v += __shfl_xor(v, o);
    return v;
  };
#pragma unroll
  for (int i = 0; i < NTRI; ++i) {
    const double v = wave_red(hacc[i]);
    if (lane == 0) red[wid * NR + i] = v;
  }
#pragma unroll
  for (int i = 0; i < NQ; ++i) {
    const double v = wave_red(gacc[i]);
    if (lane == 0) red[wid * NR + NTRI + i] = v;
  }
  {
    const double v = wave_red(llacc);
    if (lane == 0) red[wid * NR + NTRI + NQ] = v;
  }
  __syncthreads();
  double* fin = red + NW * NR;
  for (int i = tid; i < NR; i += NTHR) {
    double s = 0.0;
#pragma unroll
    for (int w = 0; w < NW; ++w) s += red[w * NR + i];
    fin[i] = s;
  }
  // the epilogue's per-entry lookups come from LDS: the factor / pair records
  // and the grids (staged over theta, which the row loop no longer reads),
  // not from the kernel arguments at a lane-dependent index (dependent memory
  // round trips; 0.015 ms per launch, profiles/r05cf_cat_epilogue_ab.jsonl)
  double* hsl = th;
  for (int i = tid; i < kCatQMax + 2; i += NTHR) hsl[i] = hs[i];
  __syncthreads();

  // factor of dummy parameter index d (0-based among dummies)
  auto factor_of = [&](int gi, int& lev) {
    int f = 0;
#pragma unroll
    for (int g = 1; g < FM; ++g)
      if (g < F && gi >= t_doff[g]) f = g;
    lev = gi - t_doff[f];
    return f;
  };
  // exact integer sums over the replicas, one rounding back to fp64
  auto nd_sum = [&](int f, int lev, int col) {
    const int4 r = ftab[f];  // {R - 1, level slots, nd offset, g offset}
    long long s = 0;
    for (int rp = 0; rp <= r.x; ++rp) s += hist_at(hist, r.z + cat_slot(r, lev, rp) * a.nd_stride + col);
    return (double)s / (col == 0 ? hsl[0] : hsl[1 + col]);
  };
  // EX: the intercept row -- the fold factor's bins over every level slot
  // (baseline included) and replica, exact in int64, one rounding.  col -1:
  // the gradient histogram
  auto fold_sum = [&](int col) {
    const int4 r = ftab[EX ? fold : 0];  // (called in EX kernels only)
    long long s = 0;
    for (int rp = 0; rp <= r.x; ++rp)
      for (int l = 0; l < r.y; ++l)
        s += col < 0 ? hist_at(hist, r.w + cat_slot(r, l, rp))
                     : hist_at(hist, r.z + cat_slot(r, l, rp) * a.nd_stride + col);
    const int si = col < 0 ? 1 : col == 0 ? 0 : 1 + col;  // its grid (hsl layout above)
    return (double)s / hsl[si];
  };

  // ---- epilogue: the partial slab in the dense pass's tile format ---------
  const int NT = a.NT;
  const int T = NT * (NT + 1) / 2;
  double* dst = a.slab_H + (int64_t)chunk * T * 256;
  for (int e = tid; e < T * 256; e += NTHR) {
    const int t = e >> 8, pos = e & 255;
    int I = 0;
    while ((I + 1) * (I + 2) / 2 <= t) ++I;
    const int J = t - I * (I + 1) / 2;
    const int gi = 16 * I + (pos >> 4), gj = 16 * J + (pos & 15);
    double v = 0.0;
    if (!(DLSA_CAT_ABLATE & 16) && gi < P && gj <= gi) {
      if (gi < Qn) {
        if (EX && gj == 0)
          v = fold_sum(gi);  // ic = 1: parameter gi >= 1 is bin column gi (w x_{gi - 1})
        else
          v = fin[(gi - Q0) * (gi - Q0 + 1) / 2 + gj - Q0];
      } else {
        int li;
        const int fi = factor_of(gi, li);
        if (gj < Qn) {
          v = nd_sum(fi, li, ic ? gj : gj + 1);
        } else {
          int lj;
          const int fj = factor_of(gj, lj);
          if (fj == fi) {
            v = li == lj ? nd_sum(fi, li, 0) : 0.0;
          } else {  // fj < fi
            // {offset, R - 1, L_fj, L_fi} at the pair's row-loop position
            const int4 r = ptab[cat_pair(fj, fi, FM)];
            long long s = 0;
            for (int rp = 0; rp <= r.y; ++rp)
              s += hist_at(hist, r.x + (DLSA_CAT_RINNER ? (lj * r.w + li) * (r.y + 1) + rp
                                                        : (rp * r.z + lj) * r.w + li));
            v = (double)s / hsl[0];
          }
        }
      }
    }
    dst[e] = v;
  }
  const int PP = 16 * NT;
  for (int e = tid; e < PP; e += NTHR) {
    double v = 0.0;
    if (e < Qn) {
      v = (EX && e == 0) ? fold_sum(-1) : fin[NTRI + e - Q0];
    } else if (e < P) {
      int l;
      const int f = factor_of(e, l);
      const int4 r = ftab[f];
      long long s = 0;
      for (int rp = 0; rp <= r.x; ++rp) s += hist_at(hist, r.w + cat_slot(r, l, rp));
      v = (double)s / hsl[1];
    }
    a.slab_g[(int64_t)chunk * PP + e] = v;
  }
  if (tid == 0) a.slab_ll[chunk] = fin[NTRI + NQ];
}

// Level presence per chunk: counts[chunk, d] = 1 if a row of the chunk
// selects dummy column d; bad[chunk] = codes outside 0..L_f-1; colmax[chunk,
// i] = max |x_i| over the finite values of the chunk (raw numeric columns:
// the fixed-point grids).  The outputs are zeroed by the launcher.
// A streaming pass, latency-bound unless many loads are in flight: each
// chunk is split over S workgroups (contiguous row ranges, ~16 per CU in
// total); every load is unconditional (out-of-range lanes load a clamped
// in-range address and discard it -- a predicated load puts each load in its
// own branch region, each closed by a vmcnt(0) wait); the codes are read as
// 16-byte units (4 per lane in flight, the factor of each byte advanced
// incrementally from one 32-bit modulo per unit) and the numeric columns as
// wave-contiguous windows of q doubles per lane, two windows (2 QS loads) in
// flight, so the column of every value is fixed per lane and slot and the
// maxima stay in registers (|x| >= 0 orders like its bits as uint64).
// Flags: plain LDS stores of 1, then plain global stores of 1.
template <int QS>
__global__ __launch_bounds__(256) void cat_presence_kernel(const CatArgs a, int S, int32_t* counts,
                                                           int32_t* bad, double* colmax) {
  __shared__ int32_t flag[kCatPMax];
  __shared__ int32_t nbad;
  __shared__ unsigned long long cmax[kCatQMax];
  __shared__ int32_t t_nd[kCatMaxFactors];  // nlev | doff << 16
  const int chunk = blockIdx.x / S, sub = blockIdx.x - chunk * S;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int F = a.F, q = a.q;
  const int D = a.P - a.intercept - q;
  const int doff0 = a.intercept + q;
  for (int i = tid; i < kCatPMax; i += 256) flag[i] = 0;
  if (tid < kCatQMax) cmax[tid] = 0ull;
  if (tid < kCatMaxFactors) t_nd[tid] = a.nlev[tid] | ((a.doff[tid] - doff0) << 16);
  if (tid == 0) nbad = 0;
  __syncthreads();
  const int nrows = a.chunk_rows[chunk];
  const int rps = (nrows + S - 1) / S;
  const int r_begin = min(nrows, sub * rps), r_end = min(nrows, r_begin + rps);
  const int64_t row0 = a.chunk_row0[chunk] + r_begin;
  const int rows = r_end - r_begin;

  // ---- codes: bytes [row0 F, (row0 + rows) F) as aligned 16-byte units ------
  if (F > 0 && rows > 0) {
    const uintptr_t cb = (uintptr_t)(a.codes + row0 * F);
    const uint4* base = (const uint4*)(cb & ~(uintptr_t)15);
    const int skew = (int)(cb & 15);
    const int nbytes = rows * F;
    const int nunits = (skew + nbytes + 15) >> 4;
    constexpr int U = 4;
    int nb = 0;
    for (int u0 = tid; u0 < nunits; u0 += 256 * U) {
      uint4 w[U];
#pragma unroll
      for (int k = 0; k < U; ++k) w[k] = base[min(u0 + 256 * k, nunits - 1)];
#pragma unroll
      for (int k = 0; k < U; ++k) {
        const int u = u0 + 256 * k;
        const int b0 = 16 * u - skew;  // chunk byte of the unit's first byte
        int f = (int)((unsigned)(b0 + 16 * F) % (unsigned)F);
        const uint32_t ws[4] = {w[k].x, w[k].y, w[k].z, w[k].w};
        const bool unit_in = u < nunits;
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const int b = b0 + i;
          const int c = (ws[i >> 2] >> (8 * (i & 3))) & 0xFF;
          const int nd = t_nd[f];
          const bool in = unit_in && (unsigned)b < (unsigned)nbytes;
          const bool isbad = in && c > (nd & 0xFFFF);
          nb += isbad ? 1 : 0;
          if (in && !isbad && c > 0) flag[(nd >> 16) + c - 1] = 1;
          f = f + 1 == F ? 0 : f + 1;
        }
      }
    }
    if (nb) atomicAdd(&nbad, nb);
  }

  // ---- numeric columns: doubles [row0 q, (row0 + rows) q) -------------------
  if (q > 0 && rows > 0) {
    const double* xb = a.Xn + row0 * q;
    const int64_t ne = (int64_t)rows * q;
    const int64_t wstride = 4LL * q * 64;  // doubles per workgroup window (a multiple of q)
    unsigned long long mx[QS];  // max |x| as bits (|x| >= 0 orders like its bits)
#pragma unroll
    for (int s = 0; s < QS; ++s) mx[s] = 0ull;
    for (int64_t e0 = (int64_t)wid * q * 64; e0 < ne; e0 += 2 * wstride) {
      double v[2][QS];
#pragma unroll
      for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int s = 0; s < QS; ++s) {
          const int64_t e = e0 + h * wstride + s * 64 + lane;
          v[h][s] = __builtin_nontemporal_load(xb + ((s < q && e < ne) ? e : 0));
        }
      // every load used unconditionally (no load sunk into a branch of its own)
#pragma unroll
      for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int s = 0; s < QS; ++s) asm volatile("" : "+v"(v[h][s]));
#pragma unroll
      for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int s = 0; s < QS; ++s) {
          const int64_t e = e0 + h * wstride + s * 64 + lane;
          // finite values only: a NaN / Inf row fails its own partition
          const unsigned long long u =
              (unsigned long long)__double_as_longlong(v[h][s]) & 0x7FFFFFFFFFFFFFFFull;
          const bool ok = s < q && e < ne && u < 0x7FF0000000000000ull;
          mx[s] = max(mx[s], ok ? u : 0ull);
        }
    }
#pragma unroll
    for (int s = 0; s < QS; ++s)
      if (s < q)
        __hip_atomic_fetch_max(&cmax[(s * 64 + lane) % q], mx[s], __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_WORKGROUP);
  }
  __syncthreads();
  for (int d = tid; d < D; d += 256)
    if (flag[d]) counts[(int64_t)chunk * D + d] = 1;
  if (tid == 0 && nbad) atomicAdd(&bad[chunk], nbad);
  if (tid < q && cmax[tid])
    __hip_atomic_fetch_max((unsigned long long*)&colmax[(int64_t)chunk * kCatQMax + tid], cmax[tid],
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Per partition: a selected dummy level with no rows -> the reference's
// all-zero frame (models.py:84-91): status MISSING_LEVEL, phase DONE, outputs
// stay zero (fit_init zeroed theta / Sig_inv).  bad_part[k] = invalid codes.
__global__ __launch_bounds__(256) void cat_mark_kernel(const CatArgs a, const int32_t* pcb,
                                                       const int32_t* counts, const int32_t* bad,
                                                       int32_t* phase, int32_t* status,
                                                       int32_t* bad_part) {
  __shared__ int32_t flag[2];
  const int k = blockIdx.x, tid = threadIdx.x;
  const int D = a.P - a.intercept - a.q;
  if (tid < 2) flag[tid] = 0;
  __syncthreads();
  const int cb = pcb[k], ce = pcb[k + 1];
  for (int d = tid; d < D; d += 256) {
    int64_t s = 0;
    for (int c = cb; c < ce; ++c) s += counts[(int64_t)c * D + d];
    if (s == 0) flag[0] = 1;
  }
  int nb = 0;
  for (int c = cb + tid; c < ce; c += 256) nb += bad[c];
  if (nb) atomicAdd(&flag[1], nb);
  __syncthreads();
  if (tid == 0) {
    bad_part[k] = flag[1];
    if (ce > cb && flag[0] && status[k] == STATUS_RUNNING) {
      status[k] = DLSA_STATUS_MISSING_LEVEL;
      phase[k] = PHASE_DONE;
    }
  }
}

template <int QN, int FM, int NTHR, bool STD>
static hipError_t launch_cat_t(const CatArgs& a, int n_chunks, size_t lds, hipStream_t s) {
  // the exact-bucket kernel only where it exists (F <= 8) and folds (F >= 1)
  const bool ex = FM == 8 && cat_exact_bucket(a) && a.fold >= 0;
  auto kern = ex ? cat_pass_kernel<QN, FM, NTHR, STD, FM == 8> : cat_pass_kernel<QN, FM, NTHR, STD, false>;
  {
    hipError_t e = ensure_max_lds((const void*)kern, 160 * 1024 - kCatStaticLds);
    if (e != hipSuccess) return e;
  }
  hipLaunchKernelGGL(kern, dim3(n_chunks), dim3(NTHR), lds, s, a);
  return hipGetLastError();
}

static int cat_qn(int Qn) { return Qn <= 4 ? 4 : Qn <= 8 ? 8 : Qn <= 10 ? 10 : Qn <= 12 ? 12 : 16; }
// the exact-bucket instantiation (EX): intercept fitted, 1 + q equal to its
// column bucket, 1 <= F <= 8 (the host layout then names a fold factor)
bool cat_exact_bucket(const CatArgs& a) {
  return a.intercept == 1 && a.F >= 1 && a.F <= 8 && a.q + 1 == cat_qn(1 + a.q);
}
static constexpr int cat_threads_t(int QN, int FM) {
  return (QN <= 4 || (QN <= 10 && FM <= 8)) ? 512 : 256;
}

size_t cat_lds_bytes(const CatArgs& a) {
  const int QN = cat_qn(a.intercept + a.q);
  const int NR = QN * (QN + 1) / 2 + QN + 1;  // (the EX kernel's NR is smaller)
  const int NW = cat_threads_t(QN, a.F <= 8 ? 8 : 16) / 64;
  return 8 * ((size_t)a.hist_doubles + kCatPMax + 2 * kCatQMax + (size_t)(NW + 1) * NR);
}

template <int QN>
static hipError_t launch_cat_q(const CatArgs& a, bool std_, int n_chunks, size_t lds,
                               hipStream_t s) {
  // 512 threads while the register blocks fit 256 VGPRs (measured: QN <= 10
  // with F <= 8), else 256 threads (512 VGPRs per lane)
  if (a.F <= 8) {
    constexpr int N8 = cat_threads_t(QN, 8);
    return std_ ? launch_cat_t<QN, 8, N8, true>(a, n_chunks, lds, s)
                : launch_cat_t<QN, 8, N8, false>(a, n_chunks, lds, s);
  }
  constexpr int N16 = cat_threads_t(QN, 16);
  return std_ ? launch_cat_t<QN, 16, N16, true>(a, n_chunks, lds, s)
              : launch_cat_t<QN, 16, N16, false>(a, n_chunks, lds, s);
}

hipError_t launch_cat_pass(const CatArgs& a, bool standardize, int n_chunks, hipStream_t s) {
  if (n_chunks <= 0) return hipSuccess;
  const size_t lds = cat_lds_bytes(a);
  if (lds + kCatStaticLds > 160 * 1024 || a.F > kCatMaxFactors || a.q + a.intercept > kCatQMax)
    return hipErrorInvalidValue;
  switch (cat_qn(a.intercept + a.q)) {
    case 4: return launch_cat_q<4>(a, standardize, n_chunks, lds, s);
    case 8: return launch_cat_q<8>(a, standardize, n_chunks, lds, s);
    case 10: return launch_cat_q<10>(a, standardize, n_chunks, lds, s);
    case 12: return launch_cat_q<12>(a, standardize, n_chunks, lds, s);
    default: return launch_cat_q<16>(a, standardize, n_chunks, lds, s);
  }
}

hipError_t launch_cat_presence(const CatArgs& a, int n_chunks, int32_t* counts, int32_t* bad,
                               double* colmax, hipStream_t s) {
  if (n_chunks <= 0) return hipSuccess;
  const int D = a.P - a.intercept - a.q;
  hipError_t e = hipMemsetAsync(counts, 0, 4LL * n_chunks * std::max(D, 1), s);
  if (e == hipSuccess) e = hipMemsetAsync(bad, 0, 4LL * n_chunks, s);
  if (e == hipSuccess) e = hipMemsetAsync(colmax, 0, 8LL * kCatQMax * n_chunks, s);
  if (e != hipSuccess) return e;
  // ~16 workgroups per CU in total (a streaming pass: loads in flight)
  const int S = std::max(1, std::min(64, (4096 + n_chunks - 1) / n_chunks));
  auto kern = a.q <= 4 ? cat_presence_kernel<4>
              : a.q <= 8 ? cat_presence_kernel<8>
              : a.q <= 12 ? cat_presence_kernel<12> : cat_presence_kernel<16>;
  hipLaunchKernelGGL(kern, dim3(n_chunks * S), dim3(256), 0, s, a, S, counts, bad, colmax);
  return hipGetLastError();
}

hipError_t launch_cat_mark(const CatArgs& a, const int32_t* pcb, const int32_t* counts,
                           const int32_t* bad, int K, int32_t* phase, int32_t* status,
                           int32_t* bad_part, hipStream_t s) {
  hipLaunchKernelGGL(cat_mark_kernel, dim3(K), dim3(256), 0, s, a, pcb, counts, bad, phase,
                     status, bad_part);
  return hipGetLastError();
}

}  // namespace dlsa
