// Wide-P IRLS path (DLSA_MAX_P_FUSED < P <= DLSA_MAX_P): BASELINE config 5
// (n = 5e6, p = 500, K = 32; mirrors projects/results/speedtest/
// logistic_LBFGS_local.py:12-13).  Same per-partition contract as the fused
// pass (dlsa/models.py:110-131: MLE theta_k, Sig_inv_k = X_k^T W X_k at
// theta_k), but the P x P Hessian no longer fits a workgroup's registers and
// LDS, so one Newton iteration is split into four launches:
//
//   wide_row_kernel     one streaming pass over X (HBM-bound): eta = x.theta,
//                       mu, w = mu(1-mu), gradient X^T (y - mu), log-lik;
//                       writes w[row] (8 B/row) and per-chunk partials.
//   wide_gram_kernel    X^T diag(w) X as 128x128 lower-triangle output tiles,
//                       split over row groups (fp64 MFMA 16x16x4, MFMA-bound).
//                       blockIdx -> (row group, tile) is XCD-aware: all tiles
//                       of a row group run on one XCD, so its rows are
//                       fetched from HBM once and re-read from that XCD's L2
//                       / the MALL.
//   wide_assemble_kernel  fixed-order sum of the row-group partials into the
//                       padded PP x PP Hessian of each partition (identity on
//                       the padding) -- deterministic.
//   wide_newton_kernel  one 1024-thread workgroup per partition: step
//                       control, publish Sig_inv, blocked right-looking
//                       Cholesky (32-column panels staged in LDS, trailing
//                       update on fp64 MFMA), blocked triangular solves,
//                       update / convergence (same state machine as
//                       newton_solve.hip).
#include <math.h>
#include <stdlib.h>

#include "dlsa_internal.hpp"

namespace dlsa {

// Broadcast lane `l` (wave-uniform, here a compile-time column index) of a
// double with two v_readlane: no LDS round trip (ds_bpermute) on the
// dependency chains of the small factorizations and solves below.
__device__ __forceinline__ double bcast_f64(double v, int l) {
  const int lo = __builtin_amdgcn_readlane(__double2loint(v), l);
  const int hi = __builtin_amdgcn_readlane(__double2hiint(v), l);
  return __hiloint2double(hi, lo);
}


typedef double d4w __attribute__((ext_vector_type(4)));

namespace {

constexpr int GT = kWideTile;  // gram output tile edge (128)
constexpr int CB = 32;         // Cholesky panel width
constexpr int LDP = CB + 1;    // padded LDS row stride of a panel (doubles)

__device__ __forceinline__ double wave_sum64(double v) {
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

__device__ __forceinline__ double bcast_first(double v) {
  const int lo = __builtin_amdgcn_readfirstlane(__double2loint(v));
  const int hi = __builtin_amdgcn_readfirstlane(__double2hiint(v));
  return __hiloint2double(hi, lo);
}

// lower-triangle tile t -> (I, J), I >= J, row-major over I
__device__ __forceinline__ void tile_ij(int t, int& I, int& J) {
  I = 0;
  while ((I + 1) * (I + 2) / 2 <= t) ++I;
  J = t - I * (I + 1) / 2;
}

}  // namespace

// ---------------------------------------------------------------------------
// row pass: one 256-thread workgroup per row chunk; wave w takes rows
// 4w .. 4w+3 of every 16-row group; lane l holds features f = l + 64 m.
// ---------------------------------------------------------------------------
template <int MB, bool STD, int FAM>
__global__ __launch_bounds__(256) void wide_row_kernel(const WideArgs a) {
  const int chunk = blockIdx.x;
  const int part = a.rc_part[chunk];
  const int ph = a.phase[part];
  if (ph != PHASE_F32 && ph != PHASE_F64) return;  // workgroup-uniform
  __shared__ double red[4 * 64 * MB + 4];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int p = a.p, P = a.P, ic = a.intercept;
  const int64_t row0 = a.rc_row0[chunk];
  const int nrows = a.rc_rows[chunk];

  double beta[MB], gacc[MB], cen[MB], isc[MB];
  int col[MB];
  bool inb[MB];
#pragma unroll
  for (int m = 0; m < MB; ++m) {
    const int f = lane + 64 * m;
    beta[m] = f < P ? a.theta[(int64_t)part * P + f] : 0.0;
    gacc[m] = 0.0;
    const int j = f - ic;
    inb[m] = j >= 0 && j < p;
    col[m] = inb[m] ? j : 0;
    cen[m] = 0.0;
    isc[m] = 1.0;
    if constexpr (STD) {
      if (inb[m]) {
        cen[m] = a.center[j];
        isc[m] = 1.0 / a.scale[j];
      }
    }
  }
  const bool icpt_lane = ic && lane == 0;
  double llacc = 0.0;
  constexpr int U = 4;  // rows per wave per step (all U rows' loads in flight)
  for (int base = wid * U; base < nrows; base += 4 * U) {
    double xv[U][MB], yv[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int r = min(base + u, nrows - 1);
      const double* xr = a.X + (row0 + r) * (int64_t)p;
#pragma unroll
      for (int m = 0; m < MB; ++m) xv[u][m] = xr[col[m]];
      yv[u] = a.y[row0 + r];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const bool valid = base + u < nrows;
      double e = 0.0;
#pragma unroll
      for (int m = 0; m < MB; ++m) {
        double v = inb[m] ? xv[u][m] : 0.0;
        if constexpr (STD) v = inb[m] ? (v - cen[m]) * isc[m] : 0.0;
        if (m == 0 && icpt_lane) v = 1.0;
        xv[u][m] = v;
        e = fma(v, beta[m], e);
      }
      e = bcast_first(wave_sum64(e));  // one value for the whole wave
      double w, r;
      if constexpr (FAM == FAMILY_LOGISTIC) {
        const double ea = exp(-fabs(e));
        const double inv = 1.0 / (1.0 + ea);
        const double mu = e >= 0.0 ? inv : ea * inv;
        w = ea * inv * inv;  // mu (1 - mu), cancellation free
        r = yv[u] - mu;
        if (valid && lane == 0) llacc += yv[u] * e - (fmax(e, 0.0) + log1p(ea));
      } else {  // gaussian (OLS): w = 1, ll = -rss/2
        w = 1.0;
        r = yv[u] - e;
        if (valid && lane == 0) llacc -= 0.5 * r * r;
      }
      if (!valid) r = 0.0;
#pragma unroll
      for (int m = 0; m < MB; ++m) gacc[m] = fma(xv[u][m], r, gacc[m]);
      if (valid && lane == 0) a.w[row0 + base + u] = w;
    }
  }
#pragma unroll
  for (int m = 0; m < MB; ++m) red[wid * 64 * MB + lane + 64 * m] = gacc[m];
  llacc = wave_sum64(llacc);
  if (lane == 0) red[4 * 64 * MB + wid] = llacc;
  __syncthreads();
  constexpr int PP = 64 * MB;
  for (int f = tid; f < PP; f += 256)
    a.slab_g[(int64_t)chunk * PP + f] =
        ((red[f] + red[PP + f]) + red[2 * PP + f]) + red[3 * PP + f];
  if (tid == 0)
    a.slab_ll[chunk] = ((red[4 * PP] + red[4 * PP + 1]) + red[4 * PP + 2]) + red[4 * PP + 3];
}

// ---------------------------------------------------------------------------
// gram pass: 512 threads = 8 waves per 128x128 output tile (I, J), I >= J.
// Wave (qi = wid >> 1, qj = wid & 1) owns rows 32 qi .. +31 and columns
// 64 qj .. +63 of the tile: 2 x 4 accumulators of v_mfma_f64_16x16x4_f64.
// K dimension = rows: per k-step of 4 rows lane l reads row (l >> 4) of the
// step at feature (l & 15) of each 16-wide sub-tile (A = w x, B = x).
// ---------------------------------------------------------------------------
template <bool STD>
__global__ __launch_bounds__(512, 1) void wide_gram_kernel(const WideArgs a) {
  const int NB = a.NB;
  const int TB = NB * (NB + 1) / 2;
  const int bid = blockIdx.x;
  const int xcd = bid & 7, j8 = bid >> 3;  // workgroups are dealt to XCDs round-robin
  const int cl = j8 / TB, t = j8 - cl * TB;
  const int chunk = cl * 8 + xcd;  // all TB tiles of a row group on one XCD
  if (chunk >= a.n_gchunks) return;
  const int part = a.gc_part[chunk];
  if (a.phase[part] != a.want_phase) return;
  int I, J;
  tile_ij(t, I, J);
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int qi = wid >> 1, qj = wid & 1;
  if (I == J && qj == 1 && qi < 2) return;  // strictly-upper quadrant of a diagonal tile
  const int p = a.p, ic = a.intercept;
  const int64_t row0 = a.gc_row0[chunk];
  const int nrows = a.gc_rows[chunk];
  const int fl = lane & 15, kq = lane >> 4;

  // per-lane feature columns of the 2 A sub-tiles and the 4 B sub-tiles
  int colA[2], colB[4];
  bool inA[2], inB[4], oneA[2], oneB[4];
  double cA[2], sA[2], cB[4], sB[4];
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    const int f = GT * I + 32 * qi + 16 * s + fl, jj = f - ic;
    inA[s] = jj >= 0 && jj < p;
    oneA[s] = ic && f == 0;
    colA[s] = inA[s] ? jj : 0;
    cA[s] = 0.0;
    sA[s] = 1.0;
    if constexpr (STD) {
      if (inA[s]) {
        cA[s] = a.center[jj];
        sA[s] = 1.0 / a.scale[jj];
      }
    }
  }
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    const int f = GT * J + 64 * qj + 16 * s + fl, jj = f - ic;
    inB[s] = jj >= 0 && jj < p;
    oneB[s] = ic && f == 0;
    colB[s] = inB[s] ? jj : 0;
    cB[s] = 0.0;
    sB[s] = 1.0;
    if constexpr (STD) {
      if (inB[s]) {
        cB[s] = a.center[jj];
        sB[s] = 1.0 / a.scale[jj];
      }
    }
  }

  d4w acc[2][4];
#pragma unroll
  for (int s = 0; s < 2; ++s)
#pragma unroll
    for (int b = 0; b < 4; ++b) acc[s][b] = d4w{0, 0, 0, 0};

  constexpr int U = 4;  // k-steps per prefetch group (16 rows)
  struct Frag {
    double xa[U][2], xb[U][4], w[U];
  };
  auto load = [&](int step0, Frag& F) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int r = 4 * (step0 + u) + kq;
      const bool valid = r < nrows;
      const int rc = valid ? r : nrows - 1;  // in-partition address, weight 0
      const double* xr = a.X + (row0 + rc) * (int64_t)p;
      F.w[u] = valid ? a.w[row0 + rc] : 0.0;
#pragma unroll
      for (int s = 0; s < 2; ++s) F.xa[u][s] = xr[colA[s]];
#pragma unroll
      for (int s = 0; s < 4; ++s) F.xb[u][s] = xr[colB[s]];
    }
  };
  auto compute = [&](const Frag& F) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      double av[2], bv[4];
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        double v = inA[s] ? F.xa[u][s] : 0.0;
        if constexpr (STD) v = (v - cA[s]) * sA[s];
        if (oneA[s]) v = 1.0;
        av[s] = v * F.w[u];
      }
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        double v = inB[s] ? F.xb[u][s] : 0.0;
        if constexpr (STD) v = (v - cB[s]) * sB[s];
        if (oneB[s]) v = 1.0;
        bv[s] = v;
      }
#pragma unroll
      for (int s = 0; s < 2; ++s)
#pragma unroll
        for (int b = 0; b < 4; ++b)
          acc[s][b] = __builtin_amdgcn_mfma_f64_16x16x4f64(av[s], bv[b], acc[s][b], 0, 0, 0);
    }
  };
  const int nsteps = (nrows + 3) / 4;
  if (nsteps > 0) {
    Frag cur, nxt;
    load(0, cur);
    for (int s0 = 0; s0 < nsteps; s0 += U) {
      if (s0 + U < nsteps) load(s0 + U, nxt);
      compute(cur);  // steps past nsteps have w = 0: no contribution
      cur = nxt;
    }
  }

  // C/D map of the f64 16x16x4 MFMA: row = (l >> 4) + 4 r, column = l & 15
  double* G = a.slab_G + ((int64_t)chunk * TB + t) * (GT * GT);
#pragma unroll
  for (int s = 0; s < 2; ++s)
#pragma unroll
    for (int b = 0; b < 4; ++b)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int i = 32 * qi + 16 * s + kq + 4 * r;
        const int jc = 64 * qj + 16 * b + fl;
        G[i * GT + jc] = acc[s][b][r];
      }
}

// ---------------------------------------------------------------------------
// approximate Gram pass (bf16 MFMA, fp32 accumulation) for the Newton steps
// before the fp64 pass (the approximate Hessian only steers
// Newton; the fp64 gradient fixes the solution).  Same (row group, tile)
// grid and XCD mapping as wide_gram_kernel.  Per 32-row block the 512
// threads stage the tile's two 128-feature column blocks through LDS:
// thread (feature f = t & 127, row octet g = t >> 7) loads rows 8g .. 8g+7
// of feature f (each load instruction = 64 consecutive features of one row,
// 512 contiguous bytes), converts to bf16 (A image: w x, B image: x) and
// writes the 8 rows as ONE 16-byte LDS store -- exactly the k-contiguous
// operand of v_mfma_f32_16x16x32_bf16 (lane (i, kg) reads feature i, rows
// 8 kg .. 8 kg + 7 with one ds_read_b128).  Feature stride 80 B: the 16
// lanes of an operand read hit 16 distinct 16-byte bank groups.
// Double-buffered images: one barrier per block.
// ---------------------------------------------------------------------------
typedef __bf16 bf16x8w __attribute__((ext_vector_type(8)));
typedef float f4w __attribute__((ext_vector_type(4)));

namespace {
constexpr int IMG_STRIDE = 80;                       // bytes per feature row of an image
constexpr int IMG_BYTES = GT * IMG_STRIDE;           // one 128-feature x 32-row image
}  // namespace

template <bool STD>
__global__ __launch_bounds__(512, 1) void wide_gram_bf16_kernel(const WideArgs a) {
  __shared__ __attribute__((aligned(16))) char img[2][2][IMG_BYTES];  // [buf][A | B]
  const int NB = a.NB;
  const int TB = NB * (NB + 1) / 2;
  const int bid = blockIdx.x;
  const int xcd = bid & 7, j8 = bid >> 3;
  const int cl = j8 / TB, t = j8 - cl * TB;
  const int chunk = cl * 8 + xcd;
  if (chunk >= a.n_gchunks) return;
  const int part = a.gc_part[chunk];
  if (a.phase[part] != a.want_phase) return;  // workgroup-uniform
  int I, J;
  tile_ij(t, I, J);
  const bool diag = I == J;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int qi = wid >> 1, qj = wid & 1;
  const bool mma = !(diag && qj == 1 && qi < 2);  // wave-uniform
  const int p = a.p, ic = a.intercept;
  const int64_t row0 = a.gc_row0[chunk];
  const int nrows = a.gc_rows[chunk];
  const int nb = (nrows + 31) / 32;

  // staging role: feature fs of both column blocks, rows 8 g .. 8 g + 7
  const int fs = tid & 127, g = tid >> 7;
  auto feat = [&](int blk, int& col, bool& in, bool& one, double& c, double& s) {
    const int f = GT * blk + fs, jj = f - ic;
    in = jj >= 0 && jj < p;
    one = ic && f == 0;
    col = in ? jj : 0;
    c = 0.0;
    s = 1.0;
    if constexpr (STD) {
      if (in) {
        c = a.center[jj];
        s = 1.0 / a.scale[jj];
      }
    }
  };
  int colI, colJ;
  bool inI, inJ, oneI, oneJ;
  double cI, sI, cJ, sJ;
  feat(I, colI, inI, oneI, cI, sI);
  feat(J, colJ, inJ, oneJ, cJ, sJ);

  double xi[8], xj[8], wv[8];
  auto load = [&](int b) {
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int r = 32 * b + 8 * g + e;
      const bool valid = r < nrows;
      const int rc = valid ? r : nrows - 1;
      const double* xr = a.X + (row0 + rc) * (int64_t)p;
      wv[e] = valid ? a.w[row0 + rc] : 0.0;
      xi[e] = xr[colI];
      if (!diag) xj[e] = xr[colJ];
    }
  };
  auto stage = [&](int buf) {
    bf16x8w va, vb;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      double v = inI ? xi[e] : 0.0;
      if constexpr (STD) v = (v - cI) * sI;
      if (oneI) v = 1.0;
      va[e] = (__bf16)(float)(v * wv[e]);
      double u = v;
      if (!diag) {
        u = inJ ? xj[e] : 0.0;
        if constexpr (STD) u = (u - cJ) * sJ;
        if (oneJ) u = 1.0;
      }
      vb[e] = (__bf16)(float)u;
    }
    *(bf16x8w*)(img[buf][0] + fs * IMG_STRIDE + 16 * g) = va;
    *(bf16x8w*)(img[buf][1] + fs * IMG_STRIDE + 16 * g) = vb;
  };

  f4w acc[2][4];
#pragma unroll
  for (int s = 0; s < 2; ++s)
#pragma unroll
    for (int b = 0; b < 4; ++b) acc[s][b] = f4w{0.f, 0.f, 0.f, 0.f};
  const int fl = lane & 15, kg = lane >> 4;

  if (nb > 0) {
    load(0);
    stage(0);
  }
  for (int b = 0; b < nb; ++b) {
    if (b + 1 < nb) load(b + 1);  // in flight during the barrier and the MFMAs
    __syncthreads();              // image b % 2 complete; image (b+1) % 2 free
    if (mma) {
      const char* A = img[b & 1][0];
      const char* B = img[b & 1][1];
      bf16x8w av[2], bv[4];
#pragma unroll
      for (int s = 0; s < 2; ++s)
        av[s] = *(const bf16x8w*)(A + (32 * qi + 16 * s + fl) * IMG_STRIDE + 16 * kg);
#pragma unroll
      for (int c = 0; c < 4; ++c)
        bv[c] = *(const bf16x8w*)(B + (64 * qj + 16 * c + fl) * IMG_STRIDE + 16 * kg);
#pragma unroll
      for (int s = 0; s < 2; ++s)
#pragma unroll
        for (int c = 0; c < 4; ++c)
          acc[s][c] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av[s], bv[c], acc[s][c], 0, 0, 0);
    }
    if (b + 1 < nb) stage((b + 1) & 1);
  }

  if (!mma) return;
  // C/D map of the f32 16x16 MFMAs: row = 4 (l >> 4) + r, column = l & 15
  double* G = a.slab_G + ((int64_t)chunk * TB + t) * (GT * GT);
#pragma unroll
  for (int s = 0; s < 2; ++s)
#pragma unroll
    for (int c = 0; c < 4; ++c)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int i = 32 * qi + 16 * s + 4 * kg + r;
        const int jc = 64 * qj + 16 * c + fl;
        G[i * GT + jc] = (double)acc[s][c][r];
      }
}


// ---------------------------------------------------------------------------
// bf16 Gram pass, one pass over a row group for ALL its tiles (approximate
// Hessian of the MIXED mode).  The per-tile kernel above re-reads each row
// once per 128 x 128 tile that needs it (5x at P = 500: L2/MALL-bound, 16 ms
// per pass at config 5); here a workgroup streams its rows once:
//   Z = bf16(sqrt(w) x),  H~ = Z^T Z   (positive semi-definite by construction)
// per 32-row block: 512 threads load x (fp64, coalesced along the features),
// scale, convert and write the feature-major image Z[PP][32] (96-byte feature
// stride: conflict-free ds_read_b128 operand reads), one barrier, then each
// wave runs one v_mfma_f32_16x16x32_bf16 per owned 16 x 16 lower-triangle
// tile.  The fp32 accumulators of all NT16 (NT16 + 1) / 2 tiles must fit the
// workgroup's registers: S workgroups share a row group, each owning a
// contiguous range of the tiles (S = 2 / 4 above PP = 256 / 384; they run on
// one XCD, so the repeated reads of the rows are L2 hits).  Output: the 128 x 128-tile
// slab layout of wide_gram_kernel (wide_assemble_kernel reads the lower
// triangle of diagonal tiles only).
// ---------------------------------------------------------------------------
namespace {
constexpr int ZS = 96;  // bytes per feature row of the Z image (32 rows of bf16 + pad)
// 16x16 tiles of the lower triangle: 136 / 300 / 528 at NT16 = 16 / 24 / 32;
// the accumulators of a group (4 VGPRs per tile per wave) stay <= ~150 VGPRs
__host__ __device__ constexpr int zall_groups(int NT16) {
  return NT16 > 24 ? 4 : (NT16 > 16 ? 2 : 1);
}
}  // namespace

template <bool STD, int NT16>
__global__ __launch_bounds__(512, 1) void wide_gram_all_bf16_kernel(const WideArgs a) {
  constexpr int S = zall_groups(NT16);
  constexpr int T = NT16 * (NT16 + 1) / 2;
  constexpr int TG = (T + S - 1) / S;    // tiles per group
  constexpr int TPW = (TG + 7) / 8;      // tiles per wave
  constexpr int PP = 16 * NT16;
  constexpr int ITEMS = PP * 4 / 512;    // (feature, 8-row group) items per thread
  extern __shared__ __attribute__((aligned(16))) char zimg[];  // [2][PP][ZS]

  const int bid = blockIdx.x;
  const int xcd = bid & 7, j8 = bid >> 3;
  const int sg = j8 % S, cl = j8 / S;
  const int chunk = cl * 8 + xcd;  // the S groups of a row group on one XCD
  if (chunk >= a.n_gchunks) return;
  const int part = a.gc_part[chunk];
  if (a.phase[part] != a.want_phase) return;  // workgroup-uniform
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int p = a.p, ic = a.intercept;
  const int64_t row0 = a.gc_row0[chunk];
  const int nrows = a.gc_rows[chunk];
  const int nb = (nrows + 31) / 32;

  // this wave's tiles (wave-uniform registers)
  int tI[TPW], tJ[TPW];
  bool tv[TPW];
#pragma unroll
  for (int i = 0; i < TPW; ++i) {
    const int t = sg * TG + wid * TPW + i;
    tv[i] = (wid * TPW + i < TG) && t < T;
    int I = 0;
    while ((I + 1) * (I + 2) / 2 <= t) ++I;
    tI[i] = __builtin_amdgcn_readfirstlane(tv[i] ? I : 0);
    tJ[i] = __builtin_amdgcn_readfirstlane(tv[i] ? t - I * (I + 1) / 2 : 0);
  }

  // staging items: feature f = (tid + 512 m) % PP, rows 8 g .. 8 g + 7
  int colx[ITEMS], fz[ITEMS], gz[ITEMS];
  bool inx[ITEMS], onex[ITEMS];
  double cx[ITEMS], sx[ITEMS];
#pragma unroll
  for (int m = 0; m < ITEMS; ++m) {
    const int idx = tid + 512 * m;
    const int f = idx % PP, g = idx / PP;
    fz[m] = f;
    gz[m] = g;
    const int jj = f - ic;
    inx[m] = jj >= 0 && jj < p;
    onex[m] = ic && f == 0;
    colx[m] = inx[m] ? jj : 0;
    cx[m] = 0.0;
    sx[m] = 1.0;
    if constexpr (STD) {
      if (inx[m]) {
        cx[m] = a.center[jj];
        sx[m] = 1.0 / a.scale[jj];
      }
    }
  }

  double xb[ITEMS][8];
  auto load = [&](int b) {
#pragma unroll
    for (int m = 0; m < ITEMS; ++m)
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        int r = 32 * b + 8 * gz[m] + e;
        r = r < nrows ? r : nrows - 1;
        xb[m][e] = a.X[(row0 + r) * (int64_t)p + colx[m]];
      }
  };
  auto stage = [&](int b) {
    char* img = zimg + (b & 1) * (PP * ZS);
    // sqrt(w) of the block's 32 rows: lane l (< 32) holds row l, broadcast by
    // v_readlane (the row of an item is wave-uniform); rows past the chunk: 0
    const int rl = 32 * b + (lane & 31);
    const float swl = rl < nrows ? sqrtf((float)a.w[row0 + rl]) : 0.f;
#pragma unroll
    for (int m = 0; m < ITEMS; ++m) {
      bf16x8w z;
      const int g8 = __builtin_amdgcn_readfirstlane(8 * gz[m]);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float sw = __builtin_bit_cast(
            float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, swl), g8 + e));
        double v = inx[m] ? xb[m][e] : 0.0;
        if constexpr (STD) v = (v - cx[m]) * sx[m];
        if (onex[m]) v = 1.0;
        float vf = (float)v;
        asm volatile("" : "+v"(vf));  // keep f64 -> f32 -> bf16 (see irls_coop_impl.hpp)
        z[e] = (__bf16)(vf * sw);
      }
      *(bf16x8w*)(img + fz[m] * ZS + 16 * gz[m]) = z;
    }
  };

  f4w acc[TPW];
#pragma unroll
  for (int i = 0; i < TPW; ++i) acc[i] = f4w{0.f, 0.f, 0.f, 0.f};
  const int fl = lane & 15, kg = lane >> 4;

  if (nb > 0) load(0);
  for (int b = 0; b < nb; ++b) {
    stage(b);
    if (b + 1 < nb) load(b + 1);  // in flight during the barrier and the MFMAs
    __syncthreads();              // image b complete; every wave is past block b-1
    const char* img = zimg + (b & 1) * (PP * ZS);
#pragma unroll
    for (int i = 0; i < TPW; ++i) {
      if (tv[i]) {  // wave-uniform
        const bf16x8w av = *(const bf16x8w*)(img + (16 * tI[i] + fl) * ZS + 16 * kg);
        const bf16x8w bv = *(const bf16x8w*)(img + (16 * tJ[i] + fl) * ZS + 16 * kg);
        acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av, bv, acc[i], 0, 0, 0);
      }
    }
  }

  // C/D map of the f32 16x16 MFMAs: row = 4 (l >> 4) + r, column = l & 15
  constexpr int NB = NT16 / 8;
  constexpr int TB = NB * (NB + 1) / 2;
#pragma unroll
  for (int i = 0; i < TPW; ++i) {
    if (!tv[i]) continue;
    const int I = tI[i], J = tJ[i];
    const int I8 = I >> 3, J8 = J >> 3;
    const int t128 = I8 * (I8 + 1) / 2 + J8;
    double* G = a.slab_G + ((int64_t)chunk * TB + t128) * (GT * GT);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int il = 16 * (I & 7) + 4 * kg + r;
      const int jl = 16 * (J & 7) + fl;
      G[il * GT + jl] = (double)acc[i][r];
    }
  }
}

template <bool STD, int NT16>
static hipError_t launch_gram_all_t(const WideArgs& a, hipStream_t s) {
  auto kern = wide_gram_all_bf16_kernel<STD, NT16>;
  const int lds = 2 * 16 * NT16 * ZS;
  {
    hipError_t e = ensure_max_lds((const void*)kern, lds);
    if (e != hipSuccess) return e;
  }
  const int grid = ((a.n_gchunks + 7) / 8) * 8 * zall_groups(NT16);
  hipLaunchKernelGGL(kern, dim3(grid), dim3(512), lds, s, a);
  return hipGetLastError();
}

// workgroups per row group of the all-tiles bf16 Gram pass (plan sizing)
int wide_gram_all_groups(int NB) { return zall_groups(8 * NB); }

hipError_t launch_wide_gram_all(const WideArgs& a, bool standardize, hipStream_t s) {
  if (a.n_gchunks <= 0) return hipSuccess;
  switch (a.NB) {
    case 2: return standardize ? launch_gram_all_t<true, 16>(a, s) : launch_gram_all_t<false, 16>(a, s);
    case 3: return standardize ? launch_gram_all_t<true, 24>(a, s) : launch_gram_all_t<false, 24>(a, s);
    case 4: return standardize ? launch_gram_all_t<true, 32>(a, s) : launch_gram_all_t<false, 32>(a, s);
    default: return hipErrorInvalidValue;
  }
}

// ---------------------------------------------------------------------------
// assemble: H[k] (PP x PP, both triangles, padding = identity) = sum of the
// row-group partials of partition k in row-group order.  grid (TB, K).
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void wide_assemble_kernel(const WideArgs a, const int32_t* gcb,
                                                            double* Hfull) {
  const int t = blockIdx.x, k = blockIdx.y;
  if (a.phase[k] != PHASE_F32 && a.phase[k] != PHASE_F64) return;
  const int NB = a.NB, TB = NB * (NB + 1) / 2, PP = GT * NB, P = a.P;
  int I, J;
  tile_ij(t, I, J);
  const int cb = gcb[k], ce = gcb[k + 1];
  double* H = Hfull + (int64_t)k * PP * PP;
  for (int e = threadIdx.x; e < GT * GT; e += 256) {
    const int il = e / GT, jl = e - il * GT;
    if (I == J && il < jl) continue;
    const int i = GT * I + il, j = GT * J + jl;
    double s = 0.0;
    for (int c = cb; c < ce; ++c) s += a.slab_G[((int64_t)c * TB + t) * (GT * GT) + e];
    if (i >= P || j >= P) s = (i == j) ? 1.0 : 0.0;
    H[(int64_t)i * PP + j] = s;
    H[(int64_t)j * PP + i] = s;
  }
}

// ---------------------------------------------------------------------------
// per-partition Newton update (one 1024-thread workgroup per partition)
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(1024) void wide_newton_kernel(const SolveArgs a, const WideArgs wa,
                                                           const int32_t* rcb, double* Hfull) {
  extern __shared__ __attribute__((aligned(16))) double sm[];
  const int k = blockIdx.x;
  if (a.status[k] != STATUS_RUNNING) return;
  if (a.phase[k] != PHASE_F32 && a.phase[k] != PHASE_F64) return;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int P = a.P, PP = GT * wa.NB;
  double* L11 = sm;             // [CB][LDP] diagonal block
  double* Lp = L11 + CB * LDP;  // [PP][LDP] panel below it (scratch in the solves)
  double* g = Lp + PP * LDP;    // [PP]
  double* z = g + PP;           // [PP]
  double* red = z + PP;         // [64]: [0..47] reductions, [40] ll, [48] flag
  int* flag = (int*)(red + 48);
  double* H = Hfull + (int64_t)k * PP * PP;

  // 1. gradient and log-likelihood of the pass (row-chunk order)
  const int cb = rcb[k], ce = rcb[k + 1];
  for (int f = tid; f < PP; f += 1024) {
    double s = 0.0;
    for (int c = cb; c < ce; ++c) s += wa.slab_g[(int64_t)c * PP + f];
    g[f] = f < P ? s : 0.0;
  }
  if (wid == 0) {
    double s = 0.0;
    for (int c = cb + lane; c < ce; c += 64) s += wa.slab_ll[c];
    s = wave_sum64(s);
    if (lane == 0) red[40] = s;
  }
  if (tid == 0) *flag = 0;
  __syncthreads();
  const double ll = red[40];
  const int it = a.iters[k];
  const int phase = a.phase[k];
  double* th = a.theta + (int64_t)k * P;

  auto level_fail = [&]() {
    for (int f = tid; f < P; f += 1024) th[f] = 0.0;
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
  // 2. step halving on a log-likelihood decrease (newton_solve.hip step 2)
  const double llp = a.ll_prev[k];
  if (a.family == FAMILY_LOGISTIC && it > 0 && ll < llp - 1e-6 * (1.0 + fabs(llp)) &&
      a.backtracks[k] < 40) {
    const int bt = a.backtracks[k] + 1;
    const double sc = ldexp(1.0, -bt);
    const double* tp = a.theta_prev + (int64_t)k * P;
    const double* dp = a.delta_prev + (int64_t)k * P;
    for (int f = tid; f < P; f += 1024) th[f] = tp[f] + sc * dp[f];
    if (tid == 0) {
      a.backtracks[k] = bt;
      a.iters[k] = it + 1;
      atomicAdd(&a.counters[phase], 1);
    }
    return;
  }
  // 3. publish the information matrix at the evaluation point (models.py:130)
  if (!a.subsample) {
    double* S = a.sig_inv + (int64_t)k * P * P;
    for (int e = tid; e < P * P; e += 1024) {
      const int i = e / P, j = e - i * P;
      S[e] = H[(int64_t)i * PP + j];
    }
    if (tid == 0) a.loglik[k] = ll;
  }
  __syncthreads();

  // 4. blocked Cholesky H = L L^T, lower, in place -------------------------
  const int fl = lane & 15, kq = lane >> 4;
  for (int jb = 0; jb < PP; jb += CB) {
    {  // diagonal block -> LDS (one element per thread)
      const int i = tid >> 5, c = tid & 31;
      L11[i * LDP + c] = c <= i ? H[(int64_t)(jb + i) * PP + jb + c] : 0.0;
    }
    __syncthreads();
    if (wid == 0) {  // unblocked right-looking factor, lane i holds row i
      const int i = lane & 31;
      double row[CB];
#pragma unroll
      for (int c = 0; c < CB; ++c) row[c] = L11[i * LDP + c];
      bool ok = true;
#pragma unroll
      for (int j = 0; j < CB; ++j) {
        const double d = bcast_f64(row[j], j);
        ok = ok && d > 0.0 && isfinite(d);
        const double ljj = sqrt(d);
        if (i == j) row[j] = ljj;
        if (i > j) row[j] = row[j] / ljj;
#pragma unroll
        for (int c = j + 1; c < CB; ++c) {
          const double lcj = bcast_f64(row[j], c);  // L[c][j]
          if (i >= c) row[c] -= row[j] * lcj;
        }
      }
      if (lane < 32) {
#pragma unroll
        for (int c = 0; c < CB; ++c) {
          const double v = c <= i ? row[c] : 0.0;
          L11[i * LDP + c] = v;
          if (c <= i) H[(int64_t)(jb + i) * PP + jb + c] = v;
        }
      }
      if (lane == 0 && !ok) *flag = 1;
    }
    __syncthreads();
    if (*flag) break;  // uniform
    const int rest = PP - jb - CB;
    if (rest <= 0) break;
    // TRSM: L21 = A21 L11^-T, one thread per row, staged into the LDS panel
    if (tid < rest) {
      double* hr = H + (int64_t)(jb + CB + tid) * PP + jb;
      double v[CB];
#pragma unroll
      for (int c = 0; c < CB; ++c) v[c] = hr[c];
#pragma unroll
      for (int c = 0; c < CB; ++c) {
        double s = v[c];
#pragma unroll
        for (int e = 0; e < c; ++e) s -= v[e] * L11[c * LDP + e];
        v[c] = s / L11[c * LDP + c];
      }
#pragma unroll
      for (int c = 0; c < CB; ++c) {
        hr[c] = v[c];
        Lp[tid * LDP + c] = v[c];
      }
    }
    __syncthreads();
    // trailing update A22 -= L21 L21^T on the lower 16x16 tiles (fp64 MFMA):
    // C[i][j] = sum_k Lp[16 ti + i][k] Lp[16 tj + j][k]
    const int m = rest / 16;
    const int ntiles = m * (m + 1) / 2;
    for (int tt = wid; tt < ntiles; tt += 16) {
      int ti, tj;
      tile_ij(tt, ti, tj);
      d4w acc = d4w{0, 0, 0, 0};
#pragma unroll
      for (int s = 0; s < CB / 4; ++s) {
        const double av = Lp[(16 * ti + fl) * LDP + 4 * s + kq];
        const double bv = Lp[(16 * tj + fl) * LDP + 4 * s + kq];
        acc = __builtin_amdgcn_mfma_f64_16x16x4f64(av, bv, acc, 0, 0, 0);
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int i = jb + CB + 16 * ti + kq + 4 * r;
        const int jj = jb + CB + 16 * tj + fl;
        H[(int64_t)i * PP + jj] -= acc[r];
      }
    }
    __syncthreads();
  }
  if (*flag) {
    if (a.subsample) {
      level_fail();
      return;
    }
    if (tid == 0) {
      if (phase == PHASE_F32 && a.family == FAMILY_LOGISTIC) {
        // approximate Hessian lost definiteness: redo this point in fp64
        a.phase[k] = PHASE_F64;
        a.iters[k] = it + 1;
        atomicAdd(&a.counters[PHASE_F64], 1);
      } else {
        a.status[k] = DLSA_STATUS_SINGULAR;
      }
    }
    return;
  }

  // 5a. forward solve L z = g, 32-row blocks ---------------------------------
  for (int f = tid; f < PP; f += 1024) z[f] = g[f];
  __syncthreads();
  for (int jb = 0; jb < PP; jb += CB) {
    if (wid == 0) {  // diagonal block by one wave: lane i = row i
      const int i = lane & 31;
      const double* hr = H + (int64_t)(jb + i) * PP + jb;
      double lrow[CB];
#pragma unroll
      for (int c = 0; c < CB; ++c) lrow[c] = c <= i ? hr[c] : 0.0;
      double zi = z[jb + i];
#pragma unroll
      for (int c = 0; c < CB; ++c) {
        if (i == c) zi = zi / lrow[c];
        const double zc = bcast_f64(zi, c);
        if (i > c) zi -= lrow[c] * zc;
      }
      if (lane < 32) z[jb + i] = zi;
    }
    __syncthreads();
    const int rest = PP - jb - CB;
    if (tid < rest) {  // rows below: z_i -= L[i][jb:jb+32] z[jb:jb+32]
      const int i = jb + CB + tid;
      const double* hr = H + (int64_t)i * PP + jb;
      double s = z[i];
#pragma unroll
      for (int c = 0; c < CB; ++c) s -= hr[c] * z[jb + c];
      z[i] = s;
    }
    __syncthreads();
  }
  // 5b. backward solve L^T d = z (d overwrites z) ----------------------------
  for (int jb = PP - CB; jb >= 0; jb -= CB) {
    {  // u_c = sum_{i >= jb + CB} L[i][jb + c] d_i, thread (c, row group)
      const int c = tid & 31, grp = tid >> 5;
      double s = 0.0;
      for (int i = jb + CB + grp; i < PP; i += 32) s += H[(int64_t)i * PP + jb + c] * z[i];
      Lp[grp * LDP + c] = s;
    }
    __syncthreads();
    if (wid == 0) {  // L11^T d = z - u by one wave: lane c = unknown c
      const int c = lane & 31;
      double u = 0.0;
#pragma unroll
      for (int q = 0; q < 32; ++q) u += Lp[q * LDP + c];
      double v = z[jb + c] - u;
      double lcol[CB];  // column c of L11: L[r][c], r >= c
#pragma unroll
      for (int r = 0; r < CB; ++r) lcol[r] = r >= c ? H[(int64_t)(jb + r) * PP + jb + c] : 0.0;
#pragma unroll
      for (int r = CB - 1; r >= 0; --r) {
        if (c == r) v = v / lcol[r];
        const double dr = bcast_f64(v, r);
        if (c < r) v -= lcol[r] * dr;
      }
      if (lane < 32) z[jb + c] = v;
    }
    __syncthreads();
  }

  // 6. update + convergence (newton_solve.hip step 6) ------------------------
  double dm = 0.0, tm = 0.0, tg = 0.0;
  double* tp = a.theta_prev + (int64_t)k * P;
  double* dp = a.delta_prev + (int64_t)k * P;
  for (int f = tid; f < P; f += 1024) {
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
  for (int o = 32; o > 0; o >>= 1) {
    dm = fmax(dm, __shfl_xor(dm, o));
    tm = fmax(tm, __shfl_xor(tm, o));
    tg += __shfl_xor(tg, o);
  }
  if (lane == 0) {
    red[wid] = dm;
    red[16 + wid] = tm;
    red[32 + wid] = tg;
  }
  __syncthreads();
  if (tid != 0) return;
  dm = red[0];
  tm = red[16];
  tg = red[32];
  for (int w = 1; w < 16; ++w) {
    dm = fmax(dm, red[w]);
    tm = fmax(tm, red[16 + w]);
    tg += red[32 + w];
  }
  a.iters[k] = it + 1;
  if (a.family == FAMILY_GAUSSIAN) {
    // OLS: rss = y^T y - theta^T X^T y = -2 ll(0) - theta . g
    a.loglik[k] = -2.0 * ll - tg;
    a.status[k] = isfinite(dm) ? DLSA_STATUS_OK : DLSA_STATUS_NONFINITE;
    if (!isfinite(dm))
      for (int f = 0; f < P; ++f) th[f] = tp[f];
    a.phase[k] = PHASE_DONE;
    return;
  }
  a.ll_prev[k] = ll;
  a.backtracks[k] = 0;
  if (a.subsample) {
    if (!isfinite(dm)) {
      for (int f = 0; f < P; ++f) th[f] = 0.0;
      a.phase[k] = PHASE_LEVEL_DONE;
    } else if (dm <= a.level_tol * (1.0 + tm)) {
      a.phase[k] = PHASE_LEVEL_DONE;
    } else {
      atomicAdd(&a.counters[phase], 1);
    }
    return;
  }
  if (!isfinite(dm)) {
    // keep the last finite iterate: the status reports the failure, and the
    // combine step excludes the partition (dlsa.py reduce)
    for (int f = 0; f < P; ++f) th[f] = tp[f];
    a.status[k] = DLSA_STATUS_NONFINITE;
    return;
  }
  int ph = phase;
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

// ---------------------------------------------------------------------------
// launchers
// ---------------------------------------------------------------------------
int wide_newton_lds_bytes(int NB) {
  const int PP = GT * NB;
  return (CB * LDP + PP * LDP + 2 * PP + 64) * (int)sizeof(double);
}

template <int MB, bool STD>
static hipError_t launch_row_t(const WideArgs& a, int family, int n_chunks, hipStream_t s) {
  if (family == FAMILY_GAUSSIAN)
    hipLaunchKernelGGL((wide_row_kernel<MB, STD, FAMILY_GAUSSIAN>), dim3(n_chunks), dim3(256), 0,
                       s, a);
  else
    hipLaunchKernelGGL((wide_row_kernel<MB, STD, FAMILY_LOGISTIC>), dim3(n_chunks), dim3(256), 0,
                       s, a);
  return hipGetLastError();
}

hipError_t launch_wide_row(const WideArgs& a, bool standardize, int family, int n_chunks,
                           hipStream_t s) {
  if (n_chunks <= 0) return hipSuccess;
  switch (2 * a.NB) {  // MB = PP / 64
    case 4: return standardize ? launch_row_t<4, true>(a, family, n_chunks, s)
                               : launch_row_t<4, false>(a, family, n_chunks, s);
    case 6: return standardize ? launch_row_t<6, true>(a, family, n_chunks, s)
                               : launch_row_t<6, false>(a, family, n_chunks, s);
    case 8: return standardize ? launch_row_t<8, true>(a, family, n_chunks, s)
                               : launch_row_t<8, false>(a, family, n_chunks, s);
    default: return hipErrorInvalidValue;
  }
}

hipError_t launch_wide_gram(const WideArgs& a, bool standardize, bool f64, hipStream_t s) {
  if (a.n_gchunks <= 0) return hipSuccess;
  const int TB = a.NB * (a.NB + 1) / 2;
  const int grid = ((a.n_gchunks + 7) / 8) * 8 * TB;
  if (!f64) {
    if (!getenv("DLSA_WIDE_GRAM_TILED")) return launch_wide_gram_all(a, standardize, s);
    if (standardize)
      hipLaunchKernelGGL(wide_gram_bf16_kernel<true>, dim3(grid), dim3(512), 0, s, a);
    else
      hipLaunchKernelGGL(wide_gram_bf16_kernel<false>, dim3(grid), dim3(512), 0, s, a);
    return hipGetLastError();
  }
  if (standardize)
    hipLaunchKernelGGL(wide_gram_kernel<true>, dim3(grid), dim3(512), 0, s, a);
  else
    hipLaunchKernelGGL(wide_gram_kernel<false>, dim3(grid), dim3(512), 0, s, a);
  return hipGetLastError();
}

hipError_t launch_wide_assemble(const WideArgs& a, const int32_t* gcb, double* Hfull, int K,
                                hipStream_t s) {
  const int TB = a.NB * (a.NB + 1) / 2;
  hipLaunchKernelGGL(wide_assemble_kernel, dim3(TB, K), dim3(256), 0, s, a, gcb, Hfull);
  return hipGetLastError();
}

hipError_t launch_wide_newton(const SolveArgs& sa, const WideArgs& wa, const int32_t* rcb,
                              double* Hfull, int K, hipStream_t s) {
  {
    hipError_t e = ensure_max_lds((const void*)wide_newton_kernel, 160 * 1024);
    if (e != hipSuccess) return e;
  }
  hipLaunchKernelGGL(wide_newton_kernel, dim3(K), dim3(1024), wide_newton_lds_bytes(wa.NB), s,
                     sa, wa, rcb, Hfull);
  return hipGetLastError();
}

}  // namespace dlsa
