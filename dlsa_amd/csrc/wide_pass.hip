// Wide-P IRLS path (DLSA_MAX_P_FUSED < P <= DLSA_MAX_P): BASELINE config 5
// (n = 5e6, p = 500, K = 32; mirrors projects/results/speedtest/
// logistic_LBFGS_local.py:12-13).  Same per-partition contract as the fused
// pass (dlsa/models.py:110-131: MLE theta_k, Sig_inv_k = X_k^T W X_k at
// theta_k), but the P x P Hessian no longer fits a workgroup's registers and
// LDS, so one Newton iteration is split into launches:
//
//   wide_fused_bf16_kernel  PHASE_F32 partitions (MIXED mode): ONE stream of X
//                       gives eta, w, the fp64 gradient / log-lik AND the
//                       approximate Hessian Z^T Z, Z = bf16(sqrt(w) x)
//                       (bf16 MFMA 16x16x32, fp32 accumulation).
//   wide_row_kernel     PHASE_F64 partitions: one streaming pass over X
//                       (HBM-bound): eta, mu, w = mu(1-mu), gradient, log-lik;
//                       writes w[row] (8 B/row) and per-chunk partials.
//   wide_gram_kernel    PHASE_F64: X^T diag(w) X as 128x128 lower-triangle
//                       output tiles, split over row groups (fp64 MFMA
//                       16x16x4, MFMA-bound).  blockIdx -> (row group, tile)
//                       is XCD-aware: all tiles of a row group run on one XCD,
//                       so its rows are fetched from HBM once and re-read from
//                       that XCD's L2 / the MALL.
//   wide_assemble_kernel  fixed-order sum of the row-group partials into the
//                       padded PP x PP Hessian of each partition (identity on
//                       the padding) -- deterministic.
//   wide_newton_kernel  one 1024-thread workgroup per partition: step
//                       control, publish Sig_inv, blocked right-looking
//                       Cholesky (32-column panels staged in LDS, trailing
//                       update on fp64 MFMA, the next diagonal block
//                       factored under the current trailing update),
//                       blocked triangular solves, update / convergence
//                       (same state machine as newton_solve.hip).
#include <math.h>
#include <stdlib.h>

#include "dlsa_internal.hpp"
#include "irls_wave_impl.hpp"  // wv_* wave helpers

// wide Newton: lookahead Cholesky with inverted diagonal blocks (1) or the
// round-4 panel sequence (0, A/B)
#ifndef DLSA_WN_LOOKAHEAD
#define DLSA_WN_LOOKAHEAD 1
#endif
// wide Newton: the trailing update of the approximate iterations on the f32
// MFMA (1) or on the fp64 MFMA like the exact ones (0, A/B)
#ifndef DLSA_WN_F32
#define DLSA_WN_F32 1
#endif
// rows per wave and step of the wide row pass (A/B builds)
#ifndef DLSA_WIDE_ROW_U
#define DLSA_WIDE_ROW_U 4
#endif

// Profiling build (DLSA_WN_PROF, tools/build_variants.sh wnprof): cycle stamps
// of the wide Newton kernel's stages, summed over workgroup runs into
// g_wn_prof (one vector atomic per stage per run; wave 1 stamps its share of
// the trailing update)
#ifdef DLSA_WN_PROF
static __device__ unsigned long long g_wn_prof[16];
#define WN_STAMP(v) uint64_t v = __builtin_readcyclecounter()
#define WN_ADD(i, d) \
  if (lane == 0) atomicAdd(&g_wn_prof[i], (unsigned long long)(d))
#else
#define WN_STAMP(v)
#define WN_ADD(i, d)
#endif

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
// padded LDS row stride of a panel (doubles).  CB + 2: the MFMA operand reads
// Lp[(16 t + fl) LDP + 4 s + kq] of a 32-lane group (fl < 16, kq < 2) then fall
// on banks 4 fl + 2 kq (+1), all 64 distinct; CB + 1 put (fl, kq = 1) and
// (fl + 1, kq = 0) on one bank pair (2-way).  The row-per-thread reads of the
// panel solve take the 2-way instead (16x fewer instructions).
#ifndef DLSA_WN_LDP
#define DLSA_WN_LDP (CB + 2)
#endif
constexpr int LDP = DLSA_WN_LDP;
static_assert(LDP > CB, "the padding slot CB holds the reciprocal pivots");
static_assert((CB * LDP + DLSA_MAX_P * LDP + 2 * DLSA_MAX_P + 64) * 8 <= 160 * 1024,
              "wide_newton_kernel LDS at PP = DLSA_MAX_P");

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
  if (a.phase[part] != PHASE_F64) return;  // workgroup-uniform (PHASE_F32: fused pass)
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
  // int8 exact Gram: running max of |sqrt(w) x| high dwords per feature
  const bool zm_on = a.slab_zmax != nullptr;
  uint32_t zmx[MB];
#pragma unroll
  for (int m = 0; m < MB; ++m) zmx[m] = 0u;
  constexpr int U = DLSA_WIDE_ROW_U;  // rows per wave per step (all U rows' loads in flight)
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
      if (zm_on) {
        const double sw = valid ? sqrt(w) : 0.0;
#pragma unroll
        for (int m = 0; m < MB; ++m)
          zmx[m] = max(zmx[m], (uint32_t)__double2hiint(xv[u][m] * sw) & 0x7FFFFFFFu);
      }
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
  if (zm_on) {
    __shared__ uint32_t zred[4 * 64 * MB];
#pragma unroll
    for (int m = 0; m < MB; ++m) zred[wid * 64 * MB + lane + 64 * m] = zmx[m];
    __syncthreads();
    for (int f = tid; f < PP; f += 256)
      a.slab_zmax[(int64_t)chunk * PP + f] =
          max(max(zred[f], zred[PP + f]), max(zred[2 * PP + f], zred[3 * PP + f]));
  }
}

// ---------------------------------------------------------------------------
// exact Gram pass: 256 threads = 4 waves per 128x128 output tile (I, J),
// I >= J; wave (qi = w >> 1, qj = w & 1) owns the 64 x 64 quadrant rows
// 64 qi .., columns 64 qj .. (the strictly-upper quadrant of a diagonal tile
// is skipped): 4 x 4 accumulators of v_mfma_f64_16x16x4_f64 (128 AGPRs), 16
// MFMAs per k-step of 4 rows against 8 operand loads + w -- fp64 VALU work
// and fp64 MFMAs do not overlap on a SIMD, so the VALU per MFMA is what the
// wave tile has to minimise.  Operands come straight from X by raw buffer
// loads: lane l reads row (l >> 4) of the k-step at feature (l & 15) of each
// 16-wide sub-tile, per-lane offsets fixed, the k-step advancing the uniform
// soffset (no address VALU); rows past the row group and columns >= p read 0
// through the buffer range check.  Four k-steps of operands in flight.
// ---------------------------------------------------------------------------
template <bool STD>
__global__ __launch_bounds__(256, 2) void wide_gram_kernel(const WideArgs a) {
  const int NB = a.NB;
  const int TB = NB * (NB + 1) / 2;
  const int bid = blockIdx.x;
  const int xcd = bid & 7, j8 = bid >> 3;  // workgroups are dealt to XCDs round-robin
  const int cl = j8 / TB, t = j8 - cl * TB;
  const int chunk = cl * 8 + xcd;  // all TB tiles of a row group on one XCD
  if (chunk >= a.n_gchunks) return;
  const int part = a.gc_part[chunk];
  if (a.phase[part] != PHASE_F64) return;
  int I, J;
  tile_ij(t, I, J);
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int qi = wid >> 1, qj = wid & 1;
  if (I == J && qi == 0 && qj == 1) return;  // strictly-upper quadrant of a diagonal tile
  const int p = a.p, ic = a.intercept;
  const int64_t row0 = a.gc_row0[chunk];
  const int nrows = __builtin_amdgcn_readfirstlane(a.gc_rows[chunk]);
  const int fl = lane & 15, kq = lane >> 4;

  // per-lane operand offsets (row kq of a k-step), 0x80000000 = column >= p
  int offA[4], offB[4];
  bool oneA = false, oneB = false;
  double cA[4], sA[4], cB[4], sB[4];
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    const int fa = GT * I + 64 * qi + 16 * s + fl, ja = fa - ic;
    const int fb = GT * J + 64 * qj + 16 * s + fl, jb = fb - ic;
    offA[s] = (ja >= 0 && ja < p) ? (kq * p + ja) * 8 : (int)0x80000000;
    offB[s] = (jb >= 0 && jb < p) ? (kq * p + jb) * 8 : (int)0x80000000;
    if (s == 0) {
      oneA = ic && fa == 0;
      oneB = ic && fb == 0;
    }
    cA[s] = cB[s] = 0.0;
    sA[s] = sB[s] = 1.0;
    if constexpr (STD) {
      if (ja >= 0 && ja < p) {
        sA[s] = 1.0 / a.scale[ja];
        cA[s] = a.center[ja] * sA[s];
      }
      if (jb >= 0 && jb < p) {
        sB[s] = 1.0 / a.scale[jb];
        cB[s] = a.center[jb] * sB[s];
      }
    }
  }
  const __amdgpu_buffer_rsrc_t xr =
      wv_rsrc((uintptr_t)(a.X + row0 * p), (uintptr_t)nrows * (uintptr_t)p * 8u);
  const __amdgpu_buffer_rsrc_t wr = wv_rsrc((uintptr_t)(a.w + row0), (uintptr_t)nrows * 8u);

  d4w acc[4][4];
#pragma unroll
  for (int s = 0; s < 4; ++s)
#pragma unroll
    for (int u = 0; u < 4; ++u) acc[s][u] = d4w{0, 0, 0, 0};

  struct Frag {
    double xa[4], xb[4], w;
  };
  auto load = [&](int step, Frag& F) {
    const int so = step * 4 * p * 8;  // k-step rows 4 step .. 4 step + 3
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      F.xa[s] = __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(xr, offA[s], so, 0));
      F.xb[s] = __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(xr, offB[s], so, 0));
    }
    F.w = __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(wr, kq * 8, step * 32, 0));
  };
  auto compute = [&](const Frag& F) {
    double av[4], bv[4];
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      double x = F.xa[s], z = F.xb[s];
      if constexpr (STD) {
        x = fma(x, sA[s], -cA[s]);
        z = fma(z, sB[s], -cB[s]);
      }
      if (s == 0) {
        if (oneA) x = 1.0;
        if (oneB) z = 1.0;
      }
      av[s] = x * F.w;  // rows past the group: w = 0
      bv[s] = z;
    }
#pragma unroll
    for (int s = 0; s < 4; ++s)
#pragma unroll
      for (int u = 0; u < 4; ++u)
        acc[s][u] = __builtin_amdgcn_mfma_f64_16x16x4f64(av[s], bv[u], acc[s][u], 0, 0, 0);
  };
  const int nsteps = (nrows + 3) / 4;
  constexpr int DEPTH = 4;  // k-steps of operands in flight
  if (nsteps > 0) {
    Frag f[DEPTH];
#pragma unroll
    for (int d = 0; d < DEPTH; ++d) load(d, f[d]);  // past the end: range-checked zeros
    for (int s0 = 0; s0 < nsteps; s0 += DEPTH) {  // a ragged last group adds zeros
#pragma unroll
      for (int d = 0; d < DEPTH; ++d) {
        compute(f[d]);
        load(s0 + DEPTH + d, f[d]);
      }
#pragma unroll
      for (int s = 0; s < 4; ++s)
#pragma unroll
        for (int u = 0; u < 4; ++u) asm volatile("" : "+a"(acc[s][u]));
    }
  }

  // C/D map of the f64 16x16x4 MFMA: row = (l >> 4) + 4 r, column = l & 15
  double* G = a.slab_G + ((int64_t)chunk * TB + t) * (GT * GT);
#pragma unroll
  for (int s = 0; s < 4; ++s)
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int i = 64 * qi + 16 * s + kq + 4 * r;
        const int jc = 64 * qj + 16 * u + fl;
        G[i * GT + jc] = acc[s][u][r];
      }
}

// ---------------------------------------------------------------------------
// fused approximate pass (MIXED mode, logistic, PHASE_F32 partitions): ONE
// stream of X per Newton iteration yields both the row quantities (eta, w, r,
// the fp64 gradient X^T (y - mu) and log-likelihood) and the approximate
// Hessian  H~ = Z^T Z,  Z = bf16(sqrt(w) x)  (positive semi-definite by
// construction; DESIGN.md 4.2: it only steers Newton, the fp64 pass fixes the
// solution and publishes Sig_inv).
//
// Register budget first: the fp32 accumulators of the P x P lower triangle
// (528 16x16 tiles = 528 KB at PP = 512) exceed a CU's register file, so
// S = 2 workgroups share a row group above PP = 256, each owning half of the
// tile rows; they are dispatched back to back onto one XCD, so the second
// stream of the rows is an L2 / MALL hit.  A workgroup is 4 waves, ONE per
// SIMD, so each wave has the full 512 registers: ~256 accumulator registers
// (AGPRs) + a 32-row block of X in flight (128 VGPRs) + the row work.
//
// Per 32-row block (wave w holds rows 8w .. 8w+7 in registers; raw buffer
// loads, 16 B per lane at even p: lane l owns columns 2l + 128 j (+1); rows or
// columns past the end read as 0 through the buffer range check):
//   1. eta of the 8 rows: lane partials, then a reduce-scatter over the lanes
//      (permlane32 / permlane16 swaps, one DPP swap, DPP within 8 lanes) --
//      lane group l >> 3 ends with row l >> 3, bitwise-identical in the group;
//   2. w, r, log-lik: ONE fp64 exp / reciprocal sequence for the 8 rows,
//      broadcast by readlane; the softplus sum is a running product
//      (frexp-normalised), one log per lane at the end;
//   3. per half of 4 rows: gradient FMAs (group 0 only), the half's Z plane
//      (see zplane_bytes), and the loads of the same half of block b+1 into
//      the freed registers -- in flight across the other half, the barrier
//      and the MFMA phase;
//   4. one LDS barrier (no vmcnt drain) and the MFMA phase:
//      v_mfma_f32_16x16x32_bf16, operand lane (i, kg) = feature i, rows
//      8 kg .. 8 kg + 7.
// Wave slot s = 4 sg + w owns the tile-row pairs q = s + 4 S k: rows q and
// NT16 - 1 - q, NT16 + 1 tiles per pair (2 pairs = 66 tiles at PP = 512).
// Double-buffered Z images: one barrier per block.  Output: the
// 128 x 128-tile slab layout of wide_gram_kernel (slab_G) and per-row-group
// gradient / log-lik partials (slab_gz / slab_llz) summed in fixed order --
// deterministic.
// ---------------------------------------------------------------------------
typedef __bf16 bf16x8w __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4w __attribute__((ext_vector_type(4)));
typedef float f4w __attribute__((ext_vector_type(4)));
typedef double d2w __attribute__((ext_vector_type(2)));

#ifndef DLSA_FUSED_ABLATE
#define DLSA_FUSED_ABLATE 0
#endif

namespace {
constexpr int FW = 4;   // waves per workgroup of the fused pass
// Z image of a 32-row block: 8 planes (wave w, half h = rows 8w + 4h .. +3),
// each [PP features][4 rows] bf16 (8 B per feature) + 64 B pad.  A half's
// store (one ds_write_b64 per lane and column, features 2 apart across the
// lanes) is 2-way conflicted; an MFMA operand (feature i, rows 8 kg .. +7) is
// two ds_read_b64 from planes 2 kg and 2 kg + 1, conflict-free: the plane
// pad moves kg = 1 (lanes 16-31) onto the other 32 banks of lanes 0-15.
__host__ __device__ constexpr int zplane_bytes(int NT16) { return 16 * NT16 * 8 + 64; }
__host__ __device__ constexpr int zimg_bytes(int NT16) { return 8 * zplane_bytes(NT16); }
__host__ __device__ constexpr int fused_groups(int NT16) { return NT16 > 16 ? 2 : 1; }
__host__ __device__ constexpr int fused_pairs_per_slot(int NT16) {
  return (NT16 / 2 + FW * fused_groups(NT16) - 1) / (FW * fused_groups(NT16));
}
// [2] Z images, [PP] scaled beta, [2][PP] 1/scale and center/scale,
// [FW][PP] gradient reduction, [32] misc
__host__ __device__ constexpr int fused_lds_bytes(int NT16) {
  return 2 * zimg_bytes(NT16) + (3 + FW) * 16 * NT16 * 8 + 256;
}

// Sum over the 64 lanes; every lane ends with the bitwise-identical total
// (each step adds a value and its partner's under a lane involution, so the
// pair computes a + b and b + a).
__device__ __forceinline__ double wave_allsum(double v) {
  v += wv_dpp<0x141>(v);  // row_half_mirror: i <-> 7 - i
  v += wv_dpp<0xB1>(v);   // quad_perm [1, 0, 3, 2]
  v += wv_dpp<0x4E>(v);   // quad_perm [2, 3, 0, 1]
  v += wv_dpp<0x140>(v);  // row_mirror: i <-> 15 - i
  v = wv_xor16(v);
  v = wv_xor32(v);
  return v;
}

// v_permlane32_swap / v_permlane16_swap of a double pair (a, b): after the
// swap, lanes of the lower half of each 2H-lane group see (a, a of lane + H),
// lanes of the upper half (b of lane - H, b)
template <int H>
__device__ __forceinline__ double swap_add(double a, double b) {
  const unsigned alo = __double2loint(a), ahi = __double2hiint(a);
  const unsigned blo = __double2loint(b), bhi = __double2hiint(b);
  if constexpr (H == 32) {
    const auto lo = __builtin_amdgcn_permlane32_swap(alo, blo, false, false);
    const auto hi = __builtin_amdgcn_permlane32_swap(ahi, bhi, false, false);
    return __hiloint2double(hi[0], lo[0]) + __hiloint2double(hi[1], lo[1]);
  } else {
    const auto lo = __builtin_amdgcn_permlane16_swap(alo, blo, false, false);
    const auto hi = __builtin_amdgcn_permlane16_swap(ahi, bhi, false, false);
    return __hiloint2double(hi[0], lo[0]) + __hiloint2double(hi[1], lo[1]);
  }
}

// 4 row partials per lane -> lane l holds the total of row l >> 4 (every lane
// of the 16-lane group bitwise-identical)
__device__ __forceinline__ double reduce_scatter4(const double (&v)[4], int lane) {
  (void)lane;
  // lanes 0-31 rows 0, 1; lanes 32-63 rows 2, 3
  const double s0 = swap_add<32>(v[0], v[2]), s1 = swap_add<32>(v[1], v[3]);
  // 16-lane groups: rows 0, 1, 2, 3
  double r = swap_add<16>(s0, s1);
  r += wv_dpp<0x141>(r);  // row_half_mirror: i <-> 7 - i
  r += wv_dpp<0xB1>(r);   // quad_perm [1, 0, 3, 2]
  r += wv_dpp<0x4E>(r);   // quad_perm [2, 3, 0, 1]
  r += wv_dpp<0x140>(r);  // row_mirror: i <-> 15 - i
  return r;
}

// 8 row partials per lane -> lane l holds the total of row l >> 3 (every lane
// of the 8-lane group bitwise-identical)
__device__ __forceinline__ double reduce_scatter8(const double (&v)[8], int lane) {
  // lanes 0-31 rows 0..3, lanes 32-63 rows 4..7
  const double s0 = swap_add<32>(v[0], v[4]), s1 = swap_add<32>(v[1], v[5]);
  const double s2 = swap_add<32>(v[2], v[6]), s3 = swap_add<32>(v[3], v[7]);
  // 16-lane groups: t0 rows 0, 2, 4, 6; t1 rows 1, 3, 5, 7
  const double t0 = swap_add<16>(s0, s2), t1 = swap_add<16>(s1, s3);
  // 8-lane groups: lanes with bit 3 clear keep t0's row, set keep t1's
  const bool b3 = (lane & 8) != 0;
  const double keep = b3 ? t1 : t0, give = b3 ? t0 : t1;
  double r = keep + wv_dpp<0x128>(give);  // row_ror 8: lane l ^ 8 within 16
  r += wv_dpp<0x141>(r);                  // row_half_mirror: i <-> 7 - i
  r += wv_dpp<0xB1>(r);                   // quad_perm [1, 0, 3, 2]
  r += wv_dpp<0x4E>(r);                   // quad_perm [2, 3, 0, 1]
  return r;
}

__device__ __forceinline__ double rdlane_f64(double v, int l) {
  const int lo = __builtin_amdgcn_readlane(__double2loint(v), l);
  const int hi = __builtin_amdgcn_readlane(__double2hiint(v), l);
  return __hiloint2double(hi, lo);
}

typedef float f2w __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2w __attribute__((ext_vector_type(2)));
__device__ __forceinline__ unsigned pack_bf16x2(float a, float b) {  // v_cvt_pk_bf16_f32
  return __builtin_bit_cast(unsigned, __builtin_convertvector(f2w{a, b}, bf16x2w));
}
}  // namespace

template <bool STD, int NT16, bool VEC2>
__global__ __launch_bounds__(64 * FW, 1) void wide_fused_bf16_kernel(const WideArgs a) {
  constexpr int S = fused_groups(NT16);
  constexpr int PP = 16 * NT16;
  constexpr int NF = PP / 64;     // columns per lane of each row
  constexpr int HALF = NT16 / 2;  // tile-row pairs
  constexpr int PPS = fused_pairs_per_slot(NT16);
  constexpr int TPP = NT16 + 1;   // tiles per pair
  constexpr int NT = 64 * FW;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int ZPL = zplane_bytes(NT16), ZIMG = zimg_bytes(NT16);
  char* zimg = smem;                            // [2] Z images
  double* bl = (double*)(smem + 2 * ZIMG);      // [PP] beta (x 1/scale) by column
  double* sd = bl + PP;                         // [2][PP] 1/scale, center/scale (STD)
  double* red = sd + 2 * PP;                    // [FW][PP] gradient of each wave
  double* misc = red + FW * PP;                 // [0] eta offset, [8..] log-lik, [16..] sum r

  const int bid = blockIdx.x;
  const int xcd = bid & 7, j8 = bid >> 3;
  const int sg = j8 % S, cl = j8 / S;
  const int chunk = cl * 8 + xcd;  // the S workgroups of a row group on one XCD
  if (chunk >= a.n_gchunks) return;
  const int part = __builtin_amdgcn_readfirstlane(a.gc_part[chunk]);
  if (a.phase[part] != PHASE_F32) return;  // workgroup-uniform
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int p = a.p, P = a.P, ic = a.intercept;
  const int64_t row0 = a.gc_row0[chunk];
  const int nrows = __builtin_amdgcn_readfirstlane(a.gc_rows[chunk]);
  const int nb = (nrows + 31) / 32;
  const double* th = a.theta + (int64_t)part * P;

  // ---- setup: zero Z images (padding features stay 0), beta, eta offset ----
  for (int o = tid * 16; o < 2 * ZIMG; o += NT * 16) *(uint4*)(zimg + o) = make_uint4(0, 0, 0, 0);
  for (int c = tid; c < PP; c += NT) {
    double is = 1.0, cs = 0.0;
    if constexpr (STD) {
      if (c < p) {
        is = 1.0 / a.scale[c];
        cs = a.center[c] * is;
      }
    }
    bl[c] = c < p ? th[c + ic] * is : 0.0;
    sd[c] = is;
    sd[PP + c] = cs;
  }
  if (wid == 0) {  // eta offset: intercept - sum_c beta_c center_c / scale_c
    double s = 0.0;
    if constexpr (STD)
      for (int c = lane; c < p; c += 64) s += th[c + ic] * (a.center[c] / a.scale[c]);
    s = wave_allsum(s);
    if (lane == 0) misc[0] = (ic ? th[0] : 0.0) - s;
  }
  __syncthreads();
  const double eoff = bcast_first(misc[0]);

  auto colf = [&](int m) { return VEC2 ? 2 * lane + 128 * (m >> 1) + (m & 1) : lane + 64 * m; };
  const int rl = lane >> 3;  // the row of the wave this lane's transcendental work is for

  // per-lane byte offset of each column group in the wave's first row (out of
  // range columns: an offset past any buffer -> reads 0); row u adds u p 8
  // through the uniform soffset
  constexpr int NV = VEC2 ? NF / 2 : NF;
  int voff[NV];
#pragma unroll
  for (int v = 0; v < NV; ++v) {
    const int c = colf(VEC2 ? 2 * v : v);
    voff[v] = c < p ? (8 * wid * p + c) * 8 : 0x7FFFFFF0;
  }
  double xv[8][NF];
  double yv = 0.0;
  // rows 4 h .. 4 h + 3 of this wave in block b (with h = 0: y of row rl).
  // Block nb (one past the last) is issued too, with an empty buffer range
  // (all loads return 0, no memory access): every loop iteration then has
  // the same loads in flight, so the compiler's vmcnt bookkeeping never
  // merges an "issued" and a "not issued" path into a full drain.
  auto issue = [&](int b, int h) {
#if DLSA_FUSED_ABLATE == 1  // profiling only: every block re-reads block 0 (L2-resident)
    const int64_t rb = row0 + 32LL * min(b, nb > 0 ? 0 : b);
#else
    const int64_t rb = row0 + 32LL * b;
#endif
    const int rows = max(0, min(32, nrows - 32 * b));
    const __amdgpu_buffer_rsrc_t xr =
        wv_rsrc((uintptr_t)(a.X + rb * p), (uintptr_t)rows * (uintptr_t)p * 8u);
    const __amdgpu_buffer_rsrc_t yr = wv_rsrc((uintptr_t)(a.y + rb), (uintptr_t)rows * 8u);
#pragma unroll
    for (int u = 4 * h; u < 4 * h + 4; ++u) {
      const int so = u * p * 8;
#pragma unroll
      for (int v = 0; v < NV; ++v) {
        if constexpr (VEC2) {
          const d2w d =
              __builtin_bit_cast(d2w, __builtin_amdgcn_raw_buffer_load_b128(xr, voff[v], so, 0));
          xv[u][2 * v] = d.x;
          xv[u][2 * v + 1] = d.y;
        } else {
          xv[u][v] =
              __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(xr, voff[v], so, 0));
        }
      }
    }
    if (h == 0)
      yv = __builtin_bit_cast(double,
                              __builtin_amdgcn_raw_buffer_load_b64(yr, (8 * wid + rl) * 8, 0, 0));
  };

  double gacc[NF];
#pragma unroll
  for (int m = 0; m < NF; ++m) gacc[m] = 0.0;
  // log-lik: sum of y eta - max(eta, 0) on the first lane of each row group,
  // and the softplus term as a running product of t = 1 + exp(-|eta|) in
  // [1, 2] kept as mantissa x 2^lexp (frexp each block: exact) -- one log per
  // lane at the end instead of one per row, and no more rounding than a sum
  // of per-row logs
  double rsum = 0.0, llacc = 0.0, lprod = 1.0;
  int lexp = 0;
  f4w acc[PPS][TPP];
#pragma unroll
  for (int k = 0; k < PPS; ++k)
#pragma unroll
    for (int i = 0; i < TPP; ++i) acc[k][i] = f4w{0.f, 0.f, 0.f, 0.f};
  const int slot = sg * FW + wid;
  const int fl = lane & 15, kg = lane >> 4;

  if (nb > 0) {
    issue(0, 0);
    issue(0, 1);
  }
  for (int b = 0; b < nb; ++b) {
    // ---- row phase: eta, w, r, log-lik of the wave's 8 rows (one
    // transcendental sequence), then per half of 4 rows the gradient, the Z
    // entries and the loads of that half of block b+1: those stay in flight
    // across the other half, the barrier and the MFMA phase ----------------
    double e8[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      double e0 = 0.0, e1 = 0.0;
#pragma unroll
      for (int m = 0; m < NF; ++m) {
        const double bm = bl[colf(m)];
        if (m & 1)
          e1 = fma(xv[u][m], bm, e1);
        else
          e0 = fma(xv[u][m], bm, e0);
      }
      e8[u] = e0 + e1;
    }
    const double eu = reduce_scatter8(e8, lane) + eoff;  // row rl of the wave
    const bool vrow = 32 * b + 8 * wid + rl < nrows;
    const double ea = exp(-fabs(eu));
    const double inv = wv_rcp(1.0 + ea);
    const double mu = eu >= 0.0 ? inv : ea * inv;
    const double w = ea * inv * inv;  // mu (1 - mu), cancellation free
    const double r = vrow ? yv - mu : 0.0;
    if (sg == 0 && (lane & 7) == 0 && vrow) {
      llacc += yv * eu - fmax(eu, 0.0);
      lprod *= 1.0 + ea;
    }
    {
      int e2;
      lprod = frexp(lprod, &e2);
      lexp += e2;
    }
    const float swl = vrow ? sqrtf((float)w) : 0.f;
    char* zb = zimg + (b & 1) * ZIMG;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      float sw[4];
#pragma unroll
      for (int u = 0; u < 4; ++u)
        sw[u] = __builtin_bit_cast(
            float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, swl), 8 * (4 * h + u)));
      if (sg == 0) {  // workgroup-uniform: group 0 accumulates the gradient
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const double ru = rdlane_f64(r, 8 * (4 * h + u));
          rsum += ru;
#pragma unroll
          for (int m = 0; m < NF; ++m) gacc[m] = fma(xv[4 * h + u][m], ru, gacc[m]);
        }
      }
      // Z entries: plane (wid, h), this half's 4 rows of each of the lane's columns
      char* zp = zb + (2 * wid + h) * ZPL;
#pragma unroll
      for (int m = 0; m < NF; ++m) {
        const int c = colf(m);
        float zf[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          double v = xv[4 * h + u][m];
          if constexpr (STD) v = fma(v, sd[c], -sd[PP + c]);
          float f = (float)v;
          asm volatile("" : "+v"(f));  // keep f64 -> f32 -> bf16 (see irls_coop_impl.hpp)
          zf[u] = f * sw[u];
        }
        // columns c >= p read as 0 and write 0 into padding features; only the
        // last column can map past the plane (c + ic = PP)
        if (m < NF - 1 || c + ic < PP)
          *(uint2*)(zp + (c + ic) * 8) = make_uint2(pack_bf16x2(zf[0], zf[1]), pack_bf16x2(zf[2], zf[3]));
      }
      if (ic && lane == 0)  // intercept column: z = sqrt(w)
        *(uint2*)zp = make_uint2(pack_bf16x2(sw[0], sw[1]), pack_bf16x2(sw[2], sw[3]));
      issue(b + 1, h);
    }
    // this wave's Z writes done; every wave's image b complete and image b-1 consumed
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");

    // ---- MFMA phase: per pair q, tile rows NT16 - 1 - q (J < nh) and q ------
    // operand (feature 16 J + fl, rows 8 kg .. 8 kg + 7): planes 2 kg, 2 kg + 1
    const char* base = zimg + (b & 1) * ZIMG + 2 * kg * ZPL + fl * 8;
    auto op = [&](int J) {
      const bf16x4w lo = *(const bf16x4w*)(base + 16 * J * 8);
      const bf16x4w hi = *(const bf16x4w*)(base + ZPL + 16 * J * 8);
      return __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
    };
    // Tile i of pair q: the upper row NT16 - 1 - q holds i < nh = NT16 - q
    // (J = i), the lower row q the rest, stored from the end (J = NT16 - i).
    // Over the slots that share pair index k, q spans [qlo, qhi], so tiles
    // i < NT16 - qhi are upper-row and i >= NT16 - qlo lower-row for every
    // slot -- compile-time operands; only the 7 tiles in between pick their
    // row at run time (uniform LDS offsets, no register selects).
    constexpr int D = 2;  // B operands read D tiles ahead of their MFMA
#pragma unroll
    for (int k = 0; k < PPS; ++k) {
      const int q = slot + FW * S * k;
      if (q < HALF) {  // wave-uniform
        const int nh = NT16 - q;
        const int qlo = FW * S * k, qhi = min(HALF - 1, FW * S * k + FW * S - 1);
        const int st_hi = NT16 - qhi, st_lo = NT16 - qlo;  // compile-time after unrolling
        const bf16x8w ahi = op(NT16 - 1 - q), alo = op(q);
        auto jof = [&](int i) { return (i < st_hi || (i < st_lo && i < nh)) ? i : NT16 - i; };
        bf16x8w bq[D + 1], aq[D + 1];
        auto rd = [&](int i) {
          bq[i % (D + 1)] = op(jof(i));
          if (i >= st_hi && i < st_lo) aq[i % (D + 1)] = op(i < nh ? NT16 - 1 - q : q);
        };
#pragma unroll
        for (int i = 0; i < D; ++i) rd(i);
#pragma unroll
        for (int i = 0; i < TPP; ++i) {
          if (i + D < TPP) rd(i + D);
          const bf16x8w av = i < st_hi ? ahi : (i >= st_lo ? alo : aq[i % (D + 1)]);
          acc[k][i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av, bq[i % (D + 1)], acc[k][i], 0, 0, 0);
          __builtin_amdgcn_sched_barrier(0);
        }
      }
    }
    // keep the accumulators in AGPRs across the loop back edge (the first 64
    // tiles: 256 AGPRs; at PP = 512 the last 2 tiles of a slot stay in VGPRs)
#pragma unroll
    for (int k = 0; k < PPS; ++k)
#pragma unroll
      for (int i = 0; i < TPP; ++i) {
        if (k * TPP + i < 64)
          asm volatile("" : "+a"(acc[k][i]));
        else
          asm volatile("" : "+v"(acc[k][i]));
      }
  }

  // ---- epilogue: Gram tiles (C/D map of the f32 16x16 MFMAs: row = 4 kg + r,
  // column = fl), 128 x 128-tile slab layout -----------------------------------
  {
    constexpr int NB = NT16 / 8;
    constexpr int TB = NB * (NB + 1) / 2;
#pragma unroll
    for (int k = 0; k < PPS; ++k) {
      const int q = slot + FW * S * k;
      if (q >= HALF) continue;
      const int nh = NT16 - q;
#pragma unroll
      for (int i = 0; i < TPP; ++i) {
        const bool hi = i < nh;
        const int I = hi ? NT16 - 1 - q : q;
        const int J = hi ? i : NT16 - i;
        const int I8 = I >> 3, J8 = J >> 3;
        double* G = a.slab_G + ((int64_t)chunk * TB + I8 * (I8 + 1) / 2 + J8) * (GT * GT);
#pragma unroll
        for (int r = 0; r < 4; ++r)
          G[(16 * (I & 7) + 4 * kg + r) * GT + 16 * (J & 7) + fl] = (double)acc[k][i][r];
      }
    }
  }
  if (sg != 0) return;  // workgroup-uniform: group 0 publishes the gradient
  // ---- gradient / log-lik partials: fixed-order sum over the waves ---------
#pragma unroll
  for (int m = 0; m < NF; ++m) red[wid * PP + colf(m)] = gacc[m];
  if ((lane & 7) == 0) llacc -= log(lprod) + lexp * 0.6931471805599453094;
  llacc = wave_allsum(llacc);
  if (lane == 0) {
    misc[8 + wid] = llacc;
    misc[16 + wid] = rsum;
  }
  __syncthreads();
  double rs = 0.0;
#pragma unroll
  for (int v = 0; v < FW; ++v) rs += misc[16 + v];
  for (int f = tid; f < PP; f += NT) {
    const int c = f - ic;
    double g = 0.0;
    if (ic && f == 0) {
      g = rs;
    } else if (c < p) {
      double s = 0.0;
#pragma unroll
      for (int v = 0; v < FW; ++v) s += red[v * PP + c];
      g = STD ? fma(sd[c], s, -sd[PP + c] * rs) : s;
    }
    a.slab_gz[(int64_t)chunk * PP + f] = g;
  }
  if (tid == 0) {
    double ll = 0.0;
#pragma unroll
    for (int v = 0; v < FW; ++v) ll += misc[8 + v];
    a.slab_llz[chunk] = ll;
  }
}

template <bool STD, int NT16>
static hipError_t launch_fused_t(const WideArgs& a, hipStream_t s) {
  const bool vec2 = (a.p % 2 == 0) && ((uintptr_t)a.X % 16 == 0);
  const void* kern = vec2 ? (const void*)wide_fused_bf16_kernel<STD, NT16, true>
                          : (const void*)wide_fused_bf16_kernel<STD, NT16, false>;
  const int lds = fused_lds_bytes(NT16);
  {
    hipError_t e = ensure_max_lds(kern, lds);
    if (e != hipSuccess) return e;
  }
  const int grid = ((a.n_gchunks + 7) / 8) * 8 * fused_groups(NT16);
  if (vec2)
    hipLaunchKernelGGL((wide_fused_bf16_kernel<STD, NT16, true>), dim3(grid), dim3(64 * FW), lds, s,
                       a);
  else
    hipLaunchKernelGGL((wide_fused_bf16_kernel<STD, NT16, false>), dim3(grid), dim3(64 * FW), lds,
                       s, a);
  return hipGetLastError();
}

hipError_t launch_wide_fused(const WideArgs& a, bool standardize, hipStream_t s) {
  if (a.n_gchunks <= 0) return hipSuccess;
  switch (a.NB) {
    case 2: return standardize ? launch_fused_t<true, 16>(a, s) : launch_fused_t<false, 16>(a, s);
    case 3: return standardize ? launch_fused_t<true, 24>(a, s) : launch_fused_t<false, 24>(a, s);
    case 4: return standardize ? launch_fused_t<true, 32>(a, s) : launch_fused_t<false, 32>(a, s);
    default: return hipErrorInvalidValue;
  }
}

// ---------------------------------------------------------------------------
// assemble: H[k] (PP x PP, both triangles, padding = identity) = sum of the
// row-group partials of partition k in row-group order.  grid (TB * 16, K):
// one workgroup per 32 x 32 block of a lower 128 x 128 tile (blocks above the
// diagonal of a diagonal tile exit); a thread sums 4 elements, all their
// row-group partials loaded before the adds (8 at a time), and the block is
// written row-major and, through LDS, transposed -- both coalesced.  (One
// workgroup per tile with one element's partials summed at a time, 320
// workgroups at config 5: 0.27 ms per launch.)
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void wide_assemble_kernel(const WideArgs a, const int32_t* gcb,
                                                            double* Hfull) {
  const int t = blockIdx.x >> 4, sb = blockIdx.x & 15, k = blockIdx.y;
  if (a.phase[k] != PHASE_F32 && a.phase[k] != PHASE_F64) return;
  const int NB = a.NB, TB = NB * (NB + 1) / 2, PP = GT * NB, P = a.P;
  int I, J;
  tile_ij(t, I, J);
  const int br = sb >> 2, bc = sb & 3;  // 32 x 32 block (br, bc) of the tile
  if (I == J && bc > br) return;
  __shared__ double tr[32][33];
  const int cb = gcb[k], ce = gcb[k + 1];
  double* H = Hfull + (int64_t)k * PP * PP;
  const int tc = threadIdx.x & 31, tr0 = threadIdx.x >> 5;
  double v[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) v[q] = 0.0;
  const double* base = a.slab_G + (int64_t)t * (GT * GT) + (32 * br + tr0) * GT + 32 * bc + tc;
  const int64_t cstride = (int64_t)TB * (GT * GT);
  int c = cb;
  for (; c + 8 <= ce; c += 8) {
    double x[8][4];
#pragma unroll
    for (int u = 0; u < 8; ++u)
#pragma unroll
      for (int q = 0; q < 4; ++q) x[u][q] = base[(int64_t)(c + u) * cstride + 8 * q * GT];
#pragma unroll
    for (int u = 0; u < 8; ++u)
#pragma unroll
      for (int q = 0; q < 4; ++q) v[q] += x[u][q];
  }
  for (; c < ce; ++c)
#pragma unroll
    for (int q = 0; q < 4; ++q) v[q] += base[(int64_t)c * cstride + 8 * q * GT];
  const bool diag = I == J && br == bc;  // a block on the matrix diagonal
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int il = 32 * br + tr0 + 8 * q, jl = 32 * bc + tc;
    const int i = GT * I + il, j = GT * J + jl;
    double s = v[q];
    if (i >= P || j >= P) s = (i == j) ? 1.0 : 0.0;
    tr[tr0 + 8 * q][tc] = s;
  }
  __syncthreads();
  // row-major block (rows 32 br .., columns 32 bc ..); on the diagonal the
  // upper triangle mirrors the lower
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int r = tr0 + 8 * q;
    const int i = GT * I + 32 * br + r, j = GT * J + 32 * bc + tc;
    H[(int64_t)i * PP + j] = (diag && tc > r) ? tr[tc][r] : tr[r][tc];
  }
  if (diag) return;
  // transposed block: H[j][i]
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int r = tr0 + 8 * q;  // row of the transposed block = column of tr
    const int j = GT * J + 32 * bc + r, i = GT * I + 32 * br + tc;
    H[(int64_t)j * PP + i] = tr[tc][r];
  }
}

// ---------------------------------------------------------------------------
// per-partition Newton update (one 1024-thread workgroup per partition)
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(1024) void wide_newton_kernel(const SolveArgs a, const WideArgs wa,
                                                           const int32_t* rcb, const int32_t* gcb,
                                                           double* Hfull) {
  extern __shared__ __attribute__((aligned(16))) double sm[];
  const int k = blockIdx.x;
  if (a.status[k] != STATUS_RUNNING) return;
  if (a.phase[k] != PHASE_F32 && a.phase[k] != PHASE_F64) return;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int P = a.P, PP = GT * wa.NB;
  WN_STAMP(t_k0);
  double* L11 = sm;             // [CB][LDP] diagonal block
  double* Lp = L11 + CB * LDP;  // [PP][LDP] panel below it (scratch in the solves)
  double* g = Lp + PP * LDP;    // [PP]
  double* z = g + PP;           // [PP]
  double* red = z + PP;         // [64]: [0..47] reductions, [40] ll, [48] flag
  int* flag = (int*)(red + 48);
  double* H = Hfull + (int64_t)k * PP * PP;

  // 1. gradient and log-likelihood of the pass, in chunk order: the fused
  // pass's row groups (PHASE_F32) or the row pass's chunks (PHASE_F64)
  const bool fz = a.phase[k] == PHASE_F32;
  const int cb = fz ? gcb[k] : rcb[k], ce = fz ? gcb[k + 1] : rcb[k + 1];
  const double* sg = fz ? wa.slab_gz : wa.slab_g;
  const double* sll = fz ? wa.slab_llz : wa.slab_ll;
  for (int f = tid; f < PP; f += 1024) {
    double s = 0.0;
    for (int c = cb; c < ce; ++c) s += sg[(int64_t)c * PP + f];
    g[f] = f < P ? s : 0.0;
  }
  if (wid == 0) {
    double s = 0.0;
    for (int c = cb + lane; c < ce; c += 64) s += sll[c];
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
  if (!a.eval_only && a.family == FAMILY_LOGISTIC && it > 0 &&
      ll < llp - 1e-6 * (1.0 + fabs(llp)) && a.backtracks[k] < 40) {
    const int bt = a.backtracks[k] + 1;
    const double sc = ldexp(1.0, -bt);
    const double* tp = a.theta_prev + (int64_t)k * P;
    const double* dp = a.delta_prev + (int64_t)k * P;
    for (int f = tid; f < P; f += 1024) th[f] = tp[f] + sc * dp[f];
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
  // 3. publish the information matrix at the evaluation point (models.py:130)
  // on exact-phase passes (the copy of P^2 values by one workgroup is skipped
  // on the approximate iterations: a partition whose budget ends in the
  // approximate phase gets its Sig_inv from the polish pass, eval_only, at
  // the theta it returns)
  if (!a.subsample) {
    if (phase == PHASE_F64) {
      double* S = a.sig_inv + (int64_t)k * P * P;
      for (int e = tid; e < P * P; e += 1024) {
        const int i = e / P, j = e - i * P;
        S[e] = H[(int64_t)i * PP + j];
      }
    }
    if (tid == 0) a.loglik[k] = ll;
  }
  if (a.eval_only) return;
  __syncthreads();

#if DLSA_WN_LOOKAHEAD
  WN_STAMP(t_f0);
  if (wid == 0) { WN_ADD(9, t_f0 - t_k0); WN_ADD(8, 1); }
  // 4. blocked Cholesky H = L L^T (lower, in place), one panel of lookahead:
  // while waves 1..15 apply panel jb's trailing update to the columns past
  // the next panel, wave 0 factors the next diagonal block (its columns were
  // updated first), so the pivot chain of a block runs under the previous
  // panel's MFMA work instead of between panels.  The reciprocal pivots are
  // kept, so the panel solve and the triangular solves multiply instead of
  // divide on their dependency chains.
  const int fl = lane & 15, kq = lane >> 4;
  const int wv = __builtin_amdgcn_readfirstlane(wid);
  // wave 0: factor diagonal block jb (lane i = row i; column j of L goes
  // through L11, column-major, to the other lanes; 1 / L[j][j] in its padding
  // slot); lanes 32..63 repeat lanes 0..31 and store the same values
  auto factor_diag = [&](int jb) {
    // the lane index re-defined opaquely: otherwise the compiler hoists the
    // lane-compare masks of the unrolled pivots and spills them (as in
    // newton_solve.hip)
    int lv = lane;
    asm volatile("" : "+v"(lv));
    const int i = lv & 31;
    const double* hr = H + (int64_t)(jb + i) * PP + jb;
    double row[CB];
#pragma unroll
    for (int c = 0; c < CB; ++c) {
      const double hv = hr[c];
      row[c] = c <= i ? hv : 0.0;
    }
    double dg = 1.0;  // this lane's diagonal entry L[i][i]
#pragma unroll
    for (int j = 0; j < CB; ++j) {
      const double d = bcast_f64(row[j], j);
      // 1 / sqrt(d) by v_rsq_f64 + two Newton steps (~1 ulp), L_jj = d / sqrt(d)
      // (NaN for a pivot that is not > 0 and finite: the flag below)
      double il = __builtin_amdgcn_rsq(d);
#pragma unroll
      for (int nr = 0; nr < 2; ++nr) il = fma(il, fma(-0.5 * d * il, il, 0.5), il);
      const double ljj = d * il;
      dg = i == j ? ljj : dg;
      row[j] = i > j ? row[j] * il : (i == j ? ljj : row[j]);
      L11[j * LDP + CB] = il;  // 1 / L[j][j] in the padding slot
#pragma unroll
      for (int c = j + 1; c < CB; ++c) {
        const double lcj = bcast_f64(row[j], c);  // L[c][j], row c's lane
        if (c <= i) row[c] = fma(-row[j], lcj, row[c]);
      }
    }
    double* hw = H + (int64_t)(jb + i) * PP + jb;
#pragma unroll
    for (int c = 0; c < CB; ++c) {
      hw[c] = row[c];
      L11[c * LDP + i] = row[c];  // column-major for the panel solve
    }
    if (__ballot(!(dg > 0.0 && isfinite(dg))) != 0 && lv == 0) *flag = 1;
  };
  // L21 = A21 L11^-T by right-looking substitution, one thread per row of the
  // panel (staged in Lp by coalesced loads): the chain per column is one
  // multiply by the stored reciprocal pivot, the updates of the later columns
  // are independent FMAs
  auto panel_copy = [&](int jb, int rest, bool to_lds) {
    for (int e = tid; e < rest * CB; e += 1024) {
      const int r = e >> 5, c = e & 31;
      double* hp = H + (int64_t)(jb + CB + r) * PP + jb + c;
      if (to_lds)
        Lp[r * LDP + c] = *hp;
      else
        *hp = Lp[r * LDP + c];
    }
  };
  // substitution of columns c0 .. c0 + 15 of every panel row (thread per row)
  auto subst16 = [&](int rest, int c0) {
    if (tid < rest) {
      double* lr = Lp + tid * LDP + c0;
      double v[16];
#pragma unroll
      for (int c = 0; c < 16; ++c) v[c] = lr[c];
#pragma unroll
      for (int c = 0; c < 16; ++c) {
        v[c] *= L11[(c0 + c) * LDP + CB];
#pragma unroll
        for (int c2 = c + 1; c2 < 16; ++c2) v[c2] = fma(-v[c], L11[(c0 + c) * LDP + c0 + c2], v[c2]);
      }
#pragma unroll
      for (int c = 0; c < 16; ++c) lr[c] = v[c];
    }
  };
  // the panel solve in two column halves: X1 by substitution, the second
  // half's right-hand side less X1 L[16..32)[0..16)^T on the fp64 MFMA, X2 by
  // substitution (16 values per thread: the broadcast reads pipeline)
  auto trsm = [&](int rest) {
    subst16(rest, 0);
    __syncthreads();
    for (int ti = wv; ti < rest / 16; ti += 16) {
      d4w acc = d4w{0, 0, 0, 0};
#pragma unroll
      for (int s4 = 0; s4 < 4; ++s4)
        acc = __builtin_amdgcn_mfma_f64_16x16x4f64(Lp[(16 * ti + fl) * LDP + 4 * s4 + kq],
                                                   L11[(4 * s4 + kq) * LDP + 16 + fl], acc, 0, 0, 0);
#pragma unroll
      for (int r = 0; r < 4; ++r) Lp[(16 * ti + kq + 4 * r) * LDP + 16 + fl] -= acc[r];
    }
    __syncthreads();
    subst16(rest, 16);
  };
  // A22 -= L21 L21^T on lower 16x16 tiles: the two tile columns of the next
  // panel (cols01) or the rest; UT tiles per wave at a time (their C reads
  // issued together: one L2 / MALL latency for UT read-modify-writes); tiles
  // past the end recompute the last tile and skip the store.  On the
  // approximate iterations (the Hessian is the bf16 pass's, ~2^-8 per value)
  // the products run on the f32 MFMA (32 cycles per 16x16x4 against ~64 for
  // fp64; C stays fp64): the trailing update is the MFMA-bound phase.  The
  // two forms' C/D maps differ: lane (kq, fl), register r holds row kq + 4 r
  // (fp64) or 4 kq + r (f32) of column fl, so C is read and written in the
  // map of the form in use.
  const bool lowp = phase == PHASE_F32 && DLSA_WN_F32;
  const int crow = lowp ? 4 * kq : kq, cstep = lowp ? 1 : 4;
  auto trail = [&](int jb, int m, bool cols01, int w0, int nw) {
    const int ntiles = cols01 ? 2 * m - 1 : (m - 2) * (m - 1) / 2;
    constexpr int UT = 4;  // 6 or 8 spill (25 / 57 VGPRs)
    for (int t0 = w0; t0 < ntiles; t0 += nw * UT) {
      int ti[UT], tj[UT];
      d4w c[UT];
#pragma unroll
      for (int u = 0; u < UT; ++u) {
        const int t = min(t0 + nw * u, ntiles - 1);
        if (cols01) {
          ti[u] = t < m ? t : t - m + 1;
          tj[u] = t < m ? 0 : 1;
        } else {
          tile_ij(t, ti[u], tj[u]);
          ti[u] += 2;
          tj[u] += 2;
        }
        const double* cp = H + (int64_t)(jb + CB + 16 * ti[u] + crow) * PP + jb + CB + 16 * tj[u] + fl;
#pragma unroll
        for (int r = 0; r < 4; ++r) c[u][r] = cp[r * cstep * PP];
      }
#pragma unroll
      for (int u = 0; u < UT; ++u) {
        d4w acc = d4w{0, 0, 0, 0};
        if (lowp) {
          f4w a32 = f4w{0, 0, 0, 0};
#pragma unroll
          for (int s = 0; s < CB / 4; ++s) {
            const float av = (float)Lp[(16 * ti[u] + fl) * LDP + 4 * s + kq];
            const float bv = (float)Lp[(16 * tj[u] + fl) * LDP + 4 * s + kq];
            a32 = __builtin_amdgcn_mfma_f32_16x16x4f32(av, bv, a32, 0, 0, 0);
          }
#pragma unroll
          for (int r = 0; r < 4; ++r) acc[r] = (double)a32[r];
        } else {
#pragma unroll
          for (int s = 0; s < CB / 4; ++s) {
            const double av = Lp[(16 * ti[u] + fl) * LDP + 4 * s + kq];
            const double bv = Lp[(16 * tj[u] + fl) * LDP + 4 * s + kq];
            acc = __builtin_amdgcn_mfma_f64_16x16x4f64(av, bv, acc, 0, 0, 0);
          }
        }
        if (t0 + nw * u < ntiles) {
          double* cp = H + (int64_t)(jb + CB + 16 * ti[u] + crow) * PP + jb + CB + 16 * tj[u] + fl;
#pragma unroll
          for (int r = 0; r < 4; ++r) cp[r * cstep * PP] = c[u][r] - acc[r];
        }
      }
    }
  };
  // the forward solve L z = g rides on the factorization: z_b of block b is
  // solved by one wave against the diagonal block while the panel below is
  // solved, and every later row takes the block's terms (z_J -= L_Jb z_b)
  // right after the panel, so no P-long substitution follows the factor
  auto zsolve = [&](int jb) {
    const int i = lane & 31;
    double zi = z[jb + i];
#pragma unroll
    for (int c = 0; c < CB; ++c) {
      if (i == c) zi *= L11[c * LDP + CB];
      const double zc = bcast_f64(zi, c);
      if (i > c) zi = fma(-L11[c * LDP + i], zc, zi);
    }
    if (lane < 32) z[jb + i] = zi;
  };
  for (int f = tid; f < PP; f += 1024) z[f] = g[f];
  if (wv == 0) factor_diag(0);
  __syncthreads();
  {
    WN_STAMP(t1);
    if (wid == 0) WN_ADD(0, t1 - t_f0);
  }
  if (!*flag) {
    for (int jb = 0; jb + CB < PP; jb += CB) {
      const int m = (PP - jb - CB) / 16;
      WN_STAMP(ta);
      panel_copy(jb, PP - jb - CB, true);
      __syncthreads();
      if (wv == 15) zsolve(jb);  // rows past 480 do not exist: wave 15 has no panel row
      trsm(PP - jb - CB);
      __syncthreads();
      WN_STAMP(tb);
      if (tid < PP - jb - CB) {
        double s = z[jb + CB + tid];
#pragma unroll
        for (int c = 0; c < CB; ++c) s = fma(-Lp[tid * LDP + c], z[jb + c], s);
        z[jb + CB + tid] = s;
      }
      trail(jb, m, true, wv, 16);
      panel_copy(jb, PP - jb - CB, false);  // L21 to H for the solves
      __syncthreads();
      WN_STAMP(tc);
      if (wv == 0)
        factor_diag(jb + CB);
      else
        trail(jb, m, false, wv - 1, 15);
      WN_STAMP(td);
      __syncthreads();
      WN_STAMP(te);
      if (wid == 0) {
        WN_ADD(1, tb - ta);
        WN_ADD(2, tc - tb);
        WN_ADD(3, td - tc);
        WN_ADD(4, te - td);
      }
      if (wid == 1) WN_ADD(5, td - tc);
      if (*flag) break;  // uniform
    }
  }
  if (*flag) {
    if (a.subsample) {
      level_fail();
      return;
    }
    if (tid == 0) {
      if (phase != PHASE_F64 && a.family == FAMILY_LOGISTIC) {
        // approximate Hessian lost definiteness: redo this point in fp64
        a.phase[k] = PHASE_F64;
        a.iters[k] = it + 1;
        a.stall[k] = 0;
        a.dm_prev[k] = 0.0;
        atomicAdd(&a.counters[PHASE_F64], 1);
      } else {
        a.status[k] = DLSA_STATUS_SINGULAR;
      }
    }
    return;
  }

  // 5a. the last diagonal block's share of the forward solve
  WN_STAMP(t_s0);
  if (wv == 0) zsolve(PP - CB);
  __syncthreads();
  WN_STAMP(t_s1);
  // 5b. backward solve L^T d = z (d overwrites z): u_c = sum_{i >= jb + CB}
  // L[i][jb + c] d_i in fixed order (4 rows in flight per thread), then
  // L11^T d_b = z_b - u by one wave (lane c = unknown c)
  for (int jb = PP - CB; jb >= 0; jb -= CB) {
    const int c = tid & 31;
    {
      const int grp = tid >> 5;
      double s = 0.0;
      int i = jb + CB + grp;
      for (; i + 96 < PP; i += 128) {
        const double h0 = H[(int64_t)i * PP + jb + c], h1 = H[(int64_t)(i + 32) * PP + jb + c];
        const double h2 = H[(int64_t)(i + 64) * PP + jb + c], h3 = H[(int64_t)(i + 96) * PP + jb + c];
        s = fma(h0, z[i], s);
        s = fma(h1, z[i + 32], s);
        s = fma(h2, z[i + 64], s);
        s = fma(h3, z[i + 96], s);
      }
      for (; i < PP; i += 32) s = fma(H[(int64_t)i * PP + jb + c], z[i], s);
      L11[grp * LDP + c] = s;
    }
    __syncthreads();
    if (wv == 0) {
      double lcol[CB];  // column c of L11: L[r][c] (zero above the diagonal)
#pragma unroll
      for (int r = 0; r < CB; ++r) lcol[r] = H[(int64_t)(jb + r) * PP + jb + c];
      const double rc = 1.0 / H[(int64_t)(jb + c) * PP + jb + c];
      double u = 0.0;
#pragma unroll
      for (int q = 0; q < 32; ++q) u += L11[q * LDP + c];
      double v = z[jb + c] - u;
#pragma unroll
      for (int r = CB - 1; r >= 0; --r) {
        if (c == r) v *= rc;
        const double dr = bcast_f64(v, r);
        if (c < r) v = fma(-lcol[r], dr, v);
      }
      z[jb + c] = v;
    }
    __syncthreads();
  }
  {
    WN_STAMP(t_s2);
    if (wid == 0) {
      WN_ADD(6, t_s1 - t_s0);
      WN_ADD(7, t_s2 - t_s1);
    }
  }
#else
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
    // UT tiles per wave at a time: their C reads are issued together, so one
    // L2 / MALL latency covers UT read-modify-writes (the update is latency-
    // bound: one CU per partition); tiles past the end recompute the last
    // tile and skip the store
    const int m = rest / 16;
    const int ntiles = m * (m + 1) / 2;
    const int wv = __builtin_amdgcn_readfirstlane(wid);
    constexpr int UT = 4;
    for (int t0 = wv; t0 < ntiles; t0 += 16 * UT) {
      int ti[UT], tj[UT];
      d4w c[UT];
#pragma unroll
      for (int u = 0; u < UT; ++u) {
        tile_ij(min(t0 + 16 * u, ntiles - 1), ti[u], tj[u]);
        const double* cp = H + (int64_t)(jb + CB + 16 * ti[u] + kq) * PP + jb + CB + 16 * tj[u] + fl;
#pragma unroll
        for (int r = 0; r < 4; ++r) c[u][r] = cp[4 * r * PP];
      }
#pragma unroll
      for (int u = 0; u < UT; ++u) {
        d4w acc = d4w{0, 0, 0, 0};
#pragma unroll
        for (int s = 0; s < CB / 4; ++s) {
          const double av = Lp[(16 * ti[u] + fl) * LDP + 4 * s + kq];
          const double bv = Lp[(16 * tj[u] + fl) * LDP + 4 * s + kq];
          acc = __builtin_amdgcn_mfma_f64_16x16x4f64(av, bv, acc, 0, 0, 0);
        }
        if (t0 + 16 * u < ntiles) {
          double* cp = H + (int64_t)(jb + CB + 16 * ti[u] + kq) * PP + jb + CB + 16 * tj[u] + fl;
#pragma unroll
          for (int r = 0; r < 4; ++r) cp[4 * r * PP] = c[u][r] - acc[r];
        }
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
      if (phase != PHASE_F64 && a.family == FAMILY_LOGISTIC) {
        // approximate Hessian lost definiteness: redo this point in fp64
        a.phase[k] = PHASE_F64;
        a.iters[k] = it + 1;
        a.stall[k] = 0;
        a.dm_prev[k] = 0.0;
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
#endif  // DLSA_WN_LOOKAHEAD

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
  if (ph != PHASE_F64) {
    if (dm <= a.switch_tol * (1.0 + tm)) {
      ph = PHASE_F64;
    } else {  // stall escalation (dlsa_internal.hpp): bf16 -> fp64 on this path
      ph = approx_next_phase(a, k, ph, dm, ll, llp);
    }
  } else if (dm <= a.tol * (1.0 + tm)) {
    a.status[k] = DLSA_STATUS_OK;
    a.phase[k] = PHASE_DONE;
    return;
  }
  a.phase[k] = ph;
  atomicAdd(&a.counters[ph], 1);
}

#ifdef DLSA_WN_PROF
extern "C" int dlsa_wn_prof_read(unsigned long long* out) {
  if (hipDeviceSynchronize() != hipSuccess) return -1;
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_wn_prof), 16 * 8) != hipSuccess) return -1;
  unsigned long long z[16] = {0};
  return hipMemcpyToSymbol(HIP_SYMBOL(g_wn_prof), z, 16 * 8) == hipSuccess ? 0 : -1;
}
#endif

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

// exact (fp64) Gram pass of the PHASE_F64 partitions
hipError_t launch_wide_gram(const WideArgs& a, bool standardize, hipStream_t s) {
  if (a.n_gchunks <= 0) return hipSuccess;
  const int TB = a.NB * (a.NB + 1) / 2;
  const int grid = ((a.n_gchunks + 7) / 8) * 8 * TB;
  if (standardize)
    hipLaunchKernelGGL(wide_gram_kernel<true>, dim3(grid), dim3(256), 0, s, a);
  else
    hipLaunchKernelGGL(wide_gram_kernel<false>, dim3(grid), dim3(256), 0, s, a);
  return hipGetLastError();
}

hipError_t launch_wide_assemble(const WideArgs& a, const int32_t* gcb, double* Hfull, int K,
                                hipStream_t s) {
  const int TB = a.NB * (a.NB + 1) / 2;
  hipLaunchKernelGGL(wide_assemble_kernel, dim3(TB * 16, K), dim3(256), 0, s, a, gcb, Hfull);
  return hipGetLastError();
}

hipError_t launch_wide_newton(const SolveArgs& sa, const WideArgs& wa, const int32_t* rcb,
                              const int32_t* gcb, double* Hfull, int K, hipStream_t s) {
  {
    hipError_t e = ensure_max_lds((const void*)wide_newton_kernel, 160 * 1024);
    if (e != hipSuccess) return e;
  }
  hipLaunchKernelGGL(wide_newton_kernel, dim3(K), dim3(1024), wide_newton_lds_bytes(wa.NB), s,
                     sa, wa, rcb, gcb, Hfull);
  return hipGetLastError();
}

}  // namespace dlsa
