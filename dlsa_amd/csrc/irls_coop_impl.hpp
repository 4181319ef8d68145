// Cooperative fused IRLS pass (gfx950 / CDNA4) -- kernel templates, included
// by the irls_coop*.hip translation units (one per group of NT values, so the
// instantiations compile in parallel).
//
// Cooperative fused IRLS pass: one 4-wave workgroup streams
// a chunk of rows of one partition through a shared LDS-DMA ring.
//
// Replaces, per Newton iteration, the per-partition work of the reference map
// stage (sklearn newton-cg Hessian-vector passes, predict_proba and
// Sig_inv = X^T diag(p(1-p)) X, dlsa/models.py:110-131) with ONE pass over X.
//
// Per 32-row block:
//   B1  barrier: the block's DMA pieces (issued by all 4 waves, each waiting
//       on its own counted vmcnt) have landed; the slot of block b-1 is free
//       and receives block b+S-1 (S-1 blocks always in flight).
//   B   row phase: rows split over the waves, 8 lanes per row.  eta = x.theta
//       (fp64, 8-lane DPP reduction), mu, w = mu(1-mu), r = y - mu, the
//       gradient x*r and the log-likelihood are computed ONCE per row; w and r
//       are published in LDS.
//   B2  barrier.
//   C   tile phase: the lower-triangle 16x16 tiles of X^T W X are split over
//       the waves (contiguous tile ranges, so each wave touches few column
//       tiles).  PREC_BF16: one v_mfma_f32_16x16x32_bf16 per tile per block;
//       PREC_F32 / PREC_F64: 8 k-steps of v_mfma_*_16x16x4 (fp32 / fp64).
// The bf16 / fp32 Hessians only steer Newton (the fp64 gradient fixes the
// fixed point); the returned Sig_inv always comes from a PREC_F64 pass.
#include <stdlib.h>

#include <type_traits>
#include <utility>

#pragma once

#include "dlsa_internal.hpp"

namespace dlsa {

typedef double d4 __attribute__((ext_vector_type(4)));
typedef float f4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x2c __attribute__((ext_vector_type(2)));
typedef float f2c __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(3))) void lds_void_t;
typedef const __attribute__((address_space(1))) void gbl_void_t;

namespace {

constexpr int RB = kCoopRows;   // rows per block

// Profiling-only ablations (tools/build_variants.sh builds them into separate
// .so files; the product build has DLSA_ABLATE = 0): 1 no tile phase, 2 no
// transcendentals in the row phase, 3 stream only, 4 no row phase.
#ifndef DLSA_ABLATE
#define DLSA_ABLATE 0
#endif
// bf16 operands (round 2): ONE image Z = bf16(sqrt(w) x), H~ = Z^T Z (positive
// semi-definite by construction, as in the wide fused pass), instead of the
// two images x and w x -- half the image stores and LDS: 9.87 -> 9.37 ms per
// config-2 launch (profiles/r02ac_zimage_ab.txt)

template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  static_assert(N >= 0 && N < 64, "vmcnt is 6 bits on gfx950");
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
template <int N>
__device__ __forceinline__ void wait_vmcnt_le(int n) {
  if constexpr (N <= 0) {
    wait_vmcnt<0>();
  } else {
    if (n >= N)
      wait_vmcnt<N>();
    else
      wait_vmcnt_le<N - 1>(n);
  }
}

// Workgroup barrier for the block loop: this wave's LDS reads/writes are
// complete (lgkmcnt(0)), then s_barrier.  Unlike __syncthreads() it carries no
// memory fence, whose lowering drains vmcnt to 0 -- that would wait for the
// LDS-DMA of the blocks still streaming in, i.e. empty the ring at every
// barrier.  The "memory" clobber keeps the compiler from moving LDS accesses
// across it; the DMA'd slot of a block is waited for by each wave's counted
// vmcnt before the first barrier that publishes it.
__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

// Buffer resource with every word wave-uniform (readfirstlane): the LDS-DMA
// loads then take it in SGPRs instead of a waterfall loop per load.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t uniform_rsrc(uintptr_t base, uintptr_t bytes) {
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)base);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)((uint64_t)base >> 32));
  const uint32_t nr = __builtin_amdgcn_readfirstlane(
      (uint32_t)(bytes < 0x7FFFFFF0u ? bytes : 0x7FFFFFF0u));
  return __builtin_amdgcn_make_buffer_rsrc((void*)(((uint64_t)hi << 32) | lo), (short)0, (int)nr,
                                           0x00020000);
}

template <int CTRL>
__device__ __forceinline__ double dpp_f64(double v) {
  const int lo = __builtin_amdgcn_mov_dpp(__double2loint(v), CTRL, 0xF, 0xF, false);
  const int hi = __builtin_amdgcn_mov_dpp(__double2hiint(v), CTRL, 0xF, 0xF, false);
  return __hiloint2double(hi, lo);
}
// Lane l and lane l ^ 16 (permlane16_swap), l and l ^ 32 (permlane32_swap):
// both operands are v, so the swapped pair (x, y) holds the two halves and
// x + y is the same sum, bitwise, in both lanes of the pair.
__device__ __forceinline__ double xor16_sum(double v) {
  const unsigned lo = __double2loint(v), hi = __double2hiint(v);
  const auto a = __builtin_amdgcn_permlane16_swap(lo, lo, false, false);
  const auto b = __builtin_amdgcn_permlane16_swap(hi, hi, false, false);
  return __hiloint2double(b[0], a[0]) + __hiloint2double(b[1], a[1]);
}
__device__ __forceinline__ double xor32_sum(double v) {
  const unsigned lo = __double2loint(v), hi = __double2hiint(v);
  const auto a = __builtin_amdgcn_permlane32_swap(lo, lo, false, false);
  const auto b = __builtin_amdgcn_permlane32_swap(hi, hi, false, false);
  return __hiloint2double(b[0], a[0]) + __hiloint2double(b[1], a[1]);
}

// Sum over the lanes l, l ^ RPW, l ^ 2 RPW, ... (the LPR feature groups of one
// row in the row phase) without LDS: row_ror 8 (and 4) inside a 16-lane DPP
// row, then the cross-row swaps.  Every lane of the row ends with the
// bitwise-identical total (each step adds a commutative pair).
template <int RPW>
__device__ __forceinline__ double red_row(double v) {
  static_assert(RPW == 8 || RPW == 4, "4 or 8 rows per wave");
  v += dpp_f64<0x128>(v);                         // row_ror 8: l ^ 8
  if constexpr (RPW == 4) v += dpp_f64<0x124>(v);  // row_ror 4: l + 4, l + 12
  v = xor16_sum(v);
  v = xor32_sum(v);
  return v;
}

constexpr int tile_I(int t) {
  int I = 0;
  while ((I + 1) * (I + 2) / 2 <= t) ++I;
  return I;
}
constexpr int tile_J(int t) { return t - tile_I(t) * (tile_I(t) + 1) / 2; }

template <int NT, int W_>
struct CG {
  static constexpr int W = W_;                // waves per workgroup (4 or 8)
  static constexpr int RPW = RB / W;          // rows per wave in the row phase
  static constexpr int LPR = 64 / RPW;        // lanes per row in the row phase (8 or 16)
  static constexpr int PMAX = 16 * NT;
  static constexpr int T = NT * (NT + 1) / 2;
  static constexpr int TPW = (T + W - 1) / W;  // tiles per wave (contiguous ranges)
  static constexpr int M = PMAX / LPR;         // features per lane in the row phase
  static constexpr int PAD = 16;
  static constexpr int OBS = RB + 16;           // bf16 image: elements per feature row; 96 B
                                               // (24 dwords) makes the ds_read_b128 operand
                                               // reads (lane groups of MI355X_MICROARCH.md
                                               // "LDS") conflict-free -- 80 B is 2-way
  static constexpr int MAX_PIECES = (RB * PMAX * 8 + 16 + 1023) / 1024;
  static constexpr int MAX_D = (MAX_PIECES + W - 1) / W;  // DMA pieces per wave per block
  // tiles of wave `wid`: t in [wid*TPW, min(T, (wid+1)*TPW))
  static constexpr unsigned col_mask(int wid) {
    unsigned m = 0;
    for (int t = wid * TPW; t < T && t < (wid + 1) * TPW; ++t)
      m |= (1u << tile_I(t)) | (1u << tile_J(t));
    return m;
  }
  static constexpr unsigned row_mask(int wid) {
    unsigned m = 0;
    for (int t = wid * TPW; t < T && t < (wid + 1) * TPW; ++t) m |= 1u << tile_I(t);
    return m;
  }
};

template <typename F, int... Is>
__device__ __forceinline__ void static_for_impl(F&& f, std::integer_sequence<int, Is...>) {
  (f(std::integral_constant<int, Is>{}), ...);
}
template <int N, typename F>
__device__ __forceinline__ void static_for(F&& f) {
  static_for_impl(f, std::make_integer_sequence<int, N>{});
}

__host__ __device__ __forceinline__ int npieces_for(int p) { return (RB * p * 8 + 16 + 1023) / 1024; }

}  // namespace

// Waves per workgroup: 4 for P <= 128 (8 lanes per row in the row phase),
// 8 above (16 lanes per row keeps the per-lane feature count <= 12).
constexpr int coop_waves(int NT) { return NT > 8 ? 8 : 4; }

// A slot holds exactly the block's pieces: a wave's surplus issues (the piece
// count is rounded up to the wave count so that every wave waits on the same
// vmcnt) re-load the last piece onto itself.
inline int coop_slot_bytes_impl(int NT, int p) {
  return 16 + npieces_for(p) * 1024 + 16 * NT * 8 + RB * 8;
}

// LDS beyond the ring: w, r of the block [2][RB] fp64, center / 1/scale
// [2][PMAX] fp64, and the bf16 MFMA operand image of the block z = sqrt(w) x,
// [PMAX][RB + 16] bf16 (feature-major, so one lane's 8 consecutive k are one
// 16-byte read).
inline int coop_extra_bytes_impl(int NT) {
  return (2 * RB + 2 * 16 * NT) * 8 + 16 * NT * (RB + 16) * 2;
}

// Tile phase of wave WID for one 32-row block.
template <int NT, int W, int PREC, bool STD, int WID, typename Acc>
__device__ __forceinline__ void tile_phase(Acc (&acc)[(CG<NT, W>::TPW)], const double* xs,
                                           const double* wr, int p, int ic, int lane,
                                           const double* stdv, const __bf16* obx) {
  using G = CG<NT, W>;
  constexpr unsigned CM = G::col_mask(WID);
  constexpr unsigned RM = G::row_mask(WID);
  const int fl = lane & 15, q = lane >> 4;
  const bool icpt_lane = ic && fl == 0;
  const double* xq = xs + q * p + (fl - ic);  // row q of the block, this lane's feature
  static_assert(PREC != PREC_BF16, "bf16 tiles are issued by the kernel body");
  {
    // 8 k-steps of 4 rows: k-step s uses block rows 4s + q (k = q)
#pragma unroll
    for (int s = 0; s < 8; ++s) {
      const double ws = wr[4 * s + q];
      double xv[NT], av[NT];
      static_for<NT>([&](auto cI) {
        constexpr int c = decltype(cI)::value;
        if constexpr ((CM >> c) & 1u) {
          double v = xq[4 * s * p + 16 * c];
          if constexpr (STD) v = (v - stdv[16 * c + fl]) * stdv[G::PMAX + 16 * c + fl];
          if (c == 0 && icpt_lane) v = 1.0;
          xv[c] = v;
          if constexpr ((RM >> c) & 1u) av[c] = v * ws;
        }
      });
      static_for<G::TPW>([&](auto iI) {
        constexpr int i = decltype(iI)::value;
        constexpr int t = WID * G::TPW + i;
        if constexpr (t < G::T) {
          constexpr int I = tile_I(t), J = tile_J(t);
          if constexpr (PREC == PREC_F64)
            acc[i] = __builtin_amdgcn_mfma_f64_16x16x4f64(av[I], xv[J], acc[i], 0, 0, 0);
          else
            acc[i] = __builtin_amdgcn_mfma_f32_16x16x4f32((float)av[I], (float)xv[J], acc[i], 0,
                                                          0, 0);
        }
      });
    }
  }
}

template <int NT, int W, int PREC, bool STD, int WID, typename Acc>
__device__ __forceinline__ void store_tiles(Acc (&acc)[(CG<NT, W>::TPW)], double* sH, int lane) {
  using G = CG<NT, W>;
  const int fl = lane & 15, q = lane >> 4;
  static_for<G::TPW>([&](auto iI) {
    constexpr int i = decltype(iI)::value;
    constexpr int t = WID * G::TPW + i;
    if constexpr (t < G::T) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        // f64 16x16x4 C/D map: row = (l>>4) + 4*reg; f32 16x16 maps: 4*(l>>4) + reg
        const int row = (PREC == PREC_F64) ? (q + 4 * r) : (4 * q + r);
        sH[t * 256 + row * 16 + fl] = (double)acc[i][r];
      }
    }
  });
}

// Profiling-only A/B (tools/build_variants.sh cmabl; product 0): the CM & 1
// pass skips its per-value max |x| update (the record reads 0).
#ifndef DLSA_CM_ABLATE
#define DLSA_CM_ABLATE 0
#endif
// CM (bits): also record the chunk's per-feature max |x| into a.colmax (1:
// the fit's first full-data bf16 pass) and max |z| (z = sqrt(w) x, the fp32
// value of the bf16 image) into a.zcolmax (2: the bf16 passes of partitions
// near convergence); the Ozaki exact pass takes its digit scales from the
// last records (irls_oz_impl.hpp)
template <int NT, int W, int PREC, bool STD, int FAM, int CM = 0>
__global__ __launch_bounds__(64 * W, (W == 8 || NT < 8) ? 2 : 1)
void irls_coop_kernel(const PassArgs a) {
  using G = CG<NT, W>;
  using Acc = typename std::conditional<PREC == PREC_F64, d4, f4>::type;
  constexpr int RPW = G::RPW, LPR = G::LPR;
  constexpr int M = G::M;
  constexpr int MAXW = 4 * (G::MAX_D + 1);  // nslot <= 6
  extern __shared__ __attribute__((aligned(16))) char smem[];

  const int chunk = blockIdx.x;
  const int part = __builtin_amdgcn_readfirstlane(a.chunk_part[chunk]);
  if (a.phase[part] != a.want_phase) return;  // workgroup-uniform

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int p = a.p, P = a.P, ic = a.intercept;
  const int64_t row0 =
      ((int64_t)__builtin_amdgcn_readfirstlane((int)(a.chunk_row0[chunk] >> 32)) << 32) |
      (uint32_t)__builtin_amdgcn_readfirstlane((int)a.chunk_row0[chunk]);
  const int nrows = __builtin_amdgcn_readfirstlane(a.chunk_rows[chunk]);
  const int nb = (nrows + RB - 1) / RB;
  const int nslot = a.nslot;
  const int slot_bytes = a.slot_bytes;
  const int npieces = npieces_for(p);
  const int d = (npieces + W - 1) / W;
  const int slot_x = G::PAD + npieces * 1024 + G::PMAX * 8;  // y follows
  double* wr = (double*)(smem + nslot * slot_bytes);       // [2][RB]: w, r of the block
  double* stdv = wr + 2 * RB;  // [2][PMAX]: center, 1/scale by feature (STD only)
  __bf16* obx = (__bf16*)(stdv + 2 * G::PMAX);  // [2][PMAX][OBS] bf16 operands (PREC_BF16)

  // ---- row-phase constants: lane = (feature group sl, row lane % RPW);
  // lane handles features f = sl + LPR m of its row.  Row-major ring reads of
  // one instruction cover RPW rows x LPR consecutive doubles per half-wave
  // (conflict-free at p = 100), and one feature's RPW rows are written to the
  // bf16 image by RPW consecutive lanes.
  const int sl = lane / RPW;
  const int rB = wid * RPW + lane % RPW;  // block row of this lane in the row phase
  double beta[M], gacc[M];
#pragma unroll
  for (int m = 0; m < M; ++m) {
    const int f = sl + LPR * m;
    beta[m] = (f < P) ? a.theta[(int64_t)part * P + f] : 0.0;
    gacc[m] = 0.0;
  }
  // re-define beta by an opaque instruction so its loads are waited for here,
  // once: otherwise the compiler's loop-carried wait for them sits inside the
  // block loop as vmcnt(1) and drains the ring
#pragma unroll
  for (int m = 0; m < M; ++m) asm volatile("" : "+v"(beta[m]));
  double llacc = 0.0;
  // CM: running max of |x| per feature, kept as the high dword of |x| (what
  // the digit exponents read: ozk::xbound sets the low dword to all ones) --
  // 32-bit integer max instead of a v_max_f64 per value, half the registers.
  // No row mask: the rows of a chunk's last block past its end are the next
  // chunk's rows (or the range check's zeros), so the recorded max is an upper
  // bound over the chunk's rows, which is all the digit exponents need (a
  // looser bound only moves the digits down a bit).
  uint32_t cmx[(CM & 1) ? M : 1];
  float zmx[(CM & 2) ? M : 1];  // running max |z| (fp32 image values; rows past the end have w = 0)
#pragma unroll
  for (int m = 0; m < (CM ? M : 1); ++m) {
    if constexpr (CM & 1) cmx[m] = 0u;
    if constexpr (CM & 2) zmx[m] = 0.0f;
  }
  int tI[G::TPW], tJ[G::TPW];  // this wave's tiles (bf16 path)
#pragma unroll
  for (int i = 0; i < G::TPW; ++i) {
    const int t = wid * G::TPW + i;
    int I = 0;
    while ((I + 1) * (I + 2) / 2 <= t) ++I;
    tI[i] = __builtin_amdgcn_readfirstlane(I);
    tJ[i] = __builtin_amdgcn_readfirstlane(t - I * (I + 1) / 2);
  }
  Acc acc[G::TPW];
#pragma unroll
  for (int i = 0; i < G::TPW; ++i) acc[i] = Acc{0, 0, 0, 0};

  // zero the ring once: pads/tails and never-DMA'd bytes must be finite
  for (int o = tid * 16; o < nslot * slot_bytes; o += 64 * W * 16)
    *(uint4*)(smem + o) = make_uint4(0, 0, 0, 0);
  if constexpr (STD) {
    for (int f = tid; f < G::PMAX; f += 64 * W) {
      const int j = f - ic;
      const bool in = j >= 0 && j < p;
      stdv[f] = in ? a.center[j] : 0.0;
      stdv[G::PMAX + f] = in ? 1.0 / a.scale[j] : 1.0;
    }
  }
  __syncthreads();

  // Buffer resources over this chunk's rows (bounds-checked raw buffers: a
  // tail piece past the end of X reads zeros instead of faulting), so a DMA
  // piece is one buffer_load ... lds with a scalar offset -- no per-lane
  // 64-bit address arithmetic.
  const uintptr_t xcb = (uintptr_t)(a.X + row0 * p) & ~(uintptr_t)15;
  const uintptr_t xend = a.x_last16 + 16;
  const __amdgpu_buffer_rsrc_t xr_rsrc = uniform_rsrc(xcb, xend - xcb);
  const uintptr_t ycb = (uintptr_t)(a.y + row0);
  const __amdgpu_buffer_rsrc_t yr_rsrc = uniform_rsrc(ycb, a.y_last4 + 4 - ycb);
  const int vx = lane * 16, vy = lane * 4;
  auto issue = [&](int blk) {
    const int bb = blk < nb ? blk : nb - 1;  // tail: harmless re-fetch, fixed counts
    char* sbase = smem + (blk % nslot) * slot_bytes;
    const uintptr_t start = (uintptr_t)(a.X + (row0 + (int64_t)bb * RB) * p);
    const int so = __builtin_amdgcn_readfirstlane((int)((start & ~(uintptr_t)15) - xcb));
    for (int i = 0; i < d; ++i) {
      int j = wid + W * i;
      const int jj = j < npieces ? j : npieces - 1;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(
          xr_rsrc, (lds_void_t*)(sbase + G::PAD + jj * 1024), 16, vx, so + jj * 1024, 0,
          DLSA_X_DMA_AUX);
    }
    __builtin_amdgcn_raw_ptr_buffer_load_lds(yr_rsrc, (lds_void_t*)(sbase + slot_x), 4, vy,
                                             bb * RB * 8, 0, 0);
  };

  for (int b = 0; b < nslot - 1; ++b) issue(b);
  const int keep = (nslot - 2) * (d + 1);

  for (int b = 0; b < nb; ++b) {
    wait_vmcnt_le<MAXW>(keep);  // this wave's pieces of block b landed
    lds_barrier();              // B1: everyone's pieces landed, block b-1 fully consumed
    issue(b + nslot - 1);

    const char* slot = smem + (b % nslot) * slot_bytes;
    const uintptr_t start = (uintptr_t)(a.X + (row0 + (int64_t)b * RB) * p);
    const double* xs = (const double*)(slot + G::PAD + (start & 15));
    const double* ys = (const double*)(slot + slot_x);
    const int rows_left = nrows - b * RB;

    // ---- B: row phase ------------------------------------------------------
    if constexpr (DLSA_ABLATE != 3 && DLSA_ABLATE != 4) {
      const bool valid = rB < rows_left;
      const double* xr = xs + rB * p + (sl - ic);
      double xv[M];
      double e0 = 0.0, e1 = 0.0;  // two FMA chains: half the latency of the dot product
#pragma unroll
      for (int m = 0; m < M; ++m) {
        double v = xr[LPR * m];
        if constexpr (STD) v = (v - stdv[sl + LPR * m]) * stdv[G::PMAX + sl + LPR * m];
        if (m == 0 && ic && sl == 0) v = 1.0;
        xv[m] = v;
        if constexpr ((CM & 1) && !DLSA_CM_ABLATE)
          cmx[m] = max(cmx[m], (uint32_t)__double2hiint(v) & 0x7FFFFFFFu);
        if (m & 1)
          e1 = fma(v, beta[m], e1);
        else
          e0 = fma(v, beta[m], e0);
      }
      const double e = red_row<RPW>(e0 + e1);  // bitwise-identical in all lanes of the row
      const double yv = ys[rB];
      double w, r;
      if constexpr (FAM == FAMILY_LOGISTIC && DLSA_ABLATE == 2) {
        w = 0.25;
        r = yv - 0.5 - 0.25 * e;
        if (valid && sl == 0) llacc += e;
      } else if constexpr (FAM == FAMILY_LOGISTIC) {
        const double ea = exp(-fabs(e));
        const double inv = 1.0 / (1.0 + ea);
        const double mu = e >= 0.0 ? inv : ea * inv;
        w = ea * inv * inv;  // mu (1 - mu), cancellation free
        r = yv - mu;
        if (valid && sl == 0) {
          // exact fp64 in the fp64 pass (its value is returned); fp32 log in
          // the approximate passes, where it only drives step halving
          const double sp = (PREC == PREC_F64) ? log1p(ea) : (double)__logf(1.0f + (float)ea);
          llacc += yv * e - (fmax(e, 0.0) + sp);
        }
      } else {  // gaussian (OLS): mu = eta, w = 1, ll = -rss/2
        w = 1.0;
        r = yv - e;
        if (valid && sl == 0) llacc -= 0.5 * r * r;
      }
      if (!valid) {
        w = 0.0;
        r = 0.0;
      }
#pragma unroll
      for (int m = 0; m < M; ++m) gacc[m] = fma(xv[m], r, gacc[m]);
      if (sl == 0) {
        wr[rB] = w;
        wr[RB + rB] = r;
      }
      if constexpr (PREC == PREC_BF16) {
        // stage the bf16 MFMA operand z = sqrt(w) x once per row; one
        // v_cvt_pk_bf16_f32 converts two of the lane's features
        const float swf = __builtin_sqrtf((float)w);
#pragma unroll
        for (int m = 0; m < M; m += 2) {
          float z0 = (float)xv[m];
          float z1 = m + 1 < M ? (float)xv[m + 1] : 0.0f;
          // opaque: otherwise (bf16)(float)x folds into a direct f64 -> bf16
          // conversion with round-to-odd fix-ups
          asm volatile("" : "+v"(z0), "+v"(z1));
          const f2c pr = {z0 * swf, z1 * swf};
          if constexpr ((CM & 2) != 0) {
            zmx[m] = __builtin_fmaxf(zmx[m], __builtin_fabsf(pr[0]));
            if (m + 1 < M) zmx[m + 1] = __builtin_fmaxf(zmx[m + 1], __builtin_fabsf(pr[1]));
          }
          const bf16x2c pk = __builtin_convertvector(pr, bf16x2c);
          obx[(sl + LPR * m) * G::OBS + rB] = pk[0];
          if (m + 1 < M) obx[(sl + LPR * (m + 1)) * G::OBS + rB] = pk[1];
        }

      }
    }
    lds_barrier();  // B2: w, r (and the bf16 operand images) of all 32 rows visible

    // ---- C: tile phase -----------------------------------------------------
    if constexpr (DLSA_ABLATE != 1 && DLSA_ABLATE != 3) {
      if constexpr (PREC == PREC_BF16) {
        // one code path for every wave: the wave's tile indices are
        // wave-uniform registers (no per-wave copies of the loop body, whose
        // merge would copy the accumulators every block)
        const int fl = lane & 15, q = lane >> 4;
#pragma unroll
        for (int i = 0; i < G::TPW; ++i) {
          if (wid * G::TPW + i < G::T) {  // wave-uniform
            const bf16x8 Av = *(const bf16x8*)(obx + (16 * tI[i] + fl) * G::OBS + 8 * q);
            const bf16x8 Bv = *(const bf16x8*)(obx + (16 * tJ[i] + fl) * G::OBS + 8 * q);
            acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(Av, Bv, acc[i], 0, 0, 0);
          }
        }
      } else {
        static_for<W>([&](auto wI) {
          constexpr int WID = decltype(wI)::value;
          if (wid == WID) tile_phase<NT, W, PREC, STD, WID>(acc, xs, wr, p, ic, lane, stdv, obx);
        });
      }
    }
  }
  wait_vmcnt<0>();  // drain the tail re-fetches
  __syncthreads();

  // ---- epilogue ------------------------------------------------------------
  double* sH = a.slab_H + (int64_t)chunk * G::T * 256;
  static_for<W>([&](auto wI) {
    constexpr int WID = decltype(wI)::value;
    if (wid == WID) store_tiles<NT, W, PREC, STD, WID>(acc, sH, lane);
  });
  // gradient: sum the row lanes of each feature group (xor 1 .. RPW/2), then the waves
  double* red = (double*)smem;  // ring is no longer needed: [W][PMAX] + [W]
#pragma unroll
  for (int m = 0; m < M; ++m) {
    double v = gacc[m];
#pragma unroll
    for (int o = 1; o < RPW; o <<= 1) v += __shfl_xor(v, o);
    if (lane % RPW == 0) red[wid * G::PMAX + sl + LPR * m] = v;
  }
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) llacc += __shfl_xor(llacc, o);
  if (lane == 0) red[W * G::PMAX + wid] = llacc;
  __syncthreads();
  for (int f = tid; f < G::PMAX; f += 64 * W) {
    double s = 0.0;
#pragma unroll
    for (int w = 0; w < W; ++w) s += red[w * G::PMAX + f];
    a.slab_g[(int64_t)chunk * G::PMAX + f] = s;
  }
  if (tid == 0) {
    double s = 0.0;
#pragma unroll
    for (int w = 0; w < W; ++w) s += red[W * G::PMAX + w];
    a.slab_ll[chunk] = s;
  }
  if constexpr (CM) {
    __syncthreads();  // red is reused
    uint32_t* cred = (uint32_t*)smem;  // [2][W][PMAX]: max |x| high dwords, max |z| fp32 bits
#pragma unroll
    for (int m = 0; m < M; ++m) {
      uint32_t v = 0, u = 0;
      if constexpr (CM & 1) v = cmx[m];
      if constexpr (CM & 2) u = __float_as_uint(zmx[m]) & 0x7FFFFFFFu;  // ordered as integers
#pragma unroll
      for (int o = 1; o < RPW; o <<= 1) {
        if constexpr (CM & 1) v = max(v, (uint32_t)__shfl_xor((int)v, o));
        if constexpr (CM & 2) u = max(u, (uint32_t)__shfl_xor((int)u, o));
      }
      if (lane % RPW == 0) {
        cred[wid * G::PMAX + sl + LPR * m] = v;
        cred[(W + wid) * G::PMAX + sl + LPR * m] = u;
      }
    }
    __syncthreads();
    // a pass enqueued before the host read the near-switch count records only
    // if that count is > 0 (the running max costs one fp32 max per value)
    const bool zon = (CM & 2) && (a.zrec_gate == nullptr || a.zrec_gate[0] > 0);
    for (int f = tid; f < G::PMAX; f += 64 * W) {
      uint32_t v = 0, u = 0;
#pragma unroll
      for (int w = 0; w < W; ++w) {
        v = max(v, cred[w * G::PMAX + f]);
        u = max(u, cred[(W + w) * G::PMAX + f]);
      }
      if constexpr (CM & 1) a.colmax[(int64_t)chunk * G::PMAX + f] = v;
      if constexpr (CM & 2)
        if (zon) a.zcolmax[(int64_t)chunk * G::PMAX + f] = u;
    }
  }
}

template <int NT, int W, int PREC, bool STD, int FAM, int CM = 0>
static hipError_t launch_c(const PassArgs& a, int n_chunks, hipStream_t s) {
  auto kern = irls_coop_kernel<NT, W, PREC, STD, FAM, CM>;
  const size_t lds =
      (size_t)a.nslot * a.slot_bytes + coop_extra_bytes_impl(NT);
  hipError_t e = ensure_max_lds((const void*)kern, 160 * 1024);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(kern, dim3(n_chunks), dim3(64 * W), lds, s, a);
  return hipGetLastError();
}

template <int NT, int W>
static hipError_t launch_coop_ntw(const PassArgs& a, int prec, bool std_, int family,
                                  int n_chunks, hipStream_t s) {
  if (family == FAMILY_GAUSSIAN) {
    if (prec != PREC_F64) return hipErrorInvalidValue;
    return std_ ? launch_c<NT, W, PREC_F64, true, FAMILY_GAUSSIAN>(a, n_chunks, s)
                : launch_c<NT, W, PREC_F64, false, FAMILY_GAUSSIAN>(a, n_chunks, s);
  }
  switch (prec) {
    case PREC_BF16:
      if constexpr (NT <= kOzMaxNT) {
        const int cm = (a.colmax ? 1 : 0) | (a.zcolmax ? 2 : 0);
        if (cm == 1)
          return std_ ? launch_c<NT, W, PREC_BF16, true, FAMILY_LOGISTIC, 1>(a, n_chunks, s)
                      : launch_c<NT, W, PREC_BF16, false, FAMILY_LOGISTIC, 1>(a, n_chunks, s);
        if (cm == 2)
          return std_ ? launch_c<NT, W, PREC_BF16, true, FAMILY_LOGISTIC, 2>(a, n_chunks, s)
                      : launch_c<NT, W, PREC_BF16, false, FAMILY_LOGISTIC, 2>(a, n_chunks, s);
        if (cm == 3)
          return std_ ? launch_c<NT, W, PREC_BF16, true, FAMILY_LOGISTIC, 3>(a, n_chunks, s)
                      : launch_c<NT, W, PREC_BF16, false, FAMILY_LOGISTIC, 3>(a, n_chunks, s);
      }
      return std_ ? launch_c<NT, W, PREC_BF16, true, FAMILY_LOGISTIC>(a, n_chunks, s)
                  : launch_c<NT, W, PREC_BF16, false, FAMILY_LOGISTIC>(a, n_chunks, s);
    case PREC_F32:
      return std_ ? launch_c<NT, W, PREC_F32, true, FAMILY_LOGISTIC>(a, n_chunks, s)
                  : launch_c<NT, W, PREC_F32, false, FAMILY_LOGISTIC>(a, n_chunks, s);
    default:
      return std_ ? launch_c<NT, W, PREC_F64, true, FAMILY_LOGISTIC>(a, n_chunks, s)
                  : launch_c<NT, W, PREC_F64, false, FAMILY_LOGISTIC>(a, n_chunks, s);
  }
}

template <int NT>
static hipError_t launch_coop_nt(const PassArgs& a, int prec, bool std_, int family,
                                 int n_chunks, hipStream_t s) {
  return launch_coop_ntw<NT, coop_waves(NT)>(a, prec, std_, family, n_chunks, s);
}

}  // namespace dlsa
