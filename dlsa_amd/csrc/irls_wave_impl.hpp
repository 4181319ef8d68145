// Per-wave fp64 IRLS pass (gfx950 / CDNA4): one 64-lane workgroup streams a
// chunk of rows of one partition through its OWN LDS-DMA ring and owns every
// lower-triangle 16x16 tile of X^T W X in registers.  Instantiated by
// irls_wave.hip.
//
// Replaces, per Newton iteration, the per-partition work of the reference map
// stage (sklearn newton-cg Hessian products, predict_proba and
// Sig_inv = X^T diag(p(1-p)) X, dlsa/models.py:110-131) with ONE pass over X;
// this is the exact (fp64-MFMA) pass whose Hessian is returned as Sig_inv
// (models.py:130) and the single pass of the OLS path.
//
// Why a wave-private design for fp64: on gfx950 fp64 VALU
// work and v_mfma_f64_16x16x4 never execute together on a SIMD
// (SQ_VALU_MFMA_COEXEC_CYCLES = 0 in profiles/r01f_pmc.csv), so the pass time
// is MFMA cycles + VALU cycles + stalls, and everything that is not an MFMA
// must be cut rather than overlapped:
//   * no barriers: a wave reads only the rows it DMA'd itself, so the row
//     phase (eta, w, r, log-lik, gradient) and the tile phase need no
//     workgroup synchronisation and the next block's DMA stays in flight
//     across both phases (s_waitcnt vmcnt counted, never drained);
//   * the row phase runs R = 64 / LPR rows at once (16 at LPR = 4), so the fp64
//     exp / division / log1p sequences cost one instruction stream per 16
//     rows instead of per 8 (the cooperative kernel) or per 4 (a k-step);
//   * the tile phase loads each column tile's operand once per k-step (NT
//     ds_read_b64), forms w*x with NT multiplies and issues all T MFMAs --
//     the same static code in every wave (no per-wave tile assignment whose
//     branch merges copy accumulators).
// T accumulators of 8 registers (224 at NT = 7) force one wave per SIMD;
// LPR = 8 (R = 8) above NT = 7 keeps the row-phase registers in budget.
#pragma once

#include <stdint.h>
#include <stdlib.h>

#include <array>
#include <type_traits>
#include <utility>

#include "dlsa_internal.hpp"

namespace dlsa {

typedef double wd4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) void wlds_void_t;

namespace {

template <int N>
__device__ __forceinline__ void wv_wait_vmcnt() {
  static_assert(N >= 0 && N < 64, "vmcnt is 6 bits on gfx950");
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
// wait until at most n (runtime, <= N) vector-memory ops of this wave are
// outstanding
template <int N>
__device__ __forceinline__ void wv_wait_vmcnt_le(int n) {
  if constexpr (N <= 0) {
    wv_wait_vmcnt<0>();
  } else {
    if (n >= N)
      wv_wait_vmcnt<N>();
    else
      wv_wait_vmcnt_le<N - 1>(n);
  }
}

__device__ __forceinline__ double wv_xor16(double v) {
  const unsigned lo = __double2loint(v), hi = __double2hiint(v);
  const auto a = __builtin_amdgcn_permlane16_swap(lo, lo, false, false);
  const auto b = __builtin_amdgcn_permlane16_swap(hi, hi, false, false);
  return __hiloint2double(b[0], a[0]) + __hiloint2double(b[1], a[1]);
}
__device__ __forceinline__ double wv_xor32(double v) {
  const unsigned lo = __double2loint(v), hi = __double2hiint(v);
  const auto a = __builtin_amdgcn_permlane32_swap(lo, lo, false, false);
  const auto b = __builtin_amdgcn_permlane32_swap(hi, hi, false, false);
  return __hiloint2double(b[0], a[0]) + __hiloint2double(b[1], a[1]);
}
// The value of lane l ^ 32.  v_permlane32_swap exchanges lanes 32-63 of vdst
// with lanes 0-31 of src: with both = v, vdst holds the partner's value in
// the upper half and src in the lower half.
__device__ __forceinline__ double wv_swap32(double v, bool upper) {
  const unsigned lo = __double2loint(v), hi = __double2hiint(v);
  const auto a = __builtin_amdgcn_permlane32_swap(lo, lo, false, false);
  const auto b = __builtin_amdgcn_permlane32_swap(hi, hi, false, false);
  return upper ? __hiloint2double(b[0], a[0]) : __hiloint2double(b[1], a[1]);
}
template <int CTRL>
__device__ __forceinline__ double wv_dpp(double v) {
  const int lo = __builtin_amdgcn_mov_dpp(__double2loint(v), CTRL, 0xF, 0xF, false);
  const int hi = __builtin_amdgcn_mov_dpp(__double2hiint(v), CTRL, 0xF, 0xF, false);
  return __hiloint2double(hi, lo);
}

// Sum over the LPR lanes of one row (lanes l, l + R, l + 2R, ...); every lane
// of the row ends with the bitwise-identical total (each step adds a
// commutative pair).
template <int R>
__device__ __forceinline__ double wv_row_sum(double v) {
  static_assert(R == 16 || R == 8 || R == 4, "16, 8 or 4 rows per block");
  if constexpr (R == 4) v += __shfl_xor(v, 4);   // l ^ 4 (no DPP form)
  if constexpr (R <= 8) v += wv_dpp<0x128>(v);  // row_ror 8: l ^ 8
  v = wv_xor16(v);
  v = wv_xor32(v);
  return v;
}

// Buffer resource with every word made wave-uniform (readfirstlane), so the
// LDS-DMA loads take it in SGPRs: without this the compiler may keep it in
// VGPRs and wrap every buffer_load ... lds in a waterfall loop.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t wv_rsrc(uintptr_t base, uintptr_t bytes) {
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)base);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)((uint64_t)base >> 32));
  const uint32_t nr = __builtin_amdgcn_readfirstlane(
      (uint32_t)(bytes < 0x7FFFFFF0u ? bytes : 0x7FFFFFF0u));
  return __builtin_amdgcn_make_buffer_rsrc((void*)(((uint64_t)hi << 32) | lo), (short)0, (int)nr,
                                           0x00020000);
}

// 1 / d for d in [1, 3]: hardware estimate + two Newton steps (~1 ulp; the
// library division's scaling / fix-up steps are for operands this never sees)
__device__ __forceinline__ double wv_rcp(double d) {
  double r = __builtin_amdgcn_rcp(d);
  r = fma(r, fma(-d, r, 1.0), r);
  r = fma(r, fma(-d, r, 1.0), r);
  return r;
}

// log(t) for t in [1, 2] (t = 1 + exp(-|eta|): the softplus of the
// log-likelihood).  t -> t / 2 above sqrt 2, then log t = k ln 2 + 2 atanh(s),
// s = (t - 1) / (t + 1) in [-0.172, 0.172], by the odd series to s^19
// (truncation < 1e-17 relative).  A few ulps, against ~70 instructions of the
// double-double library log1p; log1p's extra accuracy for tiny arguments is
// not needed here: the terms are summed, so the absolute error (~1e-16 per
// row) is what counts.
__device__ __forceinline__ double wv_log12(double t) {
  const bool hi = t > 1.4142135623730951;
  const double u = hi ? 0.5 * t : t;
  const double s = (u - 1.0) * wv_rcp(u + 1.0);
  const double s2 = s * s;
  double q = 1.0 / 19.0;
  q = fma(q, s2, 1.0 / 17.0);
  q = fma(q, s2, 1.0 / 15.0);
  q = fma(q, s2, 1.0 / 13.0);
  q = fma(q, s2, 1.0 / 11.0);
  q = fma(q, s2, 1.0 / 9.0);
  q = fma(q, s2, 1.0 / 7.0);
  q = fma(q, s2, 1.0 / 5.0);
  q = fma(q, s2, 1.0 / 3.0);
  const double l = fma(2.0 * s * s2, q, 2.0 * s);
  return hi ? l + 0.6931471805599453094 : l;
}

}  // namespace

// Ring slots per workgroup (DLSA_WAVE_NSLOT, DLSA_WAVE_NSLOT_OLS): 2 = one
// block in flight while the current one is computed; 3 = two blocks in
// flight.  Three slots for the OLS pass (8-row, 4 KiB blocks at P = 64) measured
// slower (config-4 pass 16.7-17.1 vs 14.9-15.2 ms, profiles/r04h_ols_ab.txt).
#ifndef DLSA_WAVE_NSLOT
#define DLSA_WAVE_NSLOT 2
#endif
#ifndef DLSA_WAVE_NSLOT_OLS
#define DLSA_WAVE_NSLOT_OLS 2
#endif
__host__ __device__ constexpr int wave_slots(int FAM) {
  return FAM == FAMILY_GAUSSIAN ? DLSA_WAVE_NSLOT_OLS : DLSA_WAVE_NSLOT;
}
// OLS without standardisation: a full block's row phase writes nothing the
// other wave reads (w = 1 is a constant of the tile phase), so the barrier
// between the row and tile phases can be kept for the tail block only
// (DLSA_WAVE_OLS_ONESYNC = 1; not faster: 15.2 vs 14.9-15.0 ms, r04h)
#ifndef DLSA_WAVE_OLS_ONESYNC
#define DLSA_WAVE_OLS_ONESYNC 0
#endif
// Ring slot: [16 B pad][npieces KiB of X rows][256 B: y of up to 32 rows]
__host__ __device__ __forceinline__ int wave_npieces(int RB, int p) {
  return (RB * p * 8 + 16 + 1023) / 1024;
}
__host__ __device__ __forceinline__ int wave_slot_bytes_impl(int RB, int p) {
  return 16 + wave_npieces(RB, p) * 1024 + 256;
}
// LDS of one workgroup: 2 ring slots + w of a block [RB] + theta [PMAX] +
// center / 1/scale [2][PMAX]
__host__ __device__ __forceinline__ int wave_lds_bytes_impl(int NT, int RB, int p, int FAM) {
  return wave_slots(FAM) * wave_slot_bytes_impl(RB, p) + RB * 8 + 3 * 16 * NT * 8;
}

// Waves per workgroup.  W = 2 (P <= 112): the T tiles are split over two
// waves by whole tile rows (each holds ~T/2 accumulators, <= 256 registers),
// so two workgroups' waves share every SIMD and one wave's LDS / DMA /
// dependency waits are covered by the other's MFMAs; the rows of a block are
// split between the waves in the row phase (P >= 17).  W = 1 (P <= 128): all T tiles
// in one wave, one wave per SIMD.  DLSA_WAVE_W overrides for profiling.
constexpr int wave_w_default(int NT) { return (NT >= 2 && NT <= 7) ? 2 : 1; }
// Lanes per row in the row phase: 4 (16 rows per wave) at W = 1, P <= 112; 16 (4
// rows per wave, 8-row blocks) for OLS at W = 2, P <= 64; else 8.  The OLS
// setting halves the ring (12 vs 21 KB per workgroup at P = 64: LDS allowed only
// 3.5 waves per SIMD) and runs 5 waves per SIMD (wave_min_waves): config-4 pass
// 16.2 vs 17.4 ms (profiles/r02at_lpr_ab.txt).  Logistic keeps 8: its exp / rcp /
// log sequence runs once per RW rows, and 4-row (or 16-row, RB = 32: 3.5 -> 2
// waves per SIMD by LDS) blocks measured slower at P = 64 (4.3 / 4.8 vs 3.4 ms,
// r02at / r02as).
constexpr int wave_lpr(int NT, int W, int FAM) {
  return (W > 1 && NT <= 4 && FAM == FAMILY_GAUSSIAN) ? 16 : (W == 1 && NT <= 7) ? 4 : 8;
}
constexpr int wave_rb(int NT, int W, int FAM) { return W * (64 / wave_lpr(NT, W, FAM)); }

// Edge strip (DLSA_WAVE_STRIP, default on).  The last tile row holds only
// s = P - 16 (NT - 1) parameter rows (4 at P = 100).  On the MI355X a
// v_mfma_f64_4x4x4_4b issues every ~7 ns per SIMD (75 TF/s chip-wide;
// tools/mfma4_probe.hip, profiles/r02_mfma4_probe.txt) -- a quarter of a
// 16x16x4's flops in a fraction of its issue time -- so with NS > 0 the
// strip's tiles are NS 4x4x4_4b sub-blocks each instead of one 16x16x4
// (NS = 1 for s <= 4, 2 for s <= 8).  4x4x4_4b maps (probe): A lane
// i + 4 b + 16 k, B lane j + 4 b + 16 k, D lane j + 4 b + 16 i, block b
// independent (CBSZ / ABID broadcasts have no effect on it), so the A operand
// of sub-block r is feature 16 (NT - 1) + 4 r + (l & 3) of row k in every
// block -- read from LDS -- and B is the 16x16x4 column operand unchanged:
// D lane j + 4 b + 16 i = H[16 (NT - 1) + 4 r + i][16 J + 4 b + j].
// (Computing every tile as 4x4x4_4b sub-blocks against DPP-rotated B -- the
// probe's 75 TF/s shape -- measured slower in this kernel: 31.0 vs 29.3 ms per
// config-2 exact pass, profiles/r02w_mf4_ab.txt.)
// OLS: the tile phase takes x itself as the A operand (no w * x multiplies;
// padded rows are zeroed in the ring by the row phase): 16.2-16.4 vs
// 16.4-16.5 ms per config-4 pass (profiles/r02av_ols_nomul_ab.txt)
#ifndef DLSA_WAVE_OLS_NOMUL
#define DLSA_WAVE_OLS_NOMUL 1
#endif
#ifndef DLSA_WAVE_STRIP
#define DLSA_WAVE_STRIP 1
#endif
constexpr int wave_strip_ns(int NT, int P) {
  return (!DLSA_WAVE_STRIP || NT < 2) ? 0
         : (P - 16 * (NT - 1) <= 4)   ? 1
         : (P - 16 * (NT - 1) <= 8)   ? 2
                                      : 0;
}

// MFMA time of tile row I in quarter tiles (a 4x4x4_4b ~ 1/4 of a 16x16x4
// issue slot, conservatively)
constexpr int wave_row_cost(int NT, int NS, int I) {
  return (NS > 0 && I == NT - 1) ? NT * NS : 4 * (I + 1);
}

// tile rows of wave `wid`: rows are dealt most expensive first to the lighter
// wave (NT = 7, no strip: {6, 3, 2} and {5, 4, 1, 0}, 14 tiles each; NS = 1:
// {5, 2, 1} and {4, 3, 6, 0}, 44 / 47 quarter tiles)
constexpr unsigned wave_rows_mask(int NT, int NS, int W, int wid) {
  if (W == 1) return (1u << NT) - 1;
  int load0 = 0, load1 = 0;
  unsigned m0 = 0, m1 = 0, done = 0;
  for (int n = 0; n < NT; ++n) {
    int best = -1;
    for (int I = NT - 1; I >= 0; --I)
      if (!((done >> I) & 1u) &&
          (best < 0 || wave_row_cost(NT, NS, I) > wave_row_cost(NT, NS, best)))
        best = I;
    done |= 1u << best;
    if (load0 <= load1) {
      load0 += wave_row_cost(NT, NS, best);
      m0 |= 1u << best;
    } else {
      load1 += wave_row_cost(NT, NS, best);
      m1 |= 1u << best;
    }
  }
  return wid == 0 ? m0 : m1;
}

template <int NT, int NS, int W, int WID>
struct WaveTiles {
  static constexpr unsigned RM = wave_rows_mask(NT, NS, W, WID);
  static constexpr int count() {
    int c = 0;
    for (int I = 0; I < NT; ++I)
      if ((RM >> I) & 1u) c += I + 1;
    return c;
  }
  static constexpr int TW = count();
  static constexpr int ncols() {  // B operands needed: columns 0 .. max I
    int c = 0;
    for (int I = 0; I < NT; ++I)
      if ((RM >> I) & 1u) c = I + 1;
    return c;
  }
  static constexpr int NC = ncols();
  static constexpr int I_of(int i) {  // tile i of this wave: rows ascending, J ascending
    for (int I = 0; I < NT; ++I)
      if ((RM >> I) & 1u) {
        if (i <= I) return I;
        i -= I + 1;
      }
    return -1;
  }
  static constexpr int J_of(int i) {
    for (int I = 0; I < NT; ++I)
      if ((RM >> I) & 1u) {
        if (i <= I) return i;
        i -= I + 1;
      }
    return -1;
  }
};

// MFMA issue order of a wave's tiles (DLSA_WAVE_ORDER = 1): greedy, each
// next tile taking a different A operand (tile row) AND a different B operand
// (tile column) than the previous one where one is left -- back-to-back fp64
// MFMAs on a shared operand register issue slower (tools/mfma_rate_probe.hip).
// 0: tiles in row order (the rows' A operand reused back to back).
#ifndef DLSA_WAVE_ORDER
#define DLSA_WAVE_ORDER 0
#endif
template <class TL, int TW>
struct WaveIssueOrder {
  static constexpr std::array<int, TW> make() {
    std::array<int, TW> ord{};
    bool used[TW > 0 ? TW : 1] = {};
    int pi = -1, pj = -1;
    for (int n = 0; n < TW; ++n) {
      int pick = -1;
      if (DLSA_WAVE_ORDER)
        for (int i = 0; i < TW && pick < 0; ++i)
          if (!used[i] && TL::I_of(i) != pi && TL::J_of(i) != pj) pick = i;
      for (int i = 0; i < TW && pick < 0; ++i)
        if (!used[i]) pick = i;
      used[pick] = true;
      ord[n] = pick;
      pi = TL::I_of(pick);
      pj = TL::J_of(pick);
    }
    return ord;
  }
  static constexpr std::array<int, TW> ord = make();
};

template <typename F, int... Is>
__device__ __forceinline__ void wv_static_for_impl(F&& f, std::integer_sequence<int, Is...>) {
  (f(std::integral_constant<int, Is>{}), ...);
}
template <int N, typename F>
__device__ __forceinline__ void wv_static_for(F&& f) {
  wv_static_for_impl(f, std::make_integer_sequence<int, N>{});
}

// workgroup sync of the block loop: this wave's LDS ops done, then (W > 1) a
// barrier without the vmcnt drain of __syncthreads (the next block's DMA
// stays in flight; irls_coop_impl.hpp lds_barrier)
template <int W>
__device__ __forceinline__ void wv_sync() {
  if constexpr (W > 1)
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
  else
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
}

struct WaveCtx {
  int64_t row0;
  int nrows, nb, npieces, slot_bytes, slot_y, part, chunk;
  __amdgpu_buffer_rsrc_t xr, yr;
  uintptr_t xcb;
};

// The block loop + epilogue of wave WID (a separate code path per wave: no
// branch merges of the accumulator arrays).
template <int NT, int NS, int W, int WID, bool STD, int FAM>
__device__ __forceinline__ void wave_body(const PassArgs& a, const WaveCtx& cx, char* smem) {
  using TL = WaveTiles<NT, NS, W, WID>;
  // strip tiles (the last tile row as NS 4x4x4_4b sub-blocks)
  constexpr auto strip = [](int I) { return NS > 0 && I == NT - 1; };
  constexpr bool HAS_STRIP = NS > 0 && ((TL::RM >> (NT - 1)) & 1u);
  constexpr int NSA = NS > 0 ? NS : 1;
  constexpr int LPR = wave_lpr(NT, W, FAM);
  constexpr int RW = 64 / LPR;   // rows of a block in this wave's row phase
  constexpr int RB = W * RW;     // rows per block
  constexpr int KS = RB / 4;     // MFMA k-steps per block
  constexpr int PMAX = 16 * NT;
  constexpr int M = PMAX / LPR;  // features per lane in the row phase
  constexpr int TW = TL::TW, NC = TL::NC;
  // OLS (w in {0, 1}): A operands are x itself (padded rows zeroed in the ring,
  // the intercept column = w)
  constexpr bool OLS_NOMUL = DLSA_WAVE_OLS_NOMUL && FAM == FAMILY_GAUSSIAN;
  // OLS is one pass at theta = 0 (fit_impl: fit_init zeroes theta, max_iter =
  // 1, no warm-start levels, no polish): eta = 0 and r = y, so the row phase
  // skips the x . theta dot products and their row reductions -- fp64 VALU
  // work that never co-executes with the fp64 MFMAs of the tile phase
  constexpr bool ETA0 = FAM == FAMILY_GAUSSIAN;
  constexpr int kWaveSlots = wave_slots(FAM);
  constexpr bool ONESYNC = DLSA_WAVE_OLS_ONESYNC && OLS_NOMUL && !STD;

  const int lane = threadIdx.x & 63;
  const int p = a.p, P = a.P, ic = a.intercept;
  double* wv = (double*)(smem + kWaveSlots * cx.slot_bytes);  // [RB] w of the block's rows
  double* bet = wv + RB;                             // [PMAX] theta of the partition
  double* stdv = bet + PMAX;                         // [2][PMAX] center, 1/scale (STD)

  // row-phase lane map: row = WID * RW + lane % RW, feature group sl = lane / RW;
  // the lane handles parameters f = sl + LPR m (m < M)
  const int rl = lane % RW, sl = lane / RW;
  const int row = WID * RW + rl;
  double gacc[M];
#pragma unroll
  for (int m = 0; m < M; ++m) gacc[m] = 0.0;
  double llacc = 0.0;
  wd4 acc[TW];           // 16x16x4 tiles (AGPRs)
  double sacc[TW][NSA];  // strip sub-blocks (the unused entries of either are dead)
#pragma unroll
  for (int i = 0; i < TW; ++i) {
    acc[i] = wd4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int r = 0; r < NSA; ++r) sacc[i][r] = 0.0;
  }

  // DMA: wave WID issues pieces j = WID, WID + W, ...; the last wave also y
  int my_ops = 0;
  for (int j = WID; j < cx.npieces; j += W) ++my_ops;
  if (WID == W - 1) ++my_ops;
  auto issue = [&](int blk) {
    char* sbase = smem + (blk % kWaveSlots) * cx.slot_bytes;
    const uintptr_t start = (uintptr_t)(a.X + (cx.row0 + (int64_t)blk * RB) * p);
    const int so = __builtin_amdgcn_readfirstlane((int)((start & ~(uintptr_t)15) - cx.xcb));
    for (int j = WID; j < cx.npieces; j += W)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(cx.xr, (wlds_void_t*)(sbase + 16 + j * 1024), 16,
                                               lane * 16, so + j * 1024, 0, DLSA_X_DMA_AUX);
    if (WID == W - 1)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(cx.yr, (wlds_void_t*)(sbase + cx.slot_y), 4,
                                               lane * 4, blk * RB * 8, 0, 0);
  };

  const int fl = lane & 15, q = lane >> 4;
  const bool icpt_lane = ic && fl == 0;
  for (int b = 0; b < kWaveSlots - 1 && b < cx.nb; ++b) issue(b);
  for (int b = 0; b < cx.nb; ++b) {
    // this wave's pieces of block b landed (the younger blocks' may not have)
    if constexpr (kWaveSlots == 2) {
      wv_wait_vmcnt<0>();
    } else {
      const int younger = min(kWaveSlots - 2, cx.nb - 1 - b);  // blocks issued after b
      wv_wait_vmcnt_le<2 * 8>(younger * my_ops);
    }
    wv_sync<W>();        // every wave's pieces landed; block b-1 fully consumed
    if (b + kWaveSlots - 1 < cx.nb) issue(b + kWaveSlots - 1);  // into the slot of block b-1
    const char* slot = smem + (b % kWaveSlots) * cx.slot_bytes;
    const uintptr_t start = (uintptr_t)(a.X + (cx.row0 + (int64_t)b * RB) * p);
    double* xs = (double*)(slot + 16 + (start & 15));
    const double* ys = (const double*)(slot + cx.slot_y);
    const int rows_left = cx.nrows - b * RB;

    // ---- row phase: RW rows of this wave, LPR lanes per row -------------------
    {
      const bool valid = row < rows_left;
      double* xrw = xs + row * p + (sl - ic);
      double xv[M];
      double e0 = 0.0, e1 = 0.0;
#pragma unroll
      for (int m = 0; m < M; ++m) {
        double v = xrw[LPR * m];
        if constexpr (STD) {
          v = (v - stdv[sl + LPR * m]) * stdv[PMAX + sl + LPR * m];
          const int f = sl + LPR * m;
          // standardise in place for the tile phase (own row, own features;
          // the intercept slot f = 0 is the previous row's last value)
          if (f >= ic && f < P) xrw[LPR * m] = v;
        }
        if constexpr (OLS_NOMUL) {
          // OLS: w is 1 on rows of the chunk and 0 past it; zero the padded
          // rows' features in place so the tile phase can skip w * x
          const int f = sl + LPR * m;
          if (!valid && f >= ic && f < P) xrw[LPR * m] = 0.0;
        }
        if (m == 0 && ic && sl == 0) v = 1.0;
        xv[m] = v;
        if constexpr (!ETA0) {
          const double bm = bet[sl + LPR * m];
          if (m & 1)
            e1 = fma(v, bm, e1);
          else
            e0 = fma(v, bm, e0);
        }
      }
      const double e = ETA0 ? 0.0 : wv_row_sum<RW>(e0 + e1);
      const double yv = ys[row];
      double w, r;
      if constexpr (FAM == FAMILY_LOGISTIC) {
        const double ea = exp(-fabs(e));
        const double inv = wv_rcp(1.0 + ea);
        const double mu = e >= 0.0 ? inv : ea * inv;
        w = ea * inv * inv;  // mu (1 - mu), cancellation free
        r = yv - mu;
        if (valid && sl == 0) llacc += yv * e - (fmax(e, 0.0) + wv_log12(1.0 + ea));
      } else {  // gaussian (OLS): mu = eta, w = 1, ll = -rss / 2
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
      if (sl == 0) wv[row] = w;
    }
    // w (and standardised / zeroed x) of all rows visible
    if constexpr (W > 1) {
      if (!ONESYNC || rows_left < RB) wv_sync<W>();  // workgroup-uniform
    }
    const bool w_one = ONESYNC && rows_left >= RB;  // full OLS block: w = 1 on every row

    // ---- tile phase: KS k-steps of 4 rows, this wave's TW tiles ---------------
    // operands of k-step s+1 are read while the MFMAs of k-step s run
    double xo[2][NC], xso[2][NSA], wk[2];
    auto load = [&](int s, int u) {
      const double* xq = xs + (4 * s + q) * p + (fl - ic);
#pragma unroll
      for (int c = 0; c < NC; ++c) xo[u][c] = xq[16 * c];
      if constexpr (HAS_STRIP) {
        // strip A operand of sub-block r: feature 16 (NT - 1) + 4 r + (l & 3)
        const double* xt = xq + 16 * (NT - 1) + (lane & 3) - fl;
#pragma unroll
        for (int r = 0; r < NS; ++r) xso[u][r] = xt[4 * r];
      }
      wk[u] = w_one ? 1.0 : wv[4 * s + q];
    };
    load(0, 0);
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      const int u = s & 1;
      if (s + 1 < KS) load(s + 1, u ^ 1);
      double xv[NC], av[NC];
#pragma unroll
      for (int c = 0; c < NC; ++c) {
        double v = xo[u][c];
        if (c == 0 && icpt_lane) v = OLS_NOMUL ? wk[u] : 1.0;
        xv[c] = v;
        if ((TL::RM >> c) & 1u) av[c] = OLS_NOMUL ? v : v * wk[u];
      }
      double as[NSA];
      if constexpr (HAS_STRIP) {
#pragma unroll
        for (int r = 0; r < NS; ++r) as[r] = OLS_NOMUL ? xso[u][r] : xso[u][r] * wk[u];
      }
      wv_static_for<TW>([&](auto oI) {
        constexpr int i = WaveIssueOrder<TL, TW>::ord[decltype(oI)::value];
        constexpr int I = TL::I_of(i), J = TL::J_of(i);
        if constexpr (strip(I)) {
#pragma unroll
          for (int r = 0; r < NS; ++r)
            sacc[i][r] = __builtin_amdgcn_mfma_f64_4x4x4f64(as[r], xv[J], sacc[i][r], 0, 0, 0);
        } else {
          acc[i] = __builtin_amdgcn_mfma_f64_16x16x4f64(av[I], xv[J], acc[i], 0, 0, 0);
        }
      });
    }
    // keep every 16x16x4 accumulator in AGPRs across the loop back edge (the
    // strip's 64-bit ones are left to the allocator: pinned one by one they
    // get shuffled between AGPRs; explicit capture: an asm operand alone does
    // not capture in a generic lambda)
    wv_static_for<TW>([&acc](auto iI) {
      constexpr int i = decltype(iI)::value;
      if constexpr (!(NS > 0 && TL::I_of(i) == NT - 1)) asm volatile("" : "+a"(acc[i]));
    });
  }
  wv_wait_vmcnt<0>();

  // ---- epilogue: this chunk's partials (newton_solve.hip slab layout) --------
  double* sH = a.slab_H + (int64_t)cx.chunk * (NT * (NT + 1) / 2) * 256;
  wv_static_for<TW>([&](auto iI) {
    constexpr int i = decltype(iI)::value;
    constexpr int t = TL::I_of(i) * (TL::I_of(i) + 1) / 2 + TL::J_of(i);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      if constexpr (strip(TL::I_of(i))) {
        // sub-block r: rows 4 r + (l >> 4), columns l & 15; rows past it: 0
        sH[t * 256 + (4 * r + q) * 16 + fl] = r < NS ? sacc[i][r < NSA ? r : 0] : 0.0;
      } else {  // f64 16x16x4 C/D map: row = (l >> 4) + 4 r, col = l & 15
        sH[t * 256 + (q + 4 * r) * 16 + fl] = acc[i][r];
      }
    }
  });
  // gradient: sum the RW row lanes of each feature group, then the W waves
#pragma unroll
  for (int m = 0; m < M; ++m) {
#pragma unroll
    for (int o = 1; o < RW; o <<= 1) gacc[m] += __shfl_xor(gacc[m], o);
  }
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) llacc += __shfl_xor(llacc, o);
  double* red = (double*)smem;  // the ring is no longer needed: [W - 1][PMAX + 1]
  if constexpr (W > 1) {
    __syncthreads();
    if constexpr (WID > 0) {
#pragma unroll
      for (int m = 0; m < M; ++m)
        if (rl == 0) red[(WID - 1) * (PMAX + 1) + sl + LPR * m] = gacc[m];
      if (lane == 0) red[(WID - 1) * (PMAX + 1) + PMAX] = llacc;
    }
    __syncthreads();
  }
  if constexpr (WID == 0) {
#pragma unroll
    for (int m = 0; m < M; ++m) {
      double v = gacc[m];
#pragma unroll
      for (int w = 1; w < W; ++w) v += red[(w - 1) * (PMAX + 1) + sl + LPR * m];
      if (rl == 0) a.slab_g[(int64_t)cx.chunk * PMAX + sl + LPR * m] = v;
    }
    double ll = llacc;
#pragma unroll
    for (int w = 1; w < W; ++w) ll += red[(w - 1) * (PMAX + 1) + PMAX];
    if (lane == 0) a.slab_ll[cx.chunk] = ll;
  }
}

// minimum waves per SIMD (register budget): OLS at P <= 64 fits 5 (48 VGPRs +
// <= 41 AGPRs, no scratch); the logistic kernels would spill there
constexpr int wave_min_waves(int NT, int W, int FAM) {
  return W == 1 ? 1 : (NT <= 4 && FAM == FAMILY_GAUSSIAN ? 5 : 2);
}

template <int NT, int NS, int W, bool STD, int FAM>
__global__ __launch_bounds__(64 * W, wave_min_waves(NT, W, FAM)) void irls_wave_kernel(
    const PassArgs a) {
  constexpr int RB = wave_rb(NT, W, FAM);
  constexpr int PMAX = 16 * NT;
  extern __shared__ __attribute__((aligned(16))) char smem[];

  WaveCtx cx;
  cx.chunk = blockIdx.x;
  cx.part = __builtin_amdgcn_readfirstlane(a.chunk_part[cx.chunk]);
  if (a.phase[cx.part] != a.want_phase) return;  // workgroup-uniform

  const int tid = threadIdx.x;
  const int p = a.p, P = a.P, ic = a.intercept;
  cx.row0 = ((int64_t)__builtin_amdgcn_readfirstlane((int)(a.chunk_row0[cx.chunk] >> 32)) << 32) |
            (uint32_t)__builtin_amdgcn_readfirstlane((int)a.chunk_row0[cx.chunk]);
  cx.nrows = __builtin_amdgcn_readfirstlane(a.chunk_rows[cx.chunk]);
  cx.nb = (cx.nrows + RB - 1) / RB;
  cx.npieces = wave_npieces(RB, p);
  constexpr int kWaveSlots = wave_slots(FAM);
  cx.slot_bytes = wave_slot_bytes_impl(RB, p);
  cx.slot_y = 16 + cx.npieces * 1024;
  double* wv = (double*)(smem + kWaveSlots * cx.slot_bytes);
  double* bet = wv + RB;
  double* stdv = bet + PMAX;

  // the ring must hold finite values where no DMA lands (tails, pads): a
  // padded row reads them with w = 0, and 0 * NaN would poison the tiles
  for (int o = tid * 16; o < kWaveSlots * cx.slot_bytes; o += 64 * W * 16)
    *(uint4*)(smem + o) = make_uint4(0, 0, 0, 0);
  for (int f = tid; f < PMAX; f += 64 * W)
    bet[f] = (f < P) ? a.theta[(int64_t)cx.part * P + f] : 0.0;
  if constexpr (STD) {
    for (int f = tid; f < PMAX; f += 64 * W) {
      const int j = f - ic;
      const bool in = j >= 0 && j < p;
      stdv[f] = in ? a.center[j] : 0.0;
      stdv[PMAX + f] = in ? 1.0 / a.scale[j] : 1.0;
    }
  }
  __syncthreads();

  cx.xcb = (uintptr_t)(a.X + cx.row0 * p) & ~(uintptr_t)15;
  cx.xr = wv_rsrc(cx.xcb, a.x_last16 + 16 - cx.xcb);
  const uintptr_t ycb = (uintptr_t)(a.y + cx.row0);
  cx.yr = wv_rsrc(ycb, a.y_last4 + 4 - ycb);
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  if constexpr (W == 1) {
    wave_body<NT, NS, 1, 0, STD, FAM>(a, cx, smem);
  } else {
    if (wid == 0)
      wave_body<NT, NS, W, 0, STD, FAM>(a, cx, smem);
    else
      wave_body<NT, NS, W, 1, STD, FAM>(a, cx, smem);
  }
}

// requested: dlsa_fit_options.exact_waves (0 = automatic)
static inline int wave_w(int NT, int requested = 0) {
  const int w = requested;
  if ((w == 1 && NT <= 8) || (w == 2 && NT >= 2 && NT <= 7)) return w;
  return wave_w_default(NT);
}

template <int NT, int W, bool STD, int FAM>
static hipError_t launch_wave_t(const PassArgs& a, int n_chunks, hipStream_t s) {
  const size_t lds = wave_lds_bytes_impl(NT, wave_rb(NT, W, FAM), a.p, FAM);
  switch (wave_strip_ns(NT, a.P)) {
    case 1:
      hipLaunchKernelGGL((irls_wave_kernel<NT, 1, W, STD, FAM>), dim3(n_chunks), dim3(64 * W), lds,
                         s, a);
      break;
    case 2:
      hipLaunchKernelGGL((irls_wave_kernel<NT, 2, W, STD, FAM>), dim3(n_chunks), dim3(64 * W), lds,
                         s, a);
      break;
    default:
      hipLaunchKernelGGL((irls_wave_kernel<NT, 0, W, STD, FAM>), dim3(n_chunks), dim3(64 * W), lds,
                         s, a);
  }
  return hipGetLastError();
}

template <int NT, bool STD, int FAM>
static hipError_t launch_wave_sf(const PassArgs& a, int n_chunks, hipStream_t s) {
  if constexpr (NT >= 2 && NT <= 7) {
    if (wave_w(NT, a.waves) == 2) return launch_wave_t<NT, 2, STD, FAM>(a, n_chunks, s);
  }
  return launch_wave_t<NT, 1, STD, FAM>(a, n_chunks, s);
}

template <int NT>
static hipError_t launch_wave_nt(const PassArgs& a, bool std_, int family, int n_chunks,
                                 hipStream_t s) {
  if (family == FAMILY_GAUSSIAN)
    return std_ ? launch_wave_sf<NT, true, FAMILY_GAUSSIAN>(a, n_chunks, s)
                : launch_wave_sf<NT, false, FAMILY_GAUSSIAN>(a, n_chunks, s);
  return std_ ? launch_wave_sf<NT, true, FAMILY_LOGISTIC>(a, n_chunks, s)
              : launch_wave_sf<NT, false, FAMILY_LOGISTIC>(a, n_chunks, s);
}

}  // namespace dlsa
