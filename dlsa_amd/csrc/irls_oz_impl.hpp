// Exact (fp64-accurate) IRLS pass on the int8 matrix cores (gfx950 / CDNA4):
// X^T W X by integer digit slices (the Ozaki scheme), the gradient and the
// log-likelihood in fp64.  Instantiated by irls_oz.hip / irls_oz_g2.hip.
//
// Replaces, per exact Newton iteration, the per-partition work of the
// reference map stage -- sklearn newton-cg's Hessian, predict_proba and
// Sig_inv = X^T diag(p(1-p)) X (dlsa/models.py:110-131) -- with ONE pass over
// X, like irls_wave_impl.hpp, but without the fp64 MFMA: on gfx950 a
// v_mfma_f64_16x16x4 issues every ~70 cycles per SIMD (72 TF/s,
// profiles/r03h_mfma_rate_probe.txt) and fp64 VALU work never overlaps it, so
// the fp64 pass is MFMA-bound at ~2x the HBM time of its 808 B/row (config 2:
// 24 ms against the 14 ms of a bf16 pass).  A v_mfma_i32_16x16x64_i8 issues
// every 16 cycles and accumulates exactly in int32.
//
// Numerics.  z = sqrt(w) x (the fp64 row weight times the
// fp64 feature).  Per chunk and feature f an exponent E_f with |z_f| < 2^E_f
// for every row of the chunk (digit_exponent below): from the max |z_f| that
// the partition's last full-data bf16 pass recorded at theta_rec
// (PassArgs::zcolmax), grown by exp(|theta - theta_rec|_1 max|x| / 2), the
// most sqrt(w) can grow between the two points (|d log sqrt(w) / d eta| <=
// 1/2), and never above max |x_f| / 2 (sqrt(w) <= 1/2 at every theta).
// F = round(z 2^(38 - E_f)), |F| < 2^38, by ONE fp64 FMA against
// 1.5 2^52 + B (B = 0x8080808080): the low 40 mantissa bits of the result are
// F + B, whose five bytes XOR 0x80 are the balanced signed digits d_0 (most
// significant) .. d_4 of F = sum_s d_s 2^(8(4-s)).  Then
//   sum_rows F_i F_j = 2^64 sum_k 2^(-8k) L_k,  L_k = sum_{a+b=k} sum_rows d_a(i) d_b(j),
// keeping the levels k < NL: H_ij = 2^(E_i + E_j - 12) sum_{k<NL} 2^(-8k) L_k.
// The integer sums are exact and order-free; the error is the rounding of z
// to 38 bits below 2^E_f and the dropped levels (~2^(-8 NL) of a row's leading
// product, random in sign): 2.15e-12 against the oracle at config 2, as the
// fp64 pass (profiles/r03w_bench_c2.json), and within 1e-11 of the fp64 pass at
// the same iterate (tests/test_gpu_ozaki.py).
//
// MFMA pairing.  One v_mfma_i32_16x16x64_i8 sums 64 k slots; a 32-row block
// fills them with TWO digit products: lane group g holds the 8 rows of
// producer wave g, bytes 0-7 of its fragment digit a (A features) / b (B
// features), bytes 8-15 digit a+1 / b-1 -- both products of level a+b.  A and
// B fragments of one lane hold the same k slots, so this needs no knowledge
// of the instruction's k order.  a in {0, 2, 4}: 9 MFMAs per tile per 32 rows
// cover the 15 products of levels 0-4 (out-of-range digits are zeroed in the
// register).
//
// Workgroup = 4 producer + 4 consumer waves, one workgroup per CU; an
// iteration is two 32-row blocks (b0 = 2m, b1 = 2m + 1):
//   producers: the row phase of both blocks, interleaved (8 rows per wave per
//     block, 8 lanes per row: eta, w, r, log-lik, gradient in fp64 -- two
//     independent dependency chains per wave), then the digits of those rows
//     straight from the registers: the 4 rows of a DPP quad are byte-transposed
//     (2 quad_perm moves + 2 v_perm per dword), so lane j of a quad writes
//     digit plane 4-j of its feature for 4 rows as one dword.  The image of a
//     wave's 8 rows (5 planes x 16 NT features x 8 bytes) is written over those
//     rows' own x bytes in the ring slot, once they are read;
//   consumers: the DMA of the next iteration's two blocks (LDS-DMA, 6-slot
//     ring), then the lower-triangle 16x16 tiles of X^T W X by column strips
//     from the previous iteration's two images, NL int32 level accumulators
//     per tile in registers.
// One barrier per iteration.
#pragma once

#include <stdint.h>
#include <stdlib.h>

#include <array>
#include <utility>

#include "irls_wave_impl.hpp"

namespace dlsa {

typedef int oz_i4 __attribute__((ext_vector_type(4)));

namespace ozk {

constexpr int NPW = 4;           // producer waves
constexpr int NCW = 4;           // consumer waves
constexpr int RB = 32;           // rows per DMA block
constexpr int RPW = RB / NPW;    // rows per producer wave per block (8)
constexpr int LPR = 64 / RPW;    // row-phase lanes per row (8)
constexpr int NSLOT = 6;         // ring: 2 in flight, 2 producing, 2 consuming
// Ring-slot ownership.  Between barriers B_m and B_{m+1}:
//   slots of blocks 2m+2, 2m+3: written only by the LDS-DMA (issued by the
//     consumers), read by nobody;
//   slots of blocks 2m, 2m+1: producer wave pw reads and then overwrites
//     ONLY the bytes of its own 8 rows (rows 8 pw .. 8 pw + 7 of each block)
//     -- there is no barrier between one producer wave's reads and another's
//     image stores, so a value read from another wave's rows may already be
//     digit bytes (the padding features f >= P of row 8 pw + 7 read row
//     8 pw + 8 and are zeroed, never used);
//   slots of blocks 2m-2, 2m-1: read only (the consumers' operands).
// DLSA_OZ_CHECK builds poison (NaN) any producer read of a feature f < P
// outside the reading wave's own rows, so a violation ends the partition
// nonfinite in the tests.
static_assert(NSLOT >= 6, "2 blocks in flight + 2 producing + 2 consuming");
#ifndef DLSA_OZ_CHECK
#define DLSA_OZ_CHECK 0
#endif
// digits per value (DLSA_OZ_DIGITS: 5, the product; 4: a 30-bit grid, levels
// 0-4 -- 8 MFMAs per tile and 32-row block instead of 9, one quad transpose
// per value; ~5e-11 instead of ~2e-12 per entry in the numpy restatement; A/B
// variant)
#ifndef DLSA_OZ_DIGITS
#define DLSA_OZ_DIGITS 5
#endif
constexpr int ND = DLSA_OZ_DIGITS;
static_assert(ND == 4 || ND == 5, "4 or 5 digits");
constexpr int GBITS = 8 * ND - 2;  // F = round(z 2^(GBITS - E)), |F| <= 2^GBITS
// levels k = a + b of digit products kept (DLSA_OZ_LEVELS: 5, 6 or 7)
#ifndef DLSA_OZ_LEVELS
#define DLSA_OZ_LEVELS 5
#endif
constexpr int NL = DLSA_OZ_LEVELS;
static_assert((ND == 5 && NL >= 5 && NL <= 7) || (ND == 4 && NL == 5), "levels");
constexpr int EMIN = -985;       // 2^(38 - EMIN) stays finite
constexpr int EMAX = 1009;       // MAGIC 2^(EMAX - 38) stays finite (|z| >= 2^1009
                                 // overflows the fp64 Gram anyway)
// 1.5 2^52 + B, B = 0x8080808080 (0x80808080 for 4 digits): t = fma(x, c,
// MAGIC) holds F + B in its low 8 ND bits
constexpr double MAGIC = 6755399441055744.0 + (ND == 5 ? 551911719040.0 : 2155905152.0);

// Ring slot: [16 B pad][x: the block's bytes from its 16-B-aligned start][y: 256 B].
// The x span is cut to what the block needs (the last 1-KiB DMA piece runs
// with only the lanes inside it), so six slots of p = 100 fit the CU.
__host__ __device__ constexpr int xspan(int p) { return (RB * p * 8 + 16 + 15) & ~15; }
__host__ __device__ constexpr int npieces(int p) { return (xspan(p) + 1023) / 1024; }
__host__ __device__ constexpr int slot_bytes(int p) { return 16 + xspan(p) + 256; }
// a wave's image: [feature][digit plane][8 rows] bytes, 48 B per feature (5
// planes + an unwritten sixth), so a lane's operand pair of planes (a, a+1),
// a even, is one aligned 16-byte read
constexpr int kFeatBytes = ND == 5 ? 48 : 32;
constexpr int kMaxPiecesPerWave = 7;  // 1-KiB DMA pieces of a block per consumer wave
// consumers issue the next blocks' DMA one piece per tile (1) or all before
// their MFMAs (0)
#ifndef DLSA_OZ_TICK
#define DLSA_OZ_TICK 1
#endif
// DMA schedule of the consumers: 0 the next blocks' pieces ticked through
// both images' MFMAs; 1 (the product since round 4) / 2 all of them during
// the first image's (see the consumer loop)
#ifndef DLSA_OZ_SCHED
#define DLSA_OZ_SCHED 1
#endif
// consumers at s_setprio DLSA_OZ_PRIO: the younger half of the workgroup
// otherwise gets only the producers' leftover issue slots (MI355X_MICROARCH.md
// "Two waves per SIMD", items 2 and 4)
#ifndef DLSA_OZ_PRIO
#define DLSA_OZ_PRIO 1
#endif
// producer digits (DLSA_OZ_DBATCH 1): the digit words of a block's values are
// formed for all features first, then transposed stage by stage, so the
// DPP / v_perm chains of different features interleave
#ifndef DLSA_OZ_DBATCH
#define DLSA_OZ_DBATCH 1
#endif
// byte offset of digit plane d in a feature's 48-byte image entry
__host__ __device__ constexpr int plane_off(int d) { return 8 * d; }
// producers hold 4 rows of a feature per lane (DLSA_OZ_R4 1, oz_producer_r4):
// in-register byte transposes; 0: 8 lanes per row, DPP quad transposes
#ifndef DLSA_OZ_R4
#define DLSA_OZ_R4 1
#endif
// fold the last tile row into 5 MFMAs per tile when it holds <= 5 features
// (DLSA_OZ_EDGE 1, OzConsumer)
#ifndef DLSA_OZ_EDGE
#define DLSA_OZ_EDGE 0
#endif
// the last DMA piece of a block as its final 1 KiB, overlapping the piece
// before it with the same bytes (DLSA_OZ_OVL 1: whole-wave, no lane
// predicate; 0: only the lanes inside the block; the producer schedules
// always overlap)
#ifndef DLSA_OZ_OVL
#define DLSA_OZ_OVL 0
#endif
// DMA pieces per block and wave issued by the producers (DLSA_OZ_PDMA, with
// the consumer schedules 0-2; see the DMA section of irls_oz_kernel)
#ifndef DLSA_OZ_PDMA
#define DLSA_OZ_PDMA 1
#endif
// per-feature magic constants instead of a per-value ldexp (DLSA_OZ_MAGICF 1)
#ifndef DLSA_OZ_MAGICF
#define DLSA_OZ_MAGICF 1
#endif
// profiling-only ablations (bits): 1 producers skip the row phase and digits, 2
// consumers skip the MFMAs
#ifndef DLSA_OZ_ABLATE
#define DLSA_OZ_ABLATE 0
#endif
__host__ __device__ constexpr int img_bytes(int NT) { return 16 * NT * kFeatBytes; }
// LDS after the ring: theta, center / 1/scale [PMAX] fp64, digit exponents [PMAX]
__host__ __device__ constexpr int extra_bytes(int NT) { return 3 * 16 * NT * 8 + 16 * NT * 4; }
__host__ __device__ constexpr int lds_bytes(int NT, int p) {
  return NSLOT * slot_bytes(p) + extra_bytes(NT);
}
// the pass applies when a wave's image (+ skew) fits in the x bytes of its 8
// rows and the ring fits the CU
__host__ __device__ constexpr bool fits(int NT, int p) {
  return img_bytes(NT) <= RPW * p * 8 && lds_bytes(NT, p) <= 160 * 1024 &&
         npieces(p) <= NCW * kMaxPiecesPerWave;
}

// Column strips J (tiles (I, J), I = J .. NT-1) dealt to the consumer waves,
// largest first, each to the wave with the fewest tiles (NT = 7: {0}, {1, 6},
// {2, 5}, {3, 4}: 7 tiles each).
constexpr unsigned strip_mask(int NT, int cw) {
  int load[NCW] = {0, 0, 0, 0};
  unsigned m[NCW] = {0, 0, 0, 0};
  for (int J = 0; J < NT; ++J) {
    int best = 0;
    for (int w = 1; w < NCW; ++w)
      if (load[w] < load[best]) best = w;
    load[best] += NT - J;
    m[best] |= 1u << J;
  }
  return m[cw];
}

template <int NT, int CW>
struct Tiles {
  static constexpr unsigned SM = strip_mask(NT, CW);
  static constexpr int count() {
    int c = 0;
    for (int J = 0; J < NT; ++J)
      if ((SM >> J) & 1u) c += NT - J;
    return c;
  }
  static constexpr int TW = count();
  // tile index of (I, J) in this wave (strips ascending, I ascending)
  static constexpr int index(int I, int J) {
    int c = 0;
    for (int j = 0; j < NT; ++j)
      if ((SM >> j) & 1u) {
        if (j == J) return c + (I - J);
        c += NT - j;
      }
    return -1;
  }
  static constexpr int I_of(int i) {
    for (int j = 0; j < NT; ++j)
      if ((SM >> j) & 1u) {
        if (i < NT - j) return j + i;
        i -= NT - j;
      }
    return -1;
  }
  static constexpr int J_of(int i) {
    for (int j = 0; j < NT; ++j)
      if ((SM >> j) & 1u) {
        if (i < NT - j) return j;
        i -= NT - j;
      }
    return -1;
  }
  static constexpr int strip_ordinal(int J) {  // strips of this wave before J
    int c = 0;
    for (int j = 0; j < J; ++j) c += (SM >> j) & 1u;
    return c;
  }
};

__device__ __forceinline__ void barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

// v_perm_b32: byte s of the result = byte sel_s of {a (bytes 4-7), b (0-3)}
__device__ __forceinline__ uint32_t perm(uint32_t a, uint32_t b, uint32_t sel) {
  return __builtin_amdgcn_perm(a, b, sel);
}
template <int CTRL>
__device__ __forceinline__ uint32_t dpp(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, CTRL, 0xF, 0xF, false);
}
// 4x4 byte transpose across a DPP quad: lane j of the quad ends with byte j
// of the four lanes' v (lane order = byte order).  sel1 / sel2: the lane's
// v_perm selectors (by lane & 1, lane & 2).
__device__ __forceinline__ uint32_t quad_transpose(uint32_t v, uint32_t sel1, uint32_t sel2) {
  const uint32_t s1 = perm(dpp<0xB1>(v), v, sel1);  // quad_perm [1,0,3,2]: swap with lane ^ 1
  return perm(dpp<0x4E>(s1), s1, sel2);             // quad_perm [2,3,0,1]: swap with lane ^ 2
}

// sum_k 2^(-8k) L_k of one accumulator element
__device__ __forceinline__ double level_value(const oz_i4 (&L)[NL], int r) {
  double v = (double)L[NL - 1][r];
#pragma unroll
  for (int k = NL - 2; k >= 0; --k) v = fma(v, 0x1p-8, (double)L[k][r]);
  return v;
}

// Upper bound of |x| from a recorded max |x| high dword (low dword all ones).
__device__ __forceinline__ double xbound(uint32_t hi) {
  return __hiloint2double((int)(hi & 0x7FFFFFFFu), (int)0xFFFFFFFFu);
}
// Digit exponent E (bound < 2^E) of a feature of a chunk.  xhi: recorded max
// |x| high dword; logistic: zbits = recorded max |z| (fp32 bits, z32 =
// fl32(fl32(x) sqrtf(fl32(w))), within 5 fp32 ulp of z wherever |z| >= 2^-120
// and w is an fp32 normal), growth = exp(dB / 2) >= the factor sqrt(w) can
// have grown by since the record.  Rows the fp32 record cannot see have
// |z| < 2^-120 or sqrt(w) < 2^-60 (w below the fp32 normals), hence the two
// floors; and sqrt(w) <= 1/2 always.  Gaussian: z = x.
__device__ __forceinline__ int digit_exponent(uint32_t xhi, uint32_t zbits, double growth,
                                              int fam_logistic) {
  const double xb = xbound(xhi);
  double bound = xb;
  if (fam_logistic) {
    const double zb = (double)__uint_as_float(zbits & 0x7FFFFFFFu) * (1.0 + 0x1p-16);
    bound = fmax(fmax(zb, 0x1p-120), xb * 0x1p-60) * growth;
    bound = fmin(bound, 0.5 * xb);  // (also when growth overflowed to inf)
  }
  const int e = __builtin_amdgcn_frexp_exp(bound);
  return max(e, EMIN);  // above EMAX: the caller fails the chunk (digit_overflow)
}
// |z| >= 2^EMAX: the digits of F = round(z 2^(38 - E)) would wrap at the
// clamped exponent (a finite, wrong Hessian), so such a chunk publishes a NaN
// log-likelihood instead -- the partition then fails as nonfinite, as the
// fp64 Gram's inf would make it
__device__ __forceinline__ bool digit_overflow(int e) { return e > EMAX; }

}  // namespace ozk

// Profiling build (DLSA_OZ_PROF, tools/build_variants.sh ozprof): per-wave
// cycle stamps (s_memtime) of the iteration's phases, summed over the chunk
// and added to g_oz_prof[slot] at its end (one vector atomic per wave).
#ifdef DLSA_OZ_PROF
static __device__ unsigned long long g_oz_prof[32];  // per translation unit: [4 wid + i]
static inline int oz_prof_read_impl(unsigned long long* out) {
  if (hipDeviceSynchronize() != hipSuccess) return -1;
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_oz_prof), 32 * 8) != hipSuccess) return -1;
  unsigned long long z[32] = {0};
  return hipMemcpyToSymbol(HIP_SYMBOL(g_oz_prof), z, 32 * 8) == hipSuccess ? 0 : -1;
}
#define OZ_STAMP(v) const uint64_t v = __builtin_readcyclecounter()
#define OZ_STAMP_VAR(v) uint64_t v = 0
#define OZ_STAMP_SET(v) v = __builtin_readcyclecounter()
#define OZ_ADD(i, d) prof[i] += (d)
#define OZ_DECL uint64_t prof[4] = {0, 0, 0, 0}
#define OZ_FLUSH(base)                                                        \
  if (lane == 0)                                                              \
    for (int i_ = 0; i_ < 4; ++i_) atomicAdd(&g_oz_prof[(base) + i_], prof[i_])
#else
#define OZ_STAMP(v)
#define OZ_STAMP_VAR(v)
#define OZ_STAMP_SET(v)
#define OZ_ADD(i, d)
#define OZ_DECL
#define OZ_FLUSH(base)
#endif

#if DLSA_OZ_MAGICF
#define OZ_DIGIT_T(x, s, m) fma(x, s, mg[m])
#else
#define OZ_DIGIT_T(x, s, m) fma(x, __builtin_amdgcn_ldexp(s, esc[m]), MAGIC)
#endif

// ---- consumer waves: tiles of X^T W X -------------------------------------
template <int NT, int CW>
struct OzConsumer {
  using TL = ozk::Tiles<NT, CW>;
  static constexpr int TW = TL::TW;
  static constexpr int PMAX = 16 * NT;
  static constexpr int NB = ozk::NL > 5 ? 6 : 5;  // B quads
  // Edge folding (DLSA_OZ_EDGE): the last tile row I = NT - 1 holds only
  // se = P - 16 (NT - 1) features.  When se <= 5 its 16 A rows carry three
  // groups of se rows -- group g = the digit pair (2g, 2g+1) of the se edge
  // features -- so one MFMA against B quad b adds level 2g + b to group g:
  // 5 MFMAs per edge tile and block (b = 0..4) instead of 9, and the store
  // sums L_k = acc_k[e] + acc_{k-2}[se + e] + acc_{k-4}[2 se + e], the same
  // integers the unfolded tile accumulates (bit-identical Sig_inv).
  static constexpr bool kEdge = DLSA_OZ_EDGE && ozk::ND == 5 && ozk::NL == 5;
  static constexpr int kEdgeTiles = [] {
    int c = 0;
    for (int t = 0; t < TW; ++t) c += TL::I_of(t) == NT - 1;
    return c;
  }();
  oz_i4 acc[TW > 0 ? TW : 1][ozk::NL];
  bool fold = false;    // se <= 5 (wave-uniform)
  int se = 16;          // features of the last tile row
  int e_off = 0;        // this lane's edge A operand: byte offset of (feature, pair)
  uint32_t m_lo = 0, m_hi = 0;  // its masks: group < 3, group < 2

  __device__ __forceinline__ void init(int P, int lane) {
    wv_static_for<(TW > 0 ? TW : 1)>([&](auto iI) {
      constexpr int i = decltype(iI)::value;
#pragma unroll
      for (int k = 0; k < ozk::NL; ++k) acc[i][k] = oz_i4{0, 0, 0, 0};
    });
    se = P - 16 * (NT - 1);
    fold = kEdge && kEdgeTiles > 0 && se <= 5;
    if (fold) {
      const int i = lane & 15, grp = i / se, e = i - grp * se;
      e_off = (16 * (NT - 1) + e) * ozk::kFeatBytes + 16 * (grp < 3 ? grp : 0);
      m_lo = grp < 3 ? 0xFFFFFFFFu : 0u;
      m_hi = grp < 2 ? 0xFFFFFFFFu : 0u;  // group 2: (d4, 0)
    }
  }

  // the image of one 32-row block whose x started at xs (LDS); tick() is
  // called after every tile's MFMAs (the DMA of the next blocks rides along).
  // Software-pipelined: the operands of tile t+1 (and of the next strip) are
  // read while the MFMAs of tile t issue.
  template <typename Tick>
  __device__ __forceinline__ void consume(const char* xs, int p, int lane, Tick&& tick) {
    consume_quads(xs, p, lane, tick);
  }

  template <typename Tick>
  __device__ __forceinline__ void consume_quads(const char* xs, int p, int lane, Tick&& tick) {
    if constexpr (TW > 0) {
      const int i = lane & 15, g = lane >> 4;
      // lane group g: the image of producer wave g (its 8 rows of the block)
      const char* im = xs + g * ozk::RPW * p * 8 + i * ozk::kFeatBytes;
      using u2 = unsigned __attribute__((ext_vector_type(2)));
      oz_i4 A0[2], A2[2];
      u2 A4[2];
      u2 Bd[2][ozk::ND];
      auto loadB = [&](auto jJ, int u) {
        constexpr int fo = 16 * decltype(jJ)::value * ozk::kFeatBytes;
#pragma unroll
        for (int b = 0; b < ozk::ND; ++b) Bd[u][b] = *(const u2*)(im + fo + 8 * b);
      };
      auto loadA = [&](auto tI, int u) {
        constexpr int fa = 16 * TL::I_of(decltype(tI)::value) * ozk::kFeatBytes;
        // A quad a: digits (a, a+1) of the feature -- one 16-byte read
        A0[u] = *(const oz_i4*)(im + fa);
        A2[u] = *(const oz_i4*)(im + fa + 16);
        if constexpr (ozk::ND == 5) A4[u] = *(const u2*)(im + fa + 32);
      };
      // the folded edge operand (one 16-byte read per block, all strips)
      oz_i4 Ae = oz_i4{0, 0, 0, 0};
      if constexpr (kEdge && kEdgeTiles > 0) {
        if (fold) {
          const oz_i4 q = *(const oz_i4*)(xs + g * ozk::RPW * p * 8 + e_off);
          Ae = oz_i4{(int)(q.x & m_lo), (int)(q.y & m_lo), (int)(q.z & m_hi), (int)(q.w & m_hi)};
        }
      }
      loadB(std::integral_constant<int, TL::J_of(0)>{}, 0);
      loadA(std::integral_constant<int, 0>{}, 0);
      wv_static_for<TW>([&](auto tI) {
        constexpr int t = decltype(tI)::value;
        constexpr int J = TL::J_of(t);
        constexpr int ua = t & 1;
        constexpr int ub = TL::strip_ordinal(J) & 1;
        constexpr bool edge = kEdge && TL::I_of(t) == NT - 1;
        if constexpr (t + 1 < TW) {
          constexpr int Jn = TL::J_of(t + 1);
          if constexpr (Jn != J) loadB(std::integral_constant<int, Jn>{}, ub ^ 1);
          if constexpr (kEdge && TL::I_of(t + 1) == NT - 1) {
            if (!fold) loadA(std::integral_constant<int, t + 1>{}, ua ^ 1);
          } else {
            loadA(std::integral_constant<int, t + 1>{}, ua ^ 1);
          }
        }
        __builtin_amdgcn_sched_barrier(0);
        // B quad b: bytes 0-7 digit b, bytes 8-15 digit b - 1 (zero for b = 0)
        const u2* d = Bd[ub];
        oz_i4 Bq[NB];
        Bq[0] = oz_i4{(int)d[0].x, (int)d[0].y, 0, 0};
#pragma unroll
        for (int b = 1; b < ozk::ND; ++b)
          Bq[b] = oz_i4{(int)d[b].x, (int)d[b].y, (int)d[b - 1].x, (int)d[b - 1].y};
        if constexpr (NB > 5) Bq[5] = oz_i4{0, 0, (int)d[4].x, (int)d[4].y};
        if constexpr (edge) {
          if (fold) {  // wave-uniform
#pragma unroll
            for (int b = 0; b < 5; ++b)
              acc[t][b] = __builtin_amdgcn_mfma_i32_16x16x64_i8(Ae, Bq[b], acc[t][b], 0, 0, 0);
            __builtin_amdgcn_sched_barrier(0);
            tick(std::integral_constant<int, t>{});
            return;
          }
        }
        const oz_i4 a0 = A0[ua], a2 = A2[ua];
        if constexpr (ozk::ND == 4) {  // levels 0-4: 8 MFMAs (level 4: (1,3) (2,2) (3,1))
          const oz_i4 b4 = oz_i4{0, 0, (int)d[3].x, (int)d[3].y};
          acc[t][0] = __builtin_amdgcn_mfma_i32_16x16x64_i8(a0, Bq[0], acc[t][0], 0, 0, 0);
          acc[t][1] = __builtin_amdgcn_mfma_i32_16x16x64_i8(a0, Bq[1], acc[t][1], 0, 0, 0);
          acc[t][2] = __builtin_amdgcn_mfma_i32_16x16x64_i8(a0, Bq[2], acc[t][2], 0, 0, 0);
          acc[t][3] = __builtin_amdgcn_mfma_i32_16x16x64_i8(a0, Bq[3], acc[t][3], 0, 0, 0);
          acc[t][4] = __builtin_amdgcn_mfma_i32_16x16x64_i8(a0, b4, acc[t][4], 0, 0, 0);
          acc[t][2] = __builtin_amdgcn_mfma_i32_16x16x64_i8(a2, Bq[0], acc[t][2], 0, 0, 0);
          acc[t][3] = __builtin_amdgcn_mfma_i32_16x16x64_i8(a2, Bq[1], acc[t][3], 0, 0, 0);
          acc[t][4] = __builtin_amdgcn_mfma_i32_16x16x64_i8(a2, Bq[2], acc[t][4], 0, 0, 0);
          __builtin_amdgcn_sched_barrier(0);
          tick(std::integral_constant<int, t>{});
          return;
        }
        const oz_i4 a4 = oz_i4{(int)A4[ua].x, (int)A4[ua].y, 0, 0};  // digit 5 = 0
        acc[t][0] = __builtin_amdgcn_mfma_i32_16x16x64_i8(a0, Bq[0], acc[t][0], 0, 0, 0);
        acc[t][1] = __builtin_amdgcn_mfma_i32_16x16x64_i8(a0, Bq[1], acc[t][1], 0, 0, 0);
        acc[t][2] = __builtin_amdgcn_mfma_i32_16x16x64_i8(a0, Bq[2], acc[t][2], 0, 0, 0);
        acc[t][3] = __builtin_amdgcn_mfma_i32_16x16x64_i8(a0, Bq[3], acc[t][3], 0, 0, 0);
        if constexpr (ozk::ND == 5) {
          acc[t][4] = __builtin_amdgcn_mfma_i32_16x16x64_i8(a0, Bq[4], acc[t][4], 0, 0, 0);
          acc[t][2] = __builtin_amdgcn_mfma_i32_16x16x64_i8(a2, Bq[0], acc[t][2], 0, 0, 0);
          acc[t][3] = __builtin_amdgcn_mfma_i32_16x16x64_i8(a2, Bq[1], acc[t][3], 0, 0, 0);
          acc[t][4] = __builtin_amdgcn_mfma_i32_16x16x64_i8(a2, Bq[2], acc[t][4], 0, 0, 0);
          acc[t][4] = __builtin_amdgcn_mfma_i32_16x16x64_i8(a4, Bq[0], acc[t][4], 0, 0, 0);
        }
        if constexpr (ozk::NL > 5) {  // level 5: (1,4) (2,3) (3,2) (4,1)
          acc[t][5] = __builtin_amdgcn_mfma_i32_16x16x64_i8(a0, Bq[NB - 1], acc[t][5], 0, 0, 0);
          acc[t][5] = __builtin_amdgcn_mfma_i32_16x16x64_i8(a2, Bq[3], acc[t][5], 0, 0, 0);
          acc[t][5] = __builtin_amdgcn_mfma_i32_16x16x64_i8(a4, Bq[1], acc[t][5], 0, 0, 0);
        }
        if constexpr (ozk::NL > 6) {  // level 6: (2,4) (3,3) (4,2)
          acc[t][6] = __builtin_amdgcn_mfma_i32_16x16x64_i8(a2, Bq[4], acc[t][6], 0, 0, 0);
          acc[t][6] = __builtin_amdgcn_mfma_i32_16x16x64_i8(a4, Bq[2], acc[t][6], 0, 0, 0);
        }
        __builtin_amdgcn_sched_barrier(0);
        tick(std::integral_constant<int, t>{});
      });
      // keep the level accumulators in registers across the loop
      wv_static_for<TW>([this](auto iI) {
        constexpr int t = decltype(iI)::value;
#pragma unroll
        for (int k = 0; k < ozk::NL; ++k) asm volatile("" : "+v"(acc[t][k]));
      });
    }
  }

  // H tiles into the chunk's slab (newton_solve.hip layout), scaled back.
  // scratch: this wave's LDS for the folded edge tiles (5 x 16 x 16 int32 each)
  __device__ __forceinline__ void store(double* sH, const int* ex, int lane, int* scratch) {
    if constexpr (TW > 0) {
      const int fl = lane & 15, q = lane >> 4;
      wv_static_for<TW>([&](auto iI) {
        constexpr int t = decltype(iI)::value;
        constexpr int I = TL::I_of(t), J = TL::J_of(t);
        constexpr int ts = I * (I + 1) / 2 + J;
        if constexpr (kEdge && I == NT - 1) {
          if (fold) {
            // acc[t][b] at C row R = 4 q + r, col fl -> S[b][R][fl]
#pragma unroll
            for (int b = 0; b < 5; ++b)
#pragma unroll
              for (int r = 0; r < 4; ++r) scratch[(b * 16 + 4 * q + r) * 16 + fl] = acc[t][b][r];
            const int ej = ex[16 * J + fl];
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const int row = 4 * q + r;
              double v = 0.0;  // rows past the last feature (f >= P): never read
              if (row < se) {
                oz_i4 L[1][5];
                int lv[5];
#pragma unroll
                for (int k = 0; k < 5; ++k) {
                  int x = scratch[(k * 16 + row) * 16 + fl];
                  if (k >= 2) x += scratch[((k - 2) * 16 + se + row) * 16 + fl];
                  if (k >= 4) x += scratch[((k - 4) * 16 + 2 * se + row) * 16 + fl];
                  lv[k] = x;
                }
#pragma unroll
                for (int k = 0; k < 5; ++k) L[0][k] = oz_i4{lv[k], 0, 0, 0};
                v = __builtin_amdgcn_ldexp(ozk::level_value(L[0], 0),
                                           ej + ex[16 * I + row] - 12);
              }
              sH[ts * 256 + row * 16 + fl] = v;
            }
            scratch += 5 * 256;
            return;
          }
        }
        const int ej = ex[16 * J + fl];
#pragma unroll
        for (int r = 0; r < 4; ++r) {  // i32 16x16 C/D map: row 4 (l >> 4) + r, col l & 15
          const int row = 4 * q + r;
          const double v = ozk::level_value(acc[t], r);
          sH[ts * 256 + row * 16 + fl] = __builtin_amdgcn_ldexp(v, ej + ex[16 * I + row] - 12);
        }
      });
    }
  }
};

// ---- producer waves, row quads in lanes (DLSA_OZ_R4) ------------------------
// Lane (q, s) = (lane >> 4, lane & 15) holds 4 rows of features 16 k + s,
// k = 0 .. NT-1: rows 4 (q & 1) .. 4 (q & 1) + 3 of this wave's 8 rows of
// block 2m + (q >> 1).  With the 4 rows of a feature in one lane, a digit
// plane of 4 rows is a byte transpose of the lane's own words (8 v_perm for
// the four low-dword planes, 3 for the top digit) instead of DPP quad
// exchanges across lanes (4 VALU per word), the x reads of a wave row are 16
// consecutive doubles (no bank conflicts), and theta, the gradient partials
// and the digit constants take NT registers pairs per lane instead of 2 NT.
// eta of the 4 rows: 4 FMA chains over the lane's NT features, then a
// reduce-scatter over the 16 lanes of the feature slots (DPP row_ror:8,
// row_half_mirror, 2 quad_perm) leaves lane s with row s >> 2; one
// transcendental chain for the 16 rows of the wave (4 replicas per row);
// row_newbcast brings each row's sqrt(w) and residual back to the 16 lanes.
// Same image layout, ownership rule and epilogue as the quad-transpose
// producers below.
template <int CTRL>
__device__ __forceinline__ double dpp_f64(double v) {
  const int lo = __builtin_amdgcn_mov_dpp(__double2loint(v), CTRL, 0xF, 0xF, false);
  const int hi = __builtin_amdgcn_mov_dpp(__double2hiint(v), CTRL, 0xF, 0xF, false);
  return __hiloint2double(hi, lo);
}

template <int NT, bool STD, int FAM, typename SlotX, typename Dma>
__device__ __forceinline__ void oz_producer_r4(const PassArgs& a, char* smem, int wid, int lane,
                                               int tid, int nb, int nit, int sbytes,
                                               int xs_bytes, SlotX&& slot_x, const double* bet,
                                               const double* stdv, const int* ex, int chunk,
                                               bool chunk_ovf, Dma&& issue_pair) {
  using namespace ozk;
  static_assert(ND == 5 && DLSA_OZ_MAGICF, "row-quad producers: 5 digits, magic constants");
  constexpr int PMAX = 16 * NT;
  const int p = a.p, P = a.P, ic = a.intercept;
  const int nrows = __builtin_amdgcn_readfirstlane(a.chunk_rows[blockIdx.x]);
  const int pw = wid;
  const int q = lane >> 4, s = lane & 15;
  const int Xq = q >> 1, hq = q & 1;
  const int rbase = pw * RPW + 4 * hq;  // block row of this lane's row 0
  const bool up8 = s >= 8, up4 = ((s >> 2) & 1) != 0;
  const int myrow = s >> 2;             // the row whose eta this lane ends with
  double beta[NT], gacc[NT], mg[NT];
#pragma unroll
  for (int k = 0; k < NT; ++k) {
    const int f = 16 * k + s;
    beta[k] = bet[f];
    mg[k] = __builtin_amdgcn_ldexp(MAGIC, ex[f] - GBITS);
    gacc[k] = 0.0;
  }
  const bool fin_last = 16 * (NT - 1) + s < P;  // the last tile's feature is < P
  double llacc = 0.0, lprod = 1.0;

  // producer-issued DMA (DLSA_OZ_SCHED 3: right after the barrier, 4: after
  // the row phase, 5: after the digits); each wave waits for its own pieces
  // before the next barrier, which then publishes all of them
  // (DLSA_OZ_PDMA > 0 with a consumer schedule: the producers' share of the
  // pieces, at the iteration start as in 3)
  constexpr int kSched = DLSA_OZ_SCHED >= 3 ? DLSA_OZ_SCHED : (DLSA_OZ_PDMA > 0 ? 3 : 0);
  if constexpr (kSched >= 3) {
    issue_pair(-1);
    wv_wait_vmcnt<0>();
  }
  OZ_DECL;
  for (int m = 0; m < nit; ++m) {
    OZ_STAMP(t0);
    if constexpr (kSched >= 3) wv_wait_vmcnt<0>();
    barrier();  // B_m
    OZ_STAMP(t1);
    OZ_ADD(0, t1 - t0);
    if constexpr (kSched == 3) issue_pair(m);
    if (2 * m >= nb || (DLSA_OZ_ABLATE & 1)) {  // the last iteration only consumes
      if constexpr (kSched >= 4) issue_pair(m);
      continue;
    }
    const int b = 2 * m + Xq;
    char* xq = slot_x(b);
    const double* yq = (const double*)(smem + (b % NSLOT) * sbytes + 16 + xs_bytes);
    const int leftq = nrows - b * RB;
    // workgroup-uniform: both blocks full
    const bool full = nrows - 2 * m * RB >= 2 * RB;
    double v[4][NT], e[4];
    auto row_phase = [&](auto maskI) {
      constexpr bool MASK = decltype(maskI)::value;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int rowB = rbase + r;
        const bool valid = rowB < leftq;
        const double* xr = (const double*)xq + rowB * p + (s - ic);
        double er = 0.0;
#pragma unroll
        for (int k = 0; k < NT; ++k) {
          const int f = 16 * k + s;
          double x = xr[16 * k];
          if constexpr (DLSA_OZ_CHECK) {  // ownership rule: own rows for f < P
            const int el = rowB * p + f - ic;
            if (f >= ic && f < P && (el < pw * RPW * p || el >= (pw + 1) * RPW * p))
              x = __builtin_nan("");
          }
          if constexpr (STD) x = (x - stdv[f]) * stdv[PMAX + f];
          if (k == 0 && ic && s == 0) x = 1.0;
          const bool fin = k < NT - 1 || fin_last;  // padding features f >= P: 0
          if constexpr (MASK)
            x = (valid && fin) ? x : 0.0;
          else
            x = fin ? x : 0.0;
          v[r][k] = x;
          er = fma(x, beta[k], er);
        }
        e[r] = er;
      }
    };
    if (full)
      row_phase(std::false_type{});
    else
      row_phase(std::true_type{});
    // reduce-scatter of the 4 row sums over the 16 feature slots
    double e01, e23;
    {
      const double s0 = up8 ? e[0] : e[2], s1 = up8 ? e[1] : e[3];  // the partner's rows
      const double k0 = up8 ? e[2] : e[0], k1 = up8 ? e[3] : e[1];  // kept
      e01 = k0 + dpp_f64<0x128>(s0);  // row_ror:8 = lane s ^ 8
      e23 = k1 + dpp_f64<0x128>(s1);
    }
    double eh;
    {
      const double sn = up4 ? e01 : e23, kp = up4 ? e23 : e01;
      eh = kp + dpp_f64<0x141>(sn);  // row_half_mirror: bit 2 of s flipped
    }
    eh += dpp_f64<0xB1>(eh);  // quad_perm [1,0,3,2]
    eh += dpp_f64<0x4E>(eh);  // quad_perm [2,3,0,1]
    // one transcendental chain for the wave's 16 rows (row rbase + myrow)
    double swh, rh;
    {
      const bool valid = rbase + myrow < leftq;
      const double yv = valid ? yq[rbase + myrow] : 0.0;
      if constexpr (FAM == FAMILY_LOGISTIC) {
        const double eqv = exp(-0.5 * fabs(eh));
        const double ea = eqv * eqv;
        const double inv = wv_rcp(1.0 + ea);
        const double mu = eh >= 0.0 ? inv : ea * inv;
        swh = eqv * inv;
        rh = yv - mu;
        if (valid && (s & 3) == 0) {
          llacc += yv * eh - fmax(eh, 0.0);
          lprod *= 1.0 + ea;
        }
      } else {  // gaussian (OLS): mu = eta, w = 1, ll = -rss / 2
        swh = 1.0;
        rh = yv - eh;
        if (valid && (s & 3) == 0) llacc -= 0.5 * rh * rh;
      }
      if (!valid) {
        swh = 0.0;
        rh = 0.0;
      }
    }
    double sw[4], res[4];
    sw[0] = dpp_f64<0x150>(swh);  // row_newbcast:4r -- row r's values to the 16 lanes
    sw[1] = dpp_f64<0x154>(swh);
    sw[2] = dpp_f64<0x158>(swh);
    sw[3] = dpp_f64<0x15C>(swh);
    res[0] = dpp_f64<0x150>(rh);
    res[1] = dpp_f64<0x154>(rh);
    res[2] = dpp_f64<0x158>(rh);
    res[3] = dpp_f64<0x15C>(rh);
    if constexpr (kSched == 4) issue_pair(m);
    OZ_STAMP(t2);
    OZ_ADD(1, t2 - t1);
    // ---- gradient and the digit image of the 4 rows ---------------------------
    char* img = xq + pw * RPW * p * 8 + 4 * hq;
#pragma unroll
    for (int k = 0; k < NT; ++k) {
      gacc[k] = fma(v[0][k], res[0], gacc[k]);
      gacc[k] = fma(v[1][k], res[1], gacc[k]);
      gacc[k] = fma(v[2][k], res[2], gacc[k]);
      gacc[k] = fma(v[3][k], res[3], gacc[k]);
      uint32_t lo[4], hi[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const double t = fma(v[r][k], sw[r], mg[k]);
        lo[r] = __double2loint(t);
        hi[r] = __double2hiint(t);
      }
      // byte j of lo = digit 4 - j; byte 0 of hi = digit 0 (row order = byte order)
      const uint32_t u01 = perm(lo[1], lo[0], 0x05010400u), w01 = perm(lo[1], lo[0], 0x07030602u);
      const uint32_t u23 = perm(lo[3], lo[2], 0x05010400u), w23 = perm(lo[3], lo[2], 0x07030602u);
      const uint32_t d4 = perm(u23, u01, 0x05040100u) ^ 0x80808080u;
      const uint32_t d3 = perm(u23, u01, 0x07060302u) ^ 0x80808080u;
      const uint32_t d2 = perm(w23, w01, 0x05040100u) ^ 0x80808080u;
      const uint32_t d1 = perm(w23, w01, 0x07060302u) ^ 0x80808080u;
      const uint32_t d0 = perm(perm(hi[3], hi[2], 0x05010400u), perm(hi[1], hi[0], 0x05010400u),
                               0x05040100u) ^ 0x80808080u;
      char* fe = img + (16 * k + s) * kFeatBytes;
      *(uint32_t*)(fe + plane_off(0)) = d0;
      *(uint32_t*)(fe + plane_off(1)) = d1;
      *(uint32_t*)(fe + plane_off(2)) = d2;
      *(uint32_t*)(fe + plane_off(3)) = d3;
      *(uint32_t*)(fe + plane_off(4)) = d4;
    }
    if constexpr (kSched == 5) issue_pair(m);
#ifdef DLSA_OZ_PROF
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#endif
    OZ_STAMP(t3);
    OZ_ADD(2, t3 - t2);
  }
  OZ_FLUSH(4 * pw);
  __syncthreads();  // S1 (the consumers' S1): the ring is free

  // ---- epilogue: gradient and log-likelihood partials --------------------------
  double* red = (double*)smem;  // the ring: [NPW][PMAX + 1]
#pragma unroll
  for (int k = 0; k < NT; ++k) {
    double g = gacc[k];
    g += __shfl_xor(g, 16);
    g += __shfl_xor(g, 32);
    if (q == 0) red[pw * (PMAX + 1) + 16 * k + s] = g;
  }
  if constexpr (FAM == FAMILY_LOGISTIC) llacc -= log(lprod);
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) llacc += __shfl_xor(llacc, o);
  if (lane == 0) red[pw * (PMAX + 1) + PMAX] = llacc;
  __syncthreads();  // S2
  for (int f = tid; f < PMAX; f += 64 * NPW) {
    double sg = 0.0;
#pragma unroll
    for (int w = 0; w < NPW; ++w) sg += red[w * (PMAX + 1) + f];
    a.slab_g[(int64_t)chunk * PMAX + f] = sg;
  }
  if (tid == 0) {
    double sg = 0.0;
#pragma unroll
    for (int w = 0; w < NPW; ++w) sg += red[w * (PMAX + 1) + PMAX];
    // a digit exponent past EMAX (clamped in ex[]) would publish wrapped
    // digits: the chunk's NaN log-likelihood fails its partition visibly
    // (chunk_ovf is wave 0's ballot; tid 0 is in wave 0)
    a.slab_ll[chunk] = chunk_ovf ? __builtin_nan("") : sg;
  }
}

template <int NT, bool STD, int FAM>
__global__ __launch_bounds__(64 * (ozk::NPW + ozk::NCW), 1) void irls_oz_kernel(const PassArgs a) {
  using namespace ozk;
  constexpr int PMAX = 16 * NT;
  constexpr int M = PMAX / LPR;  // row-phase features per lane
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
  const int nit = (nb + 1) / 2 + 1;  // iterations (the last only consumes)
  const int sbytes = slot_bytes(p);
  const int np = npieces(p);
  const int xs_bytes = xspan(p);
  double* bet = (double*)(smem + NSLOT * sbytes);  // [PMAX] theta of the partition
  double* stdv = bet + PMAX;                        // [2][PMAX] center, 1/scale
  int* ex = (int*)(stdv + 2 * PMAX);                // [PMAX] digit exponents E_f

  // digit scales: |theta - theta_rec|_1 and the chunk's max |x| over all
  // features (PMAX <= 112 < the 512 threads: one feature per thread), reduced
  // in a fixed order, so every thread forms the same growth factor
  double dth = 0.0;
  uint32_t xh = 0;
  bool e_ovf = false;
  if (tid < PMAX) {
    const double th = (tid < P) ? a.theta[(int64_t)part * P + tid] : 0.0;
    bet[tid] = th;
    if (tid < P) dth = fabs(th - a.theta_rec[(int64_t)part * P + tid]);
    xh = a.colmax[(int64_t)chunk * PMAX + tid] & 0x7FFFFFFFu;
    if constexpr (STD) {
      const int j = tid - ic;
      const bool in = j >= 0 && j < p;
      stdv[tid] = in ? a.center[j] : 0.0;
      stdv[PMAX + tid] = in ? 1.0 / a.scale[j] : 1.0;
    }
  }
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    dth += __shfl_xor(dth, o);
    xh = max(xh, (uint32_t)__shfl_xor((int)xh, o));
  }
  double* dred = (double*)smem;  // the ring's first bytes, before any DMA
  uint32_t* xred = (uint32_t*)(dred + (NPW + NCW));
  if (lane == 0) {
    dred[wid] = dth;
    xred[wid] = xh;
  }
  __syncthreads();
  if (tid < PMAX) {
    double sd = 0.0;
    uint32_t xm = 0;
#pragma unroll
    for (int w = 0; w < NPW + NCW; ++w) {
      sd += dred[w];
      xm = max(xm, xred[w]);
    }
    const double growth = exp(0.5 * sd * ozk::xbound(xm)) * (1.0 + 0x1p-40);
    const int e = digit_exponent(a.colmax[(int64_t)chunk * PMAX + tid],
                                 a.zcolmax[(int64_t)chunk * PMAX + tid], growth,
                                 FAM == FAMILY_LOGISTIC);
    ex[tid] = min(e, ozk::EMAX);
    if (wid == 0) {  // wave 0 (whose tid 0 publishes slab_ll) also checks wave 1's features
      e_ovf = ozk::digit_overflow(e);
      if (tid + 64 < PMAX)
        e_ovf = e_ovf || ozk::digit_overflow(digit_exponent(
                             a.colmax[(int64_t)chunk * PMAX + tid + 64],
                             a.zcolmax[(int64_t)chunk * PMAX + tid + 64], growth,
                             FAM == FAMILY_LOGISTIC));
    }
  }
  // (no __syncthreads_or: its __shared__ word would push the LDS past 160 KB)
  const bool chunk_ovf = wid == 0 && __ballot(e_ovf) != 0;
  // (the ring needs no zeroing: past-the-chunk rows are zeroed in registers
  // and nothing reads a slot's bytes that the DMA did not write)
  __syncthreads();

  auto slot_x = [&](int blk) -> char* {
    const uintptr_t start = (uintptr_t)(a.X + (row0 + (int64_t)blk * RB) * p);
    return smem + (blk % NSLOT) * sbytes + 16 + (start & 15);
  };

  // ---- LDS-DMA of the X / y blocks --------------------------------------------
  // Issued by the consumer waves (DLSA_OZ_SCHED 0-2) or by the producer waves
  // (3-5); dw = the issuing wave's index among its four.  Wave dw's pieces of
  // a block: X pieces dw, dw + 4, ... and (dw = 3) the block's y.  Scalar
  // bases per block; piece i (a compile-time index) is two scalar adds and the
  // DMA.  The last piece either runs with only the lanes inside the block
  // (consumer schedules) or is the block's final 1 KiB, overlapping the piece
  // before it with the same bytes (producer schedules: whole-wave, no lane
  // predicate -- the predicated form fails instruction selection in hipcc 7.2
  // in the producers' scope).
  constexpr bool kProdDma = DLSA_OZ_SCHED >= 3;
  static_assert(!kProdDma || DLSA_OZ_R4, "producer-issued DMA: row-quad producers");
  // DLSA_OZ_PDMA = KP > 0 with a consumer schedule: the producers issue each
  // block's pieces i < KP (their own DMA share) at the iteration start, the
  // consumers the rest -- the DMA issue cost split between the two wave types
  constexpr int KP = kProdDma ? kMaxPiecesPerWave : DLSA_OZ_PDMA;
  static_assert(KP == 0 || DLSA_OZ_R4, "producer-issued DMA: row-quad producers");
  constexpr bool kOvl = kProdDma || DLSA_OZ_OVL || KP > 0;
  const int dw = wid >= NPW ? wid - NPW : wid;
  const uintptr_t xcb = (uintptr_t)(a.X + row0 * p) & ~(uintptr_t)15;
  const __amdgpu_buffer_rsrc_t xr = wv_rsrc(xcb, a.x_last16 + 16 - xcb);
  const uintptr_t ycb = (uintptr_t)(a.y + row0);
  const __amdgpu_buffer_rsrc_t yr = wv_rsrc(ycb, a.y_last4 + 4 - ycb);
  const int npw = (np - dw + NCW - 1) / NCW;
  const int last_rem = xs_bytes - (np - 1) * 1024;  // bytes of the last piece
  // a block's slot LDS offset and the buffer offset of its 16-B-aligned start
  auto blk_lds = [&](int blk) { return __builtin_amdgcn_readfirstlane((blk % NSLOT) * sbytes); };
  auto blk_soff = [&](int blk) {
    const uintptr_t start = (uintptr_t)(a.X + (row0 + (int64_t)blk * RB) * p);
    return __builtin_amdgcn_readfirstlane((int)((start & ~(uintptr_t)15) - xcb));
  };
  auto issue_x = [&](auto iI, int lds, int soff) {
    constexpr int i = decltype(iI)::value;
    if (i < npw) {  // uniform
      const int j = dw + NCW * i;
      if constexpr (kOvl) {
        const int off = j == np - 1 ? xs_bytes - 1024 : j * 1024;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(xr, (wlds_void_t*)(smem + lds + 16 + off), 16,
                                                 lane * 16, soff + off, 0, DLSA_OZ_DMA_AUX);
      } else if (j != np - 1 || lane * 16 < last_rem) {
        __builtin_amdgcn_raw_ptr_buffer_load_lds(xr, (wlds_void_t*)(smem + lds + 16 + j * 1024),
                                                 16, lane * 16, soff + j * 1024, 0,
                                                 DLSA_OZ_DMA_AUX);
      }
    }
  };
  auto issue_y = [&](int blk, int lds) {
    if (dw == NCW - 1)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(yr, (wlds_void_t*)(smem + lds + 16 + xs_bytes), 4,
                                               lane * 4, blk * RB * 8, 0, 0);
  };
  // all of a block's pieces from piece I0 on
  auto issue_rest = [&](auto I0, int blk, int lds, int soff) {
    wv_static_for<kMaxPiecesPerWave>([&](auto iI) {
      if constexpr (decltype(iI)::value >= decltype(I0)::value) issue_x(iI, lds, soff);
    });
    issue_y(blk, lds);
  };
  // producer schedules: blocks 2m+2, 2m+3 (into the slots of 2m-4, 2m-3, free
  // since B_m), or blocks 0, 1 before the loop (m = -1)
  // (all pieces + y with kProdDma, else the pieces i < KP)
  auto issue_pair = [&](int m) {
#pragma unroll
    for (int X = 2; X < 4; ++X) {
      const int blk = 2 * m + X;
      if (blk < nb) {
        const int lds = blk_lds(blk), soff = blk_soff(blk);
        wv_static_for<kMaxPiecesPerWave>([&](auto iI) {
          if constexpr (decltype(iI)::value < KP) issue_x(iI, lds, soff);
        });
        if constexpr (kProdDma) issue_y(blk, lds);
      }
    }
  };

  if (wid >= NPW) {
    // ======================= consumer waves ==================================
    const int cw = wid - NPW;
    auto run = [&](auto cwI) {
      constexpr int CW = decltype(cwI)::value;
      constexpr int TW = OzConsumer<NT, CW>::TW;
      if constexpr (DLSA_OZ_PRIO > 0) __builtin_amdgcn_s_setprio(DLSA_OZ_PRIO);
      OzConsumer<NT, CW> C;
      C.init(P, lane);
      if constexpr (!kProdDma) {
        for (int b = 0; b < 2 && b < nb; ++b)
          issue_rest(std::integral_constant<int, KP>{}, b, blk_lds(b), blk_soff(b));
        wv_wait_vmcnt<0>();
      }
      OZ_DECL;
      for (int m = 0; m < nit; ++m) {
        OZ_STAMP(t0);
        barrier();  // B_m: blocks 2m, 2m+1 landed; the images of 2m-2, 2m-1 written
        OZ_STAMP(t1);
        // the DMA of blocks 2m+2, 2m+3 (into the slots of 2m-4, 2m-3): piece t
        // of one block after tile t's MFMAs of each image, the rest after
        const bool d0 = 2 * m + 2 < nb, d1 = 2 * m + 3 < nb;
        const int l0 = blk_lds(2 * m + 2), s0 = blk_soff(2 * m + 2);
        const int l1 = blk_lds(2 * m + 3), s1 = blk_soff(2 * m + 3);
        auto tick0 = [&](auto tI) {
          if (DLSA_OZ_TICK && d0) issue_x(tI, l0, s0);
        };
        auto tick1 = [&](auto tI) {
          if (DLSA_OZ_TICK && d1) issue_x(tI, l1, s1);
        };
        constexpr int I0 = DLSA_OZ_TICK ? TW : 0;
        const bool c0 = m >= 1 && !(DLSA_OZ_ABLATE & 2);
        const bool c1 = c0 && 2 * m - 1 < nb;
        OZ_STAMP_VAR(t2);
        if constexpr (kProdDma) {  // the producers issue the DMA
          auto tickN = [&](auto) {};
          if (c0) C.consume(slot_x(2 * m - 2), p, lane, tickN);
          if (c1) C.consume(slot_x(2 * m - 1), p, lane, tickN);
          OZ_STAMP_SET(t2);
        } else if constexpr (DLSA_OZ_SCHED == 0) {
          if (c0) C.consume(slot_x(2 * m - 2), p, lane, tick0);
          if (c1) C.consume(slot_x(2 * m - 1), p, lane, tick1);
          OZ_STAMP_SET(t2);
          // pieces not yet issued: all of a block whose image tick did not run
          if (d0) {
            if (c0)
              issue_rest(std::integral_constant<int, I0>{}, 2 * m + 2, l0, s0);
            else
              issue_rest(std::integral_constant<int, 0>{}, 2 * m + 2, l0, s0);
          }
          if (d1) {
            if (c1)
              issue_rest(std::integral_constant<int, I0>{}, 2 * m + 3, l1, s1);
            else
              issue_rest(std::integral_constant<int, 0>{}, 2 * m + 3, l1, s1);
          }
        } else {
          // both blocks' DMA during the first image's MFMAs (SCHED 1: a piece
          // of each per tile; SCHED 2: block 2m+2 at once, then a piece of
          // 2m+3 per tile), so the last pieces land while the second image's
          // MFMAs run instead of in front of the iteration's final wait
          // (pieces i < KP: the producers')
          auto tickA = [&](auto tI) {
            constexpr int i = KP + decltype(tI)::value;
            if (DLSA_OZ_SCHED == 1 && d0) issue_x(std::integral_constant<int, i>{}, l0, s0);
            if (d1) issue_x(std::integral_constant<int, i>{}, l1, s1);
          };
          auto tickN = [&](auto) {};
          if (DLSA_OZ_SCHED == 2 && d0) issue_rest(std::integral_constant<int, KP>{}, 2 * m + 2, l0, s0);
          if (c0) C.consume(slot_x(2 * m - 2), p, lane, tickA);
          if (c0) {
            if (DLSA_OZ_SCHED == 1 && d0)
              issue_rest(std::integral_constant<int, KP + TW>{}, 2 * m + 2, l0, s0);
            if (d1) issue_rest(std::integral_constant<int, KP + TW>{}, 2 * m + 3, l1, s1);
          } else {
            if (DLSA_OZ_SCHED == 1 && d0)
              issue_rest(std::integral_constant<int, KP>{}, 2 * m + 2, l0, s0);
            if (d1) issue_rest(std::integral_constant<int, KP>{}, 2 * m + 3, l1, s1);
          }
          if (c1) C.consume(slot_x(2 * m - 1), p, lane, tickN);
          OZ_STAMP_SET(t2);
        }
        OZ_STAMP(t3);
        wv_wait_vmcnt<0>();
        OZ_STAMP(t4);
        OZ_ADD(0, t1 - t0);
        OZ_ADD(1, t3 - t2);
        OZ_ADD(2, t2 - t1);
        OZ_ADD(3, t4 - t3);
      }
      OZ_FLUSH(4 * (NPW + CW));
      __syncthreads();  // S1
      // edge scratch: past the producers' reduction area at the ring's start
      C.store(a.slab_H + (int64_t)chunk * (NT * (NT + 1) / 2) * 256, ex, lane,
              (int*)(smem + 8192 + cw * 2 * 5 * 256 * 4));
      __syncthreads();  // S2 (the producers' reduction)
    };
    switch (cw) {
      case 0: run(std::integral_constant<int, 0>{}); break;
      case 1: run(std::integral_constant<int, 1>{}); break;
      case 2: run(std::integral_constant<int, 2>{}); break;
      default: run(std::integral_constant<int, 3>{}); break;
    }
    return;
  }

#if DLSA_OZ_R4
  oz_producer_r4<NT, STD, FAM>(a, smem, wid, lane, tid, nb, nit, sbytes, xs_bytes, slot_x, bet,
                               stdv, ex, chunk, chunk_ovf, issue_pair);
  return;
#endif
  // ========================= producer waves ==================================
  const int pw = wid;
  const int sl = lane / RPW;             // row phase: feature group
  const int rr = lane % RPW;             // row of this wave's 8
  const int rB = pw * RPW + rr;          // block row
  const int k4 = rr >> 2;                // row quad of the wave's 8 rows
  const uint32_t sel1 = (lane & 1) ? 0x03070105u : 0x06020400u;
  const uint32_t sel2 = (lane & 2) ? 0x03020706u : 0x05040100u;
  const int jq = lane & 3;               // lane in its quad: digit plane 4 - jq
  double beta[M], gacc[M];
  // per-feature magic MAGIC 2^(E_f - 38): fma(x, sqrt(w), mg) carries the
  // mantissa of fma(x, sqrt(w) 2^(38 - E_f), MAGIC) (a power-of-two scaling
  // of the same rounding), so no per-value ldexp
#if DLSA_OZ_MAGICF
  double mg[M];
#else
  int esc[M];
#endif
  uint32_t fmask = 0;                    // features f < P of this lane
#pragma unroll
  for (int m = 0; m < M; ++m) {
    const int f = sl + LPR * m;
    beta[m] = bet[f];
#if DLSA_OZ_MAGICF
    mg[m] = __builtin_amdgcn_ldexp(MAGIC, ex[f] - GBITS);
#else
    esc[m] = GBITS - ex[f];
#endif
    gacc[m] = 0.0;
    if (f < P) fmask |= 1u << m;
  }
  double llacc = 0.0, lprod = 1.0;

  OZ_DECL;
  for (int m = 0; m < nit; ++m) {
    OZ_STAMP(t0);
    barrier();  // B_m
    OZ_STAMP(t1);
    OZ_ADD(0, t1 - t0);
    if (2 * m >= nb || (DLSA_OZ_ABLATE & 1)) continue;  // the last iteration only consumes
    char* xsb[2];
    const double* ysb[2];
    int left[2];
#pragma unroll
    for (int X = 0; X < 2; ++X) {
      const int b = 2 * m + X;  // b = nb (odd nb): all rows invalid, nothing consumed
      xsb[X] = slot_x(b);
      ysb[X] = (const double*)(smem + (b % NSLOT) * sbytes + 16 + xs_bytes);
      left[X] = nrows - b * RB;
    }
    // ---- row phase of both blocks: 8 rows per wave, 8 lanes per row ---------
    // Two full blocks (every block but a chunk's last) need no row mask.  The
    // padding features f >= P of a row are still zeroed: their x reads land
    // on the row's successor, and the successor of a wave's last row (row
    // 8 pw + 7) is the first row of producer wave pw + 1, which overwrites
    // those bytes with its digit image as soon as it has read them -- with no
    // barrier in between, so the bytes read here may be digit bytes, i.e. any
    // double including NaN / inf, and NaN * beta_f (= 0) is NaN (ring-slot
    // ownership rule).  A chunk's last block(s) also zero the
    // rows past the chunk (they hold the next partition's rows, which must
    // not leak into this one, not even as NaN).
    const bool full = left[0] >= RB && left[1] >= RB;  // workgroup-uniform
    double xv[2][M], e[2], r[2];
    auto row_phase = [&](auto maskI) {
      constexpr bool MASK = decltype(maskI)::value;
#pragma unroll
      for (int X = 0; X < 2; ++X) {
        const bool valid = rB < left[X];
        const double* xr = (const double*)xsb[X] + rB * p + (sl - ic);
        double e0 = 0.0, e1 = 0.0;
#pragma unroll
        for (int m2 = 0; m2 < M; ++m2) {
          const int f = sl + LPR * m2;
          double v = xr[LPR * m2];
          if constexpr (DLSA_OZ_CHECK) {  // ownership rule: own rows for f < P
            const int e = rB * p + f - ic;  // element of the block this lane reads
            // a violation poisons the row (the partition ends nonfinite: the
            // tests see it without a fault)
            if (f >= ic && f < P && (e < pw * RPW * p || e >= (pw + 1) * RPW * p))
              v = __builtin_nan("");
          }
          if constexpr (STD) v = (v - stdv[f]) * stdv[PMAX + f];
          if (m2 == 0 && ic && sl == 0) v = 1.0;
          // features below the smallest P of this NT are always < P
          // (compile-time for all but the last one or two m2)
          const bool always_in = LPR * m2 + LPR - 1 < 16 * (NT - 1) + 1;
          const bool fin = always_in || ((fmask >> m2) & 1u);
          if constexpr (MASK)
            v = (valid && fin) ? v : 0.0;
          else
            v = fin ? v : 0.0;
          xv[X][m2] = v;
          if (m2 & 1)
            e1 = fma(v, beta[m2], e1);
          else
            e0 = fma(v, beta[m2], e0);
        }
        e[X] = e0 + e1;
      }
    };
    if (full)
      row_phase(std::false_type{});
    else
      row_phase(std::true_type{});
#pragma unroll
    for (int X = 0; X < 2; ++X) e[X] = wv_row_sum<RPW>(e[X]);
    // One transcendental chain for the 16 rows of both blocks: lanes 0-31 take
    // block 0's row rr (lane % 8), lanes 32-63 block 1's (every lane of a row
    // holds its eta), then each lane fetches the other block's results from
    // lane ^ 32 (the same row rr): half the chain instructions of one chain
    // per block.
    const bool hb = lane >= 32;
    double sw[2];
    {
      const double eh = hb ? e[1] : e[0];
      const int lh = hb ? left[1] : left[0];
      const bool valid = rB < lh;
      const double yv = valid ? ysb[hb ? 1 : 0][rB] : 0.0;
      // sqrt(w) = sqrt(e^-|eta|) / (1 + e^-|eta|): one exp of -|eta|/2 gives
      // both (no sqrt); the softplus log(1 + e^-|eta|) of the log-likelihood
      // goes into a running product per lane, one log at the end (a chunk is
      // <= 512 iterations, so the product of terms in [1, 2] stays < 2^512)
      double swh, rh;
      if constexpr (FAM == FAMILY_LOGISTIC) {
        const double eq = exp(-0.5 * fabs(eh));
        const double ea = eq * eq;
        const double inv = wv_rcp(1.0 + ea);
        const double mu = eh >= 0.0 ? inv : ea * inv;
        swh = eq * inv;
        rh = yv - mu;
        if (valid && (sl & 3) == 0) {
          llacc += yv * eh - fmax(eh, 0.0);
          lprod *= 1.0 + ea;
        }
      } else {  // gaussian (OLS): mu = eta, w = 1, ll = -rss / 2
        swh = 1.0;
        rh = yv - eh;
        if (valid && (sl & 3) == 0) llacc -= 0.5 * rh * rh;
      }
      if (!valid) {
        swh = 0.0;
        rh = 0.0;
      }
      const double swo = wv_swap32(swh, hb), ro = wv_swap32(rh, hb);
      sw[0] = hb ? swo : swh;
      sw[1] = hb ? swh : swo;
      r[0] = hb ? ro : rh;
      r[1] = hb ? rh : ro;
    }
    OZ_STAMP(t2);
    OZ_ADD(1, t2 - t1);
    // ---- gradient and the digit images --------------------------------------
#if DLSA_OZ_DBATCH
    static_assert(ND == 5, "batched digits: 5 digits");
    constexpr int NG = (M + 3) / 4;  // digit-0 words (4 features each)
#pragma unroll
    for (int X = 0; X < 2; ++X) {
      char* img = xsb[X] + pw * RPW * p * 8 + k4 * 4;
      uint32_t w[M + NG], hi[M];
#pragma unroll
      for (int m2 = 0; m2 < M; ++m2) {
        gacc[m2] = fma(xv[X][m2], r[X], gacc[m2]);
        const double t = OZ_DIGIT_T(xv[X][m2], sw[X], m2);
        w[m2] = __double2loint(t);
        hi[m2] = __double2hiint(t);
      }
#pragma unroll
      for (int g = 0; g < NG; ++g) {
        const int m0 = 4 * g, n = M - m0 < 4 ? M - m0 : 4;
        const uint32_t h0 = hi[m0], h1 = n > 1 ? hi[m0 + 1] : h0;
        const uint32_t h2 = n > 2 ? hi[m0 + 2] : h0, h3 = n > 3 ? hi[m0 + 3] : h0;
        w[M + g] = perm(perm(h3, h2, 0x05010400u), perm(h1, h0, 0x05010400u), 0x05040100u);
      }
      // the quad transposes stage by stage over all words (independent chains)
#pragma unroll
      for (int i = 0; i < M + NG; ++i) w[i] = perm(dpp<0xB1>(w[i]), w[i], sel1);
#pragma unroll
      for (int i = 0; i < M + NG; ++i) w[i] = perm(dpp<0x4E>(w[i]), w[i], sel2) ^ 0x80808080u;
#pragma unroll
      for (int m2 = 0; m2 < M; ++m2)
        *(uint32_t*)(img + (sl + LPR * m2) * kFeatBytes + plane_off(ND - 1 - jq)) = w[m2];
#pragma unroll
      for (int g = 0; g < NG; ++g) {
        const int m0 = 4 * g, n = M - m0 < 4 ? M - m0 : 4;
        if (jq < n)
          *(uint32_t*)(img + (sl + LPR * (m0 + jq)) * kFeatBytes + plane_off(0)) = w[M + g];
      }
    }
#else
#pragma unroll
    for (int X = 0; X < 2; ++X) {
      // this wave's image over its own rows (read above): [feature][plane][8 rows]
      char* img = xsb[X] + pw * RPW * p * 8 + k4 * 4;
      uint32_t top[4];
#pragma unroll
      for (int m2 = 0; m2 < M; ++m2) {
        gacc[m2] = fma(xv[X][m2], r[X], gacc[m2]);
        const double t = OZ_DIGIT_T(xv[X][m2], sw[X], m2);
        const uint32_t lo = __double2loint(t);
        // lane jq: byte jq of the quad's 4 rows = digit ND - 1 - jq
        const uint32_t dq = quad_transpose(lo, sel1, sel2) ^ 0x80808080u;
        *(uint32_t*)(img + (sl + LPR * m2) * kFeatBytes + plane_off(ND - 1 - jq)) = dq;
        if constexpr (ND == 4) continue;  // the low dword held all four digits
        top[m2 & 3] = __double2hiint(t);
        if ((m2 & 3) == 3 || m2 == M - 1) {  // digit 0 of up to 4 features
          const int m0 = m2 & ~3, n = m2 - m0 + 1;
#pragma unroll
          for (int u = n; u < 4; ++u) top[u] = top[0];
          const uint32_t t01 = perm(top[1], top[0], 0x05010400u);
          const uint32_t t23 = perm(top[3], top[2], 0x05010400u);
          const uint32_t tq = quad_transpose(perm(t23, t01, 0x05040100u), sel1, sel2) ^ 0x80808080u;
          if (jq < n) *(uint32_t*)(img + (sl + LPR * (m0 + jq)) * kFeatBytes + plane_off(0)) = tq;
        }
      }
    }
#endif
#ifdef DLSA_OZ_PROF
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#endif
    OZ_STAMP(t3);
    OZ_ADD(2, t3 - t2);
  }
  OZ_FLUSH(4 * pw);
  __syncthreads();  // S1 (the consumers' S1): the ring is free

  // ---- epilogue: gradient and log-likelihood partials --------------------------
  double* red = (double*)smem;  // the ring: [NPW][PMAX + 1]
#pragma unroll
  for (int m = 0; m < M; ++m) {
    double v = gacc[m];
#pragma unroll
    for (int o = 1; o < RPW; o <<= 1) v += __shfl_xor(v, o);
    if (rr == 0) red[pw * (PMAX + 1) + sl + LPR * m] = v;
  }
  if constexpr (FAM == FAMILY_LOGISTIC) llacc -= log(lprod);
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) llacc += __shfl_xor(llacc, o);
  if (lane == 0) red[pw * (PMAX + 1) + PMAX] = llacc;
  __syncthreads();  // S2
  for (int f = tid; f < PMAX; f += 64 * NPW) {
    double s = 0.0;
#pragma unroll
    for (int w = 0; w < NPW; ++w) s += red[w * (PMAX + 1) + f];
    a.slab_g[(int64_t)chunk * PMAX + f] = s;
  }
  if (tid == 0) {
    double s = 0.0;
#pragma unroll
    for (int w = 0; w < NPW; ++w) s += red[w * (PMAX + 1) + PMAX];
    a.slab_ll[chunk] = chunk_ovf ? __builtin_nan("") : s;
  }
}

template <int NT, bool STD, int FAM>
static hipError_t launch_oz_t(const PassArgs& a, int n_chunks, hipStream_t s) {
  auto kern = irls_oz_kernel<NT, STD, FAM>;
  hipError_t e = ensure_max_lds((const void*)kern, 160 * 1024);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(kern, dim3(n_chunks), dim3(64 * (ozk::NPW + ozk::NCW)),
                     ozk::lds_bytes(NT, a.p), s, a);
  return hipGetLastError();
}

template <int NT>
static hipError_t launch_oz_nt(const PassArgs& a, bool std_, int family, int n_chunks,
                               hipStream_t s) {
  if (family == FAMILY_GAUSSIAN)
    return std_ ? launch_oz_t<NT, true, FAMILY_GAUSSIAN>(a, n_chunks, s)
                : launch_oz_t<NT, false, FAMILY_GAUSSIAN>(a, n_chunks, s);
  return std_ ? launch_oz_t<NT, true, FAMILY_LOGISTIC>(a, n_chunks, s)
              : launch_oz_t<NT, false, FAMILY_LOGISTIC>(a, n_chunks, s);
}

}  // namespace dlsa
