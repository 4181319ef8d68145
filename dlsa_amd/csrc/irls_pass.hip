// Fused IRLS pass over X for a batch of row partitions (gfx950 / CDNA4).
//
// Replaces the per-partition work of the reference map stage -- sklearn's
// Newton-CG inner loop (Hessian-vector products = 2 passes over X each,
// dlsa/models.py:110-113), predict_proba (models.py:114) and the
// Sig_inv = X^T diag(p(1-p)) X product (models.py:130) -- with ONE pass over
// X per Newton iteration that produces, per chunk of rows:
//   eta = X theta, mu = sigmoid(eta), w = mu(1-mu), r = y - mu,
//   g   = X^T r                      (fp64 VALU),
//   H   = X^T diag(w) X              (lower-triangle 16x16 tiles, MFMA:
//                                     v_mfma_f64_16x16x4_f64 or
//                                     v_mfma_f32_16x16x4_f32),
//   ll  = sum y eta - log(1 + e^eta) (fp64).
//
// Geometry (DESIGN.md "Fused pass"):
//   * one workgroup = one wave64 = one chunk of consecutive rows of one
//     partition; no barriers, no inter-wave traffic.
//   * rows are streamed HBM -> LDS by LDS-DMA (global_load_lds_dwordx4, 1 KiB
//     per wave-instruction, lane-linear) into a private ring of `nslot` slots
//     of kRowsPerBlock rows; the wave waits with a COUNTED vmcnt so nslot-1
//     slots stay in flight while it computes on the oldest.
//   * MFMA operand layout: for a k-step of 4 rows, lane l holds
//     X[row 4s + (l>>4)][feature 16c + (l&15)] for every column tile c.  That
//     is exactly the A/B operand map of the 16x16x4 MFMA with K = rows, so the
//     tile (I,J) of X^T W X is mfma(w*x[I], x[J], acc) with no data movement.
//   * eta for the 4 rows of a k-step is a 16-lane fp64 reduction; the
//     logistic transcendental work is therefore done once per row-quad and
//     amortised over NT*(NT+1)/2 MFMAs.
#include "dlsa_internal.hpp"

namespace dlsa {

typedef double d4 __attribute__((ext_vector_type(4)));
typedef float f4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) void lds_void_t;
typedef const __attribute__((address_space(1))) void gbl_void_t;

template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  static_assert(N >= 0 && N < 64, "vmcnt is 6 bits on gfx950");
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// Wait until at most `n` vector-memory ops of this wave are outstanding
// (n is wave-uniform; the chain of scalar compares picks the immediate).
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

// DPP row_ror:n within each 16-lane row (dpp_ctrl 0x120 + n), on both halves
template <int CTRL>
__device__ __forceinline__ double dpp_f64(double v) {
  const int lo = __builtin_amdgcn_mov_dpp(__double2loint(v), CTRL, 0xF, 0xF, false);
  const int hi = __builtin_amdgcn_mov_dpp(__double2hiint(v), CTRL, 0xF, 0xF, false);
  return __hiloint2double(hi, lo);
}

// Sum over the 16 lanes of a row; every lane ends with the bitwise-identical
// total (each step adds a commutative pair), so all lanes of a row see the
// same eta, w and r.
__device__ __forceinline__ double red16(double v) {
  v += dpp_f64<0x128>(v);
  v += dpp_f64<0x124>(v);
  v += dpp_f64<0x122>(v);
  v += dpp_f64<0x121>(v);
  return v;
}

__device__ __forceinline__ int npieces_for(int p) {
  return (kRowsPerBlock * p * 8 + 16 + 1023) / 1024;
}

// Profiling-only ablations (tools/build_variants.sh builds them as separate
// .so files; the product build has DLSA_ABLATE = 0):
//   1 = no MFMA, 2 = no transcendentals, 3 = stream only (DMA ring, no math)
#ifndef DLSA_ABLATE
#define DLSA_ABLATE 0
#endif

template <int NT>
struct Geom {
  static constexpr int PMAX = 16 * NT;
  // dwordx4 DMA pieces needed for one block at the widest p of this NT
  static constexpr int MAX_PIECES = (kRowsPerBlock * PMAX * 8 + 16 + 1023) / 1024;
  // slot = [16 B zero pad | DMA pieces | 16*NT*8 B zero tail | y (256 B)].
  // Operand reads of padded features (f >= P) land in the pad, in a
  // neighbouring row or in the tail: always finite, and they only reach
  // Hessian entries outside P x P and zero-beta terms, so no masks are needed.
  static constexpr int PAD = 16;
  static constexpr int SLOT_X = PAD + MAX_PIECES * 1024 + PMAX * 8;
  static constexpr int SLOT_Y = 256;  // one dword DMA = 64 lanes x 4 B
  static constexpr int SLOT = SLOT_X + SLOT_Y;
  static constexpr int T = NT * (NT + 1) / 2;
};

template <int NT, bool F64, bool STD, int FAM>
__global__ __launch_bounds__(64, (F64 || NT >= 8) ? 1 : 2) void irls_pass_kernel(const PassArgs a) {
  using G = Geom<NT>;
  constexpr int T = G::T;
  constexpr int RB = kRowsPerBlock;
  constexpr int MAXW = 3 * (G::MAX_PIECES + 1);  // nslot <= 4
  extern __shared__ __attribute__((aligned(16))) char smem[];

  const int chunk = blockIdx.x;
  const int part = a.chunk_part[chunk];
  if (a.phase[part] != a.want_phase) return;  // wave-uniform

  const int lane = threadIdx.x;
  const int fl = lane & 15;  // feature within a column tile
  const int rq = lane >> 4;  // row within a k-step
  const int p = a.p, P = a.P, ic = a.intercept;
  const int64_t row0 = a.chunk_row0[chunk];
  const int nrows = a.chunk_rows[chunk];
  const int nb = (nrows + RB - 1) / RB;
  const int nslot = a.nslot;
  const int slot_bytes = a.slot_bytes;

  // per-lane feature constants: lane fl reads column 16c + fl - ic of a row
  // (column -1 = the intercept lane, overwritten by 1.0 below)
  const int xo = fl - ic;
  const bool icpt_lane = ic && fl == 0;
  double beta[NT];
  double cen[STD ? NT : 1], isd[STD ? NT : 1];
#pragma unroll
  for (int c = 0; c < NT; ++c) {
    const int f = 16 * c + fl;
    const int j = f - ic;
    beta[c] = (f < P) ? a.theta[(int64_t)part * P + f] : 0.0;
    if constexpr (STD) {
      const bool in = j >= 0 && j < p;
      cen[c] = in ? a.center[j] : 0.0;
      isd[c] = in ? 1.0 / a.scale[j] : 1.0;
    }
  }
  // zero the pad and tail bytes of every slot (the DMA never writes them)
  for (int sidx = 0; sidx < nslot; ++sidx) {
    double* sl = (double*)(smem + sidx * slot_bytes);
    if (lane < G::PAD / 8) sl[lane] = 0.0;
    const int tail0 = (G::PAD + npieces_for(p) * 1024) / 8;
    for (int q = tail0 + lane; q < G::SLOT_X / 8; q += 64) sl[q] = 0.0;
  }

  // accumulators
  d4 accd[F64 ? T : 1];
  f4 accf[F64 ? 1 : T];
#pragma unroll
  for (int t = 0; t < (F64 ? T : 1); ++t) accd[t] = d4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
  for (int t = 0; t < (F64 ? 1 : T); ++t) accf[t] = f4{0.f, 0.f, 0.f, 0.f};
  double gacc[NT];
#pragma unroll
  for (int c = 0; c < NT; ++c) gacc[c] = 0.0;
  double llacc = 0.0;

  // DMA pieces per block for this p (wave-uniform)
  const int npieces = npieces_for(p);
  const double* Xp = a.X;

  auto issue = [&](int blk) {
    const int bb = blk < nb ? blk : nb - 1;  // tail: harmless re-fetch, keeps counts fixed
    char* sbase = smem + (blk % nslot) * slot_bytes;
    const uintptr_t start = (uintptr_t)(Xp + (row0 + (int64_t)bb * RB) * p);
    const uintptr_t al = start & ~(uintptr_t)15;
    for (int j = 0; j < npieces; ++j) {
      uintptr_t src = al + (uintptr_t)j * 1024 + (uintptr_t)lane * 16;
      src = src < a.x_last16 ? src : a.x_last16;
      __builtin_amdgcn_global_load_lds((gbl_void_t*)src,
                                       (lds_void_t*)(sbase + G::PAD + j * 1024), 16, 0, 0);
    }
    uintptr_t ys = (uintptr_t)(a.y + row0 + (int64_t)bb * RB) + (uintptr_t)lane * 4;
    ys = ys < a.y_last4 ? ys : a.y_last4;
    __builtin_amdgcn_global_load_lds((gbl_void_t*)ys, (lds_void_t*)(sbase + G::SLOT_X), 4, 0, 0);
  };

  for (int b = 0; b < nslot - 1; ++b) issue(b);
  const int inflight = (nslot - 1) * (npieces + 1);

  for (int b = 0; b < nb; ++b) {
    issue(b + nslot - 1);
    wait_vmcnt_le<MAXW>(inflight);  // block b has landed

    const char* slot = smem + (b % nslot) * slot_bytes;
    const uintptr_t start = (uintptr_t)(Xp + (row0 + (int64_t)b * RB) * p);
    const double* xs = (const double*)(slot + G::PAD + (start & 15));
    const double* ysl = (const double*)(slot + G::SLOT_X);
    const int rows_left = nrows - b * RB;
    if constexpr (DLSA_ABLATE == 3) {
      llacc += xs[lane] + ysl[lane & 7];
      continue;
    }

#pragma unroll
    for (int s = 0; s < RB / 4; ++s) {
      const int rl = 4 * s + rq;
      const bool valid = rl < rows_left;
      const double* xr = xs + rl * p + xo;
      double xf[NT];
#pragma unroll
      for (int c = 0; c < NT; ++c) {
        double v = xr[16 * c];
        if constexpr (STD) v = (v - cen[c]) * isd[c];
        xf[c] = v;
      }
      if (icpt_lane) xf[0] = 1.0;
      double e = 0.0;
#pragma unroll
      for (int c = 0; c < NT; ++c) e = fma(xf[c], beta[c], e);
      e = red16(e);  // eta of row rl, in all 16 lanes of the row
      const double yv = ysl[rl];
      double w, r;
      if constexpr (FAM == FAMILY_LOGISTIC && DLSA_ABLATE == 2) {
        w = 0.25 - 0.01 * e * e;
        r = yv - 0.5 - 0.2 * e;
        if (valid && fl == 0) llacc += yv * e;
      } else if constexpr (FAM == FAMILY_LOGISTIC) {
        const double ea = exp(-fabs(e));
        const double inv = 1.0 / (1.0 + ea);
        const double mu = e >= 0.0 ? inv : ea * inv;
        w = ea * inv * inv;  // mu (1 - mu), cancellation free
        r = yv - mu;
        if (valid && fl == 0) {
          // log-likelihood: exact fp64 in the fp64 pass (its value is
          // returned); fp32 log in fp32-Hessian passes, where it only drives
          // step halving (|error| < 1e-7 per row, far below the 1e-6 relative
          // threshold of newton_solve_kernel)
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

      if constexpr (DLSA_ABLATE == 1) {
#pragma unroll
        for (int c = 0; c < NT; ++c) {
          float af = (float)(xf[c] * w);
          asm volatile("" ::"v"(af));
        }
      } else if constexpr (F64) {
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
    }
  }
  wait_vmcnt<0>();  // drain the tail re-fetches before the wave retires

  // ---- epilogue: partial sums of this chunk --------------------------------
  double* sH = a.slab_H + (int64_t)chunk * T * 256;
#pragma unroll
  for (int t = 0; t < T; ++t) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      // f64 16x16x4 C/D map: row = (l>>4) + 4*reg; f32 16x16x4: row = 4*(l>>4) + reg
      const int row = F64 ? (rq + 4 * r) : (4 * rq + r);
      const double v = F64 ? accd[t][r] : (double)accf[t][r];
      sH[t * 256 + row * 16 + fl] = v;
    }
  }
#pragma unroll
  for (int c = 0; c < NT; ++c) {
    double v = gacc[c];
    v += __shfl_xor(v, 16);
    v += __shfl_xor(v, 32);
    if (rq == 0) a.slab_g[(int64_t)chunk * (16 * NT) + 16 * c + fl] = v;
  }
  llacc += __shfl_xor(llacc, 16);
  llacc += __shfl_xor(llacc, 32);
  if (lane == 0) a.slab_ll[chunk] = llacc;
}

int pass_slot_bytes(int NT) {
  switch (NT) {
#define DLSA_SLOT(n) \
  case n:            \
    return Geom<n>::SLOT;
    DLSA_SLOT(1)
    DLSA_SLOT(2)
    DLSA_SLOT(3)
    DLSA_SLOT(4)
    DLSA_SLOT(5)
    DLSA_SLOT(6)
    DLSA_SLOT(7)
    DLSA_SLOT(8)
#undef DLSA_SLOT
    default:
      return -1;
  }
}

int pass_waves_per_cu(bool f64) { return f64 ? 4 : 8; }

template <int NT, bool F64, bool STD, int FAM>
static hipError_t launch_t(const PassArgs& a, int n_chunks, hipStream_t s) {
  auto kern = irls_pass_kernel<NT, F64, STD, FAM>;
  const size_t lds = (size_t)a.nslot * a.slot_bytes;
  static bool attr_set = false;  // per instantiation
  if (!attr_set) {
    hipError_t e = hipFuncSetAttribute((const void*)kern,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    if (e != hipSuccess) return e;
    attr_set = true;
  }
  hipLaunchKernelGGL(kern, dim3(n_chunks), dim3(64), lds, s, a);
  return hipGetLastError();
}

template <int NT>
static hipError_t launch_nt(const PassArgs& a, bool f64, bool std_, int family, int n_chunks,
                            hipStream_t s) {
  if (family == FAMILY_GAUSSIAN) {  // OLS: a single exact pass, fp64 only
    if (!f64) return hipErrorInvalidValue;
    return std_ ? launch_t<NT, true, true, FAMILY_GAUSSIAN>(a, n_chunks, s)
                : launch_t<NT, true, false, FAMILY_GAUSSIAN>(a, n_chunks, s);
  }
  if (f64)
    return std_ ? launch_t<NT, true, true, FAMILY_LOGISTIC>(a, n_chunks, s)
                : launch_t<NT, true, false, FAMILY_LOGISTIC>(a, n_chunks, s);
  return std_ ? launch_t<NT, false, true, FAMILY_LOGISTIC>(a, n_chunks, s)
              : launch_t<NT, false, false, FAMILY_LOGISTIC>(a, n_chunks, s);
}

hipError_t launch_irls_pass(const PassArgs& a, int NT, bool f64, bool standardize, int family,
                            int n_chunks, hipStream_t s) {
  switch (NT) {
    case 1: return launch_nt<1>(a, f64, standardize, family, n_chunks, s);
    case 2: return launch_nt<2>(a, f64, standardize, family, n_chunks, s);
    case 3: return launch_nt<3>(a, f64, standardize, family, n_chunks, s);
    case 4: return launch_nt<4>(a, f64, standardize, family, n_chunks, s);
    case 5: return launch_nt<5>(a, f64, standardize, family, n_chunks, s);
    case 6: return launch_nt<6>(a, f64, standardize, family, n_chunks, s);
    case 7: return launch_nt<7>(a, f64, standardize, family, n_chunks, s);
    case 8: return launch_nt<8>(a, f64, standardize, family, n_chunks, s);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace dlsa
