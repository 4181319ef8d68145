// Wave-specialised fused fp64 IRLS pass (gfx950 / CDNA4) -- the pass whose
// Hessian is returned as Sig_inv (dlsa/models.py:130) and the single OLS pass.
// Instantiated by irls_ws_g*.hip.
//
// The fp64 pass is MFMA-bound (config 2: 1.43 PFLOP-equivalent of
// v_mfma_f64_16x16x4_f64 per 1e8 rows vs 80.8 GB of X), so the design keeps
// the matrix pipes busy instead of alternating phases:
//   * 8 waves per workgroup, one workgroup per CU, two waves per SIMD;
//   * waves 0-3 PRODUCE: each streams its own 8 rows of every 32-row block
//     HBM -> LDS by LDS-DMA (global_load_lds_dwordx4, 1 KiB lane-linear
//     pieces; its own sub-slot, so it waits on its own vmcnt only, no
//     barrier), then runs the row phase of block b+1: eta = x.theta (8-lane
//     DPP reduction), mu, w = mu(1-mu), r = y - mu, the fp64 gradient x r and
//     the fp64 log-likelihood; w goes to a double-buffered LDS vector;
//   * waves 4-7 CONSUME: the lower-triangle 16x16 tiles of X^T W X for block
//     b, split in contiguous ranges; per k-step of 4 rows lane l reads
//     x[row 4s + (l >> 4)][feature 16c + (l & 15)] from the ring (the 16x16x4
//     operand map, K = rows) and issues mfma(w x[I], x[J], acc);
//   * ONE barrier per block: the producers run a block ahead, so the MFMA
//     waves never wait for the transcendental row work.
// Ring: nslot slots x 4 sub-slots; block b+nslot-1 is issued into the slot of
// block b-1 right after the barrier that retires it.
#pragma once

#include <type_traits>
#include <utility>

#include "dlsa_internal.hpp"

namespace dlsa {

typedef double d4s __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) void lds_void_ws;
typedef const __attribute__((address_space(1))) void gbl_void_ws;

namespace {

constexpr int WS_RB = 32;   // rows per block
constexpr int WS_PAD = 16;  // zero bytes in front of a sub-slot (intercept lane reads x[-1])

template <int N>
__device__ __forceinline__ void ws_wait_vmcnt() {
  static_assert(N >= 0 && N < 64, "vmcnt is 6 bits on gfx950");
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
template <int N>
__device__ __forceinline__ void ws_wait_vmcnt_le(int n) {
  if constexpr (N <= 0) {
    ws_wait_vmcnt<0>();
  } else {
    if (n >= N)
      ws_wait_vmcnt<N>();
    else
      ws_wait_vmcnt_le<N - 1>(n);
  }
}

template <int CTRL>
__device__ __forceinline__ double ws_dpp(double v) {
  const int lo = __builtin_amdgcn_mov_dpp(__double2loint(v), CTRL, 0xF, 0xF, false);
  const int hi = __builtin_amdgcn_mov_dpp(__double2hiint(v), CTRL, 0xF, 0xF, false);
  return __hiloint2double(hi, lo);
}
// sum over the 8 lanes of a row group; bitwise-identical in every lane
__device__ __forceinline__ double ws_red8(double v) {
  v += ws_dpp<0xB1>(v);   // quad_perm [1,0,3,2]
  v += ws_dpp<0x4E>(v);   // quad_perm [2,3,0,1]
  v += ws_dpp<0x141>(v);  // row_half_mirror
  return v;
}

template <typename F, int... Is>
__device__ __forceinline__ void ws_static_for_impl(F&& f, std::integer_sequence<int, Is...>) {
  (f(std::integral_constant<int, Is>{}), ...);
}
template <int N, typename F>
__device__ __forceinline__ void ws_static_for(F&& f) {
  ws_static_for_impl(f, std::make_integer_sequence<int, N>{});
}

constexpr int ws_tile_I(int t) {
  int I = 0;
  while ((I + 1) * (I + 2) / 2 <= t) ++I;
  return I;
}
constexpr int ws_tile_J(int t) { return t - ws_tile_I(t) * (ws_tile_I(t) + 1) / 2; }

}  // namespace

// pieces a producer wave DMAs per block: its 8 rows + 16-B alignment slack
__host__ __device__ __forceinline__ int ws_npieces(int p) { return (64 * p + 16 + 1023) / 1024; }
// zero tail after the pieces: padded-feature reads of the last row run up to
// 8 (16 NT - p) + 16 bytes past its end; the alignment slack inside the
// pieces already covers part of that
__host__ __device__ __forceinline__ int ws_tail_bytes(int p, int NT) {
  const int need = 8 * (16 * NT - p) + 16 - (ws_npieces(p) * 1024 - 64 * p - 16);
  return need > 0 ? (need + 15) / 16 * 16 : 0;
}
__host__ __device__ __forceinline__ int ws_sub_bytes(int p, int NT) {
  return WS_PAD + ws_npieces(p) * 1024 + ws_tail_bytes(p, NT) + 256;  // pad | pieces | tail | y
}

template <int NT, bool STD, int FAM>
__global__ __launch_bounds__(512, 1) void irls_ws_kernel(const PassArgs a) {
  constexpr int T = NT * (NT + 1) / 2;
  constexpr int TPW = (T + 3) / 4;     // tiles per consumer wave (contiguous ranges)
  constexpr int PMAX = 16 * NT;
  constexpr int M = PMAX / 8;          // features per producer lane (8 lanes per row)
  constexpr int MAXW = 4 * (10 + 1);   // vmcnt bound: nslot <= 5, npieces <= 10 (p <= 128)
  extern __shared__ __attribute__((aligned(16))) char smem[];

  const int chunk = blockIdx.x;
  const int part = a.chunk_part[chunk];
  if (a.phase[part] != a.want_phase) return;  // workgroup-uniform

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const bool producer = wid < 4;
  const int p = a.p, P = a.P, ic = a.intercept;
  const int64_t row0 = a.chunk_row0[chunk];
  const int nrows = a.chunk_rows[chunk];
  const int nb = (nrows + WS_RB - 1) / WS_RB;
  const int nslot = a.nslot;
  const int sub_bytes = a.slot_bytes;  // one producer's sub-slot
  const int slot_bytes = 4 * sub_bytes;
  const int npw = ws_npieces(p);
  const int sub_y = WS_PAD + npw * 1024 + ws_tail_bytes(p, NT);
  double* wbuf = (double*)(smem + nslot * slot_bytes);  // [2][32]
  double* stdv = wbuf + 2 * WS_RB;                        // [2][PMAX] center, 1/scale

  // zero the ring once (pads / tails are never DMA'd), stage center / scale
  for (int o = tid * 16; o < nslot * slot_bytes; o += 512 * 16)
    *(uint4*)(smem + o) = make_uint4(0, 0, 0, 0);
  if constexpr (STD) {
    for (int f = tid; f < PMAX; f += 512) {
      const int j = f - ic;
      const bool in = j >= 0 && j < p;
      stdv[f] = in ? a.center[j] : 0.0;
      stdv[PMAX + f] = in ? 1.0 / a.scale[j] : 1.0;
    }
  }
  __syncthreads();

  // ---- producer state -------------------------------------------------------
  const int sl = lane & 7, rr = lane >> 3;  // row rr of the producer's 8, lanes sl + 8 m
  double beta[M], gacc[M];
#pragma unroll
  for (int m = 0; m < M; ++m) {
    const int f = sl + 8 * m;
    beta[m] = (producer && f < P) ? a.theta[(int64_t)part * P + f] : 0.0;
    gacc[m] = 0.0;
  }
  double llacc = 0.0;

  auto sub_base = [&](int blk, int pw) -> char* {
    return smem + (blk % nslot) * slot_bytes + pw * sub_bytes;
  };
  auto row_start = [&](int blk, int pw) -> uintptr_t {
    const int bb = blk < nb ? blk : nb - 1;
    return (uintptr_t)(a.X + (row0 + (int64_t)bb * WS_RB + 8 * pw) * p);
  };
  auto issue = [&](int blk) {  // producer wave wid: its 8 rows of block blk
    char* sb = sub_base(blk, wid);
    const uintptr_t al = row_start(blk, wid) & ~(uintptr_t)15;
    for (int j = 0; j < npw; ++j) {
      uintptr_t src = al + (uintptr_t)j * 1024 + (uintptr_t)lane * 16;
      src = src < a.x_last16 ? src : a.x_last16;
      __builtin_amdgcn_global_load_lds((gbl_void_ws*)src, (lds_void_ws*)(sb + WS_PAD + j * 1024),
                                       16, 0, 0);
    }
    const int bb = blk < nb ? blk : nb - 1;
    uintptr_t ys = (uintptr_t)(a.y + row0 + (int64_t)bb * WS_RB + 8 * wid) + (uintptr_t)lane * 4;
    ys = ys < a.y_last4 ? ys : a.y_last4;
    __builtin_amdgcn_global_load_lds((gbl_void_ws*)ys, (lds_void_ws*)(sb + sub_y), 4, 0, 0);
  };
  const int keep = (nslot - 2) * (npw + 1);  // DMA ops of the blocks after the awaited one

  auto row_phase = [&](int blk) {  // producer: rows 8 wid + rr of block blk
    const char* sb = sub_base(blk, wid);
    const uintptr_t rs = row_start(blk, wid);
    const double* xs = (const double*)(sb + WS_PAD + (rs & 15));
    const double* ys = (const double*)(sb + sub_y);
    const bool valid = blk * WS_RB + 8 * wid + rr < nrows;
    const double* xr = xs + rr * p + (sl - ic);
    double xv[M];
    double e = 0.0;
#pragma unroll
    for (int m = 0; m < M; ++m) {
      double v = xr[8 * m];
      if constexpr (STD) v = (v - stdv[sl + 8 * m]) * stdv[PMAX + sl + 8 * m];
      if (m == 0 && ic && sl == 0) v = 1.0;
      xv[m] = v;
      e = fma(v, beta[m], e);
    }
    e = ws_red8(e);
    const double yv = ys[rr];
    double w, r;
    if constexpr (FAM == FAMILY_LOGISTIC) {
      const double ea = exp(-fabs(e));
      const double inv = 1.0 / (1.0 + ea);
      const double mu = e >= 0.0 ? inv : ea * inv;
      w = ea * inv * inv;  // mu (1 - mu), cancellation free
      r = yv - mu;
      if (valid && sl == 0) llacc += yv * e - (fmax(e, 0.0) + log1p(ea));
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
    if (sl == 0) wbuf[(blk & 1) * WS_RB + 8 * wid + rr] = w;
  };

  // ---- consumer state -------------------------------------------------------
  const int cw = wid - 4;  // consumer index 0..3
  const int fl = lane & 15, kq = lane >> 4;
  d4s acc[TPW];
#pragma unroll
  for (int i = 0; i < TPW; ++i) acc[i] = d4s{0.0, 0.0, 0.0, 0.0};

  auto tile_phase = [&](auto cwI, int blk) {
    constexpr int CW = decltype(cwI)::value;
    unsigned cm = 0, rm = 0;
#pragma unroll
    for (int i = 0; i < TPW; ++i) {
      const int t = CW * TPW + i;
      if (t < T) {
        cm |= (1u << ws_tile_I(t)) | (1u << ws_tile_J(t));
        rm |= 1u << ws_tile_I(t);
      }
    }
    const double* wv = wbuf + (blk & 1) * WS_RB;
    // operands of k-step s+1 are read from LDS before the MFMAs of k-step s
    // issue (register double buffer), so the matrix pipe never waits on LDS
    double xb[2][NT], wb[2];
    auto read = [&](int s, double (&xv)[NT], double& w) {
      const int pw = s >> 1;  // rows 4s .. 4s+3 belong to producer pw
      const char* sb = sub_base(blk, pw);
      const uintptr_t rs = row_start(blk, pw);
      const double* xq =
          (const double*)(sb + WS_PAD + (rs & 15)) + ((4 * s + kq) & 7) * p + (fl - ic);
      w = wv[4 * s + kq];
#pragma unroll
      for (int c = 0; c < NT; ++c)
        if ((cm >> c) & 1u) xv[c] = xq[16 * c];
    };
    read(0, xb[0], wb[0]);
#pragma unroll
    for (int s = 0; s < WS_RB / 4; ++s) {
      if (s + 1 < WS_RB / 4) read(s + 1, xb[(s + 1) & 1], wb[(s + 1) & 1]);
      double xv[NT], av[NT];
#pragma unroll
      for (int c = 0; c < NT; ++c) {
        if ((cm >> c) & 1u) {
          double v = xb[s & 1][c];
          if constexpr (STD) v = (v - stdv[16 * c + fl]) * stdv[PMAX + 16 * c + fl];
          if (c == 0 && ic && fl == 0) v = 1.0;
          xv[c] = v;
          if ((rm >> c) & 1u) av[c] = v * wb[s & 1];
        }
      }
      ws_static_for<TPW>([&](auto iI) {
        constexpr int i = decltype(iI)::value;
        constexpr int t = CW * TPW + i;
        if constexpr (t < T) {
          constexpr int I = ws_tile_I(t), J = ws_tile_J(t);
          acc[i] = __builtin_amdgcn_mfma_f64_16x16x4f64(av[I], xv[J], acc[i], 0, 0, 0);
        }
      });
    }
  };

  // ---- prologue: producers fill the ring and run the row phase of block 0 --
  if (producer) {
    for (int b = 0; b < nslot - 1; ++b) issue(b);
    ws_wait_vmcnt_le<MAXW>(keep);
    row_phase(0);
  }

  // ---- main loop: consumers on block it, producers on block it + 1 ---------
  for (int it = 0; it < nb; ++it) {
    __syncthreads();  // w of block it published; block it-1 fully consumed
    if (producer) {
      issue(it + nslot - 1);  // into the slot of block it-1
      if (it + 1 < nb) {
        ws_wait_vmcnt_le<MAXW>(keep);
        row_phase(it + 1);
      }
    } else {
      ws_static_for<4>([&](auto cI) {
        if (cw == decltype(cI)::value) tile_phase(cI, it);
      });
    }
  }
  if (producer) ws_wait_vmcnt<0>();  // drain the tail re-fetches
  __syncthreads();

  // ---- epilogue --------------------------------------------------------------
  if (!producer) {
    double* sH = a.slab_H + (int64_t)chunk * T * 256;
#pragma unroll
    for (int i = 0; i < TPW; ++i) {
      const int t = cw * TPW + i;
      if (t < T) {
#pragma unroll
        for (int r = 0; r < 4; ++r) sH[t * 256 + (kq + 4 * r) * 16 + fl] = acc[i][r];
      }
    }
  }
  double* red = (double*)smem;  // ring no longer needed: [4][PMAX] + [4]
  if (producer) {
#pragma unroll
    for (int m = 0; m < M; ++m) {
      double v = gacc[m];
      v += __shfl_xor(v, 8);
      v += __shfl_xor(v, 16);
      v += __shfl_xor(v, 32);
      if (lane < 8) red[wid * PMAX + sl + 8 * m] = v;
    }
    llacc += __shfl_xor(llacc, 8);
    llacc += __shfl_xor(llacc, 16);
    llacc += __shfl_xor(llacc, 32);
    if (lane == 0) red[4 * PMAX + wid] = llacc;
  }
  __syncthreads();
  for (int f = tid; f < PMAX; f += 512)
    a.slab_g[(int64_t)chunk * PMAX + f] =
        ((red[f] + red[PMAX + f]) + red[2 * PMAX + f]) + red[3 * PMAX + f];
  if (tid == 0)
    a.slab_ll[chunk] =
        ((red[4 * PMAX] + red[4 * PMAX + 1]) + red[4 * PMAX + 2]) + red[4 * PMAX + 3];
}

inline int ws_extra_bytes(int NT) { return (2 * WS_RB + 2 * 16 * NT) * 8; }

template <int NT, bool STD, int FAM>
static hipError_t launch_ws_t(const PassArgs& a, int n_chunks, hipStream_t s) {
  auto kern = irls_ws_kernel<NT, STD, FAM>;
  const size_t lds = (size_t)a.nslot * 4 * a.slot_bytes + ws_extra_bytes(NT);
  static bool attr_set = false;
  if (!attr_set) {
    hipError_t e = hipFuncSetAttribute((const void*)kern,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    if (e != hipSuccess) return e;
    attr_set = true;
  }
  hipLaunchKernelGGL(kern, dim3(n_chunks), dim3(512), lds, s, a);
  return hipGetLastError();
}

template <int NT>
static hipError_t launch_ws_nt(const PassArgs& a, bool std_, int family, int n_chunks,
                               hipStream_t s) {
  if (family == FAMILY_GAUSSIAN)
    return std_ ? launch_ws_t<NT, true, FAMILY_GAUSSIAN>(a, n_chunks, s)
                : launch_ws_t<NT, false, FAMILY_GAUSSIAN>(a, n_chunks, s);
  return std_ ? launch_ws_t<NT, true, FAMILY_LOGISTIC>(a, n_chunks, s)
              : launch_ws_t<NT, false, FAMILY_LOGISTIC>(a, n_chunks, s);
}

}  // namespace dlsa
