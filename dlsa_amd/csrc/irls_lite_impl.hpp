// Light-weight approximate-Hessian IRLS pass (gfx950 / CDNA4) for the Newton
// steps before the fp64 pass, P <= 112.  Instantiated by
// irls_lite.hip.
//
// The approximate pass is HBM-bound (80.8 GB of X per pass at config 2), so
// the design maximises bytes in flight and waves per CU:
//   * 16-row blocks, 4 waves per workgroup, several workgroups per CU: a
//     ring slot is ~13.6 KB (p = 100) and nothing else lives in LDS;
//   * rows stream HBM -> LDS by buffer_load ... lds (1 KiB lane-linear
//     pieces, bounds-checked buffer resource, scalar offsets);
//   * row phase: wave w owns rows 4w .. 4w+3, lane (row l >> 4, feature
//     group l & 15) holds features 16 m + (l & 15): eta = x.theta is a DPP
//     reduction inside a 16-lane row, then w, r = y - mu, the fp64 gradient
//     and the (fp32-log) log-likelihood;
//   * the bf16 MFMA operands are written IN PLACE over the wave's own rows
//     of the slot ([feature][4 rows] images of x and w x, 8 B per feature),
//     once the wave holds them in registers: no extra LDS;
//   * tile phase: v_mfma_f32_16x16x16_bf16 with K = the block's 16 rows --
//     lane (i, kg) reads rows 4 kg .. 4 kg + 3 of feature 16 c + i with one
//     ds_read_b64 from wave kg's image (16 lanes = 128 contiguous bytes).
// Two barriers per block: rows landed / slot free, images complete.
#pragma once

#include "dlsa_internal.hpp"

namespace dlsa {

typedef float f4l __attribute__((ext_vector_type(4)));
typedef short s4l __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x2l __attribute__((ext_vector_type(2)));
typedef float f2l __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(3))) void lds_void_l;

namespace {

constexpr int LT_RB = 16;   // rows per block
constexpr int LT_PAD = 16;  // zero bytes before the pieces (intercept lane reads x[-1])

template <int N>
__device__ __forceinline__ void lt_wait_vmcnt() {
  static_assert(N >= 0 && N < 64, "vmcnt is 6 bits on gfx950");
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
template <int N>
__device__ __forceinline__ void lt_wait_vmcnt_le(int n) {
  if constexpr (N <= 0) {
    lt_wait_vmcnt<0>();
  } else {
    if (n >= N)
      lt_wait_vmcnt<N>();
    else
      lt_wait_vmcnt_le<N - 1>(n);
  }
}

template <int CTRL>
__device__ __forceinline__ double lt_dpp(double v) {
  const int lo = __builtin_amdgcn_mov_dpp(__double2loint(v), CTRL, 0xF, 0xF, false);
  const int hi = __builtin_amdgcn_mov_dpp(__double2hiint(v), CTRL, 0xF, 0xF, false);
  return __hiloint2double(hi, lo);
}
// sum over the 16 lanes of a DPP row (row_ror 8, 4, 2, 1); identical in all 16
__device__ __forceinline__ double lt_red16(double v) {
  v += lt_dpp<0x128>(v);
  v += lt_dpp<0x124>(v);
  v += lt_dpp<0x122>(v);
  v += lt_dpp<0x121>(v);
  return v;
}

}  // namespace

__host__ __device__ __forceinline__ int lt_npieces(int p) {
  return (LT_RB * p * 8 + 16 + 1023) / 1024;
}
// slot: pad | pieces | zero tail for padded-feature reads of the last row | y
__host__ __device__ __forceinline__ int lt_slot_bytes(int p, int NT) {
  int tail = 8 * (16 * NT - p) + 16 - (lt_npieces(p) * 1024 - LT_RB * p * 8 - 16);
  tail = tail > 0 ? (tail + 15) / 16 * 16 : 0;
  return LT_PAD + lt_npieces(p) * 1024 + tail + 256;
}
// the in-place images (2 x 16 NT features x 4 rows x 2 B) must fit in a
// wave's 4 rows of X (4 p x 8 B)
__host__ __device__ __forceinline__ bool lt_fits(int p, int NT) {
  return NT <= 7 && 2 * 16 * NT * 8 <= 4 * p * 8;  // NT = 8 spills (launch fails)
}

template <int NT, bool STD>
__global__ __launch_bounds__(256, 4) void irls_lite_kernel(const PassArgs a) {
  constexpr int T = NT * (NT + 1) / 2;
  constexpr int TPW = (T + 3) / 4;
  constexpr int PMAX = 16 * NT;
  constexpr int MAXW = 4 * (9 + 1);  // vmcnt bound: nslot <= 5, pieces per wave <= 9 + y
  extern __shared__ __attribute__((aligned(16))) char smem[];

  const int chunk = blockIdx.x;
  const int part = a.chunk_part[chunk];
  if (a.phase[part] != a.want_phase) return;  // workgroup-uniform

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int p = a.p, P = a.P, ic = a.intercept;
  const int64_t row0 = a.chunk_row0[chunk];
  const int nrows = a.chunk_rows[chunk];
  const int nb = (nrows + LT_RB - 1) / LT_RB;
  const int nslot = a.nslot;
  const int slot_bytes = a.slot_bytes;
  const int npieces = lt_npieces(p);
  const int d = (npieces + 3) / 4;  // pieces per wave per block (duplicates clamped)
  const int slot_y = slot_bytes - 256;
  double* stdv = (double*)(smem + nslot * slot_bytes);  // [2][PMAX] (STD only)

  for (int o = tid * 16; o < nslot * slot_bytes; o += 256 * 16)
    *(uint4*)(smem + o) = make_uint4(0, 0, 0, 0);
  if constexpr (STD) {
    for (int f = tid; f < PMAX; f += 256) {
      const int j = f - ic;
      const bool in = j >= 0 && j < p;
      stdv[f] = in ? a.center[j] : 0.0;
      stdv[PMAX + f] = in ? 1.0 / a.scale[j] : 1.0;
    }
  }

  // ---- row-phase constants ------------------------------------------------
  const int rl = lane >> 4, sl = lane & 15;
  const int rB = 4 * wid + rl;  // block row of this lane
  double beta[NT], gacc[NT];
  bool inb[NT];
#pragma unroll
  for (int m = 0; m < NT; ++m) {
    const int f = sl + 16 * m;
    const int j = f - ic;
    inb[m] = j >= 0 && j < p;
    beta[m] = f < P ? a.theta[(int64_t)part * P + f] : 0.0;
    gacc[m] = 0.0;
  }
  const bool icpt_lane = ic && sl == 0;
  double llacc = 0.0;

  // ---- tile-phase constants: this wave's tiles (wave-uniform) -------------
  int tI[TPW], tJ[TPW];
#pragma unroll
  for (int i = 0; i < TPW; ++i) {
    const int t = wid * TPW + i;
    int I = 0;
    while ((I + 1) * (I + 2) / 2 <= t) ++I;
    tI[i] = __builtin_amdgcn_readfirstlane(I);
    tJ[i] = __builtin_amdgcn_readfirstlane(t - I * (I + 1) / 2);
  }
  f4l acc[TPW];
#pragma unroll
  for (int i = 0; i < TPW; ++i) acc[i] = f4l{0.f, 0.f, 0.f, 0.f};
  const int fl = lane & 15, kg = lane >> 4;
  __syncthreads();  // ring zeroed, center / scale staged

  // ---- DMA: bounds-checked buffer resources over this chunk ----------------
  const uintptr_t xcb = (uintptr_t)(a.X + row0 * p) & ~(uintptr_t)15;
  const __amdgpu_buffer_rsrc_t xrs = __builtin_amdgcn_make_buffer_rsrc(
      (void*)xcb, (short)0, (int)min<uintptr_t>(a.x_last16 + 16 - xcb, 0x7FFFFFF0u), 0x00020000);
  const uintptr_t ycb = (uintptr_t)(a.y + row0);
  const __amdgpu_buffer_rsrc_t yrs = __builtin_amdgcn_make_buffer_rsrc(
      (void*)ycb, (short)0, (int)min<uintptr_t>(a.y_last4 + 4 - ycb, 0x7FFFFFF0u), 0x00020000);
  auto blk_start = [&](int blk) -> uintptr_t {
    const int bb = blk < nb ? blk : nb - 1;
    return (uintptr_t)(a.X + (row0 + (int64_t)bb * LT_RB) * p);
  };
  auto issue = [&](int blk) {
    const int bb = blk < nb ? blk : nb - 1;  // tail: harmless re-fetch, fixed counts
    char* sb = smem + (blk % nslot) * slot_bytes;
    const int so = (int)((blk_start(blk) & ~(uintptr_t)15) - xcb);
    for (int i = 0; i < d; ++i) {
      int j = wid + 4 * i;
      j = j < npieces ? j : npieces - 1;  // duplicate of the last piece, same place
      __builtin_amdgcn_raw_ptr_buffer_load_lds(xrs, (lds_void_l*)(sb + LT_PAD + j * 1024), 16,
                                               lane * 16, so + j * 1024, 0, 0);
    }
    __builtin_amdgcn_raw_ptr_buffer_load_lds(yrs, (lds_void_l*)(sb + slot_y), 4, lane * 4,
                                             bb * LT_RB * 8, 0, 0);
  };
  for (int b = 0; b < nslot - 1; ++b) issue(b);
  const int keep = (nslot - 2) * (d + 1);

  for (int b = 0; b < nb; ++b) {
    lt_wait_vmcnt_le<MAXW>(keep);  // this wave's pieces of block b landed
    __syncthreads();               // B1: all pieces landed; slot of block b-1 retired
    issue(b + nslot - 1);

    char* slot = smem + (b % nslot) * slot_bytes;
    const double* xs = (const double*)(slot + LT_PAD + (blk_start(b) & 15));
    const double* ys = (const double*)(slot + slot_y);
    const bool valid = rB < nrows - b * LT_RB;

    // ---- row phase (registers) ----------------------------------------------
    const double* xr = xs + rB * p + (sl - ic);
    double xv[NT];
    double e = 0.0;
#pragma unroll
    for (int m = 0; m < NT; ++m) {
      double v = xr[16 * m];
      if constexpr (STD) v = (v - stdv[sl + 16 * m]) * stdv[PMAX + sl + 16 * m];
      v = inb[m] ? v : 0.0;  // select: padded reads may see another wave's images
      if (m == 0 && icpt_lane) v = 1.0;
      xv[m] = v;
      e = fma(v, beta[m], e);
    }
    e = lt_red16(e);
    const double yv = ys[rB];
    const double ea = exp(-fabs(e));
    const double inv = 1.0 / (1.0 + ea);
    const double mu = e >= 0.0 ? inv : ea * inv;
    double w = ea * inv * inv;  // mu (1 - mu), cancellation free
    double r = yv - mu;
    if (valid && sl == 0) llacc += yv * e - (fmax(e, 0.0) + (double)__logf(1.0f + (float)ea));
    if (!valid) {
      w = 0.0;
      r = 0.0;
    }
#pragma unroll
    for (int m = 0; m < NT; ++m) gacc[m] = fma(xv[m], r, gacc[m]);

    // ---- images over the wave's own rows ------------------------------------
    __bf16* img = (__bf16*)(xs + 4 * wid * p);  // [2][PMAX][4] bf16
    const float wf = (float)w;
#pragma unroll
    for (int m = 0; m < NT; ++m) {
      float xf = (float)xv[m];
      asm volatile("" : "+v"(xf));  // keep (bf16)(float)x from folding into f64 -> bf16
      const f2l pr = {xf, xf * wf};
      const bf16x2l pk = __builtin_convertvector(pr, bf16x2l);
      const int o = (sl + 16 * m) * 4 + rl;
      img[o] = pk[0];
      img[PMAX * 4 + o] = pk[1];
    }
    __syncthreads();  // B2: images of all 16 rows written

    // ---- tile phase ---------------------------------------------------------
    const char* imgk = (const char*)(xs + 4 * kg * p);  // wave kg's rows = k 4kg .. 4kg+3
#pragma unroll
    for (int i = 0; i < TPW; ++i) {
      if (wid * TPW + i < T) {  // wave-uniform
        const s4l av = *(const s4l*)(imgk + PMAX * 8 + (16 * tI[i] + fl) * 8);
        const s4l bv = *(const s4l*)(imgk + (16 * tJ[i] + fl) * 8);
        acc[i] = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(av, bv, acc[i], 0, 0, 0);
      }
    }
  }
  lt_wait_vmcnt<0>();  // drain the tail re-fetches
  __syncthreads();

  // ---- epilogue: chunk partials (newton_solve.hip layout) -------------------
  double* sH = a.slab_H + (int64_t)chunk * T * 256;
#pragma unroll
  for (int i = 0; i < TPW; ++i) {
    const int t = wid * TPW + i;
    if (t < T) {
#pragma unroll
      for (int r = 0; r < 4; ++r) sH[t * 256 + (4 * kg + r) * 16 + fl] = (double)acc[i][r];
    }
  }
  double* red = (double*)smem;  // [4][PMAX] + [4]
#pragma unroll
  for (int m = 0; m < NT; ++m) {
    double v = gacc[m];
    v += __shfl_xor(v, 16);
    v += __shfl_xor(v, 32);
    if (rl == 0) red[wid * PMAX + sl + 16 * m] = v;
  }
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) llacc += __shfl_xor(llacc, o);
  if (lane == 0) red[4 * PMAX + wid] = llacc;
  __syncthreads();
  for (int f = tid; f < PMAX; f += 256)
    a.slab_g[(int64_t)chunk * PMAX + f] =
        ((red[f] + red[PMAX + f]) + red[2 * PMAX + f]) + red[3 * PMAX + f];
  if (tid == 0)
    a.slab_ll[chunk] =
        ((red[4 * PMAX] + red[4 * PMAX + 1]) + red[4 * PMAX + 2]) + red[4 * PMAX + 3];
}

template <int NT, bool STD>
static hipError_t launch_lite_t(const PassArgs& a, int n_chunks, hipStream_t s) {
  auto kern = irls_lite_kernel<NT, STD>;
  const size_t lds = (size_t)a.nslot * a.slot_bytes + (STD ? 2 * 16 * NT * 8 : 0);
  static bool attr_set = false;
  if (!attr_set) {
    hipError_t e = hipFuncSetAttribute((const void*)kern,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    if (e != hipSuccess) return e;
    attr_set = true;
  }
  hipLaunchKernelGGL(kern, dim3(n_chunks), dim3(256), lds, s, a);
  return hipGetLastError();
}

}  // namespace dlsa
