// Exact X^T W X of the wide path (P > DLSA_MAX_P_FUSED) on the int8 matrix
// cores: the digit-slice scheme of irls_oz_impl.hpp applied
// to the 128 x 128 output tiles of wide_gram_kernel, with the digits computed
// once per row and staged through HBM instead of once per tile.
//
// Replaces, for the exact Newton iterations of a wide fit, the Sig_inv =
// X^T diag(p(1-p)) X of the reference map stage (dlsa/models.py:110-131).
//
//   wide_row_kernel      (wide_pass.hip) also records per row chunk the max
//                        |z| = |sqrt(w) x| of every feature (WideArgs::slab_zmax)
//   wide_oz_scale_kernel per Gram row group and feature E_f with |z| < 2^E_f
//                        (max over the row chunks that overlap the group: a
//                        large |z| in one row group does not coarsen the grid
//                        of the partition's other row groups)
//   wide_oz_digits_kernel  F = round(z 2^(38 - E_f)) by one FMA against
//                        1.5 2^52 + 0x8080808080; its five bytes XOR 0x80 are
//                        balanced digits d_0 .. d_4 (byte r of plane d = digit
//                        d of row r), stored per 8 rows as three slices
//                        [feature][16 B] (planes 0-1), [feature][16 B] (2-3),
//                        [feature][8 B] (4): 40 bytes per (8 rows, feature), a
//                        wave's store of a slice is contiguous, and the
//                        consumers' fragment reads are 16- / 8-byte strided
//   wide_oz_gram_kernel  per (row group, 128 x 128 tile): 8 waves, each a
//                        64 x 32 block (4 x 2 sub-tiles of 16 x 16), NL = 5
//                        int32 level accumulators per sub-tile; per 32-row step
//                        the A and B panels (4 x 128 records) come into an LDS
//                        ring by LDS-DMA; 9 v_mfma_i32_16x16x64_i8 per sub-tile
//                        per step (digit pairs (a, a+1) x (b, b-1)); the tile
//                        is written to slab_G in fp64, scaled by
//                        2^(E_i + E_j - 12) -- wide_assemble_kernel unchanged.
// A row group is at most 32767 rows (exact int32 level sums).
#include "irls_oz_impl.hpp"

namespace dlsa {

namespace {

constexpr int kRec = kWideOzRec;       // digit bytes per (8 rows, feature): 5 planes
constexpr int kOzGT = 128;             // output tile edge
constexpr int kOzStages = 3;           // LDS ring: 2 steps in flight + 1 computed
constexpr int kPanel = 4 * kOzGT * kRec;  // one panel of a step: 4 rowblocks x 128 features (20 KB)
constexpr int kPieces = kPanel / 1024;    // 1-KB DMA pieces of a panel (20)

}  // namespace

// E[g, f] for Gram row group g from the max over the row chunks of its
// partition whose rows overlap it (|z| < 2^E: the bound with the low dword all
// ones).  The row chunks of a partition are consecutive and ascending.
__global__ __launch_bounds__(256) void wide_oz_scale_kernel(const WideArgs a, const WideOzArgs o,
                                                            int PP) {
  const int g = blockIdx.x;
  const int part = a.gc_part[g];
  const int64_t r0 = a.gc_row0[g], r1 = r0 + a.gc_rows[g];
  const int c0 = o.rcb[part], c1 = o.rcb[part + 1];
  for (int f = threadIdx.x; f < PP; f += 256) {
    uint32_t m = 0;
    for (int c = c0; c < c1; ++c) {
      const int64_t s0 = a.rc_row0[c], s1 = s0 + a.rc_rows[c];
      if (s1 <= r0) continue;
      if (s0 >= r1) break;
      m = max(m, o.zmax[(int64_t)c * PP + f]);
    }
    const double bound = __hiloint2double((int)(m & 0x7FFFFFFFu), (int)0xFFFFFFFFu);
    int e = __builtin_amdgcn_frexp_exp(bound);
    // EMAX + 1 marks |z| >= 2^EMAX (digits would wrap): the tile kernel writes NaN
    o.E[(int64_t)g * PP + f] = min(max(e, ozk::EMIN), ozk::EMAX + 1);
  }
}

// one workgroup per (row group, 32-row block): wave w = rows 8w .. 8w+7 of the
// block, lane l = features l + 64 j; each lane builds its features' records
template <int MB, bool STD>
__global__ __launch_bounds__(256) void wide_oz_digits_kernel(const WideArgs a, const WideOzArgs o) {
  const int g = blockIdx.x, blk = blockIdx.y;
  const int nrows = a.gc_rows[g];
  if (blk * 32 >= nrows) return;
  const int part = a.gc_part[g];
  if (a.phase[part] != PHASE_F64) return;
  constexpr int PP = 64 * MB;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int p = a.p, ic = a.intercept;
  const int64_t row0 = a.gc_row0[g] + blk * 32 + wid * 8;
  const int left = nrows - blk * 32 - wid * 8;  // valid rows of this wave's 8
  double sw[8];
#pragma unroll
  for (int r = 0; r < 8; ++r) sw[r] = r < left ? sqrt(a.w[row0 + r]) : 0.0;
  int8_t* rec = o.D + (((int64_t)g * o.maxblk + blk) * 4 + wid) * PP * kRec;
#pragma unroll 1
  for (int m = 0; m < MB; ++m) {
    const int f = lane + 64 * m, j = f - ic;
    const bool inb = j >= 0 && j < p;
    const double sc = __builtin_amdgcn_ldexp(1.0, 38 - min(o.E[(int64_t)g * PP + f], ozk::EMAX));
    double cen = 0.0, isc = 1.0;
    if constexpr (STD) {
      if (inb) {
        cen = a.center[j];
        isc = 1.0 / a.scale[j];
      }
    }
    uint32_t lo[8], hi[8];
#pragma unroll
    for (int r = 0; r < 8; ++r) {
      double v = (inb && r < left) ? a.X[(row0 + r) * p + j] : 0.0;
      if constexpr (STD) v = inb ? (v - cen) * isc : 0.0;
      if (ic && f == 0) v = 1.0;
      const double t = fma(v, sw[r] * sc, ozk::MAGIC);
      lo[r] = __double2loint(t);
      hi[r] = __double2hiint(t);
    }
    // plane d (d = 0 the top digit: byte 0 of the high dword; d = 1 .. 4:
    // byte 4 - d of the low dword) of rows 0-3 and 4-7
    auto pack = [&](const uint32_t* src, int k, int r0) -> uint32_t {
      const uint32_t sel = (uint32_t)k | ((uint32_t)(k + 4) << 8);
      const uint32_t p01 = __builtin_amdgcn_perm(src[r0 + 1], src[r0], sel);
      const uint32_t p23 = __builtin_amdgcn_perm(src[r0 + 3], src[r0 + 2], sel);
      return __builtin_amdgcn_perm(p23, p01, 0x05040100u) ^ 0x80808080u;
    };
    uint4 q0, q1;
    uint2 q2;
    q0.x = pack(hi, 0, 0);
    q0.y = pack(hi, 0, 4);
    q0.z = pack(lo, 3, 0);
    q0.w = pack(lo, 3, 4);
    q1.x = pack(lo, 2, 0);
    q1.y = pack(lo, 2, 4);
    q1.z = pack(lo, 1, 0);
    q1.w = pack(lo, 1, 4);
    q2.x = pack(lo, 0, 0);
    q2.y = pack(lo, 0, 4);
    uint4* dst = (uint4*)(rec + (int64_t)f * 16);
    dst[0] = q0;
    dst[PP] = q1;
    *(uint2*)(rec + 32 * PP + (int64_t)f * 8) = q2;
  }
}

// grid: (row group, tile) XCD-aware like wide_gram_kernel; 512 threads
__global__ __launch_bounds__(512, 1) void wide_oz_gram_kernel(const WideArgs a, const WideOzArgs o) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int NB = a.NB;
  const int TB = NB * (NB + 1) / 2;
  const int PP = kOzGT * NB;
  const int bid = blockIdx.x;
  const int xcd = bid & 7, j8 = bid >> 3;
  const int cl = j8 / TB, t = j8 - cl * TB;
  const int g = cl * 8 + xcd;
  if (g >= a.n_gchunks) return;
  const int part = a.gc_part[g];
  if (a.phase[part] != PHASE_F64) return;
  int I = 0;
  while ((I + 1) * (I + 2) / 2 <= t) ++I;
  const int J = t - I * (I + 1) / 2;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int qi = wid >> 2, qj = wid & 3;
  // strictly-upper block of a diagonal tile: DMA and barriers only
  const bool idle = I == J && 32 * qj >= 64 * qi + 64;
  const int nrows = __builtin_amdgcn_readfirstlane(a.gc_rows[g]);
  const int nsteps = (nrows + 31) / 32;
  // the row group's records: [maxblk][4 rowblocks][slice 0 (PP x 16 B) | slice 1
  // (PP x 16 B) | slice 2 (PP x 8 B)]; a step's panel for rowblock j is the
  // 5 KB of features 128 I .. 128 I + 127 (A) / 128 J .. (B) of its 3 slices
  const uintptr_t gbase = (uintptr_t)(o.D + (int64_t)g * o.maxblk * 4 * PP * kRec);
  const __amdgpu_buffer_rsrc_t dr =
      wv_rsrc(gbase, (uintptr_t)o.maxblk * 4 * PP * kRec);
  const int stepb = 4 * PP * kRec;
  // this wave's DMA pieces of a step: 40 x 1 KB (A: 20, B: 20), 5 per wave;
  // a rowblock's panel is 5 KB: slices 0 and 1 (2 KB each), slice 2 (1 KB)
  auto issue = [&](int s) {
    char* st = smem + (s % kOzStages) * 2 * kPanel;
#pragma unroll
    for (int i = 0; i < 5; ++i) {
      const int pc = wid * 5 + i;              // 0 .. 39
      const int ab = pc / kPieces, q = pc % kPieces;  // panel, piece within it
      const int j = q / 5, e = q % 5;         // rowblock, piece within its 5 KB
      const int sl = e >> 1;                   // slice (0, 1: two pieces; 2: one)
      const int k = e & 1;
      const int src = sl < 2 ? sl * PP * 16 + (ab ? J : I) * kOzGT * 16 + k * 1024
                             : 32 * PP + (ab ? J : I) * kOzGT * 8;
      const int soff = s * stepb + j * PP * kRec + src;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(
          dr, (wlds_void_t*)(st + ab * kPanel + j * kOzGT * kRec + e * 1024), 16, lane * 16,
          __builtin_amdgcn_readfirstlane(soff), 0, 0);
    }
  };
  oz_i4 acc[4][2][ozk::NL];
#pragma unroll
  for (int si = 0; si < 4; ++si)
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
      for (int k = 0; k < ozk::NL; ++k) acc[si][u][k] = oz_i4{0, 0, 0, 0};
  const int fi = lane & 15, gq = lane >> 4;  // lane group = rowblock of the step
  using u2 = unsigned __attribute__((ext_vector_type(2)));
  issue(0);
  if (nsteps > 1) issue(1);
  if (nsteps > 1)
    wv_wait_vmcnt<5>();
  else
    wv_wait_vmcnt<0>();
  ozk::barrier();
  for (int s = 0; s < nsteps; ++s) {
    if (s + 2 < nsteps) issue(s + 2);
    if (!idle) {
      const char* st = smem + (s % kOzStages) * 2 * kPanel;
      // slices of this lane group's rowblock: [3][128 features][16 B]
      const char* pa = st + gq * kOzGT * kRec + (64 * qi + fi) * 16;
      const char* pb = st + kPanel + gq * kOzGT * kRec + (32 * qj + fi) * 16;
      // slice 2 (plane 4): 8 bytes per feature after the two 2-KB slices
      const char* pa2 = st + gq * kOzGT * kRec + 4096 + (64 * qi + fi) * 8;
      const char* pb2 = st + kPanel + gq * kOzGT * kRec + 4096 + (32 * qj + fi) * 8;
      oz_i4 Bq[2][5];
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        u2 d[5];
#pragma unroll
        for (int b = 0; b < 4; ++b)
          d[b] = *(const u2*)(pb + u * 16 * 16 + (b >> 1) * kOzGT * 16 + 8 * (b & 1));
        d[4] = *(const u2*)(pb2 + u * 16 * 8);
        Bq[u][0] = oz_i4{(int)d[0].x, (int)d[0].y, 0, 0};
#pragma unroll
        for (int b = 1; b < 5; ++b) Bq[u][b] = oz_i4{(int)d[b].x, (int)d[b].y, (int)d[b - 1].x, (int)d[b - 1].y};
      }
#pragma unroll
      for (int si = 0; si < 4; ++si) {
        const char* ra = pa + si * 16 * 16;
        const oz_i4 a0 = *(const oz_i4*)ra, a2 = *(const oz_i4*)(ra + kOzGT * 16);
        const u2 a4v = *(const u2*)(pa2 + si * 16 * 8);
        const oz_i4 a4 = oz_i4{(int)a4v.x, (int)a4v.y, 0, 0};
#pragma unroll
        for (int u = 0; u < 2; ++u) {
          oz_i4* A = acc[si][u];
          A[0] = __builtin_amdgcn_mfma_i32_16x16x64_i8(a0, Bq[u][0], A[0], 0, 0, 0);
          A[1] = __builtin_amdgcn_mfma_i32_16x16x64_i8(a0, Bq[u][1], A[1], 0, 0, 0);
          A[2] = __builtin_amdgcn_mfma_i32_16x16x64_i8(a0, Bq[u][2], A[2], 0, 0, 0);
          A[3] = __builtin_amdgcn_mfma_i32_16x16x64_i8(a0, Bq[u][3], A[3], 0, 0, 0);
          A[4] = __builtin_amdgcn_mfma_i32_16x16x64_i8(a0, Bq[u][4], A[4], 0, 0, 0);
          A[2] = __builtin_amdgcn_mfma_i32_16x16x64_i8(a2, Bq[u][0], A[2], 0, 0, 0);
          A[3] = __builtin_amdgcn_mfma_i32_16x16x64_i8(a2, Bq[u][1], A[3], 0, 0, 0);
          A[4] = __builtin_amdgcn_mfma_i32_16x16x64_i8(a2, Bq[u][2], A[4], 0, 0, 0);
          A[4] = __builtin_amdgcn_mfma_i32_16x16x64_i8(a4, Bq[u][0], A[4], 0, 0, 0);
        }
      }
    }
    // step s+1 landed (s+2 may stay in flight); everyone done with stage s
    if (s + 2 < nsteps)
      wv_wait_vmcnt<5>();
    else
      wv_wait_vmcnt<0>();
    ozk::barrier();  // (not __syncthreads: its fence would drain step s+2's DMA)
  }
  if (idle) return;
  // C/D map of the i32 16x16 MFMA: row 4 (l >> 4) + r, column l & 15
  double* G = a.slab_G + ((int64_t)g * TB + t) * (kOzGT * kOzGT);
  const int* E = o.E + (int64_t)g * PP;
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int jl = 32 * qj + 16 * u + fi;
    const int ej = E[kOzGT * J + jl];
#pragma unroll
    for (int si = 0; si < 4; ++si)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int il = 64 * qi + 16 * si + 4 * gq + r;
        const double v = ozk::level_value(acc[si][u], r);
        const int ei = E[kOzGT * I + il];
        G[il * kOzGT + jl] = (ozk::digit_overflow(ei) || ozk::digit_overflow(ej))
                                 ? __builtin_nan("")
                                 : __builtin_amdgcn_ldexp(v, ei + ej - 12);
      }
  }
}

hipError_t launch_wide_oz_scale(const WideArgs& a, const WideOzArgs& o, hipStream_t s) {
  if (a.n_gchunks <= 0) return hipSuccess;
  hipLaunchKernelGGL(wide_oz_scale_kernel, dim3(a.n_gchunks), dim3(256), 0, s, a, o, kOzGT * a.NB);
  return hipGetLastError();
}

hipError_t launch_wide_oz_digits(const WideArgs& a, const WideOzArgs& o, bool standardize,
                                 hipStream_t s) {
  if (a.n_gchunks <= 0) return hipSuccess;
  const dim3 grid(a.n_gchunks, o.maxblk);
  auto go = [&](auto kern) { hipLaunchKernelGGL(kern, grid, dim3(256), 0, s, a, o); };
  switch (2 * a.NB) {
    case 4:
      standardize ? go(wide_oz_digits_kernel<4, true>) : go(wide_oz_digits_kernel<4, false>);
      break;
    case 6:
      standardize ? go(wide_oz_digits_kernel<6, true>) : go(wide_oz_digits_kernel<6, false>);
      break;
    case 8:
      standardize ? go(wide_oz_digits_kernel<8, true>) : go(wide_oz_digits_kernel<8, false>);
      break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

hipError_t launch_wide_oz_gram(const WideArgs& a, const WideOzArgs& o, hipStream_t s) {
  if (a.n_gchunks <= 0) return hipSuccess;
  const int TB = a.NB * (a.NB + 1) / 2;
  const int grid = ((a.n_gchunks + 7) / 8) * 8 * TB;
  const int lds = kOzStages * 2 * kPanel;
  hipError_t e = ensure_max_lds((const void*)wide_oz_gram_kernel, lds);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(wide_oz_gram_kernel, dim3(grid), dim3(512), lds, s, a, o);
  return hipGetLastError();
}

}  // namespace dlsa
