// Micro-probes of the gfx950 facts the pass design depends on (not part of
// the product; built by tools/probe.sh, run on the GPU box):
//   mfma64   back-to-back v_mfma_f64_16x16x4_f64, independent accumulators
//   mfma32   back-to-back v_mfma_f32_16x16x4_f32
//   valu64   back-to-back independent v_fma_f64
//   mix      MFMA-f64 waves and VALU-f64 waves sharing the SIMDs
//   stream   plain global_load_dwordx4 read of a large buffer (grid-stride)
//   rowstream  row-major X read as 16 lanes x 8 B per row (the MFMA operand map)
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#include <chrono>

typedef double d4 __attribute__((ext_vector_type(4)));
typedef float f4 __attribute__((ext_vector_type(4)));

#define CHECK(x)                                                              \
  do {                                                                        \
    hipError_t e_ = (x);                                                      \
    if (e_ != hipSuccess) {                                                   \
      printf("HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
      exit(1);                                                                \
    }                                                                         \
  } while (0)

constexpr int NACC = 8;

__global__ __launch_bounds__(256) void k_mfma64(double* out, int iters, int valu_waves) {
  const int wid = threadIdx.x >> 6;
  double a = threadIdx.x * 1e-3, b = 1.0 + threadIdx.x * 1e-4;
  if (wid < (4 - valu_waves) || valu_waves == 0) {
    d4 acc[NACC];
    for (int i = 0; i < NACC; ++i) acc[i] = d4{0, 0, 0, 0};
    for (int it = 0; it < iters; ++it) {
#pragma unroll
      for (int i = 0; i < NACC; ++i) acc[i] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[i], 0, 0, 0);
    }
    double s = 0;
    for (int i = 0; i < NACC; ++i) s += acc[i][0] + acc[i][3];
    out[blockIdx.x * 256 + threadIdx.x] = s;
  } else {
    double v[8];
    for (int i = 0; i < 8; ++i) v[i] = a + i;
    for (int it = 0; it < iters; ++it) {
#pragma unroll
      for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int i = 0; i < 8; ++i) v[i] = fma(v[i], b, a);
    }
    double s = 0;
    for (int i = 0; i < 8; ++i) s += v[i];
    out[blockIdx.x * 256 + threadIdx.x] = s;
  }
}

template <int NA>
__global__ __launch_bounds__(256) void k_mfma64n(double* out, int iters) {
  double a = threadIdx.x * 1e-3, b = 1.0 + threadIdx.x * 1e-4;
  d4 acc[NA];
  for (int i = 0; i < NA; ++i) acc[i] = d4{0, 0, 0, 0};
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < NA; ++i) acc[i] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[i], 0, 0, 0);
  }
  double s = 0;
  for (int i = 0; i < NA; ++i) s += acc[i][0] + acc[i][3];
  out[blockIdx.x * 256 + threadIdx.x] = s;
}

// U dwordx4 loads in flight per lane per iteration, wave-contiguous 1 KiB pieces
template <int U>
__global__ __launch_bounds__(256) void k_streamu(const double* __restrict__ X, size_t n16,
                                                 double* out) {
  typedef double d2 __attribute__((ext_vector_type(2)));
  const d2* p = (const d2*)X;
  const size_t lane = threadIdx.x & 63;
  const size_t wave = (size_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const size_t nwaves = (size_t)gridDim.x * 4;
  double s = 0;
  for (size_t base = wave * 64 * U; base + 64 * U <= n16; base += nwaves * 64 * U) {
    d2 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = __builtin_nontemporal_load(p + base + 64 * u + lane);
#pragma unroll
    for (int u = 0; u < U; ++u) s += v[u].x;
  }
  if (s == 12345.678) out[0] = s;
}

// per-wave contiguous chunk (like a partition chunk), U dwordx4 loads in flight
template <int U>
__global__ __launch_bounds__(256) void k_streamchunk(const double* __restrict__ X, size_t n16_per_wave,
                                                     double* out) {
  typedef double d2 __attribute__((ext_vector_type(2)));
  const size_t lane = threadIdx.x & 63;
  const size_t wave = (size_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const d2* p = (const d2*)X + wave * n16_per_wave;
  double s = 0;
  for (size_t base = 0; base + 64 * U <= n16_per_wave; base += 64 * U) {
    d2 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = __builtin_nontemporal_load(p + base + 64 * u + lane);
#pragma unroll
    for (int u = 0; u < U; ++u) s += v[u].x;
  }
  if (s == 12345.678) out[0] = s;
}

typedef __attribute__((address_space(3))) void lds_void_t;
typedef const __attribute__((address_space(1))) void gbl_void_t;
template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// LDS-DMA ring: W waves per workgroup, each block = PIECES 1 KiB pieces split
// over the waves, NSLOT slots, optional barrier per block (coop) or none
// (per-wave rings: every wave streams its own chunk into its own ring).
template <int W, int PIECES, int NSLOT, bool COOP>
__global__ __launch_bounds__(64 * W) void k_dma(const double* __restrict__ X, size_t bytes_per_wg,
                                                double* out) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const char* base = (const char*)X + (size_t)blockIdx.x * bytes_per_wg;
  constexpr int D = COOP ? PIECES / W : PIECES;  // pieces per wave per block
  constexpr int SLOT = (COOP ? PIECES : PIECES * W) * 1024;
  const size_t blk_bytes = (size_t)PIECES * 1024 * (COOP ? 1 : W);
  const int nb = (int)(bytes_per_wg / blk_bytes);
  auto issue = [&](int b) {
    const int bb = b < nb ? b : nb - 1;
    char* sl = smem + (b % NSLOT) * SLOT;
#pragma unroll
    for (int i = 0; i < D; ++i) {
      const int j = COOP ? (wid + W * i) : (wid * PIECES + i);
      const char* src = base + (size_t)bb * blk_bytes + (size_t)j * 1024 + lane * 16;
      __builtin_amdgcn_global_load_lds((gbl_void_t*)src, (lds_void_t*)(sl + j * 1024), 16, 0, 0);
    }
  };
#pragma unroll
  for (int b = 0; b < NSLOT - 1; ++b) issue(b);
  double s = 0;
  for (int b = 0; b < nb; ++b) {
    wait_vmcnt<(NSLOT - 2) * D>();
    if (COOP) __syncthreads();
    issue(b + NSLOT - 1);
    s += ((const double*)(smem + (b % NSLOT) * SLOT))[threadIdx.x];
  }
  wait_vmcnt<0>();
  if (s == 12345.678) out[0] = s;
}

// the real coop pass's stream structure: 32-row blocks of p = 100 (25 600 B),
// 16-B aligned pieces, a y dword DMA per wave, 2 barriers per block (VAR bits:
// 1 = no y DMA, 2 = one barrier, 4 = pieces rounded to 1 KiB-aligned starts)
template <int VAR>
__global__ __launch_bounds__(256) void k_coopstream(const double* __restrict__ X, const double* __restrict__ Y,
                                                    long rows_per_wg, int p, int nslot, double* out) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const long row0 = (long)blockIdx.x * rows_per_wg;
  const int RB = 32;
  const int nb = (int)(rows_per_wg / RB);
  const int npieces = (RB * p * 8 + 16 + 1023) / 1024;
  const int d = (npieces + 3) / 4;
  const int slot_bytes = 16 + d * 4 * 1024 + 1024;
  auto issue = [&](int blk) {
    const int bb = blk < nb ? blk : nb - 1;
    char* sbase = smem + (blk % nslot) * slot_bytes;
    uintptr_t start = (uintptr_t)(X + (row0 + (long)bb * RB) * p);
    if (VAR & 4) start &= ~(uintptr_t)1023;
    const uintptr_t al = start & ~(uintptr_t)15;
    for (int i = 0; i < d; ++i) {
      int j = wid + 4 * i;
      const int jj = j < npieces ? j : npieces - 1;
      uintptr_t src = al + (uintptr_t)jj * 1024 + (uintptr_t)lane * 16;
      __builtin_amdgcn_global_load_lds((gbl_void_t*)src, (lds_void_t*)(sbase + 16 + j * 1024), 16, 0, 0);
    }
    if (!(VAR & 1)) {
      uintptr_t ys = (uintptr_t)(Y + row0 + (long)bb * RB) + (uintptr_t)lane * 4;
      __builtin_amdgcn_global_load_lds((gbl_void_t*)ys, (lds_void_t*)(sbase + 16 + d * 4096), 4, 0, 0);
    }
  };
  for (int b = 0; b < nslot - 1; ++b) issue(b);
  double s = 0;
  for (int b = 0; b < nb; ++b) {
    if (VAR & 1) {
      if (nslot == 5) wait_vmcnt<3 * 7>(); else wait_vmcnt<1 * 7>();
    } else {
      if (nslot == 5) wait_vmcnt<3 * 8>(); else wait_vmcnt<1 * 8>();
    }
    __syncthreads();
    issue(b + nslot - 1);
    s += ((const double*)(smem + (b % nslot) * slot_bytes))[threadIdx.x];
    if (!(VAR & 2)) __syncthreads();
  }
  wait_vmcnt<0>();
  if (s == 12345.678) out[0] = s;
}

__global__ __launch_bounds__(256) void k_mfma32(double* out, int iters) {
  float a = threadIdx.x * 1e-3f, b = 1.0f + threadIdx.x * 1e-4f;
  f4 acc[NACC];
  for (int i = 0; i < NACC; ++i) acc[i] = f4{0, 0, 0, 0};
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < NACC; ++i) acc[i] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc[i], 0, 0, 0);
  }
  double s = 0;
  for (int i = 0; i < NACC; ++i) s += acc[i][0] + acc[i][3];
  out[blockIdx.x * 256 + threadIdx.x] = s;
}

__global__ __launch_bounds__(256) void k_stream(const double* __restrict__ X, size_t n16,
                                                double* out) {
  typedef double d2 __attribute__((ext_vector_type(2)));
  const d2* p = (const d2*)X;
  double s = 0;
  for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n16; i += (size_t)gridDim.x * 256) {
    d2 v = __builtin_nontemporal_load(p + i);
    s += v.x;
  }
  if (s == 12345.678) out[0] = s;
}

// one wave per chunk of rows, 4 rows per k-step, lane l reads feature 16c + (l & 15)
// of row 4s + (l >> 4), NT column tiles, U k-steps of loads in flight
template <int NT, int U>
__global__ __launch_bounds__(256) void k_rowstream(const double* __restrict__ X, int p,
                                                   long rows_per_wave, double* out) {
  const int lane = threadIdx.x & 63;
  const long wave = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  const long r0 = wave * rows_per_wave;
  const int fl = lane & 15, q = lane >> 4;
  double s = 0;
  for (long s0 = 0; s0 < rows_per_wave; s0 += 4 * U) {
    double v[U][NT];
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int c = 0; c < NT; ++c) {
        const int f = 16 * c + fl;
        v[u][c] = __builtin_nontemporal_load(X + (r0 + s0 + 4 * u + q) * p + (f < p ? f : 0));
      }
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int c = 0; c < NT; ++c) s += v[u][c];
  }
  if (s == 12345.678) out[0] = s;
}

static double time_ms(hipEvent_t a, hipEvent_t b) {
  float ms;
  CHECK(hipEventElapsedTime(&ms, a, b));
  return ms;
}

int main(int argc, char** argv) {
  int cus = 256;
  double* out;
  CHECK(hipMalloc(&out, 1 << 26));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  const int iters = 4000;
  // clock estimate from a long MFMA run is not possible directly: report
  // cycles at an assumed clock and the raw per-SIMD instruction rate.
  for (int wpc : {4, 8}) {  // waves per CU -> waves per SIMD = wpc / 4
    const int grid = cus * wpc / 4;
    hipLaunchKernelGGL(k_mfma64, dim3(grid), dim3(256), 0, 0, out, 10, 0);
    CHECK(hipEventRecord(e0));
    hipLaunchKernelGGL(k_mfma64, dim3(grid), dim3(256), 0, 0, out, iters, 0);
    CHECK(hipEventRecord(e1));
    CHECK(hipEventSynchronize(e1));
    double ms = time_ms(e0, e1);
    double n_mfma = (double)grid * 4 * iters * NACC;
    double per_simd = n_mfma / (cus * 4);
    printf("mfma64 waves/SIMD=%d: %.3f ms, %.1f TFLOP/s, %.2f ns per MFMA per SIMD\n", wpc / 4,
           ms, n_mfma * 2048 / (ms * 1e-3) / 1e12, ms * 1e6 / per_simd);
    hipLaunchKernelGGL(k_mfma32, dim3(grid), dim3(256), 0, 0, out, 10);
    CHECK(hipEventRecord(e0));
    hipLaunchKernelGGL(k_mfma32, dim3(grid), dim3(256), 0, 0, out, iters);
    CHECK(hipEventRecord(e1));
    CHECK(hipEventSynchronize(e1));
    ms = time_ms(e0, e1);
    printf("mfma32 waves/SIMD=%d: %.3f ms, %.1f TFLOP/s, %.2f ns per MFMA per SIMD\n", wpc / 4,
           ms, n_mfma * 2048 / (ms * 1e-3) / 1e12, ms * 1e6 / per_simd);
  }

  for (int wps : {1, 2, 4}) {
    const int grid = cus * wps;
    auto run = [&](auto kern, int na, const char* nm) {
      hipLaunchKernelGGL(kern, dim3(grid), dim3(256), 0, 0, out, 10);
      CHECK(hipEventRecord(e0));
      hipLaunchKernelGGL(kern, dim3(grid), dim3(256), 0, 0, out, 2000);
      CHECK(hipEventRecord(e1));
      CHECK(hipEventSynchronize(e1));
      double ms = time_ms(e0, e1);
      double n_mfma = (double)grid * 4 * 2000 * na;
      printf("%s waves/SIMD=%d: %.3f ms, %.1f TFLOP/s, %.2f ns per MFMA per SIMD\n", nm, wps, ms,
             n_mfma * 2048 / (ms * 1e-3) / 1e12, ms * 1e6 / (n_mfma / (cus * 4)));
    };
    run(k_mfma64n<16>, 16, "mfma64 16acc");
    run(k_mfma64n<32>, 32, "mfma64 32acc");
  }
  // VALU f64 alone (all 4 waves VALU), then the mix (2 waves per SIMD: one
  // MFMA wave + one VALU wave per SIMD -> grid with 8 waves/CU, half of each kind)
  {
    const int grid = cus;  // 4 waves/CU, all VALU
    hipLaunchKernelGGL(k_mfma64, dim3(grid), dim3(256), 0, 0, out, 10, 4);
    CHECK(hipEventRecord(e0));
    hipLaunchKernelGGL(k_mfma64, dim3(grid), dim3(256), 0, 0, out, iters, 4);
    CHECK(hipEventRecord(e1));
    CHECK(hipEventSynchronize(e1));
    double ms = time_ms(e0, e1);
    double n_fma = (double)grid * 256 * iters * 32;
    printf("valu64 alone 1 wave/SIMD: %.3f ms, %.1f TFLOP/s\n", ms, n_fma * 2 / (ms * 1e-3) / 1e12);
    // mix: 2 blocks per CU; block layout: waves 0,1 MFMA, waves 2,3 VALU (valu_waves=2)
    const int gridm = cus * 2;
    hipLaunchKernelGGL(k_mfma64, dim3(gridm), dim3(256), 0, 0, out, 10, 2);
    CHECK(hipEventRecord(e0));
    hipLaunchKernelGGL(k_mfma64, dim3(gridm), dim3(256), 0, 0, out, iters, 2);
    CHECK(hipEventRecord(e1));
    CHECK(hipEventSynchronize(e1));
    ms = time_ms(e0, e1);
    double n_mfma = (double)gridm * 2 * iters * NACC;
    double n_fma2 = (double)gridm * 128 * iters * 32;
    printf("mix (half MFMA waves, half VALU waves, 2 waves/SIMD): %.3f ms, MFMA %.1f TF + VALU %.1f TF\n",
           ms, n_mfma * 2048 / (ms * 1e-3) / 1e12, n_fma2 * 2 / (ms * 1e-3) / 1e12);
  }
  // streaming
  size_t bytes = (size_t)80 << 30;
  double* X;
  if (hipMalloc(&X, bytes) != hipSuccess) {
    bytes = (size_t)16 << 30;
    CHECK(hipMalloc(&X, bytes));
  }
  CHECK(hipMemset(X, 0, bytes));
  for (int wpc : {8, 16, 32}) {
    const int grid = cus * wpc / 4;
    hipLaunchKernelGGL(k_stream, dim3(grid), dim3(256), 0, 0, X, bytes / 16, out);
    CHECK(hipEventRecord(e0));
    hipLaunchKernelGGL(k_stream, dim3(grid), dim3(256), 0, 0, X, bytes / 16, out);
    CHECK(hipEventRecord(e1));
    CHECK(hipEventSynchronize(e1));
    double ms = time_ms(e0, e1);
    printf("stream dwordx4 %d waves/CU: %.3f ms, %.0f GB/s\n", wpc, ms, bytes / (ms * 1e-3) / 1e9);
  }

  for (int wpc : {4, 8, 16}) {
    const int grid = cus * wpc / 4;
    auto run = [&](auto kern, const char* nm) {
      hipLaunchKernelGGL(kern, dim3(grid), dim3(256), 0, 0, X, bytes / 16, out);
      CHECK(hipEventRecord(e0));
      hipLaunchKernelGGL(kern, dim3(grid), dim3(256), 0, 0, X, bytes / 16, out);
      CHECK(hipEventRecord(e1));
      CHECK(hipEventSynchronize(e1));
      double ms = time_ms(e0, e1);
      printf("%s %d waves/CU: %.3f ms, %.0f GB/s\n", nm, wpc, ms, bytes / (ms * 1e-3) / 1e9);
    };
    run(k_streamu<4>, "streamu U=4");
    run(k_streamu<8>, "streamu U=8");
    run(k_streamu<16>, "streamu U=16");
    const size_t waves = (size_t)cus * wpc * 5;
    const size_t per = bytes / 16 / waves / 1024 * 1024;
    auto runc = [&](auto kern, const char* nm) {
      hipLaunchKernelGGL(kern, dim3(waves / 4), dim3(256), 0, 0, X, per, out);
      CHECK(hipEventRecord(e0));
      hipLaunchKernelGGL(kern, dim3(waves / 4), dim3(256), 0, 0, X, per, out);
      CHECK(hipEventRecord(e1));
      CHECK(hipEventSynchronize(e1));
      double ms = time_ms(e0, e1);
      printf("%s %d waves/CU (5 rounds of per-wave chunks): %.3f ms, %.0f GB/s\n", nm, wpc, ms,
             (double)waves * per * 16 / (ms * 1e-3) / 1e9);
    };
    runc(k_streamchunk<8>, "streamchunk U=8");
    runc(k_streamchunk<16>, "streamchunk U=16");
  }

  {
    auto rund = [&](auto kern, int wpb, size_t lds, int wgs_per_cu, const char* nm) {
      CHECK(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
      const int nwg = cus * wgs_per_cu * 5;
      const size_t per = bytes / nwg / (64 * 1024) * (64 * 1024);
      hipLaunchKernelGGL(kern, dim3(nwg), dim3(64 * wpb), lds, 0, X, per, out);
      CHECK(hipEventRecord(e0));
      hipLaunchKernelGGL(kern, dim3(nwg), dim3(64 * wpb), lds, 0, X, per, out);
      CHECK(hipEventRecord(e1));
      CHECK(hipEventSynchronize(e1));
      CHECK(hipGetLastError());
      double ms = time_ms(e0, e1);
      printf("%s: %.3f ms, %.0f GB/s\n", nm, ms, (double)nwg * per / (ms * 1e-3) / 1e9);
    };
    rund(k_dma<4, 24, 5, true>, 4, 5 * 24 * 1024, 1, "dma coop W4 24KiB blocks nslot5 1 WG/CU");
    rund(k_dma<4, 24, 3, true>, 4, 3 * 24 * 1024, 2, "dma coop W4 24KiB blocks nslot3 2 WG/CU");
    rund(k_dma<4, 8, 8, true>, 4, 8 * 8 * 1024, 2, "dma coop W4 8KiB blocks nslot8 2 WG/CU");
    rund(k_dma<8, 24, 6, true>, 8, 6 * 24 * 1024, 1, "dma coop W8 24KiB blocks nslot6 1 WG/CU");
    rund(k_dma<1, 8, 4, false>, 1, 4 * 8 * 1024, 4, "dma per-wave 8KiB blocks nslot4 4 waves/CU");
    rund(k_dma<1, 8, 4, false>, 1, 4 * 8 * 1024, 4, "dma per-wave 8KiB blocks nslot4 4 waves/CU");
    rund(k_dma<1, 4, 4, false>, 1, 4 * 4 * 1024, 8, "dma per-wave 4KiB blocks nslot4 8 waves/CU");
    rund(k_dma<1, 2, 6, false>, 1, 6 * 2 * 1024, 8, "dma per-wave 2KiB blocks nslot6 8 waves/CU");
  }

  {
    double* Y;
    CHECK(hipMalloc(&Y, (size_t)1 << 30));
    const int p = 100;
    const long rows = (long)(bytes / (8 * p));
    const long nwg = 1280;
    const long rpw = rows / nwg / 32 * 32;
    auto runc = [&](auto kern, int nslot, const char* nm) {
      CHECK(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
      const size_t lds = (size_t)nslot * (16 + 7 * 4 * 1024 + 1024);
      hipLaunchKernelGGL(kern, dim3(nwg), dim3(256), lds, 0, X, Y, rpw, p, nslot, out);
      CHECK(hipEventRecord(e0));
      hipLaunchKernelGGL(kern, dim3(nwg), dim3(256), lds, 0, X, Y, rpw, p, nslot, out);
      CHECK(hipEventRecord(e1));
      CHECK(hipEventSynchronize(e1));
      CHECK(hipGetLastError());
      double ms = time_ms(e0, e1);
      printf("%s nslot=%d: %.3f ms, %.0f GB/s\n", nm, nslot, ms, (double)nwg * rpw * (8 * p + 8) / (ms * 1e-3) / 1e9);
    };
    for (int ns : {5, 3}) {
      runc(k_coopstream<0>, ns, "coopstream as-is");
      runc(k_coopstream<1>, ns, "coopstream no-y");
      runc(k_coopstream<2>, ns, "coopstream 1-barrier");
      runc(k_coopstream<4>, ns, "coopstream 1KiB-aligned");
      runc(k_coopstream<7>, ns, "coopstream all three");
    }
  }
  {
    const int p = 100;
    const long rows = (long)(bytes / (8 * p));
    for (int wpc : {8, 16}) {
      const long waves = (long)cus * wpc * 4;  // 4 rounds of waves
      long rpw = rows / waves / 16 * 16;
      hipLaunchKernelGGL((k_rowstream<7, 4>), dim3(waves / 4), dim3(256), 0, 0, X, p, rpw, out);
      CHECK(hipEventRecord(e0));
      hipLaunchKernelGGL((k_rowstream<7, 4>), dim3(waves / 4), dim3(256), 0, 0, X, p, rpw, out);
      CHECK(hipEventRecord(e1));
      CHECK(hipEventSynchronize(e1));
      double ms = time_ms(e0, e1);
      double b = (double)waves * rpw * p * 8;
      printf("rowstream p=100 (16 lanes x 8 B per row, 4 k-steps in flight) %d waves/CU: %.3f ms, %.0f GB/s\n",
             wpc, ms, b / (ms * 1e-3) / 1e9);
      hipLaunchKernelGGL((k_rowstream<7, 8>), dim3(waves / 4), dim3(256), 0, 0, X, p, rpw, out);
      CHECK(hipEventRecord(e0));
      hipLaunchKernelGGL((k_rowstream<7, 8>), dim3(waves / 4), dim3(256), 0, 0, X, p, rpw, out);
      CHECK(hipEventRecord(e1));
      CHECK(hipEventSynchronize(e1));
      ms = time_ms(e0, e1);
      printf("rowstream p=100 8 k-steps in flight %d waves/CU: %.3f ms, %.0f GB/s\n", wpc, ms,
             b / (ms * 1e-3) / 1e9);
    }
  }
  CHECK(hipFree(X));
  CHECK(hipFree(out));
  return 0;
}
