// fp64 MFMA issue rate on the MI355X with toggling (random) operands and the
// in-kernel clock (not part of the product; the measurement behind the
// exact pass's roofline in DESIGN.md 4.1b).  tools/mfma4_probe.hip measured
// the rates with operands constant across iterations; here every MFMA takes
// a different pair out of 8 random operand registers and the accumulators
// carry random sums, as in the exact pass.  Each workgroup stamps
// s_memtime / s_memrealtime around its loop: clock = d(memtime) / d(realtime)
// x 100 MHz (median over workgroups).
//
//   hipcc --offload-arch=gfx950 -O3 -o tools/_mfma_rate_probe tools/mfma_rate_probe.hip
#include <hip/hip_runtime.h>
#include <stdio.h>

#include <algorithm>
#include <chrono>
#include <vector>

#define CHECK(x)                                                              \
  do {                                                                        \
    hipError_t e_ = (x);                                                      \
    if (e_ != hipSuccess) {                                                   \
      printf("HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
      return 1;                                                               \
    }                                                                         \
  } while (0)

typedef double d4 __attribute__((ext_vector_type(4)));

// 8 random operands per lane (a, b), NACC accumulators; every inner step of
// 8 uses pair ((i + u) & 7, (3 i + u) & 7): different data every MFMA
// operand pattern of consecutive MFMAs: 0 = both A and B change every MFMA,
// 1 = same A for runs of NACC (B changes), 2 = same B (A changes), 3 = same A
// and B every MFMA (tools/mfma4_probe.hip's pattern)
template <int NACC, bool BIG, bool RANDOM, int PAT = 0>
__global__ __launch_bounds__(256) void k_rate(const double* src, double* out, long long* stamps,
                                              int iters) {
  const int lane = threadIdx.x;
  double a[8], b[8];
#pragma unroll
  for (int u = 0; u < 8; ++u) {
    a[u] = RANDOM ? src[(blockIdx.x * 256 + lane) * 16 + u] : 1e-3 * lane;
    b[u] = RANDOM ? src[(blockIdx.x * 256 + lane) * 16 + 8 + u] : 1.0 + 1e-4 * lane;
  }
  d4 acc[BIG ? NACC : 1];
  double acc4[BIG ? 1 : NACC];
#pragma unroll
  for (int i = 0; i < (BIG ? NACC : 1); ++i) acc[i] = d4{a[i & 7], b[i & 7], a[(i + 1) & 7], 0.0};
#pragma unroll
  for (int i = 0; i < (BIG ? 1 : NACC); ++i) acc4[i] = a[i & 7];
  __syncthreads();
  const long long t0 = __builtin_amdgcn_s_memtime();
  const long long r0 = __builtin_amdgcn_s_memrealtime();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int u = 0; u < 8; ++u)
#pragma unroll
      for (int i = 0; i < NACC; ++i) {
        const int ia = PAT == 0 ? (i + u) & 7 : PAT == 1 ? u : PAT == 2 ? (i + u) & 7 : 0;
        const int ib = PAT == 0 ? (3 * i + u) & 7 : PAT == 1 ? (3 * i + u) & 7 : PAT == 2 ? u : 0;
        if constexpr (BIG)
          acc[i] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[ia], b[ib], acc[i], 0, 0, 0);
        else
          acc4[i] = __builtin_amdgcn_mfma_f64_4x4x4f64(a[ia], b[ib], acc4[i], 0, 0, 0);
      }
  }
  const long long t1 = __builtin_amdgcn_s_memtime();
  const long long r1 = __builtin_amdgcn_s_memrealtime();
  double s = 0.0;
#pragma unroll
  for (int i = 0; i < (BIG ? NACC : 1); ++i) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
#pragma unroll
  for (int i = 0; i < (BIG ? 1 : NACC); ++i) s += acc4[i];
  out[blockIdx.x * 256 + lane] = s;
  if (lane == 0) {
    stamps[blockIdx.x * 2] = t1 - t0;
    stamps[blockIdx.x * 2 + 1] = r1 - r0;
  }
}

int main() {
  hipDeviceProp_t prop;
  CHECK(hipGetDeviceProperties(&prop, 0));
  const int cus = prop.multiProcessorCount;
  const int maxg = cus * 4;
  std::vector<double> h((size_t)maxg * 256 * 16);
  unsigned long long z = 0x9E3779B97F4A7C15ull;
  for (auto& v : h) {
    z ^= z << 13;
    z ^= z >> 7;
    z ^= z << 17;
    v = (double)(z >> 11) * 0x1.0p-53 - 0.5;
  }
  double *src, *out;
  long long* st;
  CHECK(hipMalloc(&src, h.size() * 8));
  CHECK(hipMalloc(&out, (size_t)maxg * 256 * 8));
  CHECK(hipMalloc(&st, (size_t)maxg * 2 * 8));
  CHECK(hipMemcpy(src, h.data(), h.size() * 8, hipMemcpyHostToDevice));
  const int iters = 4000;
  auto run = [&](auto kern, int nacc, double flops, int wps, const char* name) -> int {
    const int g = cus * wps;  // wps workgroups of 4 waves per CU = wps waves per SIMD
    hipLaunchKernelGGL(kern, dim3(g), dim3(256), 0, 0, src, out, st, 50);
    CHECK(hipDeviceSynchronize());
    for (int warm = 0; warm < 3; ++warm)  // ~1 s of back-to-back launches first (DVFS)
      hipLaunchKernelGGL(kern, dim3(g), dim3(256), 0, 0, src, out, st, iters);
    CHECK(hipDeviceSynchronize());
    const auto t0 = std::chrono::steady_clock::now();
    hipLaunchKernelGGL(kern, dim3(g), dim3(256), 0, 0, src, out, st, iters);
    CHECK(hipDeviceSynchronize());
    const double sec = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    std::vector<long long> hs((size_t)g * 2);
    CHECK(hipMemcpy(hs.data(), st, hs.size() * 8, hipMemcpyDeviceToHost));
    std::vector<double> clk(g);
    for (int i = 0; i < g; ++i) clk[i] = (double)hs[2 * i] / (double)hs[2 * i + 1] * 0.1;  // GHz
    std::sort(clk.begin(), clk.end());
    const double per_simd = (double)iters * 8 * nacc * wps;
    const double tf = per_simd * cus * 4.0 * flops / sec * 1e-12;
    printf("%-34s waves/SIMD %d: %6.2f ns per MFMA per SIMD, %5.1f TFLOP/s, clock %.2f GHz "
           "(%.1f cycles per MFMA)\n",
           name, wps, sec * 1e9 / per_simd, tf, clk[g / 2], sec * 1e9 / per_simd * clk[g / 2]);
    return 0;
  };
  for (int wps : {2}) {
    if (run(k_rate<8, true, true, 1>, 8, 2048.0, wps, "f64 16x16x4 same A in runs of 8")) return 1;
    if (run(k_rate<8, true, true, 2>, 8, 2048.0, wps, "f64 16x16x4 same B in runs of 8")) return 1;
    if (run(k_rate<8, true, true, 3>, 8, 2048.0, wps, "f64 16x16x4 same A and B always")) return 1;
    if (run(k_rate<12, true, true, 0>, 12, 2048.0, wps, "f64 16x16x4 12 acc, A and B change")) return 1;
    if (run(k_rate<12, true, true, 1>, 12, 2048.0, wps, "f64 16x16x4 12 acc, same A runs of 12")) return 1;
  }
  for (int wps : {1, 2}) {
    if (run(k_rate<8, true, false>, 8, 2048.0, wps, "f64 16x16x4 constant operands")) return 1;
    if (run(k_rate<8, true, true>, 8, 2048.0, wps, "f64 16x16x4 random operands")) return 1;
    if (run(k_rate<16, false, false>, 16, 512.0, wps, "f64 4x4x4_4b constant operands")) return 1;
    if (run(k_rate<16, false, true>, 16, 512.0, wps, "f64 4x4x4_4b random operands")) return 1;
  }
  return 0;
}
