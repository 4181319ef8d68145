// Probe of v_mfma_f64_4x4x4_4b (gfx950): operand / result lane layout and
// issue rate against v_mfma_f64_16x16x4 (not part of the product; the exact
// pass's edge strip design depends on both).  Build + run:
//   hipcc --offload-arch=gfx950 -O3 tools/mfma4_probe.hip -o tools/_mfma4_probe && tools/_mfma4_probe
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <math.h>

#include <chrono>

typedef double d4 __attribute__((ext_vector_type(4)));

#define CHECK(x)                                                                     \
  do {                                                                               \
    hipError_t e_ = (x);                                                             \
    if (e_ != hipSuccess) {                                                          \
      printf("HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
      exit(1);                                                                       \
    }                                                                                \
  } while (0)

// out[la * 64 + lb] = bitmask of output lanes that are nonzero when only lane
// la of A and lane lb of B are 1
__global__ void k_layout(unsigned long long* out) {
  const int lane = threadIdx.x;
  for (int la = 0; la < 64; ++la)
    for (int lb = 0; lb < 64; ++lb) {
      const double a = lane == la ? 1.0 : 0.0;
      const double b = lane == lb ? 1.0 : 0.0;
      const double d = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, 0.0, 0, 0, 0);
      const unsigned long long m = __ballot(d != 0.0);
      if (lane == 0) out[la * 64 + lb] = m;
    }
}

// cbsz = 2 broadcast of A block `abid` to the 4 blocks: A[lane] = lane + 1,
// B = 1 at lane lb = 0 + 4 * 1 + 16 * 2 only; out[abid * 64 + lane] = D
template <int ABID>
__global__ void k_bcast(double* out) {
  const int lane = threadIdx.x;
  const double a = lane + 1.0;
  const double b = lane == 4 + 32 ? 1.0 : 0.0;
  out[ABID * 64 + lane] = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, 0.0, 2, ABID, 0);
}

// One 16x16 tile of A^T B over K = 4 rows (A, B: [4 rows][16 cols], lane =
// col + 16 row) as 4 v_mfma_f64_4x4x4_4b with B rotated by 4 s lanes inside
// each 16-lane row (DPP row_ror:4s).  out[s * 64 + lane] = D of rotation s.
__device__ __forceinline__ double dpp_ror(double v, int s) {
  int lo = __double2loint(v), hi = __double2hiint(v);
  if (s == 1) {
    lo = __builtin_amdgcn_mov_dpp(lo, 0x124, 0xF, 0xF, false);
    hi = __builtin_amdgcn_mov_dpp(hi, 0x124, 0xF, 0xF, false);
  } else if (s == 2) {
    lo = __builtin_amdgcn_mov_dpp(lo, 0x128, 0xF, 0xF, false);
    hi = __builtin_amdgcn_mov_dpp(hi, 0x128, 0xF, 0xF, false);
  } else if (s == 3) {
    lo = __builtin_amdgcn_mov_dpp(lo, 0x12C, 0xF, 0xF, false);
    hi = __builtin_amdgcn_mov_dpp(hi, 0x12C, 0xF, 0xF, false);
  }
  return __hiloint2double(hi, lo);
}
__global__ void k_rot(const double* A, const double* B, double* out) {
  const int lane = threadIdx.x;
  const double a = A[lane], b = B[lane];
  for (int s = 0; s < 4; ++s)
    out[s * 64 + lane] = __builtin_amdgcn_mfma_f64_4x4x4f64(a, dpp_ror(b, s), 0.0, 0, 0, 0);
}

// rate of the exact-pass pattern: per "k-step" 4 column operands, 3 DPP
// rotations each, 16 tiles x 4 rotations of 4x4x4_4b
__global__ __launch_bounds__(256) void k_rate_rot(double* out, int iters) {
  double a = threadIdx.x * 1e-3, b0 = 1.0 + threadIdx.x * 1e-4;
  double acc[16];
  for (int i = 0; i < 16; ++i) acc[i] = 0.0;
  for (int it = 0; it < iters; ++it) {
    const double b = b0 + it * 1e-9;
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const double br = dpp_ror(b, s);
#pragma unroll
      for (int i = 0; i < 4; ++i)
        acc[4 * s + i] = __builtin_amdgcn_mfma_f64_4x4x4f64(a + i, br, acc[4 * s + i], 0, 0, 0);
    }
  }
  double t = 0;
  for (int i = 0; i < 16; ++i) t += acc[i];
  out[blockIdx.x * 256 + threadIdx.x] = t;
}

template <int NACC>
__global__ __launch_bounds__(256) void k_rate4(double* out, int iters) {
  double a = threadIdx.x * 1e-3, b = 1.0 + threadIdx.x * 1e-4;
  double acc[NACC];
  for (int i = 0; i < NACC; ++i) acc[i] = 0.0;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < NACC; ++i) acc[i] = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, acc[i], 0, 0, 0);
  }
  double s = 0;
  for (int i = 0; i < NACC; ++i) s += acc[i];
  out[blockIdx.x * 256 + threadIdx.x] = s;
}

template <int NACC>
__global__ __launch_bounds__(256) void k_rate16(double* out, int iters) {
  double a = threadIdx.x * 1e-3, b = 1.0 + threadIdx.x * 1e-4;
  d4 acc[NACC];
  for (int i = 0; i < NACC; ++i) acc[i] = d4{0, 0, 0, 0};
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < NACC; ++i) acc[i] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[i], 0, 0, 0);
  }
  double s = 0;
  for (int i = 0; i < NACC; ++i) s += acc[i][0] + acc[i][3];
  out[blockIdx.x * 256 + threadIdx.x] = s;
}

int main() {
  unsigned long long* dm;
  CHECK(hipMalloc(&dm, 64 * 64 * 8));
  hipLaunchKernelGGL(k_layout, dim3(1), dim3(64), 0, 0, dm);
  CHECK(hipDeviceSynchronize());
  unsigned long long hm[64 * 64];
  CHECK(hipMemcpy(hm, dm, sizeof(hm), hipMemcpyDeviceToHost));
  // for every A lane la: the B lanes it pairs with and the output lanes
  for (int la = 0; la < 64; ++la) {
    printf("A lane %2d:", la);
    for (int lb = 0; lb < 64; ++lb)
      if (hm[la * 64 + lb]) {
        printf(" B%d->", lb);
        for (int o = 0; o < 64; ++o)
          if ((hm[la * 64 + lb] >> o) & 1ull) printf("D%d", o);
      }
    printf("\n");
  }
  {
    double* db;
    CHECK(hipMalloc(&db, 4 * 64 * 8));
    hipLaunchKernelGGL(k_bcast<0>, dim3(1), dim3(64), 0, 0, db);
    hipLaunchKernelGGL(k_bcast<1>, dim3(1), dim3(64), 0, 0, db);
    hipLaunchKernelGGL(k_bcast<2>, dim3(1), dim3(64), 0, 0, db);
    hipLaunchKernelGGL(k_bcast<3>, dim3(1), dim3(64), 0, 0, db);
    CHECK(hipDeviceSynchronize());
    double hb[256];
    CHECK(hipMemcpy(hb, db, sizeof(hb), hipMemcpyDeviceToHost));
    // expected with a broadcast of block abid: D lane (0 + 4 * 1 + 16 i) = A[i + 4 abid + 32] = i + 4 abid + 33
    for (int ab = 0; ab < 4; ++ab) {
      printf("cbsz=2 abid=%d:", ab);
      for (int o = 0; o < 64; ++o)
        if (hb[ab * 64 + o] != 0.0) printf(" D%d=%g", o, hb[ab * 64 + o]);
      printf("  (broadcast expects D4,D20,D36,D52 = %d,%d,%d,%d)\n", 33 + 4 * ab, 34 + 4 * ab,
             35 + 4 * ab, 36 + 4 * ab);
    }
  }
  {
    // rotation direction: which B column block feeds output block b under ror 4s
    double hA[64], hB[64];
    for (int l = 0; l < 64; ++l) {
      hA[l] = 1.0 + (l * 37 % 61) * 0.125;
      hB[l] = 2.0 + (l * 53 % 59) * 0.0625;
    }
    double *dA, *dB, *dO;
    CHECK(hipMalloc(&dA, 512));
    CHECK(hipMalloc(&dB, 512));
    CHECK(hipMalloc(&dO, 4 * 512));
    CHECK(hipMemcpy(dA, hA, 512, hipMemcpyHostToDevice));
    CHECK(hipMemcpy(dB, hB, 512, hipMemcpyHostToDevice));
    hipLaunchKernelGGL(k_rot, dim3(1), dim3(64), 0, 0, dA, dB, dO);
    CHECK(hipDeviceSynchronize());
    double hO[256];
    CHECK(hipMemcpy(hO, dO, sizeof(hO), hipMemcpyDeviceToHost));
    // full tile H[r][c] = sum_k A[r + 16k] B[c + 16k]
    for (int sign = -1; sign <= 1; sign += 2) {
      double maxerr = 0.0;
      for (int s = 0; s < 4; ++s)
        for (int l = 0; l < 64; ++l) {
          const int j = l & 3, b = (l >> 2) & 3, i = l >> 4;
          const int row = 4 * b + i, col = 4 * ((b + sign * s) & 3) + j;
          double ref = 0.0;
          for (int k = 0; k < 4; ++k) ref += hA[row + 16 * k] * hB[col + 16 * k];
          maxerr = fmax(maxerr, fabs(hO[s * 64 + l] - ref));
        }
      printf("rotation sign %+d (D lane j + 4b + 16i = H[4b + i][4((b %+d s) & 3) + j]): max err %g\n",
             sign, sign, maxerr);
    }
  }
  hipDeviceProp_t prop;
  CHECK(hipGetDeviceProperties(&prop, 0));
  const int grid = prop.multiProcessorCount * 4;  // 4 workgroups of 4 waves per CU: 4 waves/SIMD
  double* out;
  CHECK(hipMalloc(&out, (size_t)grid * 256 * 8));
  const int iters = 20000;
  auto run = [&](auto kern, int nacc, double flops_per_inst, const char* name) {
    hipLaunchKernelGGL(kern, dim3(grid), dim3(256), 0, 0, out, 10);
    CHECK(hipDeviceSynchronize());
    const auto t0 = std::chrono::steady_clock::now();
    hipLaunchKernelGGL(kern, dim3(grid), dim3(256), 0, 0, out, iters);
    CHECK(hipDeviceSynchronize());
    const double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    const double insts_per_simd = (double)iters * nacc * (grid * 4.0) / (prop.multiProcessorCount * 4.0);
    printf("%s: %.3f ms, %.1f TFLOP/s, %.2f ns per MFMA per SIMD\n", name, s * 1e3,
           insts_per_simd * prop.multiProcessorCount * 4.0 * flops_per_inst / s * 1e-12,
           s * 1e9 / insts_per_simd);
  };
  // waves per SIMD: grid of 1 / 2 / 4 workgroups (4 waves each) per CU
  for (int wps : {1, 2, 4}) {
    const int g = prop.multiProcessorCount * wps;
    auto runw = [&](auto kern, int nacc, double flops_per_inst, const char* name) {
      hipLaunchKernelGGL(kern, dim3(g), dim3(256), 0, 0, out, 10);
      CHECK(hipDeviceSynchronize());
      const auto t0 = std::chrono::steady_clock::now();
      hipLaunchKernelGGL(kern, dim3(g), dim3(256), 0, 0, out, iters);
      CHECK(hipDeviceSynchronize());
      const double sec = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
      const double per_simd = (double)iters * nacc * wps;
      printf("waves/SIMD %d %s: %.2f ns per MFMA per SIMD, %.1f TFLOP/s\n", wps, name,
             sec * 1e9 / per_simd, per_simd * prop.multiProcessorCount * 4.0 * flops_per_inst / sec * 1e-12);
    };
    runw(k_rate16<8>, 8, 2048.0, "f64 16x16x4 8acc");
    runw(k_rate16<16>, 16, 2048.0, "f64 16x16x4 16acc");
    runw(k_rate4<16>, 16, 512.0, "f64 4x4x4_4b 16acc");
    runw(k_rate4<32>, 32, 512.0, "f64 4x4x4_4b 32acc");
    runw(k_rate_rot, 16, 512.0, "f64 4x4x4_4b + DPP rot");
  }
  for (int rep = 0; rep < 1; ++rep) {  // alternate, so clock ramp-up shows in rep 0 only
    run(k_rate16<8>, 8, 2048.0, "f64 16x16x4 8acc");
    run(k_rate4<8>, 8, 512.0, "f64 4x4x4_4b 8acc");
    run(k_rate4<16>, 16, 512.0, "f64 4x4x4_4b 16acc");
    run(k_rate_rot, 16, 512.0, "f64 4x4x4_4b + DPP rotations (16 MFMA, 3x2 dpp per 16)");
  }
  return 0;
}
