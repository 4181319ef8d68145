// Row repartitioning in HBM: the Spark `repartition(K, "partition_id")` +
// `groupby("partition_id")` that hands each UDF call one partition's rows
// (projects/logistic_dlsa.py:303-325; partition ids from
// monotonically_increasing_id() % K, :243-245), as a stable counting sort:
//
//   1. part_count_kernel    per block of R input rows: histogram of the K ids
//                           (LDS atomics) -> counts[b, k]; ids outside [0, K)
//                           are counted as bad
//   2. part_scan_kernel     per partition: exclusive scan over blocks (block
//                           order = input order: the sort is stable); then
//                           the partition offsets (one workgroup)
//   3. part_scatter_kernel  per block: wave 0 ranks the block's rows 64 at a
//                           time (one ballot per distinct id in a segment)
//                           into destination rows; then every wave copies
//                           whole rows of each array (8-byte words when the
//                           row width allows, bytes otherwise)
//
// HBM-bound byte movement: each array is read once and written once
// (2 x row_bytes per row), plus 4 B of ids read twice.  Deterministic: the
// output order is the input order within each partition.
#include <string.h>

#include "dlsa_internal.hpp"

namespace dlsa {

__global__ __launch_bounds__(256) void part_count_kernel(const int32_t* pid, int64_t n, int K,
                                                         int64_t rows_per_block, int32_t* counts,
                                                         int32_t* bad) {
  extern __shared__ int32_t hist[];  // K + 1
  const int b = blockIdx.x, tid = threadIdx.x;
  for (int k = tid; k <= K; k += 256) hist[k] = 0;
  __syncthreads();
  const int64_t r0 = (int64_t)b * rows_per_block;
  const int64_t r1 = min(n, r0 + rows_per_block);
  for (int64_t r = r0 + tid; r < r1; r += 256) {
    const int k = pid[r];
    if (k >= 0 && k < K)
      atomicAdd(&hist[k], 1);
    else
      atomicAdd(&hist[K], 1);
  }
  __syncthreads();
  for (int k = tid; k < K; k += 256) counts[(int64_t)b * K + k] = hist[k];
  if (tid == 0) bad[b] = hist[K];
}

// counts[b, k] -> exclusive base over blocks (in place); totals[k]
__global__ __launch_bounds__(256) void part_scan_blocks_kernel(int32_t* counts, int nb, int K,
                                                               int64_t* totals) {
  const int k = blockIdx.x * 256 + threadIdx.x;
  if (k >= K) return;
  int64_t s = 0;
#pragma unroll 16
  for (int b = 0; b < nb; ++b) {
    const int32_t c = counts[(int64_t)b * K + k];
    counts[(int64_t)b * K + k] = (int32_t)s;  // < n_k <= 2^31 (checked on the host)
    s += c;
  }
  totals[k] = s;
}

// offsets[0..K] = exclusive scan of totals (one workgroup, chunks of 256)
__global__ __launch_bounds__(256) void part_offsets_kernel(const int64_t* totals, int K,
                                                           int64_t* offsets) {
  __shared__ int64_t sc[256];
  __shared__ int64_t carry;
  const int tid = threadIdx.x;
  if (tid == 0) carry = 0;
  __syncthreads();
  for (int k0 = 0; k0 < K; k0 += 256) {
    const int k = k0 + tid;
    const int64_t v = k < K ? totals[k] : 0;
    sc[tid] = v;
    __syncthreads();
    for (int o = 1; o < 256; o <<= 1) {  // Hillis-Steele inclusive scan
      const int64_t t = tid >= o ? sc[tid - o] : 0;
      __syncthreads();
      sc[tid] += t;
      __syncthreads();
    }
    if (k < K) offsets[k] = carry + sc[tid] - v;
    __syncthreads();
    if (tid == 255) carry += sc[255];
    __syncthreads();
  }
  if (tid == 0) offsets[K] = carry;
}

struct ScatterArrays {
  const char* src[kPartMaxArrays];
  char* dst[kPartMaxArrays];
  int64_t row_bytes[kPartMaxArrays];
  int32_t n_arrays;
};

constexpr int kScatterThreads = 512;

template <typename U>
__device__ __forceinline__ void copy_rows(const char* src, char* dst, const int64_t* dest, int nr,
                                          uint32_t units, int tid) {
  const U* s = (const U*)src;
  U* d = (U*)dst;
  const uint32_t total = (uint32_t)nr * units;
  for (uint32_t i = tid; i < total; i += kScatterThreads) {
    const uint32_t r = i / units;
    d[dest[r] * units + (i - r * units)] = s[i];
  }
}

__global__ __launch_bounds__(kScatterThreads) void part_scatter_kernel(
    const int32_t* pid, int64_t n, int K, int64_t rows_per_block, const int32_t* base,
    const int64_t* offsets, const ScatterArrays arr, int64_t* order) {
  extern __shared__ int64_t smem64[];
  int64_t* dest = smem64;                                  // kPartSubRows
  int32_t* cursor = (int32_t*)(smem64 + kPartSubRows);     // K
  int32_t* tag = cursor + K;                               // K: distinct-id probe
  const int b = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int64_t r0b = (int64_t)b * rows_per_block;
  const int nrb = (int)(min(n, r0b + rows_per_block) - r0b);
  for (int k = tid; k < K; k += kScatterThreads) cursor[k] = base[(int64_t)b * K + k];
  const uint64_t lt = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
  for (int sb = 0; sb < nrb; sb += kPartSubRows) {
    const int64_t r0 = r0b + sb;
    const int nr = min(kPartSubRows, nrb - sb);
    __syncthreads();  // cursors loaded / previous sub-block copied
    if (wid == 0) {
      for (int s0 = 0; s0 < nr; s0 += 64) {
        const bool valid = s0 + lane < nr;
        const int my = valid ? pid[r0 + s0 + lane] : -1;
        // fast path: all ids of the segment distinct (probe: every lane reads
        // back its own tag) -> one cursor read + write per lane, no ordering
        // question inside the segment
        if (valid) tag[my] = lane;
        __builtin_amdgcn_wave_barrier();
        const bool mine = !valid || tag[my] == lane;
        int64_t d = 0;
        if (__ballot(!mine) == 0) {
          if (valid) {
            const int c = cursor[my];
            d = offsets[my] + c;
            cursor[my] = c + 1;
          }
        } else {
          bool done = !valid;
          // one round per distinct id in the segment, lowest lane first
          while (true) {
            const uint64_t todo = __ballot(!done);
            if (todo == 0) break;
            const int leader = __builtin_ctzll(todo);
            const int v = __shfl(my, leader);
            const bool eq = !done && my == v;
            const uint64_t m = __ballot(eq);
            const int start = cursor[v];  // wave-uniform LDS read
            if (eq) {
              d = offsets[v] + start + __popcll(m & lt);
              done = true;
            }
            if (lane == leader) cursor[v] = start + __popcll(m);
          }
        }
        if (valid) dest[s0 + lane] = d;
        __builtin_amdgcn_wave_barrier();
      }
    }
    __syncthreads();
    // copy: the sub-block's source rows are contiguous, so the workgroup walks
    // (row, unit) pairs in source order -- coalesced reads, each row's units
    // written contiguously to its destination row (16-, 8-, 4- or 1-byte units)
    for (int a = 0; a < arr.n_arrays; ++a) {
      const int64_t rb = arr.row_bytes[a];
      const char* src = arr.src[a] + r0 * rb;
      char* dst = arr.dst[a];
      const uintptr_t al = (uintptr_t)src | (uintptr_t)dst;
      if ((rb & 15) == 0 && (al & 15) == 0)
        copy_rows<uint4>(src, dst, dest, nr, (uint32_t)(rb >> 4), tid);
      else if ((rb & 7) == 0 && (al & 7) == 0)
        copy_rows<uint64_t>(src, dst, dest, nr, (uint32_t)(rb >> 3), tid);
      else if ((rb & 3) == 0 && (al & 3) == 0)
        copy_rows<uint32_t>(src, dst, dest, nr, (uint32_t)(rb >> 2), tid);
      else
        copy_rows<uint8_t>(src, dst, dest, nr, (uint32_t)rb, tid);
    }
    if (order)
      for (int r = tid; r < nr; r += kScatterThreads) order[dest[r]] = r0 + r;
  }
}

hipError_t launch_partition_rows(const int32_t* pid, int64_t n, int K, int64_t rows_per_block,
                                 int nb, int32_t* counts, int32_t* bad, int64_t* totals,
                                 int64_t* offsets_dev, hipStream_t s) {
  hipLaunchKernelGGL(part_count_kernel, dim3(nb), dim3(256), (size_t)(K + 1) * 4, s, pid, n, K,
                     rows_per_block, counts, bad);
  hipLaunchKernelGGL(part_scan_blocks_kernel, dim3((K + 255) / 256), dim3(256), 0, s, counts, nb,
                     K, totals);
  hipLaunchKernelGGL(part_offsets_kernel, dim3(1), dim3(256), 0, s, totals, K, offsets_dev);
  return hipGetLastError();
}

hipError_t launch_partition_scatter(const int32_t* pid, int64_t n, int K, int64_t rows_per_block,
                                    int nb, const int32_t* base, const int64_t* offsets_dev,
                                    const void* const* src, void* const* dst,
                                    const int64_t* row_bytes, int n_arrays, int64_t* order,
                                    hipStream_t s) {
  ScatterArrays arr;
  memset(&arr, 0, sizeof(arr));
  arr.n_arrays = n_arrays;
  for (int a = 0; a < n_arrays; ++a) {
    arr.src[a] = (const char*)src[a];
    arr.dst[a] = (char*)dst[a];
    arr.row_bytes[a] = row_bytes[a];
  }
  {
    hipError_t e = ensure_max_lds((const void*)part_scatter_kernel, 160 * 1024);
    if (e != hipSuccess) return e;
  }
  const size_t lds = (size_t)kPartSubRows * 8 + (size_t)K * 8;
  hipLaunchKernelGGL(part_scatter_kernel, dim3(nb), dim3(kScatterThreads), lds, s, pid, n, K, rows_per_block,
                     base, offsets_dev, arr, order);
  return hipGetLastError();
}

}  // namespace dlsa
