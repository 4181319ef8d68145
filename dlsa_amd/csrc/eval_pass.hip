// Log-likelihood evaluation pass: one streaming pass
// over X computing, per partition and per candidate coefficient vector b,
//   ll[k, b] = sum_i y_i eta_ib - log(1 + exp(eta_ib)),  eta_ib = x_i . beta_b
// -- the per-partition work of dlsa/models.py:151-225 logistic_model_eval
// (driven by dlsa/model_eval.py:10-42 over the AIC / BIC / WLSE / ONESHOT
// columns).  HBM-bound: X and y are read once for all candidates.
//
// Geometry: one 4-wave workgroup per chunk; 32-row blocks through the same
// shared LDS-DMA ring as the fused IRLS pass; 8 lanes per row, the candidate
// vectors in LDS.
#include "dlsa_internal.hpp"

namespace dlsa {

namespace {

typedef __attribute__((address_space(3))) void lds_void_t;
typedef const __attribute__((address_space(1))) void gbl_void_t;

constexpr int EW = 4;    // waves
constexpr int ERB = 32;  // rows per block
constexpr int EMAXB = 16;

template <int N>
__device__ __forceinline__ void ev_wait() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
template <int N>
__device__ __forceinline__ void ev_wait_le(int n) {
  if constexpr (N <= 0) {
    ev_wait<0>();
  } else {
    if (n >= N)
      ev_wait<N>();
    else
      ev_wait_le<N - 1>(n);
  }
}
template <int CTRL>
__device__ __forceinline__ double ev_dpp(double v) {
  const int lo = __builtin_amdgcn_mov_dpp(__double2loint(v), CTRL, 0xF, 0xF, false);
  const int hi = __builtin_amdgcn_mov_dpp(__double2hiint(v), CTRL, 0xF, 0xF, false);
  return __hiloint2double(hi, lo);
}
__device__ __forceinline__ double ev_red8(double v) {
  v += ev_dpp<0xB1>(v);
  v += ev_dpp<0x4E>(v);
  v += ev_dpp<0x141>(v);
  return v;
}
__host__ __device__ __forceinline__ int ev_npieces(int p) {
  return (ERB * p * 8 + 16 + 1023) / 1024;
}

}  // namespace

int eval_slot_bytes(int p) {
  const int d = (ev_npieces(p) + EW - 1) / EW;
  return 16 + d * EW * 1024 + ((p + 8) / 8) * 8 * 8 + ERB * 8;
}

__global__ __launch_bounds__(256) void loglik_eval_kernel(const EvalArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int chunk = blockIdx.x;
  const int part = a.chunk_part[chunk];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int p = a.p, P = a.P, ic = a.intercept, B = a.nbeta;
  const int64_t row0 = a.chunk_row0[chunk];
  const int nrows = a.chunk_rows[chunk];
  const int nb = (nrows + ERB - 1) / ERB;
  const int nslot = a.nslot, slot_bytes = a.slot_bytes;
  const int npieces = ev_npieces(p);
  const int d = (npieces + EW - 1) / EW;
  const int slot_x = 16 + d * EW * 1024 + ((p + 8) / 8) * 8 * 8;
  const int PM = ((P + 7) / 8) * 8;  // features padded to the 8-lane stride
  double* bet = (double*)(smem + nslot * slot_bytes);  // [B][PM]
  double* stdv = bet + B * PM;                         // [2][PM]
  double* red = stdv + 2 * PM;                         // [EW][EMAXB]

  for (int o = tid * 16; o < nslot * slot_bytes; o += 256 * 16)
    *(uint4*)(smem + o) = make_uint4(0, 0, 0, 0);
  for (int e = tid; e < B * PM; e += 256) {
    const int b = e / PM, f = e - b * PM;
    bet[e] = f < P ? a.betas[(int64_t)b * P + f] : 0.0;
  }
  for (int f = tid; f < PM; f += 256) {
    const int j = f - ic;
    const bool in = a.center && j >= 0 && j < p;
    stdv[f] = in ? a.center[j] : 0.0;
    stdv[PM + f] = in ? 1.0 / a.scale[j] : 1.0;
  }
  __syncthreads();

  auto issue = [&](int blk) {
    const int bb = blk < nb ? blk : nb - 1;
    char* sbase = smem + (blk % nslot) * slot_bytes;
    const uintptr_t start = (uintptr_t)(a.X + (row0 + (int64_t)bb * ERB) * p);
    const uintptr_t al = start & ~(uintptr_t)15;
    for (int i = 0; i < d; ++i) {
      const int j = wid + EW * i;
      const int jj = j < npieces ? j : npieces - 1;
      uintptr_t src = al + (uintptr_t)jj * 1024 + (uintptr_t)lane * 16;
      src = src < a.x_last16 ? src : a.x_last16;
      __builtin_amdgcn_global_load_lds((gbl_void_t*)src, (lds_void_t*)(sbase + 16 + j * 1024), 16,
                                       0, 0);
    }
    uintptr_t ys = (uintptr_t)(a.y + row0 + (int64_t)bb * ERB) + (uintptr_t)lane * 4;
    ys = ys < a.y_last4 ? ys : a.y_last4;
    __builtin_amdgcn_global_load_lds((gbl_void_t*)ys, (lds_void_t*)(sbase + slot_x), 4, 0, 0);
  };

  const int sl = lane & 7;
  const int rB = wid * 8 + (lane >> 3);
  double llacc[EMAXB];
#pragma unroll
  for (int b = 0; b < EMAXB; ++b) llacc[b] = 0.0;

  for (int b = 0; b < nslot - 1; ++b) issue(b);
  const int keep = (nslot - 2) * (d + 1);
  for (int blk = 0; blk < nb; ++blk) {
    ev_wait_le<40>(keep);
    __syncthreads();
    issue(blk + nslot - 1);
    const char* slot = smem + (blk % nslot) * slot_bytes;
    const uintptr_t start = (uintptr_t)(a.X + (row0 + (int64_t)blk * ERB) * p);
    const double* xs = (const double*)(slot + 16 + (start & 15));
    const double* ys = (const double*)(slot + slot_x);
    const bool valid = rB < nrows - blk * ERB;
    const double* xr = xs + rB * p + (sl - ic);
    double eta[EMAXB];
#pragma unroll
    for (int b = 0; b < EMAXB; ++b) eta[b] = 0.0;
    for (int f = sl; f < PM; f += 8) {
      double v = xr[f - sl];
      v = (v - stdv[f]) * stdv[PM + f];
      if (f == 0 && ic) v = 1.0;
#pragma unroll
      for (int b = 0; b < EMAXB; ++b)
        if (b < B) eta[b] = fma(v, bet[b * PM + f], eta[b]);
    }
    const double yv = ys[rB];
#pragma unroll
    for (int b = 0; b < EMAXB; ++b) {
      if (b < B) {
        const double e = ev_red8(eta[b]);
        if (valid && sl == 0) llacc[b] += yv * e - (fmax(e, 0.0) + log1p(exp(-fabs(e))));
      }
    }
  }
  ev_wait<0>();
  __syncthreads();
#pragma unroll
  for (int b = 0; b < EMAXB; ++b) {
    if (b < B) {
      double v = llacc[b];
      v += __shfl_xor(v, 8);
      v += __shfl_xor(v, 16);
      v += __shfl_xor(v, 32);
      if (lane == 0) red[wid * EMAXB + b] = v;
    }
  }
  __syncthreads();
  if (tid < B) {
    double s = 0.0;
    for (int w = 0; w < EW; ++w) s += red[w * EMAXB + tid];
    a.partial[(int64_t)chunk * B + tid] = s;
  }
}

hipError_t launch_loglik_eval(const EvalArgs& a, int n_chunks, hipStream_t s) {
  const int PM = ((a.P + 7) / 8) * 8;
  const size_t lds = (size_t)a.nslot * a.slot_bytes +
                     ((size_t)a.nbeta * PM + 2 * PM + EW * EMAXB) * sizeof(double);
  {
    hipError_t e = ensure_max_lds((const void*)loglik_eval_kernel, 160 * 1024);
    if (e != hipSuccess) return e;
  }
  hipLaunchKernelGGL(loglik_eval_kernel, dim3(n_chunks), dim3(256), lds, s, a);
  return hipGetLastError();
}

// ll[k, b] = sum of the chunk partials of partition k (fixed order)
__global__ void loglik_reduce_kernel(const double* partial, const int32_t* pcb, int K, int B,
                                     double* out) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= K * B) return;
  const int k = e / B, b = e - k * B;
  double s = 0.0;
  for (int c = pcb[k]; c < pcb[k + 1]; ++c) s += partial[(int64_t)c * B + b];
  out[e] = s;
}

hipError_t launch_loglik_reduce(const double* partial, const int32_t* pcb, int K, int B,
                                double* out, hipStream_t s) {
  hipLaunchKernelGGL(loglik_reduce_kernel, dim3((K * B + 255) / 256), dim3(256), 0, s, partial,
                     pcb, K, B, out);
  return hipGetLastError();
}

}  // namespace dlsa
