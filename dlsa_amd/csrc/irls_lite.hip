// Light-weight approximate-Hessian pass: host entry points (kernel in
// irls_lite_impl.hpp).
#include <stdlib.h>

#include <algorithm>

#include "irls_lite_impl.hpp"

namespace dlsa {

bool lite_fits(int NT, int p) { return lt_fits(p, NT); }
int lite_slot_bytes(int NT, int p) { return lt_slot_bytes(p, NT); }

// ring depth: 3 slots (~41 KB at p = 100: three workgroups per CU, two blocks
// in flight each) unless DLSA_LITE_NSLOT says otherwise
int lite_nslot(int NT, int p) {
  int n = 3;
  if (const char* e = getenv("DLSA_LITE_NSLOT")) n = atoi(e);
  const int fit = (160 * 1024 - 2 * 16 * NT * 8) / lt_slot_bytes(p, NT);
  return std::max(2, std::min(std::min(n, 5), fit));
}

template <int NT>
static hipError_t launch_lite_nt(const PassArgs& a, bool std_, int n_chunks, hipStream_t s) {
  return std_ ? launch_lite_t<NT, true>(a, n_chunks, s) : launch_lite_t<NT, false>(a, n_chunks, s);
}

hipError_t launch_irls_lite(const PassArgs& a, int NT, bool standardize, int n_chunks,
                            hipStream_t s) {
  if (!lt_fits(a.p, NT) || lt_npieces(a.p) > 36) return hipErrorInvalidValue;
  switch (NT) {
    case 1: return launch_lite_nt<1>(a, standardize, n_chunks, s);
    case 2: return launch_lite_nt<2>(a, standardize, n_chunks, s);
    case 3: return launch_lite_nt<3>(a, standardize, n_chunks, s);
    case 4: return launch_lite_nt<4>(a, standardize, n_chunks, s);
    case 5: return launch_lite_nt<5>(a, standardize, n_chunks, s);
    case 6: return launch_lite_nt<6>(a, standardize, n_chunks, s);
    case 7: return launch_lite_nt<7>(a, standardize, n_chunks, s);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace dlsa
