// Wave-specialised fp64 pass: host entry points (kernel in irls_ws_impl.hpp,
// instantiated by irls_ws_g*.hip).
#include <algorithm>

#include "irls_ws_impl.hpp"

namespace dlsa {

hipError_t launch_irls_ws_g1(const PassArgs& a, int NT, bool std_, int family, int n_chunks,
                             hipStream_t s);
hipError_t launch_irls_ws_g2(const PassArgs& a, int NT, bool std_, int family, int n_chunks,
                             hipStream_t s);

int ws_slot_bytes(int NT, int p) { return ws_sub_bytes(p, NT); }

// ring depth: as many 4-sub-slot slots as fit next to w / center / scale,
// at most 5 (the kernel's vmcnt bound)
int ws_nslot(int NT, int p) {
  const int avail = 160 * 1024 - ws_extra_bytes(NT);
  return std::min(5, avail / (4 * ws_sub_bytes(p, NT)));
}

hipError_t launch_irls_ws(const PassArgs& a, int NT, bool standardize, int family, int n_chunks,
                          hipStream_t s) {
  if (a.nslot < 3 || ws_npieces(a.p) > 10) return hipErrorInvalidValue;
  if (NT <= 5) return launch_irls_ws_g1(a, NT, standardize, family, n_chunks, s);
  if (NT <= 8) return launch_irls_ws_g2(a, NT, standardize, family, n_chunks, s);
  return hipErrorInvalidValue;
}

}  // namespace dlsa
