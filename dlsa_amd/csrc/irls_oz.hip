// Ozaki-scheme exact pass (irls_oz_impl.hpp): host entry point; NT = 7, 8 are
// instantiated in irls_oz_g2.hip so the two halves compile in parallel.
#include "irls_oz_impl.hpp"

namespace dlsa {

hipError_t launch_irls_oz_g2(const PassArgs& a, int NT, bool std_, int family, int n_chunks,
                             hipStream_t s);

bool oz_applies(int NT, int p) { return NT >= 1 && NT <= kOzMaxNT && ozk::fits(NT, p); }

hipError_t launch_irls_oz(const PassArgs& a, int NT, bool standardize, int family, int n_chunks,
                          hipStream_t s) {
  if (!oz_applies(NT, a.p) || !a.colmax || !a.zcolmax || !a.theta_rec) return hipErrorInvalidValue;
  switch (NT) {
    case 1: return launch_oz_nt<1>(a, standardize, family, n_chunks, s);
    case 2: return launch_oz_nt<2>(a, standardize, family, n_chunks, s);
    case 3: return launch_oz_nt<3>(a, standardize, family, n_chunks, s);
    case 4: return launch_oz_nt<4>(a, standardize, family, n_chunks, s);
    case 5: return launch_oz_nt<5>(a, standardize, family, n_chunks, s);
    case 6: return launch_oz_nt<6>(a, standardize, family, n_chunks, s);
    default: return launch_irls_oz_g2(a, NT, standardize, family, n_chunks, s);
  }
}

}  // namespace dlsa



#ifdef DLSA_OZ_PROF
// profiling build only: read and reset this unit's stamp sums (producer wave
// 0: [0] barrier, [1] row phase, [2] digits + gradient; consumer wave 0:
// [8] barrier, [9] DMA issue, [10] MFMA phase, [11] DMA wait)
extern "C" int dlsa_oz_prof_read(unsigned long long* out) { return dlsa::oz_prof_read_impl(out); }
#endif
