// Ozaki-scheme exact pass: NT = 7 (see irls_oz.hip; NT = 8 would spill at 6
// levels and keeps the fp64 pass).
#include "irls_oz_impl.hpp"

namespace dlsa {

hipError_t launch_irls_oz_g2(const PassArgs& a, int NT, bool std_, int family, int n_chunks,
                             hipStream_t s) {
  switch (NT) {
    case 7: return launch_oz_nt<7>(a, std_, family, n_chunks, s);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace dlsa


#ifdef DLSA_OZ_PROF
// profiling build only: read and reset this unit's stamp sums (producer wave
// 0: [0] barrier, [1] row phase, [2] digits + gradient; consumer wave 0:
// [8] barrier, [9] DMA issue, [10] MFMA phase, [11] DMA wait)
extern "C" int dlsa_oz_prof_read_g2(unsigned long long* out) { return dlsa::oz_prof_read_impl(out); }
#endif
