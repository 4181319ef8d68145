// Per-wave fp64 IRLS pass: host entry point (kernel in irls_wave_impl.hpp;
// NT = 7, 8 are instantiated in irls_wave_g2.hip so the two halves compile in
// parallel).
#include "irls_wave_impl.hpp"

namespace dlsa {

hipError_t launch_irls_wave_g2(const PassArgs& a, int NT, bool std_, int family, int n_chunks,
                               hipStream_t s);

// (the logistic ring is the larger one)
int wave_lds_bytes(int NT, int p) {
  return wave_lds_bytes_impl(NT, wave_rb(NT, wave_w(NT), FAMILY_LOGISTIC), p, FAMILY_LOGISTIC);
}

hipError_t launch_irls_wave(const PassArgs& a, int NT, bool standardize, int family, int n_chunks,
                            hipStream_t s) {
  switch (NT) {
    case 1: return launch_wave_nt<1>(a, standardize, family, n_chunks, s);
    case 2: return launch_wave_nt<2>(a, standardize, family, n_chunks, s);
    case 3: return launch_wave_nt<3>(a, standardize, family, n_chunks, s);
    case 4: return launch_wave_nt<4>(a, standardize, family, n_chunks, s);
    case 5: return launch_wave_nt<5>(a, standardize, family, n_chunks, s);
    case 6: return launch_wave_nt<6>(a, standardize, family, n_chunks, s);
    default: return launch_irls_wave_g2(a, NT, standardize, family, n_chunks, s);
  }
}

}  // namespace dlsa
