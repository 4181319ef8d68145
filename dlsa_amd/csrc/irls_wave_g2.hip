// Instantiations of the per-wave fp64 pass for NT in {7, 8}.
#include "irls_wave_impl.hpp"

namespace dlsa {

hipError_t launch_irls_wave_g2(const PassArgs& a, int NT, bool std_, int family, int n_chunks,
                               hipStream_t s) {
  switch (NT) {
    case 7: return launch_wave_nt<7>(a, std_, family, n_chunks, s);
    case 8: return launch_wave_nt<8>(a, std_, family, n_chunks, s);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace dlsa
