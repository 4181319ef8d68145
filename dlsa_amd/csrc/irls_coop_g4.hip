// Instantiations of the cooperative pass for NT in {8}.
#include "irls_coop_impl.hpp"

namespace dlsa {

hipError_t launch_irls_coop_g4(const PassArgs& a, int NT, int prec, bool std_, int family,
                                int n_chunks, hipStream_t s) {
  switch (NT) {
    case 8: return launch_coop_nt<8>(a, prec, std_, family, n_chunks, s);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace dlsa
