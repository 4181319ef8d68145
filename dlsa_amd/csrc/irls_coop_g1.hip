// Instantiations of the cooperative pass for NT in {1, 2, 3, 4}.
#include "irls_coop_impl.hpp"

namespace dlsa {

hipError_t launch_irls_coop_g1(const PassArgs& a, int NT, int prec, bool std_, int family,
                                int n_chunks, hipStream_t s) {
  switch (NT) {
    case 1: return launch_coop_nt<1>(a, prec, std_, family, n_chunks, s);
    case 2: return launch_coop_nt<2>(a, prec, std_, family, n_chunks, s);
    case 3: return launch_coop_nt<3>(a, prec, std_, family, n_chunks, s);
    case 4: return launch_coop_nt<4>(a, prec, std_, family, n_chunks, s);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace dlsa
