// Instantiations of the cooperative pass for NT in {9, 10}.
#include "irls_coop_impl.hpp"

namespace dlsa {

hipError_t launch_irls_coop_g5(const PassArgs& a, int NT, int prec, bool std_, int family,
                                int n_chunks, hipStream_t s) {
  switch (NT) {
    case 9: return launch_coop_nt<9>(a, prec, std_, family, n_chunks, s);
    case 10: return launch_coop_nt<10>(a, prec, std_, family, n_chunks, s);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace dlsa
