// Instantiations of the register-streaming pass for NT in {1, 2, 3}.
#include "irls_reg_impl.hpp"

namespace dlsa {

hipError_t launch_irls_reg_g1(const PassArgs& a, int NT, bool f64, bool std_, int family,
                               int n_chunks, hipStream_t s) {
  switch (NT) {
    case 1: return launch_reg_nt<1>(a, f64, std_, family, n_chunks, s);
    case 2: return launch_reg_nt<2>(a, f64, std_, family, n_chunks, s);
    case 3: return launch_reg_nt<3>(a, f64, std_, family, n_chunks, s);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace dlsa
