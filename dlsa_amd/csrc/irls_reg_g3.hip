// Instantiations of the register-streaming pass for NT in {6, 7}.
#include "irls_reg_impl.hpp"

namespace dlsa {

hipError_t launch_irls_reg_g3(const PassArgs& a, int NT, bool f64, bool std_, int family,
                               int n_chunks, hipStream_t s) {
  switch (NT) {
    case 6: return launch_reg_nt<6>(a, f64, std_, family, n_chunks, s);
    case 7: return launch_reg_nt<7>(a, f64, std_, family, n_chunks, s);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace dlsa
