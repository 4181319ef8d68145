// Instantiations of the register-streaming pass for NT in {4, 5}.
#include "irls_reg_impl.hpp"

namespace dlsa {

hipError_t launch_irls_reg_g2(const PassArgs& a, int NT, bool f64, bool std_, int family,
                               int n_chunks, hipStream_t s) {
  switch (NT) {
    case 4: return launch_reg_nt<4>(a, f64, std_, family, n_chunks, s);
    case 5: return launch_reg_nt<5>(a, f64, std_, family, n_chunks, s);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace dlsa
