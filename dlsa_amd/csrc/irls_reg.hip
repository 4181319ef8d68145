// Register-streaming fused IRLS pass: host entry point (kernel in
// irls_reg_impl.hpp, instantiated by irls_reg_g*.hip).
#include "dlsa_internal.hpp"

namespace dlsa {

hipError_t launch_irls_reg_g1(const PassArgs& a, int NT, bool f64, bool std_, int family,
                              int n_chunks, hipStream_t s);
hipError_t launch_irls_reg_g2(const PassArgs& a, int NT, bool f64, bool std_, int family,
                              int n_chunks, hipStream_t s);
hipError_t launch_irls_reg_g3(const PassArgs& a, int NT, bool f64, bool std_, int family,
                              int n_chunks, hipStream_t s);

hipError_t launch_irls_reg(const PassArgs& a, int NT, bool f64, bool standardize, int family,
                           int n_chunks, hipStream_t s) {
  if (NT <= 3) return launch_irls_reg_g1(a, NT, f64, standardize, family, n_chunks, s);
  if (NT <= 5) return launch_irls_reg_g2(a, NT, f64, standardize, family, n_chunks, s);
  if (NT <= 7) return launch_irls_reg_g3(a, NT, f64, standardize, family, n_chunks, s);
  return hipErrorInvalidValue;
}

}  // namespace dlsa
