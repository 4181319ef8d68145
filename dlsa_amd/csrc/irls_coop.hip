// Cooperative fused IRLS pass: host entry points (kernels in
// irls_coop_impl.hpp, instantiated by irls_coop_g*.hip).
#include "irls_coop_impl.hpp"

namespace dlsa {

hipError_t launch_irls_coop_g1(const PassArgs& a, int NT, int prec, bool std_, int family,
                                int n_chunks, hipStream_t s);
hipError_t launch_irls_coop_g2(const PassArgs& a, int NT, int prec, bool std_, int family,
                                int n_chunks, hipStream_t s);
hipError_t launch_irls_coop_g3(const PassArgs& a, int NT, int prec, bool std_, int family,
                                int n_chunks, hipStream_t s);
hipError_t launch_irls_coop_g4(const PassArgs& a, int NT, int prec, bool std_, int family,
                                int n_chunks, hipStream_t s);
hipError_t launch_irls_coop_g5(const PassArgs& a, int NT, int prec, bool std_, int family,
                                int n_chunks, hipStream_t s);
hipError_t launch_irls_coop_g6(const PassArgs& a, int NT, int prec, bool std_, int family,
                                int n_chunks, hipStream_t s);

int coop_slot_bytes(int NT, int p) { return coop_slot_bytes_impl(NT, p); }
int coop_extra_bytes(int NT) { return coop_extra_bytes_impl(NT); }

hipError_t launch_irls_coop(const PassArgs& a, int NT, int prec, bool standardize, int family,
                            int n_chunks, hipStream_t s) {
  if (NT <= 4) return launch_irls_coop_g1(a, NT, prec, standardize, family, n_chunks, s);
  if (NT <= 6) return launch_irls_coop_g2(a, NT, prec, standardize, family, n_chunks, s);
  if (NT <= 7) return launch_irls_coop_g3(a, NT, prec, standardize, family, n_chunks, s);
  if (NT <= 8) return launch_irls_coop_g4(a, NT, prec, standardize, family, n_chunks, s);
  if (NT <= 10) return launch_irls_coop_g5(a, NT, prec, standardize, family, n_chunks, s);
  if (NT <= 12) return launch_irls_coop_g6(a, NT, prec, standardize, family, n_chunks, s);
  return hipErrorInvalidValue;
}

}  // namespace dlsa
