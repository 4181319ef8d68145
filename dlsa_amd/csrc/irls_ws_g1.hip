// Instantiations of the wave-specialised fp64 pass for NT in {1, 2, 3, 4, 5}.
#include "irls_ws_impl.hpp"

namespace dlsa {

hipError_t launch_irls_ws_g1(const PassArgs& a, int NT, bool std_, int family, int n_chunks,
                              hipStream_t s) {
  switch (NT) {
    case 1: return launch_ws_nt<1>(a, std_, family, n_chunks, s);
    case 2: return launch_ws_nt<2>(a, std_, family, n_chunks, s);
    case 3: return launch_ws_nt<3>(a, std_, family, n_chunks, s);
    case 4: return launch_ws_nt<4>(a, std_, family, n_chunks, s);
    case 5: return launch_ws_nt<5>(a, std_, family, n_chunks, s);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace dlsa
