// rtla_ksym_a.hip -- level-kernel instantiations: SYMMETRY on the run-time layout, N = 1..3 (32-state groups).
#include "rtla_kernels_common.h"

namespace rtla {

hipError_t launch_compact_sym_a(const CompactArgs& a, bool* done) {
  *done = true;
  if (!a.L.sym) {
    *done = false;
    return hipSuccess;
  }
  switch (a.L.N) {
    case 1: return launch_compact<1, 32, Layout{}, true>(a);
    case 2: return launch_compact<2, 32, Layout{}, true>(a);
    case 3: return launch_compact<3, 32, Layout{}, true>(a);
    default: break;
  }
  *done = false;
  return hipSuccess;
}

}  // namespace rtla
