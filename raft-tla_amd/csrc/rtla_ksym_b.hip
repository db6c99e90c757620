// rtla_ksym_b.hip -- level-kernel instantiations: SYMMETRY on the run-time layout, N = 4, 5 (32-state groups).
#include "rtla_kernels_common.h"

namespace rtla {

hipError_t launch_compact_sym_b(const CompactArgs& a, bool* done) {
  *done = true;
  if (!a.L.sym) {
    *done = false;
    return hipSuccess;
  }
  switch (a.L.N) {
    case 4: return launch_compact<4, 32, Layout{}, true>(a);
    case 5: return launch_compact<5, 32, Layout{}, true>(a);
    default: break;
  }
  *done = false;
  return hipSuccess;
}

}  // namespace rtla
