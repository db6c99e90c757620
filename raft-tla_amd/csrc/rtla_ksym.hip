// rtla_ksym.hip -- level-kernel instantiations: SYMMETRY on the run-time layout (N = 1..5; 32-state groups).
#include "rtla_kernels_common.h"

namespace rtla {

hipError_t launch_compact_sym(const CompactArgs& a, bool* done) {
  *done = true;
  if (!a.L.sym) {
    *done = false;
    return hipSuccess;
  }
  switch (a.L.N) {
    case 1: return launch_compact<1, 32, Layout{}, true>(a);
    case 2: return launch_compact<2, 32, Layout{}, true>(a);
    case 3: return launch_compact<3, 32, Layout{}, true>(a);
    case 4: return launch_compact<4, 32, Layout{}, true>(a);
    default: return launch_compact<5, 32, Layout{}, true>(a);
  }
  *done = false;
  return hipSuccess;
}

}  // namespace rtla
