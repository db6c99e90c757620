// rtla_kgeneric_a.hip -- level-kernel instantiations: any configuration with N = 1..3 on its run-time layout.
#include "rtla_kernels_common.h"

namespace rtla {

hipError_t launch_compact_generic_a(const CompactArgs& a, bool* done) {
  *done = true;
  const bool g64 = compact_group(a.L) == 64;
  switch (a.L.sym ? 0 : a.L.N) {
    case 1: return g64 ? launch_compact<1, 64, Layout{}>(a) : launch_compact<1, 32, Layout{}>(a);
    case 2: return g64 ? launch_compact<2, 64, Layout{}>(a) : launch_compact<2, 32, Layout{}>(a);
    case 3: return g64 ? launch_compact<3, 64, Layout{}>(a) : launch_compact<3, 32, Layout{}>(a);
    default: break;
  }
  *done = false;
  return hipSuccess;
}

}  // namespace rtla
