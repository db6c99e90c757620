// rtla_kgeneric_b.hip -- level-kernel instantiations: any configuration with N = 4, 5 on its run-time layout.
#include "rtla_kernels_common.h"

namespace rtla {

hipError_t launch_compact_generic_b(const CompactArgs& a, bool* done) {
  *done = true;
  const bool g64 = compact_group(a.L) == 64;
  switch (a.L.sym ? 0 : a.L.N) {
    case 4: return g64 ? launch_compact<4, 64, Layout{}>(a) : launch_compact<4, 32, Layout{}>(a);
    case 5: return g64 ? launch_compact<5, 64, Layout{}>(a) : launch_compact<5, 32, Layout{}>(a);
    default: break;
  }
  *done = false;
  return hipSuccess;
}

}  // namespace rtla
