// rtla_kspec_a.hip -- level-kernel instantiations: the compiled-in layouts of BASELINE configs[1], configs[0] and the exhaust model.
#include "rtla_kernels_common.h"

namespace rtla {

hipError_t launch_compact_spec_a(const CompactArgs& a, bool* done) {
  *done = true;
  if (same_layout(a.L, specs::CFG2))
    return launch_compact<specs::CFG2.N, spec_group(specs::CFG2), specs::CFG2, (bool)specs::CFG2.sym>(a);
  if (same_layout(a.L, specs::CFG1))
    return launch_compact<specs::CFG1.N, spec_group(specs::CFG1), specs::CFG1, (bool)specs::CFG1.sym>(a);
  if (same_layout(a.L, specs::EXHAUST))
    return launch_compact<specs::EXHAUST.N, spec_group(specs::EXHAUST), specs::EXHAUST, (bool)specs::EXHAUST.sym>(a);
  *done = false;
  return hipSuccess;
}

}  // namespace rtla
