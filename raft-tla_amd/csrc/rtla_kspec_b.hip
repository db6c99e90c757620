// rtla_kspec_b.hip -- level-kernel instantiations: the compiled-in layouts of BASELINE configs[2], configs[4] and configs[3] (SYMMETRY).
#include "rtla_kernels_common.h"

namespace rtla {

hipError_t launch_compact_spec_b(const CompactArgs& a, bool* done) {
  *done = true;
  if (same_layout(a.L, specs::CFG3))
    return launch_compact<specs::CFG3.N, spec_group(specs::CFG3), specs::CFG3, (bool)specs::CFG3.sym>(a);
  if (same_layout(a.L, specs::SYNTH))
    return launch_compact<specs::SYNTH.N, spec_group(specs::SYNTH), specs::SYNTH, (bool)specs::SYNTH.sym>(a);
  if (same_layout(a.L, specs::CFG4))
    return launch_compact<specs::CFG4.N, spec_group(specs::CFG4), specs::CFG4, (bool)specs::CFG4.sym>(a);
  *done = false;
  return hipSuccess;
}

}  // namespace rtla
