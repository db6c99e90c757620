// rtla_text.h -- decode packed rows into TLC-style value text.
#pragma once
#include <stdint.h>

#include <string>

#include "rtla_model.h"

namespace rtla {

// Canonical TLC-like text of a state: "/\ var = value" lines in the variable
// declaration order of raft.tla:32-85, sets and bag domains sorted by text.
std::string state_text(const Layout& L, const uint32_t* row);
// The same text written into buf (state_text_cap(L) bytes; scratch: as many
// again, for the items of the sorted collections); returns its length.
size_t state_text_cap(const Layout& L);
size_t state_text_into(const Layout& L, const uint32_t* row, char* buf, char* scratch);
// SYMMETRY: the orbit text of the state (rtla_text.cpp; the same buffers).
size_t state_orbit_text_into(const Layout& L, const uint32_t* row, char* buf, char* scratch);
// Human-readable label of an action instance (+ Receive sub-action).
std::string action_name(const Layout& L, int inst, int sub);

}  // namespace rtla
