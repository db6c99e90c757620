// rtla_launch.h -- host-side launch wrappers for the kernels in rtla_kernels.hip.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "rtla_device.h"

namespace rtla {

// LDS bytes a k_expand / k_expand_batch block of `wpb` waves needs.
size_t expand_lds_bytes(const Layout& L, int wpb);
// Waves per block of the lane-per-state row builders (k_build_winners).
int expand_lane_wpb(const Layout& L);
// Waves per block of the compacting level kernel (0: not usable).
int expand_compact_wpb(const Layout& L);
// Blocks of 4 waves that fit on one CU given the LDS footprint.
int expand_blocks_per_cu(const Layout& L);

// Arguments of one level-kernel launch (k_expand_compact).
struct CompactArgs {
  Layout L;
  bool multi;
  Ring cur;
  uint64_t s_begin, s_end, cur_base;
  Ring next;
  uint64_t* parents;
  uint64_t next_base, next_cap;
  uint64_t* table;
  int tlog2;
  DevCounters* ctr;
  ShardBox box;
  hipStream_t st;
  int xflags;
  uint64_t* sent;
  int wpb;
  int* query = nullptr;  // non-null: store {waves launched at most, GROUP} of this launch, launch nothing
};
// The level kernel's shape for layout L (multi-shard or not): the most waves
// one launch keeps resident and its frontier states per group.  false: the
// layout runs the wave-per-state kernel (no group queue).
bool level_kernel_shape(const Layout& L, bool multi, int xflags, int* waves, int* group);
// Multi-shard exchange round: move the overflow list of the previous round
// (in_fp / in_ref, *in_count records) into the outbox regions of `box` (slots
// reserved on box.out_count); records whose region is full go to box's
// overflow list.
hipError_t launch_requeue(const uint64_t* in_fp, const uint64_t* in_ref, const uint64_t* in_count, uint64_t max_count,
                          const ShardBox& box, DevCounters* ctr, hipStream_t st);
// Multi-shard exchange round: out[G] = frontier states left for the next
// round -- `rest` past the launch's range, plus those of its `span` states the
// level kernel did not take (all taken unless `grouped`: then group_next *
// group_size were) -- and out[G + 1] = records on the overflow list.
hipError_t launch_round_tail(const DevCounters* ctr, uint64_t* out, int G, uint64_t span, uint64_t rest, bool grouped,
                             const uint64_t* over_count, hipStream_t st);
// The level kernel's instantiations, one translation unit each (compiled in
// parallel): *done = false if the unit has no kernel for a.L.
hipError_t launch_compact_spec_a(const CompactArgs& a, bool* done);     // configs[1], configs[0], exhaust
hipError_t launch_compact_spec_b(const CompactArgs& a, bool* done);     // configs[2], configs[4], configs[3] (SYMMETRY)
hipError_t launch_compact_sym_a(const CompactArgs& a, bool* done);      // SYMMETRY, N = 1..3, run-time layout
hipError_t launch_compact_sym_b(const CompactArgs& a, bool* done);      // SYMMETRY, N = 4, 5, run-time layout
hipError_t launch_compact_generic_a(const CompactArgs& a, bool* done);  // N = 1..3, run-time layout
hipError_t launch_compact_generic_b(const CompactArgs& a, bool* done);  // N = 4, 5, run-time layout

hipError_t launch_expand(const Layout& L, const Ring& cur, uint64_t s_begin, uint64_t s_end,
                         uint64_t cur_base, const Ring& next, uint64_t* parents, uint64_t next_base,
                         uint64_t next_cap, uint64_t* table, int tlog2, DevCounters* ctr, const ShardBox& box,
                         int grid, hipStream_t st, int xflags = 0, uint64_t* sent = nullptr,
                         hipEvent_t mid = nullptr);  // recorded after the level kernel
// The wave-per-state level kernel (rtla_kwave.hip).
hipError_t launch_wave_expand(const Layout& L, const Ring& cur, uint64_t s_begin, uint64_t s_end, uint64_t cur_base,
                              const Ring& next, uint64_t* parents, uint64_t next_base, uint64_t next_cap,
                              uint64_t* table, int tlog2, DevCounters* ctr, const ShardBox& box, int grid,
                              hipStream_t st);
hipError_t launch_insert_remote(const uint64_t* recv_fp, const uint64_t* counts, int nshard, uint64_t cap,
                                uint64_t* table, int tlog2, uint32_t* ans, DevCounters* ctr, uint64_t max_count,
                                hipStream_t st);
hipError_t launch_build_winners(const Layout& L, const Ring& cur, uint64_t cur_base, int me, const uint64_t* send_ref,
                                const uint32_t* ans, const uint64_t* counts, int nshard, uint64_t cap,
                                const Ring& next, uint64_t* parents, uint64_t next_base, uint64_t next_cap,
                                DevCounters* ctr, uint64_t max_count, hipStream_t st);
hipError_t launch_unpack_rows(int W, const uint32_t* rows, const uint64_t* counts, const uint64_t* bases, int nshard,
                              uint64_t rows_cap, const Ring& next, uint64_t* parents, uint64_t next_base,
                              uint64_t next_cap, DevCounters* ctr, uint64_t max_count, hipStream_t st);
hipError_t launch_stage_rows(int W, const Ring& next, const uint64_t* parents, uint64_t next_base, uint64_t first,
                             uint64_t n, uint32_t* rows, hipStream_t st);
hipError_t launch_insert_rows(const Layout& L, const uint32_t* rows, uint64_t n, uint64_t* table,
                              int tlog2, int* new_flags, DevCounters* ctr, hipStream_t st);
hipError_t launch_expand_batch(const Layout& L, const uint32_t* rows, uint64_t n, uint32_t* out,
                               uint64_t* info, uint64_t cap, DevCounters* ctr, hipStream_t st);
hipError_t launch_random_rows(const Layout& L, uint64_t seed, uint64_t first, uint64_t n, uint64_t pool, uint32_t* out,
                              hipStream_t st);
hipError_t launch_probe_bench(uint64_t* table, int tlog2, uint64_t n, uint64_t seed,
                              DevCounters* ctr, hipStream_t st, int load_first = 0);
hipError_t launch_probe_mixed(uint64_t* table, int tlog2, uint64_t n, uint64_t n_present, double new_frac,
                              uint64_t seed, DevCounters* ctr, hipStream_t st);

}  // namespace rtla
