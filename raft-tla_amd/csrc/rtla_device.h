// rtla_device.h -- structures shared by the kernels and the host driver.
#pragma once
#include <stdint.h>

#include "../../include/rtla.h"
#include "rtla_model.h"

namespace rtla {

// Coverage codes: the 10 Next families, with Receive split into its 6
// sub-actions (UpdateTerm, HandleRequestVoteRequest, HandleRequestVoteResponse,
// HandleAppendEntriesRequest, HandleAppendEntriesResponse, DropStaleResponse).
constexpr int COVER_CODES = (int)F_COUNT + (int)R_NONE;

enum {
  FLAG_SPEC_ERROR = 1,      // TLC evaluation error (sequence index outside its domain)
  FLAG_ROW_OVERFLOW = 2,    // bag / elections capacity of the row format exceeded
  FLAG_FRONTIER_FULL = 4,   // next-frontier buffer too small
  FLAG_FPSET_FULL = 8,      // fingerprint set probe limit hit
  FLAG_OUTBOX_FULL = 16,    // exchange outbox region too small
  FLAG_BAD_INDEX = 32,      // RTLA_CHECKED builds: a global index outside its buffer
  FLAG_LOCAL_FAILURE = 64,  // (host) a rank's local work failed: carried to every rank in the level reduction
};
static_assert(FLAG_SPEC_ERROR == RTLA_CAP_SPEC_ERROR && FLAG_ROW_OVERFLOW == RTLA_CAP_ROW &&
                  FLAG_FRONTIER_FULL == RTLA_CAP_FRONTIER && FLAG_FPSET_FULL == RTLA_CAP_FPSET &&
                  FLAG_OUTBOX_FULL == RTLA_CAP_OUTBOX,
              "rtla.h RTLA_CAP_* mirror the device flags");

// Most shards in one job (one per GPU of an 8-GPU node, or virtual shards on
// one device): the expand kernels keep per-owner outbox state in registers /
// LDS sized by it, and rtla_open refuses more (RTLA_E_CONFIG).
constexpr int SHARD_MAX = 8;
// Outbox slots a wave of the level kernel reserves per owner at a time.
constexpr int OBOX_CHUNK = 256;

// Fingerprint ownership across shards (ranks): low 32 bits of fp.a scaled to
// [0, nshard).  The fingerprint-set home slot uses the TOP bits of fp.a, so
// ownership and placement are independent.
RTLA_HD int fp_owner(FP f, int nshard) {
  return (int)(((f.a & 0xffffffffull) * (unsigned long long)nshard) >> 32);
}

// A BFS level's rows inside the shard's row arena.  The arena (`cap` rows, a
// multiple of 64) is used as a ring: state g of the level is row
// (start + g) mod cap.  The next level starts at the first multiple of 64 past
// the current one, so one level's rows never overlap the next level's, both
// together may fill the whole arena (TLC's disk queue needs no second buffer
// either), and a group of 64 states starting at a multiple of 64 never wraps.
struct Ring {
  uint32_t* base;
  unsigned long long start, cap;
};
RTLA_HD unsigned long long ring_idx(const Ring& r, unsigned long long g) {
  const unsigned long long i = r.start + g;  // start < cap and g < cap
  return i >= r.cap ? i - r.cap : i;
}

// Outbox of one shard for one exchange round: region p (capacity `cap`
// records) holds the successors owned by shard p.  The level kernel stops
// taking frontier groups once any region holds `stop_at` records; what the
// groups already in flight still queue past a region's end goes to the
// overflow list (owner mixed, sent in the next round).  The overflow's
// capacity covers every in-flight group queueing all its candidates.
struct ShardBox {
  int nshard, me;
  unsigned long long cap;
  int slog2;                      // log2 slots of the sent cache (MULTI; 0 = no sent cache)
  unsigned long long* out_count;  // [nshard]
  unsigned long long* send_fp;    // [nshard][cap][2]
  unsigned long long* send_ref;   // [nshard][cap]: local parent index << 16 | instance
  unsigned long long stop_at;     // k_expand_compact: no new group once a region holds this many
  unsigned long long* over_fp;    // [over_cap][2]: records past their region's end
  unsigned long long* over_ref;   // [over_cap]
  unsigned long long* over_count; // its fill counter
  unsigned long long over_cap;
};

// Diagnostic switches of the expand kernels (rtla_time_expand, RTLA_XFLAGS; 0 in the BFS).
enum {
  XF_NO_PROBE = 1,        // skip the fingerprint-set CAS (every successor "seen")
  XF_NO_COVER = 2,        // skip the coverage counters
  XF_NO_HASH = 4,         // replace the fingerprint delta by a trivial sum
  XF_NO_MATERIALIZE = 8,  // compact kernel: write parent records but not the rows of new states
  XF_NO_CHUNKS = 32,      // compact kernel: load rows + per-state setup only
  XF_NO_DELTA = 64,       // compact kernel: compaction without evaluating actions
  XF_GENERIC_DELTA = 128, // compact kernel: never use the per-family specialised evaluation
  XF_BLOCK4 = 256,        // compact kernel: 4-wave workgroups instead of 1
  XF_NO_PERSIST = 512,    // compact kernel: one group per wave instead of persistent waves
  XF_CAS_ONLY = 1024,     // compact kernel: probe with CAS only (no load-first)
  XF_WAVE_KERNEL = 2048,  // use the wave-per-state k_expand (the fallback for rows too wide for the compact tile)
  XF_NO_SPECIAL = 4096,   // compact kernel: run-time layout even for a compiled-in configuration
  XF_DEDUP_ONLY = 8192,   // compact kernel: count new fingerprints, build no rows (synthetic microbench)
  XF_ALL_SUCCESSORS = 16384,  // compact kernel: no seen set -- every enabled successor (in-model or not) gets a
                              // row, its record = input index << 32 | in_model << 31 | sub << 16 | instance
                              // (rtla_expand_batch: the parity seam runs the hot kernel)
};

// Per-level device counters (zeroed before each level except `cover`).
struct DevCounters {
  unsigned long long generated;
  unsigned long long next_count;
  unsigned long long probes;
  int flags;
  int viol_mask;
  int viol_inst;
  int viol_in_model;
  unsigned long long viol_parent;
  unsigned long long viol_child;
  unsigned long long group_next;  // k_expand_compact's work queue (zeroed before each launch)
  unsigned long long group_size;  // frontier states per group of the last k_expand_compact launch
  unsigned long long stamp[8];    // RTLA_STAMPS builds: cycles per level-kernel phase, summed over waves
  unsigned long long cas;         // RTLA_COUNT_CAS builds: pipelined fingerprint-set CAS issued by the level kernel
  // buffer capacities (rows of the current / next frontier, parent records), for RTLA_CHECKED builds
  unsigned long long cap_cur, cap_next, cap_parents;
  unsigned long long cover[2 * COVER_CODES];  // [0,C): generated, [C,2C): distinct
};

}  // namespace rtla
