// rtla_kernels_common.h -- the level kernel (k_expand_compact) and the
// device helpers every kernel translation unit shares.
//
// The level kernel is a template over the server count, the group size, the
// compiled-in layout and SYMMETRY; its instantiations are spread over several
// translation units (rtla_kspec_*.hip, rtla_kgeneric_*.hip, rtla_ksym.hip)
// that compile in parallel, each exporting one launcher
// (launch_compact_*, rtla_launch.h); rtla_kernels.hip holds the other
// kernels and the dispatch.
#pragma once
#include <hip/hip_runtime.h>
#include <stdlib.h>

#include <algorithm>
#include <type_traits>

#include "rtla_device.h"

#include "rtla_model.h"
#include "rtla_synth.h"
#include "rtla_launch.h"

using namespace rtla;

namespace {

constexpr int STAGE_ROWS = 16;  // LDS staging rows per wave

__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
}

__device__ __forceinline__ unsigned long long shfl0_u64(unsigned long long v) {
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)v);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(v >> 32));
  return (unsigned long long)lo | (unsigned long long)hi << 32;
}

// Copy n contiguous words global -> LDS with 8 loads in flight per lane
// (a plain loop waits for every load before its LDS store).
__device__ __forceinline__ void copy_words_lds(uint32_t* __restrict__ dst, const uint32_t* __restrict__ src, int n,
                                               int lane) {
  int w = lane;
  for (; w + 7 * 64 < n; w += 8 * 64) {
    uint32_t v[8];
#pragma unroll
    for (int j = 0; j < 8; j++) v[j] = src[w + j * 64];
#pragma unroll
    for (int j = 0; j < 8; j++) dst[w + j * 64] = v[j];
  }
  for (; w < n; w += 64) dst[w] = src[w];
}

// The same with 16-byte accesses (dst and src 16-byte aligned): a quarter of
// the load instructions and 4x the bytes in flight per lane.
__device__ __forceinline__ void copy_words_lds16(uint32_t* __restrict__ dst, const uint32_t* __restrict__ src, int n,
                                                 int lane) {
  const uint4* __restrict__ s4 = reinterpret_cast<const uint4*>(src);
  uint4* __restrict__ d4 = reinterpret_cast<uint4*>(dst);
  const int n4 = n >> 2;
  int w = lane;
  for (; w + 7 * 64 < n4; w += 8 * 64) {
    uint4 v[8];
#pragma unroll
    for (int j = 0; j < 8; j++) v[j] = s4[w + j * 64];
#pragma unroll
    for (int j = 0; j < 8; j++) d4[w + j * 64] = v[j];
  }
  for (; w < n4; w += 64) d4[w] = s4[w];
  for (int t = (n4 << 2) + lane; t < n; t += 64) dst[t] = src[t];
}

// Gather nv rows of W words (row r from src_row(r), a wave-uniform address)
// into LDS rows dst + r * W: lane l moves words l, l + 64, ... of each row,
// 8 rows (8 loads per lane) in flight.
template <class F>
__device__ __forceinline__ void gather_rows_lds(uint32_t* __restrict__ dst, int W, int nv, F src_row, int lane) {
  for (int r0 = 0; r0 < nv; r0 += 8) {
    for (int c = lane; c < W; c += 64) {
      uint32_t v[8];
#pragma unroll
      for (int j = 0; j < 8; j++) v[j] = r0 + j < nv ? src_row(r0 + j)[c] : 0u;
#pragma unroll
      for (int j = 0; j < 8; j++)
        if (r0 + j < nv) dst[(r0 + j) * W + c] = v[j];
    }
  }
}

// Row pointer of state g of a level (see Ring, rtla_device.h).
__device__ __forceinline__ uint32_t* ring_row(const Ring& R, unsigned long long g, int W) {
  return R.base + ring_idx(R, g) * (unsigned long long)W;
}

// Store nr consecutive rows (LDS src, W words each) as states g .. g + nr - 1
// of the level R, coalesced; the range may wrap at the end of the arena.
__device__ __forceinline__ void store_rows_ring(const Ring& R, unsigned long long g, int nr, int W,
                                                const uint32_t* __restrict__ src, int lane) {
  const unsigned long long p = ring_idx(R, g);
  const int n1 = (int)min<unsigned long long>(R.cap - p, (unsigned long long)nr) * W;  // words before the wrap
  uint32_t* d1 = R.base + p * (unsigned long long)W;
  const int nw = nr * W;
  for (int w = lane; w < nw; w += 64) {
    if (w < n1) d1[w] = src[w];
    else R.base[w - n1] = src[w];
  }
}

// Insert into the fingerprint set.  1 = newly inserted, 0 = already present,
// -1 = probe limit exceeded (set too full).  Slots only ever change 0 -> key;
// the CAS both tests and claims a slot, so every probe is one round trip.
__device__ __forceinline__ int fpset_insert(unsigned long long* table, int log2, FP f) {
  const unsigned long long key = f.b | 1ull;
  const unsigned long long mask = (1ull << log2) - 1ull;
  unsigned long long idx = f.a >> (64 - log2);
  for (int probe = 0; probe < 4096; probe++) {
    unsigned long long old = atomicCAS(&table[idx], 0ull, key);
    if (old == 0ull) return 1;
    if (old == key) return 0;
    idx = (idx + 1ull) & mask;
  }
  return -1;
}

__device__ __forceinline__ void set_flag(DevCounters* c, int f) { atomicOr(&c->flags, f); }

// The first violation found wins and is never replaced.  Called by the whole
// wave (bad = this lane's violated-invariant mask, 0 if none): one CAS per
// wave -- its first violating lane -- and none once a violation has been
// recorded, so successors that all violate an invariant (random states, or
// a violation reached by many parents) do not serialise on that one word.
// Returns true on the lane whose violation was recorded.
__device__ __forceinline__ bool claim_violation(DevCounters* c, int bad, int lane) {
  const unsigned long long m = __ballot(bad != 0);
  if (!m) return false;
  if (lane != __builtin_ctzll(m)) return false;
  if (__hip_atomic_load(&c->viol_mask, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0) return false;
  return atomicCAS(&c->viol_mask, 0, bad) == 0;
}

// Finish an insert whose home slot `idx` was READ (not CAS'd) as `seen`.
// Slots only ever change 0 -> key, so a slot holding the key proves the
// state is present, and one holding another key can be skipped for good;
// only an empty slot needs the CAS (which may then find the key after all).
__device__ __forceinline__ bool fpset_resolve_loaded(unsigned long long* table, int log2, unsigned long long key,
                                                     unsigned long long idx, unsigned long long seen,
                                                     DevCounters* ctr) {
  const unsigned long long mask = (1ull << log2) - 1ull;
  for (int probe = 1;; probe++) {
    if (seen == key) return false;
    if (seen == 0ull) {
      seen = atomicCAS(&table[idx], 0ull, key);
      if (seen == 0ull) return true;
      if (seen == key) return false;
    }
    if (probe >= 4096) {
      set_flag(ctr, FLAG_FPSET_FULL);
      return false;
    }
    idx = (idx + 1ull) & mask;
    seen = __hip_atomic_load(&table[idx], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// RTLA_CHECKED builds: every global row / parent-record index is checked
// against the buffer capacities the host stores in DevCounters; a bad index
// raises FLAG_BAD_INDEX (reported by rtla_step) instead of faulting.
#ifdef RTLA_CHECKED
#define RTLA_IDX_OK(ctr, idx, cap) ((idx) < (cap) ? true : (set_flag((ctr), FLAG_BAD_INDEX), false))
#else
#define RTLA_IDX_OK(ctr, idx, cap) true
#endif

// Finish an insert whose first CAS (at home slot `idx`) returned `old`:
// continue linear probing while the slot holds another key.  true = new.
__device__ __forceinline__ bool fpset_resolve(unsigned long long* table, int log2, unsigned long long key,
                                              unsigned long long idx, unsigned long long old, DevCounters* ctr) {
  const unsigned long long mask = (1ull << log2) - 1ull;
  for (int probe = 1; old != 0ull && old != key; probe++) {
    if (probe >= 4096) {
      set_flag(ctr, FLAG_FPSET_FULL);
      return false;
    }
    idx = (idx + 1ull) & mask;
    old = atomicCAS(&table[idx], 0ull, key);
  }
  return old == 0ull;
}

// Map the q-th candidate of a parent with `nmsg` bag slots to an instance id:
// the fixed families first, then Receive / Duplicate / Drop over used slots.
__device__ __forceinline__ int candidate_inst(const Layout& L, int q, int nmsg) {
  const int fixed = L.fam[F_RECEIVE];
  if (q < fixed) return q;
  int r = q - fixed;
  int fam = r / nmsg, slot = r - fam * nmsg;
  return fam_base(L, F_RECEIVE + fam) + slot;
}

__device__ __forceinline__ int inst_family(const Layout& L, int inst) {
  int fam = 0;
#pragma unroll
  for (int f = 1; f < F_COUNT; f++) fam += inst >= L.fam[f];
  return fam;
}

__device__ __forceinline__ int cover_code(const Layout& L, int inst, int sub) {
  int fam = 0;
#pragma unroll
  for (int f = 1; f < F_COUNT; f++) fam += inst >= L.fam[f];
  return fam == F_RECEIVE ? F_COUNT + sub : fam;
}

// Per-wave LDS: parent row (W, padded to even) | new allLogs words (32) |
// parent server-record hashes (NMAX FPs = 4 * NMAX words, 8-byte aligned) |
// staging rows (STAGE_ROWS * W).  The per-wave block is a multiple of 4
// words so every wave's hash slots stay 8-byte aligned.
__host__ __device__ constexpr int even_words(int W) { return (W + 1) & ~1; }
__host__ __device__ constexpr int wave_lds_words(int W) {
  return (even_words(W) + 32 + 4 * NMAX + STAGE_ROWS * W + 3) & ~3;
}

// (the readlane builtins return a signed int: widen through uint32_t)
__device__ __forceinline__ unsigned long long readlane_u64(unsigned long long v, int l) {
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, l);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), l);
  return (unsigned long long)lo | (unsigned long long)hi << 32;
}

// SYMMETRY: the successor parent + d through sym_key's accessors (server
// records, bag slots, election records), without materialising it:
// f(rec_of, nmsg, slot_of, nelec, elec_of).
template <int NS, class P, class F>
__device__ __forceinline__ auto with_successor(const Layout& L, P prow, const DeltaT<NS>& d, F f) {
  constexpr int EW = 2 + NS;
  const int ne0 = row_nelec(L, prow);
  auto rec_of = [&](int i, uint32_t* out) {
    load_rec<NS>(L, prow, i, out);
    if (i == d.srv) {
#pragma unroll
      for (int w = 0; w < 3 + NS; w++) out[w] = d.rec[w];
    }
  };
  auto slot_of = [&](int q) { return bag_get(L, prow, d, q); };
  auto elec_of = [&](int e, uint32_t* out) {
    if (e < ne0) {
      out[0] = elec_w0(L, prow, e);
      out[1] = elec_log(L, prow, e);
#pragma unroll
      for (int j = 0; j < NS; j++) out[2 + j] = elec_vl(L, prow, e, j);
    } else {
#pragma unroll
      for (int w = 0; w < EW; w++) out[w] = d.erec[w];
    }
  };
  return f(rec_of, d.nmsg, slot_of, ne0 + (d.elec ? 1 : 0), elec_of);
}
// Orbit key of the successor parent + d (allLogs' fingerprint afp).
template <int NS, class P>
__device__ __forceinline__ FP successor_orbit_key(const Layout& L, P prow, const DeltaT<NS>& d, FP afp) {
  return with_successor<NS>(L, prow, d, [&](auto rec_of, int nmsg, auto slot_of, int nelec, auto elec_of) {
    return sym_key<NS>(L, rec_of, nmsg, slot_of, nelec, elec_of, afp);
  });
}

// The orbit key in steps of one image (key_chunk's continuations): images
// [k, k + 1) of the successor parent + d -- or [k, |C(s)|) when `all` --
// folded into best (the least image fingerprint so far).  Returns the next
// image's index, or -1 once best is the least image (the key is then
// orbit_key_finish(best) + fp(allLogs'), as sym_key's).
template <int NS, class P>
__device__ __forceinline__ int successor_orbit_step(const Layout& L, P prow, const DeltaT<NS>& d, int k, bool all,
                                                    FP& best) {
  return with_successor<NS>(L, prow, d, [&](auto rec_of, int nmsg, auto slot_of, int nelec, auto elec_of) {
    const SymRank r = sym_rank<NS>(L, rec_of, nmsg, slot_of, nelec, elec_of);
    const int k1 = all ? r.ncomb : min(k + 1, r.ncomb);
    for (int j = k; j < k1; j++) {
      const FP f = sym_image_fp<NS>(L, rec_of, nmsg, slot_of, nelec, elec_of, r, j);
      if (fp_less(f, best)) best = f;
    }
    return k1 < r.ncomb ? k1 : -1;
  });
}

// a[j] += v for a run-time j (selects)
template <int NS>
__device__ __forceinline__ void add_at(uint32_t* a, uint32_t j, uint32_t v) {
#pragma unroll
  for (int k = 0; k < NS; k++)
    if ((uint32_t)k == j) a[k] += v;
}
// successor_orbit_step with the successor's signatures PATCHED from the
// parent's parts (psg[w * S], w < 3 * NS: srv_sig, sent and received message
// sums per server, computed once per parent row): the changed server's local
// part is recomputed, each bag write moves its old slot's share out of and
// its new slot's share into the sums -- no pass over the successor's bag and
// records.  The same signatures, hence the same key, as sym_rank's.
template <int NS, int S, class P>
__device__ __forceinline__ int successor_orbit_step_sig(const Layout& L, P prow, const DeltaT<NS>& d,
                                                        const uint32_t* psg, int k, bool all, FP& best) {
  return with_successor<NS>(L, prow, d, [&](auto rec_of, int nmsg, auto slot_of, int nelec, auto elec_of) {
    uint32_t ms[NS], mr[NS];
#pragma unroll
    for (int j = 0; j < NS; j++) {
      ms[j] = psg[(NS + j) * S];
      mr[j] = psg[(2 * NS + j) * S];
    }
#pragma unroll
    for (int q = 0; q < 3; q++) {
      if (q >= d.nops) continue;
      const uint64_t o = d.op_old[q], v = d.op_new[q];
      if (o) {
        const uint32_t c = slot_sig_sent(L, o);
        add_at<NS>(ms, slot_src(L, o), 0u - c);
        add_at<NS>(mr, slot_dst(L, o), 0u - slot_sig_recv(c));
      }
      if (v) {
        const uint32_t c = slot_sig_sent(L, v);
        add_at<NS>(ms, slot_src(L, v), c);
        add_at<NS>(mr, slot_dst(L, v), slot_sig_recv(c));
      }
    }
    const uint32_t lsrv = d.srv >= 0 ? srv_sig<NS>(d.srv, d.rec) : 0u;
    uint64_t sig[NS];
#pragma unroll
    for (int i = 0; i < NS; i++) sig[i] = sig_of(i == d.srv ? lsrv : psg[i * S], ms[i], mr[i]);
    const SymRank r = sym_rank_from<NS>(L, sig, rec_of, nmsg, slot_of, nelec, elec_of);
    const int k1 = all ? r.ncomb : min(k + 1, r.ncomb);
    for (int j = k; j < k1; j++) {
      const FP f = sym_image_fp<NS>(L, rec_of, nmsg, slot_of, nelec, elec_of, r, j);
      if (fp_less(f, best)) best = f;
    }
    return k1 < r.ncomb ? k1 : -1;
  });
}

// Load the parent row into LDS and derive the per-parent data every lane
// needs.  Returns the parent fingerprint with allLogs' already applied.
template <int NS>
__device__ __forceinline__ FP load_parent(const Layout& L, const uint32_t* __restrict__ src, uint32_t* prow,
                                          uint32_t* pall, FP* hsrv, int lane) {
  const int W = L.W;
  for (int w = lane; w < W; w += 64) prow[w] = src[w];
  wave_sync();
  FP afp{0, 0};
  if (lane < NS) {
    uint32_t rec[3 + NS];
    load_rec<NS>(L, prow, lane, rec);
    hsrv[lane] = h_srv(lane, rec, 3 + NS);
  } else if (lane == NS) {
    afp = alllogs_delta<NS>(L, prow, pall);
  }
  afp.a = readlane_u64(afp.a, NS);
  afp.b = readlane_u64(afp.b, NS);
  wave_sync();
  return fp_add(row_fp(prow), afp);
}

}  // namespace

// Helpers of the lane-per-state phases (k_expand_compact, k_pack_rows).
namespace {

struct LaneWords {  // word w of a per-lane array kept word-major (stride 64: bank-conflict free)
  uint32_t* p;
  __device__ __forceinline__ uint32_t& operator[](int w) const { return p[w * 64]; }
};
template <int S>
struct StridedWords {  // the same with stride S (one array per state of an S-state group)
  uint32_t* p;
  __device__ __forceinline__ uint32_t& operator[](int w) const { return p[w * S]; }
};

__device__ __forceinline__ unsigned long long wave_or_u64(unsigned long long v) {
  uint32_t lo = (uint32_t)v, hi = (uint32_t)(v >> 32);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    lo |= (uint32_t)__shfl_xor((int)lo, o);
    hi |= (uint32_t)__shfl_xor((int)hi, o);
  }
  return (unsigned long long)lo | (unsigned long long)hi << 32;
}
__host__ __device__ constexpr int lane_lds_words(int W, int AW) { return 64 * W + 64 * AW; }

}  // namespace

// ------------------------------------------------------------------------
// k_expand_compact: the single-shard BFS level kernel with work compaction.
//
// A wave owns 64 consecutive frontier rows in LDS.  Each lane first
// computes, for its own state, the bit mask of action instances whose
// enabling guard holds (the guards of raft.tla's actions, below).  The wave
// then lists the (state, instance) pairs in instance-major order -- so
// consecutive pairs belong to the same family of Next -- and evaluates them
// 64 at a time, one pair per lane.  Every lane of a chunk does useful work
// and a chunk spans at most a few families, instead of sweeping all ~45
// instances with most lanes idle.  Fingerprint-set CAS of chunk c are
// resolved after chunk c+1 is computed; new states go to a per-wave LDS list
// and reserve next-frontier slots 64+ at a time (one atomic per flush).
namespace {

constexpr int RING = 128;   // pair ring (u16: state lane << 8 | instance - window base)
constexpr int NEWCAP = 512; // new-state list (u16: state lane << 8 | instance)
// The list is built into rows at the group's end; a group that finds more
// new states (early levels) flushes it when it holds more than this many --
// after which one chunk (<= 64) and a drain (<= 2 x 64) may still add
// entries before the flush.
constexpr int NEWFLUSH = NEWCAP - 3 * 64;


// Per-wave LDS of k_expand_compact (16-byte aligned pieces first):
// per-state fingerprint with allLogs' applied (GROUP FPs) | SYMMETRY: the
// fingerprint of each state's allLogs' (GROUP FPs) | per-owner (base, used)
// of the open outbox chunk | pending new states (NEWCAP u16 entries) |
// GROUP rows | allLogs' words of each state | pair ring | SYMMETRY: key ring,
// key continuations (64 least-image-so-far FPs, 64 entries).
// (The outbox state exists only in the MULTI kernels: one shard's tile then
// stays small enough for 12 one-wave blocks per CU on configs[1]'s 372-byte rows.)
__host__ __device__ constexpr int compact_lds_words(int W, int AW, int GROUP, bool sym, bool multi) {
  return (4 * GROUP * (sym ? 2 : 1) + (multi ? 4 * SHARD_MAX : 0) + NEWCAP / 2 + GROUP * W + GROUP * AW +
          RING / 2 * (sym ? 2 : 1) + (sym ? 5 * 64 + 3 * NMAX * GROUP : 0) + 3) & ~3;
}

// bits << off into a 64-bit window mask (off may be negative or >= 64)
__device__ __forceinline__ unsigned long long win_bits(unsigned long long bits, int off) {
  if (off >= 64 || off <= -64) return 0ull;
  return off >= 0 ? bits << off : bits >> (-off);
}

// Instances [wb, wb+64) whose enabling guard holds in `row`.  A superset is
// safe (compute_delta re-checks every guard); a subset would lose states.
// dup = false: without DuplicateMessage (counted apart, see dup_counted).
template <int NS>
__device__ __forceinline__ unsigned long long cand_mask(const Layout& L, const uint32_t* row, int nmsg, int wb,
                                                        bool dup = true) {
  constexpr int N = NS;
  unsigned long long rv = 0, bl = 0, ldr = 0, tmo = 0;
#pragma unroll
  for (int i = 0; i < N; i++) {
    const uint32_t w0 = srv_w0(L, row, i);
    const uint32_t role = s_role(w0);
    if (role == FOLLOWER || role == CANDIDATE) tmo |= 1ull << i;          // Timeout :178-181
    if (role == CANDIDATE) {
      rv |= (unsigned long long)(~s_vresp(w0) & ((1u << N) - 1u)) << (i * N);  // RequestVote :190-192
      if (__builtin_popcount(s_vgrant(w0)) * 2 > N) bl |= 1ull << i;     // BecomeLeader :229-231
    }
    if (role == LEADER) ldr |= 1ull << i;                                 // :204-206, :246-248, :259-260
  }
  unsigned long long ae = 0, cr = 0;
#pragma unroll
  for (int i = 0; i < N; i++)
    if (ldr >> i & 1ull) {
      ae |= (((1ull << N) - 1ull) & ~(1ull << i)) << (i * N);             // AppendEntries i /= j
      cr |= ((1ull << L.V) - 1ull) << (i * L.V);                           // ClientRequest(i, v)
    }
  const unsigned long long bag = nmsg >= 64 ? ~0ull : ((1ull << nmsg) - 1ull);
  unsigned long long m = 0;
  m |= win_bits((1ull << N) - 1ull, L.fam[F_RESTART] - wb);               // Restart: always
  m |= win_bits(tmo, L.fam[F_TIMEOUT] - wb);
  m |= win_bits(rv, L.fam[F_REQUESTVOTE] - wb);
  m |= win_bits(bl, L.fam[F_BECOMELEADER] - wb);
  m |= win_bits(cr, L.fam[F_CLIENTREQUEST] - wb);
  m |= win_bits(ldr, L.fam[F_ADVANCECOMMIT] - wb);
  m |= win_bits(ae, L.fam[F_APPENDENTRIES] - wb);
  m |= win_bits(bag, L.fam[F_RECEIVE] - wb);
  if (dup) m |= win_bits(bag, L.fam[F_DUPLICATE] - wb);
  m |= win_bits(bag, L.fam[F_DROP] - wb);
  return m;
}

// Zero records (fp 0:0, skipped by k_insert_remote) in outbox slots [from, to) of owner o.
__device__ __forceinline__ void outbox_holes(const ShardBox& box, int o, unsigned long long from,
                                             unsigned long long to, int lane) {
  to = min(to, box.cap);
  for (unsigned long long j = from + lane; j < to; j += 64) {
    const unsigned long long k = (unsigned long long)o * box.cap + j;
    box.send_fp[2 * k] = 0ull;
    box.send_fp[2 * k + 1] = 0ull;
  }
}

// Home slot of a key in a table of 2^lg slots (lg = 0: no table, slot 0).
__device__ __forceinline__ unsigned long long home_slot(const FP& key, int lg) {
  return lg ? key.a >> (64 - lg) : 0ull;
}

__device__ __forceinline__ unsigned long long shfl_u64(unsigned long long v, int src) {
  const uint32_t lo = (uint32_t)__shfl((int)(uint32_t)v, src);
  const uint32_t hi = (uint32_t)__shfl((int)(uint32_t)(v >> 32), src);
  return (unsigned long long)lo | (unsigned long long)hi << 32;
}

}  // namespace

#ifndef RTLA_COMPACT_WAVES_PER_EU
#define RTLA_COMPACT_WAVES_PER_EU 3  // 168 VGPRs (3 waves/SIMD); spills per instantiation: profiles/r04_*/resource_usage.txt
#endif
#ifndef RTLA_SYM_WAVES_PER_EU
#define RTLA_SYM_WAVES_PER_EU 4      // SYMMETRY, the key pass a call of its own (key_one): 128 VGPRs (configs[3]:
                                     // 311.5 ms, 16-state groups) beat 168 (343 ms) and 102 (414 ms)
#endif
#ifndef RTLA_DUP_COUNTED
#define RTLA_DUP_COUNTED 1  // 0: evaluate every DuplicateMessage successor (A/B builds)
#endif
#ifndef RTLA_DUP_NARROW
#define RTLA_DUP_NARROW 0   // 1: count them in the narrow-row kernels too (A/B builds)
#endif
#ifndef RTLA_MULTI_ASYNC
#define RTLA_MULTI_ASYNC 1  // multi-shard kernels pipeline their CAS too
#endif
#ifndef RTLA_SYM_SPLIT
#define RTLA_SYM_SPLIT 1  // SYMMETRY: orbit keys in a pass of their own (key_chunk), not inside the evaluation
#endif
// The layout the kernel runs on: the run-time argument, or (LC.N != 0) the
// configuration compiled in as a template parameter, whose fields the
// compiler then folds into every offset, bound and loop of the model code.
template <Layout LC>
__device__ __forceinline__ const Layout& pick_layout(const Layout& rt) {
  if constexpr (LC.N == 0) return rt;
  else return LC;
}

namespace {
// One key_chunk lane as a function of its own: the successor's Delta, then
// successor_orbit_step from image k with the least image so far best0.
// next >= 0: f is the least image so far and image `next` is due; next ==
// -1: f is the orbit key; next == -2: the instance is not enabled.  NOT
// inlined, so that its registers are allocated apart from the level
// kernel's: inlined, the continuation bookkeeping spilled the kernel to 712
// VGPRs (750 ms per configs[3] step); as a call, 343 ms against 355 ms for
// the inlined all-images key pass (profiles/r04_v4).
struct KeyStep {
  FP f;
  int next;
};
template <int NS, Layout LC, int S>
__device__ __noinline__ KeyStep key_one(const Layout& Lrt, const uint32_t* prow, const uint32_t* psg, int inst, int k,
                                        bool all, FP best0, FP afp) {
  const Layout& L = pick_layout<LC>(Lrt);
  DeltaT<NS> d;
  d.enabled = 0;
  compute_delta<NS>(L, prow, inst, d);
  KeyStep r{FP{0, 0}, -1};
  if (!d.enabled) {
    r.next = -2;
    return r;
  }
  FP best = best0;
  r.next = successor_orbit_step_sig<NS, S>(L, prow, d, psg, k, all, best);
  r.f = r.next < 0 ? fp_add(orbit_key_finish(best), afp) : best;
  return r;
}

// One build_all lane as a function of its own (SYMMETRY kernels): the new
// state's full Delta, fingerprint and invariants, then the words in which its
// row differs from the parent's copy (child_write; `wait`: the copies must
// land first).  NOT inlined for the same reason as key_one: at the SYMMETRY
// kernel's 128 VGPRs the inlined build pass is one of the two big spillers.
#ifndef RTLA_SYM_BUILD_CALL
#define RTLA_SYM_BUILD_CALL 1
#endif
struct BuildOut {
  int bad, sub, in_model;
};
template <int NS, Layout LC, int GROUP>
__device__ __noinline__ BuildOut build_one(const Layout& Lrt, const uint32_t* prow, int inst, FP qfp,
                                           const uint32_t* pall_p, uint32_t* d1, uint32_t* base2, int n1, int off,
                                           bool write, bool wait) {
  const Layout& L = pick_layout<LC>(Lrt);
  DeltaT<NS> d;
  d.enabled = 0;
  compute_delta<NS>(L, prow, inst, d);
  const FP cfp = fp_add(qfp, delta_fp<NS>(L, prow, d));
  BuildOut o{check_invariants_v<NS>(L, prow, d.srv, d.rec[0], d.rec[1], d.elec, d.erec[0]), d.sub, d.in_model};
  uint32_t spk[PACKW], epk[PACKW];
  child_pack(L, d, spk, epk);
  if (wait) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (write)
    child_write(L, prow, d, spk, epk, StridedWords<GROUP>{const_cast<uint32_t*>(pall_p)}, cfp, [&](int w, uint32_t v) {
      const int i = off + w;
      if (i < n1) d1[i] = v;
      else base2[i - n1] = v;
    });
  return o;
}

}  // namespace

// RTLA_STAMPS (diagnostic builds only): per-wave cycle counts of the level
// kernel's phases from s_memtime (each stamp waits for the wave's LDS
// operations in flight: a perturbation, fine for shares) summed into
// DevCounters::stamp.
#ifdef RTLA_STAMPS
#define RTLA_STAMP_DECL                                                   \
  unsigned long long st_prev_ = __builtin_amdgcn_s_memtime();              \
  unsigned long long st_acc_[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#define STAMP(k)                                                             \
  do {                                                                       \
    const unsigned long long t_ = __builtin_amdgcn_s_memtime();              \
    st_acc_[k] += t_ - st_prev_;                                             \
    st_prev_ = t_;                                                           \
  } while (0)
#define RTLA_STAMP_FLUSH(ctr, lane)                                          \
  if ((lane) == 0)                                                           \
    for (int k_ = 0; k_ < 8; k_++) atomicAdd(&(ctr)->stamp[k_], st_acc_[k_]);
#else
#define RTLA_STAMP_DECL
#define STAMP(k)
#define RTLA_STAMP_FLUSH(ctr, lane)
#endif

// GROUP: frontier states per wave-group (64, or 32 for wide rows: halves the
// LDS tile so more waves fit a CU).  LC: compiled-in layout (Layout{} = use
// the run-time argument Lrt).  SYM: SYMMETRY Permutations(Server) -- the
// probe pass evaluates the full Delta of each successor and probes its orbit
// key (successor_orbit_key) instead of its fingerprint; rows keep the states
// themselves.
// Waves per SIMD the level kernel's registers are budgeted for: narrow
// compiled-in rows (<= 32 words: the exhaust model's 84 B) fit 4 (128
// VGPRs; its 74 levels 1259 -> 1158 ms; 5 waves: 1605 ms), wider ones 3 (at 4: configs[1]
// 197.9 -> 215.6 ms, configs[2] 90.0 -> 100.0 ms, configs[0]'s 37-word rows
// 300.9 -> 328.0 ms; profiles/r04_v4/waves{3,4}_*).
#ifndef RTLA_NARROW_W
#define RTLA_NARROW_W 32  // rows of at most this many words get RTLA_NARROW_WAVES waves/SIMD
#endif
#ifndef RTLA_NARROW_WAVES
#define RTLA_NARROW_WAVES 4
#endif
constexpr int compact_waves(const Layout& L, bool sym) {
  return sym ? RTLA_SYM_WAVES_PER_EU
             : (L.N != 0 && L.W <= RTLA_NARROW_W ? RTLA_NARROW_WAVES : RTLA_COMPACT_WAVES_PER_EU);
}
template <int NS, bool MULTI, int GROUP, Layout LC, bool SYM>
__global__ void __launch_bounds__(256)
__attribute__((amdgpu_waves_per_eu(compact_waves(LC, SYM))))
k_expand_compact(Layout Lrt, Ring cur, unsigned long long s_begin, unsigned long long s_end,
                 unsigned long long cur_base, Ring next, unsigned long long* __restrict__ parents,
                 unsigned long long next_base, unsigned long long next_cap, unsigned long long* table,
                 unsigned long long* sent, int tlog2, DevCounters* ctr, ShardBox box, int xflags) {
  const Layout& L = pick_layout<LC>(Lrt);
  constexpr bool KSPLIT = SYM && RTLA_SYM_SPLIT;
  const int me = box.me;
  extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
  __shared__ unsigned int cov[2 * COVER_CODES];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int W = L.W, AW = L.all_words;
  uint32_t* wl = lds + wave * compact_lds_words(W, AW, GROUP, SYM, MULTI);
  FP* pfpl = reinterpret_cast<FP*>(wl);  // [state lane]: its fingerprint + the allLogs' change (raft.tla:465)
  FP* afpl = pfpl + GROUP;               // SYM [state lane]: fingerprint of its allLogs'
  unsigned long long* obox =             // [o] base of the open chunk, [SHARD_MAX + o] used
      reinterpret_cast<unsigned long long*>(wl + 4 * GROUP * (SYM ? 2 : 1));
  uint16_t* newl = reinterpret_cast<uint16_t*>(obox + (MULTI ? 2 * SHARD_MAX : 0));
  uint32_t* rows = reinterpret_cast<uint32_t*>(newl + NEWCAP);
  uint32_t* pall = rows + GROUP * W;  // allLogs' words of state lane l: pall[l + w * GROUP]
  const StridedWords<GROUP> pall_mine{pall + (lane & (GROUP - 1))};
  uint16_t* ring = reinterpret_cast<uint16_t*>(pall + GROUP * AW);
  // SYMMETRY: successors that need an orbit key (in-model, not the parent),
  // queued by the evaluation pass and keyed 64 at a time (key_chunk)
  uint16_t* kring = ring + RING;
  int kpos = 0, kdone = 0;
  // SYMMETRY: successors whose orbit key needs more images than key_chunk
  // computes per pass (one): entry (state lane << 8 | instance | next image
  // << 16) and the least image fingerprint so far; taken first by the next
  // key chunk (ccount of them, uniform)
  FP* cbest = reinterpret_cast<FP*>(kring + (SYM ? RING : 0));
  uint32_t* cent = reinterpret_cast<uint32_t*>(cbest + (SYM ? 64 : 0));
  int ccount = 0;
  // SYMMETRY: each tile row's signature parts (sym_sig_parts: srv_sig, sent
  // and received message sums per server), word w of row r at sigl[w * GROUP + r]
  uint32_t* sigl = cent + (SYM ? 64 : 0);
  if (MULTI) {
    if (lane < SHARD_MAX) {
      obox[lane] = ~0ull;
      obox[SHARD_MAX + lane] = OBOX_CHUNK;
    }
    wave_sync();
  }
  for (int k = threadIdx.x; k < 2 * COVER_CODES; k += blockDim.x) cov[k] = 0;
  __syncthreads();

  unsigned my_gen = 0, my_probe = 0;
  unsigned my_dup = 0;  // DuplicateMessage successors counted, not evaluated (dup_counted)
#ifdef RTLA_COUNT_CAS
  unsigned my_cas = 0;
#endif
  const int ninst = L.fam[F_COUNT];
  const unsigned long long lanes_below = (1ull << lane) - 1ull;
  // DuplicateMessage successors counted, not evaluated (see the group loop)
  // (not in the narrow-row kernels at 4 waves/SIMD: the exhaust model's spills
  // grow 39 -> 58 VGPRs with it and its run slows 1156 -> 1320 ms)
  constexpr bool narrow = !SYM && LC.N != 0 && LC.W <= RTLA_NARROW_W;
  const bool dup_counted = RTLA_DUP_COUNTED && (!narrow || RTLA_DUP_NARROW) && L.C == 1 &&
                           !(xflags & (XF_ALL_SUCCESSORS | XF_NO_CHUNKS));
  RTLA_STAMP_DECL
  // pending probe (issued by the previous chunk).  MULTI: a successor owned
  // by another shard probes this shard's SENT cache instead of the set --
  // a dedup hint, one slot per fingerprint (2^box.slog2 slots), overwritten
  // on a miss: a hit drops the copy (this shard sent it to its owner
  // already), a miss queues its (fingerprint, parent) record for the owner
  // and stores the key in the slot (a plain store, issued like the CAS of a
  // set insert and reported a chunk later).  Bounded work per probe, never
  // full; a slot overwritten by another key only costs a duplicate record,
  // which the owner deduplicates.
  bool pend = false;
  unsigned long long pold = 0;
  FP pf{0, 0};       // its fingerprint (home slot and owner derive from it)
  uint32_t pinfo = 0;  // its state lane << 16 | action instance
  // A probe whose home-slot load did not show its key issues ONE CAS -- at
  // the home slot if it read empty, else at the next slot (linear probing;
  // slots only ever go 0 -> key) -- together with the next chunk's loads,
  // and that CAS is resolved a chunk later: neither the insert nor the first
  // collision step waits for a round trip.  (MULTI, a successor another
  // shard owns: the sent-cache store instead, see above.)
  const bool async_cas = (!MULTI || RTLA_MULTI_ASYNC) && !(xflags & XF_CAS_ONLY);
  bool cpend = false;    // CAS set up by resolve(), issued by issue_cas()
  bool cflight = false;  // CAS in flight (result in cold)
  unsigned long long cold = 0, ckey = 0, cidx = 0;
  uint32_t cinfo = 0;
  FP cf{0, 0};     // MULTI: the CAS'd successor's fingerprint (its outbox record) ...
  int cowner = me; // ... and owner
  // New states found so far whose rows are not built yet: newl[head, tail)
  // (mod NEWCAP) holds (state lane, instance); their parents are rows of the
  // current group (uniform counters).  They are built when the group's probes
  // have drained (build_all), so no probe or CAS state is live while the
  // rows are built.
  int head = 0, tail = 0;
  unsigned long long dedup_new = 0;  // XF_DEDUP_ONLY: new fingerprints (uniform)
  unsigned long long s0 = 0;  // first state of the current group

  // Build the rows of every pending new state (probes drained), one
  // next-level slot reservation for all of them (slots past next_cap are
  // dropped and flagged: the level is then reported incomplete):
  //  (1) the wave copies each parent row (LDS) to its child's slot with
  //      coalesced stores, for all of them (copying per batch of 64 instead,
  //      so that the patches reach lines still in L2, was measured: no
  //      fewer HBM writes, 5 % slower);
  //  (2) per batch of 64, one state per lane: its full Delta (compute_delta
  //      with slot bookkeeping; the probe pass only folded it into a hash),
  //      fingerprint, invariants and distinct coverage -- the first batch's
  //      arithmetic overlaps the copies in flight;
  //  (3) after the copies landed (one wait), each lane stores the words in
  //      which its child differs from the parent (child_write, rtla_model.h).
  // No separate row-building kernel: no parent-record read, no parent-row
  // gather, no second launch.
  // compute_delta over a chunk of lanes, specialised for its family when the
  // whole chunk holds one (D = DeltaFpT for the probe pass, DeltaT for the
  // row build and orbit keys)
  auto chunk_delta = [&](bool active, const uint32_t* prow, int inst, auto& d) {
    const int f0 = inst_family(L, __builtin_amdgcn_readfirstlane(inst));
    const bool one_family = __ballot(active && inst_family(L, inst) != f0) == 0ull;
    if (!one_family || (xflags & XF_GENERIC_DELTA)) {
      if (active) compute_delta<NS>(L, prow, inst, d);
    } else if (active) {
      switch (f0) {  // one family in the whole chunk: its code only
        case F_RESTART: compute_delta<NS, F_RESTART>(L, prow, inst, d); break;
        case F_TIMEOUT: compute_delta<NS, F_TIMEOUT>(L, prow, inst, d); break;
        case F_REQUESTVOTE: compute_delta<NS, F_REQUESTVOTE>(L, prow, inst, d); break;
        case F_BECOMELEADER: compute_delta<NS, F_BECOMELEADER>(L, prow, inst, d); break;
        case F_CLIENTREQUEST: compute_delta<NS, F_CLIENTREQUEST>(L, prow, inst, d); break;
        case F_ADVANCECOMMIT: compute_delta<NS, F_ADVANCECOMMIT>(L, prow, inst, d); break;
        case F_APPENDENTRIES: compute_delta<NS, F_APPENDENTRIES>(L, prow, inst, d); break;
        case F_RECEIVE: compute_delta<NS, F_RECEIVE>(L, prow, inst, d); break;
        case F_DUPLICATE: compute_delta<NS, F_DUPLICATE>(L, prow, inst, d); break;
        default: compute_delta<NS, F_DROP>(L, prow, inst, d); break;
      }
    }
  };
  auto build_all = [&]() {
    const int ntot = tail - head;  // uniform
    if (ntot == 0) return;
    unsigned long long obase = 0;
    if (lane == 0) obase = atomicAdd(&ctr->next_count, (unsigned long long)ntot);
    obase = shfl0_u64(obase);
    if (obase + ntot > next_cap && lane == 0) set_flag(ctr, FLAG_FRONTIER_FULL);
    const int nrows = obase >= next_cap ? 0 : (int)min<unsigned long long>((unsigned long long)ntot, next_cap - obase);
    const bool rows_on = !(xflags & XF_NO_MATERIALIZE) && RTLA_IDX_OK(ctr, obase + nrows, ctr->cap_next + 1);
    const unsigned long long p0 = ring_idx(next, obase);
    const int n1 = (int)min<unsigned long long>(next.cap - p0, (unsigned long long)nrows) * W;  // words before the wrap
    uint32_t* d1 = next.base + p0 * (unsigned long long)W;
    // (1) for child rows [rb, re): word i of the run, lane-contiguous
    auto copy_rows = [&](int rb, int re) {
      const int nwords = re * W;
      int r = rb, w = lane;
      while (w >= W) { w -= W; r++; }
      for (int i0 = rb * W; i0 < nwords; i0 += 64) {
        const int i = i0 + lane;
        if (i < nwords) {
          const int sr = newl[(head + r) & (NEWCAP - 1)] >> 8;
          const uint32_t v = rows[sr * W + w];
          if (i < n1) d1[i] = v;
          else next.base[i - n1] = v;
        }
        w += 64;
        while (w >= W) { w -= W; r++; }
      }
    };
    if (rows_on) copy_rows(0, nrows);  // (all of them first: one pass of coalesced stores)
    for (int b = 0; b < ntot; b += 64) {  // (2), (3)
      const bool act = b + lane < ntot;
      const int e = act ? newl[(head + b + lane) & (NEWCAP - 1)] : 0;
      const int sl = e >> 8, inst = e & 255;
      const int child = b + lane;  // index in the run
      if constexpr (SYM && RTLA_SYM_BUILD_CALL) {  // the lane's work as a call of its own (build_one)
        BuildOut o{0, 0, 0};
        if (act)
          o = build_one<NS, LC, GROUP>(Lrt, rows + sl * W, inst, pfpl[sl], pall + sl, d1, next.base, n1, child * W,
                                      rows_on && child < nrows, rows_on && b == 0);
        else if (rows_on && b == 0)
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if (!(xflags & XF_ALL_SUCCESSORS) && claim_violation(ctr, o.bad, lane)) {
          ctr->viol_parent = cur_base + s0 + sl;
          ctr->viol_inst = inst;
          ctr->viol_in_model = 1;
          ctr->viol_child = child < nrows ? next_base + obase + child : ~0ull;
        }
        if (!(xflags & XF_NO_COVER)) {
          const int code = act ? cover_code(L, inst, o.sub) : -1;
          const unsigned long long am = __ballot(act);
          if (am) {
            const int c0 = __shfl(code, __builtin_ctzll(am));
            const bool same = act && code == c0;
            const int n0 = __popcll(__ballot(same));
            if (lane == 0) atomicAdd(&cov[COVER_CODES + c0], (unsigned)n0);
            if (act && !same) atomicAdd(&cov[COVER_CODES + code], 1u);
          }
        }
        if (child < nrows && RTLA_IDX_OK(ctr, next_base + obase + child, ctr->cap_parents))
          parents[next_base + obase + child] =
              (xflags & XF_ALL_SUCCESSORS)
                  ? (cur_base + s0 + sl) << 32 | (unsigned long long)(o.in_model ? 1u : 0u) << 31 |
                        (unsigned long long)o.sub << 16 | (unsigned long long)inst
                  : (unsigned long long)me << 56 | (cur_base + s0 + sl) << 16 | (unsigned long long)inst;
        continue;
      }
      DeltaT<NS> d;
      d.enabled = 0;
      if (act) compute_delta<NS>(L, rows + sl * W, inst, d);
      const FP qfp = pfpl[sl];
      FP cfp{0, 0};
      int bad = 0;
      if (act) {
        const uint32_t* prow = rows + sl * W;
        cfp = fp_add(qfp, delta_fp<NS>(L, prow, d));
        bad = check_invariants_v<NS>(L, prow, d.srv, d.rec[0], d.rec[1], d.elec, d.erec[0]);
      }
      if (!(xflags & XF_ALL_SUCCESSORS) && claim_violation(ctr, bad, lane)) {
        ctr->viol_parent = cur_base + s0 + sl;
        ctr->viol_inst = inst;
        ctr->viol_in_model = 1;
        ctr->viol_child = child < nrows ? next_base + obase + child : ~0ull;
      }
      if (!(xflags & XF_NO_COVER)) {  // distinct coverage, aggregated over equal codes
        const int code = act ? cover_code(L, inst, d.sub) : -1;
        const unsigned long long am = __ballot(act);
        if (am) {
          const int c0 = __shfl(code, __builtin_ctzll(am));
          const bool same = act && code == c0;
          const int n0 = __popcll(__ballot(same));
          if (lane == 0) atomicAdd(&cov[COVER_CODES + c0], (unsigned)n0);
          if (act && !same) atomicAdd(&cov[COVER_CODES + code], 1u);
        }
      }
      uint32_t spk[PACKW], epk[PACKW];  // the changed records, packed
      if (act) child_pack(L, d, spk, epk);
      if (rows_on) {  // (3): the copies must land first (same words, other lanes)
        if (b == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if (child < nrows) {
          const StridedWords<GROUP> pall_p{pall + sl};
          const int off = child * W;
          child_write(L, rows + sl * W, d, spk, epk, pall_p, cfp, [&](int w, uint32_t v) {
            const int i = off + w;
            if (i < n1) d1[i] = v;
            else next.base[i - n1] = v;
          });
        }
      }
      if (child < nrows && RTLA_IDX_OK(ctr, next_base + obase + child, ctr->cap_parents))
        parents[next_base + obase + child] =
            (xflags & XF_ALL_SUCCESSORS)
                ? (cur_base + s0 + sl) << 32 | (unsigned long long)(d.in_model ? 1u : 0u) << 31 |
                      (unsigned long long)d.sub << 16 | (unsigned long long)inst
                : (unsigned long long)me << 56 | (cur_base + s0 + sl) << 16 | (unsigned long long)inst;
    }
    head = tail;
  };
  auto issue_cas = [&]() {
#ifdef RTLA_COUNT_CAS
    if (cpend) my_cas++;
#endif
    if (cpend) {
      if (MULTI && cowner != me) {  // the sent cache: overwrite, report "not sent before"
        if (box.slog2) sent[cidx] = ckey;
        cold = 0ull;
      } else {
        cold = atomicCAS(&table[cidx], 0ull, ckey);
      }
    }
    cflight = cpend;
    cpend = false;
  };
  auto resolve = [&]() {
    bool isnew = false;
    // the state isnew refers to: its (tile row, instance), fingerprint and owner
    uint32_t ninfo = pinfo;
    const int powner = MULTI ? fp_owner(pf, box.nshard) : me;
    FP nf = pf;
    int nowner_r = powner;
    if (xflags & XF_ALL_SUCCESSORS) {  // every enabled successor is output (no seen set)
      isnew = pend;
    } else if (async_cas) {
      if (cflight) {  // the CAS issued one chunk ago
        if (cold == 0ull) isnew = true;
        else if (cold != ckey)  // rare: keep probing (the set only: a sent-cache store reports 0)
          isnew = fpset_resolve(table, tlog2, ckey, cidx, cold, ctr);
      }
      ninfo = cinfo;
      nf = cf;
      nowner_r = cowner;
      cflight = false;
      if (pend) {  // this chunk's load -> seen, or a CAS (sent cache: a store) for the next issue
        const bool to_sent = MULTI && powner != me;
        const int lg = to_sent ? box.slog2 : tlog2;
        const unsigned long long key = pf.b | 1ull, idx = to_sent ? home_slot(pf, lg) : pf.a >> (64 - lg);
        if (pold != key) {
          cidx = (to_sent || pold == 0ull) ? idx : ((idx + 1ull) & ((1ull << lg) - 1ull));
          ckey = key;
          cinfo = pinfo;
          if (MULTI) {
            cf = pf;
            cowner = powner;
          }
          cpend = true;
        }
      }
    } else if (pend) {
      if (MULTI && powner != me) {  // the sent cache: a miss overwrites the slot
        isnew = pold != (pf.b | 1ull);
        if (isnew && box.slog2) sent[home_slot(pf, box.slog2)] = pf.b | 1ull;
      } else {
        const unsigned long long pidx = pf.a >> (64 - tlog2);
        isnew = (xflags & XF_CAS_ONLY) ? fpset_resolve(table, tlog2, pf.b | 1ull, pidx, pold, ctr)
                                       : fpset_resolve_loaded(table, tlog2, pf.b | 1ull, pidx, pold, ctr);
      }
    }
    if (MULTI) {  // records for other owners: all owners' outbox slots reserved in one step
      const int powner = nowner_r;
      const FP pf = nf;
      const bool rem = isnew && powner != me;
      isnew = isnew && powner == me;
      if (__ballot(rem)) {
        // lane o learns how many records owner o gets (ocnt), each record its
        // rank among its owner's (r)
        unsigned long long mym = 0;
        int ocnt = 0;
        for (int o = 0; o < box.nshard; o++) {
          const unsigned long long m = __ballot(rem && powner == o);
          if (powner == o) mym = m;
          if (lane == o) ocnt = __popcll(m);
        }
        // lane o keeps owner o's open chunk of OBOX_CHUNK slots (obox[o] =
        // its base, obox[SHARD_MAX + o] = slots used); a run that does not fit
        // continues in a fresh chunk (one atomic per OBOX_CHUNK records, no holes)
        unsigned long long b1 = 0, b2 = 0;
        int room = 0;
        if (ocnt > 0) {
          const unsigned long long b = obox[lane], used = obox[SHARD_MAX + lane];
          room = b == ~0ull ? 0 : (int)(OBOX_CHUNK - used);
          b1 = b + used;
          if (ocnt > room) {
            b2 = atomicAdd(&box.out_count[lane], (unsigned long long)OBOX_CHUNK);
            obox[lane] = b2;
            obox[SHARD_MAX + lane] = (unsigned long long)(ocnt - room);
          } else {
            obox[SHARD_MAX + lane] = used + (unsigned long long)ocnt;
          }
        }
        const int src = rem ? powner : 0;
        b1 = shfl_u64(b1, src);
        b2 = shfl_u64(b2, src);
        room = __shfl(room, src);
        const int r = __popcll(mym & lanes_below);
        const unsigned long long slot = r < room ? b1 + r : b2 + (r - room);
        const unsigned long long ref = (s0 + (ninfo >> 16)) << 16 | (unsigned long long)(ninfo & 0xffffu);
        if (rem && slot < box.cap) {
          const unsigned long long k = (unsigned long long)powner * box.cap + slot;
          box.send_fp[2 * k] = pf.a;
          box.send_fp[2 * k + 1] = pf.b;
          box.send_ref[k] = ref;
        }
        // past the region's end (the groups in flight when it filled): the
        // overflow list, sent next round
        const bool ov = rem && slot >= box.cap;
        const unsigned long long om = __ballot(ov);
        if (om) {
          unsigned long long ob = 0;
          if (lane == 0) ob = atomicAdd(box.over_count, (unsigned long long)__popcll(om));
          ob = shfl0_u64(ob);
          if (ov) {
            const unsigned long long k = ob + __popcll(om & lanes_below);
            if (k < box.over_cap) {
              box.over_fp[2 * k] = pf.a;
              box.over_fp[2 * k + 1] = pf.b;
              box.over_ref[k] = ref;
            } else {
              set_flag(ctr, FLAG_OUTBOX_FULL);
            }
          }
        }
      }
    }
    const unsigned long long m = __ballot(isnew);
    if (m && (xflags & XF_DEDUP_ONLY)) {  // synthetic microbench: count, keep no row
      dedup_new += __popcll(m);
    } else if (m) {
      if (isnew) newl[(tail + __popcll(m & lanes_below)) & (NEWCAP - 1)] = (uint16_t)((ninfo >> 16) << 8 | (ninfo & 255u));
      tail += __popcll(m);
      wave_sync();
    }
    pend = false;
  };

  // ---- one chunk: lane t evaluates ring entry done + t (tile row << 8 |
  // instance).  The outcome -- whether and where it probes -- is kept for
  // issue_probe(), which runs after the previous chunk's probes resolved.
  bool nprobe = false;
  unsigned long long nidx = 0;
  FP ncf{0, 0};
  int nowner = me;
  uint32_t ninfo_new = 0;
  auto eval_chunk = [&](int done, int cnt) {
    const bool active = lane < cnt;
    const int e = active ? ring[(done + lane) & (RING - 1)] : 0;
    const int sl = e >> 8, inst = e & 255;
    const uint32_t* prow = rows + sl * W;
    const FP qfp = pfpl[sl];
    std::conditional_t<SYM && !KSPLIT, DeltaT<NS>, DeltaFpT<NS>> d;
    d.enabled = 0;
    if (!(xflags & XF_NO_DELTA)) chunk_delta(active, prow, inst, d);
    bool en = d.enabled != 0;
    if (en && d.err) {
      set_flag(ctr, d.err == 1 ? FLAG_SPEC_ERROR : FLAG_ROW_OVERFLOW);
      en = false;
    }
    my_gen += en ? 1u : 0u;
    bool kq = false;
    nprobe = false;
    nidx = 0;
    ncf = FP{0, 0};
    nowner = me;
    ninfo_new = (uint32_t)sl << 16 | (uint32_t)inst;
    if (en && (xflags & XF_ALL_SUCCESSORS)) {
      nprobe = true;  // "probe" = output it: issue_probe skips the load, resolve takes it as new
    } else if (en && d.in_model) {
      FP cfp;
      if constexpr (SYM && !KSPLIT) cfp = fp_add(qfp, delta_fp<NS>(L, prow, d));
      else
        cfp = (xflags & XF_NO_HASH) ? FP{qfp.a + d.rec[0] + (uint64_t)d.fmsg.a, qfp.b + d.rec[1]}
                                    : fp_add(qfp, delta_fp<NS>(L, prow, d));
      const FP qfp0 = row_fp(prow);
      if (cfp.a != qfp0.a || cfp.b != qfp0.b) {  // successor == parent: already in the set
        if constexpr (KSPLIT) {
          kq = true;  // its seen-set key is the orbit key: queued for key_chunk
        } else {
          // seen-set key: the fingerprint, or (SYMMETRY, not split) the orbit key
          FP key = cfp;
          if constexpr (SYM) key = successor_orbit_key<NS>(L, prow, d, afpl[sl]);
          nprobe = !(xflags & XF_NO_PROBE);
          ncf = key;
          nowner = MULTI ? fp_owner(key, box.nshard) : me;
          nidx = (MULTI && nowner != me) ? home_slot(key, box.slog2) : key.a >> (64 - tlog2);
        }
      }
    }
    if constexpr (KSPLIT) {
      const unsigned long long km = __ballot(kq);
      if (kq) kring[(kpos + __popcll(km & lanes_below)) & (RING - 1)] = (uint16_t)(sl << 8 | inst);
      kpos += __popcll(km);
    }
    if (!(xflags & XF_NO_COVER)) {  // generated coverage, aggregated over equal codes
      const int code = en ? cover_code(L, inst, d.sub) : -1;
      const unsigned long long em = __ballot(en);
      if (em) {
        const int c0 = __shfl(code, __builtin_ctzll(em));
        const bool same = en && code == c0;
        const int n0 = __popcll(__ballot(same));
        if (lane == 0) atomicAdd(&cov[c0], (unsigned)n0);
        if (en && !same) atomicAdd(&cov[code], 1u);
      }
    }
    // out-of-model successors: checked, never stored (not in the
    // synthetic microbench, whose random states are no model's)
    int bad = 0;
    if (en && !d.in_model && !(xflags & (XF_DEDUP_ONLY | XF_ALL_SUCCESSORS)))
      bad = check_invariants_v<NS>(L, prow, d.srv, d.rec[0], d.rec[1], d.elec, d.erec[0]);
    if (claim_violation(ctr, bad, lane)) {
      ctr->viol_parent = cur_base + s0 + sl;
      ctr->viol_inst = inst;
      ctr->viol_in_model = 0;
      ctr->viol_child = ~0ull;
    }
  };
  // SYMMETRY: orbit keys, one successor per lane: the ccount continuations
  // first, then kring[kd, kd + kc) -- the full Delta (the probe pass only
  // folded it into a hash), the signatures, and ONE permutation image per
  // pass (`last`: all that are left); a successor with more images left
  // continues in the next key chunk, the others' keys go through the probe
  // pipeline.  Images computed one per pass keep the wave from waiting for
  // its slowest lane: configs[3]'s successors compare 1.15 images on average
  // but the slowest lane of a 64-successor chunk 2.31 (level-15 successors,
  // tools/symstat.cpp; profiles/r04_v4/symstat.txt).
  // Kept apart from the evaluation pass so that neither holds the other's
  // registers.  (Spreading one successor's images over several lanes was
  // built and measured: 2.1-2.4x slower, the recomputed Deltas and the LDS
  // min-reduction cost more than the divergence they remove.)
  auto key_chunk = [&](int kd, int kc, bool last) {
    const int cn = ccount;
    const bool cont = lane < cn;
    const bool active = lane < cn + kc;
    int e = 0, k = 0;
    if (cont) {
      const uint32_t ce = cent[lane];
      e = (int)(ce & 0xffffu);
      k = (int)(ce >> 16);
    } else if (active) {
      e = kring[(kd + lane - cn) & (RING - 1)];
    }
    const int sl = e >> 8, inst = e & 255;
    const uint32_t* prow = rows + sl * W;
    nprobe = false;
    ninfo_new = (uint32_t)sl << 16 | (uint32_t)inst;
    int next = -1;
    FP best{~0ull, ~0ull};
    if (active) {
      const KeyStep ks = key_one<NS, LC, GROUP>(Lrt, prow, sigl + sl, inst, k, last,
                                                cont ? cbest[lane] : FP{~0ull, ~0ull}, afpl[sl]);
      next = ks.next < 0 ? -1 : ks.next;
      best = ks.f;
      if (ks.next == -1) {
        const FP key = ks.f;
        nprobe = !(xflags & XF_NO_PROBE);
        ncf = key;
        nowner = MULTI ? fp_owner(key, box.nshard) : me;
        nidx = (MULTI && nowner != me) ? home_slot(key, box.slog2) : key.a >> (64 - tlog2);
      }
    }
    const unsigned long long cm = __ballot(next >= 0);
    wave_sync();  // (every lane has read its continuation)
    if (next >= 0) {
      const int c = __popcll(cm & lanes_below);
      cent[c] = (uint32_t)e | (uint32_t)next << 16;
      cbest[c] = best;
    }
    ccount = __popcll(cm);
    wave_sync();
  };
  auto issue_probe = [&]() {
    asm volatile("" ::: "memory");
    issue_cas();
    if (nprobe) {
      my_probe++;
      pend = true;
      pf = ncf;
      pinfo = ninfo_new;
      unsigned long long* slotp = &((MULTI && nowner != me) ? sent : table)[nidx];
      // load first: most successors are already in the set, and a plain
      // load is cheaper than an atomic at the memory side; the CAS is
      // only issued (at resolve time) when the home slot reads empty
      if (MULTI && nowner != me && !box.slog2)
        pold = 0ull;  // no sent cache: every remote successor is queued for its owner
      else if (!(xflags & XF_ALL_SUCCESSORS))
        pold = ((xflags & XF_CAS_ONLY) && !(MULTI && nowner != me))
                   ? atomicCAS(slotp, 0ull, ncf.b | 1ull)
                   : __hip_atomic_load(slotp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    nprobe = false;
  };
  // Every probe in flight resolved: the last loads, then the CAS they set up.
  auto drain = [&]() {
    resolve();
    if (async_cas) {
      issue_cas();
      resolve();
    }
  };
  // Append the pairs of instance q (bit q of this window's wave-wide mask)
  // to the ring, Receive grouped by message type (one handler of
  // raft.tla:421-436 per run).
  auto append_instance = [&](int& pos, unsigned long long mask, int wb, int q, const uint32_t* prow_mine, int f) {
    const bool mine = (mask >> q) & 1ull;
    if (f == F_RECEIVE) {
      const uint32_t ty = mine ? slot_type(L, prow_mine, wb + q - L.fam[F_RECEIVE]) : 0u;
#pragma unroll
      for (uint32_t t = 0; t < 4; t++) {
        const bool b = mine && ty == t;
        const unsigned long long m = __ballot(b);
        if (b) ring[(pos + __popcll(m & lanes_below)) & (RING - 1)] = (uint16_t)(lane << 8 | (wb + q));
        pos += __popcll(m);
      }
    } else {
      const unsigned long long m = __ballot(mine);
      if (mine) ring[(pos + __popcll(m & lanes_below)) & (RING - 1)] = (uint16_t)(lane << 8 | (wb + q));
      pos += __popcll(m);
    }
  };

  // Groups are handed out by a device-wide counter (one atomic per group,
  // the next one requested while the current group is processed): a wave
  // that became resident late, or drew heavy groups, simply takes fewer --
  // no static partition, no tail.  (The occupancy API can over-report the
  // resident blocks by one per CU; a static stride would then serialise 1/k
  // of the work behind the rest.)
  // MULTI: a wave takes its next group at the end of the current one, and
  // only while no owner region of the outbox has reached box.stop_at; the
  // groups taken are always a prefix [0, group_next) of the range, so the
  // driver continues the level from there in the next exchange round.  At
  // most two groups per wave run after a region fills (the overflow list's
  // capacity covers them).
  auto take_group = [&]() -> unsigned long long {
    const bool full = MULTI && lane < box.nshard && lane != me &&
                      __hip_atomic_load(&box.out_count[lane], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= box.stop_at;
    unsigned long long g = ~0ull;
    if (!__ballot(full) && lane == 0) g = atomicAdd(&ctr->group_next, 1ull);
    return g;
  };
  if (MULTI && blockIdx.x == 0 && lane == 0 && wave == 0) ctr->group_size = GROUP;
  unsigned long long gnext = 0;
  if (MULTI) gnext = take_group();
  else if (lane == 0) gnext = atomicAdd(&ctr->group_next, 1ull);
  const unsigned long long ngroups = (s_end - s_begin + GROUP - 1) / GROUP;
  for (unsigned long long gi = shfl0_u64(gnext); gi < ngroups; gi = shfl0_u64(gnext)) {
    if (!MULTI && lane == 0) gnext = atomicAdd(&ctr->group_next, 1ull);
    s0 = s_begin + gi * GROUP;
    const int nvalid = (int)min<unsigned long long>((unsigned long long)GROUP, s_end - s0);
    {  // s0 and cur.start are multiples of GROUP: the group's rows are contiguous in the arena
      const uint32_t* src = ring_row(cur, s0, W);
      const int nw = nvalid * W;
      // 16-byte aligned: s0 * W * 4 is a multiple of 128 * W, and the row tile's LDS offset of 16
      if (RTLA_IDX_OK(ctr, ring_idx(cur, s0) + nvalid, cur.cap + 1)) copy_words_lds16(rows, src, nw, lane);
    }
    wave_sync();
    // the next group's number (its atomic returned before the tile copy's wait; MULTI: taken at the group's end)
    unsigned long long gnn = MULTI ? 0ull : shfl0_u64(gnext);
    const bool valid = lane < nvalid;
    const uint32_t* prow_mine = rows + (lane & (GROUP - 1)) * W;
    int nmsg = 0;
    if (valid) {
      pfpl[lane] = fp_add(row_fp(prow_mine), alllogs_delta<NS>(L, prow_mine, pall_mine));
      if (SYM) afpl[lane] = alllogs_fp(L, pall_mine);
      nmsg = row_nmsg(L, prow_mine);
      if constexpr (KSPLIT) {
        uint32_t loc[NS], ms[NS], mr[NS];
        sym_sig_parts<NS>(L, [&](int i, uint32_t* out) { load_rec<NS>(L, prow_mine, i, out); }, nmsg,
                          [&](int q) { return slot_raw(L, prow_mine, q); }, loc, ms, mr);
#pragma unroll
        for (int j = 0; j < NS; j++) {
          sigl[j * GROUP + lane] = loc[j];
          sigl[(NS + j) * GROUP + lane] = ms[j];
          sigl[(2 * NS + j) * GROUP + lane] = mr[j];
        }
      }
    }
    wave_sync();
    STAMP(0);  // group start: work-queue atomic, row tile load, per-state setup
    // With at most one copy of a message allowed (max copies 1), every
    // DuplicateMessage successor (raft.tla:443-445) is out of the model: its
    // one message's count becomes 2 (specs/MC.tla).  It differs from its
    // parent in the bag alone, so the invariants -- which read servers and
    // elections only -- hold on it as on the parent (every expanded state
    // passed them, or the run stopped at its level).  Such successors are
    // counted (generated, per-action coverage: one per message of the bag),
    // not evaluated -- 1/6 of configs[1]'s successors.  The successor walks
    // (XF_ALL_SUCCESSORS) still list them.
    // (kept per lane and reduced once at the end -- configs[1] 180.3 -> 178.5
    // ms; the SYMMETRY kernel keeps the per-group reduction: 292.1 -> 285.8)
    if (dup_counted) {
      if constexpr (SYM) {
        if (valid) my_gen += (unsigned)nmsg;
        if (!(xflags & XF_NO_COVER)) {
          int nd = valid ? nmsg : 0;
          for (int off = 32; off > 0; off >>= 1) nd += __shfl_down(nd, off);
          if (lane == 0 && nd) atomicAdd(&cov[F_DUPLICATE], (unsigned)nd);
        }
      } else if (valid) {
        my_dup += (unsigned)nmsg;
      }
    }
    for (int wb = 0; wb < ((xflags & XF_NO_CHUNKS) ? 0 : ninst); wb += 64) {
      const unsigned long long mask = valid ? cand_mask<NS>(L, prow_mine, nmsg, wb, !dup_counted) : 0ull;
      unsigned long long todo = wave_or_u64(mask);
      int pos = 0, done = 0;
      while (todo || pos > done) {
        // Append the pairs of the next instance(s) until a chunk is ready.  A
        // chunk is cut at a family boundary once it is a third full, so most
        // chunks hold one family and take the specialised path.
        int cfam = -1;
        while (todo && pos - done < 64) {
          const int q = __builtin_ctzll(todo);
          const int f = inst_family(L, wb + q);
          if (f != cfam && pos - done >= 22) break;
          cfam = f;
          todo &= todo - 1;
          append_instance(pos, mask, wb, q, prow_mine, f);
        }
        const int cnt = min(64, pos - done);
        wave_sync();
        STAMP(1);  // pair ring
        eval_chunk(done, cnt);
        STAMP(2);  // successor deltas, fingerprints, coverage, out-of-model invariants
        if (!KSPLIT || (xflags & XF_ALL_SUCCESSORS)) {
          resolve();  // the previous chunk's probes, after this chunk's arithmetic
          STAMP(3);
          issue_probe();
          STAMP(4);  // probe issue
        } else {
          // 64 orbit keys to compute (continuations first): key them (they
          // feed the probe pipeline) until fewer than 64 are queued (the key
          // ring holds RING = 128; an evaluation chunk adds at most 64)
          while (kpos - kdone + ccount >= 64) {
            const int kc = min(kpos - kdone, 64 - ccount);
            key_chunk(kdone, kc, kc == 0);
            kdone += kc;
            STAMP(7);  // SYMMETRY: orbit keys
            resolve();
            STAMP(3);
            issue_probe();
            STAMP(4);  // probe issue
          }
        }
        if (tail - head > NEWFLUSH) {  // rare (early levels): drain the probes, build the rows so far
          drain();
          build_all();
          STAMP(5);
        }
        done += cnt;
      }
    }
    // Group end: the last probes and every pending row (their parents are
    // this group's rows, which the next group overwrites).
    // Touch every 128-byte line of the next group's rows now, so that its
    // tile load after this drain hits the caches.  Relaxed atomic loads: the
    // compiler issues them here (it does not sink an atomic) and tracks
    // their destination registers like any load (its vmcnt waits count
    // them); the values are consumed only at the drain's end, so nothing
    // waits for them before.  (an asm-issued load's register was
    // invisible to the compiler.)
    uint32_t pfa = 0, pfb = 0;
    if (MULTI) {
      gnext = take_group();
      gnn = shfl0_u64(gnext);
    }
    while (KSPLIT && kpos - kdone + ccount > 0) {  // the group's last orbit keys (they key this group's rows)
      const int kc = min(kpos - kdone, 64 - ccount);
      key_chunk(kdone, kc, kc == 0 || kpos - kdone + ccount <= 64);  // (the last chunk: every image left)
      kdone += kc;
      STAMP(7);
      resolve();
      issue_probe();
    }
    if (gnn < ngroups) {
      const unsigned long long sn = s_begin + gnn * GROUP;
      const int lines = ((int)min<unsigned long long>((unsigned long long)GROUP, s_end - sn) * W + 31) / 32;
      const uint32_t* pa = ring_row(cur, sn, W) + 32 * min(lane, lines - 1);
      const uint32_t* pb = ring_row(cur, sn, W) + 32 * min(lane + 64, lines - 1);
      pfa = __hip_atomic_load(pa, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      pfb = __hip_atomic_load(pb, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    drain();
    if constexpr (!KSPLIT) STAMP(7);  // (non-symmetric builds: slot 7 = the group-end probe drain alone)
    build_all();
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    asm volatile("" ::"v"(pfa), "v"(pfb));
    wave_sync();
    STAMP(6);  // group-end drain
  }
  if (MULTI) {
    for (int o = 0; o < box.nshard; o++) {
      const unsigned long long b = obox[o], used = obox[SHARD_MAX + o];
      if (b != ~0ull) outbox_holes(box, o, b + used, b + OBOX_CHUNK, lane);
    }
  }
  for (int off = 32; off > 0; off >>= 1) {
    my_gen += __shfl_down(my_gen, off);
    my_probe += __shfl_down(my_probe, off);
    my_dup += __shfl_down(my_dup, off);
  }
  my_gen += my_dup;
  if (lane == 0 && my_dup && !(xflags & XF_NO_COVER)) atomicAdd(&cov[F_DUPLICATE], my_dup);
  if (lane == 0 && my_gen) atomicAdd(&ctr->generated, (unsigned long long)my_gen);
  if (lane == 0 && my_probe) atomicAdd(&ctr->probes, (unsigned long long)my_probe);
  if (lane == 0 && dedup_new) atomicAdd(&ctr->next_count, dedup_new);
#ifdef RTLA_COUNT_CAS
  for (int off = 32; off > 0; off >>= 1) my_cas += __shfl_down(my_cas, off);
  if (lane == 0 && my_cas) atomicAdd(&ctr->cas, (unsigned long long)my_cas);
#endif
  STAMP(7);  // (kernel end: negligible)
  RTLA_STAMP_FLUSH(ctr, lane)
  __syncthreads();
  for (int k = threadIdx.x; k < 2 * COVER_CODES; k += blockDim.x)
    if (cov[k]) atomicAdd(&ctr->cover[k], (unsigned long long)cov[k]);
}

namespace rtla {

#define RTLA_DISPATCH_N(L, KERNEL, ...)                        \
  switch ((L).N) {                                             \
    case 1: hipLaunchKernelGGL(KERNEL<1>, __VA_ARGS__); break; \
    case 2: hipLaunchKernelGGL(KERNEL<2>, __VA_ARGS__); break; \
    case 3: hipLaunchKernelGGL(KERNEL<3>, __VA_ARGS__); break; \
    case 4: hipLaunchKernelGGL(KERNEL<4>, __VA_ARGS__); break; \
    default: hipLaunchKernelGGL(KERNEL<5>, __VA_ARGS__); break; \
  }

static inline unsigned grid_x(uint64_t n, int per_block) {
  return (unsigned)std::max<uint64_t>(1, std::min<uint64_t>((n + per_block - 1) / per_block, 4096));
}

// States per wave-group of k_expand_compact: 64, or 32 when 64 rows would
// make the per-wave LDS tile so large that fewer than ~11 waves fit a CU.
#ifndef RTLA_GROUP64_LDS
#define RTLA_GROUP64_LDS (16 * 1024)
#endif
// SYMMETRY: always 32 (one instantiation per N; the orbit-key arithmetic,
// not the tile, bounds that kernel).
constexpr int compact_group(const Layout& L) {
  if (L.sym) return 32;
  return compact_lds_words(L.W, L.all_words, 64, false, true) * sizeof(uint32_t) <= RTLA_GROUP64_LDS ? 64 : 32;
}
// The compiled-in configurations may also run 16-state groups: wide rows
// (configs[2]: 516 B, configs[3]: 628 B) would otherwise leave the 32-row
// tile, not the registers, bounding the waves per CU (8 and 7 instead of
// 12 and 8; bench's occupancy sweep: throughput grows with resident waves).
#ifndef RTLA_GROUP32_LDS
#define RTLA_GROUP32_LDS (19 * 1024)
#endif
#ifndef RTLA_SYM_GROUP
#define RTLA_SYM_GROUP 16
#endif
constexpr int spec_group(const Layout& L) {
  if (L.sym) return RTLA_SYM_GROUP;  // configs[3]: 16 waves/CU at 128 VGPRs need the smaller tile (311.5 vs 322 ms)
  const int g = compact_group(L);
  return g == 32 && compact_lds_words(L.W, L.all_words, 32, L.sym, true) * sizeof(uint32_t) > RTLA_GROUP32_LDS ? 16 : g;
}

static inline int device_cus() {
  static int cus = 0;
  if (!cus) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
      cus = 256;
  }
  return cus;
}


// Configurations whose layout is compiled into k_expand_compact (the BASELINE
// workloads bench.py runs); any other configuration runs the same kernel on
// its run-time layout.
namespace specs {
constexpr Layout CFG2 = layout_of(3, 2, 3, 2, 1, 0, 18, 6, INV_ELECTION_SAFETY | INV_LOG_MATCHING);  // configs[1]
constexpr Layout CFG1 = layout_of(3, 1, 2, 1, 1, 0, 24, 3, INV_NO_TWO_LEADERS);                     // configs[0]
constexpr Layout EXHAUST = layout_of(3, 2, 2, 2, 1, 2, 3, 3, INV_ELECTION_SAFETY | INV_LOG_MATCHING);
constexpr Layout CFG3 = layout_of(3, 2, 4, 3, 2, 0, 20, 9, 0);                                      // configs[2]
constexpr Layout SYNTH = layout_of(3, 2, 4, 3, 2, 0, 12, 9, INV_ELECTION_SAFETY | INV_LOG_MATCHING);  // configs[4]
constexpr Layout symmetric(Layout l) {
  l.sym = 1;
  return l;
}
constexpr Layout CFG4 = symmetric(layout_of(5, 1, 3, 2, 1, 0, 20, 10, 0));  // configs[3], SYMMETRY
static_assert(CFG2.N == 3 && CFG1.N == 3 && EXHAUST.N == 3 && CFG3.N == 3 && SYNTH.N == 3 && CFG4.N == 5,
              "compiled-in layouts must be valid");
}  // namespace specs

template <int NS, int GROUP, Layout LC, bool SYM = false>
static hipError_t launch_compact(const CompactArgs& a) {
  const Layout& L = a.L;
  const bool multi = a.multi;
  const int wpb = a.wpb, xflags = a.xflags;
  const uint64_t s_begin = a.s_begin, s_end = a.s_end;
  DevCounters* ctr = a.ctr;
  hipStream_t st = a.st;
  auto kfn = multi ? k_expand_compact<NS, true, GROUP, LC, SYM> : k_expand_compact<NS, false, GROUP, LC, SYM>;
  const uint64_t groups = (s_end - s_begin + GROUP - 1) / GROUP;
  uint64_t blocks = std::min<uint64_t>((groups + wpb - 1) / wpb, 1u << 20);
  const size_t lds = (size_t)wpb * compact_lds_words(L.W, L.all_words, GROUP, SYM, multi) * sizeof(uint32_t);
  if (!(xflags & XF_NO_PERSIST) || a.query) {  // persistent waves: exactly the resident capacity, looping over groups
    static int per_cu[2][2];  // per instantiation: [multi][one-wave blocks]
    int& pc = per_cu[multi][wpb == 1];
    if (!pc) {
      if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&pc, kfn, 64 * wpb, lds) != hipSuccess || pc < 1)
        pc = 16 / wpb;
      if (const char* e = getenv("RTLA_BLOCKS_PER_CU"))  // occupancy experiments
        if (atoi(e) > 0) pc = std::min(pc, atoi(e));
    }
    blocks = std::min<uint64_t>(blocks, (uint64_t)device_cus() * pc);
    if (a.query) {  // level_kernel_shape: the waves resident at once (any launch mode) and the group size
      a.query[0] = device_cus() * pc * wpb;
      a.query[1] = GROUP;
      return hipSuccess;
    }
  }
  {
    hipError_t e = hipMemsetAsync(&ctr->group_next, 0, sizeof(ctr->group_next), st);
    if (e != hipSuccess) return e;
  }
  hipLaunchKernelGGL(kfn, dim3((unsigned)blocks), dim3(64 * wpb), lds, st, L, a.cur, (unsigned long long)s_begin,
                     (unsigned long long)s_end, (unsigned long long)a.cur_base, a.next,
                     (unsigned long long*)a.parents, (unsigned long long)a.next_base, (unsigned long long)a.next_cap,
                     (unsigned long long*)a.table, (unsigned long long*)a.sent, a.tlog2, ctr, a.box, xflags);
  return hipGetLastError();
}


}  // namespace rtla
