// rtla_kernels.hip -- gfx950 kernels of the BFS hot path.
//
// One BFS level = one launch of k_expand over the current frontier:
//   * one wavefront per frontier state: the 64 lanes copy the packed row into
//     LDS (coalesced); lanes 0..N-1 hash the parent's server records and lane
//     N derives the per-parent allLogs' (raft.tla:465), all into LDS;
//   * each lane evaluates one action instance of Next (raft.tla:454-463) as a
//     Delta against the LDS row (rtla_model.h): every lane reads the same
//     parent words (LDS broadcast, no bank conflicts) and the Delta stays in
//     VGPRs (the model is instantiated per server count, NS);
//   * the successor's 128-bit fingerprint is the parent's plus the Delta's
//     component change (no full re-hash);
//   * in-model successors probe the open-addressing fingerprint set in HBM
//     with one 8-byte CAS per probe (home slot from fp.a, key fp.b | 1):
//     one memory round trip whether the state is new or seen;
//   * new successors are compacted by ballot + popcount prefix, built in a
//     16-row LDS staging tile and written to the next frontier as contiguous,
//     coalesced ranges;
//   * invariants are checked on every new and every out-of-model successor.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <type_traits>

#include "rtla_device.h"

#include "rtla_model.h"
#include "rtla_synth.h"

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
// lossy (the MULTI sent cache, a dedup hint only): a long probe chain answers
// "not sent yet" -- the record is shipped and its owner deduplicates -- and
// never raises FLAG_FPSET_FULL.
__device__ __forceinline__ bool fpset_resolve_loaded(unsigned long long* table, int log2, unsigned long long key,
                                                     unsigned long long idx, unsigned long long seen,
                                                     DevCounters* ctr, bool lossy = false) {
  const unsigned long long mask = (1ull << log2) - 1ull;
  for (int probe = 1;; probe++) {
    if (seen == key) return false;
    if (seen == 0ull) {
      seen = atomicCAS(&table[idx], 0ull, key);
      if (seen == 0ull) return true;
      if (seen == key) return false;
    }
    if (lossy && probe >= 64) return true;
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

// SYMMETRY: orbit key of the successor parent + d (allLogs' fingerprint
// afp), without materialising it (rtla_model.h sym_key).
template <int NS, class P>
__device__ __forceinline__ FP successor_orbit_key(const Layout& L, P prow, const DeltaT<NS>& d, FP afp) {
  constexpr int EW = 2 + NS;
  const int ne0 = row_nelec(L, prow);
  return sym_key<NS>(
      [&](int i, uint32_t* out) {
        load_rec<NS>(L, prow, i, out);
        if (i == d.srv) {
#pragma unroll
          for (int w = 0; w < 3 + NS; w++) out[w] = d.rec[w];
        }
      },
      d.nmsg, [&](int q) { return bag_get(L, prow, d, q); }, ne0 + (d.elec ? 1 : 0),
      [&](int e, uint32_t* out) {
        if (e < ne0) {
#pragma unroll
          for (int w = 0; w < EW; w++) out[w] = prow[L.off_elec + e * EW + w];
        } else {
#pragma unroll
          for (int w = 0; w < EW; w++) out[w] = d.erec[w];
        }
      },
      afp);
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

template <int NS>
__global__ void __launch_bounds__(256)
k_expand(Layout L, Ring cur, unsigned long long s_begin, unsigned long long s_end,
         unsigned long long cur_base, Ring next, unsigned long long* __restrict__ parents,
         unsigned long long next_base, unsigned long long next_cap, unsigned long long* table, int tlog2,
         DevCounters* ctr, ShardBox box) {
  extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
  __shared__ unsigned int cov[2 * COVER_CODES];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int wpb = blockDim.x >> 6;
  const int W = L.W;
  uint32_t* prow = lds + wave * wave_lds_words(W);
  uint32_t* pall = prow + even_words(W);
  FP* hsrv = reinterpret_cast<FP*>(pall + 32);
  uint32_t* stage = pall + 32 + 4 * NMAX;
  for (int k = threadIdx.x; k < 2 * COVER_CODES; k += blockDim.x) cov[k] = 0;
  __syncthreads();

  unsigned long long my_gen = 0, my_probe = 0;
  const int fixed = L.fam[F_RECEIVE];
  for (unsigned long long s = s_begin + (unsigned long long)blockIdx.x * wpb + wave; s < s_end;
       s += (unsigned long long)gridDim.x * wpb) {
    const FP pfp = load_parent<NS>(L, ring_row(cur, s, W), prow, pall, hsrv, lane);
    // SYMMETRY: allLogs' is the same for every successor (raft.tla:465)
    const FP afp = L.sym ? alllogs_fp(L, pall) : FP{0, 0};
    const int nmsg = row_nmsg(L, prow);
    const int ncand = fixed + 3 * nmsg;
    for (int base = 0; base < ncand; base += 64) {
      const int q = base + lane;
      DeltaT<NS> d;
      d.enabled = 0;
      int inst = 0;
      if (q < ncand) {
        inst = candidate_inst(L, q, nmsg);
        compute_delta<NS>(L, prow, inst, d);
      }
      bool en = d.enabled != 0;
      if (en && d.err) {
        set_flag(ctr, d.err == 1 ? FLAG_SPEC_ERROR : FLAG_ROW_OVERFLOW);
        en = false;
      }
      my_gen += en ? 1 : 0;
      bool isnew = false;
      FP cfp{0, 0};
      if (en && d.in_model) {
        cfp = fp_add(pfp, delta_fp<NS>(L, prow, d, d.srv >= 0 ? &hsrv[d.srv] : nullptr));
        // seen-set key: the state's own fingerprint, or under SYMMETRY its
        // orbit key (least fingerprint over the server permutations)
        const FP key = L.sym ? successor_orbit_key<NS>(L, prow, d, afp) : cfp;
        const int owner = fp_owner(key, box.nshard);
        if (owner == box.me) {
          my_probe++;
          int r = fpset_insert(table, tlog2, key);
          if (r < 0) set_flag(ctr, FLAG_FPSET_FULL);
          isnew = r == 1;
        } else {
          // Another shard owns this fingerprint: queue (fp, parent, instance);
          // the owner answers new/seen and this shard ships it the winner.
          unsigned long long slot = atomicAdd(&box.out_count[owner], 1ull);
          if (slot < box.cap) {
            unsigned long long k = (unsigned long long)owner * box.cap + slot;
            box.send_fp[2 * k] = key.a;
            box.send_fp[2 * k + 1] = key.b;
            box.send_ref[k] = s << 16 | (unsigned long long)inst;
          } else {
            set_flag(ctr, FLAG_OUTBOX_FULL);
          }
        }
      }
      if (en) {
        int code = cover_code(L, inst, d.sub);
        atomicAdd(&cov[code], 1u);
        if (isnew) atomicAdd(&cov[COVER_CODES + code], 1u);
      }
      const unsigned long long m = __ballot(isnew);
      const int cnt = __popcll(m);
      unsigned long long obase = 0;
      int rank = 0;
      if (cnt) {
        rank = __popcll(m & ((1ull << lane) - 1ull));
        if (lane == 0) obase = atomicAdd(&ctr->next_count, (unsigned long long)cnt);
        obase = shfl0_u64(obase);
        if (obase + cnt > next_cap) {
          if (lane == 0) set_flag(ctr, FLAG_FRONTIER_FULL);
        } else {
          // stage and write out STAGE_ROWS new rows at a time
          for (int b = 0; b < cnt; b += STAGE_ROWS) {
            if (isnew && rank >= b && rank < b + STAGE_ROWS)
              materialize<NS>(L, prow, d, pall, cfp, stage + (rank - b) * W);
            wave_sync();
            store_rows_ring(next, obase + b, min(STAGE_ROWS, cnt - b), W, stage, lane);
            wave_sync();
          }
          if (isnew)
            parents[next_base + obase + rank] =
                (unsigned long long)box.me << 56 | (cur_base + s) << 16 | (unsigned long long)inst;
        }
      }
      if (en && (isnew || !d.in_model)) {
        int bad = check_invariants_v<NS>(L, prow, d.srv, d.rec[0], d.rec[1], d.elec, d.erec[0]);
        if (bad && __hip_atomic_load(&ctr->viol_mask, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0 &&
            atomicCAS(&ctr->viol_mask, 0, bad) == 0) {
          ctr->viol_parent = cur_base + s;
          ctr->viol_inst = inst;
          ctr->viol_in_model = d.in_model;
          ctr->viol_child = isnew ? next_base + obase + rank : ~0ull;
        }
      }
    }
  }
  for (int off = 32; off > 0; off >>= 1) {
    my_gen += __shfl_down(my_gen, off);
    my_probe += __shfl_down(my_probe, off);
  }
  if (lane == 0 && my_gen) atomicAdd(&ctr->generated, my_gen);
  if (lane == 0 && my_probe) atomicAdd(&ctr->probes, my_probe);
  __syncthreads();
  for (int k = threadIdx.x; k < 2 * COVER_CODES; k += blockDim.x)
    if (cov[k]) atomicAdd(&ctr->cover[k], (unsigned long long)cov[k]);
}

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
constexpr int NEWCAP = 256; // new-state list (u16: state lane << 8 | instance)

constexpr int OBOX_CHUNK = 256;  // outbox slots a wave reserves per owner at a time (MULTI)

// Per-wave LDS of k_expand_compact (16-byte aligned pieces first):
// per-state fingerprint with allLogs' applied (GROUP FPs) | SYMMETRY: the
// fingerprint of each state's allLogs' (GROUP FPs) | per-owner (base, used)
// of the open outbox chunk | pending new states (NEWCAP u16 entries) |
// GROUP rows | allLogs' words of each state | pair ring.
// (The outbox state exists only in the MULTI kernels: one shard's tile then
// stays small enough for 12 one-wave blocks per CU on configs[1]'s 372-byte rows.)
__host__ __device__ constexpr int compact_lds_words(int W, int AW, int GROUP, bool sym, bool multi) {
  return (4 * GROUP * (sym ? 2 : 1) + (multi ? 4 * SHARD_MAX : 0) + NEWCAP / 2 + GROUP * W + GROUP * AW + RING / 2 +
          3) & ~3;
}

// bits << off into a 64-bit window mask (off may be negative or >= 64)
__device__ __forceinline__ unsigned long long win_bits(unsigned long long bits, int off) {
  if (off >= 64 || off <= -64) return 0ull;
  return off >= 0 ? bits << off : bits >> (-off);
}

// Instances [wb, wb+64) whose enabling guard holds in `row`.  A superset is
// safe (compute_delta re-checks every guard); a subset would lose states.
template <int NS>
__device__ __forceinline__ unsigned long long cand_mask(const Layout& L, const uint32_t* row, int nmsg, int wb) {
  constexpr int N = NS;
  const int SW = 3 + N;
  unsigned long long rv = 0, bl = 0, ldr = 0, tmo = 0;
#pragma unroll
  for (int i = 0; i < N; i++) {
    const uint32_t w0 = row[L.off_srv + i * SW];
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
  m |= win_bits(bag, L.fam[F_DUPLICATE] - wb);
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

__device__ __forceinline__ unsigned long long shfl_u64(unsigned long long v, int src) {
  const uint32_t lo = (uint32_t)__shfl((int)(uint32_t)v, src);
  const uint32_t hi = (uint32_t)__shfl((int)(uint32_t)(v >> 32), src);
  return (unsigned long long)lo | (unsigned long long)hi << 32;
}

}  // namespace

#ifndef RTLA_COMPACT_WAVES_PER_EU
#define RTLA_COMPACT_WAVES_PER_EU 3  // 166 VGPRs for N = 3 without spills (the default allocation took 170 -> 2 waves)
#endif
#ifndef RTLA_SYM_WAVES_PER_EU
#define RTLA_SYM_WAVES_PER_EU 2      // SYMMETRY: the full Delta and the orbit-key loop stay in VGPRs
#endif
// The layout the kernel runs on: the run-time argument, or (LC.N != 0) the
// configuration compiled in as a template parameter, whose fields the
// compiler then folds into every offset, bound and loop of the model code.
template <Layout LC>
__device__ __forceinline__ const Layout& pick_layout(const Layout& rt) {
  if constexpr (LC.N == 0) return rt;
  else return LC;
}

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
template <int NS, bool MULTI, int GROUP, Layout LC, bool SYM>
__global__ void __launch_bounds__(256)
__attribute__((amdgpu_waves_per_eu(SYM ? RTLA_SYM_WAVES_PER_EU : RTLA_COMPACT_WAVES_PER_EU)))
k_expand_compact(Layout Lrt, Ring cur, unsigned long long s_begin, unsigned long long s_end,
                 unsigned long long cur_base, Ring next, unsigned long long* __restrict__ parents,
                 unsigned long long next_base, unsigned long long next_cap, unsigned long long* table,
                 unsigned long long* sent, int tlog2, DevCounters* ctr, ShardBox box, int xflags) {
  const Layout& L = pick_layout<LC>(Lrt);
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
  const int ninst = L.fam[F_COUNT];
  const unsigned long long lanes_below = (1ull << lane) - 1ull;
  RTLA_STAMP_DECL
  // pending probe (issued by the previous chunk).  MULTI: a successor owned
  // by another shard probes this shard's SENT cache instead of the set: the
  // first time this shard meets it, its (fingerprint, parent) record goes to
  // the owner's outbox; later copies are dropped (the owner already has it).
  bool pend = false;
  unsigned long long pold = 0;
  FP pf{0, 0};       // its fingerprint (home slot and owner derive from it)
  uint32_t pinfo = 0;  // its state lane << 16 | action instance
  // Single shard: a probe whose home-slot load did not show its key issues
  // ONE CAS -- at the home slot if it read empty, else at the next slot
  // (linear probing; slots only ever go 0 -> key) -- together with the next
  // chunk's loads, and that CAS is resolved a chunk later: neither the
  // insert nor the first collision step waits for a round trip.
  const bool async_cas = !MULTI && !(xflags & XF_CAS_ONLY);
  bool cpend = false;    // CAS set up by resolve(), issued by issue_cas()
  bool cflight = false;  // CAS in flight (result in cold)
  unsigned long long cold = 0, ckey = 0, cidx = 0;
  uint32_t cinfo = 0;
  // New states found so far whose rows are not built yet: newl[head, tail)
  // (mod NEWCAP) holds (state lane, instance); their parents are rows of the
  // current group (uniform counters).  A reservation of next-level slots for
  // the oldest 64 is requested one chunk before they are built (res_ob: the
  // atomic's result in lane 0, read only then).
  int head = 0, tail = 0;
  bool have_res = false;
  unsigned long long res_ob = 0;
  unsigned long long dedup_new = 0;  // XF_DEDUP_ONLY: new fingerprints (uniform)
  unsigned long long s0 = 0;  // first state of the current group

  // One atomic reserves nb next-level slots.  Slots past next_cap are
  // dropped and flagged (the level is then reported incomplete).
  auto reserve_issue = [&](int nb) {  // the atomic, not waited for
    unsigned long long ob = 0;
    if (lane == 0) ob = atomicAdd(&ctr->next_count, (unsigned long long)nb);
    return ob;
  };
  auto reserve_take = [&](unsigned long long ob, int nb) {
    ob = shfl0_u64(ob);
    if (ob + nb > next_cap && lane == 0) set_flag(ctr, FLAG_FRONTIER_FULL);
    return ob;
  };
  // Build the rows of the nb oldest pending new states into slots obase ..
  // obase + nb - 1 of the next level, one state per lane:
  //  (1) the wave copies each parent row (LDS) to its child's slot with
  //      coalesced stores;
  //  (2) each lane re-derives its successor's full Delta (compute_delta with
  //      slot bookkeeping; the probe pass only folded it into a hash), its
  //      fingerprint, invariants and distinct coverage -- arithmetic that
  //      overlaps the stores and the chunk's probe loads in flight;
  //  (3) after the stores completed, each lane stores the words in which its
  //      child differs from the parent (child_patches, rtla_model.h).
  // This replaces a separate row-building kernel: no parent-record read, no
  // parent-row gather, no second launch.
  auto build_rows = [&](unsigned long long obase, int nb) {
    const bool act = lane < nb;
    const int e = act ? newl[(head + lane) & (NEWCAP - 1)] : 0;
    const int sl = e >> 8, inst = e & 255;
    const int nrows = obase >= next_cap ? 0 : (int)min<unsigned long long>((unsigned long long)nb, next_cap - obase);
    const bool rows_on = !(xflags & XF_NO_MATERIALIZE) && RTLA_IDX_OK(ctr, obase + nrows, ctr->cap_next + 1);
    const unsigned long long p0 = ring_idx(next, obase);
    const int n1 = (int)min<unsigned long long>(next.cap - p0, (unsigned long long)nrows) * W;  // words before the wrap
    uint32_t* d1 = next.base + p0 * (unsigned long long)W;
    if (rows_on) {  // (1)
      const int nwords = nrows * W;
      int r = 0, w = lane;
      while (w >= W) { w -= W; r++; }
      for (int i0 = 0; i0 < nwords; i0 += 64) {
        const int sr = __shfl(sl, r & 63);
        const int i = i0 + lane;
        if (i < nwords) {
          const uint32_t v = rows[sr * W + w];
          if (i < n1) d1[i] = v;
          else next.base[i - n1] = v;
        }
        w += 64;
        while (w >= W) { w -= W; r++; }
      }
    }
    DeltaT<NS> d;  // (2)
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
    if (claim_violation(ctr, bad, lane)) {
      ctr->viol_parent = cur_base + s0 + sl;
      ctr->viol_inst = inst;
      ctr->viol_in_model = 1;
      ctr->viol_child = lane < nrows ? next_base + obase + lane : ~0ull;
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
    if (rows_on) {  // (3): the copies must land first (same words, other lanes)
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      if (lane < nrows) {
        const StridedWords<GROUP> pall_p{pall + sl};
        const int off = lane * W;
        child_patches<NS>(L, rows + sl * W, d, pall_p, cfp, [&](int w, uint32_t v) {
          const int i = off + w;
          if (i < n1) d1[i] = v;
          else next.base[i - n1] = v;
        });
      }
    }
    if (lane < nrows && RTLA_IDX_OK(ctr, next_base + obase + lane, ctr->cap_parents))
      parents[next_base + obase + lane] =
          (unsigned long long)me << 56 | (cur_base + s0 + sl) << 16 | (unsigned long long)inst;
    head += nb;
  };
  auto issue_cas = [&]() {
    if (cpend) cold = atomicCAS(&table[cidx], 0ull, ckey);
    cflight = cpend;
    cpend = false;
  };
  auto resolve = [&]() {
    bool isnew = false;
    uint32_t ninfo = pinfo;  // the state isnew refers to
    const int powner = MULTI ? fp_owner(pf, box.nshard) : me;
    const unsigned long long prec =
        (unsigned long long)me << 56 | (cur_base + s0 + (pinfo >> 16)) << 16 | (unsigned long long)(pinfo & 0xffffu);
    if (async_cas) {
      if (cflight) {  // the CAS issued one chunk ago
        if (cold == 0ull) isnew = true;
        else if (cold != ckey) isnew = fpset_resolve(table, tlog2, ckey, cidx, cold, ctr);  // rare: keep probing
      }
      ninfo = cinfo;
      cflight = false;
      if (pend) {  // this chunk's load -> seen, or a CAS for the next issue
        const unsigned long long key = pf.b | 1ull, idx = pf.a >> (64 - tlog2);
        if (pold != key) {
          cidx = pold == 0ull ? idx : ((idx + 1ull) & ((1ull << tlog2) - 1ull));
          ckey = key;
          cinfo = pinfo;
          cpend = true;
        }
      }
    } else if (pend) {
      const bool to_sent = MULTI && powner != me;
      unsigned long long* t = to_sent ? sent : table;
      const unsigned long long pidx = pf.a >> (64 - tlog2);
      isnew = (xflags & XF_CAS_ONLY) ? fpset_resolve(t, tlog2, pf.b | 1ull, pidx, pold, ctr)
                                     : fpset_resolve_loaded(t, tlog2, pf.b | 1ull, pidx, pold, ctr, to_sent);
    }
    if (MULTI) {  // records for other owners: one outbox reservation per (wave, owner)
      const bool rem = isnew && powner != me;
      isnew = isnew && powner == me;
      unsigned long long om = wave_or_u64(rem ? 1ull << powner : 0ull);
      while (om) {
        const int o = __builtin_ctzll(om);
        om &= om - 1;
        const unsigned long long m = __ballot(rem && powner == o);
        const int cnt = __popcll(m);
        unsigned long long b = obox[o], used = obox[SHARD_MAX + o];
        if (used + cnt > OBOX_CHUNK) {  // close the open chunk (holes = zero records), reserve the next
          if (b != ~0ull) outbox_holes(box, o, b + used, b + OBOX_CHUNK, lane);
          unsigned long long nb = 0;
          if (lane == 0) nb = atomicAdd(&box.out_count[o], (unsigned long long)OBOX_CHUNK);
          b = shfl0_u64(nb);
          used = 0;
        }
        if (rem && powner == o) {
          const unsigned long long slot = b + used + __popcll(m & lanes_below);
          if (slot < box.cap) {
            const unsigned long long k = (unsigned long long)o * box.cap + slot;
            box.send_fp[2 * k] = pf.a;
            box.send_fp[2 * k + 1] = pf.b;
            box.send_ref[k] = (((prec >> 16) & ((1ull << 40) - 1ull)) - cur_base) << 16 | (prec & 0xffffull);
          } else {
            set_flag(ctr, FLAG_OUTBOX_FULL);
          }
        }
        wave_sync();
        if (lane == 0) {
          obox[o] = b;
          obox[SHARD_MAX + o] = used + cnt;
        }
        wave_sync();
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
    std::conditional_t<SYM, DeltaT<NS>, DeltaFpT<NS>> d;
    d.enabled = 0;
    if (!(xflags & XF_NO_DELTA)) {
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
    }
    bool en = d.enabled != 0;
    if (en && d.err) {
      set_flag(ctr, d.err == 1 ? FLAG_SPEC_ERROR : FLAG_ROW_OVERFLOW);
      en = false;
    }
    my_gen += en ? 1u : 0u;
    nprobe = false;
    nidx = 0;
    ncf = FP{0, 0};
    nowner = me;
    ninfo_new = (uint32_t)sl << 16 | (uint32_t)inst;
    if (en && d.in_model) {
      FP cfp;
      if constexpr (SYM) cfp = fp_add(qfp, delta_fp<NS>(L, prow, d));
      else
        cfp = (xflags & XF_NO_HASH) ? FP{qfp.a + d.rec[0] + (uint64_t)d.fmsg.a, qfp.b + d.rec[1]}
                                    : fp_add(qfp, delta_fp<NS>(L, prow, d));
      const FP qfp0 = row_fp(prow);
      if (cfp.a != qfp0.a || cfp.b != qfp0.b) {  // successor == parent: already in the set
        // seen-set key: the fingerprint, or under SYMMETRY the orbit key
        FP key = cfp;
        if constexpr (SYM) key = successor_orbit_key<NS>(L, prow, d, afpl[sl]);
        nprobe = !(xflags & XF_NO_PROBE);
        ncf = key;
        nidx = key.a >> (64 - tlog2);
        nowner = MULTI ? fp_owner(key, box.nshard) : me;
      }
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
    if (en && !d.in_model && !(xflags & XF_DEDUP_ONLY))
      bad = check_invariants_v<NS>(L, prow, d.srv, d.rec[0], d.rec[1], d.elec, d.erec[0]);
    if (claim_violation(ctr, bad, lane)) {
      ctr->viol_parent = cur_base + s0 + sl;
      ctr->viol_inst = inst;
      ctr->viol_in_model = 0;
      ctr->viol_child = ~0ull;
    }
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
      pold = (xflags & XF_CAS_ONLY) ? atomicCAS(slotp, 0ull, ncf.b | 1ull)
                                    : __hip_atomic_load(slotp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    nprobe = false;
  };
  // Append the pairs of instance q (bit q of this window's wave-wide mask)
  // to the ring, Receive grouped by message type (one handler of
  // raft.tla:421-436 per run).
  auto append_instance = [&](int& pos, unsigned long long mask, int wb, int q, const uint32_t* prow_mine, int f) {
    const bool mine = (mask >> q) & 1ull;
    if (f == F_RECEIVE) {
      const uint32_t ty = mine ? m_type(bag_slot(L, prow_mine, wb + q - L.fam[F_RECEIVE])) : 0u;
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
  unsigned long long gnext = 0;
  if (lane == 0) gnext = atomicAdd(&ctr->group_next, 1ull);
  const unsigned long long ngroups = (s_end - s_begin + GROUP - 1) / GROUP;
  for (unsigned long long gi = shfl0_u64(gnext); gi < ngroups; gi = shfl0_u64(gnext)) {
    if (lane == 0) gnext = atomicAdd(&ctr->group_next, 1ull);
    s0 = s_begin + gi * GROUP;
    const int nvalid = (int)min<unsigned long long>((unsigned long long)GROUP, s_end - s0);
    {  // s0 and cur.start are multiples of GROUP: the group's rows are contiguous in the arena
      const uint32_t* src = ring_row(cur, s0, W);
      const int nw = nvalid * W;
      // 16-byte aligned: s0 * W * 4 is a multiple of 128 * W, and the row tile's LDS offset of 16
      if (RTLA_IDX_OK(ctr, ring_idx(cur, s0) + nvalid, cur.cap + 1)) copy_words_lds16(rows, src, nw, lane);
    }
    wave_sync();
    // the next group's number (its atomic returned before the tile copy's wait)
    const unsigned long long gnn = shfl0_u64(gnext);
    const bool valid = lane < nvalid;
    const uint32_t* prow_mine = rows + (lane & (GROUP - 1)) * W;
    int nmsg = 0;
    if (valid) {
      pfpl[lane] = fp_add(row_fp(prow_mine), alllogs_delta<NS>(L, prow_mine, pall_mine));
      if (SYM) afpl[lane] = alllogs_fp(L, pall_mine);
      nmsg = row_nmsg(L, prow_mine);
    }
    wave_sync();
    STAMP(0);  // group start: work-queue atomic, row tile load, per-state setup
    for (int wb = 0; wb < ((xflags & XF_NO_CHUNKS) ? 0 : ninst); wb += 64) {
      const unsigned long long mask = valid ? cand_mask<NS>(L, prow_mine, nmsg, wb) : 0ull;
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
        resolve();  // the previous chunk's probes, after this chunk's arithmetic
        STAMP(3);
        // Rows of the oldest 64 pending new states, into the slots reserved
        // one chunk ago -- before this chunk's probes are issued, so the
        // row stores' completion wait (build_rows step 3) never waits for
        // them.  Then reserve for the next 64 if they are pending already.
        if (have_res) {
          build_rows(reserve_take(res_ob, 64), 64);
          have_res = false;
        }
        STAMP(5);
        if (tail - head >= 64) {
          res_ob = reserve_issue(64);
          have_res = true;
        }
        issue_probe();
        STAMP(4);  // slot reservation, probe issue
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
    if (gnn < ngroups) {
      const unsigned long long sn = s_begin + gnn * GROUP;
      const int lines = ((int)min<unsigned long long>((unsigned long long)GROUP, s_end - sn) * W + 31) / 32;
      const uint32_t* pa = ring_row(cur, sn, W) + 32 * min(lane, lines - 1);
      const uint32_t* pb = ring_row(cur, sn, W) + 32 * min(lane + 64, lines - 1);
      pfa = __hip_atomic_load(pa, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      pfb = __hip_atomic_load(pb, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    resolve();
    if (async_cas) {  // the CAS this resolve set up, then its result
      issue_cas();
      resolve();
    }
    if (have_res) {
      build_rows(reserve_take(res_ob, 64), 64);
      have_res = false;
    }
    while (tail > head) {
      const int nb = min(64, tail - head);
      build_rows(reserve_take(reserve_issue(nb), nb), nb);
    }
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
  }
  if (lane == 0 && my_gen) atomicAdd(&ctr->generated, (unsigned long long)my_gen);
  if (lane == 0 && my_probe) atomicAdd(&ctr->probes, (unsigned long long)my_probe);
  if (lane == 0 && dedup_new) atomicAdd(&ctr->next_count, dedup_new);
  STAMP(7);
  RTLA_STAMP_FLUSH(ctr, lane)
  __syncthreads();
  for (int k = threadIdx.x; k < 2 * COVER_CODES; k += blockDim.x)
    if (cov[k]) atomicAdd(&ctr->cover[k], (unsigned long long)cov[k]);
}

// Owner side of the exchange: insert the fingerprints other shards sent and
// answer each record with 0 (seen) or 1 + its dense rank among the new
// fingerprints from that source (the sender uses the rank as the row slot it
// ships the materialised state into).  Region p holds counts[p] records.
__global__ void k_insert_remote(const unsigned long long* __restrict__ recv_fp,
                                const unsigned long long* __restrict__ counts, int nshard, unsigned long long cap,
                                unsigned long long* table, int tlog2, uint32_t* __restrict__ ans,
                                unsigned long long* __restrict__ new_count, DevCounters* ctr) {
  // grid.y = source shard p; lanes of a wave share p, so one atomic per wave
  // hands out the dense ranks of its new fingerprints
  const unsigned long long p = blockIdx.y;
  const unsigned long long n = counts[p];
  const int lane = threadIdx.x & 63;
  unsigned probes = 0;
  const unsigned long long stride = (unsigned long long)gridDim.x * blockDim.x;
  for (unsigned long long k0 = (unsigned long long)blockIdx.x * blockDim.x + (threadIdx.x & ~63u); k0 < n;
       k0 += stride) {
    const unsigned long long k = k0 + lane;
    int r = 0;
    if (k < n) {
      const unsigned long long i = p * cap + k;
      const FP f{recv_fp[2 * i], recv_fp[2 * i + 1]};
      if (f.a | f.b) {  // 0:0 = a hole in the sender's outbox chunk
        r = fpset_insert(table, tlog2, f);
        if (r < 0) set_flag(ctr, FLAG_FPSET_FULL);
        probes++;
      }
    }
    const unsigned long long m = __ballot(r == 1);
    unsigned long long b = 0;
    if (m) {
      if (lane == 0) b = atomicAdd(&new_count[p], (unsigned long long)__popcll(m));
      b = shfl0_u64(b);
    }
    if (k < n) ans[p * cap + k] = r == 1 ? (uint32_t)(b + __popcll(m & ((1ull << lane) - 1ull))) + 1u : 0u;
  }
  for (int off = 32; off > 0; off >>= 1) probes += __shfl_down(probes, off);
  if (lane == 0 && probes) atomicAdd(&ctr->probes, (unsigned long long)probes);
}

// Sender side: materialise the queued successors whose owner answered "new"
// with a rank in [lo, hi) into the owner's row region (row + parent record,
// RW = W + 2 words per slot).  Invariants are checked here, where parent and
// action are known; a violation is recorded against the local parent.
template <int NS>
__global__ void __launch_bounds__(256)
k_pack_rows(Layout L, Ring cur, unsigned long long cur_base, int me,
            const unsigned long long* __restrict__ send_ref, const uint32_t* __restrict__ ans,
            const unsigned long long* __restrict__ counts, int nshard, unsigned long long cap, unsigned long long lo,
            unsigned long long hi, uint32_t* __restrict__ rows, unsigned long long rows_cap, DevCounters* ctr) {
  // A wave scans 64 records of owner p (grid.y), compacts the winners of
  // this sub-round, gathers their parent rows into LDS (one coalesced read
  // per row), builds each successor in place and ships row + parent record
  // to the slot the owner's answer names (one coalesced write per row).
  extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
  __shared__ unsigned int cov[COVER_CODES];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int wpb = blockDim.x >> 6;
  const int W = L.W, AW = L.all_words, RW = W + 2;
  uint32_t* lrows = lds + wave * lane_lds_words(W, AW);
  const LaneWords pall{lrows + 64 * W + lane};
  for (int k = threadIdx.x; k < COVER_CODES; k += blockDim.x) cov[k] = 0;
  __syncthreads();
  const unsigned long long p = blockIdx.y;  // owner shard
  const unsigned long long n = counts[p];
  const unsigned long long below = (1ull << lane) - 1ull;
  for (unsigned long long k0 = ((unsigned long long)blockIdx.x * wpb + wave) * 64ull; k0 < n;
       k0 += (unsigned long long)gridDim.x * wpb * 64ull) {
    const unsigned long long k = k0 + lane;
    const unsigned long long i = p * cap + k;
    const unsigned long long a = k < n ? ans[i] : 0ull;
    const bool win = a != 0 && a - 1 >= lo && a - 1 < hi;
    const unsigned long long m = __ballot(win);
    if (!m) continue;
    const int nw = __popcll(m);
    // compact: winner number r of this wave = lane w_r
    int r_of_lane = __popcll(m & below);
    unsigned long long ref = win ? send_ref[i] : 0ull;
    unsigned long long dslot = win ? a - 1 - lo : 0ull;
    // lane r takes the r-th winner's (ref, dslot)
    int src_lane = 0;
    {
      unsigned long long mm = m;
      for (int r = 0; r < nw; r++) {
        const int l = __builtin_ctzll(mm);
        mm &= mm - 1;
        if (lane == r) src_lane = l;
      }
    }
    (void)r_of_lane;
    ref = shfl_u64(ref, src_lane);
    dslot = shfl_u64(dslot, src_lane);
    const bool act = lane < nw;
    const unsigned long long s = ref >> 16;
    const int inst = (int)(ref & 0xffffull);
    gather_rows_lds(lrows, W, nw, [&](int r) { return ring_row(cur, readlane_u64(s, r), W); }, lane);
    wave_sync();
    uint32_t* prow = lrows + lane * W;
    if (act) {
      const FP pfp = fp_add(row_fp(prow), alllogs_delta<NS>(L, prow, pall));
      DeltaT<NS> d;
      compute_delta<NS>(L, prow, inst, d);
      const FP cfp = fp_add(pfp, delta_fp<NS>(L, prow, d));
      const int bad = check_invariants_v<NS>(L, prow, d.srv, d.rec[0], d.rec[1], d.elec, d.erec[0]);
      if (bad && __hip_atomic_load(&ctr->viol_mask, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0 &&
            atomicCAS(&ctr->viol_mask, 0, bad) == 0) {
        ctr->viol_parent = cur_base + s;
        ctr->viol_inst = inst;
        ctr->viol_in_model = 1;
        ctr->viol_child = ~0ull;
      }
      atomicAdd(&cov[cover_code(L, inst, d.sub)], 1u);
      materialize<NS>(L, prow, d, pall, cfp, prow);  // in place
    }
    wave_sync();
    for (int r = 0; r < nw; r++) {
      const unsigned long long ds = readlane_u64(dslot, r);
      uint32_t* dst = rows + (p * rows_cap + ds) * (unsigned long long)RW;
      for (int w = lane; w < W; w += 64) dst[w] = lrows[r * W + w];
      if (lane == 0) {
        const unsigned long long pr =
            (unsigned long long)me << 56 | (cur_base + readlane_u64(s, r)) << 16 | (unsigned long long)__builtin_amdgcn_readlane(inst, r);
        dst[W] = (uint32_t)pr;
        dst[W + 1] = (uint32_t)(pr >> 32);
      }
    }
    wave_sync();
  }
  __syncthreads();
  for (int k = threadIdx.x; k < COVER_CODES; k += blockDim.x)
    if (cov[k]) atomicAdd(&ctr->cover[COVER_CODES + k], (unsigned long long)cov[k]);
}

// Owner side: append the received rows to the next frontier (one wave per
// row, coalesced copy) with their cross-shard parent records.
__global__ void k_unpack_rows(int W, const uint32_t* __restrict__ rows, const unsigned long long* __restrict__ counts,
                              const unsigned long long* __restrict__ bases, int nshard, unsigned long long rows_cap,
                              Ring next, unsigned long long* __restrict__ parents,
                              unsigned long long next_base, unsigned long long next_cap, DevCounters* ctr) {
  // grid.y = source shard p; its rows land at the contiguous slots bases[p] + k
  // (bases from k_part_counts: no per-row atomics)
  const unsigned long long p = blockIdx.y;
  const unsigned long long n = counts[p], base = bases[p];
  const int lane = threadIdx.x & 63;
  const int RW = W + 2;
  const unsigned long long wv = (blockIdx.x * (unsigned long long)blockDim.x + threadIdx.x) >> 6;
  const unsigned long long nw = ((unsigned long long)gridDim.x * blockDim.x) >> 6;
  for (unsigned long long k = wv; k < n; k += nw) {
    const unsigned long long o = base + k;
    if (o >= next_cap) {
      if (lane == 0) set_flag(ctr, FLAG_FRONTIER_FULL);
      continue;
    }
    const uint32_t* src = rows + (p * rows_cap + k) * (unsigned long long)RW;
    uint32_t* dst = ring_row(next, o, W);
    for (int w = lane; w < W; w += 64) dst[w] = src[w];
    if (lane == 0) parents[next_base + o] = (unsigned long long)src[W] | (unsigned long long)src[W + 1] << 32;
  }
}

// rows_in[p] = the part [lo, lo + rc) of the new_count[p] rows owner-side.
// and bases[p] = the next-frontier slot of its first row; advances next_count.
__global__ void k_part_counts(const unsigned long long* __restrict__ new_count, int nshard, unsigned long long lo,
                              unsigned long long rc, unsigned long long* __restrict__ rows_in,
                              unsigned long long* __restrict__ bases, DevCounters* ctr) {
  if (threadIdx.x != 0) return;
  unsigned long long b = ctr->next_count;
  for (int p = 0; p < nshard; p++) {
    const unsigned long long n = new_count[p];
    const unsigned long long r = n > lo ? min(n - lo, rc) : 0ull;
    rows_in[p] = r;
    bases[p] = b;
    b += r;
  }
  ctr->next_count = b;
}

// Insert the fingerprints of `n` rows (Init).  new_flags[i] = 1 if new.
__global__ void k_insert_rows(Layout L, const uint32_t* rows, unsigned long long n, unsigned long long* table,
                              int tlog2, int* new_flags, DevCounters* ctr) {
  unsigned long long i = blockIdx.x * (unsigned long long)blockDim.x + threadIdx.x;
  if (i >= n) return;
  FP f = row_fp(rows + i * (unsigned long long)L.W);
  int r = fpset_insert(table, tlog2, f);
  if (r < 0) set_flag(ctr, FLAG_FPSET_FULL);
  new_flags[i] = r == 1;
}

// Parity seam: every enabled successor of every input row (in-model or not),
// materialised.  out_info[k] = input index << 32 | in_model << 31 | sub << 16 | inst.
template <int NS>
__global__ void __launch_bounds__(256)
k_expand_batch(Layout L, const uint32_t* __restrict__ rows, unsigned long long n, uint32_t* __restrict__ out,
               unsigned long long* __restrict__ out_info, unsigned long long cap, DevCounters* ctr) {
  extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int wpb = blockDim.x >> 6;
  const int W = L.W;
  uint32_t* prow = lds + wave * wave_lds_words(W);
  uint32_t* pall = prow + even_words(W);
  FP* hsrv = reinterpret_cast<FP*>(pall + 32);
  uint32_t* stage = pall + 32 + 4 * NMAX;
  const int fixed = L.fam[F_RECEIVE];
  for (unsigned long long s = (unsigned long long)blockIdx.x * wpb + wave; s < n;
       s += (unsigned long long)gridDim.x * wpb) {
    const FP pfp = load_parent<NS>(L, rows + s * (unsigned long long)W, prow, pall, hsrv, lane);
    const int nmsg = row_nmsg(L, prow);
    const int ncand = fixed + 3 * nmsg;
    for (int base = 0; base < ncand; base += 64) {
      const int q = base + lane;
      DeltaT<NS> d;
      d.enabled = 0;
      int inst = 0;
      if (q < ncand) {
        inst = candidate_inst(L, q, nmsg);
        compute_delta<NS>(L, prow, inst, d);
      }
      bool en = d.enabled != 0;
      if (en && d.err) {
        set_flag(ctr, d.err == 1 ? FLAG_SPEC_ERROR : FLAG_ROW_OVERFLOW);
        en = false;
      }
      const unsigned long long m = __ballot(en);
      const int cnt = __popcll(m);
      if (!cnt) continue;
      const int rank = __popcll(m & ((1ull << lane) - 1ull));
      unsigned long long obase = 0;
      if (lane == 0) obase = atomicAdd(&ctr->next_count, (unsigned long long)cnt);
      obase = shfl0_u64(obase);
      if (obase + cnt > cap) {
        if (lane == 0) set_flag(ctr, FLAG_FRONTIER_FULL);
        continue;
      }
      const FP cfp = en ? fp_add(pfp, delta_fp<NS>(L, prow, d)) : FP{0, 0};
      for (int b = 0; b < cnt; b += STAGE_ROWS) {
        if (en && rank >= b && rank < b + STAGE_ROWS) materialize<NS>(L, prow, d, pall, cfp, stage + (rank - b) * W);
        wave_sync();
        const int nb = min(STAGE_ROWS, cnt - b);
        uint32_t* dst = out + (obase + b) * (unsigned long long)W;
        for (int w = lane; w < nb * W; w += 64) dst[w] = stage[w];
        wave_sync();
      }
      if (en)
        out_info[obase + rank] = s << 32 | (unsigned long long)(d.in_model ? 1u : 0u) << 31 |
                                 (unsigned long long)d.sub << 16 | (unsigned long long)inst;
    }
  }
}

// Synthetic microbench input (BASELINE configs[4], rtla_synth.h): input states
// first .. first + n - 1 as rows 0 .. n - 1 of `out`.  One lane builds one
// row in LDS; the wave stores its 64 rows with coalesced stores.
__global__ void __launch_bounds__(64)
k_random_rows(Layout L, unsigned long long seed, unsigned long long first, unsigned long long n,
              unsigned long long pool, uint32_t* __restrict__ out) {
  extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
  const int lane = threadIdx.x & 63;
  const int W = L.W;
  for (unsigned long long g = (unsigned long long)blockIdx.x * 64; g < n; g += (unsigned long long)gridDim.x * 64) {
    const int nv = (int)min<unsigned long long>(64ull, n - g);
    if (lane < nv) random_state(L, seed, synth_state_id(seed, first + g + lane, pool), lds + lane * W);
    wave_sync();
    uint32_t* dst = out + g * (unsigned long long)W;
    for (int w = lane; w < nv * W; w += 64) dst[w] = lds[w];
    wave_sync();
  }
}

// Microbenchmark kernel: random 8-B CAS inserts into a table (calibrates the
// random-access roofline of the fingerprint set).
__global__ void k_probe_bench(unsigned long long* table, int tlog2, unsigned long long n, unsigned long long seed,
                              DevCounters* ctr, int load_first) {
  unsigned long long i = blockIdx.x * (unsigned long long)blockDim.x + threadIdx.x;
  unsigned long long stride = (unsigned long long)gridDim.x * blockDim.x;
  unsigned long long got = 0;
  for (; i < n; i += stride) {
    FP f = hash_u64(seed, i);
    if (load_first) {
      const unsigned long long idx = f.a >> (64 - tlog2);
      const unsigned long long v = __hip_atomic_load(&table[idx], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      got += fpset_resolve_loaded(table, tlog2, f.b | 1ull, idx, v, ctr) ? 1 : 0;
    } else {
      got += fpset_insert(table, tlog2, f) == 1;
    }
  }
  for (int off = 32; off > 0; off >>= 1) got += __shfl_down(got, off);
  if ((threadIdx.x & 63) == 0 && got) atomicAdd(&ctr->next_count, got);
}

// ---------------------------------------------------------------- launch ----
namespace rtla {

size_t expand_lds_bytes(const Layout& L, int wpb) {
  return (size_t)wpb * (size_t)wave_lds_words(L.W) * sizeof(uint32_t);
}

int expand_lane_wpb(const Layout& L) {
  const size_t per = (size_t)lane_lds_words(L.W, L.all_words) * sizeof(uint32_t);
  if (per > 64 * 1024) return 0;
  return per * 4 <= 64 * 1024 ? 4 : (per * 2 <= 64 * 1024 ? 2 : 1);
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
constexpr int spec_group(const Layout& L) {
  const int g = compact_group(L);
  return g == 32 && compact_lds_words(L.W, L.all_words, 32, L.sym, true) * sizeof(uint32_t) > RTLA_GROUP32_LDS ? 16 : g;
}

static int device_cus() {
  static int cus = 0;
  if (!cus) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
      cus = 256;
  }
  return cus;
}


int expand_compact_wpb(const Layout& L) {
  const size_t per = (size_t)compact_lds_words(L.W, L.all_words, compact_group(L), L.sym, true) * sizeof(uint32_t);
  // one wave may use up to the CU's 160 KiB of LDS; instance ids fit 8 bits per 64-instance window
  if (per > 160 * 1024 || ((L.fam[F_COUNT] + 63) / 64) * 64 > 256) return 0;
  return per * 4 <= 64 * 1024 ? 4 : (per * 2 <= 64 * 1024 ? 2 : 1);
}

int expand_blocks_per_cu(const Layout& L) {
  size_t per = expand_lds_bytes(L, 4) + 2 * COVER_CODES * sizeof(unsigned int);
  int b = (int)((160u * 1024u) / per);
  return b < 1 ? 1 : (b > 8 ? 8 : b);
}

#define RTLA_DISPATCH_N(L, KERNEL, ...)                        \
  switch ((L).N) {                                             \
    case 1: hipLaunchKernelGGL(KERNEL<1>, __VA_ARGS__); break; \
    case 2: hipLaunchKernelGGL(KERNEL<2>, __VA_ARGS__); break; \
    case 3: hipLaunchKernelGGL(KERNEL<3>, __VA_ARGS__); break; \
    case 4: hipLaunchKernelGGL(KERNEL<4>, __VA_ARGS__); break; \
    default: hipLaunchKernelGGL(KERNEL<5>, __VA_ARGS__); break; \
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
static hipError_t launch_compact(const Layout& L, bool multi, const Ring& cur, uint64_t s_begin, uint64_t s_end,
                                 uint64_t cur_base, const Ring& next, uint64_t* parents, uint64_t next_base,
                                 uint64_t next_cap, uint64_t* table, int tlog2, DevCounters* ctr, const ShardBox& box,
                                 hipStream_t st, int xflags, uint64_t* sent, int wpb) {
  auto kfn = multi ? k_expand_compact<NS, true, GROUP, LC, SYM> : k_expand_compact<NS, false, GROUP, LC, SYM>;
  const uint64_t groups = (s_end - s_begin + GROUP - 1) / GROUP;
  uint64_t blocks = std::min<uint64_t>((groups + wpb - 1) / wpb, 1u << 20);
  const size_t lds = (size_t)wpb * compact_lds_words(L.W, L.all_words, GROUP, SYM, multi) * sizeof(uint32_t);
  if (!(xflags & XF_NO_PERSIST)) {  // persistent waves: exactly the resident capacity, looping over groups
    static int per_cu[2][2];  // per instantiation: [multi][one-wave blocks]
    int& pc = per_cu[multi][wpb == 1];
    if (!pc) {
      if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&pc, kfn, 64 * wpb, lds) != hipSuccess || pc < 1)
        pc = 16 / wpb;
      if (const char* e = getenv("RTLA_BLOCKS_PER_CU"))  // occupancy experiments
        if (atoi(e) > 0) pc = std::min(pc, atoi(e));
    }
    blocks = std::min<uint64_t>(blocks, (uint64_t)device_cus() * pc);
  }
  {
    hipError_t e = hipMemsetAsync(&ctr->group_next, 0, sizeof(ctr->group_next), st);
    if (e != hipSuccess) return e;
  }
  hipLaunchKernelGGL(kfn, dim3((unsigned)blocks), dim3(64 * wpb), lds, st, L, cur, (unsigned long long)s_begin,
                     (unsigned long long)s_end, (unsigned long long)cur_base, next, (unsigned long long*)parents,
                     (unsigned long long)next_base, (unsigned long long)next_cap, (unsigned long long*)table,
                     (unsigned long long*)sent, tlog2, ctr, box, xflags);
  return hipGetLastError();
}

hipError_t launch_expand(const Layout& L, const Ring& cur, uint64_t s_begin, uint64_t s_end, uint64_t cur_base,
                         const Ring& next, uint64_t* parents, uint64_t next_base, uint64_t next_cap, uint64_t* table,
                         int tlog2, DevCounters* ctr, const ShardBox& box, int grid, hipStream_t st, int xflags,
                         uint64_t* sent, hipEvent_t mid) {
  if (s_end <= s_begin) return hipSuccess;
  const int cwpb = expand_compact_wpb(L);
  if (cwpb > 0 && !(xflags & XF_WAVE_KERNEL) && (box.nshard == 1 || sent)) {
    const bool multi = box.nshard > 1;
    const int wpb = (xflags & XF_BLOCK4) ? cwpb : 1;  // one-wave workgroups by default
    hipError_t e = hipSuccess;
#define RTLA_ARGS L, multi, cur, s_begin, s_end, cur_base, next, parents, next_base, next_cap, table, tlog2, ctr, box, \
                  st, xflags, sent, wpb
#define RTLA_SPEC(S)                                                                               \
  if (!done && same_layout(L, specs::S)) {                                                         \
    e = launch_compact<specs::S.N, spec_group(specs::S), specs::S, (bool)specs::S.sym>(RTLA_ARGS);   \
    done = true;                                                                                   \
  }
    bool done = false;
    if (L.sym && !(xflags & XF_NO_SPECIAL)) RTLA_SPEC(CFG4)
#ifndef RTLA_EXP_MINIMAL  // perf experiments: compiled-in layouts only (fast builds)
    if (!done && L.sym) {
#define RTLA_SYMN(n) \
  case n: e = launch_compact<n, 32, Layout{}, true>(RTLA_ARGS); break;
      switch (L.N) {
        RTLA_SYMN(1)
        RTLA_SYMN(2)
        RTLA_SYMN(3)
        RTLA_SYMN(4)
        default: RTLA_SYMN(5)
      }
#undef RTLA_SYMN
      done = true;
    }
#endif
    if (!done && !(xflags & XF_NO_SPECIAL)) {
      RTLA_SPEC(CFG2)
      RTLA_SPEC(CFG1)
      RTLA_SPEC(EXHAUST)
      RTLA_SPEC(CFG3)
      RTLA_SPEC(SYNTH)
    }
    if (!done) {  // run-time layout
#ifdef RTLA_EXP_MINIMAL
      return hipErrorNotSupported;
#else
      const bool g64 = compact_group(L) == 64;
#define RTLA_GENERIC(n) \
  case n: e = g64 ? launch_compact<n, 64, Layout{}>(RTLA_ARGS) : launch_compact<n, 32, Layout{}>(RTLA_ARGS); break;
      switch (L.N) {
        RTLA_GENERIC(1)
        RTLA_GENERIC(2)
        RTLA_GENERIC(3)
        RTLA_GENERIC(4)
        default: RTLA_GENERIC(5)
      }
#undef RTLA_GENERIC
#endif
    }
#undef RTLA_SPEC
#undef RTLA_ARGS
    if (e != hipSuccess) return e;
    if (mid) {
      e = hipEventRecord(mid, st);
      if (e != hipSuccess) return e;
    }
    return hipGetLastError();
  }
  // one wave per state: rows too wide for the compacting kernel's LDS tile
  // (or forced, XF_WAVE_KERNEL)
  RTLA_DISPATCH_N(L, k_expand, dim3(grid), dim3(256), expand_lds_bytes(L, 4), st, L, cur,
                  (unsigned long long)s_begin, (unsigned long long)s_end, (unsigned long long)cur_base, next,
                  (unsigned long long*)parents, (unsigned long long)next_base, (unsigned long long)next_cap,
                  (unsigned long long*)table, tlog2, ctr, box);
  return hipGetLastError();
}

static unsigned grid_x(uint64_t n, int per_block) {
  return (unsigned)std::max<uint64_t>(1, std::min<uint64_t>((n + per_block - 1) / per_block, 4096));
}

hipError_t launch_insert_remote(const uint64_t* recv_fp, const uint64_t* counts, int nshard, uint64_t cap,
                                uint64_t* table, int tlog2, uint32_t* ans, uint64_t* new_count, DevCounters* ctr,
                                uint64_t max_count, hipStream_t st) {
  if (!max_count) return hipSuccess;
  hipLaunchKernelGGL(k_insert_remote, dim3(grid_x(max_count, 256), nshard), dim3(256), 0, st,
                     (const unsigned long long*)recv_fp, (const unsigned long long*)counts, nshard,
                     (unsigned long long)cap, (unsigned long long*)table, tlog2, ans, (unsigned long long*)new_count,
                     ctr);
  return hipGetLastError();
}

hipError_t launch_pack_rows(const Layout& L, const Ring& cur, uint64_t cur_base, int me, const uint64_t* send_ref,
                            const uint32_t* ans, const uint64_t* counts, int nshard, uint64_t cap, uint64_t lo,
                            uint64_t hi, uint32_t* rows, uint64_t rows_cap, DevCounters* ctr, uint64_t max_count,
                            hipStream_t st) {
  if (!max_count) return hipSuccess;
  const int wpb = std::max(1, expand_lane_wpb(L));
  const size_t lds = (size_t)wpb * lane_lds_words(L.W, L.all_words) * sizeof(uint32_t);
  RTLA_DISPATCH_N(L, k_pack_rows, dim3(grid_x(max_count, 64 * wpb), nshard), dim3(64 * wpb), lds, st, L, cur,
                  (unsigned long long)cur_base, me, (const unsigned long long*)send_ref, ans,
                  (const unsigned long long*)counts, nshard, (unsigned long long)cap, (unsigned long long)lo,
                  (unsigned long long)hi, rows, (unsigned long long)rows_cap, ctr);
  return hipGetLastError();
}

hipError_t launch_unpack_rows(int W, const uint32_t* rows, const uint64_t* counts, const uint64_t* bases, int nshard,
                              uint64_t rows_cap, const Ring& next, uint64_t* parents, uint64_t next_base,
                              uint64_t next_cap, DevCounters* ctr, uint64_t max_count, hipStream_t st) {
  if (!max_count) return hipSuccess;
  hipLaunchKernelGGL(k_unpack_rows, dim3(grid_x(max_count, 4), nshard), dim3(256), 0, st, W, rows,
                     (const unsigned long long*)counts, (const unsigned long long*)bases, nshard,
                     (unsigned long long)rows_cap, next, (unsigned long long*)parents, (unsigned long long)next_base,
                     (unsigned long long)next_cap, ctr);
  return hipGetLastError();
}

hipError_t launch_part_counts(const uint64_t* new_count, int nshard, uint64_t lo, uint64_t rc, uint64_t* rows_in,
                              uint64_t* bases, DevCounters* ctr, hipStream_t st) {
  hipLaunchKernelGGL(k_part_counts, dim3(1), dim3(64), 0, st, (const unsigned long long*)new_count, nshard,
                     (unsigned long long)lo, (unsigned long long)rc, (unsigned long long*)rows_in,
                     (unsigned long long*)bases, ctr);
  return hipGetLastError();
}

hipError_t launch_insert_rows(const Layout& L, const uint32_t* rows, uint64_t n, uint64_t* table, int tlog2,
                              int* new_flags, DevCounters* ctr, hipStream_t st) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(k_insert_rows, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, L, rows,
                     (unsigned long long)n, (unsigned long long*)table, tlog2, new_flags, ctr);
  return hipGetLastError();
}

hipError_t launch_expand_batch(const Layout& L, const uint32_t* rows, uint64_t n, uint32_t* out, uint64_t* info,
                               uint64_t cap, DevCounters* ctr, hipStream_t st) {
  if (n == 0) return hipSuccess;
  uint64_t blocks = (n + 3) / 4;
  int grid = (int)(blocks < 4096 ? blocks : 4096);
  RTLA_DISPATCH_N(L, k_expand_batch, dim3(grid), dim3(256), expand_lds_bytes(L, 4), st, L, rows,
                  (unsigned long long)n, out, (unsigned long long*)info, (unsigned long long)cap, ctr);
  return hipGetLastError();
}

hipError_t launch_random_rows(const Layout& L, uint64_t seed, uint64_t first, uint64_t n, uint64_t pool, uint32_t* out,
                              hipStream_t st) {
  if (!n) return hipSuccess;
  const unsigned blocks = (unsigned)std::min<uint64_t>((n + 63) / 64, 256 * 32);
  hipLaunchKernelGGL(k_random_rows, dim3(blocks), dim3(64), (size_t)64 * L.W * sizeof(uint32_t), st, L,
                     (unsigned long long)seed, (unsigned long long)first, (unsigned long long)n,
                     (unsigned long long)pool, out);
  return hipGetLastError();
}

hipError_t launch_probe_bench(uint64_t* table, int tlog2, uint64_t n, uint64_t seed, DevCounters* ctr,
                              hipStream_t st, int load_first) {
  hipLaunchKernelGGL(k_probe_bench, dim3(256 * 16), dim3(256), 0, st, (unsigned long long*)table, tlog2,
                     (unsigned long long)n, (unsigned long long)seed, ctr, load_first);
  return hipGetLastError();
}

}  // namespace rtla
