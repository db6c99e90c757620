// rtla_synth.h -- random valid packed states for the synthetic microbench
// (BASELINE.json configs[4]): "1e9 random packed
// Raft states through Next + fingerprint + dedup".
//
// Input state number i (a counter) maps to a state id: with probability 1/2
// (when a pool is given) an id drawn from [0, pool) -- those inputs repeat
// earlier ones, so dedup has hits -- otherwise the fresh id pool + i.  Every
// field of the state with that id comes from a counter-based PRNG
// (splitmix64 of seed, id and a draw counter), uniform within the bounds of
// the configuration and structurally valid, so the kernels evaluate Next on
// it exactly as on a reachable state (raft.tla:454-465):
//   currentTerm 1..T, state F/C/L, votedFor Nil or a server, log of 0..L
//   entries (term 1..T, value), commitIndex 0..Len(log), votesGranted a
//   subset of votesResponded, DOMAIN voterLog a subset of votesGranted with
//   random logs, nextIndex 1..Len(log)+1 (so AppendEntries never reads
//   outside the log: no TLC evaluation error), matchIndex 0..L; allLogs a
//   random subset of the log universe; 0..E-1 distinct random election
//   records; a bag of 0..K-1 distinct random messages of the four record
//   types with counts 1..C (one slot of each kept free: every action adds at
//   most one election record and one distinct message, so no successor
//   overflows the row format).
// Used on the GPU (k_random_rows) and on the host (rtla_random_rows, the
// tests' sample), from this one definition.
#pragma once
#include "rtla_model.h"

#if defined(__HIPCC__) || defined(__HIP__)
#define RTLA_HDM __host__ __device__ __forceinline__
#else
#define RTLA_HDM inline
#endif

namespace rtla {

struct SynthRng {
  uint64_t base, k;
  RTLA_HDM uint64_t next() { return mix_a(base + 0x9E3779B97F4A7C15ull * ++k); }
  RTLA_HDM uint32_t below(uint32_t n) { return (uint32_t)(((next() >> 32) * (uint64_t)n) >> 32); }  // [0, n)
};

RTLA_HD uint64_t synth_state_id(uint64_t seed, uint64_t i, uint64_t pool) {
  const uint64_t r = mix_b(seed ^ (i * 0xD1B54A32D192ED03ull + 0x5851F42D4C957F2Dull));
  return (pool && (r & 1)) ? (r >> 1) % pool : pool + i;
}

RTLA_HD uint32_t synth_log(const Layout& L, SynthRng& g, uint32_t maxlen) {
  const uint32_t n = g.below(maxlen + 1);
  uint32_t lg = 0;
  for (uint32_t k = 0; k < n; k++) lg = log_append(lg, (1 + g.below((uint32_t)L.T)) | g.below((uint32_t)L.V) << 3);
  return lg;
}

template <class P>
RTLA_HD void random_state(const Layout& L, uint64_t seed, uint64_t id, P row) {
  SynthRng g{mix_b(seed * 0x9E3779B97F4A7C15ull ^ mix_a(id + 0x243f6a8885a308d3ull)), 0};
  const int N = L.N, EW = L.EW;
  const uint32_t all_srv = (1u << N) - 1u;
  for (int w = 0; w < L.W; w++) row[w] = 0;
  for (int i = 0; i < N; i++) {
    uint32_t rec[3 + NMAX] = {0};
    const uint32_t lg = synth_log(L, g, (uint32_t)L.L);
    const uint32_t len = log_len(lg);
    const uint32_t vresp = g.below(all_srv + 1);
    const uint32_t vgrant = vresp & g.below(all_srv + 1);
    const uint32_t vlp = vgrant & g.below(all_srv + 1);
    const uint32_t voted = g.below((uint32_t)N + 1);
    rec[0] = s_make(1 + g.below((uint32_t)L.T), g.below(3), voted == (uint32_t)N ? NIL : voted, g.below(len + 1), vresp,
                    vgrant, vlp);
    rec[1] = lg;
    uint32_t nm = 0;
    for (int j = 0; j < N; j++) {
      nm = nm_set_next(nm, j, 1 + g.below(len + 1));
      nm = nm_set_match(nm, j, g.below((uint32_t)L.L + 1));
    }
    rec[2] = nm;
    for (int j = 0; j < N; j++)
      if (vlp >> j & 1u) rec[3 + j] = synth_log(L, g, (uint32_t)L.L);
    srv_put(L, row, i, rec);
  }
  for (int x = 0; x < L.n_logs; x++)
    if (g.below(16) == 0) row[L.off_all + (x >> 5)] |= 1u << (x & 31);
  int ne = 0;
  const int want_e = (int)g.below((uint32_t)L.E);  // < E: BecomeLeader may still append one
  for (int e = 0; e < want_e; e++) {
    uint32_t er[2 + NMAX], have[2 + NMAX];
    const uint32_t votes = g.below(all_srv + 1), dom = votes & g.below(all_srv + 1);
    er[0] = (1 + g.below((uint32_t)L.T)) | g.below((uint32_t)N) << 4 | votes << 7 | dom << 12;
    er[1] = synth_log(L, g, (uint32_t)L.L);
    for (int j = 0; j < N; j++) er[2 + j] = (dom >> j & 1u) ? synth_log(L, g, (uint32_t)L.L) : 0u;
    bool dup = false;
    for (int f = 0; f < ne; f++) {
      elec_get(L, row, f, have);
      bool same = true;
      for (int w = 0; w < EW; w++) same = same && have[w] == er[w];
      dup = dup || same;
    }
    if (dup) continue;
    elec_put(L, row, ne, er);
    ne++;
  }
  int nmsg = 0;
  const int want_m = (int)g.below((uint32_t)L.K);  // < K: an action may still add one message
  for (int q = 0; q < want_m; q++) {
    const uint32_t type = g.below(4), src = g.below((uint32_t)N), dst = g.below((uint32_t)N);
    const uint32_t term = 1 + g.below((uint32_t)L.T);
    uint64_t key;
    if (type == RVREQ) {
      key = m_rvreq(src, dst, term, g.below((uint32_t)L.T + 1), g.below((uint32_t)L.L + 1));
    } else if (type == RVRESP) {
      key = m_rvresp(src, dst, term, g.below(2), synth_log(L, g, (uint32_t)L.L));
    } else if (type == AEREQ) {
      const uint32_t has = g.below(2);
      const uint32_t entry = has ? ((1 + g.below((uint32_t)L.T)) | g.below((uint32_t)L.V) << 3) : 0u;
      key = m_aereq(src, dst, term, g.below((uint32_t)L.L + 1), g.below((uint32_t)L.T + 1), has, entry,
                    g.below((uint32_t)L.L + 1), synth_log(L, g, (uint32_t)L.L));
    } else {
      key = m_aeresp(src, dst, term, g.below(2), g.below((uint32_t)L.L + 1));
    }
    bool dup = false;
    const uint64_t pk = key_raw(L, key);
    for (int k = 0; k < nmsg; k++) dup = dup || (slot_raw(L, row, k) & slot_keymask(L)) == pk;
    if (dup) continue;
    slot_put(L, row, nmsg, key | (uint64_t)(1 + g.below((uint32_t)L.C)) << 60);
    nmsg++;
  }
  row[L.off_hdr] = (uint32_t)nmsg | (uint32_t)ne << 8;
  row_set_fp(row, row_fingerprint(L, row));
}

}  // namespace rtla
