// rtla_model.h -- packed Raft state rows and the semantics of raft.tla's Next.
//
// This header is the ONE place where the spec's actions are written for the
// product.  Every function is __host__ __device__: the GPU kernels
// (rtla_kernels.hip) evaluate it per (state, action-instance) lane, and the
// host driver uses the same code only to build Init and to decode rows to
// text.  There is no CPU expansion path in the product.
//
// Reference: /root/reference/raft.tla (sha256 683a120a...6b81).  Each action
// below cites the lines it follows.
//
// ---------------------------------------------------------------------------
// Two formats.
//
// WIDE (in registers; what the actions compute on): a server record is 3 + N
// u32 words
//       w0 scalars:   currentTerm 0-3 | state 4-5 | votedFor 6-8 (7 = Nil)
//                     | commitIndex 9-11 | votesResponded 12-16
//                     | votesGranted 17-21 | DOMAIN voterLog[i] 22-26
//       w1 log[i]     (log code, below)
//       w2            nextIndex[i][j] at 3j | matchIndex[i][j] at 15+3j
//       w3+j          voterLog[i][j] (log code; 0 unless bit j of the domain)
// an election record 2 + N words
//       w0 eterm 0-3 | eleader 4-6 | evotes 7-11 | DOMAIN evoterLog 12-16
//       w1 elog, w2+j evoterLog[j]
// a message a u64 (key | count << 60).  Log code (u32): length in bits 0-2;
// entry k (0-based) at bits 3+5k: term (3 bits) | value << 3 (2 bits).
// Message key, fields by type (raft.tla:193-198, :215-225, :294-301, :338-343):
//   type 0-1 | msource 2-4 | mdest 5-7 | mterm 8-11 |
//   RVReq:  mlastLogTerm 12-15 | mlastLogIndex 16-18
//   RVResp: mvoteGranted 12 | mlog 16-43
//   AEReq:  mprevLogIndex 12-14 | mprevLogTerm 15-18 | has-entry 19 |
//           entry 20-24 | mcommitIndex 25-27 | mlog 28-55
//   AEResp: msuccess 12 | mmatchIndex 13-15
//
// ROW (HBM, LDS, the ABI; u32 words, offsets from rtla::Layout): the same
// values bit-packed with the model's own field widths (make_layout), every
// record starting on a word boundary:
//   [0..4)                   fingerprint (a.lo, a.hi, b.lo, b.hi) of this state
//   [off_hdr]                nmsg (bits 0-7) | nelec (bits 8-15)
//   [off_srv + i*srv_w]      server i: currentTerm-1 | state | votedFor (N = Nil)
//                            | commitIndex | votesResponded | votesGranted
//                            | DOMAIN voterLog | log | per j: nextIndex-1,
//                            matchIndex | per j: voterLog[i][j]
//   [off_all]                allLogs: bitmask over the in-model log universe
//   [off_elec + e*elec_w]    election e: eterm-1 | eleader | evotes | DOMAIN
//                            evoterLog | elog | per j: evoterLog[j]
//   [off_bag + k*slot_w]     bag slot k (0 = empty): type | msource | mdest |
//                            mterm-1 | the type's fields | count
// A packed log is length | entries (term-1 | value); a server's own log has
// room for L+1 entries and its term for T+1 (the out-of-model successors of
// ClientRequest / AppendEntries and of Timeout, which the parity seam
// returns); every other log, term and index is bounded by the model (it was
// written by an in-model state).  configs[1]: 172-byte rows (372 wide).
//
// The bag, the elections list and the bag slots are NOT kept in canonical
// order.  State identity is decided only by the fingerprint, which is a sum
// over the state's components (per-server records, messages with their
// counts, allLogs members, election records) of a 128-bit PRF of each
// component -- an order-free function of the TLA+ value.  Two distinct values
// differ in at least one component, so they collide with probability 2^-128
// per pair (2^-64 per half).
// ---------------------------------------------------------------------------
#pragma once
#include <stdint.h>
#include <string.h>

#if defined(__HIPCC__) || defined(__HIP__)
#include <hip/hip_runtime.h>
#define RTLA_HD __host__ __device__ __forceinline__
#else
#define RTLA_HD static inline
#endif

namespace rtla {

constexpr int NMAX = 5;   // servers
constexpr int LMAX = 4;   // MaxLogLen (rows hold LMAX+1 entries)
constexpr int TMAX = 6;   // MaxTerm (rows hold MaxTerm+1)
constexpr int VMAX = 4;   // values
constexpr int CMAX = 14;  // MaxCopies (rows hold MaxCopies+1)
constexpr int KMAX = 64;  // bag slots
constexpr int EMAX = 32;  // election records
constexpr int WMAX = 4 + 1 + NMAX * 6 + 32 + EMAX * 6 + 2 * KMAX;  // widest row (words)

enum { FOLLOWER = 0, CANDIDATE = 1, LEADER = 2 };
enum { RVREQ = 0, RVRESP = 1, AEREQ = 2, AERESP = 3 };
constexpr uint32_t NIL = 7;

// Action families (instance ranges in Layout::fam).  Order = disjunct order of
// Next (raft.tla:454-463).
enum {
  F_RESTART = 0, F_TIMEOUT, F_REQUESTVOTE, F_BECOMELEADER, F_CLIENTREQUEST,
  F_ADVANCECOMMIT, F_APPENDENTRIES, F_RECEIVE, F_DUPLICATE, F_DROP, F_COUNT
};
// Receive sub-actions, reported for coverage / trace labels.
enum {
  R_UPDATETERM = 0, R_HRVREQ, R_HRVRESP, R_HAEREQ, R_HAERESP, R_DROPSTALE, R_NONE
};

// Invariant bits (build-defined model wrapper, specs/MC.tla).
enum { INV_NO_TWO_LEADERS = 1, INV_ELECTION_SAFETY = 2, INV_LOG_MATCHING = 4 };

// A model's row format.  Plain ints only (a C++20 structural type): the
// kernels take it either as a run-time argument or, for the configurations
// compiled in ahead of time (rtla_kernels.hip, LayoutSpecs), as a template
// parameter -- then every offset, bound and family range below is a
// compile-time constant in the generated code.
struct Layout {
  int N, V, T, L, C, M, K, E;
  int inv_mask;
  int sym;             // SYMMETRY Permutations(Server): dedup by orbit key (orbit_key)
  int SW, EW;          // WIDE record words: server 3 + N, election 2 + N
  int off_hdr, off_srv, off_all, all_words, off_elec, off_bag, W;
  int n_logs;          // |{logs of length <= L, terms 1..T}|
  int fam[F_COUNT + 1];  // first instance id of each family; fam[F_COUNT] = #instances
  int log_off[LMAX + 2];  // allLogs index offset of logs of length n
  // ROW packing: field widths in bits
  int b_tcur;  // currentTerm - 1        (0..T: Timeout's out-of-model successor reaches T+1)
  int b_tm1;   // other terms - 1        (message, entry, election terms: 1..T)
  int b_t0;    // terms 0..T             (mlastLogTerm, mprevLogTerm)
  int b_vote;  // votedFor               (0..N-1, N = Nil)
  int b_sid;   // a server id            (0..N-1)
  int b_idx;   // an index 0..L          (commitIndex, nextIndex-1, matchIndex, message indexes)
  int b_val;   // a value                (0..V-1)
  int b_ent;   // a log entry            (term-1 | value << b_tm1)
  int b_log0;  // a log of <= L entries  (length | entries): voterLog, elog, mlog
  int b_log1;  // a server's own log     (<= L+1 entries)
  int b_cnt;   // a message count        (1..C+1)
  // bit offsets inside a packed record, and its words
  int sb_log, sb_nm, sb_vl, srv_w;     // server (scalars at bit 0)
  int eb_log, eb_vl, elec_w;           // election (eterm-1 | eleader | evotes | dom at bit 0)
  int mb_term, mb_pay, mb_cnt, slot_w; // message (type at bit 0, msource 2, mdest)
};

constexpr int bits_for(int x) {  // bits to hold 0..x
  int b = 0;
  while ((1 << b) <= x) b++;
  return b;
}

// Returns 0 on success, <0 if the configuration exceeds the row format.
constexpr int make_layout(Layout* l, int N, int V, int T, int L, int C, int M, int K, int E, int inv_mask) {
  if (N < 1 || N > NMAX || V < 1 || V > VMAX || T < 1 || T > TMAX || L < 0 || L > LMAX ||
      C < 1 || C > CMAX || M < 0 || K < 1 || K > KMAX || E < 0 || E > EMAX)
    return -1;
  if (M > 0 && K < M + 1) return -1;  // out-of-model successors must stay representable
  l->N = N; l->V = V; l->T = T; l->L = L; l->C = C; l->M = M; l->K = K; l->E = E;
  l->inv_mask = inv_mask;
  l->sym = 0;
  l->SW = 3 + N;
  l->EW = 2 + N;
  int B = T * V, off = 0, pw = 1;
  for (int n = 0; n <= L + 1; n++) { l->log_off[n] = off; off += pw; pw *= B; }
  l->n_logs = l->log_off[L + 1];
  if (l->n_logs > 32 * 32) return -1;
  // field widths
  l->b_tcur = bits_for(T);
  l->b_tm1 = bits_for(T - 1);
  l->b_t0 = bits_for(T);
  l->b_vote = bits_for(N);
  l->b_sid = bits_for(N - 1);
  l->b_idx = bits_for(L);
  l->b_val = bits_for(V - 1);
  l->b_ent = l->b_tm1 + l->b_val;
  l->b_log0 = bits_for(L) + L * l->b_ent;
  l->b_log1 = bits_for(L + 1) + (L + 1) * l->b_ent;
  l->b_cnt = bits_for(C + 1);
  // server: scalars | own log | N x (nextIndex-1, matchIndex) | N x voterLog
  l->sb_log = l->b_tcur + 2 + l->b_vote + l->b_idx + 3 * N;
  l->sb_nm = l->sb_log + l->b_log1;
  l->sb_vl = l->sb_nm + 2 * N * l->b_idx;
  l->srv_w = (l->sb_vl + N * l->b_log0 + 31) / 32;
  // election: eterm-1 | eleader | evotes | dom | elog | N x evoterLog
  l->eb_log = l->b_tm1 + l->b_sid + 2 * N;
  l->eb_vl = l->eb_log + l->b_log0;
  l->elec_w = (l->eb_vl + N * l->b_log0 + 31) / 32;
  // message: type | msource | mdest | mterm-1 | payload (the largest type's) | count
  l->mb_term = 2 + 2 * l->b_sid;
  l->mb_pay = l->mb_term + l->b_tm1;
  int pay = l->b_t0 + l->b_idx;                                                      // RVReq
  if (1 + l->b_log0 > pay) pay = 1 + l->b_log0;                                      // RVResp
  const int ae = l->b_idx + l->b_t0 + 1 + l->b_ent + l->b_idx + l->b_log0;             // AEReq
  if (ae > pay) pay = ae;
  if (1 + l->b_idx > pay) pay = 1 + l->b_idx;                                        // AEResp
  l->mb_cnt = l->mb_pay + pay;
  l->slot_w = (l->mb_cnt + l->b_cnt + 31) / 32;
  if (l->slot_w > 2 || l->srv_w > 6 || l->elec_w > 6) return -1;  // (PACKW)
  // row
  l->off_hdr = 4;
  l->off_srv = 5;
  l->off_all = l->off_srv + N * l->srv_w;
  l->all_words = (l->n_logs + 31) / 32;
  l->off_elec = l->off_all + l->all_words;
  l->off_bag = l->off_elec + E * l->elec_w;
  l->W = l->off_bag + K * l->slot_w;
  l->W += !(l->W & 1);  // odd row stride: conflict-free LDS row staging
  int f = 0;
  l->fam[F_RESTART] = f; f += N;
  l->fam[F_TIMEOUT] = f; f += N;
  l->fam[F_REQUESTVOTE] = f; f += N * N;
  l->fam[F_BECOMELEADER] = f; f += N;
  l->fam[F_CLIENTREQUEST] = f; f += N * V;
  l->fam[F_ADVANCECOMMIT] = f; f += N;
  l->fam[F_APPENDENTRIES] = f; f += N * N;
  l->fam[F_RECEIVE] = f; f += K;
  l->fam[F_DUPLICATE] = f; f += K;
  l->fam[F_DROP] = f; f += K;
  l->fam[F_COUNT] = f;
  return 0;
}
// The same by value (N = 0 on a configuration outside the row format).
constexpr Layout layout_of(int N, int V, int T, int L, int C, int M, int K, int E, int inv_mask) {
  Layout l{};
  if (make_layout(&l, N, V, T, L, C, M, K, E, inv_mask) != 0) return Layout{};
  return l;
}
static inline bool same_layout(const Layout& a, const Layout& b) { return memcmp(&a, &b, sizeof(Layout)) == 0; }

// Run-time-indexed reads of the Layout tables as select chains: on the GPU a
// dynamically indexed kernel-argument array becomes a vector memory load, and
// its vmcnt wait would also wait for every fingerprint-set CAS in flight.
RTLA_HD int fam_base(const Layout& L, int fam) {
  int r = 0;
#pragma unroll
  for (int f = 0; f <= F_COUNT; f++)
    if (f == fam) r = L.fam[f];
  return r;
}
RTLA_HD int log_off_at(const Layout& L, int n) {
  int r = 0;
#pragma unroll
  for (int k = 0; k < LMAX + 2; k++)
    if (k == n) r = L.log_off[k];
  return r;
}

// ------------------------------------------------------------- fields ----
RTLA_HD uint32_t s_term(uint32_t w) { return w & 15u; }
RTLA_HD uint32_t s_role(uint32_t w) { return (w >> 4) & 3u; }
RTLA_HD uint32_t s_voted(uint32_t w) { return (w >> 6) & 7u; }
RTLA_HD uint32_t s_commit(uint32_t w) { return (w >> 9) & 7u; }
RTLA_HD uint32_t s_vresp(uint32_t w) { return (w >> 12) & 31u; }
RTLA_HD uint32_t s_vgrant(uint32_t w) { return (w >> 17) & 31u; }
RTLA_HD uint32_t s_vlp(uint32_t w) { return (w >> 22) & 31u; }
RTLA_HD uint32_t s_make(uint32_t term, uint32_t role, uint32_t voted, uint32_t commit,
                        uint32_t vresp, uint32_t vgrant, uint32_t vlp) {
  return term | role << 4 | voted << 6 | commit << 9 | vresp << 12 | vgrant << 17 | vlp << 22;
}
RTLA_HD uint32_t nm_next(uint32_t w, int j) { return (w >> (3 * j)) & 7u; }
RTLA_HD uint32_t nm_match(uint32_t w, int j) { return (w >> (15 + 3 * j)) & 7u; }
RTLA_HD uint32_t nm_set_next(uint32_t w, int j, uint32_t v) {
  return (w & ~(7u << (3 * j))) | (v << (3 * j));
}
RTLA_HD uint32_t nm_set_match(uint32_t w, int j, uint32_t v) {
  return (w & ~(7u << (15 + 3 * j))) | (v << (15 + 3 * j));
}
RTLA_HD uint32_t nm_fill(int N, uint32_t next, uint32_t match) {
  uint32_t w = 0;
  for (int j = 0; j < N; j++) w |= next << (3 * j) | match << (15 + 3 * j);
  return w;
}

// Log codes
RTLA_HD uint32_t log_len(uint32_t l) { return l & 7u; }
RTLA_HD uint32_t log_entry(uint32_t l, uint32_t k1) { return (l >> (3 + 5 * (k1 - 1))) & 31u; }
RTLA_HD uint32_t log_term(uint32_t l, uint32_t k1) { return log_entry(l, k1) & 7u; }
RTLA_HD uint32_t log_val(uint32_t l, uint32_t k1) { return log_entry(l, k1) >> 3; }
RTLA_HD uint32_t last_term(uint32_t l) { return log_len(l) ? log_term(l, log_len(l)) : 0u; }
RTLA_HD uint32_t log_append(uint32_t l, uint32_t entry) {
  uint32_t n = log_len(l);
  return ((l & ~7u) | (n + 1)) | (entry << (3 + 5 * n));
}
RTLA_HD uint32_t log_prefix(uint32_t l, uint32_t n) {  // SubSeq(l, 1, n)
  uint32_t keep = (3 + 5 * n) >= 32 ? 0xffffffffu : ((1u << (3 + 5 * n)) - 1u);
  return (l & keep & ~7u) | n;
}
// Index of an in-model log in the allLogs universe (little-endian mixed radix).
RTLA_HD int log_index(const Layout& L, uint32_t l) {
  int n = (int)log_len(l), idx = 0, pw = 1, B = L.T * L.V;
  for (int k = 1; k <= n; k++) {
    int d = ((int)log_term(l, k) - 1) * L.V + (int)log_val(l, k);
    idx += d * pw;
    pw *= B;
  }
  return log_off_at(L, n) + idx;
}
RTLA_HD uint32_t log_from_index(const Layout& L, int idx) {
  int n = 0;
  while (n + 1 <= L.L && idx >= L.log_off[n + 1]) n++;
  int r = idx - L.log_off[n], B = L.T * L.V;
  uint32_t l = 0;
  for (int k = 0; k < n; k++) {
    int d = r % B;
    r /= B;
    uint32_t t = (uint32_t)(d / L.V + 1), v = (uint32_t)(d % L.V);
    l = log_append(l, t | v << 3);
  }
  return l;
}

// Messages
RTLA_HD uint32_t m_type(uint64_t k) { return (uint32_t)(k & 3u); }
RTLA_HD uint32_t m_src(uint64_t k) { return (uint32_t)(k >> 2) & 7u; }
RTLA_HD uint32_t m_dst(uint64_t k) { return (uint32_t)(k >> 5) & 7u; }
RTLA_HD uint32_t m_term(uint64_t k) { return (uint32_t)(k >> 8) & 15u; }
RTLA_HD uint32_t m_count(uint64_t v) { return (uint32_t)(v >> 60); }
RTLA_HD uint64_t m_key(uint64_t v) { return v & ((1ull << 60) - 1); }
RTLA_HD uint64_t m_base(uint32_t type, uint32_t src, uint32_t dst, uint32_t term) {
  return (uint64_t)type | (uint64_t)src << 2 | (uint64_t)dst << 5 | (uint64_t)term << 8;
}
RTLA_HD uint64_t m_rvreq(uint32_t src, uint32_t dst, uint32_t term, uint32_t llt, uint32_t lli) {
  return m_base(RVREQ, src, dst, term) | (uint64_t)llt << 12 | (uint64_t)lli << 16;
}
RTLA_HD uint64_t m_rvresp(uint32_t src, uint32_t dst, uint32_t term, uint32_t granted, uint32_t mlog) {
  return m_base(RVRESP, src, dst, term) | (uint64_t)granted << 12 | (uint64_t)mlog << 16;
}
RTLA_HD uint64_t m_aereq(uint32_t src, uint32_t dst, uint32_t term, uint32_t prev, uint32_t prevt,
                         uint32_t has, uint32_t entry, uint32_t commit, uint32_t mlog) {
  return m_base(AEREQ, src, dst, term) | (uint64_t)prev << 12 | (uint64_t)prevt << 15 |
         (uint64_t)has << 19 | (uint64_t)entry << 20 | (uint64_t)commit << 25 | (uint64_t)mlog << 28;
}
RTLA_HD uint64_t m_aeresp(uint32_t src, uint32_t dst, uint32_t term, uint32_t success, uint32_t match) {
  return m_base(AERESP, src, dst, term) | (uint64_t)success << 12 | (uint64_t)match << 13;
}
RTLA_HD uint32_t m_f(uint64_t k, int lo, int bits) { return (uint32_t)(k >> lo) & ((1u << bits) - 1u); }

// --------------------------------------------------------------- hash ----
struct FP {
  uint64_t a, b;
};
RTLA_HD uint64_t mix_a(uint64_t z) {  // splitmix64 finalizer
  z ^= z >> 30; z *= 0xbf58476d1ce4e5b9ull;
  z ^= z >> 27; z *= 0x94d049bb133111ebull;
  z ^= z >> 31;
  return z;
}
RTLA_HD uint64_t mix_b(uint64_t z) {  // murmur3 fmix64 (independent constants)
  z ^= z >> 33; z *= 0xff51afd7ed558ccdull;
  z ^= z >> 33; z *= 0xc4ceb9fe1a85ec53ull;
  z ^= z >> 33;
  return z;
}
RTLA_HD FP fp_add(FP x, FP y) { return FP{x.a + y.a, x.b + y.b}; }
RTLA_HD FP fp_sub(FP x, FP y) { return FP{x.a - y.a, x.b - y.b}; }
RTLA_HD FP hash_u64(uint64_t tag, uint64_t x) {
  FP h;
  h.a = mix_a(mix_a(tag * 0x9E3779B97F4A7C15ull + 0x243f6a8885a308d3ull) ^ x);
  h.b = mix_b(mix_b(tag * 0xD1B54A32D192ED03ull + 0x13198a2e03707344ull) + x);
  return h;
}
template <class P>
RTLA_HD FP hash_words(uint64_t tag, P w, int n) {
  uint64_t a = mix_a(tag * 0x9E3779B97F4A7C15ull + 0x243f6a8885a308d3ull);
  uint64_t b = mix_b(tag * 0xD1B54A32D192ED03ull + 0x13198a2e03707344ull);
  for (int k = 0; k < n; k += 2) {
    uint64_t x = (uint64_t)w[k] | ((k + 1 < n) ? (uint64_t)w[k + 1] << 32 : 0ull);
    a = mix_a(a ^ x);
    b = mix_b(b + x);
  }
  return FP{a, b};
}
enum { TAG_SRV = 1, TAG_MSG = 2, TAG_ALL = 3, TAG_ELEC = 4 };
// First hash state of a record hashed at position p (run-time p < NS):
// hash_words' tag mixing of TAG_SRV << 8 | p, folded to constants.
template <int NS>
RTLA_HD FP srv_seed(int p) {
  FP s{0, 0};
#pragma unroll
  for (int k = 0; k < NS; k++) {
    const uint64_t tag = (uint64_t)(TAG_SRV << 8 | k);
    if (k == p) {
      s.a = mix_a(tag * 0x9E3779B97F4A7C15ull + 0x243f6a8885a308d3ull);
      s.b = mix_b(tag * 0xD1B54A32D192ED03ull + 0x13198a2e03707344ull);
    }
  }
  return s;
}
template <int N>
RTLA_HD FP hash_words_from(FP s, const uint32_t* w) {  // = hash_words(tag, w, N) given its seed s
#pragma unroll
  for (int k = 0; k < N; k += 2) {
    const uint64_t x = (uint64_t)w[k] | ((k + 1 < N) ? (uint64_t)w[k + 1] << 32 : 0ull);
    s.a = mix_a(s.a ^ x);
    s.b = mix_b(s.b + x);
  }
  return s;
}

// = hash_words(TAG_SRV << 8 | i, rec, SW), the tag's mixing folded to constants
RTLA_HD FP h_srv(int i, const uint32_t* rec, int SW) {
  FP s = srv_seed<NMAX>(i);
  for (int k = 0; k < SW; k += 2) {
    const uint64_t x = (uint64_t)rec[k] | ((k + 1 < SW) ? (uint64_t)rec[k + 1] << 32 : 0ull);
    s.a = mix_a(s.a ^ x);
    s.b = mix_b(s.b + x);
  }
  return s;
}
// A message with its count, as its PACKED slot value (msg_pack: a bijection of
// the model's message values, so the fingerprint stays a function of the
// state's value); 0 = empty slot.
RTLA_HD FP h_msg(uint64_t slot) { return slot ? hash_u64(TAG_MSG, slot) : FP{0, 0}; }
RTLA_HD FP h_all(int idx) { return hash_u64(TAG_ALL, (uint64_t)idx); }
RTLA_HD FP h_elec(const uint32_t* rec, int EW) { return hash_words(TAG_ELEC, rec, EW); }

// ------------------------------------------------------------ row I/O ----
// Bit fields of a packed row (widths <= 32; a field may straddle two words).
template <class P>
RTLA_HD uint32_t row_bits(P row, int word, int bit, int nbits) {
  if (nbits == 0) return 0u;
  const int w = word + (bit >> 5), s = bit & 31;
  uint64_t x = (uint64_t)row[w];
  if (s + nbits > 32) x |= (uint64_t)row[w + 1] << 32;
  return (uint32_t)(x >> s) & (uint32_t)((1ull << nbits) - 1ull);
}
// Packing into a record's words (out: zeroed, enough words).
RTLA_HD void put_bits(uint32_t* out, int bit, int nbits, uint32_t v) {
  if (nbits == 0) return;
  const int w = bit >> 5, s = bit & 31;
  const uint64_t x = (uint64_t)(v & (uint32_t)((1ull << nbits) - 1ull)) << s;
  out[w] |= (uint32_t)x;
  if (s + nbits > 32) out[w + 1] |= (uint32_t)(x >> 32);
}

// Logs: wide code <-> packed (length | entries, entry = term-1 | value << b_tm1).
RTLA_HD uint32_t log_pack(const Layout& L, uint32_t code, int lenbits) {
  const uint32_t n = log_len(code);
  uint32_t x = n;
  for (uint32_t k = 1; k <= n; k++)
    x |= ((log_term(code, k) - 1u) | log_val(code, k) << L.b_tm1) << (lenbits + (int)(k - 1) * L.b_ent);
  return x;
}
RTLA_HD uint32_t log_unpack(const Layout& L, uint32_t x, int lenbits) {
  const uint32_t n = lenbits ? x & ((1u << lenbits) - 1u) : 0u;
  uint32_t code = n;
  for (uint32_t k = 1; k <= n; k++) {
    const uint32_t e = (x >> (lenbits + (int)(k - 1) * L.b_ent)) & ((1u << L.b_ent) - 1u);
    const uint32_t term = (e & ((1u << L.b_tm1) - 1u)) + 1u, val = e >> L.b_tm1;
    code |= (term | val << 3) << (3 + 5 * (k - 1));
  }
  return code;
}
RTLA_HD int lenbits0(const Layout& L) { return L.b_log0 - L.L * L.b_ent; }
RTLA_HD int lenbits1(const Layout& L) { return L.b_log1 - (L.L + 1) * L.b_ent; }

// Server record i: the wide words from the packed row.
template <class P>
RTLA_HD uint32_t srv_w0(const Layout& L, P row, int i) {
  const int base = L.off_srv + i * L.srv_w;
  int b = 0;
  const uint32_t term = row_bits(row, base, b, L.b_tcur) + 1u; b += L.b_tcur;
  const uint32_t role = row_bits(row, base, b, 2); b += 2;
  uint32_t voted = row_bits(row, base, b, L.b_vote); b += L.b_vote;
  if (voted == (uint32_t)L.N) voted = NIL;
  const uint32_t commit = row_bits(row, base, b, L.b_idx); b += L.b_idx;
  const uint32_t masks = row_bits(row, base, b, 3 * L.N);
  const uint32_t m = (1u << L.N) - 1u;
  return s_make(term, role, voted, commit, masks & m, (masks >> L.N) & m, (masks >> (2 * L.N)) & m);
}
template <class P>
RTLA_HD uint32_t srv_log(const Layout& L, P row, int i) {
  return log_unpack(L, row_bits(row, L.off_srv + i * L.srv_w, L.sb_log, L.b_log1), lenbits1(L));
}
template <class P>
RTLA_HD uint32_t srv_nm(const Layout& L, P row, int i) {
  const int base = L.off_srv + i * L.srv_w;
  uint32_t nm = 0;
  for (int j = 0; j < L.N; j++) {
    const uint32_t x = row_bits(row, base, L.sb_nm + 2 * j * L.b_idx, 2 * L.b_idx);
    nm |= ((x & ((1u << L.b_idx) - 1u)) + 1u) << (3 * j) | (x >> L.b_idx) << (15 + 3 * j);
  }
  return nm;
}
template <class P>
RTLA_HD uint32_t srv_vl(const Layout& L, P row, int i, int j) {
  return log_unpack(L, row_bits(row, L.off_srv + i * L.srv_w, L.sb_vl + j * L.b_log0, L.b_log0), lenbits0(L));
}
// Packed words of a wide server record (out: srv_w words).
RTLA_HD void srv_pack(const Layout& L, const uint32_t* rec, uint32_t* out) {
  for (int w = 0; w < L.srv_w; w++) out[w] = 0;
  const uint32_t w0 = rec[0];
  int b = 0;
  put_bits(out, b, L.b_tcur, s_term(w0) - 1u); b += L.b_tcur;
  put_bits(out, b, 2, s_role(w0)); b += 2;
  put_bits(out, b, L.b_vote, s_voted(w0) == NIL ? (uint32_t)L.N : s_voted(w0)); b += L.b_vote;
  put_bits(out, b, L.b_idx, s_commit(w0)); b += L.b_idx;
  put_bits(out, b, 3 * L.N, s_vresp(w0) | s_vgrant(w0) << L.N | s_vlp(w0) << (2 * L.N));
  put_bits(out, L.sb_log, L.b_log1, log_pack(L, rec[1], lenbits1(L)));
  for (int j = 0; j < L.N; j++) {
    put_bits(out, L.sb_nm + 2 * j * L.b_idx, L.b_idx, nm_next(rec[2], j) - 1u);
    put_bits(out, L.sb_nm + (2 * j + 1) * L.b_idx, L.b_idx, nm_match(rec[2], j));
    put_bits(out, L.sb_vl + j * L.b_log0, L.b_log0, log_pack(L, rec[3 + j], lenbits0(L)));
  }
}

// Election record e: wide words from the packed row, and back.
template <class P>
RTLA_HD uint32_t elec_w0(const Layout& L, P row, int e) {
  const int base = L.off_elec + e * L.elec_w;
  const uint32_t x = row_bits(row, base, 0, L.b_tm1 + L.b_sid + 2 * L.N);
  const uint32_t term = (x & ((1u << L.b_tm1) - 1u)) + 1u;
  const uint32_t rest = x >> L.b_tm1;
  const uint32_t leader = rest & ((1u << L.b_sid) - 1u);
  const uint32_t masks = rest >> L.b_sid, m = (1u << L.N) - 1u;
  return term | leader << 4 | (masks & m) << 7 | ((masks >> L.N) & m) << 12;
}
template <class P>
RTLA_HD uint32_t elec_log(const Layout& L, P row, int e) {
  return log_unpack(L, row_bits(row, L.off_elec + e * L.elec_w, L.eb_log, L.b_log0), lenbits0(L));
}
template <class P>
RTLA_HD uint32_t elec_vl(const Layout& L, P row, int e, int j) {
  return log_unpack(L, row_bits(row, L.off_elec + e * L.elec_w, L.eb_vl + j * L.b_log0, L.b_log0), lenbits0(L));
}
RTLA_HD void elec_pack(const Layout& L, const uint32_t* er, uint32_t* out) {
  for (int w = 0; w < L.elec_w; w++) out[w] = 0;
  const uint32_t w0 = er[0];
  put_bits(out, 0, L.b_tm1, (w0 & 15u) - 1u);
  put_bits(out, L.b_tm1, L.b_sid, (w0 >> 4) & 7u);
  put_bits(out, L.b_tm1 + L.b_sid, 2 * L.N, ((w0 >> 7) & 31u) | ((w0 >> 12) & 31u) << L.N);
  put_bits(out, L.eb_log, L.b_log0, log_pack(L, er[1], lenbits0(L)));
  for (int j = 0; j < L.N; j++) put_bits(out, L.eb_vl + j * L.b_log0, L.b_log0, log_pack(L, er[2 + j], lenbits0(L)));
}

// Messages: wide value (key | count << 60) <-> packed slot (0 = empty).
RTLA_HD uint64_t msg_pack(const Layout& L, uint64_t v) {
  if (!v) return 0ull;
  uint32_t out[2] = {0u, 0u};
  const uint32_t type = m_type(v);
  put_bits(out, 0, 2, type);
  put_bits(out, 2, L.b_sid, m_src(v));
  put_bits(out, 2 + L.b_sid, L.b_sid, m_dst(v));
  put_bits(out, L.mb_term, L.b_tm1, m_term(v) - 1u);
  int b = L.mb_pay;
  if (type == RVREQ) {
    put_bits(out, b, L.b_t0, m_f(v, 12, 4)); b += L.b_t0;
    put_bits(out, b, L.b_idx, m_f(v, 16, 3));
  } else if (type == RVRESP) {
    put_bits(out, b, 1, m_f(v, 12, 1)); b += 1;
    put_bits(out, b, L.b_log0, log_pack(L, m_f(v, 16, 28), lenbits0(L)));
  } else if (type == AEREQ) {
    put_bits(out, b, L.b_idx, m_f(v, 12, 3)); b += L.b_idx;
    put_bits(out, b, L.b_t0, m_f(v, 15, 4)); b += L.b_t0;
    const uint32_t has = m_f(v, 19, 1), ent = m_f(v, 20, 5);
    put_bits(out, b, 1, has); b += 1;
    put_bits(out, b, L.b_ent, has ? ((ent & 7u) - 1u) | (ent >> 3) << L.b_tm1 : 0u); b += L.b_ent;
    put_bits(out, b, L.b_idx, m_f(v, 25, 3)); b += L.b_idx;
    put_bits(out, b, L.b_log0, log_pack(L, m_f(v, 28, 28), lenbits0(L)));
  } else {
    put_bits(out, b, 1, m_f(v, 12, 1)); b += 1;
    put_bits(out, b, L.b_idx, m_f(v, 13, 3));
  }
  put_bits(out, L.mb_cnt, L.b_cnt, m_count(v));
  return (uint64_t)out[0] | (uint64_t)out[1] << 32;
}
RTLA_HD uint64_t msg_unpack(const Layout& L, uint64_t x) {
  if (!x) return 0ull;
  const uint32_t p[2] = {(uint32_t)x, (uint32_t)(x >> 32)};
  const uint32_t type = row_bits(p, 0, 0, 2);
  const uint32_t src = row_bits(p, 0, 2, L.b_sid), dst = row_bits(p, 0, 2 + L.b_sid, L.b_sid);
  const uint32_t term = row_bits(p, 0, L.mb_term, L.b_tm1) + 1u;
  int b = L.mb_pay;
  uint64_t key;
  if (type == RVREQ) {
    const uint32_t llt = row_bits(p, 0, b, L.b_t0);
    key = m_rvreq(src, dst, term, llt, row_bits(p, 0, b + L.b_t0, L.b_idx));
  } else if (type == RVRESP) {
    key = m_rvresp(src, dst, term, row_bits(p, 0, b, 1), log_unpack(L, row_bits(p, 0, b + 1, L.b_log0), lenbits0(L)));
  } else if (type == AEREQ) {
    const uint32_t prev = row_bits(p, 0, b, L.b_idx); b += L.b_idx;
    const uint32_t prevt = row_bits(p, 0, b, L.b_t0); b += L.b_t0;
    const uint32_t has = row_bits(p, 0, b, 1); b += 1;
    const uint32_t e = row_bits(p, 0, b, L.b_ent); b += L.b_ent;
    const uint32_t ent = has ? ((e & ((1u << L.b_tm1) - 1u)) + 1u) | (e >> L.b_tm1) << 3 : 0u;
    const uint32_t commit = row_bits(p, 0, b, L.b_idx); b += L.b_idx;
    key = m_aereq(src, dst, term, prev, prevt, has, ent, commit, log_unpack(L, row_bits(p, 0, b, L.b_log0), lenbits0(L)));
  } else {
    key = m_aeresp(src, dst, term, row_bits(p, 0, b, 1), row_bits(p, 0, b + 1, L.b_idx));
  }
  return key | (uint64_t)row_bits(p, 0, L.mb_cnt, L.b_cnt) << 60;
}
// Bag slot k: packed (slot_raw) or wide (bag_slot).  Lookups compare packed
// keys (key_raw: the key packed with its count bits cleared) so that only a
// found message is ever unpacked.
template <class P>
RTLA_HD uint64_t slot_raw(const Layout& L, P row, int k) {
  const int w = L.off_bag + k * L.slot_w;
  return L.slot_w == 1 ? (uint64_t)row[w] : (uint64_t)row[w] | (uint64_t)row[w + 1] << 32;
}
template <class P>
RTLA_HD uint64_t bag_slot(const Layout& L, P row, int k) { return msg_unpack(L, slot_raw(L, row, k)); }
RTLA_HD uint64_t slot_keymask(const Layout& L) { return (1ull << L.mb_cnt) - 1ull; }
RTLA_HD uint64_t key_raw(const Layout& L, uint64_t key) { return msg_pack(L, key | 1ull << 60) & slot_keymask(L); }
RTLA_HD uint32_t raw_count(const Layout& L, uint64_t x) {
  return (uint32_t)(x >> L.mb_cnt) & ((1u << L.b_cnt) - 1u);
}
template <class P>
RTLA_HD uint32_t slot_type(const Layout& L, P row, int k) { return row[L.off_bag + k * L.slot_w] & 3u; }
template <class P>
RTLA_HD int row_nmsg(const Layout& L, P row) { return (int)(row[L.off_hdr] & 255u); }
template <class P>
RTLA_HD int row_nelec(const Layout& L, P row) { return (int)((row[L.off_hdr] >> 8) & 255u); }
template <class P>
RTLA_HD FP row_fp(P row) {
  return FP{(uint64_t)row[0] | (uint64_t)row[1] << 32, (uint64_t)row[2] | (uint64_t)row[3] << 32};
}
template <class P>
RTLA_HD void row_set_fp(P row, FP f) {
  row[0] = (uint32_t)f.a; row[1] = (uint32_t)(f.a >> 32);
  row[2] = (uint32_t)f.b; row[3] = (uint32_t)(f.b >> 32);
}

// Whole records in and out of a row (host-side builders: Init, permutations,
// synthetic states; the kernels patch rows through child_patches).
template <class P>
RTLA_HD void srv_get(const Layout& L, P row, int i, uint32_t* rec) {
  rec[0] = srv_w0(L, row, i);
  rec[1] = srv_log(L, row, i);
  rec[2] = srv_nm(L, row, i);
  for (int j = 0; j < L.N; j++) rec[3 + j] = srv_vl(L, row, i, j);
}
template <class P>
RTLA_HD void srv_put(const Layout& L, P row, int i, const uint32_t* rec) {
  uint32_t out[8];
  srv_pack(L, rec, out);
  for (int w = 0; w < L.srv_w; w++) row[L.off_srv + i * L.srv_w + w] = out[w];
}
template <class P>
RTLA_HD void elec_get(const Layout& L, P row, int e, uint32_t* er) {
  er[0] = elec_w0(L, row, e);
  er[1] = elec_log(L, row, e);
  for (int j = 0; j < L.N; j++) er[2 + j] = elec_vl(L, row, e, j);
}
template <class P>
RTLA_HD void elec_put(const Layout& L, P row, int e, const uint32_t* er) {
  uint32_t out[8];
  elec_pack(L, er, out);
  for (int w = 0; w < L.elec_w; w++) row[L.off_elec + e * L.elec_w + w] = out[w];
}
template <class P>
RTLA_HD void slot_put(const Layout& L, P row, int k, uint64_t v) {
  const uint64_t x = msg_pack(L, v);
  row[L.off_bag + k * L.slot_w] = (uint32_t)x;
  if (L.slot_w > 1) row[L.off_bag + k * L.slot_w + 1] = (uint32_t)(x >> 32);
}

// Full fingerprint of a row, from scratch (Init, checks).
template <class P>
RTLA_HD FP row_fingerprint(const Layout& L, P row) {
  FP f{0, 0};
  uint32_t rec[3 + NMAX];
  for (int i = 0; i < L.N; i++) {
    srv_get(L, row, i, rec);
    f = fp_add(f, h_srv(i, rec, L.SW));
  }
  int nm = row_nmsg(L, row);
  for (int k = 0; k < nm; k++) f = fp_add(f, h_msg(slot_raw(L, row, k)));
  for (int x = 0; x < L.n_logs; x++)
    if (row[L.off_all + (x >> 5)] >> (x & 31) & 1u) f = fp_add(f, h_all(x));
  int ne = row_nelec(L, row);
  uint32_t er[2 + NMAX];
  for (int e = 0; e < ne; e++) {
    elec_get(L, row, e, er);
    f = fp_add(f, h_elec(er, L.EW));
  }
  return f;
}

// Init (raft.tla:140-160): exactly one state.
template <class P>
RTLA_HD void row_init(const Layout& L, P row) {
  for (int w = 0; w < L.W; w++) row[w] = 0;
  for (int i = 0; i < L.N; i++) {
    uint32_t rec[3 + NMAX] = {0};
    rec[0] = s_make(1, FOLLOWER, NIL, 0, 0, 0, 0);  // :143-147
    rec[1] = 0;                                     // log = <<>> :153
    rec[2] = nm_fill(L.N, 1, 0);                    // :151-152
    srv_put(L, row, i, rec);
  }
  row_set_fp(row, row_fingerprint(L, row));
}

// --------------------------------------------------------------- delta ----
// The successor of one action instance, as a patch of the parent row.
//
// Every function below takes the server count as a template parameter NS
// (0 = read it from the Layout at run time: host-side decoding).  With NS
// fixed the loops over servers unroll and every array in Delta is indexed
// with compile-time constants, so the whole Delta stays in VGPRs on the GPU
// (no scratch); writes at a run-time index go through set_at().
// NR: servers the record arrays are sized for (NS in the kernels, NMAX on the host).
template <int NR = NMAX>
struct DeltaT {
  int32_t enabled;
  int32_t in_model;
  int32_t sub;             // Receive sub-action (R_*) or R_NONE
  int32_t err;             // 1: spec evaluation error, 2: row capacity overflow
  int32_t srv;             // server whose record changes, -1 = none
  uint32_t rec[3 + NR];    // its new record
  int32_t nops;            // bag slot writes (<= 3)
  int32_t op_slot[3];
  uint64_t op_old[3], op_new[3];  // PACKED slot values (msg_pack; 0 = empty)
  int32_t nmsg;            // new number of bag slots in use
  int32_t elec;            // 1: append erec to elections
  uint32_t erec[2 + NR];
};
using Delta = DeltaT<NMAX>;

#define RTLA_NSRV(L) (NS ? NS : (L).N)

// a[j] = v for a run-time j, as a chain of selects (keeps `a` in registers)
template <int CAP, class T>
RTLA_HD void set_at(T* a, int j, T v) {
#pragma unroll
  for (int k = 0; k < CAP; k++)
    if (k == j) a[k] = v;
}

// DeltaT's bag: slot writes over the parent's slots, all in PACKED form.
template <class P, int NR>
RTLA_HD uint64_t bag_get(const Layout& L, P row, const DeltaT<NR>& d, int slot) {
  uint64_t v = slot_raw(L, row, slot);
#pragma unroll
  for (int q = 0; q < 3; q++)
    if (q < d.nops && d.op_slot[q] == slot) v = d.op_new[q];
  return v;
}
template <class P, int NR>
RTLA_HD void bag_set(const Layout& L, P row, DeltaT<NR>& d, int slot, uint64_t v) {
  bool done = false;
#pragma unroll
  for (int q = 0; q < 3; q++)
    if (!done && q < d.nops && d.op_slot[q] == slot) { d.op_new[q] = v; done = true; }
  if (done) return;
  if (d.nops >= 3) { d.err = 2; return; }
  const uint64_t old = slot_raw(L, row, slot);
#pragma unroll
  for (int q = 0; q < 3; q++)
    if (q == d.nops) { d.op_slot[q] = slot; d.op_old[q] = old; d.op_new[q] = v; }
  d.nops++;
}
// slot holding packed key pk (count bits cleared), or -1
template <class P, int NR>
RTLA_HD int bag_find(const Layout& L, P row, const DeltaT<NR>& d, uint64_t pk) {
  const uint64_t km = slot_keymask(L);
  int hit = -1;
  for (int k = 0; k < d.nmsg; k++) {
    const uint64_t x = bag_get(L, row, d, k);
    if (hit < 0 && x != 0 && (x & km) == pk) hit = k;
  }
  return hit;
}
RTLA_HD uint64_t count_one(const Layout& L) { return 1ull << L.mb_cnt; }
// raft.tla:106-110 WithMessage
template <class P, int NR>
RTLA_HD void with_message(const Layout& L, P row, DeltaT<NR>& d, uint64_t key) {
  const uint64_t pk = key_raw(L, key);
  int p = bag_find(L, row, d, pk);
  if (p >= 0) {
    bag_set(L, row, d, p, bag_get(L, row, d, p) + count_one(L));
  } else {
    if (d.nmsg >= L.K) { d.err = 2; return; }
    bag_set(L, row, d, d.nmsg, pk | count_one(L));
    d.nmsg++;
  }
}
// raft.tla:114-119 WithoutMessage, of the message in slot p
template <class P, int NR>
RTLA_HD void without_slot(const Layout& L, P row, DeltaT<NR>& d, int p) {
  const uint64_t v = bag_get(L, row, d, p);
  if (raw_count(L, v) <= 1) {
    int last = d.nmsg - 1;
    if (p != last) bag_set(L, row, d, p, bag_get(L, row, d, last));
    bag_set(L, row, d, last, 0);
    d.nmsg--;
  } else {
    bag_set(L, row, d, p, v - count_one(L));
  }
}
template <class P, int NR>
RTLA_HD void without_message(const Layout& L, P row, DeltaT<NR>& d, uint64_t key) {
  const int p = bag_find(L, row, d, key_raw(L, key));
  if (p >= 0) without_slot(L, row, d, p);
}

// Fingerprint-only sink for compute_delta (the BFS probe pass).  The same
// action code runs against it, but bag updates are folded straight into the
// change of the message-multiset hash instead of being recorded as slot
// writes: the fingerprint is order-free, so only (key, old count, new count)
// matters.  Every action touches at most two distinct message keys, and the
// two keys of Reply (raft.tla:129-130) always differ in type, so each op can
// look its key up in the PARENT bag.
template <int NR = NMAX>
struct DeltaFpT {
  int32_t enabled;
  int32_t in_model;
  int32_t sub;
  int32_t err;
  int32_t srv;
  uint32_t rec[3 + NR];
  int32_t nmsg;            // new number of bag slots in use
  int32_t nmsg0;           // parent's
  int32_t dcount;          // change of BagCardinality(messages)
  int32_t elec;
  uint32_t erec[2 + NR];
  FP fmsg;                 // change of the message-multiset hash
};
using DeltaFp = DeltaFpT<NMAX>;

// Slot of packed key pk among the first n (parent) slots, its count in *count.
template <class P>
RTLA_HD int bag_find0(const Layout& L, P row, int n, uint64_t pk, uint32_t* count) {
  const uint64_t km = slot_keymask(L);
  int hit = -1;
  uint32_t c = 0;
  for (int k = 0; k < n; k++) {
    const uint64_t x = slot_raw(L, row, k);
    if (hit < 0 && x != 0 && (x & km) == pk) { hit = k; c = raw_count(L, x); }
  }
  *count = c;
  return hit;
}
// count c -> c + dc of the message with packed key pk (c = 0: absent), for the probe pass
template <int NR>
RTLA_HD void fp_bag_count(const Layout& L, DeltaFpT<NR>& d, uint64_t pk, uint32_t c, int dc) {
  const uint32_t n = (uint32_t)((int)c + dc);
  if ((int)n > L.C) d.in_model = 0;
  d.dcount += dc;
  if (c) d.fmsg = fp_sub(d.fmsg, h_msg(pk | (uint64_t)c << L.mb_cnt));
  if (n) d.fmsg = fp_add(d.fmsg, h_msg(pk | (uint64_t)n << L.mb_cnt));
}
template <class P, int NR>
RTLA_HD void with_message(const Layout& L, P row, DeltaFpT<NR>& d, uint64_t key) {  // raft.tla:106-110
  const uint64_t pk = key_raw(L, key);
  uint32_t c;
  if (bag_find0(L, row, d.nmsg0, pk, &c) >= 0) {
    fp_bag_count(L, d, pk, c, 1);
  } else {
    if (d.nmsg >= L.K) { d.err = 2; return; }
    d.nmsg++;
    fp_bag_count(L, d, pk, 0, 1);
  }
}
template <class P, int NR>
RTLA_HD void without_slot(const Layout& L, P row, DeltaFpT<NR>& d, int x) {  // raft.tla:114-119, slot x
  const uint64_t v = slot_raw(L, row, x);
  const uint32_t c = raw_count(L, v);
  if (c <= 1) d.nmsg--;
  fp_bag_count(L, d, v & slot_keymask(L), c, -1);
}
template <class P, int NR>
RTLA_HD void without_message(const Layout& L, P row, DeltaFpT<NR>& d, uint64_t key) {  // raft.tla:114-119
  const uint64_t pk = key_raw(L, key);
  uint32_t c;
  const int x = bag_find0(L, row, d.nmsg0, pk, &c);
  if (x < 0) return;
  if (c <= 1) d.nmsg--;
  fp_bag_count(L, d, pk, c, -1);
}
template <class P, int NR>
RTLA_HD void bag_dup_slot(const Layout& L, P row, DeltaFpT<NR>& d, int x) {  // DuplicateMessage :443-445
  const uint64_t v = slot_raw(L, row, x);
  fp_bag_count(L, d, v & slot_keymask(L), raw_count(L, v), 1);
}
template <class P, int NR>
RTLA_HD void bag_dup_slot(const Layout& L, P row, DeltaT<NR>& d, int x) {
  bag_set(L, row, d, x, slot_raw(L, row, x) + count_one(L));
}
template <int NR>
RTLA_HD void delta_reset(DeltaT<NR>& d) { d.nops = 0; }
template <int NR>
RTLA_HD void delta_reset(DeltaFpT<NR>& d) {
  d.nmsg0 = d.nmsg; d.dcount = 0; d.fmsg = FP{0, 0};
}
// message part of the state constraint (specs/MC.tla StateConstraint)
template <class P, int NR>
RTLA_HD void bag_constraint(const Layout& L, P row, DeltaT<NR>& d) {
  if (!d.nops) return;
  int total_delta = 0;
#pragma unroll
  for (int q = 0; q < 3; q++) {
    if (q < d.nops) {
      if ((int)raw_count(L, d.op_new[q]) > L.C) d.in_model = 0;
      total_delta += (int)raw_count(L, d.op_new[q]) - (int)raw_count(L, d.op_old[q]);
    }
  }
  if (L.M > 0 && total_delta > 0) {
    int total = 0;
    const int nm = row_nmsg(L, row);
    for (int k = 0; k < nm; k++) total += (int)raw_count(L, slot_raw(L, row, k));
    if (total + total_delta > L.M) d.in_model = 0;
  }
}
template <class P, int NR>
RTLA_HD void bag_constraint(const Layout& L, P row, DeltaFpT<NR>& d) {
  if (L.M > 0 && d.dcount > 0) {
    int total = 0;
    for (int k = 0; k < d.nmsg0; k++) total += (int)raw_count(L, slot_raw(L, row, k));
    if (total + d.dcount > L.M) d.in_model = 0;
  }
}

template <int NS, class P>
RTLA_HD void load_rec(const Layout& L, P row, int i, uint32_t* rec) {
  rec[0] = srv_w0(L, row, i);
  rec[1] = srv_log(L, row, i);
  rec[2] = srv_nm(L, row, i);
#pragma unroll
  for (int j = 0; j < (NS ? NS : NMAX); j++)
    if (j < RTLA_NSRV(L)) rec[3 + j] = srv_vl(L, row, i, j);
}

// Compute the successor of `row` under action instance `inst` (0..L.fam[F_COUNT]).
// Follows raft.tla:454-463; allLogs' (:465) is applied per parent by the caller.
// FAM >= 0: the caller guarantees inst belongs to that family (GPU chunks of
// one family); the dispatch below then folds away at compile time.
template <int NS, int FAM = -1, class P, class D>
RTLA_HD void compute_delta(const Layout& L, P row, int inst, D& d) {
  const int N = RTLA_NSRV(L);
  d.enabled = 0; d.in_model = 1; d.sub = R_NONE; d.err = 0; d.srv = -1;
  d.nmsg = row_nmsg(L, row); d.elec = 0;
  delta_reset(d);
  int fam = FAM;
  if (FAM < 0) {
    fam = 0;
#pragma unroll
    for (int f = 1; f < F_COUNT; f++) fam += inst >= L.fam[f];
  }
  const int x = inst - (FAM >= 0 ? L.fam[FAM >= 0 ? FAM : 0] : fam_base(L, fam));
  uint32_t* rec = d.rec;

  if (fam == F_RESTART) {                       // Restart(i) :167-175
    const int i = x;
    load_rec<NS>(L, row, i, rec);
    rec[0] = s_make(s_term(rec[0]), FOLLOWER, s_voted(rec[0]), 0, 0, 0, 0);
    rec[2] = nm_fill(N, 1, 0);
#pragma unroll
    for (int j = 0; j < (NS ? NS : NMAX); j++) rec[3 + j] = 0;
    d.srv = i; d.enabled = 1;
  } else if (fam == F_TIMEOUT) {                // Timeout(i) :178-187
    const int i = x;
    load_rec<NS>(L, row, i, rec);
    const uint32_t role = s_role(rec[0]);
    if (role != FOLLOWER && role != CANDIDATE) return;
    const uint32_t t = s_term(rec[0]) + 1;
    rec[0] = s_make(t, CANDIDATE, NIL, s_commit(rec[0]), 0, 0, 0);
#pragma unroll
    for (int j = 0; j < (NS ? NS : NMAX); j++) rec[3 + j] = 0;
    d.srv = i; d.enabled = 1;
    if ((int)t > L.T) d.in_model = 0;
  } else if (fam == F_REQUESTVOTE) {            // RequestVote(i, j) :190-199
    const int i = x / N, j = x - (x / N) * N;
    const uint32_t w0 = srv_w0(L, row, i);
    if (s_role(w0) != CANDIDATE || (s_vresp(w0) >> j & 1u)) return;
    const uint32_t lg = srv_log(L, row, i);
    with_message(L, row, d, m_rvreq(i, j, s_term(w0), last_term(lg), log_len(lg)));
    d.enabled = 1;
  } else if (fam == F_BECOMELEADER) {           // BecomeLeader(i) :229-243
    const int i = x;
    load_rec<NS>(L, row, i, rec);
    const uint32_t w0 = rec[0];
    if (s_role(w0) != CANDIDATE) return;
    if (!(__builtin_popcount(s_vgrant(w0)) * 2 > N)) return;   // votesGranted[i] \in Quorum :99
    d.enabled = 1; d.srv = i;
    rec[0] = (w0 & ~(3u << 4)) | (LEADER << 4);
    rec[2] = nm_fill(N, log_len(rec[1]) + 1, 0);
    // elections' = elections \cup {[eterm, eleader, elog, evotes, evoterLog]}
    d.erec[0] = s_term(w0) | (uint32_t)i << 4 | s_vgrant(w0) << 7 | s_vlp(w0) << 12;
    d.erec[1] = rec[1];
#pragma unroll
    for (int j = 0; j < (NS ? NS : NMAX); j++) d.erec[2 + j] = j < N ? rec[3 + j] : 0u;
    const int ne = row_nelec(L, row);
    uint32_t pk[8];  // the record packed: equal records have equal packed words
    elec_pack(L, d.erec, pk);
    int dup = 0;
    for (int e = 0; e < ne; e++) {
      int same = 1;
      for (int w = 0; w < L.elec_w; w++) same &= row[L.off_elec + e * L.elec_w + w] == pk[w];
      dup |= same;
    }
    if (!dup) {
      if (ne >= L.E) { d.err = 2; return; }
      d.elec = 1;
    }
  } else if (fam == F_CLIENTREQUEST) {          // ClientRequest(i, v) :246-253
    const int i = x / L.V, v = x - (x / L.V) * L.V;
    load_rec<NS>(L, row, i, rec);
    if (s_role(rec[0]) != LEADER) return;
    if (log_len(rec[1]) >= (uint32_t)LMAX + 1) { d.err = 2; return; }
    rec[1] = log_append(rec[1], s_term(rec[0]) | (uint32_t)v << 3);
    d.srv = i; d.enabled = 1;
    if ((int)log_len(rec[1]) > L.L) d.in_model = 0;
  } else if (fam == F_ADVANCECOMMIT) {          // AdvanceCommitIndex(i) :259-276
    const int i = x;
    load_rec<NS>(L, row, i, rec);
    if (s_role(rec[0]) != LEADER) return;
    const int len = (int)log_len(rec[1]);
    int maxagree = 0;
    for (int index = 1; index <= len; index++) {
      int agree = 1;                            // Agree(index) = {i} \cup {k : matchIndex[i][k] >= index}
#pragma unroll
      for (int k = 0; k < (NS ? NS : NMAX); k++)
        agree += (k < N) && (k != i) && (int)nm_match(rec[2], k) >= index;
      if (agree * 2 > N) maxagree = index;
    }
    uint32_t nci = s_commit(rec[0]);
    if (maxagree > 0 && log_term(rec[1], maxagree) == s_term(rec[0])) nci = (uint32_t)maxagree;
    rec[0] = (rec[0] & ~(7u << 9)) | nci << 9;
    d.srv = i; d.enabled = 1;
  } else if (fam == F_APPENDENTRIES) {          // AppendEntries(i, j) :204-226
    const int i = x / N, j = x - (x / N) * N;
    if (i == j) return;
    const uint32_t w0 = srv_w0(L, row, i);
    if (s_role(w0) != LEADER) return;
    const uint32_t lg = srv_log(L, row, i), nm = srv_nm(L, row, i);
    const uint32_t nxt = nm_next(nm, j), prev = nxt - 1, len = log_len(lg);
    uint32_t prevt = 0;
    if (prev > 0) {
      if (prev > len) { d.err = 1; return; }   // log[i][prevLogIndex] outside DOMAIN
      prevt = log_term(lg, prev);
    }
    const uint32_t last = len < nxt ? len : nxt;   // Min({Len(log[i]), nextIndex[i][j]})
    const uint32_t has = nxt <= last ? 1u : 0u;     // SubSeq(log[i], next, lastEntry)
    const uint32_t entry = has ? log_entry(lg, nxt) : 0u;
    const uint32_t ci = s_commit(w0);
    const uint32_t mci = ci < last ? ci : last;
    with_message(L, row, d, m_aereq(i, j, s_term(w0), prev, prevt, has, entry, mci, lg));
    d.enabled = 1;
  } else if (fam == F_RECEIVE) {                // Receive(m) :421-436
    if (x >= d.nmsg) return;
    const uint64_t key = m_key(bag_slot(L, row, x));
    const int i = (int)m_dst(key), j = (int)m_src(key);
    const uint32_t mt = m_term(key), type = m_type(key);
    load_rec<NS>(L, row, i, rec);
    const uint32_t cur = s_term(rec[0]), role = s_role(rec[0]);
    if (mt > cur) {                              // UpdateTerm :406-412 (message kept)
      rec[0] = s_make(mt, FOLLOWER, NIL, s_commit(rec[0]), s_vresp(rec[0]), s_vgrant(rec[0]), s_vlp(rec[0]));
      d.srv = i; d.enabled = 1; d.sub = R_UPDATETERM;
      return;
    }
    const uint32_t lg = rec[1], len = log_len(lg);
    if (type == RVREQ) {                         // HandleRequestVoteRequest :284-303
      const uint32_t llt = m_f(key, 12, 4), lli = m_f(key, 16, 3), lt = last_term(lg);
      const int logok = llt > lt || (llt == lt && lli >= len);
      const uint32_t vf = s_voted(rec[0]);
      const int grant = mt == cur && logok && (vf == NIL || vf == (uint32_t)j);
      if (grant) {
        rec[0] = (rec[0] & ~(7u << 6)) | (uint32_t)j << 6;
        d.srv = i;
      }
      with_message(L, row, d, m_rvresp(i, j, cur, grant ? 1u : 0u, lg));  // Reply :129-130
      without_slot(L, row, d, x);
      d.enabled = 1; d.sub = R_HRVREQ;
    } else if (type == RVRESP || type == AERESP) {
      if (mt < cur) {                            // DropStaleResponse :415-418
        without_slot(L, row, d, x);
        d.enabled = 1; d.sub = R_DROPSTALE;
      } else if (type == RVRESP) {               // HandleRequestVoteResponse :307-321
        uint32_t vr = s_vresp(rec[0]) | 1u << j, vg = s_vgrant(rec[0]), vlp = s_vlp(rec[0]);
        if (m_f(key, 12, 1)) {
          vg |= 1u << j;
          if (!(vlp >> j & 1u)) {                // voterLog[i] @@ (j :> m.mlog): left wins
            vlp |= 1u << j;
            set_at<NS ? NS : NMAX>(rec + 3, j, m_f(key, 16, 28));
          }
        }
        rec[0] = s_make(cur, role, s_voted(rec[0]), s_commit(rec[0]), vr, vg, vlp);
        without_slot(L, row, d, x);
        d.srv = i; d.enabled = 1; d.sub = R_HRVRESP;
      } else {                                   // HandleAppendEntriesResponse :393-403
        const uint32_t succ = m_f(key, 12, 1), mm = m_f(key, 13, 3);
        if (succ) {
          rec[2] = nm_set_match(nm_set_next(rec[2], j, mm + 1), j, mm);
        } else {
          const uint32_t nx = nm_next(rec[2], j);
          rec[2] = nm_set_next(rec[2], j, nx > 2 ? nx - 1 : 1);   // Max({next - 1, 1})
        }
        without_slot(L, row, d, x);
        d.srv = i; d.enabled = 1; d.sub = R_HAERESP;
      }
    } else {                                     // HandleAppendEntriesRequest :327-389
      const uint32_t prev = m_f(key, 12, 3), prevt = m_f(key, 15, 4), has = m_f(key, 19, 1);
      const uint32_t entry = m_f(key, 20, 5), mci = m_f(key, 25, 3);
      const int logok = prev == 0 || (prev > 0 && prev <= len && prevt == log_term(lg, prev));
      if (mt < cur || (mt == cur && role == FOLLOWER && !logok)) {   // reject :333-345
        with_message(L, row, d, m_aeresp(i, j, cur, 0, 0));
        without_slot(L, row, d, x);
        d.enabled = 1; d.sub = R_HAEREQ;
      } else if (mt == cur && role == CANDIDATE) {                  // return to follower :346-350
        rec[0] = (rec[0] & ~(3u << 4)) | (FOLLOWER << 4);
        d.srv = i; d.enabled = 1; d.sub = R_HAEREQ;
      } else if (mt == cur && role == FOLLOWER && logok) {          // accept :351-388
        const uint32_t index = prev + 1;
        if (!has || (len >= index && log_term(lg, index) == (entry & 7u))) {  // already done :356-374
          rec[0] = (rec[0] & ~(7u << 9)) | mci << 9;
          d.srv = i;
          with_message(L, row, d, m_aeresp(i, j, cur, 1, prev + has));
          without_slot(L, row, d, x);
          d.enabled = 1; d.sub = R_HAEREQ;
        } else if (len >= index) {               // conflict: remove 1 entry :375-382
          rec[1] = log_prefix(lg, len - 1);
          d.srv = i; d.enabled = 1; d.sub = R_HAEREQ;
        } else if (len == prev) {                // no conflict: append entry :383-388
          rec[1] = log_append(lg, entry);
          d.srv = i; d.enabled = 1; d.sub = R_HAEREQ;
        }
      }
      // AEReq with mterm = currentTerm at a Leader: no disjunct enabled.
    }
  } else if (fam == F_DUPLICATE) {              // DuplicateMessage(m) :443-445
    if (x >= d.nmsg) return;
    bag_dup_slot(L, row, d, x);
    d.enabled = 1;
  } else {                                      // DropMessage(m) :448-450
    if (x >= d.nmsg) return;
    without_slot(L, row, d, x);
    d.enabled = 1;
  }
  if (!d.enabled) return;
  // State constraint (specs/MC.tla) on the changed components.
  if (d.srv >= 0) {
    if ((int)s_term(d.rec[0]) > L.T || (int)log_len(d.rec[1]) > L.L) d.in_model = 0;
  }
  bag_constraint(L, row, d);
}

// Fingerprint change of the delta (allLogs change excluded: per parent).
// `h_old_srv` (optional) = the parent's h_srv of server d.srv, precomputed.
template <int NS, class P, int NR>
RTLA_HD FP delta_fp(const Layout& L, P row, const DeltaT<NR>& d, const FP* h_old_srv = nullptr) {
  const int SW = 3 + RTLA_NSRV(L);
  FP f{0, 0};
  if (d.srv >= 0) {
    FP old;
    if (h_old_srv) {
      old = *h_old_srv;
    } else {
      uint32_t orec[3 + NMAX];
      load_rec<NS>(L, row, d.srv, orec);
      old = h_srv(d.srv, orec, SW);
    }
    f = fp_sub(h_srv(d.srv, d.rec, SW), old);
  }
#pragma unroll
  for (int q = 0; q < 3; q++)
    if (q < d.nops) f = fp_add(f, fp_sub(h_msg(d.op_new[q]), h_msg(d.op_old[q])));
  if (d.elec) f = fp_add(f, h_elec(d.erec, 2 + RTLA_NSRV(L)));
  return f;
}

template <int NS, class P, int NR>
RTLA_HD FP delta_fp(const Layout& L, P row, const DeltaFpT<NR>& d, const FP* h_old_srv = nullptr) {
  const int SW = 3 + RTLA_NSRV(L);
  FP f = d.fmsg;
  if (d.srv >= 0) {
    FP old;
    if (h_old_srv) {
      old = *h_old_srv;
    } else {
      uint32_t orec[3 + NMAX];
      load_rec<NS>(L, row, d.srv, orec);
      old = h_srv(d.srv, orec, SW);
    }
    f = fp_add(f, fp_sub(h_srv(d.srv, d.rec, SW), old));
  }
  if (d.elec) f = fp_add(f, h_elec(d.erec, 2 + RTLA_NSRV(L)));
  return f;
}

// allLogs' = allLogs \cup {log[i] : i \in Server}   (pre-state logs, raft.tla:465)
// Writes the new allLogs words into all_out and returns the fingerprint change.
template <int NS, class P, class Q>
RTLA_HD FP alllogs_delta(const Layout& L, P row, Q all_out) {
  const int N = RTLA_NSRV(L);
  FP f{0, 0};
  for (int w = 0; w < L.all_words; w++) all_out[w] = row[L.off_all + w];
  for (int i = 0; i < N; i++) {
    const int x = log_index(L, srv_log(L, row, i));
    const uint32_t bit = 1u << (x & 31);
    if (!(all_out[x >> 5] & bit)) {
      all_out[x >> 5] |= bit;
      f = fp_add(f, h_all(x));
    }
  }
  return f;
}

// The words in which the successor row (parent + delta, with the new allLogs
// words and fingerprint) differs from its parent row, as put(word, value)
// calls; every other word of the child equals the parent's.  At most
// 4 + 1 + srv_w + all_words + elec_w + 3 * slot_w words.  In two steps:
// child_pack packs the delta's changed records (after which the wide
// records are dead: the kernels pack before they wait for the parent-row
// copies, and keep only the packed words across the wait), child_write
// emits the words.
constexpr int PACKW = 6;  // words of a packed server / election record, at most (make_layout)
template <int NR>
RTLA_HD void child_pack(const Layout& L, const DeltaT<NR>& d, uint32_t* spk, uint32_t* epk) {
  if (d.srv >= 0) srv_pack(L, d.rec, spk);
  if (d.elec) elec_pack(L, d.erec, epk);
}
template <class P, class R, class F, int NR>
RTLA_HD void child_write(const Layout& L, P row, const DeltaT<NR>& d, const uint32_t* spk, const uint32_t* epk,
                         R all_new, FP fp, F put) {
  put(0, (uint32_t)fp.a);
  put(1, (uint32_t)(fp.a >> 32));
  put(2, (uint32_t)fp.b);
  put(3, (uint32_t)(fp.b >> 32));
  const int ne = row_nelec(L, row) + (d.elec ? 1 : 0);
  put(L.off_hdr, (uint32_t)d.nmsg | (uint32_t)ne << 8);
  if (d.srv >= 0)
    for (int w = 0; w < L.srv_w; w++) put(L.off_srv + d.srv * L.srv_w + w, spk[w]);
  for (int w = 0; w < L.all_words; w++) put(L.off_all + w, all_new[w]);
  if (d.elec)
    for (int w = 0; w < L.elec_w; w++) put(L.off_elec + (ne - 1) * L.elec_w + w, epk[w]);
#pragma unroll
  for (int q = 0; q < 3; q++) {
    if (q < d.nops) {
      const uint64_t x = d.op_new[q];  // packed
      put(L.off_bag + d.op_slot[q] * L.slot_w, (uint32_t)x);
      if (L.slot_w > 1) put(L.off_bag + d.op_slot[q] * L.slot_w + 1, (uint32_t)(x >> 32));
    }
  }
}
template <int NS, class P, class R, class F, int NR>
RTLA_HD void child_patches(const Layout& L, P row, const DeltaT<NR>& d, R all_new, FP fp, F put) {
  uint32_t spk[PACKW], epk[PACKW];
  child_pack(L, d, spk, epk);
  child_write(L, row, d, spk, epk, all_new, fp, put);
}

// Materialise the successor row: child = parent + child_patches.
// `child` may alias `row` (in place) but nothing else of it.
template <int NS, class P, class Q, class R, int NR>
RTLA_HD void materialize(const Layout& L, P row, const DeltaT<NR>& d, R all_new, FP fp, Q child) {
  for (int w = 0; w < L.W; w++) child[w] = row[w];
  // (child_patches reads the parent's nelec from the copy before it rewrites the header)
  child_patches<NS>(L, child, d, all_new, fp, [&](int w, uint32_t v) { child[w] = v; });
}

// ------------------------------------------------------------ symmetry ----
// SYMMETRY Permutations(Server) (specs/MC.tla).  TLC identifies a state with
// its server-permuted images: a successor is new iff its orbit was not seen.
// The seen-set key of a state s is a function of its orbit only:
//
//   key(s) = finish( min over pi in C(s) of fp(pi(s)) ) + fp(allLogs)
//
// where pi(s) moves server record i to position pi[i] and relabels every
// server-valued field (votedFor, votesResponded/Granted, voterLog and
// next/matchIndex domains, msource/mdest, eleader, evotes, evoterLog), and
// C(s) is the set of permutations that sort the servers by a signature:
// sig_i(s) is a hash of everything server i "sees" with server names folded
// to self/other (its record, and the multisets of messages it sent and is
// sent), so sig_{pi[i]}(pi(s)) = sig_i(s) for every pi.  C(s) = { pi :
// sig_i < sig_j => pi[i] < pi[j] }; for s' = rho(s), C(s') = C(s) o rho^-1,
// so { pi(s') : pi in C(s') } = { pi(s) : pi in C(s) } and the key is
// orbit-invariant -- whatever the signature's quality.  A good signature only
// makes C small: servers tie only when they look alike, and then all |C| =
// prod(tie-group sizes)! orderings are tried.  (TLC itself fingerprints all
// N! images of every successor.)  allLogs holds no server names.
//
// The row keeps the state itself (and its own fingerprint): TLC explores the
// state it generated; the orbit key is used for the seen set and shard
// ownership only.  The same sym_key template runs in the kernels (on a parent
// row patched by a Delta, never materialised) and on the host (rows), so the
// keys agree everywhere.

// k-th permutation of 0..N-1 in lexicographic order (Lehmer code)
template <int NS>
RTLA_HD void kth_perm(int k, int* pi, int* inv) {
  int avail = (1 << NS) - 1;
  int f = 1;
#pragma unroll
  for (int i = 2; i < NS; i++) f *= i;  // (NS-1)!
#pragma unroll
  for (int i = 0; i < NS; i++) {
    const int idx = f ? k / f : 0;
    k -= idx * f;
    int pick = 0, seen = -1;
#pragma unroll
    for (int b = 0; b < NS; b++)
      if (avail >> b & 1) {
        seen++;
        if (seen == idx) pick = b;
      }
    pi[i] = pick;
    avail &= ~(1 << pick);
    if (NS - 1 - i > 0) f /= (NS - 1 - i);
  }
#pragma unroll
  for (int i = 0; i < NS; i++)
#pragma unroll
    for (int j = 0; j < NS; j++)
      if (pi[j] == i) inv[i] = j;
}
template <int NS>
RTLA_HD uint32_t perm_mask(uint32_t m, const int* pi) {
  uint32_t r = 0;
#pragma unroll
  for (int j = 0; j < NS; j++) r |= ((m >> j) & 1u) << pi[j];
  return r;
}
template <int NS>
RTLA_HD uint32_t sel_word(const uint32_t* a, int i) {  // a[i] for a run-time i, as selects
  uint32_t r = 0;
#pragma unroll
  for (int k = 0; k < NS; k++)
    if (k == i) r = a[k];
  return r;
}
template <int NS>
RTLA_HD uint32_t perm_id(uint32_t v, const int* pi) {  // a server id (or NIL) relabelled
  uint32_t r = v;
#pragma unroll
  for (int j = 0; j < NS; j++)
    if (v == (uint32_t)j) r = (uint32_t)pi[j];
  return r;
}
// server record relabelled by pi (the record of server i, now at pi[i])
template <int NS>
RTLA_HD void perm_srv_rec(const uint32_t* rec, const int* pi, const int* inv, uint32_t* out) {
  const uint32_t w0 = rec[0];
  out[0] = s_make(s_term(w0), s_role(w0), perm_id<NS>(s_voted(w0), pi), s_commit(w0), perm_mask<NS>(s_vresp(w0), pi),
                  perm_mask<NS>(s_vgrant(w0), pi), perm_mask<NS>(s_vlp(w0), pi));
  out[1] = rec[1];
  uint32_t nm = 0;
  uint32_t vl[NS];
#pragma unroll
  for (int j = 0; j < NS; j++) vl[j] = rec[3 + j];
#pragma unroll
  for (int k = 0; k < NS; k++) {
    const int j = inv[k];  // field k of the image = field inv[k] of the original
    nm |= nm_next(rec[2], j) << (3 * k) | nm_match(rec[2], j) << (15 + 3 * k);
    out[3 + k] = sel_word<NS>(vl, j);
  }
  out[2] = nm;
}
template <int NS>
RTLA_HD uint64_t perm_msg_slot(const Layout& L, uint64_t v, const int* pi) {  // a PACKED slot relabelled
  if (!v) return 0;  // empty slot (h_msg(0) = 0)
  const uint64_t m = (1ull << L.b_sid) - 1ull;
  const uint32_t src = (uint32_t)(v >> 2 & m), dst = (uint32_t)(v >> (2 + L.b_sid) & m);
  return (v & ~(m << 2 | m << (2 + L.b_sid))) | (uint64_t)perm_id<NS>(src, pi) << 2 |
         (uint64_t)perm_id<NS>(dst, pi) << (2 + L.b_sid);
}
template <int NS>
RTLA_HD void perm_elec(const uint32_t* e, const int* pi, const int* inv, uint32_t* out) {
  const uint32_t w0 = e[0];
  out[0] = (w0 & 15u) | perm_id<NS>((w0 >> 4) & 7u, pi) << 4 | perm_mask<NS>((w0 >> 7) & 31u, pi) << 7 |
           perm_mask<NS>((w0 >> 12) & 31u, pi) << 12;
  out[1] = e[1];
  uint32_t vl[NS];
#pragma unroll
  for (int j = 0; j < NS; j++) vl[j] = e[2 + j];
#pragma unroll
  for (int k = 0; k < NS; k++) out[2 + k] = sel_word<NS>(vl, inv[k]);
}

RTLA_HD uint32_t mix32(uint32_t x) {  // lowbias32 finalizer (signatures only)
  x ^= x >> 16; x *= 0x7feb352du;
  x ^= x >> 15; x *= 0x846ca68bu;
  x ^= x >> 16;
  return x;
}

// Local part of server i's signature: its record with server names folded
// to self / other / Nil; the other servers' entries (vote bits, voterLog,
// next/matchIndex) enter as an order-free sum.
template <int NS>
RTLA_HD uint32_t srv_sig(int i, const uint32_t* rec) {
  const uint32_t w0 = rec[0], nm = rec[2];
  const uint32_t vf = s_voted(w0), vr = s_vresp(w0), vg = s_vgrant(w0), vl = s_vlp(w0);
  uint32_t h = mix32(s_term(w0) | s_role(w0) << 4 | s_commit(w0) << 8 |
                     (vf == NIL ? 0u : vf == (uint32_t)i ? 1u : 2u) << 12);
  h = mix32(h ^ rec[1]);
  uint32_t others = 0;
#pragma unroll
  for (int j = 0; j < NS; j++) {
    const uint32_t t = (vr >> j & 1u) | (vg >> j & 1u) << 1 | (vl >> j & 1u) << 2 | (vf == (uint32_t)j ? 8u : 0u) |
                       nm_next(nm, j) << 4 | nm_match(nm, j) << 8;
    const uint32_t x = mix32(t ^ mix32(rec[3 + j] + 0x9e3779b9u));
    if (j == i) h = mix32(h ^ x);
    else others += x;
  }
  return mix32(h ^ mix32(others + 0x85ebca6bu));
}

RTLA_HD bool fp_less(FP x, FP y) { return x.a < y.a || (x.a == y.a && x.b < y.b); }

// The least of several fingerprints is skewed towards 0, which would pile
// the orbit keys into the low slots of the open-addressing set.  Re-mix it
// with a bijection of the 128 bits (mix_b and mix_a are bijective; a'
// depends on b only through an xor) so home slots and shard ownership are
// uniform again and no two orbit keys merge.
RTLA_HD FP orbit_key_finish(FP m) {
  return FP{mix_a(m.a ^ (m.b >> 29 | m.b << 35)), mix_b(m.b)};
}

// Permutations packed 3 bits per server (pim: pi[j] at bits 3j, invm: its
// inverse), so a loop over servers indexes them with shifts: the orbit-key
// loops below stay rolled (one record live at a time) instead of unrolling
// into N records' worth of registers.  Same values as the array forms above.
template <int NS>
RTLA_HD uint32_t pk_get(uint32_t pm, int j) { return pm >> (3 * j) & 7u; }
template <int NS>
RTLA_HD uint32_t perm_id_p(uint32_t v, uint32_t pim) {
  uint32_t r = v;
#pragma unroll
  for (int j = 0; j < NS; j++)
    if (v == (uint32_t)j) r = pk_get<NS>(pim, j);
  return r;
}
template <int NS>
RTLA_HD uint32_t perm_mask_p(uint32_t m, uint32_t pim) {
  uint32_t r = 0;
#pragma unroll
  for (int j = 0; j < NS; j++) r |= ((m >> j) & 1u) << pk_get<NS>(pim, j);
  return r;
}
template <int NS>
RTLA_HD void perm_srv_rec_p(const uint32_t* rec, uint32_t pim, uint32_t invm, uint32_t* out) {
  const uint32_t w0 = rec[0];
  out[0] = s_make(s_term(w0), s_role(w0), perm_id_p<NS>(s_voted(w0), pim), s_commit(w0),
                  perm_mask_p<NS>(s_vresp(w0), pim), perm_mask_p<NS>(s_vgrant(w0), pim),
                  perm_mask_p<NS>(s_vlp(w0), pim));
  out[1] = rec[1];
  uint32_t nm = 0;
#pragma unroll
  for (int k = 0; k < NS; k++) {
    const int j = (int)pk_get<NS>(invm, k);  // field k of the image = field j of the original
    nm |= nm_next(rec[2], j) << (3 * k) | nm_match(rec[2], j) << (15 + 3 * k);
    out[3 + k] = sel_word<NS>(rec + 3, j);
  }
  out[2] = nm;
}
template <int NS>
RTLA_HD uint64_t perm_msg_slot_p(const Layout& L, uint64_t v, uint32_t pim) {
  if (!v) return 0;  // empty slot (h_msg(0) = 0)
  const uint64_t m = (1ull << L.b_sid) - 1ull;
  const uint32_t src = (uint32_t)(v >> 2 & m), dst = (uint32_t)(v >> (2 + L.b_sid) & m);
  return (v & ~(m << 2 | m << (2 + L.b_sid))) | (uint64_t)perm_id_p<NS>(src, pim) << 2 |
         (uint64_t)perm_id_p<NS>(dst, pim) << (2 + L.b_sid);
}
template <int NS>
RTLA_HD void perm_elec_p(const uint32_t* e, uint32_t pim, uint32_t invm, uint32_t* out) {
  const uint32_t w0 = e[0];
  out[0] = (w0 & 15u) | perm_id_p<NS>((w0 >> 4) & 7u, pim) << 4 | perm_mask_p<NS>((w0 >> 7) & 31u, pim) << 7 |
           perm_mask_p<NS>((w0 >> 12) & 31u, pim) << 12;
  out[1] = e[1];
#pragma unroll
  for (int k = 0; k < NS; k++) out[2 + k] = sel_word<NS>(e + 2, (int)pk_get<NS>(invm, k));
}

// The orbit key of a state given through accessors:
//   rec_of(i, out)  server i's record (3 + NS words)
//   slot_of(q)      bag slot q < nmsg, PACKED (0 = empty)
//   elec_of(e, out) election record e < nelec (2 + NS words)
//   afp             fingerprint of allLogs (permutation-free)
// in two phases: sym_rank (the signatures and the tie groups they leave:
// C(s) has `ncomb` members) and sym_image_fp (the fingerprint of pi_k(s)
// for the k-th member), so that a kernel can spread the images of a chunk's
// states over its lanes.  sym_key = both.
#ifndef RTLA_TWIN_MIN
#define RTLA_TWIN_MIN 3  // smallest tie group sym_rank tests for interchangeable members
#endif
struct SymRank {
  uint32_t lom, cntm, radm;  // per server (3 bits each): first position, tie-group size, choices left
  int ncomb;                 // |C(s)|
};
// Is the transposition (i j) an automorphism of s -- tau(s) = s -- by a
// SUFFICIENT test: no message names i or j, every election record and every
// other server's record is unchanged by the relabelling, and i's record
// relabelled is j's.  (Then all orderings of a tie group whose consecutive
// members pass give the same image: the transpositions generate the group's
// permutations.  A test that fails merely keeps all of them.)
template <int NS, class RecF, class SlotF, class ElecF>
RTLA_HD bool sym_twins(const Layout& L, RecF rec_of, int nmsg, SlotF slot_of, int nelec, ElecF elec_of, int i,
                       int j) {
  constexpr int SW = 3 + NS, EW = 2 + NS;
  const uint64_t sm = (1ull << L.b_sid) - 1ull;
  for (int q = 0; q < nmsg; q++) {
    const uint64_t v = slot_of(q);
    if (!v) continue;
    const uint32_t src = (uint32_t)(v >> 2 & sm), dst = (uint32_t)(v >> (2 + L.b_sid) & sm);
    if (src == (uint32_t)i || src == (uint32_t)j || dst == (uint32_t)i || dst == (uint32_t)j) return false;
  }
  uint32_t tau = 0;  // the transposition, packed (its own inverse)
#pragma unroll
  for (int k = 0; k < NS; k++) tau |= (uint32_t)(k == i ? j : k == j ? i : k) << (3 * k);
  bool same = true;
#pragma unroll 1
  for (int p = 0; p < NS; p++) {  // relabel(rec_p) == rec_{tau(p)}
    uint32_t a[SW], b[SW], out[SW];
    rec_of(p, a);
    rec_of(p == i ? j : p == j ? i : p, b);
    perm_srv_rec_p<NS>(a, tau, tau, out);
#pragma unroll
    for (int w = 0; w < SW; w++) same = same && out[w] == b[w];
  }
  for (int e = 0; e < nelec && same; e++) {
    uint32_t er[EW], out[EW];
    elec_of(e, er);
    perm_elec_p<NS>(er, tau, tau, out);
#pragma unroll
    for (int w = 0; w < EW; w++) same = same && out[w] == er[w];
  }
  return same;
}
// A bag slot's share of its sender's / receiver's signature: the message
// with both names dropped (msource /= mdest in every message), hashed.
RTLA_HD uint32_t slot_sig_sent(const Layout& L, uint64_t v) {
  const uint64_t sm = (1ull << L.b_sid) - 1ull;
  const uint64_t anon = v & ~(sm << 2 | sm << (2 + L.b_sid));
  return mix32((uint32_t)anon ^ mix32((uint32_t)(anon >> 32) + 0x632be5abu));
}
RTLA_HD uint32_t slot_sig_recv(uint32_t sent) { return mix32(sent ^ 0x5bd1e995u); }
RTLA_HD uint32_t slot_src(const Layout& L, uint64_t v) { return (uint32_t)(v >> 2 & ((1ull << L.b_sid) - 1ull)); }
RTLA_HD uint32_t slot_dst(const Layout& L, uint64_t v) {
  return (uint32_t)(v >> (2 + L.b_sid) & ((1ull << L.b_sid) - 1ull));
}
// Server i's signature from its parts: the local part (srv_sig, high half)
// and the sums of slot_sig_sent / slot_sig_recv over the messages it sent /
// is sent.
RTLA_HD uint64_t sig_of(uint32_t local, uint32_t ms, uint32_t mr) {
  return (uint64_t)local << 32 | mix32(ms ^ mix32(mr + 0x27d4eb2fu));
}
// The signature parts of a state: loc[i], ms[i], mr[i] per server.
template <int NS, class RecF, class SlotF>
RTLA_HD void sym_sig_parts(const Layout& L, RecF rec_of, int nmsg, SlotF slot_of, uint32_t* loc, uint32_t* ms,
                           uint32_t* mr) {
  constexpr int SW = 3 + NS;
#pragma unroll
  for (int j = 0; j < NS; j++) ms[j] = mr[j] = 0;
  for (int q = 0; q < nmsg; q++) {
    const uint64_t v = slot_of(q);
    if (!v) continue;
    const uint32_t src = slot_src(L, v), dst = slot_dst(L, v);
    const uint32_t c = slot_sig_sent(L, v), cr = slot_sig_recv(c);
#pragma unroll
    for (int j = 0; j < NS; j++) {
      ms[j] += src == (uint32_t)j ? c : 0u;
      mr[j] += dst == (uint32_t)j ? cr : 0u;
    }
  }
#pragma unroll 1
  for (int i = 0; i < NS; i++) {  // one record live at a time
    uint32_t rec[SW];
    rec_of(i, rec);
    set_at<NS>(loc, i, srv_sig<NS>(i, rec));
  }
}
// Ranking from the signatures: C(s)'s tie groups (and |C(s)|).
template <int NS, class RecF, class SlotF, class ElecF>
RTLA_HD SymRank sym_rank_from(const Layout& L, const uint64_t* sig, RecF rec_of, int nmsg, SlotF slot_of, int nelec,
                              ElecF elec_of) {
  // pi[i] ranges over [lo_i, lo_i + cnt_i); server i picks among the
  // positions its tie group has left: rad_i = cnt_i - (tied servers before i)
  SymRank r{0, 0, 0, 1};
#pragma unroll
  for (int i = 0; i < NS; i++) {
    int l = 0, c = 0, b = 0;
#pragma unroll
    for (int j = 0; j < NS; j++) {
      l += sig[j] < sig[i] ? 1 : 0;
      c += sig[j] == sig[i] ? 1 : 0;
      if (j < i) b += sig[j] == sig[i] ? 1 : 0;
    }
    r.lom |= (uint32_t)l << (3 * i);
    r.cntm |= (uint32_t)c << (3 * i);
    r.radm |= (uint32_t)(c - b) << (3 * i);
    r.ncomb *= c - b;
  }
  if (r.ncomb > 1) {
    // tie groups whose members are interchangeable (sym_twins for each
    // member and the next one of its group) need one ordering only
#pragma unroll 1
    for (int i = 0; i < NS; i++) {
      const uint32_t li = pk_get<NS>(r.lom, i), ci = pk_get<NS>(r.cntm, i);
      // i: first member of a tie group of >= RTLA_TWIN_MIN (a pair's test
      // costs about what its second image does)
      if (ci < RTLA_TWIN_MIN || pk_get<NS>(r.radm, i) != ci) continue;
      bool all = true;
      int prev = i;
      for (int j = i + 1; j < NS && all; j++) {
        if (pk_get<NS>(r.lom, j) != li) continue;  // (same first position <=> same group)
        all = sym_twins<NS>(L, rec_of, nmsg, slot_of, nelec, elec_of, prev, j);
        prev = j;
      }
      if (!all) continue;
      for (int j = i; j < NS; j++)
        if (pk_get<NS>(r.lom, j) == li) r.radm = (r.radm & ~(7u << (3 * j))) | 1u << (3 * j);
    }
    r.ncomb = 1;
#pragma unroll
    for (int i = 0; i < NS; i++) r.ncomb *= (int)pk_get<NS>(r.radm, i);
  }
  return r;
}
template <int NS, class RecF, class SlotF, class ElecF>
RTLA_HD SymRank sym_rank(const Layout& L, RecF rec_of, int nmsg, SlotF slot_of, int nelec, ElecF elec_of) {
  uint32_t loc[NS], ms[NS], mr[NS];
  sym_sig_parts<NS>(L, rec_of, nmsg, slot_of, loc, ms, mr);
  uint64_t sig[NS];
#pragma unroll
  for (int i = 0; i < NS; i++) sig[i] = sig_of(loc[i], ms[i], mr[i]);
  return sym_rank_from<NS>(L, sig, rec_of, nmsg, slot_of, nelec, elec_of);
}
// Fingerprint of pi_k(s), the k-th member (0 <= k < r.ncomb) of C(s).
template <int NS, class RecF, class SlotF, class ElecF>
RTLA_HD FP sym_image_fp(const Layout& L, RecF rec_of, int nmsg, SlotF slot_of, int nelec, ElecF elec_of,
                        const SymRank& r, int k) {
  constexpr int SW = 3 + NS, EW = 2 + NS;
  uint32_t pim = 0, invm = 0, used = 0;
  int rem = k;
#pragma unroll
  for (int i = 0; i < NS; i++) {
    const int rad = (int)pk_get<NS>(r.radm, i), cnt = (int)pk_get<NS>(r.cntm, i), lo = (int)pk_get<NS>(r.lom, i);
    int dgt = 0;
    if (rad > 1) {
      dgt = rem % rad;
      rem /= rad;
    }
    const uint32_t free = ((1u << cnt) - 1u) << lo & ~used;
    int p = 0, c = dgt;
#pragma unroll
    for (int b = 0; b < NS; b++)
      if (free >> b & 1u) {
        if (c == 0) p = b;
        c--;
      }
    pim |= (uint32_t)p << (3 * i);
    invm |= (uint32_t)i << (3 * p);
    used |= 1u << p;
  }
  FP f{0, 0};
#pragma unroll 1
  for (int i = 0; i < NS; i++) {
    uint32_t rec[SW], out[SW];
    rec_of(i, rec);
    perm_srv_rec_p<NS>(rec, pim, invm, out);
    f = fp_add(f, hash_words_from<SW>(srv_seed<NS>((int)pk_get<NS>(pim, i)), out));
  }
  for (int q = 0; q < nmsg; q++) f = fp_add(f, h_msg(perm_msg_slot_p<NS>(L, slot_of(q), pim)));
  for (int e = 0; e < nelec; e++) {
    uint32_t er[EW], out[EW];
    elec_of(e, er);
    perm_elec_p<NS>(er, pim, invm, out);
    f = fp_add(f, h_elec(out, EW));
  }
  return f;
}
template <int NS, class RecF, class SlotF, class ElecF>
RTLA_HD FP sym_key(const Layout& L, RecF rec_of, int nmsg, SlotF slot_of, int nelec, ElecF elec_of, FP afp,
                   int* perms = nullptr) {
  const SymRank r = sym_rank<NS>(L, rec_of, nmsg, slot_of, nelec, elec_of);
  if (perms) *perms = r.ncomb;
  FP best{~0ull, ~0ull};
  for (int k = 0; k < r.ncomb; k++) {
    const FP f = sym_image_fp<NS>(L, rec_of, nmsg, slot_of, nelec, elec_of, r, k);
    if (fp_less(f, best)) best = f;
  }
  return fp_add(orbit_key_finish(best), afp);
}

// allLogs part of a fingerprint: sum of h_all over the set bits of the words
template <class Q>
RTLA_HD FP alllogs_fp(const Layout& L, Q words) {
  FP f{0, 0};
  for (int w = 0; w < L.all_words; w++) {
    uint32_t m = words[w];
    while (m) {
      const int b = __builtin_ctz(m);
      m &= m - 1;
      f = fp_add(f, h_all(w * 32 + b));
    }
  }
  return f;
}

// Orbit key of a materialised row (host: rtla_orbit_key, tests).
template <int NS, class P>
RTLA_HD FP orbit_key_row(const Layout& L, P row, int* perms = nullptr) {
  return sym_key<NS>(L, [&](int i, uint32_t* out) { load_rec<NS>(L, row, i, out); }, row_nmsg(L, row),
                     [&](int q) { return slot_raw(L, row, q); }, row_nelec(L, row),
                     [&](int e, uint32_t* out) {
                       elec_get(L, row, e, out);
                     },
                     alllogs_fp(L, row + L.off_all), perms);
}

// pi(row): the server-permuted image of a row, with its own fingerprint
// (host: rtla_permute_row, the symmetry tests).  Bag slots and election
// records keep their order (both are multisets in the fingerprint).
template <int NS, class P, class Q>
RTLA_HD void permute_row(const Layout& L, P row, const int* pi, Q out) {
  constexpr int SW = 3 + NS, EW = 2 + NS;
  int inv[NS];
  for (int i = 0; i < NS; i++)
    for (int j = 0; j < NS; j++)
      if (pi[j] == i) inv[i] = j;
  for (int w = 0; w < L.W; w++) out[w] = row[w];
  for (int i = 0; i < NS; i++) {
    uint32_t rec[SW], img[SW];
    load_rec<NS>(L, row, i, rec);
    perm_srv_rec<NS>(rec, pi, inv, img);
    srv_put(L, out, pi[i], img);
  }
  const int nm = row_nmsg(L, row), ne = row_nelec(L, row);
  for (int q = 0; q < nm; q++) {
    const uint64_t x = perm_msg_slot<NS>(L, slot_raw(L, row, q), pi);
    out[L.off_bag + q * L.slot_w] = (uint32_t)x;
    if (L.slot_w > 1) out[L.off_bag + q * L.slot_w + 1] = (uint32_t)(x >> 32);
  }
  for (int e = 0; e < ne; e++) {
    uint32_t er[EW], img[EW];
    elec_get(L, row, e, er);
    perm_elec<NS>(er, pi, inv, img);
    elec_put(L, out, e, img);
  }
  row_set_fp(out, row_fingerprint(L, out));
}

// ---------------------------------------------------------- invariants ----
// Evaluated on the successor (parent + delta) without materialising it; the
// delta is passed as the few words the invariants read (srv < 0: none).
// Returns the mask of VIOLATED invariants among L.inv_mask.
template <int NS, class P>
RTLA_HD int check_invariants_v(const Layout& L, P row, int dsrv, uint32_t drec0, uint32_t drec1, int delec,
                               uint32_t derec0) {
  const int N = RTLA_NSRV(L);
  constexpr int NC = NS ? NS : NMAX;
  int bad = 0;
  uint32_t w0[NC], lg[NC];
#pragma unroll
  for (int i = 0; i < NC; i++) {
    w0[i] = i < N ? srv_w0(L, row, i) : 0u;
    lg[i] = i < N ? srv_log(L, row, i) : 0u;
    if (i == dsrv) { w0[i] = drec0; lg[i] = drec1; }
  }
  if (L.inv_mask & INV_NO_TWO_LEADERS) {
    // NoTwoLeaders == \A i, j \in Server : state[i] = Leader /\ state[j] = Leader => i = j
    int nl = 0;
#pragma unroll
    for (int i = 0; i < NC; i++) nl += (i < N) && s_role(w0[i]) == LEADER;
    if (nl > 1) bad |= INV_NO_TWO_LEADERS;
  }
  if (L.inv_mask & INV_ELECTION_SAFETY) {
    // ElectionSafety == \A e, f \in elections : e.eterm = f.eterm => e.eleader = f.eleader
    const int ne = row_nelec(L, row);
    const int tot = ne + (delec ? 1 : 0);
    for (int a = 0; a < tot; a++) {
      const uint32_t ea = a < ne ? elec_w0(L, row, a) : derec0;
      for (int b = a + 1; b < tot; b++) {
        const uint32_t eb = b < ne ? elec_w0(L, row, b) : derec0;
        if ((ea & 15u) == (eb & 15u) && ((ea >> 4) & 7u) != ((eb >> 4) & 7u)) bad |= INV_ELECTION_SAFETY;
      }
    }
  }
  if (L.inv_mask & INV_LOG_MATCHING) {
    // LogMatching == \A i, j \in Server : \A n \in 1..Min({Len(log[i]), Len(log[j])}) :
    //   log[i][n].term = log[j][n].term => SubSeq(log[i],1,n) = SubSeq(log[j],1,n)
#pragma unroll
    for (int i = 0; i < NC; i++)
#pragma unroll
      for (int j = i + 1; j < NC; j++) {
        if (j >= N) continue;
        const uint32_t a = lg[i], b = lg[j];
        const uint32_t m = log_len(a) < log_len(b) ? log_len(a) : log_len(b);
        for (uint32_t n = 1; n <= m; n++)
          if (log_term(a, n) == log_term(b, n) && log_prefix(a, n) != log_prefix(b, n)) bad |= INV_LOG_MATCHING;
      }
  }
  return bad;
}

template <int NS, class P, int NR = NMAX>
RTLA_HD int check_invariants(const Layout& L, P row, const DeltaT<NR>* d) {
  if (!d) return check_invariants_v<NS>(L, row, -1, 0u, 0u, 0, 0u);
  return check_invariants_v<NS>(L, row, d->srv, d->rec[0], d->rec[1], d->elec, d->erec[0]);
}

#undef RTLA_NSRV

}  // namespace rtla
