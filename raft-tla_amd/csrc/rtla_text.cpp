// rtla_text.cpp -- TLC-style state printer for packed rows.
//
// TLC prints a state as one "/\ var = value" line per variable
// (raft.tla:32-85 declaration order).  Values use TLA+ syntax: records
// [f |-> v], functions (a :> x @@ b :> y), sequences <<...>>, sets {...};
// the empty function prints as <<>>.  Sets and the bag's domain are printed
// sorted by their text so the output is canonical (the row itself keeps the
// bag and the elections list unordered).
//
// The printer writes into a flat character buffer (no per-field string
// temporaries): it also produces the per-level parity digests over hundreds
// of millions of states (rtla_level_text_hash), so it is written for speed.
#include "rtla_text.h"

#include <string.h>

#include <algorithm>
#include <vector>

namespace rtla {

namespace {

// Append-only text buffer; items of the sorted collections are written into
// a second buffer and referenced by (offset, length).
struct Out {
  char* p;
  size_t n = 0;
  template <size_t K>
  void s(const char (&t)[K]) {  // a literal: its length is known at compile time
    memcpy(p + n, t, K - 1);
    n += K - 1;
  }
  void str(const char* t) {  // a run-time string
    const size_t k = strlen(t);
    memcpy(p + n, t, k);
    n += k;
  }
  void c(char ch) { p[n++] = ch; }
  void u(uint32_t v) {  // decimal
    char t[12];
    int k = 0;
    do {
      t[k++] = (char)('0' + v % 10);
      v /= 10;
    } while (v);
    while (k) p[n++] = t[--k];
  }
  void srv(uint32_t i) {  // server name s<i+1>
    c('s');
    u(i + 1);
  }
};

void text_log(Out& o, uint32_t l) {
  const uint32_t n = log_len(l);
  if (!n) return o.s("<<>>");
  o.s("<<");
  for (uint32_t k = 1; k <= n; k++) {
    if (k > 1) o.s(", ");
    o.s("[term |-> ");
    o.u(log_term(l, k));
    o.s(", value |-> v");
    o.u(log_val(l, k) + 1);
    o.c(']');
  }
  o.s(">>");
}

void text_srvset(Out& o, uint32_t mask, int N) {
  o.c('{');
  bool first = true;
  for (int j = 0; j < N; j++)
    if (mask >> j & 1u) {
      if (!first) o.s(", ");
      o.srv((uint32_t)j);
      first = false;
    }
  o.c('}');
}

void text_vl(Out& o, uint32_t dom, const uint32_t* vl, int N) {
  if (!dom) return o.s("<<>>");
  o.c('(');
  bool first = true;
  for (int j = 0; j < N; j++)
    if (dom >> j & 1u) {
      if (!first) o.s(" @@ ");
      o.srv((uint32_t)j);
      o.s(" :> ");
      text_log(o, vl[j]);
      first = false;
    }
  o.c(')');
}

const char* BOOL(uint32_t b) { return b ? "TRUE" : "FALSE"; }

void text_msg(Out& o, uint64_t k, const int* pi = nullptr) {
  static const char* TN[4] = {"RequestVoteRequest", "RequestVoteResponse", "AppendEntriesRequest",
                              "AppendEntriesResponse"};
  o.s("[mtype |-> \"");
  o.str(TN[m_type(k)]);
  o.s("\", mterm |-> ");
  o.u(m_term(k));
  o.s(", ");
  switch (m_type(k)) {
    case RVREQ:
      o.s("mlastLogTerm |-> ");
      o.u(m_f(k, 12, 4));
      o.s(", mlastLogIndex |-> ");
      o.u(m_f(k, 16, 3));
      o.s(", ");
      break;
    case RVRESP:
      o.s("mvoteGranted |-> ");
      o.str(BOOL(m_f(k, 12, 1)));
      o.s(", mlog |-> ");
      text_log(o, m_f(k, 16, 28));
      o.s(", ");
      break;
    case AEREQ: {
      o.s("mprevLogIndex |-> ");
      o.u(m_f(k, 12, 3));
      o.s(", mprevLogTerm |-> ");
      o.u(m_f(k, 15, 4));
      o.s(", mentries |-> ");
      if (m_f(k, 19, 1)) {
        const uint32_t e = m_f(k, 20, 5);
        o.s("<<[term |-> ");
        o.u(e & 7u);
        o.s(", value |-> v");
        o.u((e >> 3) + 1);
        o.s("]>>");
      } else {
        o.s("<<>>");
      }
      o.s(", mlog |-> ");
      text_log(o, m_f(k, 28, 28));
      o.s(", mcommitIndex |-> ");
      o.u(m_f(k, 25, 3));
      o.s(", ");
      break;
    }
    case AERESP:
      o.s("msuccess |-> ");
      o.str(BOOL(m_f(k, 12, 1)));
      o.s(", mmatchIndex |-> ");
      o.u(m_f(k, 13, 3));
      o.s(", ");
      break;
  }
  o.s("msource |-> ");
  o.srv(pi ? (uint32_t)pi[m_src(k)] : m_src(k));
  o.s(", mdest |-> ");
  o.srv(pi ? (uint32_t)pi[m_dst(k)] : m_dst(k));
  o.c(']');
}

// Items of one sorted collection: their texts live in `scratch`.
struct Items {
  Out scratch;
  uint32_t off[KMAX + EMAX + 32 * 32 + 1], len[KMAX + EMAX + 32 * 32 + 1];
  int n = 0;
  size_t mark = 0;
  void begin() { mark = scratch.n; }
  void end() {
    off[n] = (uint32_t)mark;
    len[n] = (uint32_t)(scratch.n - mark);
    n++;
  }
  // std::string ordering: bytewise, a proper prefix first
  void emit(Out& o, const char* open, const char* sep, const char* close, const char* empty) {
    if (!n) return o.str(empty);
    uint16_t ord[KMAX + EMAX + 32 * 32 + 1];
    for (int k = 0; k < n; k++) ord[k] = (uint16_t)k;
    const char* base = scratch.p;
    std::sort(ord, ord + n, [&](uint16_t a, uint16_t b) {
      const uint32_t la = len[a], lb = len[b];
      const int r = memcmp(base + off[a], base + off[b], std::min(la, lb));
      return r < 0 || (r == 0 && la < lb);
    });
    o.str(open);
    for (int k = 0; k < n; k++) {
      if (k) o.str(sep);
      memcpy(o.p + o.n, base + off[ord[k]], len[ord[k]]);
      o.n += len[ord[k]];
    }
    o.str(close);
    n = 0;
    scratch.n = 0;
  }
};

// Upper bound of one state's text: every variable at its widest.
size_t text_cap(const Layout& L) {
  const size_t log = 8 + (size_t)(LMAX + 1) * 40;
  const size_t msg = 300 + 2 * log;
  const size_t vl = 4 + (size_t)L.N * (16 + log);
  return 4096 + (size_t)L.K * (msg + 16) + (size_t)L.E * (200 + log + vl + 16 * L.N) +
         (size_t)L.n_logs * (log + 2) + (size_t)L.N * (400 + log + 2 * vl + 40 * L.N);
}

// A row decoded once; the text of any server-permuted image pi(s) is
// rendered from it (pi relabels every server-valued field, sg = pi^-1 gives
// the server whose record lands at each position; nullptr = the state).
struct Dec {
  int N, nm, ne;
  uint32_t rec[NMAX][3 + NMAX];
  uint64_t key[KMAX];
  uint32_t cnt[KMAX];
  uint32_t er[EMAX][2 + NMAX];
};

void decode(const Layout& L, const uint32_t* row, Dec& d) {
  d.N = L.N;
  d.nm = row_nmsg(L, row);
  d.ne = row_nelec(L, row);
  for (int i = 0; i < L.N; i++) srv_get(L, row, i, d.rec[i]);
  for (int k = 0; k < d.nm; k++) {
    const uint64_t v = bag_slot(L, row, k);
    d.key[k] = m_key(v);
    d.cnt[k] = m_count(v);
  }
  for (int e = 0; e < d.ne; e++) elec_get(L, row, e, d.er[e]);
}

uint32_t pmask(uint32_t m, const int* pi, int N) {  // {pi[j] : j \in m}
  if (!pi) return m;
  uint32_t r = 0;
  for (int j = 0; j < N; j++)
    if (m >> j & 1u) r |= 1u << pi[j];
  return r;
}

void line_messages(Out& o, Items& it, const Dec& d, const int* pi) {
  for (int k = 0; k < d.nm; k++) {
    it.begin();
    text_msg(it.scratch, d.key[k], pi);
    it.scratch.s(" :> ");
    it.scratch.u(d.cnt[k]);
    it.end();
  }
  o.s("/\\ messages = ");
  it.emit(o, "(", " @@ ", ")", "<<>>");
}

void line_elections(Out& o, Items& it, const Dec& d, const int* pi) {
  const int N = d.N;
  for (int e = 0; e < d.ne; e++) {
    const uint32_t* r = d.er[e];
    const uint32_t w0 = r[0];
    uint32_t vl[NMAX];
    for (int j = 0; j < N; j++) vl[pi ? pi[j] : j] = r[2 + j];
    Out& s = it.scratch;
    it.begin();
    s.s("[eterm |-> ");
    s.u(w0 & 15u);
    s.s(", eleader |-> ");
    const uint32_t ld = (w0 >> 4) & 7u;
    s.srv(pi ? (uint32_t)pi[ld] : ld);
    s.s(", elog |-> ");
    text_log(s, r[1]);
    s.s(", evotes |-> ");
    text_srvset(s, pmask((w0 >> 7) & 31u, pi, N), N);
    s.s(", evoterLog |-> ");
    text_vl(s, pmask((w0 >> 12) & 31u, pi, N), vl, N);
    s.c(']');
    it.end();
  }
  o.s("/\\ elections = ");
  it.emit(o, "{", ", ", "}", "{}");
}

void line_alllogs(Out& o, Items& it, const Layout& L, const uint32_t* row) {
  for (int x = 0; x < L.n_logs; x++)
    if (row[L.off_all + (x >> 5)] >> (x & 31) & 1u) {
      it.begin();
      text_log(it.scratch, log_from_index(L, x));
      it.end();
    }
  o.s("/\\ allLogs = ");
  it.emit(o, "{", ", ", "}", "{}");
}

// The k-th per-server line (raft.tla:50-85 order): currentTerm, state,
// votedFor, log, commitIndex, votesResponded, votesGranted, voterLog,
// nextIndex, matchIndex.
constexpr int SRV_LINES = 10;
void line_server(Out& o, const Dec& d, int k, const int* pi, const int* sg) {
  static const char* NAME[SRV_LINES] = {"currentTerm", "state", "votedFor", "log", "commitIndex",
                                        "votesResponded", "votesGranted", "voterLog", "nextIndex", "matchIndex"};
  static const char* RN[4] = {"\"Follower\"", "\"Candidate\"", "\"Leader\"", "\"?\""};
  const int N = d.N;
  o.s("/\\ ");
  o.str(NAME[k]);
  o.s(" = (");
  for (int p = 0; p < N; p++) {
    const uint32_t* r = d.rec[sg ? sg[p] : p];
    if (p) o.s(" @@ ");
    o.srv((uint32_t)p);
    o.s(" :> ");
    switch (k) {
      case 0: o.u(s_term(r[0])); break;
      case 1: o.str(RN[s_role(r[0])]); break;
      case 2:
        if (s_voted(r[0]) == NIL) o.s("\"Nil\"");
        else o.srv(pi ? (uint32_t)pi[s_voted(r[0])] : s_voted(r[0]));
        break;
      case 3: text_log(o, r[1]); break;
      case 4: o.u(s_commit(r[0])); break;
      case 5: text_srvset(o, pmask(s_vresp(r[0]), pi, N), N); break;
      case 6: text_srvset(o, pmask(s_vgrant(r[0]), pi, N), N); break;
      case 7: {
        uint32_t vl[NMAX];
        for (int q = 0; q < N; q++) vl[q] = r[3 + (sg ? sg[q] : q)];
        text_vl(o, pmask(s_vlp(r[0]), pi, N), vl, N);
        break;
      }
      default: {
        o.c('(');
        for (int q = 0; q < N; q++) {
          if (q) o.s(" @@ ");
          o.srv((uint32_t)q);
          o.s(" :> ");
          const int j = sg ? sg[q] : q;
          o.u(k == 8 ? nm_next(r[2], j) : nm_match(r[2], j));
        }
        o.c(')');
      }
    }
  }
  o.c(')');
}

// The text of the image pi(s), lines in TLC order.
size_t image_text(const Layout& L, const uint32_t* row, const Dec& d, const int* pi, const int* sg, char* buf,
                  char* scratch) {
  Out o{buf};
  Items it;
  it.scratch.p = scratch;
  line_messages(o, it, d, pi);
  o.c('\n');
  line_elections(o, it, d, pi);
  o.c('\n');
  line_alllogs(o, it, L, row);
  for (int k = 0; k < SRV_LINES; k++) {
    o.c('\n');
    line_server(o, d, k, pi, sg);
  }
  return o.n;
}

}  // namespace

size_t state_text_cap(const Layout& L) { return text_cap(L); }

size_t state_text_into(const Layout& L, const uint32_t* row, char* buf, char* scratch) {
  Dec d;
  decode(L, row, d);
  return image_text(L, row, d, nullptr, nullptr, buf, scratch);
}

// The orbit text (the per-orbit item of a SYMMETRY level's digest,
// DESIGN.md section 3): the text of the image pi(s) whose ROTATED text --
// the ten per-server lines first, then messages, elections, allLogs -- is
// least over all N! permutations.  Defined on the value text alone, so the
// CPU oracle (oracle/raft_cpu.c orbit_text) and the value oracle compute it
// independently of this code; nothing here uses the kernels' orbit key.
//
// The images are compared line by line, each dropped at its first line
// above the best so far.  One exact shortcut: the first two rotated lines
// (currentTerm, state) print a relabel-free token per position (a decimal
// term, a quoted role; neither token set has one token a proper prefix of
// another followed by a character that sorts below the delimiters " @@ " /
// ")"), so their least text lists the servers sorted by (term text, role
// text), and every image that does not is above it there: only the
// orderings within ties of (term, role) are rendered.
size_t state_orbit_text_into(const Layout& L, const uint32_t* row, char* buf, char* scratch) {
  Dec d;
  decode(L, row, d);
  const int N = d.N;
  // servers sorted by (term text, role text): the key packs the term's
  // decimal text (two digits, a one-digit term's second digit below '0')
  // and the role's rank in text order ("Candidate" < "Follower" < "Leader")
  static const int RRANK[4] = {1, 0, 2, 3};
  int key[NMAX];
  for (int i = 0; i < N; i++) {
    const uint32_t t = s_term(d.rec[i][0]);
    const int d0 = t >= 10 ? (int)(t / 10) : (int)t, d1 = t >= 10 ? (int)(t % 10) : -1;
    key[i] = (d0 * 11 + (d1 + 1)) * 4 + RRANK[s_role(d.rec[i][0])];
  }
  int sg[NMAX], pi[NMAX], best_sg[NMAX];
  for (int i = 0; i < N; i++) sg[i] = i;
  std::stable_sort(sg, sg + N, [&](int a, int b) { return key[a] < key[b]; });
  int gb[NMAX + 1], ng = 0;  // tie groups [gb[g], gb[g+1]) of positions
  for (int p = 0; p < N; p++)
    if (p == 0 || key[sg[p]] != key[sg[p - 1]]) gb[ng++] = p;
  gb[ng] = N;
  // rotated text minus the first two lines (equal for every candidate),
  // compared line by line with the best so far
  const size_t cap = text_cap(L);
  thread_local std::vector<char> work;  // two rotated texts (candidate, best)
  if (work.size() < 2 * cap) work.resize(2 * cap);
  char* bufs[2] = {work.data(), work.data() + cap};
  int bi = -1;
  size_t bn = 0, bmsg = 0;  // the best's length and the offset of its messages line ("\n" before it)
  Items it;
  it.scratch.p = scratch;
  for (;;) {
    for (int p = 0; p < N; p++) pi[sg[p]] = p;
    const int ci = bi < 0 ? 0 : bi ^ 1;
    Out o{bufs[ci]};
    bool below = bi < 0, above = false;
    size_t msg_off = 0;
    auto cmp_line = [&](size_t from) {  // the line just written: below / above / equal to best's bytes
      if (below) return;
      const int r = memcmp(o.p + from, bufs[bi] + from, o.n - from);
      if (r < 0) below = true;
      else if (r > 0) above = true;
    };
    for (int k = 2; k < SRV_LINES + 3 && !above; k++) {
      const size_t from = o.n;
      if (k == SRV_LINES) msg_off = from;
      o.c('\n');
      if (k < SRV_LINES) line_server(o, d, k, pi, sg);
      else if (k == SRV_LINES) line_messages(o, it, d, pi);
      else if (k == SRV_LINES + 1) line_elections(o, it, d, pi);
      else line_alllogs(o, it, L, row);
      cmp_line(from);
    }
    if (below) {
      bi = ci;
      bn = o.n;
      bmsg = msg_off;
      for (int p = 0; p < N; p++) best_sg[p] = sg[p];
    }
    // next ordering: an odometer over the tie groups' permutations
    int g = ng - 1;
    while (g >= 0 && !std::next_permutation(sg + gb[g], sg + gb[g + 1])) g--;
    if (g < 0) break;
  }
  // the best image's text in TLC order, from its rotated text: messages,
  // elections, allLogs, then the two lines every candidate shares, then the
  // other eight per-server lines
  for (int p = 0; p < N; p++) pi[best_sg[p]] = p;
  Out o{buf};
  memcpy(o.p, bufs[bi] + bmsg + 1, bn - bmsg - 1);
  o.n = bn - bmsg - 1;
  for (int k = 0; k < 2; k++) {
    o.c('\n');
    line_server(o, d, k, pi, best_sg);
  }
  memcpy(o.p + o.n, bufs[bi], bmsg);
  o.n += bmsg;
  return o.n;
}

std::string state_text(const Layout& L, const uint32_t* row) {
  const size_t cap = text_cap(L);
  std::string buf(2 * cap, '\0');
  const size_t n = state_text_into(L, row, &buf[0], &buf[cap]);
  buf.resize(n);
  return buf;
}

std::string action_name(const Layout& L, int inst, int sub) {
  static const char* SUB[R_NONE + 1] = {"UpdateTerm",
                                        "HandleRequestVoteRequest",
                                        "HandleRequestVoteResponse",
                                        "HandleAppendEntriesRequest",
                                        "HandleAppendEntriesResponse",
                                        "DropStaleResponse",
                                        "?"};
  int fam = 0;
  while (fam + 1 < F_COUNT && inst >= L.fam[fam + 1]) fam++;
  int x = inst - L.fam[fam];
  const int N = L.N;
  switch (fam) {
    case F_RESTART: return "Restart(" + std::string("s") + std::to_string(x + 1) + ")";
    case F_TIMEOUT: return "Timeout(s" + std::to_string(x + 1) + ")";
    case F_REQUESTVOTE: return "RequestVote(s" + std::to_string(x / N + 1) + ", s" + std::to_string(x % N + 1) + ")";
    case F_BECOMELEADER: return "BecomeLeader(s" + std::to_string(x + 1) + ")";
    case F_CLIENTREQUEST: return "ClientRequest(s" + std::to_string(x / L.V + 1) + ", v" + std::to_string(x % L.V + 1) + ")";
    case F_ADVANCECOMMIT: return "AdvanceCommitIndex(s" + std::to_string(x + 1) + ")";
    case F_APPENDENTRIES: return "AppendEntries(s" + std::to_string(x / N + 1) + ", s" + std::to_string(x % N + 1) + ")";
    case F_RECEIVE: return std::string("Receive -> ") + SUB[sub < 0 || sub > R_NONE ? R_NONE : sub];
    case F_DUPLICATE: return "DuplicateMessage";
    default: return "DropMessage";
  }
}

}  // namespace rtla
