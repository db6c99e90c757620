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

namespace rtla {

namespace {

// Append-only text buffer; items of the sorted collections are written into
// a second buffer and referenced by (offset, length).
struct Out {
  char* p;
  size_t n = 0;
  void s(const char* t) {
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

void text_msg(Out& o, uint64_t k) {
  static const char* TN[4] = {"RequestVoteRequest", "RequestVoteResponse", "AppendEntriesRequest",
                              "AppendEntriesResponse"};
  o.s("[mtype |-> \"");
  o.s(TN[m_type(k)]);
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
      o.s(BOOL(m_f(k, 12, 1)));
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
      o.s(BOOL(m_f(k, 12, 1)));
      o.s(", mmatchIndex |-> ");
      o.u(m_f(k, 13, 3));
      o.s(", ");
      break;
  }
  o.s("msource |-> ");
  o.srv(m_src(k));
  o.s(", mdest |-> ");
  o.srv(m_dst(k));
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
    if (!n) return o.s(empty);
    uint16_t ord[KMAX + EMAX + 32 * 32 + 1];
    for (int k = 0; k < n; k++) ord[k] = (uint16_t)k;
    const char* base = scratch.p;
    std::sort(ord, ord + n, [&](uint16_t a, uint16_t b) {
      const uint32_t la = len[a], lb = len[b];
      const int r = memcmp(base + off[a], base + off[b], std::min(la, lb));
      return r < 0 || (r == 0 && la < lb);
    });
    o.s(open);
    for (int k = 0; k < n; k++) {
      if (k) o.s(sep);
      memcpy(o.p + o.n, base + off[ord[k]], len[ord[k]]);
      o.n += len[ord[k]];
    }
    o.s(close);
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

}  // namespace

size_t state_text_cap(const Layout& L) { return text_cap(L); }

size_t state_text_into(const Layout& L, const uint32_t* row, char* buf, char* scratch) {
  const int N = L.N;
  Out o{buf};
  Items it;
  it.scratch.p = scratch;
  const int nm = row_nmsg(L, row);
  for (int k = 0; k < nm; k++) {
    const uint64_t v = bag_slot(L, row, k);
    it.begin();
    text_msg(it.scratch, m_key(v));
    it.scratch.s(" :> ");
    it.scratch.u(m_count(v));
    it.end();
  }
  o.s("/\\ messages = ");
  it.emit(o, "(", " @@ ", ")", "<<>>");
  const int ne = row_nelec(L, row);
  for (int e = 0; e < ne; e++) {
    uint32_t r[2 + NMAX];
    elec_get(L, row, e, r);
    const uint32_t w0 = r[0];
    Out& s = it.scratch;
    it.begin();
    s.s("[eterm |-> ");
    s.u(w0 & 15u);
    s.s(", eleader |-> ");
    s.srv((w0 >> 4) & 7u);
    s.s(", elog |-> ");
    text_log(s, r[1]);
    s.s(", evotes |-> ");
    text_srvset(s, (w0 >> 7) & 31u, N);
    s.s(", evoterLog |-> ");
    text_vl(s, (w0 >> 12) & 31u, r + 2, N);
    s.c(']');
    it.end();
  }
  o.s("\n/\\ elections = ");
  it.emit(o, "{", ", ", "}", "{}");
  for (int x = 0; x < L.n_logs; x++)
    if (row[L.off_all + (x >> 5)] >> (x & 31) & 1u) {
      it.begin();
      text_log(it.scratch, log_from_index(L, x));
      it.end();
    }
  o.s("\n/\\ allLogs = ");
  it.emit(o, "{", ", ", "}", "{}");
  uint32_t recs[NMAX][3 + NMAX];  // the server records, unpacked
  for (int i = 0; i < N; i++) srv_get(L, row, i, recs[i]);
  auto per = [&](const char* name, auto fn) {
    o.s("\n/\\ ");
    o.s(name);
    o.s(" = (");
    for (int i = 0; i < N; i++) {
      if (i) o.s(" @@ ");
      o.srv((uint32_t)i);
      o.s(" :> ");
      fn(recs[i]);
    }
    o.c(')');
  };
  static const char* RN[4] = {"\"Follower\"", "\"Candidate\"", "\"Leader\"", "\"?\""};
  per("currentTerm", [&](const uint32_t* r) { o.u(s_term(r[0])); });
  per("state", [&](const uint32_t* r) { o.s(RN[s_role(r[0])]); });
  per("votedFor", [&](const uint32_t* r) {
    if (s_voted(r[0]) == NIL) o.s("\"Nil\"");
    else o.srv(s_voted(r[0]));
  });
  per("log", [&](const uint32_t* r) { text_log(o, r[1]); });
  per("commitIndex", [&](const uint32_t* r) { o.u(s_commit(r[0])); });
  per("votesResponded", [&](const uint32_t* r) { text_srvset(o, s_vresp(r[0]), N); });
  per("votesGranted", [&](const uint32_t* r) { text_srvset(o, s_vgrant(r[0]), N); });
  per("voterLog", [&](const uint32_t* r) { text_vl(o, s_vlp(r[0]), r + 3, N); });
  auto idx = [&](const uint32_t* r, bool match) {
    o.c('(');
    for (int j = 0; j < N; j++) {
      if (j) o.s(" @@ ");
      o.srv((uint32_t)j);
      o.s(" :> ");
      o.u(match ? nm_match(r[2], j) : nm_next(r[2], j));
    }
    o.c(')');
  };
  per("nextIndex", [&](const uint32_t* r) { idx(r, false); });
  per("matchIndex", [&](const uint32_t* r) { idx(r, true); });
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
