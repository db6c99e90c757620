// rtla_text.cpp -- TLC-style state printer for packed rows.
//
// TLC prints a state as one "/\ var = value" line per variable
// (raft.tla:32-85 declaration order).  Values use TLA+ syntax: records
// [f |-> v], functions (a :> x @@ b :> y), sequences <<...>>, sets {...};
// the empty function prints as <<>>.  Sets and the bag's domain are printed
// sorted by their text so the output is canonical (the row itself keeps the
// bag and the elections list unordered).
#include "rtla_text.h"

#include <stdio.h>

#include <algorithm>
#include <vector>

namespace rtla {

static std::string sname(uint32_t i) { return "s" + std::to_string(i + 1); }

static std::string text_log(uint32_t l) {
  uint32_t n = log_len(l);
  if (!n) return "<<>>";
  std::string s = "<<";
  for (uint32_t k = 1; k <= n; k++) {
    if (k > 1) s += ", ";
    s += "[term |-> " + std::to_string(log_term(l, k)) + ", value |-> v" + std::to_string(log_val(l, k) + 1) + "]";
  }
  return s + ">>";
}

static std::string text_srvset(uint32_t mask, int N) {
  std::string s = "{";
  bool first = true;
  for (int j = 0; j < N; j++)
    if (mask >> j & 1u) {
      if (!first) s += ", ";
      s += sname((uint32_t)j);
      first = false;
    }
  return s + "}";
}

static std::string text_vl(uint32_t dom, const uint32_t* vl, int N) {
  if (!dom) return "<<>>";
  std::string s = "(";
  bool first = true;
  for (int j = 0; j < N; j++)
    if (dom >> j & 1u) {
      if (!first) s += " @@ ";
      s += sname((uint32_t)j) + " :> " + text_log(vl[j]);
      first = false;
    }
  return s + ")";
}

static const char* BOOL(uint32_t b) { return b ? "TRUE" : "FALSE"; }

static std::string text_msg(uint64_t k) {
  static const char* TN[4] = {"RequestVoteRequest", "RequestVoteResponse", "AppendEntriesRequest",
                              "AppendEntriesResponse"};
  std::string s = "[mtype |-> \"" + std::string(TN[m_type(k)]) + "\", mterm |-> " + std::to_string(m_term(k)) + ", ";
  switch (m_type(k)) {
    case RVREQ:
      s += "mlastLogTerm |-> " + std::to_string(m_f(k, 12, 4)) + ", mlastLogIndex |-> " + std::to_string(m_f(k, 16, 3)) + ", ";
      break;
    case RVRESP:
      s += std::string("mvoteGranted |-> ") + BOOL(m_f(k, 12, 1)) + ", mlog |-> " + text_log(m_f(k, 16, 28)) + ", ";
      break;
    case AEREQ: {
      s += "mprevLogIndex |-> " + std::to_string(m_f(k, 12, 3)) + ", mprevLogTerm |-> " + std::to_string(m_f(k, 15, 4)) +
           ", mentries |-> ";
      if (m_f(k, 19, 1)) {
        uint32_t e = m_f(k, 20, 5);
        s += "<<[term |-> " + std::to_string(e & 7u) + ", value |-> v" + std::to_string((e >> 3) + 1) + "]>>";
      } else {
        s += "<<>>";
      }
      s += ", mlog |-> " + text_log(m_f(k, 28, 28)) + ", mcommitIndex |-> " + std::to_string(m_f(k, 25, 3)) + ", ";
      break;
    }
    case AERESP:
      s += std::string("msuccess |-> ") + BOOL(m_f(k, 12, 1)) + ", mmatchIndex |-> " + std::to_string(m_f(k, 13, 3)) + ", ";
      break;
  }
  s += "msource |-> " + sname(m_src(k)) + ", mdest |-> " + sname(m_dst(k)) + "]";
  return s;
}

static std::string join_sorted(std::vector<std::string> v, const char* open, const char* sep, const char* close,
                               const char* empty) {
  if (v.empty()) return empty;
  std::sort(v.begin(), v.end());
  std::string s = open;
  for (size_t k = 0; k < v.size(); k++) {
    if (k) s += sep;
    s += v[k];
  }
  return s + close;
}

std::string state_text(const Layout& L, const uint32_t* row) {
  const int N = L.N;
  std::string o;
  std::vector<std::string> items;
  int nm = row_nmsg(L, row);
  for (int k = 0; k < nm; k++) {
    uint64_t v = bag_slot(L, row, k);
    items.push_back(text_msg(m_key(v)) + " :> " + std::to_string(m_count(v)));
  }
  o += "/\\ messages = " + join_sorted(items, "(", " @@ ", ")", "<<>>");
  items.clear();
  int ne = row_nelec(L, row);
  for (int e = 0; e < ne; e++) {
    const uint32_t* r = row + L.off_elec + e * L.EW;
    uint32_t w0 = r[0];
    items.push_back("[eterm |-> " + std::to_string(w0 & 15u) + ", eleader |-> " + sname((w0 >> 4) & 7u) +
                    ", elog |-> " + text_log(r[1]) + ", evotes |-> " + text_srvset((w0 >> 7) & 31u, N) +
                    ", evoterLog |-> " + text_vl((w0 >> 12) & 31u, r + 2, N) + "]");
  }
  o += "\n/\\ elections = " + join_sorted(items, "{", ", ", "}", "{}");
  items.clear();
  for (int x = 0; x < L.n_logs; x++)
    if (row[L.off_all + (x >> 5)] >> (x & 31) & 1u) items.push_back(text_log(log_from_index(L, x)));
  o += "\n/\\ allLogs = " + join_sorted(items, "{", ", ", "}", "{}");
  auto per = [&](const char* name, auto fn) {
    o += "\n/\\ ";
    o += name;
    o += " = (";
    for (int i = 0; i < N; i++) {
      if (i) o += " @@ ";
      o += sname((uint32_t)i) + " :> " + fn(row + L.off_srv + i * L.SW);
    }
    o += ")";
  };
  static const char* RN[4] = {"\"Follower\"", "\"Candidate\"", "\"Leader\"", "\"?\""};
  per("currentTerm", [&](const uint32_t* r) { return std::to_string(s_term(r[0])); });
  per("state", [&](const uint32_t* r) { return std::string(RN[s_role(r[0])]); });
  per("votedFor", [&](const uint32_t* r) {
    return s_voted(r[0]) == NIL ? std::string("\"Nil\"") : sname(s_voted(r[0]));
  });
  per("log", [&](const uint32_t* r) { return text_log(r[1]); });
  per("commitIndex", [&](const uint32_t* r) { return std::to_string(s_commit(r[0])); });
  per("votesResponded", [&](const uint32_t* r) { return text_srvset(s_vresp(r[0]), N); });
  per("votesGranted", [&](const uint32_t* r) { return text_srvset(s_vgrant(r[0]), N); });
  per("voterLog", [&](const uint32_t* r) { return text_vl(s_vlp(r[0]), r + 3, N); });
  auto idx = [&](const uint32_t* r, bool match) {
    std::string s = "(";
    for (int j = 0; j < N; j++) {
      if (j) s += " @@ ";
      s += sname((uint32_t)j) + " :> " + std::to_string(match ? nm_match(r[2], j) : nm_next(r[2], j));
    }
    return s + ")";
  };
  per("nextIndex", [&](const uint32_t* r) { return idx(r, false); });
  per("matchIndex", [&](const uint32_t* r) { return idx(r, true); });
  return o;
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
    case F_RESTART: return "Restart(" + sname(x) + ")";
    case F_TIMEOUT: return "Timeout(" + sname(x) + ")";
    case F_REQUESTVOTE: return "RequestVote(" + sname(x / N) + ", " + sname(x % N) + ")";
    case F_BECOMELEADER: return "BecomeLeader(" + sname(x) + ")";
    case F_CLIENTREQUEST: return "ClientRequest(" + sname(x / L.V) + ", v" + std::to_string(x % L.V + 1) + ")";
    case F_ADVANCECOMMIT: return "AdvanceCommitIndex(" + sname(x) + ")";
    case F_APPENDENTRIES: return "AppendEntries(" + sname(x / N) + ", " + sname(x % N) + ")";
    case F_RECEIVE: return std::string("Receive -> ") + SUB[sub < 0 || sub > R_NONE ? R_NONE : sub];
    case F_DUPLICATE: return "DuplicateMessage";
    default: return "DropMessage";
  }
}

}  // namespace rtla
