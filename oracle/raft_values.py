"""Value-semantics oracle for raft.tla -- TEST INFRASTRUCTURE ONLY.

This module is the checker, never the product.  Only ``tests/``,
``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may use
anything under ``oracle/``.

It is a literal, slow transcription of the reference spec
``/root/reference/raft.tla`` (Diego Ongaro's Raft spec, sha256 683a120a...6b81)
over immutable Python values that follow TLA+ value equality:

* records are functions on field names  -> ``Rec`` (frozenset of items)
* functions / bags                      -> ``FMap`` (frozenset of items)
* sequences                             -> ``tuple``
* sets                                  -> ``frozenset``
* the empty function ``[x \\in {} |-> e]`` -> ``FMap()``

Server ids are the ints ``0..N-1`` (model values r1..rN); values are ``0..V-1``
(model values v1..vV).  Role and message-type constants are the strings bound
in ``/root/reference/raft.cfg:8-15``.

Every action cites the raft.tla line it transcribes.  The model-checking
wrapper (state constraint and invariants) is NOT part of the reference
(``raft.cfg:3`` names an undefined ``NoTwoLeaders`` and there is no
CONSTRAINT); the definitions used here are the build's own and are recorded
verbatim in ``specs/MC.tla`` and DESIGN.md.

Parity status: TLC (the reference's engine) cannot run in this container or on
the GPU box (no JVM), and the reference ships no tests or fixtures, so this
oracle is pinned only by hand-derived known-answer tests and by
agreement with the independent C restatement ``oracle/raft_cpu.c`` -- i.e.
"parity unpinned" against TLC itself.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Dict, Iterable, List, Optional, Tuple

# raft.cfg:8-15 -- string constants
FOLLOWER, CANDIDATE, LEADER = "Follower", "Candidate", "Leader"
NIL = "Nil"
RVREQ, RVRESP = "RequestVoteRequest", "RequestVoteResponse"
AEREQ, AERESP = "AppendEntriesRequest", "AppendEntriesResponse"


class FMap:
    """An immutable TLA+ function (also used for records and bags)."""

    __slots__ = ("_items", "_d", "_h")

    def __init__(self, d: Optional[Dict] = None):
        d = dict(d or {})
        self._d = d
        self._items = frozenset(d.items())
        self._h = hash(self._items)

    def __getitem__(self, k):
        return self._d[k]

    def __contains__(self, k):
        return k in self._d

    def domain(self):
        return self._d.keys()

    def items(self):
        return self._d.items()

    def __len__(self):
        return len(self._d)

    def __eq__(self, o):
        return isinstance(o, FMap) and self._items == o._items

    def __hash__(self):
        return self._h

    def except_(self, k, v) -> "FMap":
        d = dict(self._d)
        d[k] = v
        return FMap(d)

    def __repr__(self):
        return "FMap(%r)" % (self._d,)


def Rec(**fields) -> FMap:
    return FMap(fields)


def fn_tuple(t: tuple, i: int, v) -> tuple:
    """[f EXCEPT ![i] = v] for a function on Server represented as a tuple."""
    return t[:i] + (v,) + t[i + 1:]


@dataclass(frozen=True)
class Cfg:
    n_server: int
    n_value: int
    max_term: int
    max_log: int
    max_copies: int
    invariants: Tuple[str, ...] = ()
    max_msgs: int = 0   # 0 = unbounded; else BagCardinality(messages) <= max_msgs


# State: the 13 variables of raft.tla:32-85, as a tuple in this fixed order.
VARS = ("messages", "elections", "allLogs", "currentTerm", "state", "votedFor",
        "log", "commitIndex", "votesResponded", "votesGranted", "voterLog",
        "nextIndex", "matchIndex")
IX = {n: k for k, n in enumerate(VARS)}


def mk(s: tuple, **changes) -> tuple:
    lst = list(s)
    for k, v in changes.items():
        lst[IX[k]] = v
    return tuple(lst)


# ---------------------------------------------------------------- helpers --
def quorum(n: int, subset: frozenset) -> bool:
    """raft.tla:99  Quorum == {i \\in SUBSET(Server) : Cardinality(i)*2 > Cardinality(Server)}"""
    return len(subset) * 2 > n


def last_term(xlog: tuple) -> int:
    """raft.tla:102"""
    return 0 if len(xlog) == 0 else xlog[-1]["term"]


def with_message(m, msgs: FMap) -> FMap:
    """raft.tla:106-110"""
    if m in msgs:
        return msgs.except_(m, msgs[m] + 1)
    d = dict(msgs.items())
    d[m] = 1
    return FMap(d)


def without_message(m, msgs: FMap) -> FMap:
    """raft.tla:114-119"""
    if m in msgs:
        if msgs[m] <= 1:
            d = dict(msgs.items())
            del d[m]
            return FMap(d)
        return msgs.except_(m, msgs[m] - 1)
    return msgs


# ------------------------------------------------------------------- init --
def init_state(cfg: Cfg) -> tuple:
    """raft.tla:140-160 -- exactly one initial state."""
    n = cfg.n_server
    return (
        FMap(),                                   # messages = [m \in {} |-> 0]  :155
        frozenset(),                              # elections = {}               :140
        frozenset(),                              # allLogs = {}                 :141
        (1,) * n,                                 # currentTerm                  :143
        (FOLLOWER,) * n,                          # state                        :144
        (NIL,) * n,                               # votedFor                     :145
        ((),) * n,                                # log                          :153
        (0,) * n,                                 # commitIndex                  :154
        (frozenset(),) * n,                       # votesResponded               :146
        (frozenset(),) * n,                       # votesGranted                 :147
        (FMap(),) * n,                            # voterLog                     :142
        ((1,) * n,) * n,                          # nextIndex                    :151
        ((0,) * n,) * n,                          # matchIndex                   :152
    )


class SpecError(Exception):
    """A TLC evaluation error (e.g. a sequence index outside its domain)."""


def _seq_at(s: tuple, k: int):
    if not 1 <= k <= len(s):
        raise SpecError("sequence index %d out of domain 1..%d" % (k, len(s)))
    return s[k - 1]


# ---------------------------------------------------------------- actions --
# Each generator yields (label, successor-without-allLogs).  Next (:454-465)
# then conjoins allLogs' = allLogs \cup {log[i] : i \in Server}.

def restart(cfg, s, i):
    """raft.tla:167-175"""
    n = cfg.n_server
    g = lambda k: s[IX[k]]
    return mk(s,
              state=fn_tuple(g("state"), i, FOLLOWER),
              votesResponded=fn_tuple(g("votesResponded"), i, frozenset()),
              votesGranted=fn_tuple(g("votesGranted"), i, frozenset()),
              voterLog=fn_tuple(g("voterLog"), i, FMap()),
              nextIndex=fn_tuple(g("nextIndex"), i, (1,) * n),
              matchIndex=fn_tuple(g("matchIndex"), i, (0,) * n),
              commitIndex=fn_tuple(g("commitIndex"), i, 0))


def timeout(cfg, s, i):
    """raft.tla:178-187"""
    g = lambda k: s[IX[k]]
    if g("state")[i] not in (FOLLOWER, CANDIDATE):
        return None
    return mk(s,
              state=fn_tuple(g("state"), i, CANDIDATE),
              currentTerm=fn_tuple(g("currentTerm"), i, g("currentTerm")[i] + 1),
              votedFor=fn_tuple(g("votedFor"), i, NIL),
              votesResponded=fn_tuple(g("votesResponded"), i, frozenset()),
              votesGranted=fn_tuple(g("votesGranted"), i, frozenset()),
              voterLog=fn_tuple(g("voterLog"), i, FMap()))


def request_vote(cfg, s, i, j):
    """raft.tla:190-199"""
    g = lambda k: s[IX[k]]
    if g("state")[i] != CANDIDATE or j in g("votesResponded")[i]:
        return None
    lg = g("log")[i]
    m = Rec(mtype=RVREQ, mterm=g("currentTerm")[i], mlastLogTerm=last_term(lg),
            mlastLogIndex=len(lg), msource=i, mdest=j)
    return mk(s, messages=with_message(m, g("messages")))


def append_entries(cfg, s, i, j):
    """raft.tla:204-226"""
    g = lambda k: s[IX[k]]
    if i == j or g("state")[i] != LEADER:
        return None
    lg = g("log")[i]
    nxt = g("nextIndex")[i][j]
    prev_idx = nxt - 1
    prev_term = _seq_at(lg, prev_idx)["term"] if prev_idx > 0 else 0
    last_entry = min(len(lg), nxt)
    entries = tuple(lg[nxt - 1:last_entry]) if nxt <= last_entry else ()  # SubSeq(log, nxt, lastEntry)
    m = Rec(mtype=AEREQ, mterm=g("currentTerm")[i], mprevLogIndex=prev_idx,
            mprevLogTerm=prev_term, mentries=entries, mlog=lg,
            mcommitIndex=min(g("commitIndex")[i], last_entry), msource=i, mdest=j)
    return mk(s, messages=with_message(m, g("messages")))


def become_leader(cfg, s, i):
    """raft.tla:229-243"""
    n = cfg.n_server
    g = lambda k: s[IX[k]]
    if g("state")[i] != CANDIDATE or not quorum(n, g("votesGranted")[i]):
        return None
    lg = g("log")[i]
    e = Rec(eterm=g("currentTerm")[i], eleader=i, elog=lg,
            evotes=g("votesGranted")[i], evoterLog=g("voterLog")[i])
    return mk(s,
              state=fn_tuple(g("state"), i, LEADER),
              nextIndex=fn_tuple(g("nextIndex"), i, (len(lg) + 1,) * n),
              matchIndex=fn_tuple(g("matchIndex"), i, (0,) * n),
              elections=g("elections") | {e})


def client_request(cfg, s, i, v):
    """raft.tla:246-253"""
    g = lambda k: s[IX[k]]
    if g("state")[i] != LEADER:
        return None
    entry = Rec(term=g("currentTerm")[i], value=v)
    return mk(s, log=fn_tuple(g("log"), i, g("log")[i] + (entry,)))


def advance_commit_index(cfg, s, i):
    """raft.tla:259-276"""
    n = cfg.n_server
    g = lambda k: s[IX[k]]
    if g("state")[i] != LEADER:
        return None
    lg = g("log")[i]
    mi = g("matchIndex")[i]

    def agree(index):
        return frozenset([i]) | frozenset(k for k in range(n) if mi[k] >= index)

    agree_indexes = [index for index in range(1, len(lg) + 1) if quorum(n, agree(index))]
    if agree_indexes and _seq_at(lg, max(agree_indexes))["term"] == g("currentTerm")[i]:
        nci = max(agree_indexes)
    else:
        nci = g("commitIndex")[i]
    return mk(s, commitIndex=fn_tuple(g("commitIndex"), i, nci))


def handle_request_vote_request(cfg, s, i, j, m):
    """raft.tla:284-303"""
    g = lambda k: s[IX[k]]
    lg = g("log")[i]
    log_ok = (m["mlastLogTerm"] > last_term(lg)) or (
        m["mlastLogTerm"] == last_term(lg) and m["mlastLogIndex"] >= len(lg))
    grant = m["mterm"] == g("currentTerm")[i] and log_ok and g("votedFor")[i] in (NIL, j)
    if not m["mterm"] <= g("currentTerm")[i]:
        return None
    vf = fn_tuple(g("votedFor"), i, j) if grant else g("votedFor")
    resp = Rec(mtype=RVRESP, mterm=g("currentTerm")[i], mvoteGranted=grant,
               mlog=lg, msource=i, mdest=j)
    return mk(s, votedFor=vf,
              messages=without_message(m, with_message(resp, g("messages"))))


def handle_request_vote_response(cfg, s, i, j, m):
    """raft.tla:307-321"""
    g = lambda k: s[IX[k]]
    if m["mterm"] != g("currentTerm")[i]:
        return None
    vr = fn_tuple(g("votesResponded"), i, g("votesResponded")[i] | {j})
    if m["mvoteGranted"]:
        vg = fn_tuple(g("votesGranted"), i, g("votesGranted")[i] | {j})
        # voterLog[i] @@ (j :> m.mlog): @@ keeps the LEFT operand's value on overlap
        old = g("voterLog")[i]
        if j in old:
            new_vl = old
        else:
            d = dict(old.items())
            d[j] = m["mlog"]
            new_vl = FMap(d)
        vl = fn_tuple(g("voterLog"), i, new_vl)
    else:
        vg, vl = g("votesGranted"), g("voterLog")
    return mk(s, votesResponded=vr, votesGranted=vg, voterLog=vl,
              messages=without_message(m, g("messages")))


def handle_append_entries_request(cfg, s, i, j, m):
    """raft.tla:327-389"""
    g = lambda k: s[IX[k]]
    lg = g("log")[i]
    cur = g("currentTerm")[i]
    st = g("state")[i]
    pli = m["mprevLogIndex"]
    log_ok = pli == 0 or (pli > 0 and pli <= len(lg) and m["mprevLogTerm"] == _seq_at(lg, pli)["term"])
    if not m["mterm"] <= cur:
        return None
    results = []
    # reject request  :333-345
    if m["mterm"] < cur or (m["mterm"] == cur and st == FOLLOWER and not log_ok):
        resp = Rec(mtype=AERESP, mterm=cur, msuccess=False, mmatchIndex=0, msource=i, mdest=j)
        results.append(mk(s, messages=without_message(m, with_message(resp, g("messages")))))
    # return to follower state  :346-350
    if m["mterm"] == cur and st == CANDIDATE:
        results.append(mk(s, state=fn_tuple(g("state"), i, FOLLOWER)))
    # accept request  :351-388
    if m["mterm"] == cur and st == FOLLOWER and log_ok:
        index = pli + 1
        ents = m["mentries"]
        # already done with request  :356-374
        if ents == () or (ents != () and len(lg) >= index and _seq_at(lg, index)["term"] == ents[0]["term"]):
            resp = Rec(mtype=AERESP, mterm=cur, msuccess=True, mmatchIndex=pli + len(ents),
                       msource=i, mdest=j)
            results.append(mk(s, commitIndex=fn_tuple(g("commitIndex"), i, m["mcommitIndex"]),
                              messages=without_message(m, with_message(resp, g("messages")))))
        # conflict: remove 1 entry  :375-382
        if ents != () and len(lg) >= index and _seq_at(lg, index)["term"] != ents[0]["term"]:
            new = tuple(lg[:len(lg) - 1])
            results.append(mk(s, log=fn_tuple(g("log"), i, new)))
        # no conflict: append entry  :383-388
        if ents != () and len(lg) == pli:
            results.append(mk(s, log=fn_tuple(g("log"), i, lg + (ents[0],))))
    if len(results) > 1:
        raise SpecError("HandleAppendEntriesRequest: %d branches enabled" % len(results))
    return results[0] if results else None


def handle_append_entries_response(cfg, s, i, j, m):
    """raft.tla:393-403"""
    g = lambda k: s[IX[k]]
    if m["mterm"] != g("currentTerm")[i]:
        return None
    ni, mi = g("nextIndex"), g("matchIndex")
    if m["msuccess"]:
        ni = fn_tuple(ni, i, fn_tuple(ni[i], j, m["mmatchIndex"] + 1))
        mi = fn_tuple(mi, i, fn_tuple(mi[i], j, m["mmatchIndex"]))
    else:
        ni = fn_tuple(ni, i, fn_tuple(ni[i], j, max(ni[i][j] - 1, 1)))
    return mk(s, nextIndex=ni, matchIndex=mi, messages=without_message(m, g("messages")))


def update_term(cfg, s, i, j, m):
    """raft.tla:406-412"""
    g = lambda k: s[IX[k]]
    if not m["mterm"] > g("currentTerm")[i]:
        return None
    return mk(s,
              currentTerm=fn_tuple(g("currentTerm"), i, m["mterm"]),
              state=fn_tuple(g("state"), i, FOLLOWER),
              votedFor=fn_tuple(g("votedFor"), i, NIL))


def drop_stale_response(cfg, s, i, j, m):
    """raft.tla:415-418"""
    g = lambda k: s[IX[k]]
    if not m["mterm"] < g("currentTerm")[i]:
        return None
    return mk(s, messages=without_message(m, g("messages")))


def receive(cfg, s, m):
    """raft.tla:421-436 -- returns the (unique) successor or None."""
    i, j = m["mdest"], m["msource"]
    out = []
    r = update_term(cfg, s, i, j, m)
    if r is not None:
        out.append(("UpdateTerm", r))
    t = m["mtype"]
    if t == RVREQ:
        r = handle_request_vote_request(cfg, s, i, j, m)
        if r is not None:
            out.append(("HandleRequestVoteRequest", r))
    elif t == RVRESP:
        for name, fn in (("DropStaleResponse", drop_stale_response),
                         ("HandleRequestVoteResponse", handle_request_vote_response)):
            r = fn(cfg, s, i, j, m)
            if r is not None:
                out.append((name, r))
    elif t == AEREQ:
        r = handle_append_entries_request(cfg, s, i, j, m)
        if r is not None:
            out.append(("HandleAppendEntriesRequest", r))
    elif t == AERESP:
        for name, fn in (("DropStaleResponse", drop_stale_response),
                         ("HandleAppendEntriesResponse", handle_append_entries_response)):
            r = fn(cfg, s, i, j, m)
            if r is not None:
                out.append((name, r))
    if len(out) > 1:
        raise SpecError("Receive: %d disjuncts enabled" % len(out))
    return out[0] if out else None


def duplicate_message(cfg, s, m):
    """raft.tla:443-445"""
    return mk(s, messages=with_message(m, s[IX["messages"]]))


def drop_message(cfg, s, m):
    """raft.tla:448-450"""
    return mk(s, messages=without_message(m, s[IX["messages"]]))


def next_states(cfg: Cfg, s: tuple) -> List[Tuple[str, tuple]]:
    """raft.tla:454-465 -- one (label, successor) per enabled instance.

    The enumeration order of the families follows the disjunct order of Next;
    within a family servers/values ascend.  Message instances enumerate
    DOMAIN messages (distinct messages, not copies)."""
    n, nv = cfg.n_server, cfg.n_value
    out: List[Tuple[str, tuple]] = []

    def add(label, r):
        if r is not None:
            out.append((label, r))

    for i in range(n):
        add("Restart(%d)" % i, restart(cfg, s, i))
    for i in range(n):
        add("Timeout(%d)" % i, timeout(cfg, s, i))
    for i in range(n):
        for j in range(n):
            add("RequestVote(%d,%d)" % (i, j), request_vote(cfg, s, i, j))
    for i in range(n):
        add("BecomeLeader(%d)" % i, become_leader(cfg, s, i))
    for i in range(n):
        for v in range(nv):
            add("ClientRequest(%d,%d)" % (i, v), client_request(cfg, s, i, v))
    for i in range(n):
        add("AdvanceCommitIndex(%d)" % i, advance_commit_index(cfg, s, i))
    for i in range(n):
        for j in range(n):
            add("AppendEntries(%d,%d)" % (i, j), append_entries(cfg, s, i, j))
    msgs = list(s[IX["messages"]].domain())
    for m in msgs:
        r = receive(cfg, s, m)
        if r is not None:
            out.append(("Receive:" + r[0], r[1]))
    for m in msgs:
        add("DuplicateMessage", duplicate_message(cfg, s, m))
    for m in msgs:
        add("DropMessage", drop_message(cfg, s, m))
    # allLogs' = allLogs \cup {log[i] : i \in Server}   (pre-state log!)  :465
    al = s[IX["allLogs"]] | frozenset(s[IX["log"]])
    return [(lab, mk(r, allLogs=al)) for lab, r in out]


# -------------------------------------------- build-defined MC wrapper ----
# Recorded verbatim in specs/MC.tla.  NOT part of the reference.

def in_model(cfg: Cfg, s: tuple) -> bool:
    """StateConstraint == /\\ \\A i \\in Server : currentTerm[i] <= MaxTerm
                          /\\ \\A i \\in Server : Len(log[i]) <= MaxLogLen
                          /\\ \\A m \\in DOMAIN messages : messages[m] <= MaxCopies
                          /\\ MaxInFlight = 0 \\/ BagCardinality(messages) <= MaxInFlight"""
    msgs = s[IX["messages"]]
    return (all(t <= cfg.max_term for t in s[IX["currentTerm"]])
            and all(len(l) <= cfg.max_log for l in s[IX["log"]])
            and all(c <= cfg.max_copies for _, c in msgs.items())
            and (cfg.max_msgs == 0 or sum(c for _, c in msgs.items()) <= cfg.max_msgs))


def inv_no_two_leaders(cfg, s) -> bool:
    """NoTwoLeaders == \\A i, j \\in Server : (state[i] = Leader /\\ state[j] = Leader) => i = j"""
    return sum(1 for r in s[IX["state"]] if r == LEADER) <= 1


def inv_election_safety(cfg, s) -> bool:
    """ElectionSafety == \\A e, f \\in elections : e.eterm = f.eterm => e.eleader = f.eleader"""
    seen = {}
    for e in s[IX["elections"]]:
        if seen.setdefault(e["eterm"], e["eleader"]) != e["eleader"]:
            return False
    return True


def inv_log_matching(cfg, s) -> bool:
    """LogMatching == \\A i, j \\in Server : \\A n \\in 1..Min({Len(log[i]), Len(log[j])}) :
                        log[i][n].term = log[j][n].term => SubSeq(log[i],1,n) = SubSeq(log[j],1,n)"""
    logs = s[IX["log"]]
    n = cfg.n_server
    for i in range(n):
        for j in range(n):
            a, b = logs[i], logs[j]
            for k in range(1, min(len(a), len(b)) + 1):
                if a[k - 1]["term"] == b[k - 1]["term"] and a[:k] != b[:k]:
                    return False
    return True


INVARIANTS = {
    "NoTwoLeaders": inv_no_two_leaders,
    "ElectionSafety": inv_election_safety,
    "LogMatching": inv_log_matching,
}


@dataclass
class BfsResult:
    levels: List[Tuple[int, int]]  # per level: (distinct new, generated from the previous level)
    distinct: int
    generated: int
    depth: int
    violation: Optional[str] = None
    trace: Optional[List[Tuple[str, tuple]]] = None
    max_msgs: int = 0


def bfs(cfg: Cfg, max_states: Optional[int] = None) -> BfsResult:
    """Level-synchronous BFS with TLC's counting conventions:

    * generated counts the initial state plus every enabled instance of Next,
      including successors outside the state constraint;
    * out-of-model successors are invariant-checked but never stored;
    * invariants are checked on every newly seen state;
    * depth = number of BFS levels, Init = level 1."""
    s0 = init_state(cfg)
    parent: Dict[tuple, Optional[Tuple[tuple, str]]] = {s0: None}
    levels = [(1, 1)]
    generated = 1
    frontier = [s0]
    max_msgs = 0

    def check(st):
        for name in cfg.invariants:
            if not INVARIANTS[name](cfg, st):
                return name
        return None

    def trace_to(st, last=None):
        tr = []
        cur = st
        while cur is not None:
            p = parent[cur]
            tr.append((p[1] if p else "Init", cur))
            cur = p[0] if p else None
        tr.reverse()
        if last is not None:
            tr.append(last)
        return tr

    bad = check(s0)
    if bad:
        return BfsResult(levels, 1, 1, 1, bad, trace_to(s0))
    while frontier:
        nxt = []
        gen = 0
        for s in frontier:
            for lab, t in next_states(cfg, s):
                gen += 1
                if in_model(cfg, t):
                    if t in parent:
                        continue
                    parent[t] = (s, lab)
                    nxt.append(t)
                    max_msgs = max(max_msgs, len(t[IX["messages"]]))
                    bad = check(t)
                    if bad:
                        levels.append((len(nxt), gen))
                        return BfsResult(levels, len(parent), generated + gen, len(levels), bad,
                                         trace_to(t), max_msgs)
                else:
                    bad = check(t)
                    if bad:
                        levels.append((len(nxt), gen))
                        return BfsResult(levels, len(parent), generated + gen, len(levels), bad,
                                         trace_to(s, (lab, t)), max_msgs)
            if max_states and len(parent) > max_states:
                raise RuntimeError("state budget exceeded")
        generated += gen
        if not nxt:
            # the final level generated only already-seen states
            levels.append((0, gen))
            break
        levels.append((len(nxt), gen))
        frontier = nxt
    depth = sum(1 for d, _ in levels if d > 0)
    return BfsResult(levels, len(parent), generated, depth, None, None, max_msgs)


# --------------------------------------------------------------- symmetry --
# SYMMETRY Permutations(Server) (specs/MC.tla).  pi maps server i to pi[i];
# every server-valued field is relabelled and every function on Server
# re-indexed.  An independent restatement of oracle/raft_cpu.c's orbit key.
def permute_state(s: tuple, pi) -> tuple:
    def srv(x):
        return x if x == NIL else pi[x]

    def sset(fs):
        return frozenset(pi[x] for x in fs)

    def on_server(t):  # a function on Server, as a tuple
        out = [None] * len(t)
        for i, v in enumerate(t):
            out[pi[i]] = v
        return tuple(out)

    def msg(m):
        d = dict(m.items())
        d["msource"], d["mdest"] = pi[d["msource"]], pi[d["mdest"]]
        return FMap(d)

    def elec(e):
        d = dict(e.items())
        d["eleader"] = pi[d["eleader"]]
        d["evotes"] = sset(d["evotes"])
        d["evoterLog"] = FMap({pi[k]: v for k, v in d["evoterLog"].items()})
        return FMap(d)

    msgs = FMap({msg(m): c for m, c in s[IX["messages"]].items()})
    return (
        msgs,
        frozenset(elec(e) for e in s[IX["elections"]]),
        s[IX["allLogs"]],
        on_server(s[IX["currentTerm"]]),
        on_server(s[IX["state"]]),
        on_server(tuple(srv(v) for v in s[IX["votedFor"]])),
        on_server(s[IX["log"]]),
        on_server(s[IX["commitIndex"]]),
        on_server(tuple(sset(v) for v in s[IX["votesResponded"]])),
        on_server(tuple(sset(v) for v in s[IX["votesGranted"]])),
        on_server(tuple(FMap({pi[k]: v for k, v in f.items()}) for f in s[IX["voterLog"]])),
        on_server(tuple(on_server(row) for row in s[IX["nextIndex"]])),
        on_server(tuple(on_server(row) for row in s[IX["matchIndex"]])),
    )


def orbit_key(cfg: Cfg, s: tuple) -> str:
    """The least canonical text over all server permutations of s."""
    import itertools
    return min(state_text(cfg, permute_state(s, pi)) for pi in itertools.permutations(range(cfg.n_server)))


def rotated_text(cfg: Cfg, s: tuple) -> str:
    """The state text with its three lines that are no function on Server
    (messages, elections, allLogs) moved after the ten per-server lines."""
    lines = state_text(cfg, s).split("\n")
    return "\n".join(lines[3:] + lines[:3])


def orbit_text(cfg: Cfg, s: tuple) -> str:
    """The orbit text of s: the state text of the image whose rotated text is
    least over all server permutations -- a function of the orbit alone, the
    per-orbit item of a SYMMETRY level's digest (oracle/raft_cpu.c orbit_text,
    the product's rtla_level_orbit_hash).  Brute force over every image."""
    import itertools
    imgs = (permute_state(s, pi) for pi in itertools.permutations(range(cfg.n_server)))
    return state_text(cfg, min(imgs, key=lambda t: rotated_text(cfg, t)))


def bfs_symmetric(cfg: Cfg, orbit_hashes: Optional[List[int]] = None) -> List[Tuple[int, int]]:
    """Per-level (new orbits, generated) of the BFS under SYMMETRY
    Permutations(Server): a successor is new iff no state of its orbit was
    seen; the state itself (not a representative) is explored, as in TLC.
    orbit_hashes (a list) receives each level's digest: the sum mod 2^64 of
    FNV-1a(orbit_text) over its new orbits."""
    s0 = init_state(cfg)
    seen = {orbit_key(cfg, s0)}
    levels, frontier = [(1, 1)], [s0]
    if orbit_hashes is not None:
        orbit_hashes.append(fnv1a64(orbit_text(cfg, s0)))
    while frontier:
        nxt, gen = [], 0
        for s in frontier:
            for _lab, t in next_states(cfg, s):
                gen += 1
                if in_model(cfg, t):
                    k = orbit_key(cfg, t)
                    if k not in seen:
                        seen.add(k)
                        nxt.append(t)
        levels.append((len(nxt), gen))
        if orbit_hashes is not None:
            orbit_hashes.append(sum(fnv1a64(orbit_text(cfg, t)) for t in nxt) & 0xFFFFFFFFFFFFFFFF)
        frontier = nxt
    return levels


# ------------------------------------------------------------ state text --
# Canonical TLC-like text; must be byte-identical to oracle/raft_cpu.c's
# state_text (sets and the bag's domain sorted by their text).
def _t_log(lg) -> str:
    if not lg:
        return "<<>>"
    return "<<" + ", ".join("[term |-> %d, value |-> v%d]" % (e["term"], e["value"] + 1) for e in lg) + ">>"


def _t_srvset(s) -> str:
    return "{" + ", ".join("s%d" % (j + 1) for j in sorted(s)) + "}"


def _t_vl(f: FMap) -> str:
    if len(f) == 0:
        return "<<>>"
    return "(" + " @@ ".join("s%d :> %s" % (j + 1, _t_log(f[j])) for j in sorted(f.domain())) + ")"


def _t_bool(b) -> str:
    return "TRUE" if b else "FALSE"


def _t_msg(m) -> str:
    t = m["mtype"]
    s = '[mtype |-> "%s", mterm |-> %d, ' % (t, m["mterm"])
    if t == RVREQ:
        s += "mlastLogTerm |-> %d, mlastLogIndex |-> %d, " % (m["mlastLogTerm"], m["mlastLogIndex"])
    elif t == RVRESP:
        s += "mvoteGranted |-> %s, mlog |-> %s, " % (_t_bool(m["mvoteGranted"]), _t_log(m["mlog"]))
    elif t == AEREQ:
        s += "mprevLogIndex |-> %d, mprevLogTerm |-> %d, mentries |-> %s, mlog |-> %s, mcommitIndex |-> %d, " % (
            m["mprevLogIndex"], m["mprevLogTerm"], _t_log(m["mentries"]), _t_log(m["mlog"]), m["mcommitIndex"])
    else:
        s += "msuccess |-> %s, mmatchIndex |-> %d, " % (_t_bool(m["msuccess"]), m["mmatchIndex"])
    return s + "msource |-> s%d, mdest |-> s%d]" % (m["msource"] + 1, m["mdest"] + 1)


def _join(items, op, sep, cl, empty):
    if not items:
        return empty
    return op + sep.join(sorted(items)) + cl


def state_text(cfg: Cfg, s: tuple) -> str:
    n = cfg.n_server
    g = lambda k: s[IX[k]]
    out = "/\\ messages = " + _join(["%s :> %d" % (_t_msg(m), c) for m, c in g("messages").items()],
                                    "(", " @@ ", ")", "<<>>")
    els = []
    for e in g("elections"):
        els.append("[eterm |-> %d, eleader |-> s%d, elog |-> %s, evotes |-> %s, evoterLog |-> %s]" % (
            e["eterm"], e["eleader"] + 1, _t_log(e["elog"]), _t_srvset(e["evotes"]), _t_vl(e["evoterLog"])))
    out += "\n/\\ elections = " + _join(els, "{", ", ", "}", "{}")
    out += "\n/\\ allLogs = " + _join([_t_log(l) for l in g("allLogs")], "{", ", ", "}", "{}")

    def per(name, fn):
        return "\n/\\ %s = (" % name + " @@ ".join("s%d :> %s" % (i + 1, fn(i)) for i in range(n)) + ")"

    out += per("currentTerm", lambda i: str(g("currentTerm")[i]))
    out += per("state", lambda i: '"%s"' % g("state")[i])
    out += per("votedFor", lambda i: '"Nil"' if g("votedFor")[i] == NIL else "s%d" % (g("votedFor")[i] + 1))
    out += per("log", lambda i: _t_log(g("log")[i]))
    out += per("commitIndex", lambda i: str(g("commitIndex")[i]))
    out += per("votesResponded", lambda i: _t_srvset(g("votesResponded")[i]))
    out += per("votesGranted", lambda i: _t_srvset(g("votesGranted")[i]))
    out += per("voterLog", lambda i: _t_vl(g("voterLog")[i]))
    fn2 = lambda f: "(" + " @@ ".join("s%d :> %d" % (j + 1, f[j]) for j in range(n)) + ")"
    out += per("nextIndex", lambda i: fn2(g("nextIndex")[i]))
    out += per("matchIndex", lambda i: fn2(g("matchIndex")[i]))
    return out


def fnv1a64(text: str) -> int:
    h = 0xcbf29ce484222325
    for b in text.encode():
        h ^= b
        h = (h * 0x100000001b3) & 0xFFFFFFFFFFFFFFFF
    return h


def level_text_hashes(cfg: Cfg, max_states: Optional[int] = None) -> List[int]:
    """Per BFS level: sum mod 2^64 of FNV-1a(state_text) over the new states."""
    s0 = init_state(cfg)
    seen = {s0}
    out = [fnv1a64(state_text(cfg, s0))]
    frontier = [s0]
    while frontier:
        nxt = []
        for s in frontier:
            for _, t in next_states(cfg, s):
                if in_model(cfg, t) and t not in seen:
                    seen.add(t)
                    nxt.append(t)
        if not nxt:
            break
        out.append(sum(fnv1a64(state_text(cfg, t)) for t in nxt) & 0xFFFFFFFFFFFFFFFF)
        frontier = nxt
        if max_states and len(seen) > max_states:
            raise RuntimeError("state budget exceeded")
    return out


def bfs_prefix(cfg: Cfg, max_levels: int, symmetric: bool = False) -> Tuple[List[Tuple[int, int]], List[int]]:
    """The first `max_levels` BFS levels (Init = level 1): per level (new,
    generated) and its content digest -- the sum mod 2^64 of FNV-1a over the
    new states' texts, or (symmetric: SYMMETRY Permutations(Server)) over the
    new orbits' orbit texts.  The same conventions as bfs / bfs_symmetric, cut
    after a level count instead of run to exhaustion: pins the C oracle's
    fixtures of the BASELINE configs (which no oracle exhausts) on their
    first levels (tests/golden/make_golden.py PY_PINS)."""
    s0 = init_state(cfg)
    key = (lambda t: orbit_key(cfg, t)) if symmetric else (lambda t: t)
    text = (lambda t: orbit_text(cfg, t)) if symmetric else (lambda t: state_text(cfg, t))
    seen = {key(s0)}
    levels, hashes, frontier = [(1, 1)], [fnv1a64(text(s0))], [s0]
    while frontier and len(levels) < max_levels:
        nxt, gen = [], 0
        for s in frontier:
            for _lab, t in next_states(cfg, s):
                gen += 1
                if in_model(cfg, t):
                    k = key(t)
                    if k not in seen:
                        seen.add(k)
                        nxt.append(t)
        levels.append((len(nxt), gen))
        hashes.append(sum(fnv1a64(text(t)) for t in nxt) & 0xFFFFFFFFFFFFFFFF)
        frontier = nxt
    return levels, hashes
