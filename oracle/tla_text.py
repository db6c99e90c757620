"""Parse a state printed in TLC's value syntax (rtla_state_text /
raft_values.state_text) back into the value oracle's state tuple --
TEST INFRASTRUCTURE ONLY (tests/ use it to run the value oracle's Next on
arbitrary packed states, e.g. the synthetic microbench's random ones).

The grammar is the subset those printers emit: integers, strings, model
values s<k> (servers) and v<k> (values), TRUE/FALSE, sequences <<...>>,
sets {...}, records [f |-> e, ...] and functions (k :> e @@ ...), with
<<>> also standing for the empty function (raft.tla:155 `[m \\in {} |-> 0]`).
"""
from __future__ import annotations

import re

import raft_values as rv

_TOK = re.compile(r'\s*(<<|>>|\|->|:>|@@|/\\|"[^"]*"|[A-Za-z_][A-Za-z_0-9]*|-?\d+|[\[\]{}(),=])')


def _tokens(text):
    pos, out = 0, []
    text = text.rstrip()
    while pos < len(text):
        m = _TOK.match(text, pos)
        if not m:
            raise ValueError("bad token at %r" % text[pos:pos + 20])
        out.append(m.group(1))
        pos = m.end()
    return out


class _P:
    def __init__(self, toks):
        self.t, self.k = toks, 0

    def peek(self):
        return self.t[self.k] if self.k < len(self.t) else None

    def eat(self, x=None):
        tok = self.t[self.k]
        if x is not None and tok != x:
            raise ValueError("expected %r, got %r" % (x, tok))
        self.k += 1
        return tok

    def value(self):
        tok = self.peek()
        if tok == "<<":
            self.eat()
            items = []
            while self.peek() != ">>":
                items.append(self.value())
                if self.peek() == ",":
                    self.eat()
            self.eat(">>")
            return ("seq", tuple(items))
        if tok == "{":
            self.eat()
            items = []
            while self.peek() != "}":
                items.append(self.value())
                if self.peek() == ",":
                    self.eat()
            self.eat("}")
            return ("set", items)
        if tok == "[":
            self.eat()
            rec = {}
            while self.peek() != "]":
                f = self.eat()
                self.eat("|->")
                rec[f] = self.value()
                if self.peek() == ",":
                    self.eat()
            self.eat("]")
            return ("rec", rec)
        if tok == "(":
            self.eat()
            fn = []
            while True:
                k = self.value()
                self.eat(":>")
                fn.append((k, self.value()))
                if self.peek() == "@@":
                    self.eat()
                    continue
                break
            self.eat(")")
            return ("fn", fn)
        self.eat()
        if tok.startswith('"'):
            return ("str", tok[1:-1])
        if tok in ("TRUE", "FALSE"):
            return ("bool", tok == "TRUE")
        if re.fullmatch(r"-?\d+", tok):
            return ("int", int(tok))
        m = re.fullmatch(r"([sv])(\d+)", tok)
        if m:
            return ("srv" if m.group(1) == "s" else "val", int(m.group(2)) - 1)
        raise ValueError("unexpected %r" % tok)


def _int(v):
    assert v[0] == "int", v
    return v[1]


def _srv(v):
    assert v[0] == "srv", v
    return v[1]


def _fn(v):
    """(k :> e @@ ...) or <<>> (the empty function) -> [(k, e)]."""
    if v[0] == "seq":
        assert v[1] == (), v
        return []
    assert v[0] == "fn", v
    return v[1]


def _log(v):
    assert v[0] == "seq", v
    return tuple(rv.Rec(term=_int(e[1]["term"]), value=e[1]["value"][1]) for e in v[1])


def _msg(v):
    r = v[1]
    t = r["mtype"][1]
    f = dict(mtype=t, mterm=_int(r["mterm"]), msource=_srv(r["msource"]), mdest=_srv(r["mdest"]))
    if t == rv.RVREQ:
        f.update(mlastLogTerm=_int(r["mlastLogTerm"]), mlastLogIndex=_int(r["mlastLogIndex"]))
    elif t == rv.RVRESP:
        f.update(mvoteGranted=r["mvoteGranted"][1], mlog=_log(r["mlog"]))
    elif t == rv.AEREQ:
        f.update(mprevLogIndex=_int(r["mprevLogIndex"]), mprevLogTerm=_int(r["mprevLogTerm"]),
                 mentries=_log(r["mentries"]), mlog=_log(r["mlog"]), mcommitIndex=_int(r["mcommitIndex"]))
    else:
        f.update(msuccess=r["msuccess"][1], mmatchIndex=_int(r["mmatchIndex"]))
    return rv.Rec(**f)


def _per_server(v, n, conv):
    d = {_srv(k): conv(e) for k, e in _fn(v)}
    assert sorted(d) == list(range(n)), d
    return tuple(d[i] for i in range(n))


def parse_state(cfg: rv.Cfg, text: str) -> tuple:
    """The value oracle's state tuple (raft_values.VARS order) for `text`."""
    toks = _tokens(text)
    p = _P(toks)
    vals = {}
    while p.peek() is not None:
        p.eat("/\\")
        name = p.eat()
        p.eat("=")
        vals[name] = p.value()
    n = cfg.n_server
    srvset = lambda v: frozenset(_srv(x) for x in v[1])
    voter_log = lambda v: rv.FMap({_srv(k): _log(e) for k, e in _fn(v)})
    elections = frozenset(
        rv.Rec(eterm=_int(e[1]["eterm"]), eleader=_srv(e[1]["eleader"]), elog=_log(e[1]["elog"]),
               evotes=srvset(e[1]["evotes"]), evoterLog=voter_log(e[1]["evoterLog"]))
        for e in vals["elections"][1])
    return (
        rv.FMap({_msg(k): _int(c) for k, c in _fn(vals["messages"])}),
        elections,
        frozenset(_log(x) for x in vals["allLogs"][1]),
        _per_server(vals["currentTerm"], n, _int),
        _per_server(vals["state"], n, lambda v: v[1]),
        _per_server(vals["votedFor"], n, lambda v: rv.NIL if v[0] == "str" else _srv(v)),
        _per_server(vals["log"], n, _log),
        _per_server(vals["commitIndex"], n, _int),
        _per_server(vals["votesResponded"], n, srvset),
        _per_server(vals["votesGranted"], n, srvset),
        _per_server(vals["voterLog"], n, voter_log),
        _per_server(vals["nextIndex"], n, lambda v: _per_server(v, n, _int)),
        _per_server(vals["matchIndex"], n, lambda v: _per_server(v, n, _int)),
    )
