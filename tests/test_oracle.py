"""CPU tests of the oracle itself (no GPU): known-answer tests, agreement of the
two independent restatements, and the committed golden fixtures."""
import json
import os

import pytest

import raft_cpu
import raft_values as rv

GOLD = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "bfs_counts.json")))


def level_counts_py(cfg, max_level):
    """First `max_level` BFS levels of the value oracle: (new, generated)."""
    s0 = rv.init_state(cfg)
    seen = {s0}
    out = [(1, 1)]
    frontier = [s0]
    for _ in range(max_level - 1):
        nxt, gen = [], 0
        for s in frontier:
            for _, t in rv.next_states(cfg, s):
                gen += 1
                if rv.in_model(cfg, t) and t not in seen:
                    seen.add(t)
                    nxt.append(t)
        out.append((len(nxt), gen))
        frontier = nxt
    return out


def test_kat_survey_levels_1_to_3():
    """SURVEY.md §4.3 hand-derived KATs for N=3, T=2 (raft.cfg-style):
    level 2 = 4 new / 6 generated, level 3 = 15 new / 33 generated."""
    cfg = rv.Cfg(3, 1, 2, 1, 1, ("NoTwoLeaders",))
    assert level_counts_py(cfg, 3) == [(1, 1), (4, 6), (15, 33)]
    r = raft_cpu.bfs(raft_cpu.cfg_of(3, 1, 2, 1, 1, 0, ("NoTwoLeaders",), max_distinct=20))
    assert r["levels"][:3] == [[1, 1], [4, 6], [15, 33]]


def test_init_is_unique_and_not_revisited():
    """raft.tla:155-160 has one initial state; every successor has <<>> in allLogs (:465)."""
    cfg = rv.Cfg(2, 1, 2, 1, 1, ())
    s0 = rv.init_state(cfg)
    for _, t in rv.next_states(cfg, s0):
        assert () in t[rv.IX["allLogs"]]
        assert t != s0


def test_restart_always_enabled_and_receive_exclusive():
    cfg = rv.Cfg(2, 1, 3, 1, 1, (), 1)
    # a few BFS levels: every state has >= N successors (Restart), Receive never
    # has two disjuncts enabled (SpecError would be raised)
    s0 = rv.init_state(cfg)
    seen, frontier = {s0}, [s0]
    for _ in range(8):
        nxt = []
        for s in frontier:
            succ = rv.next_states(cfg, s)
            assert sum(1 for lab, _ in succ if lab.startswith("Restart")) == cfg.n_server
            for _, t in succ:
                if rv.in_model(cfg, t) and t not in seen:
                    seen.add(t)
                    nxt.append(t)
        frontier = nxt


@pytest.mark.parametrize("name", [k for k, v in GOLD.items() if "raft_values" in v["source"]])
def test_value_oracle_matches_golden(name):
    g = GOLD[name]
    cfg = rv.Cfg(g["n_server"], g["n_value"], g["max_term"], g["max_log"], g["max_copies"],
                 tuple(g["invariants"]), g["max_msgs"])
    if g.get("symmetry"):
        assert [list(x) for x in rv.bfs_symmetric(cfg)] == g["levels"]
        return
    r = rv.bfs(cfg)
    assert [list(x) for x in r.levels] == g["levels"]
    assert r.distinct == g["distinct"] and r.generated == g["generated"] and r.depth == g["depth"]


SMALL = [k for k, v in GOLD.items() if v["distinct"] < 3_000_000 and not v.get("prefix")]


@pytest.mark.parametrize("name", SMALL)
def test_c_oracle_matches_golden(name):
    g = GOLD[name]
    cfg = raft_cpu.cfg_of(g["n_server"], g["n_value"], g["max_term"], g["max_log"], g["max_copies"],
                          g["max_msgs"], g["invariants"], symmetry=g.get("symmetry", False))
    r = raft_cpu.bfs(cfg, threads=os.cpu_count() or 4, text_hash="level_text_hash" in g)
    assert r["levels"] == g["levels"]
    assert (r["distinct"], r["generated"], r["depth"], r["violated"]) == \
        (g["distinct"], g["generated"], g["depth"], g["violated"])
    if "level_text_hash" in g:
        assert ["%016x" % h for h in r["level_text_hash"]] == g["level_text_hash"]


def test_text_format_agrees_between_oracles():
    cfg = rv.Cfg(2, 2, 3, 2, 1, (), 1)
    h_py = rv.level_text_hashes(cfg, max_states=None)[:6]
    r = raft_cpu.bfs(raft_cpu.cfg_of(2, 2, 3, 2, 1, 1, ()), text_hash=True)
    assert h_py == r["level_text_hash"][:6]


def test_c_oracle_violation_trace():
    """T=3 lets a stale term-2 leader coexist with a term-3 leader: strict
    NoTwoLeaders fails; the shortest counterexample has `depth` states."""
    g = GOLD["n3_v1_t3_l1_m1_ntl"]
    r = raft_cpu.bfs(raft_cpu.cfg_of(3, 1, 3, 1, 1, 1, ("NoTwoLeaders",)), keep_trace=True)
    assert r["violated"] == 1 and r["depth"] == g["depth"] == 19
    assert r["trace_len"] == g["depth"]
    states = r["trace_text"].strip().split("\n\n")
    assert states[0].startswith("<Initial predicate>")
    assert states[-1].count('"Leader"') >= 2


def test_walk_api_lockstep_consistency():
    w = raft_cpu.Walk(raft_cpu.cfg_of(3, 2, 3, 2, 1, 2, ()))
    succ = w.successors()
    assert len(succ) == 6                      # 3 Restart + 3 Timeout from Init
    texts = sorted(t for _, t in succ)
    w.goto(texts[-1])
    assert w.text() == texts[-1]


def test_symmetry_orbit_keys_are_permutation_invariant():
    """The two oracles' orbit machinery: every server permutation of a
    reachable state has the same orbit key, and the orbit count of a small
    model is the number of distinct orbit keys over all its states."""
    import itertools
    cfg = rv.Cfg(2, 1, 2, 1, 1, ("NoTwoLeaders",), 1)
    r = rv.bfs(cfg)
    assert r.distinct == 1760
    # all states of the non-symmetric search, by BFS
    s0 = rv.init_state(cfg)
    seen, frontier = {s0}, [s0]
    while frontier:
        nxt = []
        for s in frontier:
            for _, t in rv.next_states(cfg, s):
                if rv.in_model(cfg, t) and t not in seen:
                    seen.add(t)
                    nxt.append(t)
        frontier = nxt
    keys = {rv.orbit_key(cfg, s) for s in seen}
    assert len(keys) == GOLD["n2_v1_t2_l1_m1_sym"]["distinct"]
    some = sorted(seen, key=lambda s: rv.state_text(cfg, s))[::97]
    for s in some:
        for pi in itertools.permutations(range(2)):
            assert rv.orbit_key(cfg, rv.permute_state(s, pi)) == rv.orbit_key(cfg, s)


@pytest.mark.parametrize("shape", [(3, 1, 3, 2, 1, 0), (4, 1, 2, 1, 1, 2)])
def test_walk_orbit_texts_match_value_oracle(shape):
    """The C oracle's per-successor orbit texts (its early-exit minimum over
    all N! images) equal the value oracle's brute force, and its seen-set key
    (least orbit serialisation) groups the successors into the same orbits as
    the value oracle's least text over permutations."""
    import random
    import tla_text
    n, v, t, l, c, m = shape
    vc = rv.Cfg(n, v, t, l, c, (), m)
    w = raft_cpu.Walk(raft_cpu.cfg_of(n, v, t, l, c, m, (), symmetry=True))
    rnd = random.Random(7)
    for _ in range(25):
        succ = w.successors()
        orb = w.orbits()
        assert len(orb) == len(succ)
        by_key = {}
        for (im, tx), (key, otext) in zip(succ, orb):
            s = tla_text.parse_state(vc, tx)
            assert otext == rv.orbit_text(vc, s)
            by_key.setdefault(key, set()).add(rv.orbit_key(vc, s))
        assert all(len(x) == 1 for x in by_key.values())
        assert len(by_key) == len({k for x in by_key.values() for k in x})
        inm = [tx for im, tx in succ if im]
        if not inm:
            break
        w.goto(rnd.choice(inm))


# The BASELINE configs' shapes (N, V, MaxTerm, MaxLogLen, MaxCopies, MaxInFlight):
# configs[0] (raft.cfg bounds), configs[1], configs[2] (Duplicate/Drop live),
# configs[3] (N = 5).
BASELINE_SHAPES = [(3, 1, 2, 1, 1, 0), (3, 2, 3, 2, 1, 0), (3, 2, 4, 3, 2, 0), (5, 1, 3, 2, 1, 0)]


@pytest.mark.parametrize("shape", BASELINE_SHAPES)
def test_walk_successors_match_value_oracle(shape):
    """Along a random walk at every BASELINE shape, N = 5 included: the C
    oracle's successor multiset (state texts + in-model flags) of each state
    equals the value oracle's (raft_values.next_states, the literal
    transcription of raft.tla's Next) on the same state parsed from its text."""
    import random
    import tla_text
    n, v, t, l, c, m = shape
    vc = rv.Cfg(n, v, t, l, c, (), m)
    w = raft_cpu.Walk(raft_cpu.cfg_of(n, v, t, l, c, m, ()))
    rnd = random.Random(sum(shape) * 31 + n)
    checked = 0
    for step in range(60):
        s = tla_text.parse_state(vc, w.text())
        ref = sorted((rv.in_model(vc, x), rv.state_text(vc, x)) for _, x in rv.next_states(vc, s))
        got = sorted(w.successors())
        assert got == ref, "shape %s step %d" % (shape, step)
        checked += len(got)
        inm = [tx for im, tx in got if im]
        if not inm:
            break
        w.goto(rnd.choice(inm))
    assert checked > 300


@pytest.mark.parametrize("name,levels", [("n3_v2_t3_l2_c1_prefix", 6), ("n5_v1_t3_l2_c1_sym_prefix", 5)])
def test_value_oracle_pins_baseline_prefix(name, levels):
    """The C oracle's BASELINE fixtures are pinned by the value oracle's own
    BFS on their first levels (make_golden.py PY_PINS: every BASELINE prefix
    carries py_levels >= 7); a short prefix is re-run here: per-level counts
    and content digests (configs[3]: orbit counts and orbit-text digests)."""
    for k in ("n3_v1_t2_l1_c1_prefix", "n3_v2_t3_l2_c1_prefix", "n3_v2_t4_l3_c2_prefix",
              "n5_v1_t3_l2_c1_sym_prefix"):
        assert GOLD[k].get("py_levels", 0) >= 7, k
    g = GOLD[name]
    sym = bool(g.get("symmetry"))
    pc = rv.Cfg(g["n_server"], g["n_value"], g["max_term"], g["max_log"], g["max_copies"], tuple(g["invariants"]),
                g["max_msgs"])
    lv, hs = rv.bfs_prefix(pc, levels, symmetric=sym)
    assert [list(x) for x in lv] == g["levels"][:levels]
    assert ["%016x" % h for h in hs] == g["level_orbit_hash" if sym else "level_text_hash"][:levels]
