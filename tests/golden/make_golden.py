"""Generate the golden BFS fixtures in tests/golden/bfs_counts.json.

Each case is run through the C oracle (oracle/raft_cpu.c); cases marked
"py" are also run through the value-semantics oracle (oracle/raft_values.py)
and the two must agree on every level's counts and state-text hash before the
case is written.  The configs are the build's bounded models (specs/MC.tla);
the reference ships no fixtures of its own.

    python tests/golden/make_golden.py [--big] [--py-pins] [--only=name,name]
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import raft_cpu  # noqa: E402
import raft_values as rv  # noqa: E402

NTL, ES, LM = "NoTwoLeaders", "ElectionSafety", "LogMatching"
# name: (N, V, T, L, C, M, invariants, py, big)
CASES = {
    "n1_v1_t2_l1": (1, 1, 2, 1, 1, 0, (NTL,), True, False),
    "n1_v2_t3_l2": (1, 2, 3, 2, 1, 0, (NTL, ES, LM), True, False),
    "n2_v1_t2_l1_m1": (2, 1, 2, 1, 1, 1, (NTL,), True, False),
    "n2_v1_t3_l1_m1": (2, 1, 3, 1, 1, 1, (NTL, ES, LM), True, False),
    "n2_v1_t2_l1_c2_m2": (2, 1, 2, 1, 2, 2, (NTL,), False, False),
    "n2_v2_t3_l2_m1": (2, 2, 3, 2, 1, 1, (ES, LM), False, False),
    "n3_v1_t3_l1_m1_ntl": (3, 1, 3, 1, 1, 1, (NTL,), False, False),
    "n3_v1_t2_l1_m1": (3, 1, 2, 1, 1, 1, (NTL,), False, False),
    "n2_v1_t2_l1": (2, 1, 2, 1, 1, 0, (NTL,), False, True),
    "n3_v1_t2_l1_m2": (3, 1, 2, 1, 1, 2, (NTL,), False, True),
    "n3_v2_t2_l1_m2": (3, 2, 2, 1, 1, 2, (ES, LM), False, True),
}
# SYMMETRY Permutations(Server) (specs/MC.tla): per-level orbit counts.  "py"
# cases are also run through the value oracle's independent orbit BFS.
# name: (N, V, T, L, C, M, invariants, py, big)
SYM_CASES = {
    "n2_v1_t2_l1_m1_sym": (2, 1, 2, 1, 1, 1, (NTL,), True, False),
    "n2_v1_t3_l1_m1_sym": (2, 1, 3, 1, 1, 1, (NTL, ES, LM), True, False),
    "n3_v1_t2_l1_m1_sym": (3, 1, 2, 1, 1, 1, (NTL,), False, False),
    "n3_v1_t3_l1_m1_ntl_sym": (3, 1, 3, 1, 1, 1, (NTL,), False, False),
    "n3_v1_t2_l1_m2_sym": (3, 1, 2, 1, 1, 2, (NTL,), False, True),
}
# Models too large for the CPU oracle to exhaust here: a bounded prefix of
# complete BFS levels, with each level's state-text hash.  The oracle stops
# after the first level that passes max_distinct, or after max_levels levels
# (its last level counted, hashed and deduplicated but not kept: one level
# deeper in the same memory).  The BASELINE configs are pinned to the depth
# bench.py times them at (the levels that fit one MI355X's HBM).
# name: (N, V, T, L, C, M, invariants, max_distinct, max_levels)
PREFIXES = {
    # bench.py's exhaust model (wall time to exhaust)
    "n3_v2_t2_l2_m2_prefix": (3, 2, 2, 2, 1, 2, (ES, LM), 200_000_000, 0),
    # BASELINE.json configs[1] and configs[0] exactly as stated (no in-flight bound)
    "n3_v2_t3_l2_c1_prefix": (3, 2, 3, 2, 1, 0, (ES, LM), 0, 17),
    "n3_v1_t2_l1_c1_prefix": (3, 1, 2, 1, 1, 0, (NTL,), 0, 23),
    # BASELINE.json configs[2] as stated (2 copies per message: Duplicate/Drop live)
    "n3_v2_t4_l3_c2_prefix": (3, 2, 4, 3, 2, 0, (), 0, 14),
}
# SYMMETRY prefixes: orbit counts and orbit-text digests per level (the
# orbit text is the same whichever member of an orbit an implementation
# keeps).  N = 4, and BASELINE configs[3] (N = 5) as stated to the 15 levels
# bench.py times.
# name: (N, V, T, L, C, M, invariants, max_distinct, max_levels)
SYM_PREFIXES = {
    "n4_v1_t2_l1_m1_sym_prefix": (4, 1, 2, 1, 1, 1, (NTL,), 3_000_000, 0),
    "n5_v1_t3_l2_c1_sym_prefix": (5, 1, 3, 2, 1, 0, (), 0, 15),
}


# The value oracle's own BFS over the first levels of the BASELINE prefixes
# (the C oracle's fixtures above): per-level counts and content digests must
# agree before "py_levels" is recorded -- the value semantics touch every
# BASELINE shape (configs[0]-[3]; configs[3] through its orbit texts).
# name: levels (as many as the pure-Python transcription finishes in minutes)
PY_PINS = {
    "n3_v1_t2_l1_c1_prefix": 11,      # configs[0]: 103,165 states
    "n3_v2_t3_l2_c1_prefix": 9,       # configs[1]: 74,048 states
    "n3_v2_t4_l3_c2_prefix": 8,       # configs[2]: 48,290 states
    "n5_v1_t3_l2_c1_sym_prefix": 7,   # configs[3]: 1,501 orbits (all 120 images of every successor)
}


def pin_with_value_oracle(out, only):
    for name, k in PY_PINS.items():
        if (only and name not in only) or name not in out:
            continue
        g = out[name]
        sym = bool(g.get("symmetry"))
        pc = rv.Cfg(g["n_server"], g["n_value"], g["max_term"], g["max_log"], g["max_copies"],
                    tuple(g["invariants"]), g["max_msgs"])
        levels, hashes = rv.bfs_prefix(pc, k, symmetric=sym)
        want = g["level_orbit_hash" if sym else "level_text_hash"]
        assert [list(x) for x in levels] == g["levels"][:k], name
        assert ["%016x" % h for h in hashes] == want[:k], name
        g["py_levels"] = k
        print(name, "value oracle agrees on the first %d levels" % k, flush=True)


def main():
    big = "--big" in sys.argv
    only = [a.split("=", 1)[1] for a in sys.argv if a.startswith("--only=")]
    only = set(only[0].split(",")) if only else None
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "bfs_counts.json")
    out = json.load(open(path)) if os.path.exists(path) else {}
    raft_cpu.build()
    for name, (n, v, t, l, c, m, inv, py, is_big) in CASES.items():
        if (is_big and not big) or (only and name not in only):
            continue
        cfg = raft_cpu.cfg_of(n, v, t, l, c, m, inv)
        r = raft_cpu.bfs(cfg, threads=os.cpu_count() or 8, keep_trace=not is_big, text_hash=True)
        assert r["rc"] >= 0, (name, r["rc"])
        case = {"n_server": n, "n_value": v, "max_term": t, "max_log": l, "max_copies": c,
                "max_msgs": m, "invariants": list(inv), "distinct": r["distinct"],
                "generated": r["generated"], "depth": r["depth"], "levels": r["levels"],
                "violated": r["violated"], "trace_len": r["trace_len"], "source": "oracle/raft_cpu.c",
                "level_text_hash": ["%016x" % h for h in r["level_text_hash"]]}
        if py:
            pc = rv.Cfg(n, v, t, l, c, inv, m)
            pr = rv.bfs(pc)
            assert [list(x) for x in pr.levels] == r["levels"], name
            assert (pr.violation is not None) == bool(r["violated"]), name
            if not r["violated"]:
                ph = rv.level_text_hashes(pc)
                assert ph == r["level_text_hash"][:len(ph)], name
            case["source"] += " + oracle/raft_values.py"
        out[name] = case
        print(name, r["distinct"], r["generated"], r["depth"], r["violated"], "%.1fs" % r["seconds"], flush=True)
    for name, (n, v, t, l, c, m, inv, py, is_big) in SYM_CASES.items():
        if (is_big and not big) or (only and name not in only):
            continue
        cfg = raft_cpu.cfg_of(n, v, t, l, c, m, inv, symmetry=True)
        r = raft_cpu.bfs(cfg, threads=os.cpu_count() or 8, keep_trace=not is_big, text_hash=True)
        assert r["rc"] >= 0, (name, r["rc"])
        case = {"n_server": n, "n_value": v, "max_term": t, "max_log": l, "max_copies": c, "max_msgs": m,
                "invariants": list(inv), "symmetry": True, "distinct": r["distinct"], "generated": r["generated"],
                "depth": r["depth"], "levels": r["levels"], "violated": r["violated"], "trace_len": r["trace_len"],
                "level_orbit_hash": ["%016x" % h for h in r["level_text_hash"]],
                "source": "oracle/raft_cpu.c (orbit key: least orbit serialisation over server permutations; "
                          "level_orbit_hash: sum of FNV-1a of each new orbit's orbit text)"}
        if py and not r["violated"]:
            ph = []
            pl = rv.bfs_symmetric(rv.Cfg(n, v, t, l, c, inv, m), ph)
            assert [list(x) for x in pl] == r["levels"], name
            assert ph == r["level_text_hash"], name
            case["source"] += " + oracle/raft_values.py (orbit key: least text over permutations; orbit texts)"
        out[name] = case
        print(name, r["distinct"], r["generated"], r["depth"], r["violated"], "%.1fs" % r["seconds"], flush=True)
    for name, (n, v, t, l, c, m, inv, cap, depth) in PREFIXES.items():
        if not big or (only and name not in only):
            continue
        cfg = raft_cpu.cfg_of(n, v, t, l, c, m, inv, max_distinct=cap, max_levels=depth)
        cfg.verbose = 1
        r = raft_cpu.bfs(cfg, threads=os.cpu_count() or 8, text_hash=True)
        assert r["rc"] in (0, -4), (name, r["rc"])
        out[name] = {"n_server": n, "n_value": v, "max_term": t, "max_log": l, "max_copies": c, "max_msgs": m,
                     "invariants": list(inv), "prefix": True, "levels": r["levels"],
                     "distinct": r["distinct"], "generated": r["generated"], "max_msgs_seen": r["max_msgs"],
                     "level_text_hash": ["%016x" % h for h in r["level_text_hash"]],
                     "source": "oracle/raft_cpu.c, first %d complete levels" % len(r["levels"])}
        print(name, r["distinct"], len(r["levels"]), "%.1fs" % r["seconds"], flush=True)
        with open(path, "w") as f:  # each prefix is long: keep what is done
            json.dump(out, f, indent=1, sort_keys=True)
    for name, (n, v, t, l, c, m, inv, cap, depth) in SYM_PREFIXES.items():
        if not big or (only and name not in only):
            continue
        cfg = raft_cpu.cfg_of(n, v, t, l, c, m, inv, max_distinct=cap, symmetry=True, max_levels=depth)
        cfg.verbose = 1
        r = raft_cpu.bfs(cfg, threads=os.cpu_count() or 8, text_hash=True)
        assert r["rc"] in (0, -4), (name, r["rc"])
        out[name] = {"n_server": n, "n_value": v, "max_term": t, "max_log": l, "max_copies": c, "max_msgs": m,
                     "invariants": list(inv), "prefix": True, "symmetry": True, "levels": r["levels"],
                     "distinct": r["distinct"], "generated": r["generated"], "max_msgs_seen": r["max_msgs"],
                     "level_orbit_hash": ["%016x" % h for h in r["level_text_hash"]],
                     "source": "oracle/raft_cpu.c (orbit key: least orbit serialisation over server permutations; "
                               "level_orbit_hash: orbit texts), first %d complete levels" % len(r["levels"])}
        print(name, r["distinct"], len(r["levels"]), "%.1fs" % r["seconds"], flush=True)
        with open(path, "w") as f:
            json.dump(out, f, indent=1, sort_keys=True)
    if "--py-pins" in sys.argv or big:
        pin_with_value_oracle(out, only)
    with open(path, "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
