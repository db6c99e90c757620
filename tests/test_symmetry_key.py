"""The SYMMETRY orbit key on the CPU (rtla_model.h sym_key through
rtla_orbit_key / rtla_permute_row): every server permutation of a state has
its state's key, and two states share a key exactly when some permutation
maps one onto the other (checked against the least TLC text over all
permutations, the value oracle's notion of an orbit).  The states are the
synthetic microbench's random rows (few ties between servers), copies of
them with servers made look-alike and the bag emptied (many ties: the
signature-pruned search must then try every ordering of the tied servers),
and Init (all servers alike and interchangeable: sym_rank's twin test then
keeps one ordering).  The GPU side -- orbit counts of whole BFS runs
against the C oracle -- is in test_gpu.py."""
import itertools
import random

import pytest

import rtla



def cfg_of(n):
    t, l = (3, 2) if n <= 3 else (2, 1)
    return rtla.Config(n_server=n, n_value=1, max_term=t, max_log=l, max_copies=1, max_msgs=0,
                       invariants=(), bag_cap=12, symmetry=True)


def look_alike(cfg, row, k):
    """Servers 1..k take server 0's record relabelled into their place (the
    image of record 0 under the transposition (0 i)); the bag is emptied."""
    n, g = cfg.n_server, rtla.row_layout(cfg)
    off, sw = g["off_srv"], g["srv_words"]
    out = list(row)
    for i in range(1, k + 1):
        pi = list(range(n))
        pi[0], pi[i] = i, 0
        img = rtla.permute_row(cfg, row, pi)
        out[off + i * sw:off + (i + 1) * sw] = img[off + i * sw:off + (i + 1) * sw]
    out[g["off_hdr"]] &= ~0xFF
    return out


def min_text(cfg, row, perms):
    return min(rtla.state_text(cfg, rtla.permute_row(cfg, row, pi)) for pi in perms)


@pytest.mark.parametrize("n", [2, 3, 4, 5])
def test_orbit_key_is_a_function_of_the_orbit(n):
    cfg = cfg_of(n)
    all_perms = [list(p) for p in itertools.permutations(range(n))]
    rng = random.Random(n)
    base = rtla.random_rows(cfg, 0, 40 if n < 5 else 16, pool=0)
    rows = base + [look_alike(cfg, r, rng.randrange(1, n)) for r in base[:12]] + [rtla.init_row(cfg)]
    # permuted copies: equal orbits under different names
    rows += [rtla.permute_row(cfg, r, rng.choice(all_perms)) for r in rows[:20]]
    keys, orbits, nperm = [], [], []
    for r in rows:
        key, c = rtla.orbit_key(cfg, r)
        nperm.append(c)
        for pi in (all_perms if n <= 4 else rng.sample(all_perms, 12)):
            assert rtla.orbit_key(cfg, rtla.permute_row(cfg, r, pi))[0] == key
        keys.append(key)
        orbits.append(min_text(cfg, r, all_perms))
    # same key <=> same orbit
    by_key = {}
    for k, o in zip(keys, orbits):
        by_key.setdefault(k, set()).add(o)
    assert all(len(v) == 1 for v in by_key.values())
    assert len(by_key) == len(set(orbits))
    # Init: every server alike, and interchangeable (each transposition maps
    # Init onto itself): sym_rank's twin test (tie groups of >= 3) keeps one
    # ordering, a pair keeps both; random states: mostly one
    assert nperm[len(base) + 12] == (1 if n >= 3 else len(all_perms))
    assert sum(nperm[:len(base)]) <= 1.5 * len(base), nperm[:len(base)]


def test_permute_row_keeps_state_validity():
    cfg = cfg_of(3)
    for r in rtla.random_rows(cfg, 0, 30):
        img = rtla.permute_row(cfg, r, [2, 0, 1])
        assert rtla.row_fingerprint(cfg, img) == rtla.stored_fingerprint(img)
        back = rtla.permute_row(cfg, img, [1, 2, 0])  # the inverse permutation
        assert back == r
    with pytest.raises(rtla.RtlaError):
        rtla.permute_row(cfg, r, [0, 0, 1])


@pytest.mark.parametrize("n", [2, 3, 4, 5])
def test_orbit_text_matches_value_oracle(n):
    """The SYMMETRY level digest's per-orbit item (rtla_orbit_text, host C++
    over the packed row, with its exact shortcut on the first two rotated
    lines) equals the value oracle's brute force over every permutation
    (raft_values.orbit_text on the parsed state), is the same for every
    image of a state, and rtla_rows_orbit_hash sums FNV-1a of exactly these
    texts."""
    import os
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle"))
    import raft_values as rv
    import tla_text
    cfg = cfg_of(n)
    vc = rv.Cfg(n, 1, cfg.max_term, cfg.max_log, 1, (), 0)
    all_perms = [list(p) for p in itertools.permutations(range(n))]
    rng = random.Random(100 + n)
    base = rtla.random_rows(cfg, 0, 24 if n < 5 else 8, pool=0)
    rows = base + [look_alike(cfg, r, rng.randrange(1, n)) for r in base[:8]] + [rtla.init_row(cfg)]
    rows += [rtla.permute_row(cfg, r, rng.choice(all_perms)) for r in rows[:10]]
    texts = []
    for r in rows:
        t = rtla.orbit_text(cfg, r)
        assert t == rv.orbit_text(vc, tla_text.parse_state(vc, rtla.state_text(cfg, r)))
        for pi in rng.sample(all_perms, min(len(all_perms), 6)):
            assert rtla.orbit_text(cfg, rtla.permute_row(cfg, r, pi)) == t
        texts.append(t)
    assert rtla.rows_orbit_hash(cfg, rows, threads=2) == sum(rv.fnv1a64(t) for t in texts) & (2 ** 64 - 1)
