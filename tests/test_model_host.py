"""CPU checks of the model code the level kernel evaluates (rtla_model.h,
compiled for the host by tests/hostmodel.py -- test infrastructure): the
successor multisets of lockstep random walks equal the C oracle's, the
successors of random synthetic states equal the value oracle's, and every
incrementally derived fingerprint equals a from-scratch hash.  The same
checks run on the GPU through the hot kernel (tests/test_gpu.py)."""
import collections
import random

import pytest

import hostmodel
import raft_cpu
import raft_values as rv
import rtla
import tla_text

INV = ("NoTwoLeaders", "ElectionSafety", "LogMatching")
WALKS = [(2, 2, 3, 2, 1, 1), (3, 1, 2, 1, 1, 2), (3, 2, 3, 2, 1, 3), (3, 2, 4, 3, 2, 4),
         (5, 1, 3, 2, 1, 3), (2, 1, 3, 1, 2, 0), (4, 2, 3, 2, 1, 0)]


@pytest.mark.parametrize("shape", WALKS)
def test_host_model_walk_matches_oracle(shape):
    n, v, t, l, c, m = shape
    cfg = rtla.Config(n, v, t, l, c, m, INV, bag_cap=16 if m == 0 else 0)
    w = rtla.row_words(cfg)
    walk = raft_cpu.Walk(raft_cpu.cfg_of(n, v, t, l, c, m, INV))
    rnd = random.Random(hash(shape) & 0xFFFF)
    row = rtla.init_row(cfg)
    for step in range(150):
        succ = hostmodel.expand(cfg, [row], w)
        mine = sorted((im, rtla.state_text(cfg, r)) for _, _, _, im, r in succ)
        assert mine == sorted(walk.successors()), "successor multiset differs at step %d" % step
        for _, _, _, _, r in succ:
            assert rtla.stored_fingerprint(r) == rtla.row_fingerprint(cfg, r)
        inm = [x for x in succ if x[3]]
        if not inm:
            break
        row = rnd.choice(inm)[4]
        walk.goto(rtla.state_text(cfg, row))


def test_host_model_synthetic_states_match_value_oracle():
    cfg = rtla.Config(3, 2, 4, 3, 2, 0, ("ElectionSafety", "LogMatching"), bag_cap=12)
    vc = rv.Cfg(3, 2, 4, 3, 2, ("ElectionSafety", "LogMatching"), 0)
    w = rtla.row_words(cfg)
    rows = rtla.random_rows(cfg, 0, 120, pool=30)
    by = collections.defaultdict(list)
    for k, inst, sub, im, r in hostmodel.expand(cfg, rows, w):
        by[k].append((im, rtla.state_text(cfg, r)))
        assert rtla.stored_fingerprint(r) == rtla.row_fingerprint(cfg, r)
    for k, r in enumerate(rows):
        s = tla_text.parse_state(vc, rtla.state_text(cfg, r))
        ref = sorted((rv.in_model(vc, t), rv.state_text(vc, t)) for _, t in rv.next_states(vc, s))
        assert sorted(by[k]) == ref, "input state %d" % k
