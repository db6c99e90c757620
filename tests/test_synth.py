"""The synthetic microbench's input states (BASELINE.json configs[4],
raft-tla_amd/csrc/rtla_synth.h) on the CPU: every random row is a valid
packed state -- its TLC text parses into the value oracle's state and prints
back identically, its stored fingerprint is the from-scratch one -- and the
input numbering is deterministic with half of the inputs drawn from the
pool.  (The GPU side -- Next on these states against the value oracle, and the
dedup counts of rtla_synthetic_step -- is in test_gpu.py.)"""
import pytest

import raft_values as rv
import rtla
import tla_text

# the cfg-3 layout SURVEY.md section 8(d) prescribes: 3 servers, 2 values, term <= 4, log <= 3, 2 copies
SYNTH = dict(n_server=3, n_value=2, max_term=4, max_log=3, max_copies=2, max_msgs=0,
             invariants=("ElectionSafety", "LogMatching"), bag_cap=12)


def vcfg(c):
    return rv.Cfg(c.n_server, c.n_value, c.max_term, c.max_log, c.max_copies, c.invariants, c.max_msgs)


@pytest.mark.parametrize("shape", [SYNTH, dict(SYNTH, max_term=3, max_log=2, max_copies=1, bag_cap=18),
                                   dict(SYNTH, n_server=5, n_value=1, max_term=3, max_log=2, max_copies=1)])
def test_random_rows_are_valid_states(shape):
    cfg = rtla.Config(**shape)
    rows = rtla.random_rows(cfg, 0, 400, pool=50)
    for r in rows:
        text = rtla.state_text(cfg, r)
        assert rv.state_text(vcfg(cfg), tla_text.parse_state(vcfg(cfg), text)) == text
        assert rtla.row_fingerprint(cfg, r) == rtla.stored_fingerprint(r)


def test_input_numbering_is_deterministic_with_pool_repeats():
    cfg = rtla.Config(**SYNTH)
    a = rtla.random_rows(cfg, 0, 600, pool=40)
    assert rtla.random_rows(cfg, 200, 50, pool=40) == a[200:250]
    texts = [rtla.state_text(cfg, r) for r in a]
    distinct = len(set(texts))
    # ~half the inputs are fresh, the rest fall into 40 pool states
    assert 250 < distinct < 350, distinct
    assert rtla.random_rows(cfg, 0, 10, pool=40, seed=1) != a[:10]
