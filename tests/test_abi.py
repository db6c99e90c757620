"""CPU tests of the C-ABI library: it loads, exports every symbol that
include/rtla.h declares, and its host-only helpers (row layout, Init row,
state printer) agree with the oracle.  No kernel is launched here."""
import ctypes
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "raft-tla_amd", "librtla.so")


def declared_symbols():
    hdr = open(os.path.join(ROOT, "include", "rtla.h")).read()
    hdr = re.sub(r"/\*.*?\*/", "", hdr, flags=re.S)
    return sorted(set(re.findall(r"\b(rtla_[a-z_0-9]+)\s*\(", hdr)))


def test_library_exports_every_declared_symbol():
    assert os.path.exists(LIB), "build librtla.so first (__graft_entry__.build())"
    nm = subprocess.check_output(["nm", "-D", "--defined-only", LIB]).decode()
    exported = set(re.findall(r"\bT (rtla_[a-z_0-9]+)", nm))
    missing = [s for s in declared_symbols() if s not in exported]
    assert not missing, missing
    lib = ctypes.CDLL(LIB)
    for s in declared_symbols():
        getattr(lib, s)


def test_python_mirror_binds_every_symbol():
    import rtla
    assert sorted(rtla.EXPORTED) == declared_symbols()
    assert rtla._lib.rtla_abi_version() == 9


def test_row_layout_and_config_errors():
    import rtla
    assert rtla.row_words(rtla.Config(3, 1, 2, 1, 1, 2)) % 2 == 1   # odd stride for LDS staging
    with pytest.raises(rtla.RtlaError):
        rtla.row_words(rtla.Config(n_server=6))
    with pytest.raises(rtla.RtlaError):
        rtla.row_words(rtla.Config(max_log=5))


@pytest.mark.parametrize("n", [1, 2, 3, 5])
def test_init_row_text_matches_value_oracle(n):
    import raft_values as rv
    import rtla
    cfg = rtla.Config(n, 2, 3, 2, 1, 2)
    row = rtla.init_row(cfg)
    assert rtla.state_text(cfg, row) == rv.state_text(rv.Cfg(n, 2, 3, 2, 1), rv.init_state(rv.Cfg(n, 2, 3, 2, 1)))
    assert rtla.invariants_violated(rtla.Config(n, invariants=("NoTwoLeaders", "ElectionSafety", "LogMatching")), row) == 0


def test_action_names():
    import rtla
    cfg = rtla.Config(3, 2, 2, 1, 1, 2)
    assert rtla.action_name(cfg, 0, 6) == "Restart(s1)"
    assert rtla.action_name(cfg, 3 + 2, 6) == "Timeout(s3)"
    assert rtla.action_name(cfg, 6 + 1, 6) == "RequestVote(s1, s2)"


def test_open_refuses_more_shards_than_the_outbox_holds():
    """rtla_open checks the shard count before touching a device:
    more than SHARD_MAX = 8 owners would overflow the kernels' per-owner state."""
    import rtla
    for kw in ({"shards": 9}, {"shards": 16}):
        with pytest.raises(rtla.RtlaError) as e:
            rtla.Checker(rtla.Config(2, 1, 2, 1, 1, 1, **kw))
        assert e.value.status == -1


def test_rows_text_hash_is_the_oracle_digest():
    """rtla_rows_text_hash (host threads) = the sum of FNV-1a-64 of each row's
    text, the digest the C oracle records per level (raft_cpu.text_hash)."""
    import raft_cpu
    import rtla
    cfg = rtla.Config(3, 2, 4, 3, 2, 0, ("ElectionSafety",), bag_cap=12)
    rows = rtla.random_rows(cfg, 0, 3000, pool=500)
    want = sum(raft_cpu.text_hash(rtla.state_text(cfg, r)) for r in rows) & (2**64 - 1)
    assert rtla.rows_text_hash(cfg, rows) == want
    assert rtla.rows_text_hash(cfg, rows, threads=1) == want
    assert rtla.rows_text_hash(cfg, []) == 0
