"""Python host-side mirror of the C ABI (include/rtla.h) over ctypes.

This is the user-facing API of the MI355X model checker for Python callers
(tests, bench.py).  It mirrors TLC's model-checking contract for
/root/reference/raft.tla + a raft.cfg-style model (raft.cfg:1-15):

    res = rtla.check(rtla.Config(n_server=3, n_value=1, max_term=2, max_log=1,
                                 max_copies=1, max_msgs=2,
                                 invariants=("NoTwoLeaders",)))
    res.distinct, res.generated, res.depth, res.violation, res.trace

There is no CPU fallback: every entry point runs the HIP kernels in
librtla.so, and importing this module raises if the library is missing.
"""
from __future__ import annotations

import ctypes as C
import os
from dataclasses import dataclass, field
from typing import List, Optional, Sequence, Tuple

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("RTLA_LIB") or os.path.join(HERE, "librtla.so")  # RTLA_LIB: perf-experiment builds only

OK, DONE, VIOLATION = 0, 1, 2
E_CONFIG, E_HIP, E_OVERFLOW, E_SPEC, E_STATE, E_ARG, E_COMM = -1, -2, -3, -4, -5, -6, -7  # include/rtla.h
INV_BITS = {"NoTwoLeaders": 1, "ElectionSafety": 2, "LogMatching": 4}
COVER_NAMES = ["Restart", "Timeout", "RequestVote", "BecomeLeader", "ClientRequest",
               "AdvanceCommitIndex", "AppendEntries", "Receive", "DuplicateMessage",
               "DropMessage", "UpdateTerm", "HandleRequestVoteRequest",
               "HandleRequestVoteResponse", "HandleAppendEntriesRequest",
               "HandleAppendEntriesResponse", "DropStaleResponse"]


# rtla_level_stats.flags: which capacity ran out (include/rtla.h RTLA_CAP_*)
CAP_NAMES = {1: "spec-error", 2: "row", 4: "frontier", 8: "fpset", 16: "outbox"}


class RtlaError(RuntimeError):
    def __init__(self, status: int, what: str = "", flags: int = 0):
        self.status = status
        self.flags = flags
        msg = _lib.rtla_strerror(status).decode() if _lib else str(status)
        caps = [n for b, n in CAP_NAMES.items() if flags & b]
        super().__init__("%s: %s (status %d%s)" % (what, msg, status, ", " + "+".join(caps) if caps else ""))


class _Cfg(C.Structure):
    _fields_ = [("n_server", C.c_int32), ("n_value", C.c_int32), ("max_term", C.c_int32),
                ("max_log", C.c_int32), ("max_copies", C.c_int32), ("max_msgs", C.c_int32),
                ("bag_cap", C.c_int32), ("elec_cap", C.c_int32), ("inv_mask", C.c_int32),
                ("symmetry", C.c_int32), ("fpset_log2", C.c_int32), ("shards", C.c_int32),
                ("frontier_cap", C.c_uint64), ("mem_budget", C.c_uint64), ("chunk", C.c_uint64),
                ("mode", C.c_int32), ("reserved", C.c_int32)]


class _Stats(C.Structure):
    _fields_ = [("level", C.c_int32), ("status", C.c_int32), ("frontier", C.c_uint64),
                ("new_states", C.c_uint64), ("generated", C.c_uint64),
                ("distinct_total", C.c_uint64), ("generated_total", C.c_uint64),
                ("seconds", C.c_double), ("kernel_ms", C.c_double), ("probes", C.c_uint64),
                ("row_bytes", C.c_uint64), ("expand_ms", C.c_double), ("flags", C.c_int32),
                ("reserved", C.c_int32)]


def _load():
    if not os.path.exists(LIB_PATH):
        raise ImportError("librtla.so not built at %s (run `make -C raft-tla_amd` or "
                          "__graft_entry__.build())" % LIB_PATH)
    lib = C.CDLL(LIB_PATH)
    P = C.POINTER
    sig = {
        "rtla_open": (C.c_int, [P(_Cfg), C.c_int, C.c_int, C.c_void_p, P(C.c_void_p)]),
        "rtla_close": (None, [C.c_void_p]),
        "rtla_init": (C.c_int, [C.c_void_p, P(_Stats)]),
        "rtla_step": (C.c_int, [C.c_void_p, P(_Stats)]),
        "rtla_reset": (C.c_int, [C.c_void_p]),
        "rtla_violation": (C.c_int, [C.c_void_p, P(C.c_int32), P(C.c_int32)]),
        "rtla_trace": (C.c_int, [C.c_void_p, P(C.c_uint32), P(C.c_int32), C.c_size_t, P(C.c_size_t)]),
        "rtla_frontier": (C.c_int, [C.c_void_p, P(C.c_uint32), C.c_size_t, P(C.c_size_t)]),
        "rtla_coverage": (C.c_int, [C.c_void_p, P(C.c_uint64), P(C.c_uint64), C.c_int]),
        "rtla_device_info": (C.c_int, [C.c_void_p, C.c_char_p, C.c_size_t]),
        "rtla_time_expand": (C.c_int, [C.c_void_p, C.c_int, C.c_int, P(C.c_double)]),
        "rtla_checkpoint": (C.c_int, [C.c_void_p, C.c_char_p]),
        "rtla_recover": (C.c_int, [C.c_void_p, C.c_char_p]),
        "rtla_probe_bench2": (C.c_int, [C.c_int, C.c_uint64, P(C.c_double), P(C.c_double), P(C.c_double),
                                        P(C.c_uint64)]),
        "rtla_probe_bench3": (C.c_int, [C.c_int, C.c_uint64, C.c_uint64, C.c_double, P(C.c_double),
                                        P(C.c_uint64)]),
        "rtla_random_texts": (C.c_int, [P(_Cfg), C.c_uint64, C.c_uint64, C.c_uint64, C.c_uint64, C.c_char_p,
                                        C.c_size_t, P(C.c_size_t)]),
        "rtla_row_words": (C.c_int, [P(_Cfg)]),
        "rtla_row_layout": (C.c_int, [P(_Cfg), P(C.c_int32), C.c_int]),
        "rtla_init_row": (C.c_int, [P(_Cfg), P(C.c_uint32)]),
        "rtla_expand_batch": (C.c_int, [P(_Cfg), P(C.c_uint32), C.c_size_t, P(C.c_uint32),
                                        P(C.c_uint64), C.c_size_t, P(C.c_size_t)]),
        "rtla_state_text": (C.c_int, [P(_Cfg), P(C.c_uint32), C.c_char_p, C.c_size_t]),
        "rtla_action_name": (C.c_int, [P(_Cfg), C.c_int32, C.c_int32, C.c_char_p, C.c_size_t]),
        "rtla_invariants": (C.c_int, [P(_Cfg), P(C.c_uint32)]),
        "rtla_row_fingerprint": (C.c_int, [P(_Cfg), P(C.c_uint32), P(C.c_uint64)]),
        "rtla_strerror": (C.c_char_p, [C.c_int]),
        "rtla_abi_version": (C.c_int, []),
        "rtla_comm_id": (C.c_int, [C.c_void_p]),
        "rtla_probe_bench": (C.c_int, [C.c_int, C.c_uint64, P(C.c_double), P(C.c_uint64)]),
        "rtla_random_rows": (C.c_int, [P(_Cfg), C.c_uint64, C.c_uint64, C.c_uint64, C.c_uint64, P(C.c_uint32)]),
        "rtla_synthetic_step": (C.c_int, [C.c_void_p, C.c_uint64, C.c_uint64, C.c_uint64, C.c_uint64, P(_Stats)]),
        "rtla_synthetic_generate": (C.c_int, [C.c_void_p, C.c_uint64, C.c_uint64, C.c_uint64, C.c_uint64, C.c_uint64]),
        "rtla_synthetic_dedup": (C.c_int, [C.c_void_p, C.c_uint64, C.c_uint64, P(_Stats)]),
        "rtla_orbit_key": (C.c_int, [P(_Cfg), P(C.c_uint32), P(C.c_uint64), P(C.c_int)]),
        "rtla_permute_row": (C.c_int, [P(_Cfg), P(C.c_uint32), P(C.c_int), P(C.c_uint32)]),
        "rtla_rows_text_hash": (C.c_int, [P(_Cfg), P(C.c_uint32), C.c_size_t, C.c_int, P(C.c_uint64)]),
        "rtla_level_text_hash": (C.c_int, [C.c_void_p, C.c_int, P(C.c_uint64)]),
        "rtla_rows_orbit_hash": (C.c_int, [P(_Cfg), P(C.c_uint32), C.c_size_t, C.c_int, P(C.c_uint64)]),
        "rtla_level_orbit_hash": (C.c_int, [C.c_void_p, C.c_int, P(C.c_uint64)]),
        "rtla_orbit_text": (C.c_int, [P(_Cfg), P(C.c_uint32), C.c_char_p, C.c_size_t]),
    }
    for name, (res, args) in sig.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    return lib


_lib = _load()

EXPORTED = ["rtla_open", "rtla_close", "rtla_comm_id", "rtla_init", "rtla_reset", "rtla_step", "rtla_violation",
            "rtla_trace", "rtla_frontier", "rtla_coverage", "rtla_device_info", "rtla_row_words", "rtla_init_row",
            "rtla_expand_batch", "rtla_state_text", "rtla_action_name", "rtla_invariants", "rtla_row_fingerprint",
            "rtla_strerror", "rtla_abi_version", "rtla_probe_bench", "rtla_time_expand",
            "rtla_probe_bench2", "rtla_checkpoint", "rtla_recover", "rtla_random_rows", "rtla_synthetic_step",
            "rtla_synthetic_generate", "rtla_synthetic_dedup", "rtla_orbit_key", "rtla_permute_row",
            "rtla_rows_text_hash", "rtla_level_text_hash", "rtla_row_layout", "rtla_rows_orbit_hash",
            "rtla_level_orbit_hash", "rtla_orbit_text", "rtla_probe_bench3", "rtla_random_texts"]

SYNTH_SEED = 0x5AF72025  # the synthetic microbench's PRNG seed


@dataclass(frozen=True)
class Config:
    """A raft.cfg-style model: constants + the build's StateConstraint bounds."""
    n_server: int = 3
    n_value: int = 1
    max_term: int = 2
    max_log: int = 1
    max_copies: int = 1
    max_msgs: int = 0
    invariants: Tuple[str, ...] = ("NoTwoLeaders",)
    bag_cap: int = 0
    elec_cap: int = 0
    fpset_log2: int = 0
    frontier_cap: int = 0
    mem_budget: int = 0
    shards: int = 0
    chunk: int = 0
    symmetry: bool = False  # SYMMETRY Permutations(Server) (specs/MC.tla)
    dedup_only: bool = False  # RTLA_MODE_DEDUP: the synthetic microbench's context (no BFS, no parent records)

    @property
    def inv_mask(self) -> int:
        m = 0
        for n in self.invariants:
            m |= INV_BITS[n]
        return m

    def c(self) -> _Cfg:
        return _Cfg(self.n_server, self.n_value, self.max_term, self.max_log, self.max_copies,
                    self.max_msgs, self.bag_cap, self.elec_cap, self.inv_mask, int(self.symmetry),
                    self.fpset_log2, self.shards, self.frontier_cap, self.mem_budget, self.chunk,
                    1 if self.dedup_only else 0, 0)


@dataclass
class Level:
    level: int
    frontier: int
    new: int
    generated: int
    seconds: float
    kernel_ms: float = 0.0
    probes: int = 0
    row_bytes: int = 0
    expand_ms: float = 0.0  # of kernel_ms: the probe kernel alone


@dataclass
class Result:
    distinct: int = 0
    generated: int = 0
    depth: int = 0
    levels: List[Level] = field(default_factory=list)
    violation: Optional[str] = None
    violation_in_model: bool = True
    trace: Optional[List[Tuple[str, str]]] = None   # (action label, state text)
    coverage: Optional[dict] = None
    seconds: float = 0.0


def _check(st: int, what: str):
    if st < 0:
        raise RtlaError(st, what)
    return st


def row_words(cfg: Config) -> int:
    cc = cfg.c()
    return _check(_lib.rtla_row_words(C.byref(cc)), "rtla_row_words")


ROW_LAYOUT_KEYS = ("W", "off_hdr", "off_srv", "srv_words", "off_all", "all_words", "off_elec", "elec_words",
                   "off_bag", "slot_words")


def row_layout(cfg: Config) -> dict:
    """Geometry of the packed row (rtla_model.h make_layout): word offsets and record sizes."""
    cc = cfg.c()
    out = (C.c_int32 * len(ROW_LAYOUT_KEYS))()
    n = _check(_lib.rtla_row_layout(C.byref(cc), out, len(ROW_LAYOUT_KEYS)), "rtla_row_layout")
    return dict(zip(ROW_LAYOUT_KEYS[:n], list(out)[:n]))


def init_row(cfg: Config):
    cc = cfg.c()
    w = row_words(cfg)
    buf = (C.c_uint32 * w)()
    _check(_lib.rtla_init_row(C.byref(cc), buf), "rtla_init_row")
    return list(buf)


def state_text(cfg: Config, row: Sequence[int]) -> str:
    cc = cfg.c()
    arr = (C.c_uint32 * len(row))(*row)
    cap = 1 << 16
    while True:
        buf = C.create_string_buffer(cap)
        st = _lib.rtla_state_text(C.byref(cc), arr, buf, cap)
        if st >= 0:
            return buf.value.decode()
        cap *= 4
        if cap > 1 << 26:
            raise RtlaError(st, "rtla_state_text")


def action_name(cfg: Config, inst: int, sub: int) -> str:
    cc = cfg.c()
    buf = C.create_string_buffer(256)
    _check(_lib.rtla_action_name(C.byref(cc), inst, sub, buf, 256), "rtla_action_name")
    return buf.value.decode()


def invariants_violated(cfg: Config, row: Sequence[int]) -> int:
    cc = cfg.c()
    arr = (C.c_uint32 * len(row))(*row)
    return _check(_lib.rtla_invariants(C.byref(cc), arr), "rtla_invariants")


def row_fingerprint(cfg: Config, row: Sequence[int]):
    """(a, b) recomputed from scratch; the row stores the incrementally derived one in words 0-3."""
    cc = cfg.c()
    arr = (C.c_uint32 * len(row))(*row)
    out = (C.c_uint64 * 2)()
    _check(_lib.rtla_row_fingerprint(C.byref(cc), arr, out), "rtla_row_fingerprint")
    return out[0], out[1]


def orbit_key(cfg: Config, row: Sequence[int]):
    """SYMMETRY seen-set key of the row's orbit and the number of permutation
    images it compared (rtla_model.h sym_key; host)."""
    cc = cfg.c()
    arr = (C.c_uint32 * len(row))(*row)
    out = (C.c_uint64 * 2)()
    n = C.c_int(0)
    _check(_lib.rtla_orbit_key(C.byref(cc), arr, out, C.byref(n)), "rtla_orbit_key")
    return (out[0], out[1]), n.value


def permute_row(cfg: Config, row: Sequence[int], pi: Sequence[int]):
    """The server-permuted image of a row (server i moved to pi[i])."""
    cc = cfg.c()
    arr = (C.c_uint32 * len(row))(*row)
    p = (C.c_int * len(pi))(*pi)
    out = (C.c_uint32 * len(row))()
    _check(_lib.rtla_permute_row(C.byref(cc), arr, p, out), "rtla_permute_row")
    return list(out)


def rows_text_hash(cfg: Config, rows: Sequence[Sequence[int]], threads: int = 0) -> int:
    """Sum mod 2^64 of FNV-1a-64(state_text) over the rows: the oracle's
    per-level digest of a set of states (host threads, rtla_rows_text_hash)."""
    cc = cfg.c()
    w = row_words(cfg)
    n = len(rows)
    flat = (C.c_uint32 * max(1, n * w))()
    for k, r in enumerate(rows):
        flat[k * w:(k + 1) * w] = list(r)
    out = C.c_uint64(0)
    _check(_lib.rtla_rows_text_hash(C.byref(cc), flat, n, threads, C.byref(out)), "rtla_rows_text_hash")
    return out.value


def rows_orbit_hash(cfg: Config, rows: Sequence[Sequence[int]], threads: int = 0) -> int:
    """Sum mod 2^64 of FNV-1a-64 of each row's ORBIT TEXT (rtla_rows_orbit_hash):
    a SYMMETRY level's digest, whichever member of each orbit a row holds."""
    cc = cfg.c()
    w = row_words(cfg)
    n = len(rows)
    flat = (C.c_uint32 * max(1, n * w))()
    for k, r in enumerate(rows):
        flat[k * w:(k + 1) * w] = list(r)
    out = C.c_uint64(0)
    _check(_lib.rtla_rows_orbit_hash(C.byref(cc), flat, n, threads, C.byref(out)), "rtla_rows_orbit_hash")
    return out.value


def orbit_text(cfg: Config, row: Sequence[int]) -> str:
    """The text of the orbit representative whose rotated text is least
    (rtla_orbit_text; the item of a SYMMETRY level digest)."""
    cc = cfg.c()
    arr = (C.c_uint32 * len(row))(*row)
    cap = 1 << 16
    while True:
        buf = C.create_string_buffer(cap)
        st = _lib.rtla_orbit_text(C.byref(cc), arr, buf, cap)
        if st >= 0:
            return buf.value.decode()
        cap *= 4
        if cap > 1 << 26:
            raise RtlaError(st, "rtla_orbit_text")


def random_texts(cfg: Config, first: int, n: int, pool: int = 0, seed: int = SYNTH_SEED) -> bytes:
    """The synthetic input states first .. first + n - 1 as state texts, each
    terminated by '\x1e' (rtla_random_texts; host)."""
    cc = cfg.c()
    need = C.c_size_t(0)
    cap = n * 2048  # a random state's text is ~1 KB; the rare larger batch is rendered again at its exact size
    buf = C.create_string_buffer(cap)
    if _lib.rtla_random_texts(C.byref(cc), seed, first, n, pool, buf, cap, C.byref(need)) != OK:
        buf = C.create_string_buffer(need.value + 1)
        _check(_lib.rtla_random_texts(C.byref(cc), seed, first, n, pool, buf, need.value, C.byref(need)),
               "rtla_random_texts")
    return buf.raw[:need.value]


def stored_fingerprint(row: Sequence[int]):
    return row[0] | row[1] << 32, row[2] | row[3] << 32


def random_rows(cfg: Config, first: int, n: int, pool: int = 0, seed: int = SYNTH_SEED):
    """Rows of the synthetic microbench's input states first .. first + n - 1
    (rtla_synth.h; computed on the host)."""
    w = row_words(cfg)
    cc = cfg.c()
    buf = (C.c_uint32 * max(1, n * w))()
    _check(_lib.rtla_random_rows(C.byref(cc), seed, first, n, pool, buf), "rtla_random_rows")
    return [list(buf[k * w:(k + 1) * w]) for k in range(n)]


def expand_batch(cfg: Config, rows: Sequence[Sequence[int]]):
    """GPU successor generation (TLC getNextStates) for a batch of rows.

    Returns a list of (input index, instance, receive-sub, in_model, row),
    sorted by (input, instance)."""
    cc = cfg.c()
    w = row_words(cfg)
    n = len(rows)
    flat = (C.c_uint32 * (max(n, 1) * w))()
    for k, r in enumerate(rows):
        assert len(r) == w, "row width mismatch"
        flat[k * w:(k + 1) * w] = list(r)
    cap = max(n, 1) * 512
    succ = (C.c_uint32 * (cap * w))()
    info = (C.c_uint64 * cap)()
    nout = C.c_size_t(0)
    _check(_lib.rtla_expand_batch(C.byref(cc), flat, n, succ, info, cap, C.byref(nout)),
           "rtla_expand_batch")
    out = []
    for k in range(nout.value):
        v = info[k]
        out.append((v >> 32, v & 0xFFFF, (v >> 16) & 0x7FFF, bool(v >> 31 & 1),
                    list(succ[k * w:(k + 1) * w])))
    return out


class Checker:
    """One BFS context on one GPU (rank)."""

    def __init__(self, cfg: Config, rank: int = 0, world: int = 1, comm_id: bytes = None):
        self.cfg = cfg
        self._cc = cfg.c()
        h = C.c_void_p()
        cid = C.create_string_buffer(comm_id, 128) if comm_id else None
        _check(_lib.rtla_open(C.byref(self._cc), rank, world, cid, C.byref(h)), "rtla_open")
        self._h = h
        self._recovered = False
        self.levels: List[Level] = []
        self.status = OK

    def close(self):
        if self._h:
            _lib.rtla_close(self._h)
            self._h = None

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def device_info(self) -> str:
        buf = C.create_string_buffer(4096)
        _check(_lib.rtla_device_info(self._h, buf, 4096), "rtla_device_info")
        return buf.value.decode()

    def _rec(self, st: _Stats):
        self.levels.append(Level(st.level, st.frontier, st.new_states, st.generated, st.seconds,
                                 st.kernel_ms, st.probes, st.row_bytes, st.expand_ms))
        self.distinct, self.generated = st.distinct_total, st.generated_total

    def init(self) -> int:
        st = _Stats()
        self.status = _check(_lib.rtla_init(self._h, C.byref(st)), "rtla_init")
        self._rec(st)
        return self.status

    def reset(self):
        _check(_lib.rtla_reset(self._h), "rtla_reset")
        self.levels = []
        self.status = OK

    def step(self) -> int:
        """One BFS level.  Raises RtlaError (with .flags naming the capacity
        that ran out) if the level could not be completed."""
        st = _Stats()
        rc = _lib.rtla_step(self._h, C.byref(st))
        if rc < 0:
            self.status = rc
            raise RtlaError(rc, "rtla_step", st.flags)
        self.status = rc
        self._rec(st)
        return self.status

    def run(self, max_levels: int = 100000) -> int:
        if not self.levels and not self._recovered:
            if self.init() != OK:
                return self.status
        while self.status == OK and len(self.levels) < max_levels:
            self.step()
        return self.status

    def violation(self):
        m, im = C.c_int32(0), C.c_int32(0)
        _lib.rtla_violation(self._h, C.byref(m), C.byref(im))
        names = [n for n, b in INV_BITS.items() if m.value & b]
        return (names[0] if names else None), bool(im.value)

    def trace(self) -> List[Tuple[str, str]]:
        w = row_words(self.cfg)
        n = C.c_size_t(0)
        _lib.rtla_trace(self._h, None, None, 0, C.byref(n))
        cap = n.value
        rows = (C.c_uint32 * (cap * w))()
        labels = (C.c_int32 * cap)()
        _check(_lib.rtla_trace(self._h, rows, labels, cap, C.byref(n)), "rtla_trace")
        out = []
        for k in range(n.value):
            lab = labels[k]
            name = "Initial predicate" if lab < 0 else action_name(self.cfg, lab & 0xFFFF, (lab >> 16) & 0x7FFF)
            out.append((name, state_text(self.cfg, list(rows[k * w:(k + 1) * w]))))
        return out

    def frontier(self):
        """Rows of the level last produced (debug / parity)."""
        w = row_words(self.cfg)
        n = C.c_size_t(0)
        _check(_lib.rtla_frontier(self._h, None, 0, C.byref(n)), "rtla_frontier")
        buf = (C.c_uint32 * max(1, n.value * w))()
        _check(_lib.rtla_frontier(self._h, buf, n.value, C.byref(n)), "rtla_frontier")
        return [list(buf[k * w:(k + 1) * w]) for k in range(n.value)]

    def level_text_hash(self, threads: int = 0) -> int:
        """Digest of the level last produced (all shards / ranks): sum mod 2^64
        of FNV-1a-64 of each state's text, decoded on the host from the device
        rows in chunks -- compared with the oracle's level_text_hash."""
        out = C.c_uint64(0)
        _check(_lib.rtla_level_text_hash(self._h, threads, C.byref(out)), "rtla_level_text_hash")
        return out.value

    def level_orbit_hash(self, threads: int = 0) -> int:
        """SYMMETRY: the level's digest over orbit texts (rtla_level_orbit_hash),
        compared with the oracle's per-level orbit digest."""
        out = C.c_uint64(0)
        _check(_lib.rtla_level_orbit_hash(self._h, threads, C.byref(out)), "rtla_level_orbit_hash")
        return out.value

    def checkpoint(self, prefix: str):
        """TLC -checkpoint: write the search to <prefix>.shard<id>.rtla (between levels)."""
        _check(_lib.rtla_checkpoint(self._h, prefix.encode()), "rtla_checkpoint")

    def recover(self, prefix: str):
        """TLC -recover: resume a checkpoint written by a context of the same configuration."""
        _check(_lib.rtla_recover(self._h, prefix.encode()), "rtla_recover")
        self.status = OK
        self._recovered = True

    def time_expand(self, xflags: int, reps: int = 3) -> float:
        """Diagnostic: mean ms of re-expanding the current frontier (pollutes the search)."""
        ms = C.c_double()
        _check(_lib.rtla_time_expand(self._h, xflags, reps, C.byref(ms)), "rtla_time_expand")
        return ms.value

    def synthetic_step(self, first: int, n: int, pool: int = 0, seed: int = SYNTH_SEED) -> Level:
        """BASELINE configs[4]: n random states through Next + fingerprint +
        dedup (one level-kernel launch; the set accumulates across calls)."""
        st = _Stats()
        rc = _lib.rtla_synthetic_step(self._h, seed, first, n, pool, C.byref(st))
        if rc < 0:
            raise RtlaError(rc, "rtla_synthetic_step", st.flags)
        return Level(0, st.frontier, st.new_states, st.generated, st.seconds, st.kernel_ms, st.probes, st.row_bytes,
                     st.expand_ms)

    def synthetic_generate(self, first: int, n: int, pool: int = 0, at: int = 0, seed: int = SYNTH_SEED):
        """Input states first .. first + n - 1 into row-arena rows at .. at + n - 1 (on the device)."""
        _check(_lib.rtla_synthetic_generate(self._h, seed, first, n, pool, at), "rtla_synthetic_generate")

    def synthetic_dedup(self, begin: int, end: int) -> Level:
        """One dedup-only level-kernel launch over the resident arena rows [begin, end)."""
        st = _Stats()
        rc = _lib.rtla_synthetic_dedup(self._h, begin, end, C.byref(st))
        if rc < 0:
            raise RtlaError(rc, "rtla_synthetic_dedup", st.flags)
        return Level(0, st.frontier, st.new_states, st.generated, st.seconds, st.kernel_ms, st.probes, st.row_bytes,
                     st.expand_ms)

    def coverage(self) -> dict:
        n = len(COVER_NAMES)
        g, d = (C.c_uint64 * n)(), (C.c_uint64 * n)()
        _check(_lib.rtla_coverage(self._h, g, d, n), "rtla_coverage")
        return {COVER_NAMES[k]: (g[k], d[k]) for k in range(n)}


def check(cfg: Config, trace: bool = True) -> Result:
    """Exhaustive BFS of the model (TLC `-workers N` breadth-first mode)."""
    with Checker(cfg) as ck:
        st = ck.run()
        res = Result(distinct=ck.distinct, generated=ck.generated, levels=list(ck.levels))
        res.depth = sum(1 for lv in ck.levels if lv.new > 0)
        res.seconds = sum(lv.seconds for lv in ck.levels)
        res.coverage = ck.coverage()
        if st == VIOLATION:
            res.violation, res.violation_in_model = ck.violation()
            if trace:
                res.trace = ck.trace()
        return res


def comm_id() -> bytes:
    """A fresh RCCL unique id (rank 0 makes it, every rank passes it to Checker)."""
    buf = C.create_string_buffer(128)
    _check(_lib.rtla_comm_id(buf), "rtla_comm_id")
    return buf.raw


def probe_bench2(log2: int, n: int):
    """(s_insert, s_seen_cas, s_seen_load, inserted) for n random keys, see rtla.h."""
    a, b, c, ins = C.c_double(0), C.c_double(0), C.c_double(0), C.c_uint64(0)
    _check(_lib.rtla_probe_bench2(log2, n, C.byref(a), C.byref(b), C.byref(c), C.byref(ins)), "rtla_probe_bench2")
    return a.value, b.value, c.value, ins.value


def probe_mixed(log2: int, n_present: int, n: int, new_frac: float):
    """(seconds, inserted): n load-first probes into a 2^log2 table holding
    n_present keys, a fraction new_frac of them new keys (rtla_probe_bench3)."""
    sec, ins = C.c_double(0), C.c_uint64(0)
    _check(_lib.rtla_probe_bench3(log2, n_present, n, new_frac, C.byref(sec), C.byref(ins)), "rtla_probe_bench3")
    return sec.value, ins.value


def probe_bench(log2: int, n: int):
    s, ins = C.c_double(0), C.c_uint64(0)
    _check(_lib.rtla_probe_bench(log2, n, C.byref(s), C.byref(ins)), "rtla_probe_bench")
    return s.value, ins.value
