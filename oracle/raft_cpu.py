"""ctypes wrapper of the C oracle (oracle/raft_cpu.c) -- TEST INFRASTRUCTURE ONLY.

Used by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg as the
checker / CPU baseline.  Never imported by the product (raft-tla_amd/).
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "libraft_cpu.so")

INV = {"NoTwoLeaders": 1, "ElectionSafety": 2, "LogMatching": 4}
MAX_LEVELS = 1024


class OrcCfg(C.Structure):
    _fields_ = [("n_server", C.c_int), ("n_value", C.c_int), ("max_term", C.c_int),
                ("max_log", C.c_int), ("max_copies", C.c_int), ("inv_mask", C.c_int),
                ("verbose", C.c_int), ("max_msgs", C.c_int), ("max_distinct", C.c_uint64),
                ("symmetry", C.c_int), ("max_levels", C.c_int)]


class OrcResult(C.Structure):
    _fields_ = [("n_levels", C.c_int), ("depth", C.c_int), ("violated", C.c_int),
                ("trace_len", C.c_int), ("distinct", C.c_uint64), ("generated", C.c_uint64),
                ("level_new", C.c_uint64 * MAX_LEVELS), ("level_gen", C.c_uint64 * MAX_LEVELS),
                ("level_text_hash", C.c_uint64 * MAX_LEVELS), ("coverage", C.c_uint64 * 16),
                ("max_msgs", C.c_uint64), ("max_state_bytes", C.c_uint64), ("seconds", C.c_double),
                ("trace_text", C.c_void_p)]


def build():
    subprocess.check_call(["make", "-s", "-C", HERE], stdout=subprocess.DEVNULL)


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            build()
        _lib = C.CDLL(LIB)
        _lib.orc_bfs.argtypes = [C.POINTER(OrcCfg), C.c_int, C.c_int, C.c_int, C.POINTER(OrcResult)]
        _lib.orc_bfs.restype = C.c_int
        _lib.orc_free.argtypes = [C.c_void_p]
        _lib.orc_text_hash.argtypes = [C.c_char_p]
        _lib.orc_text_hash.restype = C.c_uint64
        _lib.orc_walk_new.argtypes = [C.POINTER(OrcCfg)]
        _lib.orc_walk_new.restype = C.c_void_p
        _lib.orc_walk_free.argtypes = [C.c_void_p]
        _lib.orc_walk_successors.argtypes = [C.c_void_p, C.c_char_p, C.c_size_t]
        _lib.orc_walk_successors.restype = C.c_long
        _lib.orc_walk_goto.argtypes = [C.c_void_p, C.c_char_p]
        _lib.orc_walk_text.argtypes = [C.c_void_p, C.c_char_p, C.c_size_t]
        _lib.orc_walk_text.restype = C.c_long
        _lib.orc_walk_inv.argtypes = [C.c_void_p]
        _lib.orc_walk_orbits.argtypes = [C.c_void_p, C.c_char_p, C.c_size_t]
        _lib.orc_walk_orbits.restype = C.c_long
        _lib.orc_dedup_new.argtypes = [C.POINTER(OrcCfg)]
        _lib.orc_dedup_new.restype = C.c_void_p
        _lib.orc_dedup_free.argtypes = [C.c_void_p]
        _lib.orc_dedup_texts.argtypes = [C.c_void_p, C.c_char_p, C.c_size_t, C.c_int, C.POINTER(C.c_uint64),
                                         C.POINTER(C.c_double)]
    return _lib


def cfg_of(n_server, n_value, max_term, max_log, max_copies, max_msgs=0, invariants=(),
           max_distinct=0, symmetry=False, max_levels=0):
    m = 0
    for n in invariants:
        m |= INV[n]
    return OrcCfg(n_server, n_value, max_term, max_log, max_copies, m, 0, max_msgs, max_distinct, int(symmetry), max_levels)


def bfs(cfg: OrcCfg, threads=8, keep_trace=False, text_hash=False):
    r = OrcResult()
    rc = lib().orc_bfs(C.byref(cfg), threads, int(keep_trace), int(text_hash), C.byref(r))
    out = {
        "rc": rc, "distinct": r.distinct, "generated": r.generated, "depth": r.depth,
        "violated": r.violated,
        "levels": [[r.level_new[k], r.level_gen[k]] for k in range(r.n_levels)],
        "coverage": list(r.coverage)[:15], "seconds": r.seconds,
        "max_msgs": r.max_msgs, "trace_len": r.trace_len,
    }
    if text_hash:
        out["level_text_hash"] = [r.level_text_hash[k] for k in range(r.n_levels)]
    if r.trace_text:
        out["trace_text"] = C.string_at(r.trace_text).decode()
        lib().orc_free(r.trace_text)
    return out


def text_hash(text: str) -> int:
    return lib().orc_text_hash(text.encode())


class Walk:
    """Lockstep walker: the oracle's view of one current state."""

    def __init__(self, cfg: OrcCfg):
        self.h = lib().orc_walk_new(C.byref(cfg))

    def successors(self):
        cap = 1 << 20
        while True:
            buf = C.create_string_buffer(cap)
            n = lib().orc_walk_successors(self.h, buf, cap)
            if n >= 0:
                break
            if n > -(1 << 40) and -n > cap:
                cap = -n + 16
                continue
            raise RuntimeError("oracle walk error %d" % n)
        items = [x for x in buf.raw[:buf.raw.index(b"\0")].decode().split("\x1e") if x]
        return [(it[0] == "1", it[2:]) for it in items]

    def orbits(self):
        """SYMMETRY: for each successor of the last successors() call, its
        oracle seen-set key (hash of the least orbit serialisation, hex) and
        its orbit text."""
        cap = 1 << 20
        while True:
            buf = C.create_string_buffer(cap)
            n = lib().orc_walk_orbits(self.h, buf, cap)
            if n >= 0:
                break
            cap = -n + 16
        items = [x for x in buf.raw[:buf.raw.index(b"\0")].decode().split("\x1e") if x]
        return [tuple(it.split("\x1f", 1)) for it in items]

    def goto(self, text: str):
        if lib().orc_walk_goto(self.h, text.encode()) != 0:
            raise KeyError("successor not found")

    def text(self) -> str:
        buf = C.create_string_buffer(1 << 20)
        lib().orc_walk_text(self.h, buf, 1 << 20)
        return buf.value.decode()

    def invariants(self) -> int:
        return lib().orc_walk_inv(self.h)

    def close(self):
        if self.h:
            lib().orc_walk_free(self.h)
            self.h = None

    def __del__(self):
        self.close()


class Dedup:
    """Next + dedup of arbitrary states given as state texts (the synthetic
    microbench's CPU leg): counts (generated, probes, new) accumulate over
    batches that share one seen set."""

    def __init__(self, cfg: OrcCfg):
        self.h = lib().orc_dedup_new(C.byref(cfg))
        self.counts = [0, 0, 0]
        self.seconds = 0.0

    def batch(self, texts: bytes, n: int, threads: int = 8):
        out = (C.c_uint64 * 3)(*self.counts)
        sec = C.c_double(0)
        if lib().orc_dedup_texts(self.h, texts, n, threads, out, C.byref(sec)) != 0:
            raise RuntimeError("oracle dedup: unparsable state text or capacity overflow")
        self.counts = list(out)
        self.seconds += sec.value
        return self.counts

    def close(self):
        if self.h:
            lib().orc_dedup_free(self.h)
            self.h = None

    def __del__(self):
        self.close()
