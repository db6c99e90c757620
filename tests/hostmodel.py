"""TEST INFRASTRUCTURE: ctypes access to tests/hostmodel.cpp -- the product's
model header (rtla_model.h) compiled for the host -- so the CPU suite checks
the semantics the level kernel evaluates against the oracles without a GPU.
The library is built on first use into tests/_build/ (git-ignored)."""
import ctypes as C
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
SRC = os.path.join(HERE, "hostmodel.cpp")
CSRC = os.path.join(ROOT, "raft-tla_amd", "csrc")
OUT = os.path.join(HERE, "_build", "libhostmodel.so")
_lib = None


def lib():
    global _lib
    if _lib is None:
        deps = [SRC, os.path.join(CSRC, "rtla_model.h")]
        if not os.path.exists(OUT) or os.path.getmtime(OUT) < max(os.path.getmtime(d) for d in deps):
            os.makedirs(os.path.dirname(OUT), exist_ok=True)
            subprocess.check_call(["g++", "-O2", "-std=c++20", "-shared", "-fPIC", "-I", CSRC, "-o", OUT + ".tmp", SRC])
            os.replace(OUT + ".tmp", OUT)
        _lib = C.CDLL(OUT)
        P = C.POINTER
        ints = [C.c_int] * 9
        _lib.hm_expand.argtypes = ints + [P(C.c_uint32), C.c_size_t, P(C.c_uint32), P(C.c_uint64), C.c_size_t]
        _lib.hm_expand.restype = C.c_long
        _lib.hm_fingerprint.argtypes = ints + [P(C.c_uint32), P(C.c_uint64)]
    return _lib


def _params(cfg):
    k = cfg.bag_cap or (cfg.max_msgs + 1 if cfg.max_msgs > 0 else 32)
    e = max(1, cfg.elec_cap or (cfg.max_term - 1) * cfg.n_server)
    return (cfg.n_server, cfg.n_value, cfg.max_term, cfg.max_log, cfg.max_copies, cfg.max_msgs, k, e, cfg.inv_mask)


def expand(cfg, rows, words):
    """Every enabled successor, as rtla.expand_batch returns them:
    (input index, instance, receive-sub, in_model, row), sorted by (input, instance)."""
    n = len(rows)
    flat = (C.c_uint32 * max(1, n * words))()
    for k, r in enumerate(rows):
        flat[k * words:(k + 1) * words] = list(r)
    cap = max(1, n) * 512
    out = (C.c_uint32 * (cap * words))()
    info = (C.c_uint64 * cap)()
    got = lib().hm_expand(*_params(cfg), flat, n, out, info, cap)
    if got < 0:
        raise RuntimeError("hm_expand: %d" % got)
    res = []
    for k in range(got):
        v = info[k]
        res.append((v >> 32, v & 0xFFFF, (v >> 16) & 0x7FFF, bool(v >> 31 & 1), list(out[k * words:(k + 1) * words])))
    return res


def fingerprint(cfg, row):
    arr = (C.c_uint32 * len(row))(*row)
    out = (C.c_uint64 * 2)()
    lib().hm_fingerprint(*_params(cfg), arr, out)
    return out[0], out[1]
