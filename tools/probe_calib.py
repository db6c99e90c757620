"""Calibrate the random-access roofline of the fingerprint set (8-byte slots
at uniformly random positions of tables far larger than the 256 MiB Infinity
Cache, all CUs): inserts (CAS, every key new), re-probes by CAS and re-probes
by the load-first protocol the BFS kernel uses (every key present).  Prints
one JSON line per table size; the result is recorded in profiles/ and
DESIGN.md section 5 and used as bench.py's random-access ceiling."""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "raft-tla_amd"))
import rtla  # noqa: E402

for log2, n in [(28, 1 << 26), (30, 1 << 28), (32, 1 << 30)]:
    si, sc, sl, ins = rtla.probe_bench2(log2, n)
    print(json.dumps({"table_bytes": 8 << log2, "keys": n, "inserted": ins, "load": n / (1 << log2),
                      "insert_cas_per_s": n / si, "seen_cas_per_s": n / sc, "seen_load_per_s": n / sl}), flush=True)
