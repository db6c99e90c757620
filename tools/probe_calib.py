"""Calibrate the random-access roofline of the fingerprint set: random 8-byte
CAS inserts (k_probe_bench) into tables far larger than the 256 MiB Infinity
Cache.  Prints one JSON line per table size."""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "raft-tla_amd"))
import rtla  # noqa: E402

for log2, n in [(24, 1 << 22), (28, 1 << 26), (30, 1 << 28), (32, 1 << 29)]:
    s, ins = rtla.probe_bench(log2, n)
    print(json.dumps({"table_bytes": 8 << log2, "inserts": n, "inserted": ins, "seconds": s,
                      "cas_per_s": n / s, "load_after": n / (1 << log2)}), flush=True)
