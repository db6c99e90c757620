"""How many permutations the orbit key tries per state (|C(s)|, rtla_orbit_key's
`perms`) on reachable configs[3] states: run the symmetric search on the GPU
for some levels, sample the frontier, count on the host.  Also the per-wave
maximum over 64 consecutive states (a key pass iterates as long as its
slowest lane).

    python tools/sym_perms.py [levels] [sample]
"""
import collections
import json
import os
import random
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "raft-tla_amd"))
import rtla  # noqa: E402

levels = int(sys.argv[1]) if len(sys.argv) > 1 else 11
sample = int(sys.argv[2]) if len(sys.argv) > 2 else 64 * 2000
cfg = rtla.Config(5, 1, 3, 2, 1, 0, (), symmetry=True, bag_cap=20, fpset_log2=28, mem_budget=40 << 30)
with rtla.Checker(cfg) as ck:
    st = ck.init()
    while st == rtla.OK and len(ck.levels) < levels:
        st = ck.step()
    rows = ck.frontier()
n = len(rows)
start = random.Random(1).randrange(0, max(1, n - sample))
sel = rows[start:start + sample]
perms = [rtla.orbit_key(cfg, r)[1] for r in sel]
hist = collections.Counter(perms)
waves = [max(perms[i:i + 64]) for i in range(0, len(perms) - 63, 64)]
out = {"levels": levels, "frontier": n, "sample": len(perms), "mean_perms": sum(perms) / len(perms),
       "hist": dict(sorted(hist.items())), "mean_wave_max": sum(waves) / max(1, len(waves)),
       "wave_max_hist": dict(sorted(collections.Counter(waves).items()))}
print(json.dumps(out))
