"""Debug: compare stored vs recomputed fingerprints for rows built by
k_expand_batch and by a one-level k_expand, for the same Init parent."""
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "raft-tla_amd"))
import rtla
cfg = rtla.Config(2, 2, 3, 2, 1, 1, (), fpset_log2=16, mem_budget=64 << 20)
init = rtla.init_row(cfg)
print("W", len(init), "init ok", rtla.stored_fingerprint(init) == rtla.row_fingerprint(cfg, init))
for (_, inst, sub, im, r) in rtla.expand_batch(cfg, [init]):
    print("batch inst", inst, rtla.stored_fingerprint(r) == rtla.row_fingerprint(cfg, r), ["%08x" % x for x in r[:8]])
with rtla.Checker(cfg) as ck:
    ck.init(); ck.step()
    for r in ck.frontier():
        s, f = rtla.stored_fingerprint(r), rtla.row_fingerprint(cfg, r)
        print("expand", s == f, "%016x %016x / %016x %016x" % (s[0], s[1], f[0], f[1]), ["%08x" % x for x in r[:8]])
        print("   diff a %016x b %016x" % ((s[0] - f[0]) % 2**64, (s[1] - f[1]) % 2**64))
