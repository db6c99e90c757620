"""Ablation of the BFS level kernel on one real frontier: run the bench model
to level --level, then re-expand that frontier with k_expand_lane switches
(rtla_time_expand) and print the mean device time of each variant."""
import argparse, json, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "raft-tla_amd"))
import rtla  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--level", type=int, default=34)
ap.add_argument("--reps", type=int, default=3)
a = ap.parse_args()
cfg = rtla.Config(3, 2, 2, 1, 1, 2, ("ElectionSafety", "LogMatching"), fpset_log2=30)
with rtla.Checker(cfg) as ck:
    ck.init()
    while len(ck.levels) < a.level:
        ck.step()
    lv = ck.levels[-1]
    print("frontier", lv.new, flush=True)
    variants = [("full", 0), ("no_materialize", 8), ("block4_nopersist", 256 | 512 | 8),
                ("block1_nopersist", 512 | 8), ("block4_persist", 256 | 8), ("generic", 128 | 8),
                ("noprobe_nocover", 1 | 2 | 8), ("compaction_only", 64 | 8 | 2)]
    for name, xf in variants:
        ms = ck.time_expand(xf, a.reps)
        print(json.dumps({"variant": name, "xflags": xf, "ms": ms, "states_per_s": lv.new / ms * 1e3}), flush=True)
