import os, sys, json, time
sys.path.insert(0, "raft-tla_amd")
import rtla
cfg = rtla.Config(3, 2, 2, 1, 1, 2, ("ElectionSafety", "LogMatching"), fpset_log2=30, mem_budget=60 << 30)
for mode in ["step", "time", "step"]:
    with rtla.Checker(cfg) as ck:
        ck.init()
        while len(ck.levels) < 34:
            ck.step()
        if mode == "step":
            ck.step()
            lv = ck.levels[-1]
            print(json.dumps({"mode": mode, "frontier": lv.frontier, "new": lv.new, "kernel_ms": lv.kernel_ms, "sec": lv.seconds}), flush=True)
        else:
            print(json.dumps({"mode": mode, "ms": ck.time_expand(0, 1), "ms2": ck.time_expand(0, 1)}), flush=True)
