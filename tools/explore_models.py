"""Size candidate bench models on the GPU: BFS until done, a distinct-state
cap or a time cap; prints per-model totals as JSON lines (exploration tool)."""
import json, os, sys, time
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "raft-tla_amd"))
import rtla  # noqa: E402

CANDS = [  # name: N, V, T, L, C, M
    ("raft3_v2_t2_l1_m3", (3, 2, 2, 1, 1, 3)),
    ("raft3_v2_t3_l1_m2", (3, 2, 3, 1, 1, 2)),
    ("raft3_v2_t2_l2_m2", (3, 2, 2, 2, 1, 2)),
    ("raft3_v2_t3_l2_m2", (3, 2, 3, 2, 1, 2)),
    ("raft3_v1_t3_l2_m2", (3, 1, 3, 2, 1, 2)),
]
cap_states = float(os.environ.get("CAP_STATES", 4e9))
cap_sec = float(os.environ.get("CAP_SEC", 40))
only = os.environ.get("ONLY")
for name, (n, v, t, l, c, m) in CANDS:
    if only and name not in only.split(","):
        continue
    cfg = rtla.Config(n, v, t, l, c, m, ("ElectionSafety", "LogMatching"), fpset_log2=int(os.environ.get("FPLOG2", 32)))
    t0 = time.time()
    with rtla.Checker(cfg) as ck:
        st = ck.init()
        status = "running"
        while st == rtla.OK:
            try:
                st = ck.step()
            except rtla.RtlaError as e:
                st = -1
                status = "error: %s" % e
                break
            d = sum(lv.new for lv in ck.levels)
            if d > cap_states or time.time() - t0 > cap_sec:
                status = "capped"
                break
        if st == rtla.DONE:
            status = "done"
        elif st == rtla.VIOLATION:
            status = "violation"
        lv = ck.levels
        out = {"model": name, "status": status, "levels": len(lv), "distinct": sum(x.new for x in lv),
               "generated": sum(x.generated for x in lv), "row_bytes": lv[0].row_bytes,
               "last_new": lv[-1].new, "kernel_ms": sum(x.kernel_ms for x in lv), "wall_s": time.time() - t0,
               "tail": [[x.new, round(x.kernel_ms, 2)] for x in lv[-6:]]}
        print(json.dumps(out), flush=True)
