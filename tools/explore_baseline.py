"""Run BASELINE.json configs[0]/configs[1] as stated (no MaxInFlight) on one
GPU until the search is exhausted or device memory runs out; print the
per-level table.  Evidence for DESIGN.md section 2 (committed under
profiles/).

    python tools/explore_baseline.py cfg2 [fpset_log2] [bag_cap]
"""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "raft-tla_amd"))
import rtla  # noqa: E402

SHAPES = {
    "cfg1": (3, 1, 2, 1, 1, 0, ("NoTwoLeaders",)),                  # raft.cfg bounds, BASELINE configs[0]
    "cfg2": (3, 2, 3, 2, 1, 0, ("ElectionSafety", "LogMatching")),  # BASELINE configs[1]
}
name = sys.argv[1]
fpl = int(sys.argv[2]) if len(sys.argv) > 2 else 31
bag = int(sys.argv[3]) if len(sys.argv) > 3 else 0
n, v, t, l, c, m, inv = SHAPES[name]
cfg = rtla.Config(n, v, t, l, c, m, inv, fpset_log2=fpl, bag_cap=bag)
t0 = time.time()
with rtla.Checker(cfg) as ck:
    print(ck.device_info(), flush=True)
    st = ck.init()
    status = "running"
    while st == rtla.OK:
        try:
            st = ck.step()
        except rtla.RtlaError as e:
            status = "stopped: %s" % e
            break
        lv = ck.levels[-1]
        print("level %3d frontier %12d new %12d generated %13d kernel %9.3f ms (probe %9.3f ms) wall %.3f s"
              % (lv.level, lv.frontier, lv.new, lv.generated, lv.kernel_ms, lv.expand_ms, lv.seconds), flush=True)
    if st == rtla.DONE:
        status = "exhausted"
    elif st == rtla.VIOLATION:
        status = "violation %s" % (ck.violation(),)
    lv = ck.levels
    print("%s: %s after %d complete levels, %d distinct, %d generated, row %d B, kernel %.1f ms, wall %.2f s"
          % (name, status, len(lv), sum(x.new for x in lv), sum(x.generated for x in lv), lv[0].row_bytes,
             sum(x.kernel_ms for x in lv), time.time() - t0), flush=True)
