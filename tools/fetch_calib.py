"""Calibrate rocprofv3 FETCH_SIZE / WRITE_SIZE on gfx950 for the two access
shapes of the level kernel, by running kernels whose byte counts are known
exactly (run under `rocprofv3 --pmc FETCH_SIZE` and `--pmc WRITE_SIZE`, one
pass each; tools/prof_summary.py divides the counters by these):

  1. k_probe_bench x3 (rtla_probe_bench2): n 8-byte accesses at uniformly
     random slots of a 2^30-slot table -- CAS inserts, CAS re-probes, load
     re-probes (the fingerprint-set access shape);
  2. k_expand_compact with XF_NO_CHUNKS|XF_NO_COVER (rtla_time_expand): the
     level kernel reading its frontier rows and doing nothing else -- E rows
     of S bytes, dword loads coalesced over 64 lanes (the row-stream shape).

Prints one JSON line with the known byte counts per dispatch, in dispatch order."""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "raft-tla_amd"))
import rtla  # noqa: E402

out = {}
n = 1 << 27
rtla.probe_bench2(30, n)
out["probe_bench"] = {"accesses_per_dispatch": n, "access_bytes": 8,
                      "dispatches": ["insert CAS (all new)", "re-probe CAS (all present)", "re-probe load (all present)"]}
cfg = rtla.Config(3, 2, 3, 2, 1, 0, ("ElectionSafety", "LogMatching"), bag_cap=18, fpset_log2=31)
with rtla.Checker(cfg) as ck:
    ck.init()
    while ck.levels[-1].new < 40_000_000:
        ck.step()
    E = ck.levels[-1].new
    S = ck.levels[-1].row_bytes
    ms = ck.time_expand(32 | 2, 1)
    out["row_stream"] = {"rows": E, "row_bytes": S, "bytes": E * S, "ms": ms,
                         "dispatch": "k_expand_compact XF_NO_CHUNKS|XF_NO_COVER (last k_expand_compact dispatch)"}
print(json.dumps(out), flush=True)
