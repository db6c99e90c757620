"""Summarise a tools/profile.sh run (gpurun_out/prof): per workload the
kernel-trace stats and PMC counters of k_expand_compact, HBM bytes per launch
from FETCH_SIZE / WRITE_SIZE corrected by the calibration of
tools/fetch_calib.py (known byte counts, same gfx950 counters), and a
traffic.json for bench.py's roofline.traffic.

    python tools/prof_summary.py gpurun_out/prof profiles/r02_XX
"""
import collections
import csv
import glob
import json
import os
import sys

root, dest = sys.argv[1], sys.argv[2]
os.makedirs(dest, exist_ok=True)


def dispatches(path, kernel_prefix=None):
    """[(dispatch id, kernel name, {counter: value})] in dispatch order."""
    d = collections.OrderedDict()
    for r in csv.DictReader(open(path)):
        k = int(r["Dispatch_Id"])
        if k not in d:
            d[k] = (r["Kernel_Name"], collections.defaultdict(float))
        d[k][1][r["Counter_Name"]] += float(r["Counter_Value"])
    out = [(k, n, c) for k, (n, c) in d.items()]
    if kernel_prefix:
        out = [x for x in out if kernel_prefix in x[1]]
    return out


lines = []
calib = {}
cal_log = open(os.path.join(root, "calib.fetch.log")).read()
known = json.loads([l for l in cal_log.splitlines() if l.startswith("{")][-1])
for ctr, sub in (("FETCH_SIZE", "p1"), ("WRITE_SIZE", "p2")):
    f = os.path.join(root, "calib", sub, "p_counter_collection.csv")
    pb = dispatches(f, "k_probe_bench")
    ex = dispatches(f, "k_expand_compact")
    n = known["probe_bench"]["accesses_per_dispatch"]
    calib[ctr] = {"probe_insert_cas_bytes_per_access": pb[0][2][ctr] * 1024 / n,
                  "probe_seen_cas_bytes_per_access": pb[1][2][ctr] * 1024 / n,
                  "probe_seen_load_bytes_per_access": pb[2][2][ctr] * 1024 / n,
                  "row_stream_counted_over_true": ex[-1][2][ctr] * 1024 / known["row_stream"]["bytes"]}
lines.append("calibration (counter KiB x 1024 / known): " + json.dumps(calib, indent=1))
stream_f = calib["FETCH_SIZE"]["row_stream_counted_over_true"]
for wdir in sorted(glob.glob(os.path.join(root, "*", "kt"))):
    wd = os.path.dirname(wdir)
    w = os.path.basename(wd)
    lines.append("\n== %s" % w)
    for r in csv.DictReader(open(os.path.join(wdir, "kt_kernel_stats.csv"))):
        lines.append("%-60s calls %5s total %10.3f ms avg %10.1f us %5.1f%%" % (
            r["Name"][:60], r["Calls"], float(r["TotalDurationNs"]) / 1e6, float(r["AverageNs"]) / 1e3,
            float(r["Percentage"])))
    agg = collections.defaultdict(float)
    nd = {}
    for sub in ("p1", "p2", "p3", "p4"):
        f = os.path.join(wd, sub, "p_counter_collection.csv")
        if not os.path.exists(f):
            continue
        ds = dispatches(f, "k_expand_compact")
        for _, _, c in ds:
            for k, v in c.items():
                if k == "SQ_WAVE_CYCLES" and sub == "p4":
                    k = "SQ_WAVE_CYCLES_p4"
                agg[k] += v
        nd[sub] = len(ds)
    wc = agg.get("SQ_WAVE_CYCLES")
    wc4 = agg.get("SQ_WAVE_CYCLES_p4")
    lines.append("k_expand_compact counters (sum over %s launches)" % nd)
    for c, v in sorted(agg.items()):
        base = wc4 if c in ("SQ_WAIT_INST_ANY", "SQ_WAIT_INST_LDS") else wc
        extra = "  (%.3f of wave cycles)" % (v / base) if base and c.startswith(("SQ_WAIT", "SQ_ACTIVE")) else ""
        lines.append("   %-26s %.4g%s" % (c, v, extra))
    if "FETCH_SIZE" in agg and "WRITE_SIZE" in agg:
        fetch = agg["FETCH_SIZE"] * 1024 / nd["p1"]
        write = agg["WRITE_SIZE"] * 1024 / nd["p2"]
        # probes per launch from the bench line of the kernel-trace run
        probes = None
        try:
            kt_log = open(os.path.join(root, "%s.kt.log" % w)).read()
            b = json.loads([l for l in kt_log.splitlines() if l.startswith('{"metric"')][-1])
            ra = b["roofline"]["random_access"]
            probes = ra["probes_per_s"] * b["roofline"]["kernel_ms_avg"] / 1e3
        except (OSError, ValueError, KeyError, IndexError):
            pass
        per_load = calib["FETCH_SIZE"]["probe_seen_load_bytes_per_access"]
        if probes is not None:  # random probe loads count ~64 B each; the rest is the row streams
            probe_fetch = probes * per_load
            fetch_true = probe_fetch + max(0.0, fetch - probe_fetch) / stream_f
        else:
            fetch_true = fetch / stream_f
        t = {"workload": w, "kernel": "k_expand_compact", "launches": nd["p1"],
             "fetch_bytes_per_launch_raw": fetch, "write_bytes_per_launch_raw": write,
             "probes_per_launch": probes,
             "fetch_bytes_per_launch": fetch_true, "write_bytes_per_launch": write,
             "calibration": calib,
             "note": "FETCH_SIZE: the fingerprint-set probe loads (probes per launch from the bench line x the "
                     "calibrated counted bytes per random load, ~64 B) plus the remainder divided by the "
                     "counted/true ratio of a known row stream (tools/fetch_calib.py: the level kernel reading E "
                     "rows and nothing else).  WRITE_SIZE as counted (each fingerprint-set CAS counts ~68 B)."}
        t["bytes_per_launch"] = t["fetch_bytes_per_launch"] + t["write_bytes_per_launch"]
        json.dump(t, open(os.path.join(dest, "traffic_%s.json" % w), "w"), indent=1)
        lines.append("   HBM bytes per launch: fetch %.4g (raw %.4g) + write %.4g = %.4g" % (
            t["fetch_bytes_per_launch"], fetch, write, t["bytes_per_launch"]))
open(os.path.join(dest, "pmc_summary.txt"), "w").write("\n".join(lines) + "\n")
print("\n".join(lines))
