"""Summarise a gpurun_out/pmc directory (tools/gpu_pmc.sh): per-kernel time
from the kernel trace and counter sums per kernel.  With --traffic-out FILE
it also writes the probe kernel's HBM bytes per launch (FETCH_SIZE +
WRITE_SIZE passes) for bench.py's roofline.traffic.

    python tools/pmc_summary.py [gpurun_out/pmc] [--workload W --traffic-out profiles/rNN/traffic.json]
"""
import argparse
import collections
import csv
import glob
import json
import os

ap = argparse.ArgumentParser()
ap.add_argument("root", nargs="?", default="gpurun_out/pmc")
ap.add_argument("--workload", default="raft3_v2_t2_l2_m2")
ap.add_argument("--traffic-out")
a = ap.parse_args()
for r in csv.DictReader(open(os.path.join(a.root, "kt", "kt_kernel_stats.csv"))):
    print("%-44s calls %5s total %10.3f ms avg %10.1f us" % (r["Name"][:44], r["Calls"],
                                                            float(r["TotalDurationNs"]) / 1e6,
                                                            float(r["AverageNs"]) / 1e3))
agg = collections.defaultdict(lambda: collections.defaultdict(float))
disp = collections.defaultdict(lambda: collections.defaultdict(set))
for f in sorted(glob.glob(os.path.join(a.root, "p*", "p_counter_collection.csv"))):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].replace("void ", "")[:44]
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
        disp[k][r["Counter_Name"]].add((f, r["Dispatch_Id"]))
for k, d in agg.items():
    if "fill" in k or "copy" in k:
        continue
    print(k)
    wc = d.get("SQ_WAVE_CYCLES")
    for c, v in sorted(d.items()):
        extra = "  (%.3f of wave cycles)" % (v / wc) if wc and c.startswith(("SQ_WAIT", "SQ_ACTIVE")) else ""
        print("   %-28s %.4g%s" % (c, v, extra))
if a.traffic_out:
    k = next(k for k in agg if k.startswith("k_expand_compact"))
    d = agg[k]
    n_f = len(disp[k]["FETCH_SIZE"])
    n_w = len(disp[k]["WRITE_SIZE"])
    out = {"workload": a.workload, "kernel": "k_expand_compact",
           "launches_fetch_pass": n_f, "launches_write_pass": n_w,
           "fetch_bytes_per_launch": d["FETCH_SIZE"] * 1024 / n_f,
           "write_bytes_per_launch": d["WRITE_SIZE"] * 1024 / n_w,
           "note": "rocprofv3 FETCH_SIZE / WRITE_SIZE (KiB) in separate passes, summed over XCDs, per dispatch. "
                   "The probe kernel's traffic is 8-B loads and CAS at random slots plus dword row reads: the "
                   "guide's x2 FETCH correction applies to 16-B/lane streaming reads only and is NOT applied; "
                   "per-access units are calibrated against tools/probe_calib.py in DESIGN.md section 5."}
    out["bytes_per_launch"] = out["fetch_bytes_per_launch"] + out["write_bytes_per_launch"]
    os.makedirs(os.path.dirname(a.traffic_out), exist_ok=True)
    json.dump(out, open(a.traffic_out, "w"), indent=1)
    print("wrote", a.traffic_out, out["bytes_per_launch"])
