"""Summarise gpurun_out/pmc: per-kernel time (kernel trace) and counter sums."""
import collections, csv, glob, os, sys
root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc"
for r in csv.DictReader(open(os.path.join(root, "kt", "kt_kernel_stats.csv"))):
    print("%-40s calls %5s total %9.3f ms avg %9.1f us" % (r["Name"][:40], r["Calls"], float(r["TotalDurationNs"]) / 1e6,
                                                        float(r["AverageNs"]) / 1e3))
agg = collections.defaultdict(lambda: collections.defaultdict(float))
for f in sorted(glob.glob(os.path.join(root, "p*", "p_counter_collection.csv"))):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0][:40]
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
for k, d in agg.items():
    if "fill" in k or "copy" in k:
        continue
    print(k)
    wc = d.get("SQ_WAVE_CYCLES")
    for c, v in sorted(d.items()):
        extra = "  (%.3f of wave cycles)" % (v / wc) if wc and c.startswith(("SQ_WAIT", "SQ_ACTIVE")) else ""
        print("   %-28s %.4g%s" % (c, v, extra))
