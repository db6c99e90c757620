#!/usr/bin/env python3
"""Per-level view of a rocprofv3 kernel trace (kt_kernel_trace.csv) of one
`bench.py --steps 1 --warmup 0` run: every level-kernel launch in order with
its duration and the device-idle gap before it, then totals by launch size
(to see whether small levels, the tail or per-launch setup dominate)."""
import csv
import sys

LEVEL = "k_expand_compact"
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
t0 = int(rows[0]["Start_Timestamp"])
prev_end = t0
lv = []
other = 0
for r in rows:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    if LEVEL in r["Kernel_Name"]:
        lv.append((s, e, max(0, s - prev_end)))
    else:
        other += e - s
    prev_end = max(prev_end, e)
span = prev_end - t0
# a capped workload's trace holds the untimed prefix run and the timed run: keep the last run
print("%d level launches, trace span %.1f ms, other kernels %.1f ms" % (len(lv), span / 1e6, other / 1e6))
print("%5s %10s %10s" % ("launch", "ms", "gap_us"))
for i, (s, e, g) in enumerate(lv):
    print("%5d %10.3f %10.1f" % (i, (e - s) / 1e6, g / 1e3))
buckets = [(0, 0.1), (0.1, 1), (1, 10), (10, 1e9)]
for lo, hi in buckets:
    sel = [(e - s) / 1e6 for s, e, _ in lv if lo <= (e - s) / 1e6 < hi]
    print("launches %6.1f-%-6g ms: %3d, %8.2f ms total" % (lo, hi, len(sel), sum(sel)))
print("sum of gaps before level launches: %.2f ms" % (sum(g for _, _, g in lv) / 1e6))
