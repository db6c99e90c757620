#!/usr/bin/env python3
"""Summarise a rocprofv3 kernel_stats.csv: per kernel (short name) calls,
total ms, share, average us."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
tot = sum(int(r["TotalDurationNs"]) for r in rows)
print("total device time %.1f ms" % (tot / 1e6))
for r in sorted(rows, key=lambda r: -int(r["TotalDurationNs"])):
    name = r["Name"].split("(")[0].replace("void ", "")[:40]
    print("%-40s %7s calls %9.2f ms %5.1f%% avg %9.1f us" % (name, r["Calls"], int(r["TotalDurationNs"]) / 1e6,
                                                           100.0 * int(r["TotalDurationNs"]) / tot,
                                                           float(r["AverageNs"]) / 1e3))
