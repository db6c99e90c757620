#!/usr/bin/env python3
"""Device-side resource usage of kernel translation units (hipcc
-Rpass-analysis=kernel-resource-usage): one line per function with its
VGPRs, AGPRs, spilled VGPRs, scratch bytes per lane, occupancy and LDS.

    python tools/resource_usage.py [unit ...] [-D...]   (units: csrc/*.hip names, default all)
"""
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "raft-tla_amd", "csrc")
FIELDS = [("VGPRs", "vgpr"), ("AGPRs", "agpr"), ("VGPRs Spill", "spill"), ("ScratchSize [bytes/lane]", "scratch"),
          ("Occupancy [waves/SIMD]", "occ"), ("LDS Size [bytes/block]", "lds")]


def usage(unit, flags):
    cmd = ["/opt/rocm/bin/hipcc", "-O3", "-std=c++20", "-fPIC", "--offload-arch=gfx950", "-Wno-unused-result",
           "-Rpass-analysis=kernel-resource-usage", "-c", "-o", "/dev/null", os.path.join(SRC, unit + ".hip")] + flags
    err = subprocess.run(cmd, capture_output=True, text=True).stderr
    rows, cur = [], None
    for line in err.splitlines():
        m = re.search(r"remark: +Function Name: (\S+)", line)
        if m:
            cur = {"name": m.group(1)}
            rows.append(cur)
            continue
        for key, short in FIELDS:
            m = re.search(r"remark: +%s: (\d+)" % re.escape(key), line)
            if m and cur is not None:
                cur[short] = int(m.group(1))
    return rows


def main():
    units = [a for a in sys.argv[1:] if not a.startswith("-")]
    flags = [a for a in sys.argv[1:] if a.startswith("-")]
    if not units:
        units = sorted(f[:-4] for f in os.listdir(SRC) if f.endswith(".hip"))
    print("# unit | function (mangled prefix) | VGPRs AGPRs | spill VGPR | scratch B/lane | waves/SIMD | LDS B")
    for u in units:
        for r in usage(u, flags):
            print("%s | %s | %s %s | %s | %s | %s | %s" % (u, r["name"][:90], r.get("vgpr"), r.get("agpr"),
                                                        r.get("spill"), r.get("scratch"), r.get("occ"), r.get("lds")))


if __name__ == "__main__":
    main()
