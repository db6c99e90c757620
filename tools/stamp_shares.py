"""Weighted per-phase shares of the level kernel's wave-cycles from an
RTLA_STAMPS build's stderr (stamps lines); for capped workloads only the
timed run's levels (the second half of the lines) are counted."""
import re
import sys

for path in sys.argv[1:]:
    lines = [l for l in open(path) if l.startswith("stamps")]
    if "cfg" in path:
        lines = lines[len(lines) // 2:]
    tot, allc = {}, 0.0
    for line in lines:
        m = re.match(r"stamps level (\d+): (.*) \(([\d.e+]+) wave-cycles\)", line)
        c = float(m.group(3))
        allc += c
        for k, v in re.findall(r"([\w+]+) ([\d.]+)", m.group(2)):
            tot[k] = tot.get(k, 0.0) + float(v) * c
    print(path, " ".join("%s %.3f" % (k, v / allc) for k, v in tot.items()), "%.3g wave-cycles" % allc)
