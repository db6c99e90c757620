#!/bin/bash
# bench.py under several RTLA_XFLAGS kernel variants (perf experiments).
set -u
for xf in ${XFS:-0 16 256}; do
  echo "== RTLA_XFLAGS=$xf"
  RTLA_XFLAGS=$xf timeout -k 10 120 python bench.py --no-cpu --steps 3 --warmup 1 > /tmp/b.json 2>/tmp/b.err || { tail -3 /tmp/b.err; exit 1; }
  python -c "
import json; r=json.load(open('/tmp/b.json'))
print('  value %.4g  kernel_ms %.2f  wall_ms %.2f distinct %d' % (r['value'], r['roofline']['kernel_ms_total'], r['ms_per_step'], r['config']['distinct']))"
done
