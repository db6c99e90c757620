#!/bin/bash
# Time each exp/<variant>/librtla.so on the bench workload (perf experiments).
set -u
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out/variants; mkdir -p $OUT
for d in ${VARIANTS:-$(ls exp)}; do
  echo "== $d"
  RTLA_LIB=$PWD/exp/$d/librtla.so timeout -k 10 120 python bench.py --no-cpu --steps 2 --warmup 1 ${BENCHARGS:-} > $OUT/$d.json 2> $OUT/$d.err
  rc=$?
  if [ $rc -ne 0 ]; then echo "rc=$rc"; tail -3 $OUT/$d.err; exit $rc; fi
  python -c "
import json,sys; r=json.load(open('$OUT/$d.json'))
print('  value %.4g  kernel_ms %.2f  wall_ms %.2f distinct %d probes/s %.3g' % (r['value'], r['roofline']['kernel_ms_total'], r['ms_per_step'], r['config']['distinct'], r['roofline']['probes_per_s']))"
done
