#!/bin/bash
# One bench line per BASELINE workload (capped ones from Init to the deepest level that fits).
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out/wl; mkdir -p $OUT
for w in ${WORKLOADS:-cfg1 cfg3 cfg4 synthetic}; do
  echo "== $w $(date +%T)"
  timeout -k 10 300 python bench.py --workload $w --steps ${STEPS:-1} --warmup ${WARMUP:-1} --no-secondary --levels > $OUT/$w.json 2> $OUT/$w.err || { tail -5 $OUT/$w.err; exit 1; }
  python -c "import json; r=json.load(open('$OUT/$w.json')); c=r['config']; print('  %.4g %s  %.1f ms/step  levels %s distinct %s' % (r['value'], r['unit'], r['ms_per_step'], c.get('levels'), c.get('distinct')))"
done
