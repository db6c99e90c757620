#!/bin/bash
# GPU session: bench lines side by side (perf experiments).  Each line is
# "name|env|bench args"; every step has its own time limit, the first failure ends it.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/cmp; mkdir -p $O
while IFS='|' read -r name envs args; do
  [ -z "$name" ] && continue
  echo "== $name $(date +%T)"
  env $envs timeout -k 10 ${LIMIT:-300} python -u bench.py --no-cpu --no-secondary $args > $O/$name.json 2> $O/$name.err \
    || { tail -5 $O/$name.err; exit 1; }
  python -c "
import json; r=json.loads([l for l in open('$O/$name.json') if l.startswith('{')][-1]); f=r['roofline']; c=r['config']
print('%-14s value %.4g ms/step %.1f kernel_ms_avg %.2f frac %.3f ra %.3f levels %s distinct %s' % ('$name', r['value'], r['ms_per_step'], f['kernel_ms_avg'], f['frac'], f['random_access']['frac'], c.get('levels'), c.get('distinct')))"
done < ${CMP_FILE:-/dev/stdin}
