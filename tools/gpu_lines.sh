#!/bin/bash
# GPU session: one bench.py line per entry of LINES ("tag|bench args"), each
# under its own time limit, without the CPU leg; JSON lines and stderr
# progress go to gpurun_out/lines/.  The first failure ends the session.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/lines; mkdir -p $O
IFS=';' read -ra ENTRIES <<< "${LINES:-cfg2|--workload cfg2}"
for ent in "${ENTRIES[@]}"; do
  tag=${ent%%|*}; args=${ent#*|}
  timeout -k 10 ${LIMIT:-400} python -u bench.py --no-cpu --no-secondary $args > $O/$tag.json 2> $O/$tag.err \
    || { echo "FAILED $tag"; tail -20 $O/$tag.err; exit 1; }
  python -c "
import json; r=json.load(open('$O/$tag.json')); f=r['roofline']; ra=f['random_access']
print('%-14s value %.4g %s ms/step %.1f kernel_ms_avg %.2f frac %.3f ra %.3f (ceil %.3g/s) levels %s' % ('$tag', r['value'], r['unit'], r['ms_per_step'], f['kernel_ms_avg'], f['frac'], ra['frac'], ra['ceiling_per_s'], r['config'].get('levels')))"
done
