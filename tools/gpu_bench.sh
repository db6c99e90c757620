#!/bin/bash
# GPU session: bench lines (default line, then per-workload lines without the CPU
# leg), each under its own time limit; stderr progress goes to gpurun_out/bench/.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/bench; mkdir -p $O
for w in ${WORKLOADS:-default}; do
  if [ "$w" = default ]; then
    timeout -k 10 ${LIMIT:-600} python -u bench.py ${BENCH_ARGS:-} > $O/default.json 2> $O/default.err || { tail -20 $O/default.err; exit 1; }
    cat $O/default.json
  else
    timeout -k 10 ${LIMIT:-600} python -u bench.py --no-cpu --no-secondary --workload $w ${BENCH_ARGS:-} > $O/$w.json 2> $O/$w.err || { tail -20 $O/$w.err; exit 1; }
    python -c "
import json; r=json.load(open('$O/$w.json')); f=r['roofline']
print('%-18s value %.4g %s ms/step %.1f kernel_ms_avg %.2f frac %.3f ra %.3f levels %s' % ('$w', r['value'], r['unit'], r['ms_per_step'], f['kernel_ms_avg'], f['frac'], f['random_access']['frac'], r['config'].get('levels')))"
  fi
done
