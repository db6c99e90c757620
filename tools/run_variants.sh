#!/bin/bash
# Time each exp/<variant>/librtla.so on the bench workloads (perf experiments).
#   VARIANTS="a b" WORKLOADS="cfg2 raft3_v2_t2_l2_m2" bash tools/run_variants.sh
set -u
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out/variants; mkdir -p $OUT
for w in ${WORKLOADS:-cfg2 raft3_v2_t2_l2_m2}; do
  for v in ${VARIANTS:-$(ls exp)}; do  # <variant>[@<RTLA_XFLAGS>]
    d=${v%@*}; xf=0; [ "$v" != "$d" ] && xf=${v#*@}
    echo "== $v $w"
    RTLA_XFLAGS=$xf RTLA_LIB=$PWD/exp/$d/librtla.so timeout -k 10 150 python bench.py --no-cpu --no-secondary --steps 2 --warmup 1 \
      --workload $w ${BENCHARGS:-} > $OUT/$v.$w.json 2> $OUT/$v.$w.err
    rc=$?
    if [ $rc -ne 0 ]; then echo "rc=$rc"; tail -3 $OUT/$v.$w.err; exit $rc; fi
    python -c "
import json,sys; r=json.load(open('$OUT/$v.$w.json')); f=r['roofline']
print('  value %.4g  kernel_ms %.2f  wall_ms %.2f distinct %d probes/s %.3g' % (r['value'], f['kernel_ms_total'], r['ms_per_step'], r['config']['distinct'], f['random_access']['probes_per_s']))"
  done
done
