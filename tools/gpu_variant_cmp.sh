# exp/$V against the default build: a parity subset for the variant, then paired benches.
set -o pipefail
export TMPDIR=/tmp
V=${V:-tpf}; O=gpurun_out/cmp_$V; rm -rf $O; mkdir -p $O
RTLA_LIB=$PWD/exp/$V/librtla.so timeout -k 10 400 python -u -m pytest tests/test_gpu.py -x -q --timeout 120 --timeout-method thread \
  -k "prefix_levels and (c1_prefix or m2_prefix)" > $O/tests.log 2>&1; rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
for w in ${WORKLOADS:-cfg2 raft3_v2_t2_l2_m2 cfg1}; do
  for v in base $V; do
    lib=$PWD/raft-tla_amd/librtla.so; [ $v = base ] || lib=$PWD/exp/$v/librtla.so
    RTLA_LIB=$lib timeout -k 10 300 python bench.py --no-cpu --no-secondary --steps 2 --warmup 1 --workload $w > $O/$v.$w.json 2> $O/$v.$w.err || { tail -5 $O/$v.$w.err; exit 1; }
    python -c "
import json; r=json.load(open('$O/$v.$w.json')); f=r['roofline']
print('%-6s %-18s value %.4g ms/step %.1f kernel_ms %.2f' % ('$v', '$w', r['value'], r['ms_per_step'], f['kernel_ms_total']))"
  done
done
