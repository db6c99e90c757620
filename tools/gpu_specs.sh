# Compiled-in layouts for BASELINE configs[2]/[3]/[4]: parity of the kernels
# they select, then each workload with the compiled-in 16-state groups
# (default), the run-time layout (RTLA_XFLAGS=4096, 32-state groups) and the
# compiled-in layout at 32-state groups (exp/g32).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/specs; rm -rf $O; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu.py -x -v --timeout 400 --timeout-method thread \
  -k "prefix_levels or synthetic or symmetry" > $O/tests.log 2>&1; rc=$?; tail -4 $O/tests.log; [ $rc -eq 0 ] || exit $rc
run() {  # name workload [env...]
  local name=$1 w=$2; shift 2
  env "$@" timeout -k 10 200 python bench.py --no-cpu --no-secondary --steps 2 --warmup 1 --workload $w \
    > $O/$name.json 2> $O/$name.err || { echo "rc=$? $name"; tail -3 $O/$name.err; return 1; }
  python -c "
import json; r=json.load(open('$O/$name.json')); f=r['roofline']
print('%-16s value %.4g %s ms/step %.1f kernel_ms %.2f distinct %d levels %s' % ('$name', r['value'], r['unit'], r['ms_per_step'], f['kernel_ms_total'], r['config'].get('distinct', 0), r['config'].get('levels')))"
}
run cfg4.sym1 cfg4 RTLA_LIB=$PWD/exp/sym1/librtla.so || exit 1
for w in cfg3 cfg4 synthetic; do
  run $w.spec16 $w X=1 && run $w.runtime $w RTLA_XFLAGS=4096 && run $w.spec32 $w RTLA_LIB=$PWD/exp/g32/librtla.so || exit 1
done
