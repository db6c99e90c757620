# A tiny model first (short limit), the GPU suite, then cfg2 / exhaust benches.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/suite; rm -rf $O; mkdir -p $O
timeout -k 10 180 python -u -m pytest tests/test_gpu.py -x -v --timeout 60 --timeout-method thread -k "bfs_counts and n1_v1" \
  > $O/tiny.log 2>&1; rc=$?; tail -4 $O/tiny.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1; rc=$?
tail -4 $O/tests.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" $O/tests.log | head -20; exit $rc; }
for w in cfg2 raft3_v2_t2_l2_m2 cfg1 cfg3 synthetic; do
  timeout -k 10 300 python bench.py --no-cpu --no-secondary --steps 2 --warmup 1 --workload $w > $O/$w.json 2> $O/$w.err || { tail -5 $O/$w.err; exit 1; }
  python -c "
import json; r=json.load(open('$O/$w.json')); f=r['roofline']
print('%-18s value %.4g %s ms/step %.1f kernel_ms %.2f frac %.3f ra %.3f' % ('$w', r['value'], r['unit'], r['ms_per_step'], f['kernel_ms_total'], f['frac'], f['random_access']['frac']))"
done
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { cat $O/smoke.log; exit 1; }
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
cat $O/bench.json
