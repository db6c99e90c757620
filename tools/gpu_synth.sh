# configs[4] path: synthetic parity tests, then the bench line (inputs resident in HBM).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/synth; rm -rf $O; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu.py -x -v --timeout 200 --timeout-method thread -k "synthetic" \
  > $O/tests.log 2>&1; rc=$?; tail -5 $O/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --workload synthetic --no-cpu > $O/synthetic.json 2> $O/synthetic.err || { tail -5 $O/synthetic.err; exit 1; }
cat $O/synthetic.json
