#!/bin/bash
# GPU session: the -m gpu suite (per-test durations), smoke, then the default
# bench line.  Every GPU step has its own time limit; the first failure ends it.
# PYTEST_K: a -k expression selecting tests; NO_BENCH=1 skips the bench.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/suite; rm -rf $O; mkdir -p $O
K=(); [ -n "${PYTEST_K:-}" ] && K=(-k "$PYTEST_K")
timeout -k 10 ${SUITE_LIMIT:-1100} python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread \
  --durations=40 "${K[@]}" > $O/tests.log 2>&1; rc=$?
tail -45 $O/tests.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" $O/tests.log | head -20; exit $rc; }
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { cat $O/smoke.log; exit 1; }
[ "${NO_BENCH:-0}" = 1 ] && exit 0
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
cat $O/bench.json
