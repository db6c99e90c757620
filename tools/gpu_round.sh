#!/bin/bash
# One GPU session: gpu tests, bench, kernel-trace profile.  Each GPU step has
# its own limit; any crash-type exit ends the script (no further GPU steps).
set -u
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out/round
mkdir -p "$OUT"
export TMPDIR=/tmp
W=${WORKLOAD:-raft3_v2_t2_l2_m2}
step() {  # name, limit, cmd...
  local name=$1 lim=$2; shift 2
  echo "== $name $(date +%T)"
  timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?; echo "   rc=$rc"; tail -5 "$OUT/$name.log"
  if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
}
[ "${SKIP_TESTS:-0}" = 1 ] || step tests 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ${TESTK:+-k "$TESTK"}
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench 600 python bench.py --levels
[ "${SKIP_TRACE:-0}" = 1 ] || step trace 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/kt" -o kt -- python bench.py --steps 2 --warmup 1 --no-cpu --workload "$W"
echo done
