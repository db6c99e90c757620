#!/bin/bash
# Quick GPU iteration: parity subset, bench, one SQ counter pass on the bench.
set -u
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out/quick
rm -rf "$OUT"; mkdir -p "$OUT"
export TMPDIR=/tmp
step() {
  local name=$1 lim=$2; shift 2
  echo "== $name $(date +%T)"
  timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?; echo "   rc=$rc"; tail -4 "$OUT/$name.log" | cut -c1-1500
  if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
}
step tests 600 python -u -m pytest tests/test_gpu.py -x -q --timeout 200 --timeout-method thread -k "${TESTK:-bfs_counts or level_contents or virtual_shards_match or counterexample or coverage or out_of_model}"
step bench 300 python bench.py --levels --no-cpu --steps 3
[ -n "${PMC:-}" ] && step pmc 120 rocprofv3 --pmc $PMC --output-format csv -d "$OUT/pmc" -o pmc -- python bench.py --steps 1 --warmup 0 --no-cpu
echo done
