#!/bin/bash
# Kernel trace + PMC passes over one bench step (each pass its own run and time limit).
set -u
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out/pmc
rm -rf "$OUT"; mkdir -p "$OUT"
export TMPDIR=/tmp
B="python bench.py --steps 1 --warmup 0 --no-cpu ${BENCHARGS:-}"
step() {
  local name=$1 lim=$2; shift 2
  echo "== $name $(date +%T)"
  timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?; echo "   rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 "$OUT/$name.log"; echo "stopping after $name (rc=$rc)"; exit $rc; fi
}
step kt 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/kt" -o kt -- $B
i=0
while IFS= read -r ctrs; do
  [ -z "$ctrs" ] && continue
  i=$((i+1))
  step p$i 120 rocprofv3 --pmc $ctrs --output-format csv -d "$OUT/p$i" -o p -- $B
done <<< "${PASSES:-}"
echo done
