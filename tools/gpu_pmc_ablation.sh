#!/bin/bash
# PMC passes over tools/expand_ablation.py (each pass its own run + time limit).
set -u
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out/pmca
rm -rf "$OUT"; mkdir -p "$OUT"
export TMPDIR=/tmp
i=0
while IFS= read -r ctrs; do
  [ -z "$ctrs" ] && continue
  i=$((i+1))
  echo "== pass $i: $ctrs"
  timeout -k 10 120 rocprofv3 --pmc $ctrs --output-format csv -d "$OUT/p$i" -o p -- python tools/expand_ablation.py --reps 1 > "$OUT/p$i.log" 2>&1
  rc=$?; echo "   rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 "$OUT/p$i.log"; exit $rc; fi
done <<< "${PASSES:-}"
echo done
