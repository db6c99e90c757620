#!/bin/bash
# PC sampling of the ablation run (beta rocprofv3 feature); each attempt time-limited.
set -u
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out/pcs
rm -rf "$OUT"; mkdir -p "$OUT"
export TMPDIR=/tmp
rocprofv3 -L > "$OUT/list.txt" 2>&1 || true
grep -i -A3 "pc_sampl\|PC sampling\|method" "$OUT/list.txt" | head -40
timeout -k 10 180 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method ${METHOD:-stochastic} \
  --pc-sampling-unit ${UNIT:-cycles} --pc-sampling-interval ${IVL:-1048576} --output-format csv -d "$OUT/run" -o pcs \
  -- python tools/expand_ablation.py --reps 2 > "$OUT/run.log" 2>&1
rc=$?; echo "rc=$rc"; tail -5 "$OUT/run.log"; ls -la "$OUT/run" 2>/dev/null | head
exit $rc
