#!/bin/bash
# Profiling session for the committed profiles/: probe calibration, kernel
# trace with stats, and one PMC pass per counter group (FETCH_SIZE and
# WRITE_SIZE in passes of their own), all on the default bench workload.
# Each GPU step has its own time limit; any failure ends the script.
set -u
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out/pmc
rm -rf "$OUT"; mkdir -p "$OUT"
export TMPDIR=/tmp
B="python bench.py --steps 1 --warmup 0 --no-cpu ${BENCHARGS:-}"
step() {
  local name=$1 lim=$2; shift 2
  echo "== $name $(date +%T)"
  timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?; echo "   rc=$rc"; tail -3 "$OUT/$name.log" | cut -c1-300
  if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
}
step calib 300 python tools/probe_calib.py
step kt 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/kt" -o kt -- $B
step p1 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/p1" -o p -- $B
step p2 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/p2" -o p -- $B
step p3 200 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM --output-format csv -d "$OUT/p3" -o p -- $B
step bench 300 python bench.py --levels
echo done
