#!/bin/bash
# Profiling session (round 2 onwards): for each workload a kernel trace with stats and
# PMC passes (FETCH_SIZE and WRITE_SIZE in passes of their own, two SQ
# groups), plus the FETCH/WRITE calibration of tools/fetch_calib.py.  Each GPU
# step has its own time limit; any failure ends the script.
set -u
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out/prof
rm -rf "$OUT"; mkdir -p "$OUT"
export TMPDIR=/tmp
step() {
  local name=$1 lim=$2; shift 2
  echo "== $name $(date +%T)"
  timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?; echo "   rc=$rc"; tail -2 "$OUT/$name.log" | cut -c1-300
  if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
}
SQ1="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM"
SQ2="SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SMEM"
for W in ${WORKLOADS:-cfg2 raft3_v2_t2_l2_m2}; do
  # the benched depth without a sizing run inside the profile (cfg4: no oracle-pinned depth)
  CAP=""; [ "$W" = cfg2 ] && CAP="--cap-levels 17"; [ "$W" = cfg4 ] && CAP="--cap-levels 15"
  B="python bench.py --steps 1 --warmup 0 --no-cpu --no-secondary --workload $W $CAP"
  step $W.kt 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/$W/kt" -o kt -- $B
  step $W.fetch 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/$W/p1" -o p -- $B
  step $W.write 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/$W/p2" -o p -- $B
  step $W.sq1 200 rocprofv3 --pmc $SQ1 --output-format csv -d "$OUT/$W/p3" -o p -- $B
  [ "${SKIP_SQ2:-0}" = 1 ] || step $W.sq2 200 rocprofv3 --pmc $SQ2 --output-format csv -d "$OUT/$W/p4" -o p -- $B
done
if [ "${SKIP_CALIB:-0}" != 1 ]; then
  step calib.fetch 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/calib/p1" -o p -- python tools/fetch_calib.py
  step calib.write 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/calib/p2" -o p -- python tools/fetch_calib.py
fi
echo done
