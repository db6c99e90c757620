#!/bin/bash
# One profiling session on the GPU box (run from the repo root via gpurun).
# Each GPU step has its own time limit; any crash-type exit stops the script.
set -u
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out/prof
mkdir -p "$OUT"
export TMPDIR=/tmp
W=${WORKLOAD:-raft3_v2_t2_l2_m2}
run() {  # name, limit, cmd...
  local name=$1 lim=$2; shift 2
  echo "== $name"; timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?; echo "   rc=$rc"; tail -3 "$OUT/$name.log"
  if [ $rc -gt 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
}
run calib 300 python tools/probe_calib.py
run trace 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/kt" -o kt -- python bench.py --steps 1 --warmup 0 --no-cpu --workload "$W"
run pmc_fetch 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pf" -o pf -- python bench.py --steps 1 --warmup 0 --no-cpu --workload "$W"
run pmc_write 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pw" -o pw -- python bench.py --steps 1 --warmup 0 --no-cpu --workload "$W"
run pmc_sq 400 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VMEM --output-format csv -d "$OUT/ps" -o ps -- python bench.py --steps 1 --warmup 0 --no-cpu --workload "$W"
echo done
