set -o pipefail
bash tools/gpu_stamps.sh > gpurun_out/stamps.log 2>&1 || { cat gpurun_out/stamps.log | tail; exit 1; }
cat gpurun_out/stamps.log
KT="c3|-|--workload cfg3;ex|-|--workload raft3_v2_t2_l2_m2" LIMIT=300 bash tools/gpu_kt.sh
