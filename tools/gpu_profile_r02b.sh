# Profile of the refactored level kernel (tools/profile_r02.sh) and the configs[3] bench line.
set -o pipefail
export TMPDIR=/tmp
WORKLOADS="cfg2 raft3_v2_t2_l2_m2" bash tools/profile_r02.sh || exit 1
mkdir -p gpurun_out/prof
timeout -k 10 300 python bench.py --no-cpu --no-secondary --steps 2 --warmup 1 --workload cfg4 > gpurun_out/prof/cfg4.json 2> gpurun_out/prof/cfg4.err || { tail -5 gpurun_out/prof/cfg4.err; exit 1; }
tail -c 400 gpurun_out/prof/cfg4.json
