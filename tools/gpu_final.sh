# Round-end record: GPU suite, smoke, per-workload lines, the default bench line, then the profile.
set -o pipefail
export TMPDIR=/tmp
bash tools/gpu_suite_bench.sh || exit 1
cp gpurun_out/suite/bench.json gpurun_out/suite/bench_default.json
WORKLOADS="cfg2 raft3_v2_t2_l2_m2" SKIP_CALIB=0 bash tools/profile_r02.sh || exit 1
timeout -k 10 300 python bench.py --no-cpu --no-secondary --steps 2 --warmup 1 --workload cfg4 > gpurun_out/suite/cfg4.json 2> gpurun_out/suite/cfg4.err || { tail -5 gpurun_out/suite/cfg4.err; exit 1; }
echo final ok
