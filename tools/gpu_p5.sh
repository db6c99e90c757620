set -o pipefail
mkdir -p gpurun_out/p5 && export TMPDIR=/tmp
B="python bench.py --steps 1 --warmup 0 --no-cpu --no-secondary --no-calib"
RTLA_SYM_QUEUE=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/p5/q1 -o kt -- $B --workload cfg4 > gpurun_out/p5/q1.json 2>gpurun_out/p5/q1.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/p5/s2 -o kt -- $B --workload cfg2 --cap-levels 15 --shards 2 > gpurun_out/p5/s2.json 2>gpurun_out/p5/s2.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/p5/s1 -o kt -- $B --workload cfg2 --cap-levels 15 > gpurun_out/p5/s1.json 2>gpurun_out/p5/s1.err
