set -o pipefail
mkdir -p gpurun_out/baseline
timeout -k 10 60 ./tools/lds_occupancy > gpurun_out/baseline/occ.txt 2>&1 && cat gpurun_out/baseline/occ.txt &&
timeout -k 10 300 python bench.py --no-cpu --no-secondary --steps 3 --warmup 1 --levels > gpurun_out/baseline/cfg2.json 2> gpurun_out/baseline/cfg2.err && tail -c 600 gpurun_out/baseline/cfg2.json &&
timeout -k 10 300 python bench.py --no-cpu --no-secondary --steps 2 --warmup 1 --workload raft3_v2_t2_l2_m2 > gpurun_out/baseline/exh.json 2> gpurun_out/baseline/exh.err && tail -c 300 gpurun_out/baseline/exh.json
