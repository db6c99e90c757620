# Level-kernel change check: parity subset, bench cfg2 + exhaust, stamps variant on cfg2.
set -o pipefail
O=gpurun_out/check; rm -rf $O; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu.py -x -q --timeout 200 --timeout-method thread \
  -k "bfs_counts or level_contents or virtual_shards_match or counterexample or coverage or out_of_model or prefix_levels or synthetic or overflow or ring_arena" > $O/tests.log 2>&1 && tail -3 $O/tests.log &&
timeout -k 10 300 python bench.py --no-cpu --no-secondary --steps 3 --warmup 1 > $O/cfg2.json 2> $O/cfg2.err &&
timeout -k 10 300 python bench.py --no-cpu --no-secondary --steps 2 --warmup 1 --workload raft3_v2_t2_l2_m2 > $O/exh.json 2> $O/exh.err &&
RTLA_STAMPS_PRINT=1 RTLA_LIB=$PWD/exp/stamps/librtla.so timeout -k 10 300 python bench.py --no-cpu --no-secondary --steps 1 --warmup 1 > $O/stamps_cfg2.json 2> $O/stamps_cfg2.err &&
python tools/stamp_shares.py $O/stamps_cfg2.err &&
grep -o '"kernel_ms_avg": [0-9.]*' $O/*.json && grep -o '"value": [0-9.e+]*' $O/*.json
