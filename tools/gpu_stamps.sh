# Per-phase cycle shares of the level kernel (RTLA_STAMPS build in exp/stamps) on cfg2 and the exhaust model.
set -o pipefail
O=gpurun_out/stamps; mkdir -p $O
for w in cfg2 raft3_v2_t2_l2_m2; do
  RTLA_STAMPS_PRINT=1 RTLA_LIB=$PWD/exp/stamps/librtla.so timeout -k 10 300 python bench.py --no-cpu --no-secondary --steps 1 --warmup 0 --workload $w > $O/$w.json 2> $O/$w.err || { tail -5 $O/$w.err; exit 1; }
done
python tools/stamp_shares.py $O/cfg2.err $O/raft3_v2_t2_l2_m2.err
