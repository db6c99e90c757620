# The multi-shard protocol on one GPU (virtual shards, device copies as transport): bench lines at 2 shards.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/vshards; mkdir -p $O
for w in raft3_v2_t2_l2_m2 cfg2; do
  timeout -k 10 400 python bench.py --no-cpu --no-secondary --steps 1 --warmup 0 --shards 2 --workload $w > $O/$w.json 2> $O/$w.err || { tail -5 $O/$w.err; exit 1; }
  python -c "
import json; r=json.load(open('$O/$w.json')); print('$w', r['value'], r['ms_per_step'], r['config'].get('distinct'), r['config'].get('levels'), r['config'].get('parallelism'))"
done
