set -u
for fb in ${FBS:-32 33}; do
  echo "== fpset-log2 $fb"
  timeout -k 10 150 python bench.py --no-cpu --steps 3 --warmup 1 --fpset-log2 $fb > gpurun_out/exp_$fb.json 2>gpurun_out/exp_$fb.err || { tail -3 gpurun_out/exp_$fb.err; exit 1; }
  python -c "
import json; r=json.load(open('gpurun_out/exp_$fb.json'))
print('  value %.4g  kernel_ms %.2f  wall_ms %.2f mat_ms %.2f distinct %d' % (r['value'], r['roofline']['kernel_ms_total'], r['ms_per_step'], r['roofline']['k_materialize']['ms_total'], r['config']['distinct']))"
done
