#!/bin/bash
# GPU session (round 5): the multi-shard parity tests, then the cost of
# fingerprint ownership on configs[1]'s 17 benched levels with 1, 2, 4 and 8
# virtual shards, with and without the sent cache; JSON lines and stderr go
# to gpurun_out/shards/.  Every GPU step has its own time limit; the first
# failure ends the session.  SKIP_TESTS=1: the bench lines only.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/shards; mkdir -p $O
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  timeout -k 10 ${TEST_LIMIT:-900} python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
    -k "${PYTEST_K:-shard or ranks or ring or checkpoint or wave_kernel or digest_equals or sharding_invariant}" \
    > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
  grep -E "passed|failed" $O/tests.log | tail -2
fi
line() {  # tag, env assignments (or -), bench args
  local tag=$1 envs=$2; shift 2
  [ "$envs" = - ] && envs=""
  env $envs timeout -k 10 ${LIMIT:-400} python -u bench.py --no-cpu --no-secondary --no-calib --levels "$@" \
    > $O/$tag.json 2> $O/$tag.err || { echo "FAILED $tag"; tail -20 $O/$tag.err; exit 1; }
  python -c "
import json; r=json.load(open('$O/$tag.json')); c=r['config']
print('%-12s %.4g distinct/s  %.1f ms/step  levels %d' % ('$tag', r['value'], r['ms_per_step'], c['levels']))"
}
DEF="s1|-|--workload cfg2;s2|-|--workload cfg2 --shards 2;s4|-|--workload cfg2 --shards 4;s8|-|--workload cfg2 --shards 8"
DEF="$DEF;s2n|RTLA_SENT_CACHE=0|--workload cfg2 --shards 2;s8n|RTLA_SENT_CACHE=0|--workload cfg2 --shards 8"
IFS=';' read -ra SPECS <<< "${LINES:-$DEF}"
for spec in "${SPECS[@]}"; do
  IFS='|' read -r tag envs args <<< "$spec"
  line "$tag" "$envs" $args
done
