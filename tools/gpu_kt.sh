#!/bin/bash
# GPU session: rocprofv3 kernel traces (--kernel-trace --stats) of bench.py lines,
# one per entry of KT ("tag|env|bench args"), into gpurun_out/kt/<tag>/.
set -o pipefail
export TMPDIR=/tmp
O=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out/kt; mkdir -p $O
IFS=';' read -ra SPECS <<< "$KT"
for spec in "${SPECS[@]}"; do
  IFS='|' read -r tag envs args <<< "$spec"
  [ "$envs" = - ] && envs=""
  for e in $envs; do export "$e"; done
  timeout -k 10 ${LIMIT:-300} rocprofv3 --kernel-trace --stats --output-format csv -d $O/$tag -o kt -- \
    python bench.py --no-cpu --no-secondary --no-calib --steps 1 --warmup 0 $args > $O/$tag.json 2> $O/$tag.err \
    || { echo "FAILED $tag"; tail -20 $O/$tag.err; exit 1; }
  for e in $envs; do unset "${e%%=*}"; done
  python tools/kt_summary.py $O/$tag/kt_kernel_stats.csv | head -12
done
