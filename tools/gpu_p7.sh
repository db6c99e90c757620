#!/bin/bash
# Profiling session (round 4): the set-clearing kernel (k_clear, 16-B
# nontemporal stores) against plain stores (exp/clr0) -- kernel traces of
# configs[1] at 15 levels on 1 and 2 shards and of the synthetic microbench.
set -o pipefail
O=gpurun_out/p7; rm -rf $O; mkdir -p $O && export TMPDIR=/tmp
B="python bench.py --steps 1 --warmup 0 --no-cpu --no-secondary --no-calib"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/s1 -o kt -- $B --workload cfg2 --cap-levels 15 > $O/s1.json 2>$O/s1.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/s2 -o kt -- $B --workload cfg2 --cap-levels 15 --shards 2 > $O/s2.json 2>$O/s2.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/syn -o kt -- $B --workload synthetic > $O/syn.json 2>$O/syn.err &&
RTLA_LIB=exp/clr0/librtla.so timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/s1c0 -o kt -- $B --workload cfg2 --cap-levels 15 > $O/s1c0.json 2>$O/s1c0.err &&
RTLA_LIB=exp/clr0/librtla.so timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/sync0 -o kt -- $B --workload synthetic > $O/sync0.json 2>$O/sync0.err
