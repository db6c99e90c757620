#!/bin/bash
# Profiling session (round 4): the 2-shard exchange's kernel split, and the
# level kernel's HBM writes with and without register spills (3 waves/SIMD
# in-tree vs the 2-wave exp/w2 build) -- configs[1] at 15 levels.
set -o pipefail
O=gpurun_out/p6; rm -rf $O; mkdir -p $O && export TMPDIR=/tmp
B="python bench.py --steps 1 --warmup 0 --no-cpu --no-secondary --no-calib --workload cfg2 --cap-levels 15"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/s2 -o kt -- $B --shards 2 > $O/s2.json 2>$O/s2.err &&
timeout -k 10 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/w3 -o p -- $B > $O/w3.json 2>$O/w3.err &&
RTLA_LIB=exp/w2/librtla.so timeout -k 10 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/w2 -o p -- $B > $O/w2.json 2>$O/w2.err &&
RTLA_LIB=exp/w2/librtla.so timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/w2kt -o kt -- $B > $O/w2kt.json 2>$O/w2kt.err &&
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/w3kt -o kt -- $B > $O/w3kt.json 2>$O/w3kt.err
