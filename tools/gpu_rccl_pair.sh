#!/bin/bash
# Two RCCL ranks on the box's GPU(s): the multi-GPU exchange path end to end.
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out/rccl; mkdir -p $OUT
M=${1:-n3_v1_t2_l1_m1}
rm -f /tmp/rccl_id_$$
for r in 0 1; do
  NCCL_DEBUG=${NCCL_DEBUG:-WARN} timeout -k 10 120 python -u tests/rccl_pair.py $r 2 /tmp/rccl_id_$$ $M > $OUT/r$r.json 2> $OUT/r$r.err &
done
wait %1; a=$?; wait %2; b=$?
echo "rc $a $b"; cat $OUT/r0.json; tail -n 5 $OUT/r0.err; tail -n 5 $OUT/r1.err
[ $a -eq 0 ] && [ $b -eq 0 ]
