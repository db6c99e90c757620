#!/bin/bash
# Build a perf-experiment variant of librtla.so into exp/<name>/ (extra -D flags),
# all translation units in parallel.  UNITS="u1 u2": compile only these units
# with the flags and link them with the in-tree build's other objects
# (raft-tla_amd/build/*.o, from make).
set -e
name=$1; shift
ROOT=$(cd "$(dirname "$0")/.." && pwd)
D=$ROOT/exp/$name; rm -rf $D; mkdir -p $D
H=/opt/rocm/bin/hipcc
F="-O3 -std=c++20 -fPIC --offload-arch=gfx950 -Wno-unused-result $*"
S=${SRC:-$ROOT/raft-tla_amd/csrc}  # SRC: a modified copy of csrc/ (its ../../include must hold rtla.h)
ALL=${ALL_UNITS:-"rtla_kernels rtla_kwave rtla_kpack rtla_kspec_a rtla_kspec_b rtla_ksym_a rtla_ksym_b rtla_kgeneric_a rtla_kgeneric_b"}
pids=""
if [ -n "$UNITS" ]; then
  for u in $ALL rtla_host rtla_text; do cp $ROOT/raft-tla_amd/build/$u.o $D/$u.o; done
  for u in $UNITS; do $H $F -c -o $D/$u.o $S/$u.hip & pids="$pids $!"; done
else
  for u in $ALL; do $H $F -c -o $D/$u.o $S/$u.hip & pids="$pids $!"; done
  $H $F -c -o $D/rtla_host.o $S/rtla_host.cpp & pids="$pids $!"
  $H $F -c -o $D/rtla_text.o $S/rtla_text.cpp & pids="$pids $!"
fi
for p in $pids; do wait $p || { echo "build_variant: a unit failed"; exit 1; }; done
$H -shared -fPIC --offload-arch=gfx950 -o $D/librtla.so $D/*.o -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
rm -f $D/*.o
