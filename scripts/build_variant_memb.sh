#!/bin/bash
# Experiment builds of the membership kernels: raft-tla_amd/_build_var/NAME/libraftmc.so with extra
# -D flags on memb_backend.hip (the rest linked from _build).  Select with RAFTMC_LIB=<path>.
#   scripts/build_variant_memb.sh NAME "-DRMC_FP_DUP_MINPERM"
set -e
NAME=$1; DEFS=$2
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT=$ROOT/raft-tla_amd/_build_var/$NAME
mkdir -p "$OUT"
H=/opt/rocm/bin/hipcc
F="-O3 -std=c++17 -fPIC -Wall -Wno-unused-function"
C=$ROOT/raft-tla_amd/csrc
B=$ROOT/raft-tla_amd/_build
$H $F --offload-arch=gfx950 -munsafe-fp-atomics $DEFS -I$C -c -o "$OUT/memb_backend.o" $C/memb_backend.hip
$H -shared --offload-arch=gfx950 -o "$OUT/libraftmc.so" $B/orig_backend.o "$OUT/memb_backend.o" \
   $B/mc_api.o $B/model.o $B/orig_model.o $B/memb_model.o $B/tla_value.o \
   $B/tla_parse.o $B/tla_gen.o $B/tlagen_backend.o $B/tlagen_sort.o \
   -ldl -L/opt/rocm/lib -lhiprtc -Wl,-rpath,/opt/rocm/lib
rm -f "$OUT/memb_backend.o"
echo "$OUT/libraftmc.so"
