#!/bin/bash
# Experiment builds (C2 shape only): raft-tla_amd/_build_var/NAME/libraftmc.so with extra -D flags.
#   scripts/build_variant.sh NAME "-DRMC_DEDUP_PER=8 -DRMC_LDS_SLOTS=2048"
# Select one at run time with RAFTMC_LIB=raft-tla_amd/_build_var/NAME/libraftmc.so.
# The rejected experiment switches live in scripts/variants/orig_backend_experiments.hip (third argument):
#   scripts/build_variant.sh binned "-DRMC_GEN_BINNED" scripts/variants/orig_backend_experiments.hip
set -e
NAME=$1; DEFS=$2
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT=$ROOT/raft-tla_amd/_build_var/$NAME
mkdir -p "$OUT"
H=/opt/rocm/bin/hipcc
F="-O3 -std=c++17 -fPIC -Wall -Wno-unused-function"
C=$ROOT/raft-tla_amd/csrc
SRC=${3:-$C/orig_backend.hip}
$H $F --offload-arch=gfx950 -munsafe-fp-atomics -DRMC_QUICK_BUILD $DEFS -I$C -c -o "$OUT/orig_backend.o" "$SRC"
$H -shared --offload-arch=gfx950 -o "$OUT/libraftmc.so" "$OUT/orig_backend.o" $ROOT/raft-tla_amd/_build/memb_backend.o \
   $ROOT/raft-tla_amd/_build/mc_api.o $ROOT/raft-tla_amd/_build/model.o $ROOT/raft-tla_amd/_build/orig_model.o \
   $ROOT/raft-tla_amd/_build/memb_model.o $ROOT/raft-tla_amd/_build/tla_value.o \
   $ROOT/raft-tla_amd/_build/tla_parse.o $ROOT/raft-tla_amd/_build/tla_gen.o $ROOT/raft-tla_amd/_build/tlagen_backend.o $ROOT/raft-tla_amd/_build/tlagen_sort.o \
   -ldl -L/opt/rocm/lib -lhiprtc -Wl,-rpath,/opt/rocm/lib
rm -f "$OUT/orig_backend.o"
echo "$OUT/libraftmc.so"
