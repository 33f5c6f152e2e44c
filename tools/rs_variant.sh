#!/bin/bash
# Variant library with pwg_rstack.hip rebuilt under extra flags, every other object from the main
# build (build/libpwg_hip): bash tools/rs_variant.sh NAME -DRS_ORDER=1 ...
# -> parallelwavegan_amd/lib/rsv/libpwg_NAME.so (A/B runs: PWG_LIB_PATH=...; delete the directory
# before the round ends)
set -e
NAME=$1; shift
R=$(cd "$(dirname "$0")/.." && pwd)
OUT=$R/parallelwavegan_amd/lib/rsv
mkdir -p "$OUT" "$R/build/rsv"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -mllvm -amdgpu-atomic-optimizer-strategy=None -Wall "$@" \
  -c "$R/parallelwavegan_amd/csrc/pwg_rstack.hip" -o "$R/build/rsv/rstack_$NAME.o"
objs=$(ls "$R"/build/libpwg_hip/*.o | grep -v pwg_rstack)
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$OUT/libpwg_$NAME.so" $objs "$R/build/rsv/rstack_$NAME.o" -ldl
echo "$OUT/libpwg_$NAME.so"
