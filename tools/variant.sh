#!/bin/bash
# Variant library with one source rebuilt under extra flags, every other object from the main build
# (build/libpwg_hip): bash tools/variant.sh SOURCE NAME -DFLAG=V ...
# -> parallelwavegan_amd/lib/abv/libpwg_NAME.so (A/B runs: PWG_LIB_PATH=...; delete the directory
# after the A/B)
set -e
SRC=$1; NAME=$2; shift 2
R=$(cd "$(dirname "$0")/.." && pwd)
OUT=$R/parallelwavegan_amd/lib/abv
mkdir -p "$OUT" "$R/build/abv"
base=$(basename "$SRC" .hip)
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -fvisibility=hidden -mcode-object-version=5 -mllvm -amdgpu-atomic-optimizer-strategy=None -Wall "$@" \
  -c "$R/parallelwavegan_amd/csrc/$base.hip" -o "$R/build/abv/${base}_$NAME.o"
objs=$(ls "$R"/build/libpwg_hip/*.o | grep -v "/$base.hip.o")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$OUT/libpwg_$NAME.so" $objs "$R/build/abv/${base}_$NAME.o" -ldl
echo "$OUT/libpwg_$NAME.so"
