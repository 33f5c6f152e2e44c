#!/bin/bash
# Round 4 pass H (GPU box): B = 1 vocoder latency A/B over library variants (lib/variants/libpwg_<v>.so).
set -e
OUT=${1:-gpurun_out/r04_h}; shift
mkdir -p "$OUT"
export PWG_NO_BUILD=1 TMPDIR=/tmp
if [ -n "$PARITY_LIB" ]; then
  PWG_LIB_PATH=parallelwavegan_amd/lib/variants/libpwg_$PARITY_LIB.so timeout -k 10 400 python -u -m pytest tests/test_gpu_vocoders.py \
    -x -q --timeout 120 --timeout-method thread > "$OUT/pytest_$PARITY_LIB.log" 2>&1 || { tail -30 "$OUT/pytest_$PARITY_LIB.log"; exit 1; }
  tail -1 "$OUT/pytest_$PARITY_LIB.log"
fi
for v in "$@"; do
  if [ "$v" = base ]; then lib=parallelwavegan_amd/lib/libpwg_hip.so; else lib=parallelwavegan_amd/lib/variants/libpwg_$v.so; fi
  PWG_LIB_PATH=$lib timeout -k 10 300 python -u tools/diag/voc_lat_ab.py "$OUT/lat_$v.json" > "$OUT/lat_$v.log" 2>&1
  grep -E "^(hifigan|mb_melgan|melgan)_?v?[0-9]* [0-9]+ 1 1" "$OUT/lat_$v.log" | sed "s/^/$v /"
done
