#!/bin/bash
# Round 4 pass P (GPU box): DMA-ring knob variants (ring cap, K = 1 chunks per step): vocoder
# parity per variant, then B = 1 latency of base and each variant. Usage: OUT v1 v2 ...
set -e
OUT=${1:-gpurun_out/r04_p}; shift
mkdir -p "$OUT"
export PWG_NO_BUILD=1 TMPDIR=/tmp
for v in "$@"; do
  PWG_LIB_PATH=parallelwavegan_amd/lib/variants/libpwg_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_vocoders.py \
    -x -q --timeout 120 --timeout-method thread > "$OUT/pytest_$v.log" 2>&1 || { tail -30 "$OUT/pytest_$v.log"; exit 1; }
  echo "$v $(tail -1 "$OUT/pytest_$v.log")"
done
for v in base "$@" base; do
  if [ "$v" = base ]; then lib=parallelwavegan_amd/lib/libpwg_hip.so; else lib=parallelwavegan_amd/lib/variants/libpwg_$v.so; fi
  PWG_LIB_PATH=$lib timeout -k 10 300 python -u tools/diag/voc_lat_ab.py "$OUT/lat_$v.json" > "$OUT/lat_$v.log" 2>&1
  grep -E "^(hifigan|mb_melgan|melgan)_?v?[0-9]* [0-9]+ 1 1" "$OUT/lat_$v.log" | sed "s/^/$v /"
done
