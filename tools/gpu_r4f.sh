#!/bin/bash
# Round 4 pass F (GPU box): vocoder parity (incl. narrow bitwise), B = 1 latency A/B, DMA-ring timelines.
set -e
OUT=${1:-gpurun_out/r04_f}
mkdir -p "$OUT"
export PWG_NO_BUILD=1 TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_vocoders.py -x -v --timeout 120 --timeout-method thread \
  > "$OUT/pytest_voc.log" 2>&1 || { tail -30 "$OUT/pytest_voc.log"; exit 1; }
tail -1 "$OUT/pytest_voc.log"
timeout -k 10 300 python -u tools/diag/voc_lat_ab.py "$OUT/voc_lat_ab.json" > "$OUT/voc_lat_ab.log" 2>&1
grep -E "^(hifigan|mb_melgan|melgan)" "$OUT/voc_lat_ab.log"
for spec in hifigan_v1:64 mb_melgan_v2:64; do
  IFS=: read cfg T <<< "$spec"
  PWG_LIB_PATH=parallelwavegan_amd/lib/variants/libpwg_probe.so timeout -k 10 120 python -u tools/diag/xdma_probe.py "$cfg" "$T" \
    > "$OUT/probe_${cfg}_T$T.txt" 2>&1
done
grep phase "$OUT/probe_hifigan_v1_T64.txt" | head -30
