#!/bin/bash
# Round 4 pass E (GPU box): DMA-ring kernel timelines (probe build) at B = 1.
set -e
OUT=${1:-gpurun_out/r04_e}
mkdir -p "$OUT"
export PWG_NO_BUILD=1 TMPDIR=/tmp
for spec in hifigan_v1:64 mb_melgan_v2:64 hifigan_v1:512; do
  IFS=: read cfg T <<< "$spec"
  PWG_LIB_PATH=parallelwavegan_amd/lib/variants/libpwg_probe.so timeout -k 10 120 python -u tools/diag/xdma_probe.py "$cfg" "$T" \
    > "$OUT/probe_${cfg}_T$T.txt" 2>&1
  grep phase "$OUT/probe_${cfg}_T$T.txt" | head -40
done
