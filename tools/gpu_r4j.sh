#!/bin/bash
# Round 4 pass J (GPU box): DMA-ring timelines (probe build) at B = 1 after the ring cap / K = 1 changes.
set -e
OUT=${1:-gpurun_out/r04_j}
mkdir -p "$OUT"
export PWG_NO_BUILD=1 TMPDIR=/tmp
for spec in mb_melgan_v2:64 hifigan_v1:64; do
  IFS=: read cfg T <<< "$spec"
  PWG_LIB_PATH=parallelwavegan_amd/lib/variants/libpwg_probe.so timeout -k 10 120 python -u tools/diag/xdma_probe.py "$cfg" "$T" \
    > "$OUT/probe_${cfg}_T$T.txt" 2>&1
done
grep phase "$OUT/probe_mb_melgan_v2_T64.txt"
