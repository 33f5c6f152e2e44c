#!/bin/bash
# Round 4 pass M (GPU box): kernel trace of the concurrent B = 1 HiFiGAN forward.
set -e
OUT=${1:-gpurun_out/r04_m}
mkdir -p "$OUT"
export PWG_NO_BUILD=1 TMPDIR=/tmp
ROOT=$(pwd)
for spec in hifigan_v1:64:1 mb_melgan_v2:64:1; do
  IFS=: read cfg T dma <<< "$spec"
  d="$ROOT/$OUT/trace_${cfg}_T${T}"
  (cd /tmp && timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d "$d" -o kt -- \
    python3 "$ROOT/tools/diag/voc_trace.py" run "$cfg" "$T" "$dma") > "$OUT/trace_${cfg}_T${T}.log" 2>&1
done
python3 tools/diag/voc_trace.py concurrent "$ROOT/$OUT/trace_hifigan_v1_T64" 81 > "$OUT/hifigan_T64_concurrent.txt"
python3 tools/diag/voc_trace.py concurrent "$ROOT/$OUT/trace_mb_melgan_v2_T64" 32 > "$OUT/mb_melgan_T64.txt"
tail -1 "$OUT/hifigan_T64_concurrent.txt"; tail -1 "$OUT/mb_melgan_T64.txt"
