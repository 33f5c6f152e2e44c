#!/bin/bash
# Round 4 pass C (GPU box): narrow-launch bitwise tests, the B = 1 vocoder latency A/B (DMA-ring
# kernel vs the narrow x-tile ones), launch floor / graph replay, then the PWG per-layer PMC +
# same-box A/B of the split16 prefetch phase (PWG_S16_PF variant builds).
set -e
OUT=${1:-gpurun_out/r04_c}
mkdir -p "$OUT"
export PWG_NO_BUILD=1 TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_vocoders.py -x -v --timeout 120 --timeout-method thread \
  -k "narrow or golden or ragged or full_size" > "$OUT/pytest_voc.log" 2>&1 || { tail -30 "$OUT/pytest_voc.log"; exit 1; }
tail -2 "$OUT/pytest_voc.log"
timeout -k 10 300 python -u tools/diag/voc_lat_ab.py "$OUT/voc_lat_ab.json" > "$OUT/voc_lat_ab.log" 2>&1
cat "$OUT/voc_lat_ab.log"
timeout -k 10 300 python -u tools/diag/launch_floor.py "$OUT/launch_floor.json" > "$OUT/launch_floor.log" 2>&1
tail -3 "$OUT/launch_floor.log"
timeout -k 10 300 python -u tools/cnet_profile.py hifigan_v1 --utts 32 --steps 3 > "$OUT/hifigan_batch_ops.txt" 2>&1
tail -1 "$OUT/hifigan_batch_ops.txt"
timeout -k 10 900 bash tools/gpu_r4_diag_pwg.sh "$OUT/diag"
