#!/bin/bash
# Per-op times of the vocoders at the B = 1 latency shapes (LJ, T' = 64 / 512), GPU box.
# Usage: bash tools/diag/voc_lat_ops.sh OUT [lib]
set -e
OUT=$1; LIB=${2:-parallelwavegan_amd/lib/libpwg_hip.so}
mkdir -p "$OUT"
export PWG_NO_BUILD=1 PWG_LIB_PATH=$LIB
for c in hifigan_v1 mb_melgan_v2; do
  for f in 64 512; do
    timeout -k 10 120 python tools/cnet_profile.py $c --frames $f --batch 1 --steps 10 > "$OUT/${c}_T$f.txt" 2>&1
    tail -1 "$OUT/${c}_T$f.txt"
  done
done
