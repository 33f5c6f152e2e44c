#!/bin/bash
# Per-layer HBM traffic and same-box A/B of the split16 tap-0 prefetch phase (PWG_S16_PF builds).
set -e
OUT=${1:-gpurun_out/r04_diag}
mkdir -p "$OUT"
export TMPDIR=/tmp PWG_NO_BUILD=1
V=parallelwavegan_amd/lib/variants
bash tools/diag/layer_fetch.sh "$OUT/lf" base pf1=$V/libpwg_pf1.so pf2=$V/libpwg_pf2.so > "$OUT/layer_fetch.txt" 2>&1
cat "$OUT/layer_fetch.txt"
bash tools/ab_variants.sh "$OUT/ab" base pf1 pf2 base pf1 pf2
