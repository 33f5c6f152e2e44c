#!/bin/bash
# Per-layer HBM traffic of the PWG bench batch (round 4: the tap-0 prefetch A/B builds are gone,
# their winner -- the load just before GEMM 2 -- is the only path).
set -e
OUT=${1:-gpurun_out/r04_diag}
mkdir -p "$OUT"
export TMPDIR=/tmp PWG_NO_BUILD=1
bash tools/diag/layer_fetch.sh "$OUT/lf" base > "$OUT/layer_fetch.txt" 2>&1
cat "$OUT/layer_fetch.txt"
