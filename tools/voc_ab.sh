#!/bin/bash
# A/B library variants on the HiFiGAN v1 per-op profile (GPU box). Usage: bash tools/voc_ab.sh OUT name...
set -e
OUT=$1; shift
mkdir -p "$OUT"
export TMPDIR=/tmp PWG_NO_BUILD=1
for v in "$@"; do
  if [ "$v" = base ]; then lib=parallelwavegan_amd/lib/libpwg_hip.so; else lib=parallelwavegan_amd/lib/variants/libpwg_$v.so; fi
  PWG_LIB_PATH=$lib timeout -k 10 200 python tools/cnet_profile.py hifigan_v1 > "$OUT/ops_$v.txt" 2>&1
  echo "$v $(grep total $OUT/ops_$v.txt)"
done
