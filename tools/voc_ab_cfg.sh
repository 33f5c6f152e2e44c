#!/bin/bash
# A/B library variants on one vocoder's per-op profile (GPU box).
# Usage: bash tools/voc_ab_cfg.sh OUT CONFIG name...   (name = libpwg_<name>.so; "base" = default lib)
set -e
OUT=$1; CFG=$2; shift 2
mkdir -p "$OUT"
export TMPDIR=/tmp PWG_NO_BUILD=1
for v in "$@"; do
  if [ "$v" = base ]; then lib=parallelwavegan_amd/lib/libpwg_hip.so; else lib=parallelwavegan_amd/lib/variants/libpwg_$v.so; fi
  PWG_LIB_PATH=$lib timeout -k 10 200 python tools/cnet_profile.py $CFG > "$OUT/ops_${CFG}_$v.txt" 2>&1
  echo "$v $(grep total $OUT/ops_${CFG}_$v.txt)"
done
