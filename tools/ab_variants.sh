#!/bin/bash
# A/B the prebuilt library variants under parallelwavegan_amd/lib/variants on the bench workload.
# Usage (GPU box): bash tools/ab_variants.sh OUT name1 name2 ...   (name = libpwg_<name>.so; "base" = default lib)
set -e
OUT=$1; shift
mkdir -p "$OUT"
for v in "$@"; do
  if [ "$v" = base ]; then lib=parallelwavegan_amd/lib/libpwg_hip.so; else lib=parallelwavegan_amd/lib/variants/libpwg_$v.so; fi
  PWG_NO_BUILD=1 PWG_LIB_PATH=$lib timeout -k 10 300 python bench.py --cpu-seconds 0 --steps 5 --warmup 2 > "$OUT/$v.json" 2> "$OUT/$v.err"
  python -c "import json,sys; d=json.load(open('$OUT/$v.json')); print('$v', d['value'], d['roofline']['avg_launch_ms'], d['kernel_ms_per_step'])"
done
