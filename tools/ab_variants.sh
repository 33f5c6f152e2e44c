#!/bin/bash
# A/B the prebuilt library variants under parallelwavegan_amd/lib/variants on the bench workload.
# Usage (GPU box): bash tools/ab_variants.sh OUT spec1 spec2 ...
#   spec = name[:bench args with , for spaces]   (name = libpwg_<name>.so; "base" = default lib)
#   e.g.  base  w12:--waves-per-wg,12
set -e
OUT=$1; shift
mkdir -p "$OUT"
i=0
for spec in "$@"; do
  i=$((i+1))
  v=${spec%%:*}
  extra=""
  if [ "$spec" != "$v" ]; then extra=$(echo "${spec#*:}" | tr ',' ' '); fi
  if [ "$v" = base ]; then lib=parallelwavegan_amd/lib/libpwg_hip.so; else lib=parallelwavegan_amd/lib/variants/libpwg_$v.so; fi
  PWG_NO_BUILD=1 PWG_LIB_PATH=$lib timeout -k 10 300 python bench.py --cpu-seconds 0 --steps 5 --warmup 2 --no-latency --no-vocoders --no-exact --pmc off $extra > "$OUT/$i-$v.json" 2> "$OUT/$i-$v.err"
  python -c "import json,sys; d=json.load(open('$OUT/$i-$v.json')); print('$spec', d['value'], d['roofline']['avg_launch_ms'], d['kernel_ms_per_step'])"
done
