#!/bin/bash
# A/B library variants on the three vocoder benches (GPU box). Usage: bash tools/voc_bench_ab.sh OUT name...
set -e
OUT=$1; shift
mkdir -p "$OUT"
export TMPDIR=/tmp PWG_NO_BUILD=1
for rep in 1 2; do
for v in "$@"; do
  if [ "$v" = base ]; then lib=parallelwavegan_amd/lib/libpwg_hip.so; else lib=parallelwavegan_amd/lib/variants/libpwg_$v.so; fi
  for c in hifigan_v1 mb_melgan_v2 melgan_v1; do
    PWG_LIB_PATH=$lib timeout -k 10 200 python bench.py --config $c --cpu-seconds 0 > "$OUT/$v-$c-$rep.json" 2> "$OUT/$v-$c-$rep.err"
    python -c "import json; d=json.load(open('$OUT/$v-$c-$rep.json')); print('$v $c $rep', round(d['value']/1e6,1))"
  done
done
done
