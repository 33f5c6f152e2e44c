#!/bin/bash
# FETCH_SIZE / WRITE_SIZE / TCC hit-miss passes of the bench for several library variants (GPU box).
# Usage: bash tools/pmc_variants.sh OUT name1 name2 ...   (name = libpwg_<name>.so under lib/variants; base = default)
set -e
OUT=$1; shift
export TMPDIR=/tmp PWG_NO_BUILD=1
mkdir -p "$OUT"
for v in "$@"; do
  if [ "$v" = base ]; then lib=parallelwavegan_amd/lib/libpwg_hip.so; else lib=parallelwavegan_amd/lib/variants/libpwg_$v.so; fi
  i=0
  mkdir -p "$OUT/$v"
  for group in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum"; do
    i=$((i+1))
    PWG_LIB_PATH=$lib timeout -k 10 120 rocprofv3 --pmc $group --output-format csv -d "$OUT/$v/p$i" -o pmc -- python bench.py --utts 32 --steps 1 --warmup 1 --cpu-seconds 0 --no-latency > "$OUT/$v/p$i.log" 2>&1
  done
  python tools/pmc_summary.py "$OUT/$v" "$OUT/$v/summary.json" > /dev/null
  python - "$OUT/$v/summary.json" "$v" <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
for k, v in d.items():
    if "split16_kernel<false, 1, false>" in k:
        print(sys.argv[2], "fetch GB", round(v["FETCH_BYTES_corrected"] / 1e9, 3), "write GB", round(v["WRITE_BYTES"] / 1e9, 3),
              "l2 hit", round(v["TCC_HIT_sum"] / (v["TCC_HIT_sum"] + v["TCC_MISS_sum"]), 3))
PY
done
