#!/bin/bash
# FETCH_SIZE / WRITE_SIZE per split-layer launch (middle layers) for prebuilt variants (GPU box).
# Usage: bash tools/fetch_ab.sh OUT spec1 spec2 ...   spec = name[:bench args with , for spaces]
#        ("base" = default library)
set -e
OUT=$1; shift
mkdir -p "$OUT"
export TMPDIR=/tmp PWG_NO_BUILD=1
i=0
for spec in "$@"; do
  i=$((i+1))
  v=${spec%%:*}
  extra=""
  if [ "$spec" != "$v" ]; then extra=$(echo "${spec#*:}" | tr ',' ' '); fi
  if [ "$v" = base ]; then lib=parallelwavegan_amd/lib/libpwg_hip.so; else lib=parallelwavegan_amd/lib/variants/libpwg_$v.so; fi
  d="$OUT/$i-$v"
  mkdir -p "$d"
  for c in FETCH_SIZE WRITE_SIZE; do
    PWG_LIB_PATH=$lib timeout -k 10 120 rocprofv3 --pmc $c --output-format csv -d "$d/$c" -o pmc -- python bench.py --steps 1 --warmup 1 --cpu-seconds 0 $extra > "$d/$c.log" 2>&1
  done
  python - "$d" "$spec" <<'PY'
import csv, glob, sys, collections
root, name = sys.argv[1], sys.argv[2]
tot = collections.defaultdict(lambda: collections.defaultdict(float))
for p in glob.glob(root + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(p)):
        k = r["Kernel_Name"]
        if "_kernel<false" not in k or "layer_split" not in k: continue
        tot[r["Counter_Name"]][r["Dispatch_Id"]] += float(r["Counter_Value"])
f = tot["FETCH_SIZE"]; w = tot["WRITE_SIZE"]
print(name, "fetch GB/launch (x2)", round(sum(f.values()) / max(len(f), 1) * 2048 / 1e9, 3), "write GB/launch", round(sum(w.values()) / max(len(w), 1) * 1024 / 1e9, 3))
PY
done
