#!/bin/bash
# Average shader clock of the middle layer kernel per library variant (GPU box): one
# GRBM_GUI_ACTIVE + SQ_BUSY_CYCLES pass with kernel timestamps; clock = GRBM_GUI_ACTIVE / duration.
# Usage: bash tools/clock_variants.sh OUT name1 name2 ...
set -e
OUT=$1; shift
export TMPDIR=/tmp PWG_NO_BUILD=1
mkdir -p "$OUT"
for v in "$@"; do
  if [ "$v" = base ]; then lib=parallelwavegan_amd/lib/libpwg_hip.so; else lib=parallelwavegan_amd/lib/variants/libpwg_$v.so; fi
  mkdir -p "$OUT/$v"
  PWG_LIB_PATH=$lib timeout -k 10 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES --output-format csv -d "$OUT/$v/p1" -o pmc -- python bench.py --utts 32 --steps 1 --warmup 1 --cpu-seconds 0 --no-latency > "$OUT/$v/p1.log" 2>&1
  python - "$OUT/$v" "$v" <<'PY'
import csv, glob, sys
from collections import defaultdict
f = glob.glob(sys.argv[1] + "/p1/**/*counter_collection.csv", recursive=True)[0]
d = defaultdict(lambda: {"dur": 0, "ctr": defaultdict(float)})
for r in csv.DictReader(open(f)):
    if "split16_kernel<false, 1, false>" not in r["Kernel_Name"]:
        continue
    e = d[r["Dispatch_Id"]]
    e["dur"] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    e["ctr"][r["Counter_Name"]] += float(r["Counter_Value"])
ghz = [e["ctr"]["GRBM_GUI_ACTIVE"] / e["dur"] for e in d.values() if e["dur"] > 0]
print(sys.argv[2], "dispatches", len(ghz), "GRBM_GUI_ACTIVE/ns mean", round(sum(ghz) / len(ghz), 3),
      "min", round(min(ghz), 3), "max", round(max(ghz), 3),
      "dur_ms", round(sum(e["dur"] for e in d.values()) / len(d) / 1e6, 4))
PY
done
