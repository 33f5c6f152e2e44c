#!/bin/bash
# Latency A/B (GPU box): parity suite on the default library, then the drop-in latency rows and the
# default bench for each library variant. Usage: bash tools/gpu_latency_ab.sh OUT [variant ...]
set -e
OUT=$1; shift
mkdir -p "$OUT"
export PWG_NO_BUILD=1 TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_streaming.py -m gpu -x -q --timeout 200 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
for v in base "$@"; do
  if [ "$v" = base ]; then lib=parallelwavegan_amd/lib/libpwg_hip.so; else lib=parallelwavegan_amd/lib/variants/libpwg_$v.so; fi
  PWG_LIB_PATH=$lib timeout -k 10 200 python tools/latency.py > "$OUT/lat_$v.json"
  python - "$OUT/lat_$v.json" "$v" <<'PY'
import json, sys
for r in json.load(open(sys.argv[1]))["rows"]:
    print(sys.argv[2], r["frames"], r["batch"], "median_ms", r["median_ms"], "kernel_ms", r["kernel_ms"], "samples/s", r["samples_per_s"])
PY
  PWG_LIB_PATH=$lib timeout -k 10 300 python bench.py --cpu-seconds 0 --no-latency --steps 5 --warmup 2 > "$OUT/bench_$v.json"
  python -c "import json; d=json.load(open('$OUT/bench_$v.json')); print('$v bench', d['value'], d['roofline']['avg_launch_ms'], d['kernel_ms_per_step'])"
done
