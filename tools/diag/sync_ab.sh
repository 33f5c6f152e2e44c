#!/bin/bash
# Grid-synchronised forward A/B (GPU box): sync parity tests, then the latency plans per-layer vs
# synchronised (same library, PWG_OPT_SYNC). Usage: bash tools/diag/sync_ab.sh OUT
set -e
OUT=$1
mkdir -p "$OUT"
export PWG_NO_BUILD=1 TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_sync.py tests/test_gpu_half_blocks.py tests/test_gpu_parity.py tests/test_streaming.py tests/test_gpu_sharding.py -m gpu -rP -x -v --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
for rep in 1 2; do
  PLANS=${PLANS:-lat} timeout -k 10 200 python tools/diag/opt_bench.py '{"sync": 0}' '{"sync": 1073741824}' '{}' > "$OUT/lat_$rep.jsonl"
  python - "$OUT/lat_$rep.jsonl" <<'PY'
import json, sys
for l in open(sys.argv[1]):
    r = json.loads(l)
    print(r["frames"], "per-layer", r["m0"]["median_ms"], "sync", r["m1"]["median_ms"], "default", r["m2"]["median_ms"])
PY
done
