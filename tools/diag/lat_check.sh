#!/bin/bash
# Latency-path check (GPU box): parity subset, drop-in latency rows, kernel trace of T' = 64 calls.
# Usage: bash tools/diag/lat_check.sh OUT
set -e
OUT=$1
mkdir -p "$OUT"
export PWG_NO_BUILD=1 TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_streaming.py tests/test_gpu_sync.py tests/test_gpu_half_blocks.py tests/test_gpu_pipeline.py tests/test_decode_cli.py -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
timeout -k 10 300 python tools/latency.py > "$OUT/lat.json"
python - "$OUT/lat.json" <<'PY'
import json, sys
for r in json.load(open(sys.argv[1]))["rows"]:
    print(r["frames"], r["batch"], "median_ms", r["median_ms"], "graph", r["graph_replay_median_ms"], "samples/s", r["samples_per_s"])
PY
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$GRAFT_REPO_ROOT/$OUT/trace" -o run -- python3 "$GRAFT_REPO_ROOT/tools/diag/lat_trace.py" 64 > /dev/null 2>&1
cd "$GRAFT_REPO_ROOT" && python tools/diag/lat_gaps.py $(find "$OUT/trace" -name "*kernel_trace.csv" | head -1) | tail -3
