#!/bin/bash
# Quick GPU iteration (GPU box): split-kernel parity subset + bench (no CPU baseline).
# Usage: bash tools/gpu_quick.sh OUTDIR [pytest -k expr]
set -e
OUT=${1:-gpurun_out/quick}; K=${2:-split}
mkdir -p "$OUT"
export TMPDIR=/tmp PWG_NO_BUILD=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread -k "$K" > "$OUT/pytest.log" 2>&1 || { tail -40 "$OUT/pytest.log"; exit 1; }
tail -3 "$OUT/pytest.log"
timeout -k 10 300 python bench.py --cpu-seconds 0 > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail -20 "$OUT/bench.err"; exit 1; }
cat "$OUT/bench.json"
