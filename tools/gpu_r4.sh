#!/bin/bash
# Round-4 verification pass (GPU box): full GPU suite, smoke, the default bench line (PWG + exact
# fp32 + embedded vocoders + CPU baseline + latency rows), rocprofv3 kernel stats of the PWG bench.
# Usage: bash tools/gpu_r4.sh OUTDIR [skip-tests|tests-only]
set -e
OUT=${1:-gpurun_out/r4}
mkdir -p "$OUT"
export TMPDIR=/tmp PWG_NO_BUILD=1
if [ "$2" != "skip-tests" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 || { tail -60 "$OUT/pytest_gpu.log"; exit 1; }
  tail -3 "$OUT/pytest_gpu.log"
fi
[ "$2" == "tests-only" ] && exit 0
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
tail -1 "$OUT/smoke.log"
timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 > "$OUT/bench.json" 2> "$OUT/bench.err"
tail -c 3000 "$OUT/bench.json"
echo bench done
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$OUT/prof" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 3 --warmup 1 --cpu-seconds 0 --no-latency --no-vocoders --no-exact --pmc off > "$GRAFT_REPO_ROOT/$OUT/bench_prof.json" 2> "$GRAFT_REPO_ROOT/$OUT/prof.err"
echo round-check done
