#!/bin/bash
# Round-4 pass B (GPU box): the GPU test files changed since pass A, smoke, the default bench line,
# per-op vocoder times at the latency shapes, then the PWG layer diagnostics.
set -e
OUT=${1:-gpurun_out/r04_b}
mkdir -p "$OUT"
export TMPDIR=/tmp PWG_NO_BUILD=1
if [ "$2" != "skip-tests" ]; then
  timeout -k 10 600 python -u -m pytest tests/test_gpu_vocoders.py tests/test_gpu_vocoder_range.py tests/test_gpu_sharding.py -m gpu -x -v --timeout 200 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 || { tail -60 "$OUT/pytest_gpu.log"; exit 1; }
  tail -2 "$OUT/pytest_gpu.log"
fi
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
tail -1 "$OUT/smoke.log"
timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 > "$OUT/bench.json" 2> "$OUT/bench.err"
echo bench done
python - "$OUT/bench.json" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("PWG", d["value"], "frac", d["roofline"]["frac"], "traffic", d["roofline"]["traffic"])
print("exact", json.dumps(d.get("exact_fp32")))
print("cpu", json.dumps(d.get("cpu_baseline")))
for k, v in (d.get("vocoders") or {}).items():
    print(k, v["value"], v["roofline"]["frac"], v["roofline"]["traffic"], [(r["frames"], r["batch"], r["median_ms"]) for r in v["latency"]["rows"]])
print("lat", [(r["frames"], r["batch"], r["median_ms"]) for r in d["latency"]["rows"]])
PY
mkdir -p "$OUT/voc" && timeout -k 10 300 python tools/diag/voc_lat_ab.py "$OUT/voc/lat_ab.json"
bash tools/gpu_r4_diag_pwg.sh "$OUT/diag"
echo pass-b done
