#!/bin/bash
# Round 4 pass G (GPU box). tests: the whole GPU suite + smoke. bench: the default bench line, a
# rocprofv3 kernel-trace summary of the PWG bench leg, the B = 1 vocoder latency A/B.
set -e
OUT=${1:-gpurun_out/r04_g}
mkdir -p "$OUT"
export TMPDIR=/tmp PWG_NO_BUILD=1
ROOT=$(pwd)
if [ "$2" == "tests" ]; then
  timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 || { tail -60 "$OUT/pytest_gpu.log"; exit 1; }
  tail -2 "$OUT/pytest_gpu.log"
  timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
  tail -1 "$OUT/smoke.log"
  exit 0
fi
timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 > "$OUT/bench.json" 2> "$OUT/bench.err"
python - "$OUT/bench.json" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("PWG", d["value"], "frac", d["roofline"]["frac"], "traffic", d["roofline"]["traffic"], d["roofline"].get("avg_launch_ms"))
print("exact", json.dumps(d.get("exact_fp32"))[:400])
print("cpu", json.dumps(d.get("cpu_baseline"))[:400])
for k, v in (d.get("vocoders") or {}).items():
    print(k, v["value"], v["roofline"]["frac"], v["roofline"]["traffic"], [(r["frames"], r["batch"], r["median_ms"]) for r in v["latency"]["rows"]])
print("lat", [(r["frames"], r["batch"], r["median_ms"]) for r in d["latency"]["rows"]])
PY
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/$OUT/prof" -o bench -- \
  python3 "$ROOT/bench.py" --steps 10 --warmup 3 --no-vocoders --no-exact --no-latency --cpu-seconds 0 --pmc off) > "$OUT/prof.log" 2>&1
find "$OUT/prof" -name "*kernel_stats.csv" | head -2
timeout -k 10 300 python -u tools/diag/voc_lat_ab.py "$OUT/voc_lat_ab.json" > "$OUT/voc_lat_ab.log" 2>&1
grep -E "^(hifigan|mb_melgan)" "$OUT/voc_lat_ab.log"
for st in 0 2; do
  timeout -k 10 300 python bench.py --config hifigan_v1 --steps 10 --warmup 3 --cpu-seconds 0 --no-latency --pmc off --cnet-streams $st > "$OUT/hifi_streams$st.json" 2>/dev/null
  python -c "import json; d=json.loads(open('$OUT/hifi_streams$st.json').read().strip().splitlines()[-1]); print('hifigan streams $st', d['value'], d['ms_per_step'])"
done
