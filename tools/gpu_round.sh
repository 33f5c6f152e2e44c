#!/bin/bash
# Round verification pass (GPU box): full GPU suite, smoke, default bench (latency rows + CPU
# baseline), strong-scaling bench of the 512-utterance list, rocprofv3 kernel stats.
# Usage: bash tools/gpu_round.sh OUTDIR [skip-tests]
set -e
OUT=${1:-gpurun_out/round}
mkdir -p "$OUT"
export TMPDIR=/tmp PWG_NO_BUILD=1
if [ "$2" != "skip-tests" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 || { tail -60 "$OUT/pytest_gpu.log"; exit 1; }
  tail -3 "$OUT/pytest_gpu.log"
fi
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
tail -1 "$OUT/smoke.log"
timeout -k 10 400 python bench.py > "$OUT/bench.json" 2> "$OUT/bench.err"
cat "$OUT/bench.json"
timeout -k 10 300 python bench.py --strong --steps 2 --warmup 1 --cpu-seconds 0 --no-latency > "$OUT/strong.json" 2> "$OUT/strong.err"
cat "$OUT/strong.json"
for c in hifigan_v1 mb_melgan_v2 melgan_v1; do
  timeout -k 10 300 python bench.py --config $c > "$OUT/$c.json" 2> "$OUT/$c.err"
  python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['roofline']['frac'])" "$OUT/$c.json" $c
done
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$OUT/prof" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 3 --warmup 1 --cpu-seconds 0 --no-latency > "$GRAFT_REPO_ROOT/$OUT/bench_prof.json" 2> "$GRAFT_REPO_ROOT/$OUT/prof.err"
cd "$GRAFT_REPO_ROOT"
python - <<'PY' "$OUT"
import os, sys
out = sys.argv[1]
print("cpus: os.cpu_count", os.cpu_count(), "affinity", len(os.sched_getaffinity(0)))
try:
    print("cgroup cpu.max", open("/sys/fs/cgroup/cpu.max").read().strip())
except OSError as e:
    print("no cgroup cpu.max", e)
PY
echo round-check done
