#!/bin/bash
# One GPU verification pass (GPU box): parity suite, smoke, default bench, rocprofv3 kernel stats.
# Usage: bash tools/gpu_check.sh OUTDIR
set -e
OUT=${1:-gpurun_out/check}
mkdir -p "$OUT"
export TMPDIR=/tmp PWG_NO_BUILD=1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1
tail -3 "$OUT/pytest_gpu.log"
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
cat "$OUT/smoke.log" | tail -1
timeout -k 10 300 python bench.py > "$OUT/bench.json" 2> "$OUT/bench.err"
cat "$OUT/bench.json"
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$OUT/prof" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 3 --warmup 1 --cpu-seconds 0 --no-latency > "$GRAFT_REPO_ROOT/$OUT/bench_prof.json" 2> "$GRAFT_REPO_ROOT/$OUT/prof.err"

cd "$GRAFT_REPO_ROOT"
# PMC passes (separate rocprofv3 runs) -> HBM traffic per split-layer launch
bash tools/profile_pmc.sh "$OUT/pmc" && python tools/pmc_summary.py "$OUT/pmc" "$OUT/pmc_summary.json" > /dev/null && python tools/make_traffic_json.py "$OUT/pmc_summary.json" "$OUT/layer_traffic.json" split16
echo done
timeout -k 10 300 python bench.py --config ljspeech_v1 --cpu-seconds 8 > "$OUT/ljspeech_v1.json" 2> "$OUT/ljspeech_v1.err"
# vocoder configs (BASELINE configs 3-4 and MelGAN v1) and the HiFiGAN per-op profile
for c in mb_melgan_v2 hifigan_v1 melgan_v1; do
  timeout -k 10 300 python bench.py --config $c --cpu-seconds 8 > "$OUT/$c.json" 2> "$OUT/$c.err"
done
timeout -k 10 200 python tools/cnet_profile.py hifigan_v1 > "$OUT/ops_hifigan_split.txt" 2>&1
echo vocoders done
