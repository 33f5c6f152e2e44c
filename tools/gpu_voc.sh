#!/bin/bash
# Vocoder iteration (GPU box): conv-network parity suite, HiFiGAN bench fused / unfused, per-op profile.
# Usage: bash tools/gpu_voc.sh OUTDIR [extra bench args]
set -e
OUT=${1:-gpurun_out/voc}; shift || true
mkdir -p "$OUT"
export TMPDIR=/tmp PWG_NO_BUILD=1
timeout -k 10 400 python -u -m pytest tests/test_gpu_vocoders.py -x -v --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { tail -40 "$OUT/pytest.log"; exit 1; }
tail -3 "$OUT/pytest.log"
timeout -k 10 300 python bench.py --config hifigan_v1 --cpu-seconds 0 "$@" > "$OUT/hifigan_v1.json" 2> "$OUT/hifigan_v1.err" || { tail -20 "$OUT/hifigan_v1.err"; exit 1; }
timeout -k 10 300 python bench.py --config hifigan_v1 --cpu-seconds 0 --cnet-nofuse > "$OUT/hifigan_v1_nofuse.json" 2> "$OUT/hifigan_v1_nofuse.err" || { tail -20 "$OUT/hifigan_v1_nofuse.err"; exit 1; }
python -c "import json; [print(f, json.load(open('$OUT/'+f+'.json'))['value']/1e6) for f in ['hifigan_v1','hifigan_v1_nofuse']]"
timeout -k 10 200 python tools/cnet_profile.py hifigan_v1 > "$OUT/ops_hifigan.txt" 2>&1
for s in 4 16; do
  timeout -k 10 200 python tools/cnet_profile.py hifigan_v1 --pair-steps $s > "$OUT/ops_hifigan_ps$s.txt" 2>&1
done
grep total "$OUT"/ops_*.txt
