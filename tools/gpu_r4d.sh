#!/bin/bash
# Round 4 pass D (GPU box): kernel traces of the B = 1 vocoder forwards (DMA-ring kernel on / off),
# the batched HiFiGAN program's per-kernel stats, then the default bench line.
set -e
OUT=${1:-gpurun_out/r04_d}
mkdir -p "$OUT"
export PWG_NO_BUILD=1 TMPDIR=/tmp
ROOT=$(pwd)
timeout -k 10 400 python -u -m pytest tests/test_gpu_vocoders.py -x -v --timeout 120 --timeout-method thread \
  > "$OUT/pytest_voc.log" 2>&1 || { tail -30 "$OUT/pytest_voc.log"; exit 1; }
tail -1 "$OUT/pytest_voc.log"
timeout -k 10 300 python -u tools/diag/voc_lat_ab.py "$OUT/voc_lat_ab.json" > "$OUT/voc_lat_ab.log" 2>&1
grep -E "^(hifigan|mb_melgan)" "$OUT/voc_lat_ab.log"
for spec in hifigan_v1:64:1 hifigan_v1:64:0 mb_melgan_v2:64:1 mb_melgan_v2:64:0 hifigan_v1:512:1; do
  IFS=: read cfg T dma <<< "$spec"
  d="$ROOT/$OUT/trace_${cfg}_T${T}_dma${dma}"
  (cd /tmp && timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d "$d" -o kt -- \
    python3 "$ROOT/tools/diag/voc_trace.py" run "$cfg" "$T" "$dma") > "$OUT/trace_${cfg}_T${T}_dma${dma}.log" 2>&1
  python3 tools/diag/voc_trace.py summarize "$d" > "$OUT/trace_${cfg}_T${T}_dma${dma}.txt"
  tail -1 "$OUT/trace_${cfg}_T${T}_dma${dma}.txt"
done
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/$OUT/hifi_batch" -o kt -- \
  python3 "$ROOT/tools/cnet_profile.py" hifigan_v1 --utts 32 --steps 3) > "$OUT/hifi_batch.log" 2>&1
grep -E "total|input_conv" "$OUT/hifi_batch.log" || true
timeout -k 10 600 python -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.err"
tail -c 600 "$OUT/bench.json"
