#!/bin/bash
# Per-launch HBM traffic of one vocoder forward (GPU box): FETCH_SIZE and WRITE_SIZE passes (one
# counter block per run) plus a kernel-trace pass over `bench.py --pmc-child` (two forwards of the
# bench plan); tools/traffic_summary.py joins them per dispatch of the second forward.
# Usage: bash tools/voc_traffic.sh OUT [CONFIG]
set -e
OUT=$1; CFG=${2:-hifigan_v1}
export TMPDIR=/tmp PWG_NO_BUILD=1
mkdir -p "$OUT"
R=$GRAFT_REPO_ROOT
cd /tmp
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$R/$OUT/fetch" -o pmc -- python3 "$R/bench.py" --pmc-child --config $CFG > "$R/$OUT/fetch.log" 2>&1
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$R/$OUT/write" -o pmc -- python3 "$R/bench.py" --pmc-child --config $CFG > "$R/$OUT/write.log" 2>&1
timeout -k 10 150 rocprofv3 --kernel-trace --output-format csv -d "$R/$OUT/trace" -o kt -- python3 "$R/bench.py" --pmc-child --config $CFG > "$R/$OUT/trace.log" 2>&1
cd "$R"
python tools/traffic_summary.py "$OUT" > "$OUT/summary.txt"
head -60 "$OUT/summary.txt"
