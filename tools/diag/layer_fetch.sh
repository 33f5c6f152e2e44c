#!/bin/bash
# Per-layer HBM traffic of the PWG bench batch (LibriTTS v1, 32 ragged utterances): FETCH_SIZE (x2,
# gfx950 correction) and WRITE_SIZE per residual-layer dispatch of the second of two forwards, by
# dilation, for each library given (A/B builds under parallelwavegan_amd/lib/variants).
# Usage (GPU box): bash tools/diag/layer_fetch.sh OUT name[=lib path relative to the repo] ...
set -e
OUT=$1; shift
mkdir -p "$OUT"
export TMPDIR=/tmp PWG_NO_BUILD=1
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
for spec in "$@"; do
  v=${spec%%=*}; lib=${spec#*=}; [ "$lib" == "$spec" ] && lib=parallelwavegan_amd/lib/libpwg_hip.so
  for ctr in FETCH_SIZE WRITE_SIZE; do
    (cd /tmp && PWG_LIB_PATH=$ROOT/$lib timeout -s KILL 120 rocprofv3 --pmc $ctr --kernel-trace --output-format csv \
      -d "$ROOT/$OUT/$v/$ctr" -o pmc -- python3 "$ROOT/bench.py" --pmc-child --config libritts_v1 --utts 32) \
      > "$OUT/$v.$ctr.log" 2>&1
  done
done
python3 tools/diag/layer_fetch.py "$OUT" "$@"
