#!/bin/bash
# Parity subset + bench for a prebuilt variant library (GPU box). Usage: bash tools/gpu_variant_test.sh NAME OUTDIR
set -e
V=$1; OUT=${2:-gpurun_out/var}
mkdir -p "$OUT"
export TMPDIR=/tmp PWG_NO_BUILD=1 PWG_LIB_PATH=parallelwavegan_amd/lib/variants/libpwg_$V.so
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread -k "split or full or ragged or causal" > "$OUT/pytest.log" 2>&1 || { tail -40 "$OUT/pytest.log"; exit 1; }
tail -2 "$OUT/pytest.log"
