#!/bin/bash
# PMC passes over a short bench run (one rocprofv3 invocation per counter group; FETCH_SIZE and
# WRITE_SIZE need separate passes on gfx950, MI355X_MICROARCH.md "rocprofv3 PMC slots").
# Usage (on the GPU box): bash tools/profile_pmc.sh OUTDIR [bench args...]
set -e
OUT=${1:-gpurun_out/pmc}; shift || true
ARGS="$@"
[ -z "$ARGS" ] && ARGS="--utts 32 --steps 1 --warmup 1 --cpu-seconds 0 --no-latency"
export TMPDIR=/tmp
mkdir -p "$OUT"
i=0
for group in "FETCH_SIZE" "WRITE_SIZE" \
  "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES" \
  "SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE" \
  "TCC_HIT_sum TCC_MISS_sum SQ_INSTS_VALU_TRANS_F32 SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM_RD SQ_LDS_IDX_ACTIVE"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $group --output-format csv -d "$OUT/p$i" -o pmc -- python bench.py $ARGS > "$OUT/p$i.log" 2>&1
done
echo "pmc passes done: $i"
