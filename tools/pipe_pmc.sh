#!/bin/bash
# PMC of the layer pipeline vs the per-layer launches (GPU box): FETCH_SIZE, WRITE_SIZE and a
# clock / matrix-pipe / wait pass per (mode, workload), each its own rocprofv3 run over
# tools/diag/pipe_pmc.py child. Usage: bash tools/pipe_pmc.sh OUT
set -e
OUT=$1
export TMPDIR=/tmp PWG_NO_BUILD=1
R=$GRAFT_REPO_ROOT
mkdir -p "$OUT"
cd /tmp
for work in bench lj512; do
  for mode in per_layer pipeline; do
    D="$R/$OUT/${mode}_$work"
    mkdir -p "$D"
    timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$D/fetch" -o pmc -- python3 "$R/tools/diag/pipe_pmc.py" child $mode $work > "$D/fetch.log" 2>&1
    timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$D/write" -o pmc -- python3 "$R/tools/diag/pipe_pmc.py" child $mode $work > "$D/write.log" 2>&1
    timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_MFMA --output-format csv -d "$D/clk" -o pmc -- python3 "$R/tools/diag/pipe_pmc.py" child $mode $work > "$D/clk.log" 2>&1
  done
done
cd "$R"
python tools/diag/pipe_pmc.py summary "$OUT"
