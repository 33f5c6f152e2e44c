#!/bin/bash
# PMC passes over one vocoder forward (GPU box): per-kernel MFMA busy, LDS bank conflicts, LDS
# waits and barrier-ish idle of the conv-network kernels. Usage: bash tools/voc_pmc.sh OUT [CONFIG]
set -e
OUT=$1; CFG=${2:-hifigan_v1}
export TMPDIR=/tmp PWG_NO_BUILD=1
mkdir -p "$OUT"
i=0
for group in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE" \
             "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_LDS SQ_INSTS_VALU SQ_ACTIVE_INST_VALU"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --pmc $group --output-format csv -d "$OUT/p$i" -o pmc -- python tools/cnet_profile.py $CFG --steps 1 > "$OUT/p$i.log" 2>&1
done
python tools/pmc_summary.py "$OUT" "$OUT/summary.json" > /dev/null
python - "$OUT/summary.json" <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
rows = []
for k, v in d.items():
    if "GRBM_GUI_ACTIVE" not in v or "SQ_WAVE_CYCLES" not in v or "SQ_WAIT_ANY" not in v:
        continue
    gui = v["GRBM_GUI_ACTIVE"]
    wc = max(v["SQ_WAVE_CYCLES"], 1)
    rows.append((gui, k.split("(")[0].replace("void pwg::", "").replace("(anonymous namespace)::", ""),
                 v["SQ_VALU_MFMA_BUSY_CYCLES"] / (gui / 8 * 1024),
                 v["SQ_LDS_BANK_CONFLICT"] / max(v["SQ_LDS_IDX_ACTIVE"], 1),
                 v["SQ_WAIT_INST_LDS"] / wc, v["SQ_WAIT_ANY"] / wc, v["SQ_ACTIVE_INST_ANY"] / wc))
rows.sort(reverse=True)
print(f"{'kernel':60s} {'gui_cyc':>10s} {'mfma_busy':>9s} {'lds_conf':>8s} {'wait_lds':>8s} {'wait_any':>8s} {'active':>7s}")
for gui, k, mb, lc, wl, wa, ac in rows[:16]:
    print(f"{k[:60]:60s} {gui:10.0f} {mb:9.3f} {lc:8.3f} {wl:8.3f} {wa:8.3f} {ac:7.3f}")
PY
