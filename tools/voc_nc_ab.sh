#!/bin/bash
# x-tile NC (column tiles per workgroup) A/B on the GPU box: per-op profiles of each library variant
# and a bitwise comparison of their outputs (NC = 2 must be bit-identical to NC = 1).
# Usage: bash tools/voc_nc_ab.sh OUT name...   (name = libpwg_<name>.so; "base" = default lib)
set -e
OUT=$1; shift
mkdir -p "$OUT"
export TMPDIR=/tmp PWG_NO_BUILD=1
for c in hifigan_v1 melgan_v1 mb_melgan_v2; do
  for v in "$@"; do
    if [ "$v" = base ]; then lib=parallelwavegan_amd/lib/libpwg_hip.so; else lib=parallelwavegan_amd/lib/variants/libpwg_$v.so; fi
    PWG_LIB_PATH=$lib timeout -k 10 200 python tools/cnet_profile.py $c --dump "/tmp/nc_ab_${c}_$v.npy" > "$OUT/ops_${c}_$v.txt" 2>&1
    echo "$c $v $(grep total $OUT/ops_${c}_$v.txt)"
  done
  python - "$OUT" "$c" "$@" <<'PY'
import sys, numpy as np
out, c, vs = sys.argv[1], sys.argv[2], sys.argv[3:]
ref = np.load(f"/tmp/nc_ab_{c}_{vs[0]}.npy")
for v in vs[1:]:
    o = np.load(f"/tmp/nc_ab_{c}_{v}.npy")
    print(c, v, "vs", vs[0], "bit-identical" if np.array_equal(ref.view(np.uint32), o.view(np.uint32)) else f"DIFFERS max|d|={np.abs(ref-o).max():.3e}")
PY
done
rm -f /tmp/nc_ab_*.npy
