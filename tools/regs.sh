#!/bin/bash
# Register / spill summary of one HIP source for gfx950: bash tools/regs.sh FILE [extra hipcc flags]
f=$1; shift
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -c -mllvm -amdgpu-atomic-optimizer-strategy=None \
  "$@" "$f" -o /tmp/regs.o -Rpass-analysis=kernel-resource-usage 2>&1 | sed 's/ \[-Rpass-analysis=kernel-resource-usage\]//' |
  awk '/error/ {print} /Function Name/ {n=$NF} / VGPRs:/ {v=$NF} /VGPRs Spill/ {print n, "vgpr", v, "spill", $NF}'
