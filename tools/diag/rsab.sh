export PWG_NO_BUILD=1
mkdir -p gpurun_out/r06h
for v in base nobar nomfma1; do
  if [ $v = base ]; then L=parallelwavegan_amd/lib/libpwg_hip.so; else L=parallelwavegan_amd/lib/rsv/libpwg_$v.so; fi
  PWG_LIB_PATH=$L timeout -k 10 100 python tools/cnet_profile.py mb_melgan_v2 --nocheck > gpurun_out/r06h/$v.txt 2>&1 || exit 1
  echo "== $v"; grep "stack.2+\|total" gpurun_out/r06h/$v.txt | awk '{print $1, $(NF-3)}' | tr '\n' ' '; echo
done
