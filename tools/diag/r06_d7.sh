set -e
O=gpurun_out/r06d7; mkdir -p $O; export PWG_NO_BUILD=1
L=parallelwavegan_amd/lib/abv
for v in main tpc2 main2 tpc2b; do
  case $v in main|main2) lib=parallelwavegan_amd/lib/libpwg_hip.so;; *) lib=$L/libpwg_tpc2.so;; esac
  PWG_LIB_PATH=$lib timeout -k 10 120 python tools/cnet_profile.py mb_melgan_v2 > $O/mb_$v.txt 2>&1
done
for v in main ctdb1; do
  case $v in main) lib=parallelwavegan_amd/lib/libpwg_hip.so;; *) lib=$L/libpwg_ctdb1.so;; esac
  PWG_LIB_PATH=$lib timeout -k 10 150 python tools/cnet_profile.py hifigan_v1 > $O/hifi_$v.txt 2>&1
done
PWG_LIB_PATH=$L/libpwg_tpc2.so timeout -k 10 300 python -u -m pytest tests/test_gpu_vocoders.py -x -q --timeout 120 --timeout-method thread -k "golden or oracle" > $O/pytest_tpc2.log 2>&1 && tail -1 $O/pytest_tpc2.log
for f in $O/mb_*.txt; do echo "$f $(grep -E 'melgan.22 ' $f | awk '{print $(NF-3)}') $(grep total $f)"; done
for f in $O/hifi_*.txt; do echo "$f $(grep -E '^upsamples.3.1' $f | awk '{print $(NF-3)}') $(grep total $f)"; done
