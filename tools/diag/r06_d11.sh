set -e
O=gpurun_out/r06d11; mkdir -p $O; export PWG_NO_BUILD=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_vocoders.py -x -q --timeout 120 --timeout-method thread -k "rstack or golden or oracle" > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 120 python tools/cnet_profile.py mb_melgan_v2 --bitwise-rstack > $O/mb.txt 2>&1
timeout -k 10 120 python tools/cnet_profile.py melgan_v1 > $O/mg.txt 2>&1
PWG_LIB_PATH=parallelwavegan_amd/lib/abv/libpwg_mg0.so timeout -k 10 120 python tools/cnet_profile.py mb_melgan_v2 > $O/mb_mg0.txt 2>&1
PWG_LIB_PATH=parallelwavegan_amd/lib/abv/libpwg_mg0.so timeout -k 10 120 python tools/cnet_profile.py melgan_v1 > $O/mg_mg0.txt 2>&1
for f in $O/mb.txt $O/mb_mg0.txt; do echo "$f $(grep total $f)"; grep -E "bitwise|melgan.[45].stack" $f; done
for f in $O/mg.txt $O/mg_mg0.txt; do echo "$f $(grep total $f)"; grep -E "melgan.(4|9).stack.2 " $f; done
