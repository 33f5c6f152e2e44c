set -e
O=gpurun_out/r06d10; mkdir -p $O; export PWG_NO_BUILD=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_vocoders.py -x -q --timeout 120 --timeout-method thread -k "rstack or golden or oracle" > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 120 python tools/cnet_profile.py mb_melgan_v2 --bitwise-rstack > $O/mb.txt 2>&1
timeout -k 10 120 python tools/cnet_profile.py mb_melgan_v2 --rstack 2 > $O/mb_rs2.txt 2>&1
timeout -k 10 120 python tools/cnet_profile.py melgan_v1 > $O/mg.txt 2>&1
grep -E "bitwise|total|melgan.4.stack" $O/mb.txt; grep -E "total|melgan.4.stack" $O/mb_rs2.txt; grep -E "total|stack.4" $O/mg.txt | head -8
