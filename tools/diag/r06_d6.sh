set -e
O=gpurun_out/r06d6; mkdir -p $O; export PWG_NO_BUILD=1
timeout -k 10 600 python -u -m pytest tests/test_gpu_vocoders.py tests/test_gpu_vocoder_range.py -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 120 python tools/cnet_profile.py mb_melgan_v2 > $O/mb.txt 2>&1
timeout -k 10 150 python tools/cnet_profile.py hifigan_v1 > $O/hifi.txt 2>&1
grep -E "total|melgan.(3|9|15) " $O/mb.txt; grep -E "total|^ups" $O/hifi.txt
