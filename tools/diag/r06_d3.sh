set -e
O=gpurun_out/r06d3; mkdir -p $O; export PWG_NO_BUILD=1
timeout -k 10 400 python -u -m pytest tests/test_gpu_vocoders.py -x -q --timeout 120 --timeout-method thread -k "dma or xcd or narrow or golden or oracle or ragged" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for o in xt_dma=9 xt_dma=8; do
  timeout -k 10 120 python tools/cnet_profile.py mb_melgan_v2 --opt $o > $O/mb_$o.txt 2>&1
  timeout -k 10 150 python tools/cnet_profile.py hifigan_v1 --opt $o > $O/hifi_$o.txt 2>&1
done
for f in $O/mb_*.txt; do echo "$f $(grep total $f)"; grep -E "melgan.(3|9|15) " $f; done
for f in $O/hifi_*.txt; do echo "$f $(grep total $f)"; grep -E "^ups" $f; done
