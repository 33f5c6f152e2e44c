set -e
O=gpurun_out/r06d1; mkdir -p $O; export PWG_NO_BUILD=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_vocoders.py -x -q --timeout 120 --timeout-method thread -k "thinw or golden or oracle or ragged" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 200 python tools/diag/first_call_voc.py hifigan_v1 > $O/fc_hifi.json 2>$O/fc_hifi.err
timeout -k 10 200 python tools/diag/first_call_voc.py mb_melgan_v2 > $O/fc_mb.json 2>$O/fc_mb.err
timeout -k 10 120 python tools/cnet_profile.py mb_melgan_v2 > $O/mb_def.txt 2>&1
for o in thinw=0 xt_dma=2 xt_dma=11 xt_dma=13 xt_dma=1 xcd_order=0 narrow=0; do
  timeout -k 10 120 python tools/cnet_profile.py mb_melgan_v2 --opt $o > $O/mb_$o.txt 2>&1
done
timeout -k 10 150 python tools/cnet_profile.py hifigan_v1 > $O/hifi_def.txt 2>&1
cat $O/fc_*.json
