set -e
O=gpurun_out/r06d2; mkdir -p $O; export PWG_NO_BUILD=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_vocoders.py -x -q --timeout 120 --timeout-method thread -k "thinw" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for o in thinw=0 thinw=1 thinw=2; do
  timeout -k 10 120 python tools/cnet_profile.py mb_melgan_v2 --opt $o > $O/mb_$o.txt 2>&1
done
timeout -k 10 250 python tools/diag/voc_latency_twice.py hifigan_v1 --exact > $O/lat2_hifi.json 2> $O/lat2_hifi.err
cat $O/lat2_hifi.json
for f in $O/mb_*.txt; do echo "$f $(grep -E 'melgan.22 ' $f)"; done
