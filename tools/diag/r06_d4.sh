set -e
O=gpurun_out/r06d4; mkdir -p $O; export PWG_NO_BUILD=1 TMPDIR=/tmp
R=$(pwd)
timeout -k 10 400 python -u -m pytest tests/test_gpu_vocoders.py -x -q --timeout 120 --timeout-method thread -k "fused_stack_chain" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for o in narrow=2 narrow=1; do
  timeout -k 10 120 python tools/cnet_profile.py mb_melgan_v2 --opt $o > $O/mb_$o.txt 2>&1
done
(cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace -d $R/$O/kt -o run --output-format csv -- python3 $R/tools/cnet_profile.py mb_melgan_v2 --steps 1 > $R/$O/kt.log 2>&1)
ls $O/kt
for f in $O/mb_*.txt; do echo "$f $(grep total $f)"; done
