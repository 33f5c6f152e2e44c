set -e
export PWG_NO_BUILD=1
mkdir -p gpurun_out/r02_sub
for k in 1 32 16 8 4 2 1 32; do
  timeout -k 10 200 python bench.py --cpu-seconds 0 --no-latency --sub-plans $k > gpurun_out/r02_sub/k$k.json 2>gpurun_out/r02_sub/k$k.err
  python -c "import json; d=json.load(open('gpurun_out/r02_sub/k$k.json')); print($k, d['value'], d['roofline']['avg_launch_ms'], d['roofline']['launches_timed'])"
done
