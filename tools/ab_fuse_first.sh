set -e
export TMPDIR=/tmp PWG_NO_BUILD=1
mkdir -p gpurun_out/ff2
for i in 1 2; do
timeout -k 10 300 python bench.py --cpu-seconds 0 > gpurun_out/ff2/fused$i.json 2> gpurun_out/ff2/fused$i.err
timeout -k 10 300 python bench.py --cpu-seconds 0 --no-fuse-first > gpurun_out/ff2/unfused$i.json 2> gpurun_out/ff2/unfused$i.err
done
for f in gpurun_out/ff2/*.json; do python -c "import json; d=json.load(open('$f')); print('$f', round(d['value']/1e6,2), d['kernel_ms_per_step'], d['roofline']['avg_launch_ms'])"; done
