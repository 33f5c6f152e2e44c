set -e
O=gpurun_out/r06d5; mkdir -p $O; export PWG_NO_BUILD=1 TMPDIR=/tmp
timeout -k 10 400 python bench.py --config hifigan_v1 --steps 3 --pmc off > $O/hifi_pmcoff.json 2> $O/a.err
timeout -k 10 400 python bench.py --config hifigan_v1 --steps 3 > $O/hifi_pmcauto.json 2> $O/b.err
python - <<'PY'
import json
for f in ["hifi_pmcoff", "hifi_pmcauto"]:
    d = json.loads(open(f"gpurun_out/r06d5/{f}.json").read().strip().splitlines()[-1])
    print(f, [(r["frames"], r["batch"], r["first_call_ms"], r["median_ms"]) for r in d["latency"]["rows"]])
PY
