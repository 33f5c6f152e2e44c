"""Engine-option A/B on the LJ v1 / LibriTTS plans (diagnostic, GPU box): median wall ms per
forward (device-resident inputs, no range check) for each option set given as JSON on the command
line, e.g. python tools/diag/opt_bench.py '{"waves_per_wg": 8}' '{"waves_per_wg": 4}'"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from parallelwavegan_amd import Engine, configs, synthetic  # noqa: E402

modes = [json.loads(a) for a in sys.argv[1:]] or [{}]
dev = torch.device("cuda", 0)
plans = [("ljspeech_v1", [64]), ("ljspeech_v1", [512]), ("ljspeech_v1", [1024]), ("ljspeech_v1", [2048]), ("ljspeech_v1", [512] * 16),
         ("libritts_v1", synthetic.libritts_lengths(32, seed=3).tolist())]
if os.environ.get("PLANS") == "small":
    plans = plans[:4]
elif os.environ.get("PLANS") == "lat":
    plans = [("ljspeech_v1", [f]) for f in (64, 96, 128, 192, 256, 384, 512)]
elif os.environ.get("PLANS") == "latx":
    plans = [("ljspeech_v1", [f]) for f in (64, 128, 256, 512, 768, 1024, 1536, 2048)]
    plans += [("ljspeech_v1", [64] * 4), ("ljspeech_v1", [512] * 4), ("libritts_v1", [300, 120, 40])]
for cfg, lengths in plans:
    params = configs.generator_params(cfg)
    row = {"config": cfg, "frames": lengths if len(lengths) <= 2 else f"{len(lengths)} utts, {sum(lengths)} frames"}
    for mi, opts in enumerate(modes):
        eng = Engine(params, dev)
        eng.load_state_dict(synthetic.make_state_dict(params, seed=0))
        for k, v in opts.items():
            eng.set_option(k, v)
        plan = eng.plan(lengths)
        rs = np.random.RandomState(1)
        mel = torch.from_numpy(rs.standard_normal(sum(lengths) * 80).astype(np.float32)).to(dev)
        noise = torch.from_numpy(rs.standard_normal(plan.total_samples).astype(np.float32)).to(dev)
        out = torch.empty(plan.total_samples, device=dev)
        for _ in range(3):
            eng.run(plan, mel, noise, out, check=False)
        torch.cuda.synchronize()
        n = 30 if plan.total_samples < 1e6 else 8
        ts = []
        for _ in range(n):
            t0 = time.perf_counter()
            eng.run(plan, mel, noise, out, check=False)
            torch.cuda.synchronize()
            ts.append((time.perf_counter() - t0) * 1e3)
        eng.run_status(plan)
        ts.sort()
        med = ts[len(ts) // 2]
        row[f"m{mi}"] = {"opts": opts, "median_ms": round(med, 3), "min_ms": round(ts[0], 3),
                         "Msamples_per_s": round(plan.total_samples / med / 1e3, 2)}
    print(json.dumps(row), flush=True)
