"""Layer pipeline vs per-layer launches (diagnostic, GPU box): median wall ms per forward with
device-resident inputs, LJ v1 B = 1 at T' = 64 / 512 / 2048, B = 16 at T' = 512, and the bench's
32-utterance LibriTTS batch. Usage: python tools/diag/pipe_bench.py [reps]"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from parallelwavegan_amd import Engine, configs, synthetic  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
dev = torch.device("cuda", 0)
res = []
for cfg, lengths in [("ljspeech_v1", [64]), ("ljspeech_v1", [512]), ("ljspeech_v1", [2048]),
                     ("ljspeech_v1", [512] * 16), ("libritts_v1", synthetic.libritts_lengths(32, seed=3).tolist())]:
    params = configs.generator_params(cfg)
    row = {"config": cfg, "frames": lengths if len(lengths) <= 2 else f"{len(lengths)} utts, {sum(lengths)} frames"}
    for mode, lim in (("per_layer", 0), ("pipeline", 1 << 24)):
        eng = Engine(params, dev)
        eng.load_state_dict(synthetic.make_state_dict(params, seed=0))
        eng.set_option("pipeline", lim)
        plan = eng.plan(lengths)
        rs = np.random.RandomState(1)
        mel = torch.from_numpy(rs.standard_normal(sum(lengths) * 80).astype(np.float32)).to(dev)
        noise = torch.from_numpy(rs.standard_normal(plan.total_samples).astype(np.float32)).to(dev)
        out = torch.empty(plan.total_samples, device=dev)
        for _ in range(3):
            eng.run(plan, mel, noise, out, check=False)
        torch.cuda.synchronize()
        ts = []
        n = reps if plan.total_samples < 4e6 else max(3, reps // 4)
        for _ in range(n):
            t0 = time.perf_counter()
            eng.run(plan, mel, noise, out, check=False)
            torch.cuda.synchronize()
            ts.append((time.perf_counter() - t0) * 1e3)
        eng.set_timing(True)
        eng.collect_timing()
        eng.run(plan, mel, noise, out, check=False)
        torch.cuda.synchronize()
        t = eng.collect_timing()
        eng.set_timing(False)
        eng.run_status(plan)
        ts.sort()
        med = ts[len(ts) // 2]
        row[mode] = {"median_ms": round(med, 3), "min_ms": round(ts[0], 3),
                     "samples_per_s": round(plan.total_samples / med * 1e3, 1),
                     "kernel_ms": {k: round(v[0], 3) for k, v in t.items() if v[1]}}
    print(json.dumps(row), flush=True)
