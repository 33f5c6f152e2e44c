"""Where a new batch shape's first drop-in call spends its time (diagnostic, GPU box): after a
warm B = 1 call, for each new (T', B): plan creation, workspace growth, the first run and the
steady run, each synchronised and timed separately. Usage: python tools/diag/first_call.py"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from parallelwavegan_amd import ParallelWaveGANGenerator, configs, synthetic  # noqa: E402

dev = torch.device("cuda", 0)
params = configs.generator_params("ljspeech_v1")
m = ParallelWaveGANGenerator(**params)
m.remove_weight_norm()
m.load_state_dict({k: torch.from_numpy(v) for k, v in synthetic.make_state_dict(params, seed=0).items()})
m = m.eval().to(dev)


def t(fn):
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    r = fn()
    torch.cuda.synchronize(dev)
    return (time.perf_counter() - t0) * 1e3, r


with torch.no_grad():
    mel = torch.from_numpy(synthetic.make_mel(64, 80, seed=1)).to(dev)
    warm = [t(lambda: m.inference(mel))[0] for _ in range(3)]
    eng = m.engine()
    for F, B in [(64, 16), (512, 16), (2048, 16), (100, 1), (700, 3), (300, 5)]:
        mels = [torch.from_numpy(synthetic.make_mel(F, 80, seed=10 + b)).to(dev) for b in range(B)]
        row = {"frames": F, "batch": B}
        row["plan_ms"], plan = t(lambda: eng.plan([F] * B))
        row["workspace_ms"], _ = t(lambda: eng.workspace(plan.workspace_bytes))
        row["workspace_MB"] = round(plan.workspace_bytes / 2**20, 1)
        mel_d = torch.cat([x.reshape(-1) for x in mels])
        noise_d = torch.randn(plan.total_samples, device=dev)
        out_d = torch.empty(plan.total_samples, device=dev)
        row["engine_run_first_ms"], _ = t(lambda: eng.run(plan, mel_d, noise_d, out_d))
        row["engine_run_second_ms"], _ = t(lambda: eng.run(plan, mel_d, noise_d, out_d))
        call = (lambda: m.inference(mels[0])) if B == 1 else (lambda: m.inference_batch(mels))
        seg0 = torch.cuda.memory_stats(dev).get("segment.all.allocated", 0)
        row["first_call_ms"], _ = t(call)
        row["new_segments"] = torch.cuda.memory_stats(dev).get("segment.all.allocated", 0) - seg0
        row["second_call_ms"], _ = t(call)
        row["steady_ms"] = round(float(np.median([t(call)[0] for _ in range(5)])), 3)
        print(json.dumps({k: (round(v, 3) if isinstance(v, float) else v) for k, v in row.items()}), flush=True)
    print(json.dumps({"warm_B1_T64_ms": [round(x, 3) for x in warm]}))
