"""The bench's PWG latency order (B = 1 then B = 16 at T' = 64) with the B = 16 first call split into
its parts (diagnostic, GPU box): python tools/diag/first_call_b16.py"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from parallelwavegan_amd import ParallelWaveGANGenerator, _lib, configs, synthetic  # noqa: E402

dev = torch.device("cuda", 0)
params = configs.generator_params("ljspeech_v1")
m = ParallelWaveGANGenerator(**params)
m.remove_weight_norm()
m.load_state_dict({k: torch.from_numpy(v) for k, v in synthetic.make_state_dict(params, seed=0).items()})
m = m.eval().to(dev)
H = m.upsample_factor


def t(fn):
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    r = fn()
    torch.cuda.synchronize(dev)
    return round((time.perf_counter() - t0) * 1e3, 3), r


res = {}
with torch.no_grad():
    m.inference(torch.from_numpy(synthetic.make_mel(7, 80, seed=1)).to(dev), torch.from_numpy(synthetic.make_noise(7 * H, seed=1)).to(dev))
    mel1 = torch.from_numpy(synthetic.make_mel(64, 80, seed=30)).to(dev)
    n1 = torch.from_numpy(synthetic.make_noise(64 * H, seed=60)).to(dev)
    res["b1_first"], _ = t(lambda: m.inference(mel1, n1))
    res["b1_steady"] = [t(lambda: m.inference(mel1, n1))[0] for _ in range(3)]
    eng = m.engine()
    for B in (16, 8):
        F = 64
        mels = [torch.from_numpy(synthetic.make_mel(F, 80, seed=30 + b)).to(dev) for b in range(B)]
        noises = [torch.from_numpy(synthetic.make_noise(F * H, seed=60 + b)).to(dev) for b in range(B)]
        r = {}
        r["plan_ms"], plan = t(lambda: eng.plan([F] * B))
        r["ws_bytes_MB"] = round(plan.workspace_bytes / 2**20, 1)
        r["ws_have_MB"] = round(max((w.numel() for w in eng._workspaces.values()), default=0) / 2**20, 1)
        r["cat_ms"], mel_d = t(lambda: torch.cat([x.reshape(-1) for x in mels]))
        r["cat2_ms"], noise_d = t(lambda: torch.cat([x.reshape(-1) for x in noises]))
        r["out_ms"], out_d = t(lambda: torch.empty(plan.total_samples, device=dev))
        r["run_first_ms"], _ = t(lambda: eng.run(plan, mel_d, noise_d, out_d))
        r["run_second_ms"], _ = t(lambda: eng.run(plan, mel_d, noise_d, out_d))
        r["first_call_ms"], _ = t(lambda: m.inference_batch(mels, noises))
        r["steady_ms"] = [t(lambda: m.inference_batch(mels, noises))[0] for _ in range(3)]
        eng.set_timing(2)
        eng.collect_timing()
        eng.run(plan, mel_d, noise_d, out_d)
        torch.cuda.synchronize(dev)
        r["span_ms"] = round(eng.timing_span(), 3)
        eng.collect_timing()
        eng.set_timing(False)
        res[f"B{B}"] = r
print(json.dumps(res))
