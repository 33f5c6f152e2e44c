"""A vocoder's first inference_batch call at a new shape split into its parts (diagnostic, GPU box),
after the bench's batched leg has run: python tools/diag/first_call_voc.py hifigan_v1"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from parallelwavegan_amd import configs, synthetic  # noqa: E402
from parallelwavegan_amd.hifigan import HiFiGANGenerator  # noqa: E402
from parallelwavegan_amd.melgan import PQMF, MelGANGenerator  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "hifigan_v1"
dev = torch.device("cuda", 0)
cls, p = configs.vocoder_params(name)
m = {"MelGANGenerator": MelGANGenerator, "HiFiGANGenerator": HiFiGANGenerator}[cls](**p)
m.load_state_dict({k: torch.from_numpy(v) for k, v in synthetic.make_module_state_dict(m, seed=0).items()})
if name in configs.VOCODER_PQMF:
    m.pqmf = PQMF(**configs.VOCODER_PQMF[name])
m = m.eval().to(dev)


def t(fn):
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    r = fn()
    torch.cuda.synchronize(dev)
    return round((time.perf_counter() - t0) * 1e3, 3), r


res = {}
with torch.no_grad():
    eng = m.engine()
    # the bench's batched leg first (its plan is larger than any row's)
    lengths = synthetic.libritts_lengths(32, seed=3).tolist()
    big = eng.plan(lengths)
    mel = torch.randn(sum(lengths) * 80, device=dev)
    out = torch.empty(big.out_rows * eng.out_channels, device=dev)
    for _ in range(3):
        eng.run(big, mel, out, check=False)
    torch.cuda.synchronize(dev)
    m.inference(torch.from_numpy(synthetic.make_mel(7, 80, seed=1)).to(dev))
    mel1 = torch.from_numpy(synthetic.make_mel(64, 80, seed=30)).to(dev)
    res["b1_first"], _ = t(lambda: m.inference(mel1))
    res["b1_steady"] = [t(lambda: m.inference(mel1))[0] for _ in range(3)]
    for B, F in ((16, 64), (8, 64), (16, 96)):
        mels = [torch.from_numpy(synthetic.make_mel(F, 80, seed=30 + b)).to(dev) for b in range(B)]
        r = {}
        r["plan_ms"], plan = t(lambda: eng.plan([F] * B))
        r["ws_bytes_MB"] = round(plan.workspace_bytes / 2**20, 1)
        r["ws_have_MB"] = round(max((w.numel() for w in eng._workspaces.values()), default=0) / 2**20, 1)
        r["cat_ms"], mel_d = t(lambda: torch.cat([x.reshape(-1) for x in mels]))
        r["out_ms"], out_d = t(lambda: torch.empty(plan.out_rows * eng.out_channels, device=dev))
        r["run_first_ms"], _ = t(lambda: eng.run(plan, mel_d, out_d))
        r["run_second_ms"], _ = t(lambda: eng.run(plan, mel_d, out_d))
        r["run_third_ms"], _ = t(lambda: eng.run(plan, mel_d, out_d))
        r["call_ms"] = [t(lambda: m.inference_batch(mels))[0] for _ in range(3)]
        res[f"B{B}_T{F}"] = r
    # a fresh plan at a shape already seen by the schedule cache: plan build alone
    eng._plans.clear()
    r = {}
    mels = [torch.from_numpy(synthetic.make_mel(64, 80, seed=30 + b)).to(dev) for b in range(16)]
    r["plan_ms"], plan = t(lambda: eng.plan([64] * 16))
    mel_d = torch.cat([x.reshape(-1) for x in mels])
    out_d = torch.empty(plan.out_rows * eng.out_channels, device=dev)
    r["run_first_ms"], _ = t(lambda: eng.run(plan, mel_d, out_d))
    r["run_second_ms"], _ = t(lambda: eng.run(plan, mel_d, out_d))
    res["B16_T64_replanned"] = r
print(json.dumps({name: res}))
