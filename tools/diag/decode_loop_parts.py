"""Where a vocoder's decode-loop call goes (diagnostic, GPU box): the bench's 32 distinct LibriTTS
lengths at B = 1, (a) as the bench runs them, (b) with every plan built beforehand (host only), and
(c) the device span of each call (timing mode 2). python tools/diag/decode_loop_parts.py hifigan_v1"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np  # noqa: E402
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
eng = m.engine()


def loop(lengths, seed):
    ms = []
    for i, f in enumerate(lengths):
        mel = torch.from_numpy(synthetic.make_mel(int(f), 80, seed=seed + i)).to(dev)
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        m.inference(mel)
        torch.cuda.synchronize(dev)
        ms.append((time.perf_counter() - t0) * 1e3)
    return np.array(ms)


res = {}
with torch.no_grad():
    m.inference(torch.from_numpy(synthetic.make_mel(7, 80, seed=1)).to(dev))
    base = [int(f) for f in synthetic.libritts_lengths(32, seed=3)]
    short = [f for f in base if f <= 512]
    res["bench_order_le512"] = round(float(loop(short, 500).mean()), 3)
    # other distinct lengths (no plan reuse), plans built first on the host
    lens2 = [f + 1 for f in short]
    t0 = time.perf_counter()
    for f in lens2:
        eng.plan([f])
    res["plan_build_ms_each"] = round((time.perf_counter() - t0) * 1e3 / len(lens2), 3)
    res["prebuilt_plans_le512"] = round(float(loop(lens2, 600).mean()), 3)
    # device span of each call and the host's share
    eng.set_timing(2)
    spans = []
    for i, f in enumerate(short):
        mel = torch.from_numpy(synthetic.make_mel(int(f) + 2, 80, seed=700 + i)).to(dev)
        eng.collect_timing()
        m.inference(mel)
        torch.cuda.synchronize(dev)
        spans.append(eng.timing_span())
        eng.collect_timing()
    eng.set_timing(False)
    res["span_ms_le512"] = round(float(np.mean(spans)), 3)
    res["n_short"] = len(short)
print(json.dumps({name: res}))
