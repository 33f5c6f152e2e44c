"""HiFiGAN v1 B = 1 decode loop (utterances <= 512 frames of the bench's 512-utterance list) under
run-time option combinations (diagnostic, GPU box): python tools/diag/hifi_loop_ab.py [CFG]"""
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

cfg = sys.argv[1] if len(sys.argv) > 1 else "hifigan_v1"
dev = torch.device("cuda", 0)
cls, p = configs.vocoder_params(cfg)
m = {"MelGANGenerator": MelGANGenerator, "HiFiGANGenerator": HiFiGANGenerator}[cls](**p)
m.load_state_dict({k: torch.from_numpy(v) for k, v in synthetic.make_module_state_dict(m, seed=0).items()})
if cfg in configs.VOCODER_PQMF:
    m.pqmf = PQMF(**configs.VOCODER_PQMF[cfg])
m = m.to(dev)
eng = m.engine()
L = [int(f) for f in synthetic.libritts_lengths(512, seed=3)[:128] if f <= 512][:24]
mels = [torch.from_numpy(synthetic.make_mel(f, 80, seed=500 + i)).to(dev) for i, f in enumerate(L)]


def loop():
    ms = []
    for x in mels:
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        m.inference(x)
        torch.cuda.synchronize(dev)
        ms.append((time.perf_counter() - t0) * 1e3)
    return ms


res = []
with torch.no_grad():
    m.inference(mels[0])
    for narrow, ndma, streams in [(1, 1, 1), (1, 0, 1), (1, 1, 2), (1, 1, 0), (2, 1, 1), (0, 1, 1), (1, 1, 1)]:
        eng.set_narrow(narrow)
        eng.set_narrow_dma(ndma)
        eng.set_streams(streams)
        eng._plans.clear()
        first = loop()  # new plans
        steady = loop()  # cached plans (eager: fewer than GRAPH_AFTER runs)
        res.append({"narrow": narrow, "narrow_dma": ndma, "streams": streams,
                    "first_mean_ms": round(float(np.mean(first)), 3), "steady_mean_ms": round(float(np.mean(steady)), 3)})
        print(json.dumps(res[-1]), flush=True)
print(json.dumps({"frames": L}))
