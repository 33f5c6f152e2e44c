"""B = 1 latency of a vocoder drop-in under values of one CnetEngine option (diagnostic, GPU box).

  python tools/diag/opt_lat.py CFG SETTER V1,V2,.. [T1,T2,..]   e.g. mb_melgan_v2 set_mstack 0,1 64,512
  (several setters: SETTER s1:s2 and values a1:a2,b1:b2 -- each value sets every setter in turn)

Per (value, T'): median wall ms of 30 synchronised inference() calls, the device span of one call
(timing mode 2) and, for the first value, whether every later value's output is bit-identical.
One JSON line."""
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


def main():
    cfg, setter = sys.argv[1], sys.argv[2]
    values = sys.argv[3].split(",")
    frames = [int(v) for v in (sys.argv[4] if len(sys.argv) > 4 else "64,512").split(",")]
    dev = torch.device("cuda", 0)
    cls, params = configs.vocoder_params(cfg)
    m = {"MelGANGenerator": MelGANGenerator, "HiFiGANGenerator": HiFiGANGenerator}[cls](**params)
    m.load_state_dict({k: torch.from_numpy(v) for k, v in synthetic.make_module_state_dict(m, seed=0).items()})
    if cfg in configs.VOCODER_PQMF:
        m.pqmf = PQMF(**configs.VOCODER_PQMF[cfg])
    m = m.to(dev)
    eng = m.engine()
    res = {"config": cfg, "option": setter, "rows": []}
    ref = {}
    with torch.no_grad():
        for v in values:
            for st, sv in zip(setter.split(":"), v.split(":")):
                getattr(eng, st)(int(sv))
            for F in frames:
                mel = torch.from_numpy(synthetic.make_mel(F, 80, seed=7)).to(dev)
                for _ in range(5):
                    y = m.inference(mel)
                ts = []
                for _ in range(30):
                    torch.cuda.synchronize(dev)
                    t0 = time.perf_counter()
                    m.inference(mel)
                    torch.cuda.synchronize(dev)
                    ts.append((time.perf_counter() - t0) * 1e3)
                eng.set_timing(2)
                eng.collect_timing()
                m.inference(mel)
                torch.cuda.synchronize(dev)
                span = eng.timing_span()
                eng.collect_timing()
                eng.set_timing(False)
                out = y.cpu().numpy()
                same = None
                if F in ref:
                    same = bool(np.array_equal(out, ref[F]))
                else:
                    ref[F] = out
                res["rows"].append({"value": v, "frames": F, "median_ms": round(float(np.median(ts)), 4),
                                    "min_ms": round(float(np.min(ts)), 4), "span_ms": round(span, 4),
                                    "bit_identical_to_first": same})
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
