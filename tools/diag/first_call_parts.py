"""Where a first B = 1 call at a new length goes (diagnostic, GPU box).

  python tools/diag/first_call_parts.py CFG

For the decode loop's utterances of <= 512 frames: the first inference() at the length (fresh plan),
the plan build alone (host), a second call (plan cached, eager: graphs start on the second run's
capture... so the third call), and the steady graph-replayed call; one JSON line, ms."""
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
    cfg = sys.argv[1]
    dev = torch.device("cuda", 0)
    cls, p = configs.vocoder_params(cfg)
    m = {"MelGANGenerator": MelGANGenerator, "HiFiGANGenerator": HiFiGANGenerator}[cls](**p)
    m.load_state_dict({k: torch.from_numpy(v) for k, v in synthetic.make_module_state_dict(m, seed=0).items()})
    if cfg in configs.VOCODER_PQMF:
        m.pqmf = PQMF(**configs.VOCODER_PQMF[cfg])
    m = m.to(dev)
    eng = m.engine()
    lengths = [int(f) for f in synthetic.libritts_lengths(32, seed=3) if f <= 512]
    rows = []

    def call(mel):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        m.inference(mel)
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) * 1e3

    with torch.no_grad():
        m.inference(torch.from_numpy(synthetic.make_mel(7, 80, seed=1)).to(dev))
        for i, f in enumerate(lengths):
            mel = torch.from_numpy(synthetic.make_mel(f, 80, seed=500 + i)).to(dev)
            first = call(mel)
            # a fresh plan object of another length, built on the host only (timing the build)
            t0 = time.perf_counter()
            eng.plan([f + 1000])
            build = (time.perf_counter() - t0) * 1e3
            eng._plans.pop((f + 1000,), None)
            second = call(mel)   # eager, plan cached (this run is the capture's trigger: counts 2)
            third = call(mel)    # captured and replayed
            steady = float(np.median([call(mel) for _ in range(5)]))
            eng.set_graphs(False)
            eager = float(np.median([call(mel) for _ in range(5)]))
            eng.set_graphs(True)
            rows.append({"frames": f, "first": round(first, 3), "plan_build": round(build, 3), "second": round(second, 3),
                         "third": round(third, 3), "steady_graph": round(steady, 3), "steady_eager": round(eager, 3)})
    print(json.dumps({"config": cfg, "rows": rows,
                      "mean": {k: round(float(np.mean([r[k] for r in rows])), 3) for k in rows[0] if k != "frames"}}))


if __name__ == "__main__":
    main()
