"""Vocoder B = 1 latency A/B on the GPU box: the drop-in's inference() at T' = 64 / 512 with
PWG_CNET_OPT_NARROW 0 / 1 / 2 and PWG_CNET_OPT_NARROW_DMA 0 / 1 (same library), median wall ms per synchronised call, the kernels'
summed ms, and the per-op ms of the automatic mode (tools/diag/voc_lat_ops.sh's table, one line).
Usage: python tools/diag/voc_lat_ab.py OUT.json"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch  # noqa: E402

from parallelwavegan_amd import configs, synthetic  # noqa: E402
from parallelwavegan_amd.hifigan import HiFiGANGenerator  # noqa: E402
from parallelwavegan_amd.melgan import PQMF, MelGANGenerator  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    res = {}
    for cfg in ("hifigan_v1", "mb_melgan_v2", "melgan_v1"):
        cls, params = configs.vocoder_params(cfg)
        m = {"MelGANGenerator": MelGANGenerator, "HiFiGANGenerator": HiFiGANGenerator}[cls](**params)
        m.load_state_dict({k: torch.from_numpy(v) for k, v in synthetic.make_module_state_dict(m, seed=0).items()})
        if cfg in configs.VOCODER_PQMF:
            m.pqmf = PQMF(**configs.VOCODER_PQMF[cfg])
        m = m.to(dev)
        eng = m.engine()
        for F in (64, 512):
            mel = torch.from_numpy(synthetic.make_mel(F, 80, seed=30)).to(dev)
            for mode, dma in ((0, 1), (1, 0), (1, 1), (2, 1)):
                eng.set_narrow(mode)
                eng.set_narrow_dma(dma)
                with torch.no_grad():
                    for _ in range(3):
                        m.inference(mel)
                    ts = []
                    for _ in range(15):
                        torch.cuda.synchronize(dev)
                        t0 = time.perf_counter()
                        m.inference(mel)
                        torch.cuda.synchronize(dev)
                        ts.append((time.perf_counter() - t0) * 1e3)
                    eng.set_timing(True)
                    eng.collect_timing()
                    m.inference(mel)
                    torch.cuda.synchronize(dev)
                    eng.set_timing(False)
                    t = eng.collect_timing()
                ts.sort()
                row = {"median_ms": round(ts[len(ts) // 2], 4), "min_ms": round(ts[0], 4),
                       "kernel_ms": round(sum(ms for _, ms, _ in t), 4),
                       "launches": int(sum(n for _, _, n in t))}
                if mode == 1 and dma == 1:
                    row["ops"] = [(name, round(ms, 4), int(n)) for name, ms, n in t]
                res[f"{cfg}_T{F}_narrow{mode}_dma{dma}"] = row
                print(cfg, F, mode, dma, {k: v for k, v in row.items() if k != "ops"}, flush=True)
            eng.set_narrow(1)
            eng.set_narrow_dma(1)
    json.dump(res, open(sys.argv[1], "w"), indent=1)


if __name__ == "__main__":
    main()
