"""Per-op time of a vocoder program under two option settings (diagnostic, GPU box): same plan,
same input, interleaved repetitions; prints the per-op ms of both and the step totals, and checks
the outputs bitwise. Usage: python tools/diag/voc_opt_ab.py CONFIG OPTION [reps] [on-value] [off-value]
(OPTION = a CnetEngine setter name, e.g. set_xt_dma)"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from parallelwavegan_amd import configs, synthetic  # noqa: E402
from parallelwavegan_amd.hifigan import HiFiGANGenerator  # noqa: E402
from parallelwavegan_amd.melgan import PQMF, MelGANGenerator  # noqa: E402

cfg, opt = sys.argv[1], sys.argv[2]
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 3
val_on = int(sys.argv[4]) if len(sys.argv) > 4 else 1  # the setter's "on" value
val_off = int(sys.argv[5]) if len(sys.argv) > 5 else 0  # ... and its "off" value
cls, p = configs.vocoder_params(cfg)
m = {"MelGANGenerator": MelGANGenerator, "HiFiGANGenerator": HiFiGANGenerator}[cls](**p)
m.load_state_dict({k: torch.from_numpy(v) for k, v in synthetic.make_module_state_dict(m, seed=0).items()})
if cfg in configs.VOCODER_PQMF:
    m.pqmf = PQMF(**configs.VOCODER_PQMF[cfg])
dev = torch.device("cuda", 0)
m = m.to(dev)
eng = m.engine()
lengths = synthetic.libritts_lengths(32, seed=3)
plan = eng.plan(lengths.tolist())
mel = torch.randn(int(lengths.sum()) * 80, device=dev, generator=torch.Generator(dev).manual_seed(0))
outs = {}
tot = {0: [], 1: []}
per = {0: None, 1: None}
for r in range(reps + 1):
    for v in (0, 1):
        getattr(eng, opt)(val_on if v else val_off)
        out = torch.empty(plan.out_rows * eng.out_channels, device=dev)
        eng.set_timing(True)
        eng.collect_timing()
        eng.run(plan, mel, out, check=False)
        torch.cuda.synchronize()
        t = eng.collect_timing()
        eng.set_timing(False)
        if r == 0:
            outs[v] = out.cpu().numpy()
            continue
        tot[v].append(sum(ms for _, ms, _ in t))
        if per[v] is None:
            per[v] = [[name, ms, n] for name, ms, n in t]
        else:
            for row, (_, ms, _) in zip(per[v], t):
                row[1] = min(row[1], ms)
print(cfg, opt, val_off, "->", val_on, "bitwise equal:", bool(np.array_equal(outs[0], outs[1])),
      "max|d|", float(np.abs(outs[0] - outs[1]).max()))
print(f"step ms  off {min(tot[0]):.3f}  on {min(tot[1]):.3f}")
for (name, a, n), (_, b, _) in zip(per[0], per[1]):
    if a > 0.05 or b > 0.05:
        print(f"  {name:40s} {a:7.3f} {b:7.3f}  {b / a if a else 0:5.2f}")
