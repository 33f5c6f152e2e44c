"""The bench's vocoder latency rows twice in one process, after the batched leg (and, with --exact,
the exact-fp32 leg), to tell one-time first-call costs from per-shape ones (diagnostic, GPU box):
python tools/diag/voc_latency_twice.py hifigan_v1 [--exact]"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

import bench  # noqa: E402
from parallelwavegan_amd import configs, synthetic  # noqa: E402
from parallelwavegan_amd.hifigan import HiFiGANGenerator  # noqa: E402
from parallelwavegan_amd.melgan import PQMF, MelGANGenerator  # noqa: E402

name = sys.argv[1]
dev = torch.device("cuda", 0)
cls, p = configs.vocoder_params(name)
m = {"MelGANGenerator": MelGANGenerator, "HiFiGANGenerator": HiFiGANGenerator}[cls](**p)
m.load_state_dict({k: torch.from_numpy(v) for k, v in synthetic.make_module_state_dict(m, seed=0).items()})
if name in configs.VOCODER_PQMF:
    m.pqmf = PQMF(**configs.VOCODER_PQMF[name])
m = m.eval().to(dev)
eng = m.engine()
with torch.no_grad():
    lengths = synthetic.libritts_lengths(32, seed=3).tolist()
    big = eng.plan(lengths)
    mel = torch.randn(sum(lengths) * 80, device=dev)
    out = torch.empty(big.out_rows * eng.out_channels, device=dev)
    for _ in range(3):
        eng.run(big, mel, out, check=False)
    eng.set_timing(True)
    eng.run(big, mel, out, check=False)
    torch.cuda.synchronize(dev)
    eng.collect_timing()
    eng.set_timing(False)
    if "--exact" in sys.argv:
        fl = bench.program_flops_per_frame(eng.program) * sum(lengths)
        bench.vocoder_exact_fp32_leg(eng, big, mel, out, fl, sum(lengths) * eng.hop, 2)
res = {}
for rep in range(2):
    lat = bench.vocoder_latency_rows(m, dev)
    res[f"pass{rep}"] = {f"B{r['batch']}_T{r['frames']}": (r["first_call_ms"], r["median_ms"]) for r in lat["rows"]}
    res[f"pass{rep}"]["loop_le512"] = lat["decode_loop"]["mean_ms_per_call_le512_frames"]
print(json.dumps({name: res}))
