"""B=1 drop-in calls of LJ v1 at T' = 64 and 512 (diagnostic; run under rocprofv3 --kernel-trace):
20 calls each after warm-up, so the kernel trace shows per-layer durations and the gaps between
launches. Usage (GPU box): rocprofv3 --kernel-trace --output-format csv -d DIR -- python
tools/diag/lat_trace.py"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from parallelwavegan_amd import ParallelWaveGANGenerator, configs, synthetic  # noqa: E402

params = configs.generator_params("ljspeech_v1")
m = ParallelWaveGANGenerator(**params)
m.remove_weight_norm()
m.load_state_dict({k: torch.from_numpy(v) for k, v in synthetic.make_state_dict(params, seed=0).items()})
dev = torch.device("cuda", 0)
m = m.eval().to(dev)
frames = [int(x) for x in (sys.argv[1:] or ["64", "512"])]
with torch.no_grad():
    for F in frames:
        mel = torch.from_numpy(synthetic.make_mel(F, 80, seed=30)).to(dev)
        noise = torch.from_numpy(synthetic.make_noise(F * 256, seed=60)).to(dev)
        for _ in range(25):
            m.inference(mel, noise)
        torch.cuda.synchronize()
