"""B = 1 forwards of one vocoder at one length, for a kernel trace (diagnostic, GPU box).

  rocprofv3 --kernel-trace --output-format csv -d DIR -o run -- python tools/diag/voc_kt.py CFG T [N]

N (default 6) synchronised inference() calls; the trace's last forward is the steady one."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch  # noqa: E402

from parallelwavegan_amd import configs, synthetic  # noqa: E402
from parallelwavegan_amd.hifigan import HiFiGANGenerator  # noqa: E402
from parallelwavegan_amd.melgan import PQMF, MelGANGenerator  # noqa: E402


def main():
    cfg, T = sys.argv[1], int(sys.argv[2])
    n = int(sys.argv[3]) if len(sys.argv) > 3 else 6
    dev = torch.device("cuda", 0)
    cls, p = configs.vocoder_params(cfg)
    m = {"MelGANGenerator": MelGANGenerator, "HiFiGANGenerator": HiFiGANGenerator}[cls](**p)
    m.load_state_dict({k: torch.from_numpy(v) for k, v in synthetic.make_module_state_dict(m, seed=0).items()})
    if cfg in configs.VOCODER_PQMF:
        m.pqmf = PQMF(**configs.VOCODER_PQMF[cfg])
    m = m.to(dev)
    mel = torch.from_numpy(synthetic.make_mel(T, 80, seed=7)).to(dev)
    with torch.no_grad():
        for _ in range(n):
            m.inference(mel)
            torch.cuda.synchronize()


if __name__ == "__main__":
    main()
