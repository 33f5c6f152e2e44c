"""Timeline of the fused stack-chain kernel's workgroup 0, wave 0 (diagnostic, GPU box, probe build).

  python -c "from parallelwavegan_amd import _lib; _lib.build(extra_flags=['-DPWG_MSTACK_PROBE'],
             out_path='parallelwavegan_amd/lib/probe/libpwg_probe.so')"          (here, CPU)
  PWG_NO_BUILD=1 PWG_LIB_PATH=parallelwavegan_amd/lib/probe/libpwg_probe.so \\
      python tools/diag/mstack_probe.py CFG T MODE                                 (GPU box)

Runs one B = 1 forward with PWG_CNET_OPT_MSTACK = MODE (the LAST chain launch leaves its stamps) and
prints the prologue, then per step the mean shader cycles of: the wait for the step's fragments,
the barrier, and the step's work (issue + operands + MFMAs) -- and the epilogue."""
import ctypes
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from parallelwavegan_amd import _lib, configs, synthetic  # noqa: E402
from parallelwavegan_amd.melgan import PQMF, MelGANGenerator  # noqa: E402

N = 512


def main():
    cfg, T, mode = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
    dev = torch.device("cuda", 0)
    _, p = configs.vocoder_params(cfg)
    m = MelGANGenerator(**p)
    m.load_state_dict({k: torch.from_numpy(v) for k, v in synthetic.make_module_state_dict(m, seed=0).items()})
    if cfg in configs.VOCODER_PQMF:
        m.pqmf = PQMF(**configs.VOCODER_PQMF[cfg])
    m = m.to(dev)
    eng = m.engine()
    eng.set_mstack(mode)
    mel = torch.from_numpy(synthetic.make_mel(T, 80, seed=1)).to(dev)
    with torch.no_grad():
        for _ in range(3):
            m.inference(mel)
    torch.cuda.synchronize()
    buf = (ctypes.c_ulonglong * N)()
    rc = _lib.load().pwg_mstack_debug_probe(buf, N)
    a = np.frombuffer(buf, dtype=np.uint64).astype(np.int64)
    hdr = int(a[0])
    npr, nsteps, cs = hdr & 0xFFFF, (hdr >> 16) & 0xFFFF, hdr >> 32
    t = a[1:npr]
    # stamps: start, then per step (end of previous work, after wait, after barrier), end
    steps = []
    for k in range(nsteps):
        b = 1 + 3 * k
        work_prev = t[b] - t[b - 1]
        steps.append((int(t[b + 1] - t[b]), int(t[b + 2] - t[b + 1]), int(work_prev)))
    w = np.array(steps)
    res = {"rc": rc, "cs": int(cs), "steps": int(nsteps), "stamps": int(npr),
           "total_cycles": int(t[-1] - t[0]), "prologue_to_first_wait": int(steps[0][2]),
           "mean_wait": float(w[1:, 0].mean()), "mean_barrier": float(w[1:, 1].mean()),
           "mean_work": float(w[1:, 2].mean()), "epilogue": int(t[-1] - t[-2]),
           "per_step": steps}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
