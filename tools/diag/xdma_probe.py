"""Timeline of the DMA-ring kernel's workgroup 0 per launch (diagnostic, GPU box, probe build).

  python -c "from parallelwavegan_amd import _lib; _lib.build(extra_flags=['-DPWG_XDMA_PROBE'],
             out_path='parallelwavegan_amd/lib/variants/libpwg_probe.so')"        (here, CPU)
  PWG_NO_BUILD=1 PWG_LIB_PATH=parallelwavegan_amd/lib/variants/libpwg_probe.so \\
      python tools/diag/xdma_probe.py CFG T                                        (GPU box)

Per narrow launch of one B = 1 forward (program phase order): the kernel shape, shader cycles
from start to the ring's first wait, the first wait, step 0's conversion, then per step the mean
cycles of issue / wait+barrier / MFMAs / conversion+barrier, and the epilogue."""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from parallelwavegan_amd import _lib, configs, synthetic  # noqa: E402
from parallelwavegan_amd.hifigan import HiFiGANGenerator  # noqa: E402
from parallelwavegan_amd.melgan import PQMF, MelGANGenerator  # noqa: E402

SLOTS, N = 128, 96


def main():
    cfg, T = sys.argv[1], int(sys.argv[2])
    dev = torch.device("cuda", 0)
    cls, p = configs.vocoder_params(cfg)
    m = {"MelGANGenerator": MelGANGenerator, "HiFiGANGenerator": HiFiGANGenerator}[cls](**p)
    m.load_state_dict({k: torch.from_numpy(v) for k, v in synthetic.make_module_state_dict(m, seed=0).items()})
    if cfg in configs.VOCODER_PQMF:
        m.pqmf = PQMF(**configs.VOCODER_PQMF[cfg])
    m = m.to(dev)
    eng = m.engine()
    plan = eng.plan([T])
    mel = torch.randn(T * 80, device=dev)
    out = torch.empty(plan.out_rows * eng.out_channels, device=dev)
    for _ in range(3):
        eng.run(plan, mel, out, check=False)
    torch.cuda.synchronize()
    lib = _lib.load()
    buf = (ctypes.c_ulonglong * (SLOTS * N))()
    _lib.check(lib.pwg_cnet_debug_probe(buf, SLOTS * N))
    a = np.frombuffer(buf, dtype=np.uint64).reshape(SLOTS, N).astype(np.int64)
    names = eng.program.ops
    for slot in range(SLOTS):
        hdr = int(a[slot, 0])
        np_ = hdr & 0xFFFF
        if np_ == 0:
            continue
        K, MT, NWV, ns, P = (hdr >> 16) & 0xFF, (hdr >> 24) & 0xFF, (hdr >> 32) & 0xFF, (hdr >> 40) & 0xFFFF, hdr >> 56
        t = a[slot, 1:1 + np_]
        t = t - t[0]
        d = np.diff(t)
        head = d[:3]  # issue prologue, first wait, convert 0
        steps = d[3:3 + 4 * ns]
        per = steps[:4 * (len(steps) // 4)].reshape(-1, 4).mean(axis=0) if len(steps) >= 4 else np.zeros(4)
        tail = d[3 + 4 * ns:]
        if K == 1:  # per step: wait + barrier, issue, MFMAs (in-register split), -
            cols = f"per step wait {per[0]:6.0f} issue {per[1]:6.0f} mma {per[2]:6.0f}"
        else:
            cols = f"per step issue {per[0]:6.0f} wait {per[1]:6.0f} mma {per[2]:6.0f} conv {per[3]:6.0f}"
        print(f"phase {slot:3d} K{K:<2d} MT{MT} W{NWV} steps {ns:3d} P{P}  total {t[-1]:7d} cyc  "
              f"prologue issue {head[0]:5d} wait {head[1]:6d} conv0 {head[2]:5d} | {cols} | "
              f"epilogue {int(tail.sum()) if len(tail) else 0:6d}", flush=True)
    print("ops:", len(names))


if __name__ == "__main__":
    main()
