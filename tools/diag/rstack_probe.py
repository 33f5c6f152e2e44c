"""Timeline of the batched ResidualStack kernel (pwg_rstack.hip), one workgroup's wave 0 (diagnostic,
GPU box; the probe is compiled in and armed at run time, no variant build).

  PWG_NO_BUILD=1 python tools/diag/rstack_probe.py CFG CS [WG]

Runs the bench's ragged batch (32 LibriTTS lengths) through CFG (mb_melgan_v2 / melgan_v1) with the
probe armed for stacks of CS 16-channel blocks; the last such launch leaves its stamps. Prints the mean
shader cycles between consecutive phase stamps per step kind, and per tile."""
import ctypes
import json
import os
import sys
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from parallelwavegan_amd import _lib, configs, synthetic  # noqa: E402
from parallelwavegan_amd.melgan import PQMF, MelGANGenerator  # noqa: E402

N = 4096
NAMES = {1: "tile", 2: "tile.waited", 3: "tile.barrier", 4: "conv", 5: "conv.waited", 6: "conv.barrier",
         7: "conv.issued", 8: "conv.mfma", 9: "mm", 10: "mm.waited", 11: "mm.barrier", 12: "mm.issued",
         13: "mm.pass", 14: "mm.end"}


def main():
    cfg, cs = sys.argv[1], int(sys.argv[2])
    wg = int(sys.argv[3]) if len(sys.argv) > 3 else 0
    dev = torch.device("cuda", 0)
    _, p = configs.vocoder_params(cfg)
    m = MelGANGenerator(**p)
    m.load_state_dict({k: torch.from_numpy(v) for k, v in synthetic.make_module_state_dict(m, seed=0).items()})
    if cfg in configs.VOCODER_PQMF:
        m.pqmf = PQMF(**configs.VOCODER_PQMF[cfg])
    m = m.to(dev)
    eng = m.engine()
    lengths = synthetic.libritts_lengths(32, seed=3)
    plan = eng.plan(lengths.tolist())
    mel = torch.randn(int(lengths.sum()) * 80, device=dev)
    out = torch.empty(plan.out_rows * eng.out_channels, device=dev)
    lib = _lib.load()
    f = lib.pwg_rstack_debug_probe
    f.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_int]
    eng.run(plan, mel, out)
    torch.cuda.synchronize()
    assert f(cs, wg, None, 0) == 0
    eng.run(plan, mel, out)
    torch.cuda.synchronize()
    buf = (ctypes.c_ulonglong * N)()
    assert f(0, 0, ctypes.cast(buf, ctypes.c_void_p), N) == 0
    a = np.frombuffer(buf, dtype=np.uint64)
    hdr = int(a[0])
    npr, nt, kcs = hdr & 0xFFFF, (hdr >> 16) & 0xFFFF, hdr >> 32
    tags = (a[1:npr] >> np.uint64(56)).astype(int)
    t = (a[1:npr] & np.uint64((1 << 56) - 1)).astype(np.int64)
    seg = defaultdict(list)
    for i in range(1, len(t)):
        seg[(NAMES.get(tags[i - 1]), NAMES.get(tags[i]))].append(int(t[i] - t[i - 1]))
    tile_starts = t[tags == 1]
    res = {"cfg": cfg, "cs": int(kcs), "wg": wg, "tiles": int(nt), "stamps": int(npr),
           "total_cycles": int(t[-1] - t[0]),
           "cycles_per_tile": float(np.diff(tile_starts).mean()) if len(tile_starts) > 1 else None,
           "segments": {f"{k[0]} -> {k[1]}": {"n": len(v), "mean": round(float(np.mean(v)), 1),
                                              "max": int(np.max(v))} for k, v in seg.items()}}
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
