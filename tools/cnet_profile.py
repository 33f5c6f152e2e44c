"""Per-op time and MFMA rate of a MelGAN-family program on the GPU (diagnostic).
Usage: python tools/cnet_profile.py mb_melgan_v2 [--utts 32] [--steps 3] [--frames 64 --batch 1]
(--frames: B equal-length utterances of that many frames instead of the bench's ragged list)"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from parallelwavegan_amd import cnet, configs, synthetic  # noqa: E402
from parallelwavegan_amd.hifigan import HiFiGANGenerator  # noqa: E402
from parallelwavegan_amd.melgan import PQMF, MelGANGenerator  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("config")
    ap.add_argument("--utts", type=int, default=32)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--nofuse", action="store_true")
    ap.add_argument("--pair-steps", type=int, default=None)
    ap.add_argument("--frames", type=int, default=None)
    ap.add_argument("--batch", type=int, default=1)
    ap.add_argument("--mstack", type=int, default=None, help="PWG_CNET_OPT_MSTACK (fused stack chains) 0/1/2")
    ap.add_argument("--presplit", type=int, default=None, help="PWG_CNET_OPT_PRESPLIT 0/1")
    ap.add_argument("--rstack", type=int, default=None, help="PWG_CNET_OPT_RSTACK 0/1/2")
    ap.add_argument("--nocheck", action="store_true", help="no range check / exact-fp32 rerun (diagnostic builds)")
    ap.add_argument("--bitwise-rstack", action="store_true",
                    help="first compare one forward with PWG_CNET_OPT_RSTACK 0 and 1 bit for bit")
    ap.add_argument("--opt", action="append", default=[],
                    help="NAME=VALUE: eng.set_NAME(VALUE) before planning (e.g. xt_dma=2, xcd_order=0)")
    ap.add_argument("--dump", default=None, help="save the first forward's output (.npy) for a bitwise A/B")
    a = ap.parse_args()
    cls, p = configs.vocoder_params(a.config)
    m = {"MelGANGenerator": MelGANGenerator, "HiFiGANGenerator": HiFiGANGenerator}[cls](**p)
    m.load_state_dict({k: torch.from_numpy(v) for k, v in synthetic.make_module_state_dict(m, seed=0).items()})
    if a.config in configs.VOCODER_PQMF:
        m.pqmf = PQMF(**configs.VOCODER_PQMF[a.config])
    dev = torch.device("cuda", 0)
    m = m.to(dev)
    eng = m.engine()
    eng.set_fuse_pairs(not a.nofuse)
    if a.mstack is not None:
        eng.set_mstack(a.mstack)
    if a.presplit is not None:
        eng.set_presplit(a.presplit)
    if a.rstack is not None:
        eng.set_rstack(a.rstack)
    if a.pair_steps:
        eng.set_pair_steps(a.pair_steps)
    for o in a.opt:
        k, v = o.split("=")
        getattr(eng, "set_" + k)(int(v))
    P = eng.program
    lengths = (np.full(a.batch, a.frames) if a.frames else synthetic.libritts_lengths(a.utts, seed=3))
    frames = int(lengths.sum())
    plan = eng.plan(lengths.tolist())
    torch.manual_seed(0)
    mel = torch.randn(frames * 80, device=dev)
    out = torch.empty(plan.out_rows * eng.out_channels, device=dev)
    if a.bitwise_rstack:
        eng.set_rstack(0)
        eng.run(plan, mel, out)
        ref = out.clone()
        eng.set_rstack(2)
        out.fill_(float("nan"))
        eng.run(plan, mel, out)
        torch.cuda.synchronize()
        print(f"bitwise rstack 0 vs 2: {'equal' if torch.equal(ref, out) else 'DIFFER'}", flush=True)
        eng.set_rstack(1)
        out.fill_(float("nan"))
        eng.run(plan, mel, out)
        torch.cuda.synchronize()
        same = bool(torch.equal(ref, out))
        print(f"bitwise rstack 0 vs 1: {'equal' if same else 'DIFFER'} max|d| {(ref - out).abs().max().item():.3e}"
              f" finite {bool(torch.isfinite(out).all())}", flush=True)
    eng.run(plan, mel, out, check=not a.nocheck)
    torch.cuda.synchronize()
    if a.dump:
        np.save(a.dump, out.cpu().numpy())
    eng.set_timing(True)
    eng.collect_timing()
    for _ in range(a.steps):
        eng.run(plan, mel, out, check=not a.nocheck)
    t = eng.collect_timing()
    tot = 0.0
    rows = []
    for i, (name, ms, n) in enumerate(t):
        op = P.ops[i]
        r = P.rate[op["dst"]]
        if op["kind"] == cnet.CONV:
            k = sum(s["channels"] * s["taps"] for s in op["srcs"])
        elif op["kind"] == cnet.CONVT:
            k = op["srcs"][0]["channels"] * 2
        else:
            k = op["padding"]
        fl = 2.0 * op["out_channels"] * k * r * frames
        ms /= a.steps
        tot += ms
        if n == 0 and rows:  # fused into the previous op's launch (pwg_cnet_pair_kernel)
            prev = rows[-1]
            rows[-1] = (prev[0] + "+", prev[1], prev[2] + k, r, prev[4], prev[5] + fl)
            continue
        rows.append((name, op["out_channels"], k, r, ms, fl))
    for name, M, K, r, ms, fl in rows:
        print(f"{name:28s} M {M:4d} K {K:5d} rate {r:4d}  {ms:7.3f} ms  {fl / (ms * 1e-3) / 1e12:6.1f} TF")
    print(f"total {tot:.3f} ms")


if __name__ == "__main__":
    main()
