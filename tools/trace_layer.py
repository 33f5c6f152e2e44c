"""Per-wave timeline of the persistent layer kernel (diagnostic; not part of the engine).

Builds a PWG_TRACE variant of the library (per-wave wall-clock start/end, block count and
s_memtime cycles spent in GEMM 1 / aux+gate / GEMM 2+stores), runs the bench workload once
and prints, per layer: kernel span, wave start/end spread, mean per-block phase cycles, and the
effective shader clock.  Usage (GPU box): python tools/trace_layer.py [--utts 32] [--out FILE]
"""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
VARIANT = os.path.join(REPO, "parallelwavegan_amd", "lib", "variants", "libpwg_trace.so")
os.environ["PWG_LIB_PATH"] = VARIANT
sys.path.insert(0, REPO)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from parallelwavegan_amd import Engine, _lib, configs, synthetic  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--utts", type=int, default=32)
    ap.add_argument("--config", default="libritts_v1")
    ap.add_argument("--out", default=os.path.join(REPO, "gpurun_out", "layer_trace.bin"))
    ap.add_argument("--flags", default="", help="extra hipcc flags for the variant")
    args = ap.parse_args()
    if not (os.environ.get("PWG_NO_BUILD") == "1" and os.path.exists(VARIANT)):
        _lib.build(force=True, extra_flags=["-DPWG_TRACE=1"] + args.flags.split(), out_path=VARIANT)
    os.environ["PWG_TRACE_FILE"] = args.out
    os.makedirs(os.path.dirname(args.out), exist_ok=True)
    params = configs.generator_params(args.config)
    dev = torch.device("cuda", 0)
    eng = Engine(params, dev)
    eng.load_state_dict(synthetic.make_state_dict(params, seed=0))
    lengths = synthetic.libritts_lengths(args.utts, seed=3)
    plan = eng.plan(lengths.tolist())
    A = params["aux_channels"]
    rs = np.random.RandomState(100)
    mel = torch.from_numpy(rs.standard_normal(int(lengths.sum()) * A).astype(np.float32)).to(dev)
    noise = torch.from_numpy(rs.standard_normal(plan.total_samples).astype(np.float32)).to(dev)
    out = torch.empty(plan.total_samples * params["out_channels"], dtype=torch.float32, device=dev)
    for _ in range(3):
        eng.run(plan, mel, noise, out)
    torch.cuda.synchronize()
    raw = np.fromfile(args.out, dtype=np.int64)
    L, nwg, wpw, nf = raw[:4]
    rec = raw[4:].reshape(L, nwg * wpw, nf).astype(np.float64)
    print(f"layers {L}, workgroups {nwg}, waves/wg {wpw}")
    xcd = (np.arange(nwg * wpw) // wpw) % 8
    for l in range(L):
        r = rec[l]
        live = r[:, 2] > 0
        s0, e0 = r[:, 0], r[:, 1]
        t0 = s0.min()
        span = (e0.max() - t0) / 100.0  # 100 MHz -> us
        dur = (e0 - s0)[live] / 100.0
        clk = ((r[:, 7] - r[:, 6]) / ((e0 - s0) / 100e6))[live].mean() / 1e9
        n = r[live, 2]
        g1, gt, g2 = (r[live, 3] / n).mean(), (r[live, 4] / n).mean(), (r[live, 5] / n).mean()
        endx = [((e0[xcd == x] - t0) / 100.0).max() for x in range(8)]
        if l in (0, 1, 9, 15, L - 1) or l == L - 2:
            print(f"layer {l:2d}: span {span:7.1f} us | wave start spread {(s0.max() - t0) / 100:5.1f} us | "
                  f"wave dur min/mean/max {dur.min():7.1f}/{dur.mean():7.1f}/{dur.max():7.1f} us | "
                  f"blocks/wave {n.min():.0f}-{n.max():.0f} | cyc/block g1 {g1:7.0f} gate {gt:6.0f} g2 {g2:6.0f} "
                  f"| clk {clk:.2f} GHz | xcd end {min(endx):.0f}-{max(endx):.0f} us")


if __name__ == "__main__":
    main()
