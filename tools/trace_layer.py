"""Per-wave timeline of the split16 residual-layer launches (diagnostic; not part of the engine).

With PWG_TRACE_FILE set, pwg_run records per wave [start, staged, first block done, end, blocks,
shader clock at start / end, XCC id] for every layer launch and dumps them after the run. This
script runs one plan a few times and prints, per layer: launch span, staging time (start ->
barrier), time to the first finished block, wave end spread, blocks per computing wave and the
effective shader clock. Usage (GPU box): python tools/trace_layer.py [--config ljspeech_v1]
[--frames 64] [--utts 1] [--out FILE]   (--utts > 1: that many LibriTTS bench lengths)
"""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from parallelwavegan_amd import Engine, configs, synthetic  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="ljspeech_v1")
    ap.add_argument("--frames", type=int, default=64)
    ap.add_argument("--utts", type=int, default=1)
    ap.add_argument("--out", default=os.path.join(REPO, "gpurun_out", "layer_trace.bin"))
    ap.add_argument("--layers", default="0,1,9,15,28,29")
    args = ap.parse_args()
    os.makedirs(os.path.dirname(args.out), exist_ok=True)
    params = configs.generator_params(args.config)
    dev = torch.device("cuda", 0)
    eng = Engine(params, dev)
    eng.load_state_dict(synthetic.make_state_dict(params, seed=0))
    lengths = [args.frames] if args.utts == 1 else synthetic.libritts_lengths(args.utts, seed=3).tolist()
    plan = eng.plan(lengths)
    rs = np.random.RandomState(100)
    mel = torch.from_numpy(rs.standard_normal(sum(lengths) * params["aux_channels"]).astype(np.float32)).to(dev)
    noise = torch.from_numpy(rs.standard_normal(plan.total_samples).astype(np.float32)).to(dev)
    out = torch.empty(plan.total_samples * params["out_channels"], dtype=torch.float32, device=dev)
    for _ in range(3):
        eng.run(plan, mel, noise, out, check=False)
    torch.cuda.synchronize()
    os.environ["PWG_TRACE_FILE"] = args.out
    eng.run(plan, mel, noise, out, check=False)
    torch.cuda.synchronize()
    del os.environ["PWG_TRACE_FILE"]
    raw = np.fromfile(args.out, dtype=np.int64)
    L, nwg, wpw, nf = (int(v) for v in raw[:4])
    rec = raw[4:].reshape(L, nwg * wpw, nf).astype(np.float64)
    print(f"{args.config} {lengths if len(lengths) < 4 else f'{len(lengths)} utts'}: {L} layers, {nwg} workgroups x "
          f"{wpw} waves, {plan.total_samples} samples")
    k0 = rec[:, :, 0].min()
    for l in [int(x) for x in args.layers.split(",") if int(x) < L]:
        r = rec[l]
        st, sg, fb, en, nb = r[:, 0], r[:, 1], r[:, 2], r[:, 3], r[:, 4]
        comp = nb > 0
        t0 = st.min()
        us = lambda v: v / 100.0  # noqa: E731  (100 MHz real-time counter)
        clk = ((r[:, 6] - r[:, 5]) / (us(en - st) * 1e-6))[comp].mean() / 1e9
        print(f"layer {l:2d}: at {us(t0 - k0):8.1f} us | span {us(en.max() - t0):6.1f} | start spread {us(st.max() - t0):5.1f} | "
              f"staging {us((sg - st)[comp]).mean():5.1f} (max {us((sg - st).max()):5.1f}) | first block "
              f"{us((fb - sg)[comp]).mean():5.1f} | compute end {us(en[comp].min() - t0):6.1f}-{us(en[comp].max() - t0):6.1f} | "
              f"blocks/wave {nb[comp].min():.0f}-{nb[comp].max():.0f} on {comp.sum():.0f} waves | clk {clk:.2f} GHz")
    gaps = [us_ for us_ in ((rec[l + 1, :, 0].min() - rec[l, :, 3].max()) / 100.0 for l in range(L - 1))]
    print(f"launch gaps (first start of l+1 - last end of l): mean {np.mean(gaps):.2f} us, min {min(gaps):.2f}, max {max(gaps):.2f}")


if __name__ == "__main__":
    main()
