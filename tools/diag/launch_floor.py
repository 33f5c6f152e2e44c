"""Launch floor and graph replay of the B = 1 vocoder path (diagnostic, GPU box).

Prints one JSON line: the per-kernel cost of back-to-back tiny kernels (eager and hipGraph
replay), and the vocoders' T' = 64 / B = 1 forward eager vs replayed from a captured graph.
Usage: python tools/diag/launch_floor.py [OUT.json]"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from parallelwavegan_amd import configs, synthetic  # noqa: E402
from parallelwavegan_amd.hifigan import HiFiGANGenerator  # noqa: E402
from parallelwavegan_amd.melgan import PQMF, MelGANGenerator  # noqa: E402


def timed(fn, reps, s):
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ts = []
    for _ in range(reps):
        a.record(s)
        fn()
        b.record(s)
        b.synchronize()
        ts.append(a.elapsed_time(b))
    return float(np.median(ts)), float(np.min(ts))


def main():
    out_path = sys.argv[1] if len(sys.argv) > 1 else None
    dev = torch.device("cuda", 0)
    res = {}
    s = torch.cuda.Stream(dev)
    x = torch.zeros(1, device=dev)
    N = 200
    with torch.cuda.stream(s):
        def tiny():
            for _ in range(N):
                x.add_(1.0)
        tiny()
        torch.cuda.synchronize()
        med, mn = timed(tiny, 10, s)
        res["tiny_eager_us"] = med * 1e3 / N
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            tiny()
        g.replay()
        torch.cuda.synchronize()
        med, mn = timed(g.replay, 20, s)
        res["tiny_graph_us"] = med * 1e3 / N

    for name in ("hifigan_v1", "mb_melgan_v2"):
        cls, p = configs.vocoder_params(name)
        m = {"MelGANGenerator": MelGANGenerator, "HiFiGANGenerator": HiFiGANGenerator}[cls](**p)
        m.load_state_dict({k: torch.from_numpy(v) for k, v in synthetic.make_module_state_dict(m, seed=0).items()})
        if name in configs.VOCODER_PQMF:
            m.pqmf = PQMF(**configs.VOCODER_PQMF[name])
        m = m.to(dev)
        eng = m.engine()
        for T in (64, 512):
            plan = eng.plan([T])
            torch.manual_seed(0)
            mel = torch.randn(T * 80, device=dev)
            out = torch.empty(plan.out_rows * eng.out_channels, device=dev)
            with torch.cuda.stream(s):
                eng.run(plan, mel, out, stream=s)  # checked once (allocates the stream's workspace)
                torch.cuda.synchronize()
                ref = out.clone()

                def fwd():
                    eng.run(plan, mel, out, stream=s, check=False)
                for _ in range(3):
                    fwd()
                torch.cuda.synchronize()
                e_med, e_min = timed(fwd, 30, s)
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g, stream=s):
                    fwd()
                out.zero_()
                g.replay()
                torch.cuda.synchronize()
                same = bool(torch.equal(out, ref))
                g_med, g_min = timed(g.replay, 30, s)
                # host cost of one eager enqueue
                t0 = time.perf_counter()
                for _ in range(20):
                    fwd()
                host_us = (time.perf_counter() - t0) / 20 * 1e6
                torch.cuda.synchronize()
            res[f"{name}_T{T}"] = {"eager_ms": e_med, "eager_min_ms": e_min, "graph_ms": g_med, "graph_min_ms": g_min,
                                   "graph_bitwise_equal": same, "host_enqueue_us": host_us}
            print(name, T, res[f"{name}_T{T}"], flush=True)
    line = json.dumps(res)
    print(line)
    if out_path:
        with open(out_path, "w") as f:
            f.write(line + "\n")


if __name__ == "__main__":
    main()
