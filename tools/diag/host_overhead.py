"""Host-side cost of one B = 1 vocoder call (diagnostic, GPU box).

  python tools/diag/host_overhead.py CFG [T]

Median over 50 calls (us): the full inference() with its synchronisation; eng.run(check=False)
enqueue time alone (host returns before the GPU finishes) and with a sync; the range-status read
(pwg_cnet_run_status) after a synced run; the device span of one eager run (timing mode 2)."""
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


def med(fn, n=50):
    ts = []
    for _ in range(n):
        t = fn()
        ts.append(t)
    return round(float(np.median(ts)) * 1e6, 1)


def main():
    cfg = sys.argv[1]
    T = int(sys.argv[2]) if len(sys.argv) > 2 else 64
    dev = torch.device("cuda", 0)
    cls, p = configs.vocoder_params(cfg)
    m = {"MelGANGenerator": MelGANGenerator, "HiFiGANGenerator": HiFiGANGenerator}[cls](**p)
    m.load_state_dict({k: torch.from_numpy(v) for k, v in synthetic.make_module_state_dict(m, seed=0).items()})
    if cfg in configs.VOCODER_PQMF:
        m.pqmf = PQMF(**configs.VOCODER_PQMF[cfg])
    m = m.to(dev)
    eng = m.engine()
    mel = torch.from_numpy(synthetic.make_mel(T, 80, seed=7)).to(dev)
    res = {"config": cfg, "frames": T, "graphs_used": None}
    with torch.no_grad():
        for _ in range(5):
            m.inference(mel)
        torch.cuda.synchronize()

        def full():
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            m.inference(mel)
            torch.cuda.synchronize()
            return time.perf_counter() - t0
        res["inference_us"] = med(full)
        plan = eng.plan([T])
        flat = mel.reshape(-1).contiguous()
        out = torch.empty(plan.out_rows * eng.out_channels, device=dev)
        res["graphs_used"] = bool(eng._graph_ok(plan, None, torch.cuda.current_stream()))

        def enq():
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            eng.run(plan, flat, out, check=False)
            t1 = time.perf_counter()
            torch.cuda.synchronize()
            return t1 - t0
        res["run_enqueue_us"] = med(enq)

        def run_sync():
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            eng.run(plan, flat, out, check=False)
            torch.cuda.synchronize()
            return time.perf_counter() - t0
        res["run_nocheck_synced_us"] = med(run_sync)

        def run_check():
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            eng.run(plan, flat, out, check=True)
            torch.cuda.synchronize()
            return time.perf_counter() - t0
        res["run_check_synced_us"] = med(run_check)

        def status():
            eng.run(plan, flat, out, check=False)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            eng.run_status(plan)
            return time.perf_counter() - t0
        res["status_read_us"] = med(status)
        eng.set_timing(2)
        eng.collect_timing()
        m.inference(mel)
        torch.cuda.synchronize()
        res["eager_span_us"] = round(eng.timing_span() * 1e3, 1)
        eng.collect_timing()
        eng.set_timing(False)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
