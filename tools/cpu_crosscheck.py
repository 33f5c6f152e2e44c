"""Dev-container cross-check of bench.py's CPU baseline: the torch-CPU
restatement (oracle/pwg_torch_cpu.py, the "port" bench.py times on the GPU box, where the
reference is absent) against the REFERENCE generator itself, imported read-only with the
SURVEY.md sec 8(c) shim, on the same cores, inputs and weights. Warm-up 1, best of 3, B=1
through inference(c, x) like bin/decode.py. Runs only where /root/reference exists.

    PYTHONDONTWRITEBYTECODE=1 python tools/cpu_crosscheck.py [--threads 8] > profiles/<round>/cpu_crosscheck.json
"""

import argparse
import json
import os
import subprocess
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests", "golden"))

from make_golden import build_reference, import_reference  # noqa: E402

from oracle.pwg_torch_cpu import TorchCPUGenerator  # noqa: E402
from parallelwavegan_amd import configs, synthetic  # noqa: E402


def best_of(fn, n=3):
    fn()  # warm-up
    ts = []
    for _ in range(n):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    return min(ts)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--threads", type=int, default=os.cpu_count())
    ap.add_argument("--frames", type=int, default=400)
    args = ap.parse_args()
    torch.set_num_threads(args.threads)
    cls = import_reference()
    model_name = subprocess.run(["lscpu"], capture_output=True, text=True).stdout
    model_name = next((ln.split(":", 1)[1].strip() for ln in model_name.splitlines() if ln.startswith("Model name")), "?")
    rows = []
    for cfg in ("ljspeech_v1", "libritts_v1"):
        params = configs.generator_params(cfg)
        sd = synthetic.make_state_dict(params, seed=0)
        ref = build_reference(cls, configs.generator_params(cfg), sd, False)
        port = TorchCPUGenerator(sd, params)
        H = int(np.prod(params["upsample_params"]["upsample_scales"]))
        mel = synthetic.make_mel(args.frames, 80, seed=1)
        noise = synthetic.make_noise(args.frames * H, seed=2)
        with torch.no_grad():
            y_ref = ref.inference(torch.from_numpy(mel), torch.from_numpy(noise)).numpy()
            y_port = port.inference(mel, noise).numpy()
            t_ref = best_of(lambda: ref.inference(torch.from_numpy(mel), torch.from_numpy(noise)))
            t_port = best_of(lambda: port.inference(mel, noise))
        n = args.frames * H
        rows.append({
            "config": cfg, "frames": args.frames, "samples": n,
            "reference_samples_per_s": round(n / t_ref, 1), "port_samples_per_s": round(n / t_port, 1),
            "port_over_reference": round(t_ref / t_port, 4),
            "max_abs_diff": float(np.abs(y_ref - y_port).max()),
        })
    print(json.dumps({"threads": args.threads, "os_cpu_count": os.cpu_count(), "cpu_model": model_name,
                      "torch": torch.__version__, "method": "warm-up 1, best of 3, B=1 inference(c, x)",
                      "rows": rows}, indent=1))


if __name__ == "__main__":
    main()
