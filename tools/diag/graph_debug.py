"""Diagnostic: replay a captured pwg_graph and compare with Engine.run (raw output, range flag).
Usage: python tools/diag/graph_debug.py SEQ   (SEQ: letters c=capture, r=Engine.run, g=replay+compare)"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from parallelwavegan_amd import Engine, GraphedRun, configs, synthetic  # noqa: E402

dev = torch.device("cuda", 0)
params = configs.generator_params("libritts_v1")
eng = Engine(params, dev)
eng.load_state_dict(synthetic.make_state_dict(params, seed=5))
frames = [37, 5, 120]
plan = eng.plan(frames)
rs = np.random.RandomState(1)
mel = torch.from_numpy(rs.standard_normal(sum(frames) * 80).astype(np.float32)).to(dev)
noise = torch.from_numpy(rs.standard_normal(plan.total_samples).astype(np.float32)).to(dev)
ref = torch.empty(plan.total_samples, dtype=torch.float32, device=dev)
lib = eng._lib
g = None
out = []
for step in sys.argv[1]:
    if step == "c":
        g = GraphedRun(eng, plan)
    elif step == "n":  # fresh inputs allocated now
        rs = np.random.RandomState(len(out) + 7)
        mel = torch.from_numpy(rs.standard_normal(sum(frames) * 80).astype(np.float32)).to(dev)
        noise = torch.from_numpy(rs.standard_normal(plan.total_samples).astype(np.float32)).to(dev)
        ref = torch.empty(plan.total_samples, dtype=torch.float32, device=dev)
    elif step == "r":
        eng.run(plan, mel, noise, ref)
    elif step == "g":
        got = g(mel, noise, check=False).clone()
        rc = lib.pwg_run_status(plan._p, g.ws.data_ptr(), torch.cuda.current_stream().cuda_stream)
        chk = torch.empty_like(ref)
        eng.run(plan, mel, noise, chk, check=False)
        d = (got - chk).abs()
        out.append(f"g: rc {rc} eq {torch.equal(got, chk)} max|d| {float(d.max()):.3g} "
                   f"bad {int((d > 0).sum())} first {int(torch.nonzero(d > 0)[0]) if (d > 0).any() else -1}")
print(sys.argv[1], " | ".join(out))
