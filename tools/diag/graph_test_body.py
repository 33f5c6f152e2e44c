import numpy as np, torch, sys, os
sys.path.insert(0, os.getcwd())
from parallelwavegan_amd import Engine, GraphedRun, configs, synthetic
cuda_device = torch.device("cuda:0")
params = configs.generator_params("libritts_v1")
eng = Engine(params, cuda_device)
eng.load_state_dict(synthetic.make_state_dict(params, seed=5))
frames = [37, 5, 120]
plan = eng.plan(frames)
g = GraphedRun(eng, plan)
for seed in (1, 2):
    rs = np.random.RandomState(seed)
    mel = torch.from_numpy(rs.standard_normal(sum(frames) * 80).astype(np.float32)).to(cuda_device)
    noise = torch.from_numpy(rs.standard_normal(plan.total_samples).astype(np.float32)).to(cuda_device)
    ref = torch.empty(plan.total_samples, dtype=torch.float32, device=cuda_device)
    eng.run(plan, mel, noise, ref)
    got = g(mel, noise, check=False).clone()
    rc = eng._lib.pwg_run_status(plan._p, g.ws.data_ptr(), torch.cuda.current_stream().cuda_stream)
    d = (got - ref).abs()
    print("seed", seed, "rc", rc, "eq", torch.equal(got, ref), "max", float(d.max()), "bad", int((d > 0).sum()), "nonfinite", int((~torch.isfinite(got)).sum()))
