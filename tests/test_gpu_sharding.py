"""The multi-GPU decode path (BASELINE config 5) executed on the HIP engine.

test_sharded_decode_two_ranks: two fresh child processes (torch.distributed.run, started by the
test as a subprocess) share cuda:0 over gloo, broadcast rank 0's packed weights, decode their LPT
shards of a ragged LibriTTS v1 list and gather on rank 0; the result must be bit-identical to one
single-process ragged decode of the whole list (utterances are independent and the engine's
segment padding isolates them); and one long utterance split in time over the
two ranks (sharding.decode_long_sharded) must equal its unsplit decode bit for bit.

test_rccl_broadcast_capi: the C-ABI RCCL path (pwg_rccl_unique_id / pwg_rccl_comm_create /
pwg_broadcast_weights) in a one-rank process group: the image arrives intact and decodes as the
locally packed one. (Two RCCL ranks cannot share one GPU; the 8-GPU driver run covers N > 1.)"""

import os
import socket
import subprocess
import sys

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_sharded_decode_two_ranks(built_lib, cuda_device, tmp_path):
    sys.path.insert(0, HERE)
    import sharded_worker as w

    from parallelwavegan_amd import Engine, configs, sharding, synthetic

    env = dict(os.environ, PWG_NO_BUILD="1", OMP_NUM_THREADS="4")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}",
           os.path.join(HERE, "sharded_worker.py"), str(tmp_path)]
    res = subprocess.run(cmd, env=env, cwd=REPO, capture_output=True, text=True, timeout=100)
    assert res.returncode == 0, res.stdout[-3000:] + res.stderr[-3000:]
    got = np.load(os.path.join(tmp_path, "sharded.npz"))

    shards = sharding.lpt_partition(w.LENGTHS, 2)
    assert list(got["rank0"]) == shards[0]
    assert list(got["loads"]) == sharding.shard_loads(w.LENGTHS, shards)
    params = configs.generator_params("libritts_v1")
    eng = Engine(params, cuda_device)
    eng.load_state_dict(synthetic.make_state_dict(params, seed=0))
    mels, noises = [], []
    for i, f in enumerate(w.LENGTHS):
        m, n = w.inputs(i, f)
        mels.append(torch.from_numpy(m).to(cuda_device))
        noises.append(torch.from_numpy(n).to(cuda_device))
    ref = [y.cpu().numpy() for y in eng.infer(mels, noises)]
    for i, y in enumerate(ref):
        np.testing.assert_array_equal(got[f"y{i}"], y)
    # one long utterance split in time over the two ranks: every rank ends
    # with the whole waveform, bit-identical to one unsplit decode
    m, n = w.inputs(99, w.LONG)
    ref_long = eng.infer([torch.from_numpy(m).to(cuda_device)], [torch.from_numpy(n).to(cuda_device)])[0].cpu().numpy()
    for r in range(2):
        np.testing.assert_array_equal(np.load(os.path.join(tmp_path, f"long{r}.npy")), ref_long)


def test_rccl_broadcast_capi(built_lib, cuda_device):
    import torch.distributed as dist

    from parallelwavegan_amd import Engine, configs, sharding, synthetic

    params = configs.generator_params("ljspeech_v1")
    eng = Engine(params, cuda_device)
    packed = torch.from_numpy(eng.pack(synthetic.make_state_dict(params, seed=3))).to(cuda_device)
    ref = packed.clone()
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ["MASTER_PORT"] = str(_free_port())
    dist.init_process_group("gloo", rank=0, world_size=1)
    try:
        sharding.broadcast_weights_rccl(eng, packed, src=0)
    finally:
        dist.destroy_process_group()
    assert torch.equal(packed, ref)
    eng.set_packed(packed)
    mel = torch.from_numpy(synthetic.make_mel(9, 80, seed=1)).to(cuda_device)
    noise = torch.from_numpy(synthetic.make_noise(9 * 256, seed=2)).to(cuda_device)
    y = eng.infer([mel], [noise])[0]
    eng.set_packed(ref)
    assert torch.equal(y, eng.infer([mel], [noise])[0])


def test_bench_self_launches_ranks(built_lib, cuda_device):
    """`bench.py --gpus 2` as ONE command starts its two ranks itself (a torch.distributed.run
    child); on this 1-GPU box they share cuda:0 over gloo. The line reports 2 ranks, 1 device and
    both ranks' seconds."""
    import json

    env = dict(os.environ, PWG_NO_BUILD="1", PWG_BENCH_BACKEND="gloo", OMP_NUM_THREADS="4")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        env.pop(k, None)
    cmd = [sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", "--steps", "1", "--warmup", "1",
           "--utts", "8", "--no-latency", "--cpu-seconds", "0", "--pmc", "off"]
    res = subprocess.run(cmd, env=env, cwd=REPO, capture_output=True, text=True, timeout=110)
    assert res.returncode == 0, res.stdout[-3000:] + res.stderr[-3000:]
    lines = [ln for ln in res.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, res.stdout
    line = json.loads(lines[0])
    assert line["ranks"] == 2 and line["n_gpus"] == 1
    assert len(line["rank_seconds"]) == 2 and all(t > 0 for t in line["rank_seconds"])
    assert line["config"]["global_batch"] == 16
    assert line["value"] > 0
