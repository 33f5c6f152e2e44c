"""Host-side logic that needs no GPU: the drop-in modules' weight-change tracker
(engine.WeightTracker) and bench.py's self-launch of N ranks (launch_command / launch_ranks)."""

import os
import subprocess
import sys

import torch

from parallelwavegan_amd.engine import WeightTracker

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_weight_tracker_sees_inplace_updates_and_storage_swaps():
    m = torch.nn.Sequential(torch.nn.Conv1d(4, 4, 3), torch.nn.Conv1d(4, 2, 1))
    t = WeightTracker()
    assert t.changed(m)
    t.mark_packed()
    assert not t.changed(m)
    with torch.no_grad():
        m[0].weight.add_(1.0)  # in-place through the parameter: _version bumps
    assert t.changed(m)
    t.mark_packed()
    m[1].bias.data = torch.zeros(2)  # storage swap: _version unchanged, data_ptr changes
    assert t.changed(m)
    t.mark_packed()
    assert not t.changed(m)
    m.load_state_dict({k: v + 1 for k, v in m.state_dict().items()})  # copy_ into the parameters
    assert t.changed(m)
    t.mark_packed()
    m[0].weight = torch.nn.Parameter(torch.ones_like(m[0].weight))  # re-registration
    assert t.changed(m)
    t.mark_packed()
    t.invalidate()
    assert t.changed(m)


def test_bench_launch_command_form():
    sys.path.insert(0, REPO)
    import bench

    cmd = bench.launch_command(4, ["--gpus", "4", "--steps", "3"], 29555)
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert "--nproc-per-node=4" in cmd and "--master-addr=127.0.0.1" in cmd and "--master-port=29555" in cmd
    assert cmd[-4:] == ["--gpus", "4", "--steps", "3"]
    assert cmd[-5] == os.path.join(REPO, "bench.py")


def test_bench_refuses_more_ranks_than_gpus_on_nccl():
    """`bench.py --gpus 2` as one process on the nccl backend with fewer than 2 visible GPUs
    (none here) exits non-zero before touching a GPU instead of timing one process."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK",
                                                            "PWG_BENCH_BACKEND")}
    env["PWG_NO_BUILD"] = "1"
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", "--steps", "1"],
                       env=env, capture_output=True, text=True, timeout=120)
    assert r.returncode == 2, r.stdout + r.stderr
    assert "one process per GPU needs 2" in r.stderr
    assert r.stdout.strip() == ""
