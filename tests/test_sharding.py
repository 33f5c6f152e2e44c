"""Utterance sharding (parallelwavegan_amd/sharding.py) on CPU: LPT balance, and a world-size-2
gloo rehearsal of the multi-GPU path: weight-image broadcast from rank 0, per-rank decode of the
LPT shard (with the NumPy oracle standing in for the GPU engine, as test infrastructure only),
gather on rank 0 equal to the unsharded decode, max/sum timing reductions."""

import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from parallelwavegan_amd import sharding


def test_lpt_partition_covers_and_balances():
    rs = np.random.RandomState(3)
    lengths = rs.randint(80, 1200, size=512)
    for world in (1, 2, 3, 4, 8):
        shards = sharding.lpt_partition(lengths, world)
        flat = sorted(i for s in shards for i in s)
        assert flat == list(range(len(lengths)))
        loads = sharding.shard_loads(lengths, shards)
        # LPT bound: max - min <= longest job
        assert max(loads) - min(loads) <= lengths.max()
        assert max(loads) <= lengths.sum() / world * 4 / 3 + lengths.max()
    assert sharding.lpt_partition([5, 5], 2) == [[0], [1]]
    assert sharding.lpt_partition([], 3) == [[], [], []]
    with pytest.raises(ValueError):
        sharding.lpt_partition([1], 0)


def test_shard_for_rank_is_disjoint():
    lengths = [100, 7, 300, 300, 1, 50, 49]
    parts = [sharding.shard_for_rank(lengths, r, 3) for r in range(3)]
    assert sorted(sum(parts, [])) == list(range(len(lengths)))
    with pytest.raises(ValueError):
        sharding.shard_for_rank(lengths, 3, 3)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, result_dir):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from oracle import pwg_numpy
        from parallelwavegan_amd import HostHandle, configs, synthetic

        params = configs.generator_params("yesno_debug")
        host = HostHandle(params)
        # rank 0 packs, everyone receives the same image
        if rank == 0:
            sd = synthetic.make_state_dict(params, seed=0)
            packed = torch.from_numpy(host.pack(sd))
        else:
            packed = torch.zeros(host.packed_weight_count, dtype=torch.float32)
        sharding.broadcast_packed_weights(packed, src=0)
        own = host.pack(synthetic.make_state_dict(params, seed=0))
        assert np.array_equal(packed.numpy(), own)

        lengths = [3, 1, 5, 2, 4]
        sd = synthetic.make_state_dict(params, seed=0)
        H = host.upsample_factor
        mels = [synthetic.make_mel(f, 80, seed=10 + i) for i, f in enumerate(lengths)]
        noises = [synthetic.make_noise(f * H, seed=20 + i) for i, f in enumerate(lengths)]

        def decode(idx):
            return [pwg_numpy.inference(mels[i], noises[i], sd, params).astype(np.float32) for i in idx]

        local = sharding.decode_sharded(lengths, decode)
        assert set(local) == set(sharding.shard_for_rank(lengths, rank, world))
        gathered = sharding.gather_outputs(local, len(lengths))
        tmax = sharding.max_over_ranks(float(rank + 1))
        tsum = sharding.sum_over_ranks(float(rank + 1))
        # collective agreement of the RCCL broadcast's phases: one failing rank fails all
        assert sharding.all_ranks_ok(True)
        assert not sharding.all_ranks_ok(rank != 1)
        if rank == 0:
            ref = decode(range(len(lengths)))
            for a, b in zip(gathered, ref):
                np.testing.assert_array_equal(a, b)
            assert tmax == world and tsum == world * (world + 1) / 2
            open(os.path.join(result_dir, "ok"), "w").write("ok")
        else:
            assert gathered is None
        dist.barrier()
    finally:
        dist.destroy_process_group()


def test_world2_gloo_broadcast_decode_gather(tmp_path, built_lib):
    world = 2
    mp.spawn(_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    assert (tmp_path / "ok").exists()


def test_long_utterance_ranges_partition_and_align():
    """Cores of one long utterance partition [0, F) in rank order, chunk starts sit on the
    engine's alignment (hop 300: 8 frames), halos cover at least ``halo`` frames where the
    utterance allows, causal chunks have no right halo; more ranks than cores leave empty ranks."""
    for F, world, hop, causal in ((1000, 2, 300, False), (1000, 8, 300, True), (9, 4, 256, False),
                                  (5, 8, 300, False), (60000, 8, 256, False)):
        halo = 14
        rng = sharding.long_utterance_ranges(F, world, halo, hop, causal)
        assert len(rng) == world
        align = 32 // np.gcd(hop, 32)
        pos = 0
        for lo, s, e, hi in rng:
            assert s == pos and e >= s
            pos = e
            assert lo % align == 0 and lo <= max(0, s - halo)
            assert hi == (e if causal else min(F, e + halo))
        assert pos == F


def _long_worker(rank, world, port, result_dir):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from oracle import pwg_numpy  # test infrastructure: stands in for the GPU engine
        from parallelwavegan_amd import HostHandle, configs, synthetic

        params = configs.generator_params("yesno_debug")
        host = HostHandle(params)
        sd = synthetic.make_state_dict(params, seed=0)

        class OracleEngine:
            config = host.config
            receptive_field_size = host.receptive_field_size
            upsample_factor = host.upsample_factor

            @staticmethod
            def infer(mels, noises, mean=None, scale=None):
                return [torch.from_numpy(pwg_numpy.inference(m.numpy(), z.numpy(), sd, params).astype(np.float32))
                        for m, z in zip(mels, noises)]

        F, H = 37, host.upsample_factor
        mel = torch.from_numpy(synthetic.make_mel(F, 80, seed=5))
        noise = torch.from_numpy(synthetic.make_noise(F * H, seed=6)).reshape(-1)
        y = sharding.decode_long_sharded(OracleEngine, mel, noise)
        ref = OracleEngine.infer([mel], [noise])[0]
        assert y.shape == ref.shape
        np.testing.assert_allclose(y.numpy(), ref.numpy(), rtol=0, atol=1e-6)
        open(os.path.join(result_dir, f"ok{rank}"), "w").write("ok")
        dist.barrier()
    finally:
        dist.destroy_process_group()


def test_world2_gloo_long_utterance_split(tmp_path, built_lib):
    """decode_long_sharded on two gloo ranks (the NumPy oracle standing in for each rank's GPU
    engine): each rank computes its core with recomputed halos, the cores are all-gathered, and
    every rank holds the whole waveform, equal to the unsplit decode."""
    world = 2
    mp.spawn(_long_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    assert (tmp_path / "ok0").exists() and (tmp_path / "ok1").exists()
