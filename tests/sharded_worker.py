"""Worker of tests/test_gpu_sharding.py (GPU box; not collected by pytest): one rank of the
multi-GPU decode path on the HIP engine, launched by the test as
``python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 ...``.

Ranks share cuda:0 (the test box has one GPU), so the process group is gloo: rank 0 packs the
generator weights, broadcast_packed_weights ships the image, every rank decodes its LPT shard of
a ragged LibriTTS v1 utterance list with Engine.infer (one ragged plan per rank), and rank 0
gathers the outputs (utterance order) into OUT/sharded.npz with the per-rank shards and loads.
Then both ranks decode ONE long utterance together (sharding.decode_long_sharded: a core each,
recomputed halos, all-gather of the cores) and each saves the whole waveform to OUT/long<rank>.npy."""

import os
import sys

import numpy as np
import torch
import torch.distributed as dist

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

from parallelwavegan_amd import Engine, configs, sharding, synthetic  # noqa: E402

LENGTHS = [143, 17, 600, 88, 1, 250, 311, 45, 90]
LONG = 3001  # frames of the utterance split in time across the ranks (37.5 s at 24 kHz)


def inputs(i, f):
    return synthetic.make_mel(f, 80, seed=500 + i), synthetic.make_noise(f * 300, seed=600 + i)


def main():
    out_dir = sys.argv[1]
    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    params = configs.generator_params("libritts_v1")
    eng = Engine(params, dev)
    if rank == 0:
        packed = torch.from_numpy(eng.pack(synthetic.make_state_dict(params, seed=0))).to(dev)
    else:
        packed = torch.zeros(eng.packed_weight_count, dtype=torch.float32, device=dev)
    sharding.broadcast_packed_weights(packed, src=0)
    eng.set_packed(packed)

    def decode(indices):
        mels, noises = [], []
        for i in indices:
            m, n = inputs(i, LENGTHS[i])
            mels.append(torch.from_numpy(m).to(dev))
            noises.append(torch.from_numpy(n).to(dev))
        return [y.cpu().numpy() for y in eng.infer(mels, noises)]

    local = sharding.decode_sharded(LENGTHS, decode)
    shards = [sharding.shard_for_rank(LENGTHS, r, world) for r in range(world)]
    outs = sharding.gather_outputs(local, len(LENGTHS))
    if rank == 0:
        arrays = {f"y{i}": y for i, y in enumerate(outs)}
        arrays["loads"] = np.array(sharding.shard_loads(LENGTHS, shards))
        arrays["rank0"] = np.array(shards[0])
        np.savez(os.path.join(out_dir, "sharded.npz"), **arrays)
    m, n = inputs(99, LONG)
    y = sharding.decode_long_sharded(eng, torch.from_numpy(m).to(dev), torch.from_numpy(n).to(dev))
    np.save(os.path.join(out_dir, f"long{rank}.npy"), y.cpu().numpy())
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
