"""Utterance-parallel multi-GPU execution: one process per GPU, torch.distributed over RCCL.

The reference decodes one utterance at a time on one GPU (bin/decode.py:236-268;
egs/*/voc1/run.sh:147 forces n_gpus=1 for decoding), so this layer is new. Utterances are
independent, so the data path has NO collective: each rank runs its own shard. The one
collective is a broadcast of the packed fp32 weight image (5.3 MB for PWG v1) from rank 0
over xGMI at start-up.
"""

import heapq

import numpy as np
import torch
import torch.distributed as dist


def lpt_partition(lengths, n_shards):
    """Longest-processing-time greedy: assign utterances (by length, descending) to the
    currently lightest shard. Returns a list of index lists, each sorted ascending.
    Deterministic (ties broken by shard index, then utterance index)."""
    lengths = np.asarray(lengths, dtype=np.int64)
    if n_shards < 1:
        raise ValueError("n_shards must be >= 1")
    order = sorted(range(len(lengths)), key=lambda i: (-int(lengths[i]), i))
    heap = [(0, s) for s in range(n_shards)]
    shards = [[] for _ in range(n_shards)]
    for i in order:
        load, s = heapq.heappop(heap)
        shards[s].append(i)
        heapq.heappush(heap, (load + int(lengths[i]), s))
    return [sorted(s) for s in shards]


def shard_loads(lengths, shards):
    lengths = np.asarray(lengths, dtype=np.int64)
    return [int(lengths[s].sum()) if len(s) else 0 for s in shards]


def broadcast_packed_weights(packed, src=0, group=None):
    """Broadcast the packed weight image (a contiguous float32 tensor on this rank's device)
    from ``src`` to every rank, in place. With the nccl backend this is one RCCL broadcast over
    xGMI; with gloo (CPU tests) a host broadcast."""
    if not dist.is_available() or not dist.is_initialized():
        return packed
    if not packed.is_contiguous():
        raise ValueError("packed weights must be contiguous")
    dist.broadcast(packed, src=src, group=group)
    return packed


def max_over_ranks(value, device=None):
    """Max of a float over all ranks (timing reduction for bench.py)."""
    if not dist.is_available() or not dist.is_initialized():
        return float(value)
    t = torch.tensor([float(value)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def sum_over_ranks(value, device=None):
    if not dist.is_available() or not dist.is_initialized():
        return float(value)
    t = torch.tensor([float(value)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return float(t.item())
