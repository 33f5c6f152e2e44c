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


def broadcast_weights_rccl(engine, packed, src=0, group=None):
    """The same broadcast through the C-ABI's RCCL entry points (include/pwg.h
    pwg_rccl_unique_id / pwg_rccl_comm_create / pwg_broadcast_weights), i.e. the path a
    non-Python host uses: rank ``src`` makes the RCCL id, the 128 bytes travel over the existing
    process group, every rank joins a one-shot RCCL communicator on its engine's device and
    receives the image in place on the current stream. Returns ``packed``.

    Failure is collective: every phase ends with an agreement (MIN over the process group of a
    per-rank success flag), so either every rank returns or every rank raises RcclBroadcastError
    and the caller can fall back on all ranks together. Phase 1, before any rank enters RCCL, has
    every rank load librccl and make an id (the src rank's is the one used), so a rank that
    cannot reach RCCL never leaves the others waiting in the communicator's collective init."""
    if not dist.is_available() or not dist.is_initialized():
        return packed
    import ctypes

    from . import _lib

    lib = _lib.load()
    rank, world = dist.get_rank(group), dist.get_world_size(group)

    def agree(ok, what):
        if not all_ranks_ok(ok, group, packed.device):
            raise RcclBroadcastError(f"RCCL weight broadcast: {what} failed on at least one rank")

    buf = ctypes.create_string_buffer(_lib.PWG_RCCL_UNIQUE_ID_BYTES)
    ok = lib.pwg_rccl_unique_id(buf) == _lib.PWG_OK
    agree(ok, "librccl / ncclGetUniqueId")
    obj = [bytes(buf.raw) if rank == src else None]
    dist.broadcast_object_list(obj, src=src, group=group)
    buf = ctypes.create_string_buffer(obj[0], _lib.PWG_RCCL_UNIQUE_ID_BYTES)
    dev = packed.device.index if packed.device.index is not None else torch.cuda.current_device()
    comm = ctypes.c_void_p()
    ok = lib.pwg_rccl_comm_create(world, buf, rank, dev, ctypes.byref(comm)) == _lib.PWG_OK
    try:
        agree(ok, "ncclCommInitRank")
        stream = torch.cuda.current_stream(packed.device)
        ok = lib.pwg_broadcast_weights(engine._h, comm, src, packed.data_ptr(), stream.cuda_stream) == _lib.PWG_OK
        if ok:
            stream.synchronize()
        agree(ok, "pwg_broadcast_weights")
    finally:
        if comm.value:
            lib.pwg_rccl_comm_destroy(comm)
    return packed


class RcclBroadcastError(RuntimeError):
    """The C-ABI RCCL weight broadcast failed on at least one rank (raised on every rank)."""


def all_ranks_ok(ok, group=None, device=None):
    """Collective AND of a per-rank boolean (all_reduce MIN); host tensor on gloo."""
    if not dist.is_available() or not dist.is_initialized():
        return bool(ok)
    on_host = dist.get_backend(group) == "gloo" or device is None or torch.device(device).type != "cuda"
    t = torch.tensor([1 if ok else 0], dtype=torch.int32, device="cpu" if on_host else device)
    dist.all_reduce(t, op=dist.ReduceOp.MIN, group=group)
    return bool(t.item())


def _reduce_device(device):
    """Where a small reduction tensor lives: the host on gloo, else the rank's device."""
    if device is None or dist.get_backend() == "gloo":
        return "cpu"
    return device


def max_over_ranks(value, device=None):
    """Max of a float over all ranks (timing reduction for bench.py)."""
    if not dist.is_available() or not dist.is_initialized():
        return float(value)
    t = torch.tensor([float(value)], dtype=torch.float64, device=_reduce_device(device))
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def sum_over_ranks(value, device=None):
    if not dist.is_available() or not dist.is_initialized():
        return float(value)
    t = torch.tensor([float(value)], dtype=torch.float64, device=_reduce_device(device))
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return float(t.item())


def shard_for_rank(lengths, rank, world):
    """Utterance indices this rank decodes (LPT over frame counts, identical on every rank)."""
    if not 0 <= rank < world:
        raise ValueError(f"rank {rank} outside world of {world}")
    return lpt_partition(lengths, world)[rank]


def decode_sharded(lengths, decode_fn, rank=None, world=None):
    """Decode this rank's share of a fixed utterance list.

    ``decode_fn(indices) -> list of per-utterance outputs`` runs the local batch (on a GPU rank:
    ``Engine.infer`` over the selected mels/noises, one ragged plan). Returns {index: output} for
    this rank's utterances only; no data-path collective is involved."""
    if rank is None or world is None:
        init = dist.is_available() and dist.is_initialized()
        rank = dist.get_rank() if init else 0
        world = dist.get_world_size() if init else 1
    mine = shard_for_rank(lengths, rank, world)
    outs = decode_fn(mine) if mine else []
    if len(outs) != len(mine):
        raise RuntimeError(f"decode_fn returned {len(outs)} outputs for {len(mine)} utterances")
    return dict(zip(mine, outs))


def gather_outputs(local, n_utts, dst=0):
    """Collect every rank's {index: output} on ``dst`` as a list in utterance order (host
    objects, e.g. CPU tensors / arrays). Other ranks get None. Off the timed path: the reference's
    decode writes each utterance to disk from the process that produced it (bin/decode.py:262-266),
    so this exists for callers that want one list."""
    if not dist.is_available() or not dist.is_initialized():
        return [local[i] for i in range(n_utts)]
    world = dist.get_world_size()
    parts = [None] * world if dist.get_rank() == dst else None
    dist.gather_object(local, parts, dst=dst)
    if dist.get_rank() != dst:
        return None
    merged = {}
    for p in parts:
        overlap = merged.keys() & p.keys()
        if overlap:
            raise RuntimeError(f"utterances decoded twice: {sorted(overlap)[:5]}")
        merged.update(p)
    if len(merged) != n_utts:
        raise RuntimeError(f"gathered {len(merged)} of {n_utts} utterances")
    return [merged[i] for i in range(n_utts)]


def long_utterance_ranges(frames, world, halo, hop, causal=False):
    """one very long utterance split over ``world`` ranks in time. Returns one
    (lo, s, e, hi) frame range per rank: the rank computes frames [lo, hi) (its core [s, e) plus
    ``halo`` frames of recomputed context, left only when causal) and keeps the core. Cores are
    ceil(frames / world) frames rounded up to the engine's chunk alignment (streaming.align_frames:
    a chunk that starts off the 32-sample block phase sums in another order), and ``lo`` is rounded
    down to it, so the concatenated cores are BIT-IDENTICAL to one whole-utterance run. Ranks past
    the end get an empty core (s == e)."""
    from .streaming import align_frames

    align = align_frames(hop)
    per = -(-int(frames) // int(world))
    per = -(-per // align) * align
    out = []
    for r in range(int(world)):
        s = min(int(frames), r * per)
        e = min(int(frames), s + per)
        lo = max(0, (s - halo) // align * align)
        hi = e if causal else min(int(frames), e + halo)
        out.append((lo, s, e, hi))
    return out


def decode_long_sharded(engine, mel, noise, rank=None, world=None, halo=None, mean=None, scale=None):
    """One long utterance decoded by every rank together (SURVEY.md sec 8(e) "split time into P
    chunks whose inputs overlap by the receptive halo... no exchange" on the input side): each rank
    runs its core plus recomputed halos (long_utterance_ranges) on its own GPU, then the cores are
    all-gathered (RCCL on the nccl backend: the one data-path collective of this path, 4 B per
    output sample over xGMI) and every rank returns the whole (T, out_channels) waveform,
    bit-identical to ``engine.infer([mel], [noise])``. ``engine`` is an Engine (or anything with its
    ``infer``, ``upsample_factor``, ``config``); mel (T', A) and noise (T,) live on the rank's device
    (every rank holds the whole input, as every rank reads its own input in bin/decode.py)."""
    from .streaming import halo_frames

    init = dist.is_available() and dist.is_initialized()
    if rank is None or world is None:
        rank = dist.get_rank() if init else 0
        world = dist.get_world_size() if init else 1
    H = int(engine.upsample_factor)
    O = int(engine.config.out_channels)
    F = int(mel.shape[0])
    noise = noise.reshape(-1)
    if noise.numel() != F * H:
        raise ValueError("noise must have frames * upsample_factor samples")
    causal = bool(engine.config.use_causal_conv) and int(getattr(engine.config, "interpolate_mode", 0)) != 1
    halo = halo_frames(engine) if halo is None else int(halo)
    ranges = long_utterance_ranges(F, world, halo, H, causal)
    per = max(e - s for _, s, e, _ in ranges)
    lo, s, e, hi = ranges[rank]
    piece = torch.zeros(per * H * O, dtype=torch.float32, device=mel.device)
    if e > s:
        y = engine.infer([mel[lo:hi].contiguous()], [noise[lo * H:hi * H].contiguous()], mean, scale)[0]
        piece[:(e - s) * H * O] = y[(s - lo) * H:(e - lo) * H].reshape(-1)
    if world == 1 or not init:
        parts = [piece]
    elif dist.get_backend() == "gloo":
        host = piece.cpu()
        parts = [torch.empty_like(host) for _ in range(world)]
        dist.all_gather(parts, host)
        parts = [p.to(mel.device) for p in parts]
    else:
        flat = torch.empty(world * piece.numel(), dtype=torch.float32, device=mel.device)
        dist.all_gather_into_tensor(flat, piece)
        parts = list(flat.view(world, -1))
    out = torch.cat([p[:(e_ - s_) * H * O] for p, (_, s_, e_, _) in zip(parts, ranges)])
    return out.view(F * H, O)
