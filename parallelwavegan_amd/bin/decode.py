#!/usr/bin/env python3
"""Decode dumped features with the MI355X engine: the ``parallel-wavegan-decode`` CLI
(/root/reference/parallel_wavegan/bin/decode.py:31-268) for the accelerated generator types.

Same arguments for the mel-to-wave case (--dumpdir with ``*-feats.npy`` files, --outdir,
--checkpoint, --config, --normalize-before, --verbose) and the same outputs
(``{outdir}/{utt_id}_gen.wav``, PCM_16, and the mean per-utterance RTF in the log). Differences:
  * utterances are decoded in ragged BATCHES of up to --batch-frames mel frames per engine pass
    (the reference runs one utterance per call), by default sized from the free device memory;
    the logged RTF is per batch wall time / audio;
  * features are read lazily: lengths from the .npy headers, data per batch of the rank's shard;
  * under ``torch.distributed.run`` every rank decodes its LPT share of the utterances on its own
    GPU (sharding.decode_sharded) and writes its own wavs;
  * --scp (kaldiio), hdf5 dumps and --use-f0 are not available in this image: they raise.
"""

import argparse
import logging
import os
import sys
import time

import numpy as np
import torch


def engines_of(model):
    """The HIP engine(s) a drop-in module holds (PWG: one; MelGAN: one per PQMF setting)."""
    if hasattr(model, "_engines"):
        return [e[0] for e in model._engines.values()]
    return [model.engine()]


def batch_cost_model(model, device, frac=0.25, cap_gib=8.0, probe_frames=512, probe_utts=8):
    """Bytes of one engine pass as a function of (mel frames, utterances) and the budget they must
    fit: ``frac`` of the free device memory, at most ``cap_gib``. Per frame: the plan workspace of
    a one-utterance probe, plus the caller's mel input (4 B x input channels) and noise / output
    (4 B per audio sample and output channel, the noise for PWG only). Per utterance: what a probe
    of ``probe_utts`` equal utterances of the same total length adds over the one-utterance probe
    (segment gaps and tile padding). Channel counts and samples per frame come from the model."""
    eng = model.engine()
    if hasattr(model, "aux_channels"):  # ParallelWaveGANGenerator: mel in, noise in, audio out
        in_ch, hop, out_ch, noise = model.aux_channels, model.upsample_factor, model.out_channels, 1
    else:  # MelGAN family: the program's input channels, output rate (PQMF included) and channels
        in_ch, hop, out_ch, noise = eng.program.channels[0], eng.hop, eng.out_channels, 0
    one = eng.plan([probe_frames]).workspace_bytes
    many = eng.plan([probe_frames // probe_utts] * probe_utts).workspace_bytes
    per_frame = one / probe_frames + 4 * in_ch + 4 * hop * (out_ch + noise)
    per_utt = max(0.0, (many - one) / (probe_utts - 1))
    free, _ = torch.cuda.mem_get_info(device)
    budget = min(free * frac, cap_gib * (1 << 30))
    return per_frame, per_utt, budget


def main(argv=None):
    ap = argparse.ArgumentParser(description="Decode dumped features with the MI355X generator engine.")
    ap.add_argument("--scp", default=None, type=str)
    ap.add_argument("--dumpdir", default=None, type=str)
    ap.add_argument("--segments", default=None, type=str)
    ap.add_argument("--outdir", type=str, required=True)
    ap.add_argument("--checkpoint", type=str, required=True)
    ap.add_argument("--config", default=None, type=str)
    ap.add_argument("--normalize-before", default=False, action="store_true")
    ap.add_argument("--verbose", type=int, default=1)
    ap.add_argument("--use-f0", default=False, action="store_true")
    ap.add_argument("--batch-frames", type=int, default=None,
                    help="max mel frames per engine pass (ragged batch); default: sized from free device "
                         "memory (--batch-mem-frac of it, at most --batch-mem-gib)")
    ap.add_argument("--batch-mem-frac", type=float, default=0.25)
    ap.add_argument("--batch-mem-gib", type=float, default=8.0)
    args = ap.parse_args(argv)

    level = logging.DEBUG if args.verbose > 1 else (logging.INFO if args.verbose > 0 else logging.WARN)
    logging.basicConfig(level=level, format="%(asctime)s (%(module)s:%(lineno)d) %(levelname)s: %(message)s")

    from parallelwavegan_amd import sharding
    from parallelwavegan_amd.utils import find_files, load_model, log_rtf, read_config, write_pcm16_wav

    if args.scp is not None or args.segments is not None:
        raise NotImplementedError("--scp/--segments need kaldiio, which is not available; use --dumpdir")
    if args.use_f0:
        raise NotImplementedError("--use-f0 generators are not accelerated")
    if args.dumpdir is None:
        raise ValueError("Please specify either --dumpdir or --feats-scp.")
    os.makedirs(args.outdir, exist_ok=True)
    cfg_path = args.config or os.path.join(os.path.dirname(args.checkpoint), "config.yml")
    config = read_config(cfg_path)
    config.update(vars(args))
    if config.get("format", "npy") != "npy":
        raise NotImplementedError("hdf5 dumps need h5py, which is not available; dump with format: npy")

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = 0
    if world > 1:
        import torch.distributed as dist

        local = int(os.environ.get("LOCAL_RANK", "0"))
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        rank = dist.get_rank()
    if not torch.cuda.is_available():
        raise RuntimeError("the MI355X engine needs a ROCm GPU (no CPU fallback)")
    device = torch.device("cuda", torch.cuda.current_device())

    model = load_model(args.checkpoint, config)
    if args.normalize_before:
        assert hasattr(model, "mean"), "Feature stats are not registered."
        assert hasattr(model, "scale"), "Feature stats are not registered."
    model.remove_weight_norm()
    model = model.eval().to(device)

    files = find_files(args.dumpdir, "*-feats.npy")
    utt_ids = [os.path.basename(f).replace("-feats.npy", "") for f in files]
    # lengths from the .npy headers only (memory-mapped, nothing read); each rank loads the
    # features of its own shard, one batch at a time
    lengths = [int(np.load(f, mmap_mode="r", allow_pickle=False).shape[0]) for f in files]
    logging.info(f"The number of features to be decoded = {len(files)}.")
    sr = config["sampling_rate"]
    if args.batch_frames is None:
        per_frame, per_utt, budget = batch_cost_model(model, device, args.batch_mem_frac, args.batch_mem_gib)
        logging.info(f"batch budget: {budget / 2**30:.2f} GiB, {per_frame:.0f} B per mel frame + {per_utt:.0f} B "
                     f"per utterance")

        def fits(nfr, nutt):
            return nfr * per_frame + nutt * per_utt <= budget
    else:
        def fits(nfr, nutt):
            return nfr <= args.batch_frames

    def decode(idx):
        outs = [None] * len(idx)
        batch, nfr = [], 0
        total_rtf, n = 0.0, 0

        def flush():
            nonlocal batch, nfr, total_rtf, n
            if not batch:
                return
            cs = [torch.from_numpy(np.ascontiguousarray(np.load(files[i], allow_pickle=False), np.float32))
                  for _, i in batch]
            start = time.time()
            with torch.no_grad():
                ys = model.inference_batch(cs, normalize_before=args.normalize_before)
                ys = [y.view(-1).cpu().numpy() for y in ys]
            el = time.time() - start
            audio = sum(len(y) for y in ys) / sr
            total_rtf += el / audio * len(ys)
            n += len(ys)
            for (slot, i), y in zip(batch, ys):
                write_pcm16_wav(os.path.join(config["outdir"], f"{utt_ids[i]}_gen.wav"), y, sr)
                outs[slot] = len(y)
            batch, nfr = [], 0

        for slot, i in enumerate(idx):
            if batch and not fits(nfr + lengths[i], len(batch) + 1):
                flush()
            batch.append((slot, i))
            nfr += lengths[i]
        flush()
        log_rtf(n, total_rtf)
        return outs

    local = sharding.decode_sharded(lengths, decode)
    logging.info(f"rank {rank}: wrote {len(local)} utterances to {config['outdir']}")
    for eng in engines_of(model):
        eng.release_workspace()
    if world > 1:
        import torch.distributed as dist

        dist.barrier()
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
