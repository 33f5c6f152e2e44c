#!/usr/bin/env python3
"""Decode dumped features with the MI355X engine: the ``parallel-wavegan-decode`` CLI
(/root/reference/parallel_wavegan/bin/decode.py:31-268) for the accelerated generator types.

Same arguments for the mel-to-wave case (--dumpdir with ``*-feats.npy`` files, --outdir,
--checkpoint, --config, --normalize-before, --verbose) and the same outputs
(``{outdir}/{utt_id}_gen.wav``, PCM_16, and the mean per-utterance RTF in the log). Differences:
  * utterances are decoded in ragged BATCHES of up to --batch-frames mel frames per engine pass
    (the reference runs one utterance per call); the logged RTF is per batch wall time / audio;
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
    ap.add_argument("--batch-frames", type=int, default=200000,
                    help="max mel frames per engine pass (ragged batch)")
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
    feats = [np.load(f, allow_pickle=False) for f in files]
    lengths = [int(f.shape[0]) for f in feats]
    logging.info(f"The number of features to be decoded = {len(files)}.")
    sr = config["sampling_rate"]

    def decode(idx):
        outs = [None] * len(idx)
        batch, nfr = [], 0
        total_rtf, n = 0.0, 0

        def flush():
            nonlocal batch, nfr, total_rtf, n
            if not batch:
                return
            cs = [torch.from_numpy(np.ascontiguousarray(feats[i], np.float32)) for _, i in batch]
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
            if batch and nfr + lengths[i] > args.batch_frames:
                flush()
            batch.append((slot, i))
            nfr += lengths[i]
        flush()
        log_rtf(n, total_rtf)
        return outs

    local = sharding.decode_sharded(lengths, decode)
    logging.info(f"rank {rank}: wrote {len(local)} utterances to {config['outdir']}")
    if world > 1:
        import torch.distributed as dist

        dist.barrier()
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
