"""Checkpoint / config / stats ingestion for the drop-in generators.

``load_model`` mirrors parallel_wavegan.utils.load_model
(/root/reference/parallel_wavegan/utils/utils.py:294-360): the generator class comes from
``config["generator_type"]``, the weights from ``checkpoint["model"]["generator"]``, the stats from
``stats.npy`` next to the checkpoint, and a PQMF is attached for multi-band generators (with the
<= 0.4.2 compatibility defaults). Differences, by design:
  * the checkpoint is read with ``torch.load(weights_only=True)`` (tensors only, nothing executed);
  * ``config.yml`` is read with ``yaml.SafeLoader``;
  * ``stats.h5`` / ``format: hdf5`` need h5py, which this image lacks: they raise ImportError.
"""

import fnmatch
import logging
import os

import numpy as np
import torch
import yaml

GENERATORS = ("ParallelWaveGANGenerator", "MelGANGenerator", "HiFiGANGenerator")


def generator_class(name):
    from .hifigan import HiFiGANGenerator
    from .melgan import MelGANGenerator
    from .models import ParallelWaveGANGenerator

    table = {"ParallelWaveGANGenerator": ParallelWaveGANGenerator, "MelGANGenerator": MelGANGenerator,
             "HiFiGANGenerator": HiFiGANGenerator}
    if name not in table:
        raise NotImplementedError(f"generator_type {name!r} is not accelerated (supported: {', '.join(GENERATORS)})")
    return table[name]


def _version_tuple(v):
    out = []
    for part in str(v).split("."):
        digits = "".join(ch for ch in part if ch.isdigit())
        out.append(int(digits) if digits else 0)
    return tuple(out)


def read_config(path):
    with open(path) as f:
        return yaml.load(f, Loader=yaml.SafeLoader)


def load_model(checkpoint, config=None, stats=None):
    """utils/utils.py:294-360 for the accelerated generator types. Returns the module on the CPU
    (call ``.to('cuda')``, as bin/decode.py does)."""
    if config is None:
        config = read_config(os.path.join(os.path.dirname(checkpoint), "config.yml"))
    generator_type = config.get("generator_type", "ParallelWaveGANGenerator")
    cls = generator_class(generator_type)
    # workaround for the reference's typo #295 (utils.py:322-326)
    params = {k.replace("upsample_kernal_sizes", "upsample_kernel_sizes"): v
              for k, v in config["generator_params"].items()}
    model = cls(**params)
    state = torch.load(checkpoint, map_location="cpu", weights_only=True)
    model.load_state_dict(state["model"]["generator"])
    if stats is None:
        ext = "h5" if config.get("format", "npy") == "hdf5" else "npy"
        cand = os.path.join(os.path.dirname(checkpoint), f"stats.{ext}")
        if os.path.exists(cand):
            stats = cand
    if stats is not None:
        model.register_stats(stats)
    if config["generator_params"].get("out_channels", 1) > 1:
        from .melgan import PQMF

        pqmf_params = {}
        if _version_tuple(config.get("version", "0.1.0")) <= (0, 4, 2):
            pqmf_params.update(taps=62, cutoff_ratio=0.15, beta=9.0)  # utils.py:349-353
        model.pqmf = PQMF(subbands=config["generator_params"]["out_channels"],
                          **config.get("pqmf_params", pqmf_params))
    return model


def find_files(root_dir, query="*-feats.npy"):
    """Recursive fnmatch search, like utils/utils.py:61-80, sorted."""
    files = []
    for root, _, names in os.walk(root_dir, followlinks=True):
        for n in fnmatch.filter(names, query):
            files.append(os.path.join(root, n))
    return sorted(files)


def write_pcm16_wav(path, y, sampling_rate):
    """PCM_16 mono wav (what bin/decode.py writes with soundfile, absent here): float samples in
    [-1, 1] scaled by 32767 with clipping, little-endian."""
    import wave

    y = np.asarray(y, dtype=np.float64).reshape(-1)
    pcm = np.clip(np.round(y * 32767.0), -32768, 32767).astype("<i2")
    with wave.open(path, "wb") as w:
        w.setnchannels(1)
        w.setsampwidth(2)
        w.setframerate(int(sampling_rate))
        w.writeframes(pcm.tobytes())


def read_pcm16_wav(path):
    import wave

    with wave.open(path, "rb") as w:
        n = w.getnframes()
        data = np.frombuffer(w.readframes(n), dtype="<i2")
        return data.astype(np.float32) / 32767.0, w.getframerate()


def log_rtf(n, total_rtf):
    logging.info(f"Finished generation of {n} utterances (RTF = {total_rtf / max(n, 1):.03f}).")
