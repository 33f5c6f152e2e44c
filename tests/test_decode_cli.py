"""Checkpoint/config/stats ingestion (utils.load_model, mirrors reference utils/utils.py:294-360)
and the decode CLI (bin/decode.py). CPU tests build and load; the GPU test decodes a dump dir."""

import os

import numpy as np
import pytest
import torch
import yaml

from parallelwavegan_amd import configs, synthetic
from parallelwavegan_amd.utils import load_model, read_pcm16_wav, write_pcm16_wav


def _make_ckpt(tmp, name, version="0.5.4", stats=True):
    if name in configs.GENERATOR_PARAMS:
        gtype, params = "ParallelWaveGANGenerator", configs.generator_params(name)
    else:
        gtype, params = configs.vocoder_params(name)
    from parallelwavegan_amd.utils import generator_class

    m = generator_class(gtype)(**params)
    if gtype == "ParallelWaveGANGenerator":
        sd = synthetic.make_state_dict(params, seed=4, weight_norm=True)
    else:
        sd = synthetic.make_module_state_dict(m, seed=4)
    state = {k: torch.from_numpy(v) for k, v in sd.items()}
    torch.save({"model": {"generator": state}, "steps": 10}, os.path.join(tmp, "checkpoint-10steps.pkl"))
    cfg = dict(generator_type=gtype, generator_params=params, sampling_rate=16000, format="npy", version=version)
    with open(os.path.join(tmp, "config.yml"), "w") as f:
        yaml.safe_dump(cfg, f)
    A = params.get("aux_channels", params.get("in_channels", 80))
    if stats:
        rs = np.random.RandomState(0)
        np.save(os.path.join(tmp, "stats.npy"), np.stack([rs.standard_normal(A), rs.uniform(0.5, 2, A)]).astype(np.float32))
    return os.path.join(tmp, "checkpoint-10steps.pkl"), state, A


@pytest.mark.parametrize("name", ["reference_test", "mb_melgan_test", "hifigan_noadd_test"])
def test_load_model_round_trip(name, tmp_path):
    ckpt, state, A = _make_ckpt(str(tmp_path), name)
    m = load_model(ckpt)
    got = m.state_dict()
    for k, v in state.items():
        assert torch.equal(got[k], v), k
    assert m.mean.shape == (A,) and m.scale.shape == (A,)
    if name == "mb_melgan_test":
        assert m.pqmf is not None and m.pqmf.subbands == 4


def test_load_model_pqmf_version_defaults(tmp_path):
    ckpt, _, _ = _make_ckpt(str(tmp_path), "mb_melgan_test", version="0.4.2", stats=False)
    from parallelwavegan_amd.melgan import pqmf_filters

    m = load_model(ckpt)
    _, syn = pqmf_filters(4, 62, 0.15, 9.0)  # utils.py:349-353 compatibility values
    np.testing.assert_allclose(m.pqmf.synthesis_taps(), syn.astype(np.float32))
    assert not hasattr(m, "mean")


def test_unsupported_generator_type(tmp_path):
    ckpt, _, _ = _make_ckpt(str(tmp_path), "reference_test")
    cfg = yaml.safe_load(open(os.path.join(str(tmp_path), "config.yml")))
    cfg["generator_type"] = "StyleMelGANGenerator"
    with pytest.raises(NotImplementedError):
        load_model(ckpt, cfg)


def test_pcm16_wav_round_trip(tmp_path):
    y = np.linspace(-1.2, 1.2, 1001).astype(np.float32)
    p = str(tmp_path / "a.wav")
    write_pcm16_wav(p, y, 22050)
    z, sr = read_pcm16_wav(p)
    assert sr == 22050 and z.shape == y.shape
    np.testing.assert_allclose(z, np.clip(y, -1, 1), atol=1.0 / 32767)


@pytest.mark.gpu
@pytest.mark.parametrize("batch", ["20", None], ids=["batch20", "auto"])
@pytest.mark.parametrize("name", ["reference_test", "mb_melgan_test", "hifigan_noadd_test"])
def test_decode_cli_end_to_end(name, batch, tmp_path, built_lib, cuda_device):
    from parallelwavegan_amd.bin import decode

    ckpt, state, A = _make_ckpt(str(tmp_path), name)
    dump = tmp_path / "dump"
    dump.mkdir()
    lengths = {"utt_a": 9, "utt_b": 23, "utt_c": 5}
    for i, (u, f) in enumerate(lengths.items()):
        np.save(dump / f"{u}-feats.npy", synthetic.make_mel(f, A, seed=50 + i))
    out = tmp_path / "wav"
    torch.manual_seed(0)
    argv = ["--dumpdir", str(dump), "--outdir", str(out), "--checkpoint", ckpt, "--verbose", "0"]
    if batch is not None:
        argv += ["--batch-frames", batch]  # else sized from free device memory
    assert decode.main(argv) == 0
    m = load_model(ckpt)
    m.remove_weight_norm()
    m = m.eval().to(cuda_device)
    hop = m.upsample_factor * (m.pqmf.subbands if getattr(m, "pqmf", None) is not None else 1)
    for i, (u, f) in enumerate(lengths.items()):
        z, sr = read_pcm16_wav(str(out / f"{u}_gen.wav"))
        assert sr == 16000 and z.shape == (f * hop,)
        if name != "reference_test":  # PWG draws random noise per utterance; the others are deterministic
            with torch.no_grad():
                y = m.inference(synthetic.make_mel(f, A, seed=50 + i)).view(-1).cpu().numpy()
            np.testing.assert_allclose(z, np.clip(y, -1, 1), atol=1.5 / 32767)
