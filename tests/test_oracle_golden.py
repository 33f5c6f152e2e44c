"""Pin the CPU oracle (oracle/) to golden vectors produced by the reference itself
(tests/golden/make_golden.py). CPU only."""

import numpy as np
import pytest

from conftest import golden_names, golden_params, golden_state, load_golden
from oracle import pwg_numpy
from oracle.pwg_torch_cpu import TorchCPUGenerator

# fp64 oracle vs the reference's fp32 output: measured fp32-vs-fp64 floor of the reference is
# ~2e-6; 2e-5 leaves margin while staying 5x under the 1e-4 product bar.
ORACLE_ATOL = 2e-5


def _run_oracle(g, params, sd):
    if g["meta"]["mode"] == "inference":
        return pwg_numpy.inference(g["mel"], g["noise"], sd, params, g.get("mean"), g.get("scale"))
    return pwg_numpy.forward(g["z"], g["c"], sd, params)


@pytest.mark.parametrize("name", golden_names())
def test_numpy_oracle_matches_reference(name):
    g = load_golden(name)
    params = golden_params(g["meta"])
    sd = golden_state(g["meta"], params)
    y = _run_oracle(g, params, sd)
    assert y.shape == g["y"].shape
    np.testing.assert_allclose(y, g["y"], rtol=0, atol=ORACLE_ATOL)


@pytest.mark.parametrize("name", golden_names())
def test_torch_cpu_restatement_matches_reference(name):
    """The CPU-baseline restatement runs the reference's aten op sequence: it must agree."""
    g = load_golden(name)
    if "mean" in g:
        pytest.skip("normalize_before is exercised by the numpy oracle")
    params = golden_params(g["meta"])
    sd = golden_state(g["meta"], params)
    gen = TorchCPUGenerator(sd, params)
    if g["meta"]["mode"] == "inference":
        y = gen.inference(g["mel"], g["noise"]).numpy()
    else:
        import torch

        y = gen.forward(torch.from_numpy(g["z"]), torch.from_numpy(g["c"])).numpy()
    np.testing.assert_allclose(y, g["y"], rtol=0, atol=1e-5)


def test_upsampler_intermediate_matches_reference():
    g = load_golden("libritts_T4")
    params = golden_params(g["meta"])
    sd = pwg_numpy.fold_weight_norm(golden_state(g["meta"], params))
    cp = pwg_numpy.pad_inference_features(g["mel"], params)
    cup = pwg_numpy.upsample_net(cp, sd, params)
    np.testing.assert_allclose(cup, g["cup"], rtol=0, atol=1e-5)


def test_golden_set_covers_edge_cases():
    names = set(golden_names())
    # single frame, causal, weight norm, normalize_before, batched forward, bias=False,
    # UpsampleNetwork, non-uniform 24 kHz scales
    for n in ("ljspeech_T1", "reftest_causal_T16", "yesno_wn_T24", "yesno_norm_T10",
              "ljspeech_fwd_B2_T5", "reftest_nobias_T8", "reftest_upnet_T12", "libritts_T7"):
        assert n in names


# ------------------------------------------------------------------ MelGAN family (sec 8(f))
from conftest import vocoder_golden_names, vocoder_holder  # noqa: E402


@pytest.mark.parametrize("name", vocoder_golden_names())
def test_vocoder_oracle_matches_reference_golden(name):
    """oracle/melgan_numpy.py (float64) against the reference's fp32 outputs."""
    from oracle import melgan_numpy

    g = load_golden(name)
    meta = g["meta"]
    m, params, folded = vocoder_holder(meta)
    is_melgan = type(m).__name__ == "MelGANGenerator"
    if meta["options"].get("forward"):
        fwd = melgan_numpy.melgan_forward if is_melgan else melgan_numpy.hifigan_forward
        y = np.stack([fwd(c, folded, params) for c in g["c"]])
    else:
        mean, scale = g.get("mean"), g.get("scale")
        if is_melgan:
            syn = m.pqmf.synthesis_taps() if m.pqmf is not None else None
            y = melgan_numpy.melgan_inference(g["mel"], folded, params, syn, mean, scale)
        else:
            y = melgan_numpy.hifigan_inference(g["mel"], folded, params, mean, scale)
    assert y.shape == g["y"].shape
    err = np.abs(y - g["y"]).max()
    assert err < 2e-5, f"{name}: max|d| = {err:.3e}"


def test_pqmf_filters_match_scipy_kaiser():
    """The restated Kaiser window equals scipy.signal.windows.kaiser (layers/pqmf.py:11,44)."""
    import scipy.signal.windows

    from parallelwavegan_amd.melgan import _kaiser

    for m, beta in ((63, 9.0), (31, 5.0), (64, 8.6)):
        np.testing.assert_allclose(_kaiser(m, beta), scipy.signal.windows.kaiser(m, beta), rtol=0, atol=1e-13)


@pytest.mark.parametrize("name", vocoder_golden_names())
def test_vocoder_torch_cpu_restatement_matches_golden(name):
    """oracle/melgan_torch_cpu.py (the vocoder CPU baseline) reproduces the reference outputs."""
    from oracle.melgan_torch_cpu import TorchCPUVocoder

    g = load_golden(name)
    meta = g["meta"]
    if meta["options"].get("forward") or meta["options"].get("normalize"):
        pytest.skip("inference() without normalization only")
    m, params, folded = vocoder_holder(meta)
    syn = m.pqmf.synthesis_taps() if getattr(m, "pqmf", None) is not None else None
    y = TorchCPUVocoder(type(m).__name__, folded, params, syn).inference(g["mel"]).numpy()
    err = np.abs(y - g["y"]).max()
    assert err < 1e-5, f"{name}: max|d| = {err:.3e}"
