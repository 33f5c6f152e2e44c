"""Chunked and causal-streaming inference (parallelwavegan_amd/streaming.py) reproduce the
whole-utterance engine output BIT FOR BIT (SURVEY.md sec 8(e) long-utterance split, sec 8(f) row 3)."""

import numpy as np
import pytest
import torch

from parallelwavegan_amd import streaming


def test_chunk_ranges_cover_exactly():
    for causal in (False, True):
        r = streaming.chunk_ranges(1000, 64, 17, causal)
        assert r[0][1] == 0 and r[-1][2] == 1000
        for (lo, s, e, hi), nxt in zip(r, r[1:] + [None]):
            assert lo == max(0, s - 17) and (hi == e if causal else hi == min(1000, e + 17))
            if nxt:
                assert nxt[1] == e
    # aligned starts: lo a multiple of align, at least halo frames of context
    for lo, s, e, hi in streaming.chunk_ranges(1000, 61, 15, False, align=8):
        assert lo % 8 == 0 and (lo == 0 or s - lo >= 15) and s - lo < 15 + 8


def test_align_frames():
    assert streaming.align_frames(256) == 1  # LJSpeech hop: every frame starts a block
    assert streaming.align_frames(300) == 8  # LibriTTS hop: 8 x 300 = 75 x 32
    assert streaming.align_frames(120) == 4


def _engine(name, cuda_device, **over):
    from parallelwavegan_amd import Engine, configs, synthetic

    params = configs.generator_params(name, **over)
    eng = Engine(params, cuda_device)
    eng.load_state_dict(synthetic.make_state_dict(params, seed=0))
    return eng


@pytest.mark.gpu
@pytest.mark.parametrize("name, frames, chunk", [("ljspeech_v1", 300, 64), ("libritts_v1", 161, 40),
                                                 ("libritts_v1", 171, 37)])
def test_chunked_equals_whole_utterance(name, frames, chunk, built_lib, cuda_device):
    from parallelwavegan_amd import synthetic

    eng = _engine(name, cuda_device)
    H = eng.upsample_factor
    mel = torch.from_numpy(synthetic.make_mel(frames, 80, seed=3)).to(cuda_device)
    noise = torch.from_numpy(synthetic.make_noise(frames * H, seed=4)).to(cuda_device)
    full = eng.infer([mel], [noise])[0].cpu().numpy()
    y = streaming.infer_chunked(eng, mel, noise, chunk).cpu().numpy()
    np.testing.assert_array_equal(y, full)
    # a halo that is too short must show (the test has teeth)
    y_bad = streaming.infer_chunked(eng, mel, noise, chunk, halo=1).cpu().numpy()
    assert not np.array_equal(y_bad, full)


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["reference_test", "ljspeech_v1", "libritts_v1"])
def test_causal_stream_equals_whole_utterance(name, built_lib, cuda_device):
    from parallelwavegan_amd import synthetic

    eng = _engine(name, cuda_device, use_causal_conv=True)
    A, H = eng.config.aux_channels, eng.upsample_factor
    frames = 150
    mel = torch.from_numpy(synthetic.make_mel(frames, A, seed=5)).to(cuda_device)
    noise = torch.from_numpy(synthetic.make_noise(frames * H, seed=6)).to(cuda_device).reshape(-1)
    full = eng.infer([mel], [noise])[0].cpu().numpy()
    st = streaming.CausalStream(eng)
    outs, f = [], 0
    for n in (1, 7, 30, 2, 50, 60):
        outs.append(st.push(mel[f:f + n], noise[f * H:(f + n) * H]).cpu().numpy())
        f += n
    assert f == frames
    np.testing.assert_array_equal(np.concatenate(outs, 0), full)


def test_upsample_reach_frames():
    assert streaming.upsample_reach_frames([4, 4, 4, 4], False) == pytest.approx(1 + 1 / 4 + 1 / 16 + 1 / 64)
    assert streaming.upsample_reach_frames([2] * 8, True) == pytest.approx(2 * (2 - 2 ** -7))


@pytest.mark.gpu
@pytest.mark.parametrize("causal", [False, True], ids=["noncausal", "causal"])
def test_many_small_scales_chunked_and_streamed(causal, built_lib, cuda_device):
    """Eight x2 upsample stages (hop 256): the FIR chain reaches ~2 frames (~4 causal), more than
    a constant allowance covered; chunking and streaming stay bit-identical."""
    from parallelwavegan_amd import synthetic

    eng = _engine("reference_test", cuda_device, use_causal_conv=causal,
                  upsample_params={"upsample_scales": [2] * 8})
    A, H = eng.config.aux_channels, eng.upsample_factor
    frames = 90
    mel = torch.from_numpy(synthetic.make_mel(frames, A, seed=7)).to(cuda_device)
    noise = torch.from_numpy(synthetic.make_noise(frames * H, seed=8)).to(cuda_device).reshape(-1)
    full = eng.infer([mel], [noise])[0].cpu().numpy()
    np.testing.assert_array_equal(streaming.infer_chunked(eng, mel, noise, 11).cpu().numpy(), full)
    if causal:
        st = streaming.CausalStream(eng)
        outs, f = [], 0
        for n in (1, 3, 17, 5, 64):
            outs.append(st.push(mel[f:f + n], noise[f * H:(f + n) * H]).cpu().numpy())
            f += n
        np.testing.assert_array_equal(np.concatenate(outs, 0), full)


@pytest.mark.gpu
def test_causal_stream_rejects_noncausal(built_lib, cuda_device):
    eng = _engine("reference_test", cuda_device)
    with pytest.raises(ValueError):
        streaming.CausalStream(eng)


@pytest.mark.gpu
@pytest.mark.parametrize("causal", [False, True], ids=["noncausal", "causal"])
def test_bilinear_upsampler_chunked(causal, built_lib, cuda_device):
    """interpolate_mode="bilinear" (layers/upsample.py:43-45): the stretch reaches one more input
    sample per stage (upsample_reach_frames) and looks ahead even in a causal generator, so chunks
    take right halos then too; chunked decoding stays bit-identical to the whole utterance, and
    CausalStream refuses the configuration."""
    from parallelwavegan_amd import synthetic

    eng = _engine("ljspeech_v1", cuda_device, use_causal_conv=causal,
                  upsample_params={"upsample_scales": [4, 4, 4, 4], "interpolate_mode": "bilinear"})
    H = eng.upsample_factor
    mel = torch.from_numpy(synthetic.make_mel(203, 80, seed=13)).to(cuda_device)
    noise = torch.from_numpy(synthetic.make_noise(203 * H, seed=14)).to(cuda_device)
    full = eng.infer([mel], [noise])[0].cpu().numpy()
    np.testing.assert_array_equal(streaming.infer_chunked(eng, mel, noise, 48).cpu().numpy(), full)
    if causal:
        with pytest.raises(ValueError):
            streaming.CausalStream(eng)
