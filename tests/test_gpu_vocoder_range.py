"""Split-f16 range guard, stress cases and long / maximum-size parity of the conv-network
executor (MelGAN-family drop-ins), GPU only, through
include/pwg_cnet.h.

The split-f16 mode carries every fp32 operand as an fp16 pair (hi, lo): fp32's mantissa, fp16's
exponent range. Two guards make a value outside that range fail loudly instead of silently:
- pack time: pwg_cnet_pack_weights returns PWG_ERR_RANGE for a weight |w| >= 65520; the engine
  then runs exact fp32 from the start and refuses set_split_f16(True);
- run time: an activation beyond the range splits into (inf, -inf), every later product is NaN and
  nothing downstream clears it, so the launch writing the program output flags a non-finite value;
  pwg_cnet_run_status reports it and CnetEngine.run(check=True) (the drop-ins' path) reruns the
  forward in exact fp32 (range_reruns).

Bar: max|d| < max(1e-4, 3 x the error of the reference's own fp32 op sequence) against the float64
oracle (oracle/melgan_numpy.py); the second term only matters where the network itself is
ill-conditioned in fp32. Cases the reference handles well must also pass max(1e-4, 1.25 x that fp32
error): no worse than the reference's own fp32 arithmetic (mel x 30 on MB-MelGAN v2: output
amplitude 6.3, the reference's fp32 error 9.7e-5).
Reference: models/hifigan.py:173-207 (forward, N(0, 0.01) init), models/melgan.py:159-170,
layers/pqmf.py:133-149."""

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

ATOL = 1e-4


def _holder(cfg, sd_fn, seed=3):
    """(module on no device yet, params, folded state dict, PQMF synthesis taps or None) with the
    state dict drawn by synthetic.make_module_state_dict and transformed by ``sd_fn``."""
    from parallelwavegan_amd import configs, synthetic
    from parallelwavegan_amd.hifigan import HiFiGANGenerator
    from parallelwavegan_amd.melgan import PQMF, MelGANGenerator

    cls_name, params = configs.vocoder_params(cfg, use_weight_norm=False)
    m = {"MelGANGenerator": MelGANGenerator, "HiFiGANGenerator": HiFiGANGenerator}[cls_name](**params)
    sd = sd_fn(synthetic.make_module_state_dict(m, seed=seed), m)
    m.load_state_dict({k: torch.from_numpy(np.ascontiguousarray(v)) for k, v in sd.items()})
    syn = None
    if cfg in configs.VOCODER_PQMF:
        m.pqmf = PQMF(**configs.VOCODER_PQMF[cfg])
        syn = m.pqmf.synthesis_taps()
    return m, cls_name, params, sd, syn


def _oracles(cls_name, mel, sd, params, syn):
    from oracle import melgan_numpy
    from oracle.melgan_torch_cpu import TorchCPUVocoder

    if cls_name == "MelGANGenerator":
        ref = melgan_numpy.melgan_inference(mel, sd, params, syn)
    else:
        ref = melgan_numpy.hifigan_inference(mel, sd, params)
    torch.set_num_threads(min(16, torch.get_num_threads()))
    fp32 = TorchCPUVocoder(cls_name, sd, params, syn).inference(mel)
    fp32 = fp32.numpy() if torch.is_tensor(fp32) else np.asarray(fp32)
    return ref, np.abs(fp32.reshape(ref.shape) - ref).max()


def _scale_convs(k, only=None):
    def fn(sd, m):
        return {key: (v * k if key.endswith(".weight") and (only is None or key.startswith(only)) else v)
                for key, v in sd.items()}
    return fn


def _ref_init(sd, m):
    """The reference HiFiGAN's own init (models/hifigan.py:194-207): conv weights ~ N(0, 0.01).
    Pushes most lo halves of the weight pairs into fp16 subnormals (2^-24 absolute resolution)."""
    rs = np.random.RandomState(77)
    return {key: ((0.01 * rs.standard_normal(v.shape)).astype(np.float32) if key.endswith(".weight") else v)
            for key, v in sd.items()}


def _big_weight(sd, m):
    sd = dict(sd)
    key = next(k for k in sd if k.endswith(".weight") and ("blocks.0." in k or "melgan.3." in k))
    w = sd[key].copy()
    w.reshape(-1)[5] = 7e4
    sd[key] = w
    return sd


CASES = {
    # name: (state-dict transform, mel factor, expect a run-time rerun, expect pack refusal, 1e-4 outright)
    "mel_x30": (lambda sd, m: sd, 30.0, False, False, True),
    "w_x2": (_scale_convs(2.0), 1.0, None, False, False),
    "ref_init_n001": (_ref_init, 1.0, False, False, True),
    "act_overflow": (None, 1.0, True, False, False),  # first conv x1e5: its output leaves the pair range
    "weight_overflow": (_big_weight, 1.0, False, True, False),
}
FRAMES = {"hifigan_v1": 12, "mb_melgan_v2": 24}


@pytest.mark.parametrize("case", list(CASES))
@pytest.mark.parametrize("cfg", ["hifigan_v1", "mb_melgan_v2"])
def test_vocoder_split_range_guard(cfg, case, built_lib, cuda_device):
    from parallelwavegan_amd import _lib, synthetic

    fn, mel_k, rerun, refused, outright = CASES[case]
    if case == "act_overflow":
        first = "input_conv." if cfg.startswith("hifigan") else "melgan.1."
        fn = _scale_convs(1e5, only=first)
    m, cls_name, params, sd, syn = _holder(cfg, fn)
    m = m.to(cuda_device)
    eng = m.engine()
    mel = synthetic.make_mel(FRAMES[cfg], 80, seed=9) * mel_k
    with torch.no_grad():
        y = m.inference(mel).cpu().numpy()
    if refused:
        assert not eng.split_range_ok and not eng.split_f16
        with pytest.raises(_lib.RangeError):
            eng.set_split_f16(True)
    else:
        assert eng.split_range_ok and eng.split_f16
    if rerun is not None:
        assert eng.range_reruns == (1 if rerun else 0), f"{cfg}/{case}: range_reruns {eng.range_reruns}"
    ref, fp32_err = _oracles(cls_name, mel, sd, params, syn)
    assert np.isfinite(ref).all() and np.isfinite(y).all()
    err = np.abs(y.reshape(ref.shape) - ref).max()
    assert err < max(ATOL, 3 * fp32_err), f"{cfg}/{case}: max|d| = {err:.3e}, fp32 reference {fp32_err:.3e}"
    if outright:
        assert err < max(ATOL, 1.25 * fp32_err), f"{cfg}/{case}: max|d| = {err:.3e}, fp32 reference {fp32_err:.3e}"
    if rerun:
        # the raw C-ABI path reports the flag instead of rerunning
        plan = eng.plan([FRAMES[cfg]])
        out = torch.empty(plan.out_rows * eng.out_channels, device=cuda_device)
        eng.run(plan, torch.from_numpy(mel).to(cuda_device).reshape(-1), out, check=False)
        with pytest.raises(_lib.RangeError):
            eng.run_status(plan)


@pytest.mark.parametrize("cfg", ["hifigan_v1", "mb_melgan_v2"])
def test_full_length_ragged_batch_against_torch_cpu(cfg, built_lib, cuda_device):
    """The bench's utterance lengths: a ragged batch with a full-length utterance (T' = 1199, the
    longest of the bench list) plus two shorter ones, each against the reference's fp32 op
    sequence on the CPU (oracle/melgan_torch_cpu.py), |d| < 1e-4 (split-f16 default path)."""
    from oracle.melgan_torch_cpu import TorchCPUVocoder
    from parallelwavegan_amd import synthetic

    m, cls_name, params, sd, syn = _holder(cfg, lambda sd, m: sd, seed=11)
    m = m.to(cuda_device)
    lengths = [1199, 80, 517]
    mels = [synthetic.make_mel(f, 80, seed=300 + i) for i, f in enumerate(lengths)]
    from test_gpu_vocoders import _rstack_launches
    n0 = _rstack_launches()
    with torch.no_grad():
        ys = [y.cpu().numpy() for y in m.inference_batch(mels)]
    assert m.engine().range_reruns == 0
    if cfg == "mb_melgan_v2":  # its 48-channel stage runs batched: the LDS-ring stack kernel
        assert _rstack_launches() > n0
    torch.set_num_threads(min(16, torch.get_num_threads()))
    gen = TorchCPUVocoder(cls_name, sd, params, syn)
    for f, mel, y in zip(lengths, mels, ys):
        ref = gen.inference(mel)
        ref = ref.numpy() if torch.is_tensor(ref) else np.asarray(ref)
        err = np.abs(y.reshape(ref.shape) - ref).max()
        assert err < ATOL, f"{cfg} T'={f}: max|d| = {err:.3e}"


def test_long_utterance_prefix_is_position_independent(built_lib, cuda_device):
    """A 30,000-frame HiFiGAN v1 utterance (7.7 M samples, ~5.8 min at 22.05 kHz): finite, and
    its first 2,900 frames of audio are bit-identical to those of a 3,000-frame prefix utterance
    (every kernel tiles an utterance from its own start, and the receptive field is a few frames)."""
    from parallelwavegan_amd import synthetic

    m, _, params, _, _ = _holder("hifigan_v1", lambda sd, m: sd, seed=12)
    m = m.to(cuda_device)
    hop = int(np.prod(params["upsample_scales"]))
    mel = synthetic.make_mel(30000, 80, seed=5)
    with torch.no_grad():
        y_long = m.inference(mel)
        assert torch.isfinite(y_long).all()
        y_short = m.inference(mel[:3000])
    k = 2900 * hop
    torch.testing.assert_close(y_long[:k], y_short[:k], rtol=0, atol=0)
