"""Half-block work units (PWG_OPT_HALF_BLOCKS; csrc/pwg_split16.hip pwg_layer_split16_kernel with
NTN = 1): one wave takes one 16-column n-tile of a 32-sample block, so a small plan spreads over
twice the waves and each wave's dependent chain runs half the MFMAs. Every column's accumulators
sum the same products in the same order as with whole blocks, and the aux K slots stay anchored at
the block's first frame, so the forward must be BIT-IDENTICAL to the whole-block kernel on every
plan: ragged batches, utterances shorter than a block, causal configs, first_conv fused or not,
the batched forward() layout, the bench's full batch, graph replay and the drop-in's B = 1 call
(bin/decode.py:236-268). GPU only; every forward goes through include/pwg.h."""

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _engines(params, dev, seed=0):
    from parallelwavegan_amd import Engine, synthetic

    sd = synthetic.make_state_dict(params, seed=seed)
    whole = Engine(params, dev)
    whole.load_state_dict(sd)
    whole.set_option("half_blocks", 0)
    half = Engine(params, dev)
    half.load_state_dict(sd)
    half.set_option("half_blocks", 1 << 30)
    return whole, half


def _inputs(lengths, hop, dev, seed=5):
    rs = np.random.RandomState(seed)
    mels = [torch.from_numpy(rs.standard_normal((f, 80)).astype(np.float32)).to(dev) for f in lengths]
    noises = [torch.from_numpy(rs.standard_normal((f * hop, 1)).astype(np.float32)).to(dev) for f in lengths]
    return mels, noises


@pytest.mark.parametrize("cfg, lengths, over", [
    ("ljspeech_v1", [64], {}),
    ("ljspeech_v1", [512], {}),
    ("libritts_v1", [143, 17, 600, 1, 88, 250], {}),
    ("libritts_v1", [3, 1, 40], {"use_causal_conv": True}),
    ("ljspeech_v1", [7, 300, 2], {"use_causal_conv": True}),
])
def test_half_blocks_bitwise_equal_to_whole_blocks(cfg, lengths, over, built_lib, cuda_device):
    from parallelwavegan_amd import configs

    params = configs.generator_params(cfg, **over)
    whole, half = _engines(params, cuda_device)
    hop = whole.upsample_factor
    mels, noises = _inputs(lengths, hop, cuda_device)
    ref = [y.cpu().numpy() for y in whole.infer(mels, noises)]
    got = [y.cpu().numpy() for y in half.infer(mels, noises)]
    for a, b in zip(got, ref):
        np.testing.assert_array_equal(a, b)


def test_half_blocks_unfused_first_conv_forward_layout_and_full_batch(built_lib, cuda_device):
    """First_conv as its own kernel, the batched forward(z, c) layout (models/parallel_wavegan.py:
    144-173), and the bench's 32-utterance LibriTTS batch (many units per wave, the work queues'
    stealing included) on half blocks: bit-identical to whole blocks."""
    from parallelwavegan_amd import _lib, configs, synthetic

    params = configs.generator_params("ljspeech_v1")
    whole, half = _engines(params, cuda_device, seed=2)
    for e in (whole, half):
        e.set_option("fuse_first_conv", 0)
    mels, noises = _inputs([33, 5], 256, cuda_device, seed=7)
    got = [y.cpu().numpy() for y in half.infer(mels, noises)]
    ref = [y.cpu().numpy() for y in whole.infer(mels, noises)]
    for a, b in zip(got, ref):
        np.testing.assert_array_equal(a, b)
    B, F, w = 2, 9, params["aux_context_window"]
    rs = np.random.RandomState(3)
    c = torch.from_numpy(rs.standard_normal((B, 80, F + 2 * w)).astype(np.float32)).to(cuda_device)
    z = torch.from_numpy(rs.standard_normal((B, 1, F * 256)).astype(np.float32)).to(cuda_device)
    outs = []
    for e in (whole, half):
        plan = e.plan([F] * B, _lib.PWG_LAYOUT_FORWARD)
        out = torch.empty(B, 1, F * 256, device=cuda_device)
        e.run(plan, c, z, out)
        outs.append(out.cpu().numpy())
    np.testing.assert_array_equal(outs[1], outs[0])

    params = configs.generator_params("libritts_v1")
    whole, half = _engines(params, cuda_device, seed=0)
    lengths = synthetic.libritts_lengths(32, seed=3).tolist()
    plan_a, plan_b = whole.plan(lengths), half.plan(lengths)
    rs = np.random.RandomState(100)
    mel = torch.from_numpy(rs.standard_normal(sum(lengths) * 80).astype(np.float32)).to(cuda_device)
    noise = torch.from_numpy(rs.standard_normal(plan_a.total_samples).astype(np.float32)).to(cuda_device)
    ya = torch.empty(plan_a.total_samples, device=cuda_device)
    yb = torch.empty_like(ya)
    whole.run(plan_a, mel, noise, ya)
    half.run(plan_b, mel, noise, yb)
    assert torch.equal(ya, yb)


def test_half_blocks_graph_replay_and_decode_pattern(built_lib, cuda_device):
    """A half-block run captured as a HIP graph replays bit-identically, and the drop-in's B = 1
    inference() on the default options matches the whole-block engine."""
    from parallelwavegan_amd import GraphedRun, ParallelWaveGANGenerator, configs, synthetic

    params = configs.generator_params("ljspeech_v1")
    whole, half = _engines(params, cuda_device, seed=4)
    plan = half.plan([64])
    g = GraphedRun(half, plan)
    for seed in (1, 2):
        mels, noises = _inputs([64], 256, cuda_device, seed=seed)
        y = g(mels[0], noises[0]).clone()
        ref = whole.infer(mels, noises)[0].reshape(-1)
        assert torch.equal(y, ref)
    del g
    m = ParallelWaveGANGenerator(**params)
    m.remove_weight_norm()
    m.load_state_dict({k: torch.from_numpy(v) for k, v in synthetic.make_state_dict(params, seed=4).items()})
    m = m.eval().to(cuda_device)
    mel = synthetic.make_mel(100, 80, seed=8)
    noise = synthetic.make_noise(100 * 256, seed=9)
    with torch.no_grad():
        y = m.inference(mel, noise).reshape(-1)
    ref = whole.infer([torch.from_numpy(mel).to(cuda_device)], [torch.from_numpy(noise).to(cuda_device)])[0]
    assert torch.equal(y, ref.reshape(-1))
