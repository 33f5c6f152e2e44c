"""The layer-pipelined split16 forward (PWG_OPT_PIPELINE, pwg_split16.hip pwg_pipe_split16_kernel):
all 30 residual layers in ONE launch, each CU keeping one layer's weights, blocks handed from layer
to layer through per-block progress words. It runs the same per-block arithmetic as the per-layer
launches, so its output must be BIT-IDENTICAL to them on every plan it accepts: ragged batches,
utterances shorter than a block, causal configs, the batched forward() layout, first_conv fused
or not, and the bench's full 32-utterance LibriTTS batch. Plus: graph capture/replay of a
pipelined run, and the reference's B = 1 decode call pattern (bin/decode.py:236-268) on it.
GPU only; every forward goes through include/pwg.h."""

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _engines(params, dev, seed=0):
    from parallelwavegan_amd import Engine, synthetic

    sd = synthetic.make_state_dict(params, seed=seed)
    per = Engine(params, dev)
    per.load_state_dict(sd)
    per.set_option("pipeline", 0)
    pipe = Engine(params, dev)
    pipe.load_state_dict(sd)
    pipe.set_option("pipeline", 1 << 24)
    return per, pipe


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
def test_pipeline_bitwise_equal_to_per_layer(cfg, lengths, over, built_lib, cuda_device):
    from parallelwavegan_amd import configs

    params = configs.generator_params(cfg, **over)
    per, pipe = _engines(params, cuda_device)
    hop = per.upsample_factor
    mels, noises = _inputs(lengths, hop, cuda_device)
    ref = [y.cpu().numpy() for y in per.infer(mels, noises)]
    pipe.set_timing(True)
    got = [y.cpu().numpy() for y in pipe.infer(mels, noises)]
    t = pipe.collect_timing()
    pipe.set_timing(False)
    assert t["residual_layer"][1] == 1, "the plan did not run on the layer pipeline"
    for a, b in zip(got, ref):
        np.testing.assert_array_equal(a, b)


def test_pipeline_unfused_first_conv_and_forward_layout(built_lib, cuda_device):
    """First_conv as its own kernel (layer 0 then reads plane 0), and the batched forward(z, c)
    layout (models/parallel_wavegan.py:144-173) on the pipeline: bit-identical to per-layer."""
    from parallelwavegan_amd import _lib, configs

    params = configs.generator_params("ljspeech_v1")
    per, pipe = _engines(params, cuda_device, seed=2)
    for e in (per, pipe):
        e.set_option("fuse_first_conv", 0)
    mels, noises = _inputs([33, 5], 256, cuda_device, seed=7)
    ref = [y.cpu().numpy() for y in per.infer(mels, noises)]
    got = [y.cpu().numpy() for y in pipe.infer(mels, noises)]
    for a, b in zip(got, ref):
        np.testing.assert_array_equal(a, b)
    B, F, w = 2, 9, params["aux_context_window"]
    rs = np.random.RandomState(3)
    c = torch.from_numpy(rs.standard_normal((B, 80, F + 2 * w)).astype(np.float32)).to(cuda_device)
    z = torch.from_numpy(rs.standard_normal((B, 1, F * 256)).astype(np.float32)).to(cuda_device)
    outs = []
    for e in (per, pipe):
        plan = e.plan([F] * B, _lib.PWG_LAYOUT_FORWARD)
        out = torch.empty(B, 1, F * 256, device=cuda_device)
        e.run(plan, c, z, out)
        outs.append(out.cpu().numpy())
    np.testing.assert_array_equal(outs[1], outs[0])


def test_pipeline_full_bench_batch(built_lib, cuda_device):
    """The bench workload (32 ragged LibriTTS utterances, 7.29 M samples) forced onto the pipeline:
    bit-identical to the per-layer launches at full size."""
    from parallelwavegan_amd import configs, synthetic

    params = configs.generator_params("libritts_v1")
    per, pipe = _engines(params, cuda_device, seed=0)
    lengths = synthetic.libritts_lengths(32, seed=3).tolist()
    plan_a, plan_b = per.plan(lengths), pipe.plan(lengths)
    rs = np.random.RandomState(100)
    mel = torch.from_numpy(rs.standard_normal(sum(lengths) * 80).astype(np.float32)).to(cuda_device)
    noise = torch.from_numpy(rs.standard_normal(plan_a.total_samples).astype(np.float32)).to(cuda_device)
    ya = torch.empty(plan_a.total_samples, device=cuda_device)
    yb = torch.empty_like(ya)
    per.run(plan_a, mel, noise, ya)
    pipe.run(plan_b, mel, noise, yb)
    assert per.range_reruns == 0 and pipe.range_reruns == 0
    assert torch.equal(ya, yb)


def test_pipeline_graph_replay_and_decode_pattern(built_lib, cuda_device):
    """A pipelined run captured as a HIP graph replays bit-identically for two inputs, and the
    drop-in's B = 1 inference() (the default path for small plans) matches the per-layer engine."""
    from parallelwavegan_amd import GraphedRun, ParallelWaveGANGenerator, configs, synthetic

    params = configs.generator_params("ljspeech_v1")
    per, pipe = _engines(params, cuda_device, seed=4)
    plan = pipe.plan([64])
    g = GraphedRun(pipe, plan)
    for seed in (1, 2):
        mels, noises = _inputs([64], 256, cuda_device, seed=seed)
        y = g(mels[0], noises[0]).clone()
        ref = per.infer(mels, noises)[0].reshape(-1)
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
    ref = per.infer([torch.from_numpy(mel).to(cuda_device)], [torch.from_numpy(noise).to(cuda_device)])[0]
    assert torch.equal(y, ref.reshape(-1))

