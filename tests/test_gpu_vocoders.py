"""Parity of the conv-network executor (MelGAN / multi-band MelGAN + PQMF / HiFiGAN drop-ins,
SURVEY.md sec 8(f) rows 1-2) with the reference's golden vectors and the float64 oracle.
GPU only; every forward goes through include/pwg_cnet.h.

Tolerance: |d| < 1e-4 absolute (BASELINE.json north_star's fp32 bar), ATOL below."""

import numpy as np
import pytest
import torch

from conftest import load_golden, vocoder_golden_names, vocoder_holder

pytestmark = pytest.mark.gpu

ATOL = 1e-4


def _rstack_launches():
    """Batched ResidualStack (pwg_rstack.hip) launches enqueued so far (test hook)."""
    import ctypes

    from parallelwavegan_amd import _lib
    f = _lib.load().pwg_rstack_debug_launches
    f.restype = ctypes.c_longlong
    return int(f())


@pytest.mark.parametrize("split", [True, False], ids=["split_f16", "fp32"])
@pytest.mark.parametrize("name", vocoder_golden_names())
def test_vocoder_golden_vectors(name, split, built_lib, cuda_device):
    g = load_golden(name)
    meta = g["meta"]
    m, params, _ = vocoder_holder(meta)
    m = m.to(cuda_device)
    m.engine().set_split_f16(split)
    with torch.no_grad():
        if meta["options"].get("forward"):
            y = m(torch.from_numpy(g["c"]).to(cuda_device))
        else:
            norm = "mean" in g
            if norm:
                m.register_buffer("mean", torch.from_numpy(g["mean"]).to(cuda_device))
                m.register_buffer("scale", torch.from_numpy(g["scale"]).to(cuda_device))
            y = m.inference(g["mel"], normalize_before=norm)
    y = y.cpu().numpy()
    assert y.shape == g["y"].shape
    assert np.isfinite(y).all()
    err = np.abs(y - g["y"]).max()
    assert err < ATOL, f"{name}: max|d| = {err:.3e}"


@pytest.mark.parametrize("split", [True, False], ids=["split_f16", "fp32"])
@pytest.mark.parametrize("cfg, frames", [("mb_melgan_v2", 40), ("hifigan_v1", 12), ("melgan_v1", 16),
                                         ("mb_melgan_v2_causal", 40), ("hifigan_v1_causal", 12),
                                         ("melgan_v1_causal", 16)])
def test_full_size_configs_against_oracle(cfg, frames, split, built_lib, cuda_device):
    from oracle import melgan_numpy
    from parallelwavegan_amd import configs, synthetic
    from parallelwavegan_amd.engine import fold_weight_norm
    from parallelwavegan_amd.hifigan import HiFiGANGenerator
    from parallelwavegan_amd.melgan import PQMF, MelGANGenerator

    cls_name, params = configs.vocoder_params(cfg)
    m = {"MelGANGenerator": MelGANGenerator, "HiFiGANGenerator": HiFiGANGenerator}[cls_name](**params)
    sd = synthetic.make_module_state_dict(m, seed=3)
    m.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()})
    syn = None
    if cfg in configs.VOCODER_PQMF:
        m.pqmf = PQMF(**configs.VOCODER_PQMF[cfg])
        syn = m.pqmf.synthesis_taps()
    m = m.to(cuda_device)
    m.engine().set_split_f16(split)
    mel = synthetic.make_mel(frames, 80, seed=9)
    with torch.no_grad():
        y = m.inference(mel).cpu().numpy()
    folded = fold_weight_norm(sd)
    if cls_name == "MelGANGenerator":
        ref = melgan_numpy.melgan_inference(mel, folded, params, syn)
    else:
        ref = melgan_numpy.hifigan_inference(mel, folded, params)
    assert y.shape == ref.shape
    err = np.abs(y - ref).max()
    assert err < ATOL, f"{cfg}: max|d| = {err:.3e}"


@pytest.mark.parametrize("cfg", ["mb_melgan_test", "hifigan_test", "mb_melgan_causal_test", "hifigan_causal_test"])
def test_ragged_batch_is_bitwise_equal_to_single_utterances(cfg, built_lib, cuda_device):
    from parallelwavegan_amd import configs, synthetic
    from parallelwavegan_amd.hifigan import HiFiGANGenerator
    from parallelwavegan_amd.melgan import PQMF, MelGANGenerator

    cls_name, params = configs.vocoder_params(cfg)
    m = {"MelGANGenerator": MelGANGenerator, "HiFiGANGenerator": HiFiGANGenerator}[cls_name](**params)
    m.load_state_dict({k: torch.from_numpy(v) for k, v in synthetic.make_module_state_dict(m, seed=1).items()})
    if cfg in configs.VOCODER_PQMF:
        m.pqmf = PQMF(**configs.VOCODER_PQMF[cfg])
    m = m.to(cuda_device)
    lengths = [7, 37, 8, 130, 9] if params.get("use_causal_conv") else [4, 37, 5, 130, 9]
    mels = [synthetic.make_mel(f, 80, seed=30 + i) for i, f in enumerate(lengths)]
    with torch.no_grad():
        batch = [y.cpu().numpy() for y in m.inference_batch(mels)]
        for i in range(len(lengths)):
            np.testing.assert_array_equal(batch[i], m.inference(mels[i]).cpu().numpy())


def test_vocoder_timing_and_weight_update(built_lib, cuda_device):
    from parallelwavegan_amd import configs, synthetic
    from parallelwavegan_amd.hifigan import HiFiGANGenerator

    _, params = configs.vocoder_params("hifigan_noadd_test")
    m = HiFiGANGenerator(**params)
    m.load_state_dict({k: torch.from_numpy(v) for k, v in synthetic.make_module_state_dict(m, seed=2).items()})
    m = m.to(cuda_device)
    mel = synthetic.make_mel(12, 80, seed=5)
    eng = m.engine()
    eng.set_timing(True)
    with torch.no_grad():
        y1 = m.inference(mel).cpu().numpy()
        t = eng.collect_timing()
        assert len(t) == len(eng.program.ops) and all(n >= 1 for _, _, n in t)
        m.output_conv[1].bias.add_(0.25)  # re-packed on the next call
        y2 = m.inference(mel).cpu().numpy()
    assert np.abs(y2 - y1).max() > 1e-3


@pytest.mark.parametrize("causal", [False, True], ids=["noncausal", "causal"])
def test_xtile_pairs_bitwise_equal_to_unfused(causal, built_lib, cuda_device):
    """pwg_cnet_xpair_kernel (HiFiGAN ResBlock conv pairs of 32/64 channels on the x-tile scheme,
    h in LDS, 224-column workgroups) against the same two convs as two x-tile launches: same
    chunk order, pair split and epilogue order, so bit-identical; ragged utterances exercise
    utterance edges inside a workgroup (conv 2's zero padding of h)."""
    from parallelwavegan_amd import configs, synthetic
    from parallelwavegan_amd.hifigan import HiFiGANGenerator

    _, params = configs.vocoder_params("hifigan_v1_causal" if causal else "hifigan_v1")
    m = HiFiGANGenerator(**params)
    m.load_state_dict({k: torch.from_numpy(v) for k, v in synthetic.make_module_state_dict(m, seed=4).items()})
    m = m.to(cuda_device)
    eng = m.engine()
    eng.set_narrow(0)  # the default (8-wave) launches themselves, not their small-plan form
    mels = [synthetic.make_mel(f, 80, seed=90 + i) for i, f in enumerate([3, 1, 14, 5])]
    with torch.no_grad():
        eng.set_fuse_pairs(False)
        ref = [y.cpu().numpy() for y in m.inference_batch(mels)]
        eng.set_fuse_pairs(True)
        eng.set_timing(True)
        got = [y.cpu().numpy() for y in m.inference_batch(mels)]
        t = eng.collect_timing()
        eng.set_timing(False)
    assert sum(1 for _, _, n in t if n == 0) == 21  # the 64- and 32-channel stages' 3 x 3 pairs + the 128-channel k = 3 block's 3
    for a, b in zip(got, ref):
        np.testing.assert_array_equal(a, b)


@pytest.mark.parametrize("steps", [1, 3, 8])
def test_fused_conv_pairs_bitwise_equal_to_unfused(steps, built_lib, cuda_device):
    """pwg_cnet_pair_kernel (ResBlock conv pairs with the intermediate in LDS) against the two
    unfused split-f16 ops: same chunk order, pair split and epilogue order, so bit-identical.
    Ragged utterances (1..14 frames -> 256..3584 columns at the 32-channel stage) with strips of
    1, 3 and 8 tiles exercise strip starts, partial last strips and utterance edges."""
    from parallelwavegan_amd import configs, synthetic
    from parallelwavegan_amd.hifigan import HiFiGANGenerator

    _, params = configs.vocoder_params("hifigan_v1")
    m = HiFiGANGenerator(**params)
    m.load_state_dict({k: torch.from_numpy(v) for k, v in synthetic.make_module_state_dict(m, seed=4).items()})
    m = m.to(cuda_device)
    eng = m.engine()
    eng.set_pair_steps(steps)
    eng.set_xtile(False)  # pairs of x-tile convs run unfused (PWG_CNET_OPT_XTILE)
    mels = [synthetic.make_mel(f, 80, seed=60 + i) for i, f in enumerate([3, 1, 14, 5])]
    with torch.no_grad():
        eng.set_fuse_pairs(False)
        ref = [y.cpu().numpy() for y in m.inference_batch(mels)]
        eng.set_fuse_pairs(True)
        eng.set_timing(True)
        got = [y.cpu().numpy() for y in m.inference_batch(mels)]
        t = eng.collect_timing()
        eng.set_timing(False)
    # the 64- (streamed weights) and 32-channel (resident weights) stages' 3 ResBlocks x 3
    # (conv1, conv2) pairs run fused (128 channels: PWG_PAIR_STREAM128, off)
    assert sum(1 for _, _, n in t if n == 0) == 18
    for a, b in zip(got, ref):
        np.testing.assert_array_equal(a, b)


@pytest.mark.parametrize("cfg, over", [
    ("hifigan_v1_causal", {"upsample_scales": [5, 5, 4, 3], "upsample_kernel_sizes": [10, 10, 8, 6]}),
    ("hifigan_v1_causal", {"upsample_scales": [4, 5, 4, 3], "upsample_kernel_sizes": [8, 10, 8, 6]}),
    ("hifigan_v1_causal", {}),
    ("melgan_v1_causal", {}),
    ("melgan_v1_causal", {"upsample_scales": [4, 5, 4, 3]}),
])
def test_causal_generators_are_causal(cfg, over, built_lib, cuda_device):
    """Restates test/test_hifigan.py:198-225 and test/test_melgan.py:275-301: B = 4 utterances of
    8192 (HiFiGAN) / 4096 (MelGAN) samples through forward(); replacing the second half of the
    frames leaves the first half of the output bit-identical, and T_out = T' * hop."""
    from parallelwavegan_amd import configs, synthetic
    from parallelwavegan_amd.hifigan import HiFiGANGenerator
    from parallelwavegan_amd.melgan import MelGANGenerator

    cls_name, params = configs.vocoder_params(cfg, **over)
    m = {"MelGANGenerator": MelGANGenerator, "HiFiGANGenerator": HiFiGANGenerator}[cls_name](**params)
    m.load_state_dict({k: torch.from_numpy(v) for k, v in synthetic.make_module_state_dict(m, seed=8).items()})
    m = m.to(cuda_device).eval()
    hop = int(np.prod(params["upsample_scales"]))
    T = (8192 if cls_name == "HiFiGANGenerator" else 4096) // hop
    g = torch.Generator().manual_seed(0)
    c = torch.randn(4, 80, T, generator=g)
    c2 = c.clone()
    c2[..., T // 2:] = torch.randn(c[..., T // 2:].shape, generator=g)
    with torch.no_grad():
        y = m(c.to(cuda_device)).cpu().numpy()
        y2 = m(c2.to(cuda_device)).cpu().numpy()
    assert y.shape[2] == T * hop
    np.testing.assert_array_equal(y[..., :T // 2 * hop], y2[..., :T // 2 * hop])
    assert not np.array_equal(y, y2)


@pytest.mark.parametrize("xtile", [False, True])
@pytest.mark.parametrize("cfg", ["mb_melgan_v2", "mb_melgan_v2_causal", "melgan_v1", "mb_melgan_test"])
def test_fused_residual_stacks_bitwise_equal_to_unfused(cfg, xtile, built_lib, cuda_device):
    """pwg_cnet_stack_kernel (MelGAN ResidualStack: dilated conv + the two-source 1x1 in one
    launch, h in LDS; x-tile off) and pwg_cnet_xstack_kernel (the same on the x-tile scheme; x-tile
    on) against the two unfused split-f16 ops of the same mode: same chunk order, pair split and
    epilogue order, so bit-identical; every ResidualStack runs fused."""
    from parallelwavegan_amd import configs, synthetic
    from parallelwavegan_amd.melgan import PQMF, MelGANGenerator

    _, params = configs.vocoder_params(cfg)
    m = MelGANGenerator(**params)
    m.load_state_dict({k: torch.from_numpy(v) for k, v in synthetic.make_module_state_dict(m, seed=4).items()})
    if cfg in configs.VOCODER_PQMF:
        m.pqmf = PQMF(**configs.VOCODER_PQMF[cfg])
    m = m.to(cuda_device)
    eng = m.engine()
    eng.set_narrow(0)  # the default (8-wave) launches themselves, not their small-plan form
    eng.set_xtile(xtile)  # off: conv A unfused on the tap-major kernel; on: on the x-tile kernel
    mels = [synthetic.make_mel(f, 80, seed=70 + i) for i, f in enumerate([9, 40, 7, 23, 300])]
    with torch.no_grad():
        eng.set_fuse_pairs(False)
        ref = [y.cpu().numpy() for y in m.inference_batch(mels)]
        eng.set_fuse_pairs(True)
        # x-tile on: the x-tile stack kernel (PWG_CNET_OPT_RSTACK 0) and the batched LDS-ring kernel
        eng.set_rstack(False)
        got0 = [y.cpu().numpy() for y in m.inference_batch(mels)]
        eng.set_rstack(True)
        n0 = _rstack_launches()
        eng.set_timing(True)
        got = [y.cpu().numpy() for y in m.inference_batch(mels)]
        t = eng.collect_timing()
        eng.set_timing(False)
    if xtile and cfg != "melgan_v1":  # (MelGAN v1's fused stacks: 64 and 32 channels, also covered)
        assert _rstack_launches() > n0
    for a, b in zip(got0, ref):
        np.testing.assert_array_equal(a, b)
    # stacks of <= 96 channels run fused (PWG_STACK_MAX_MT)
    ch, stacks = params["channels"], 0
    for _ in params["upsample_scales"]:
        ch //= 2
        stacks += params["stacks"] if ch <= 96 else 0
    assert stacks > 0
    assert sum(1 for name, _, n in t if n == 0 and "skip_layer" in name) == stacks
    for a, b in zip(got, ref):
        np.testing.assert_array_equal(a, b)


@pytest.mark.parametrize("cfg", ["hifigan_v1", "melgan_v1", "hifigan_v1_causal"])
def test_xtile_kernel_matches_tap_major(cfg, built_lib, cuda_device):
    """PWG_CNET_OPT_XTILE: the channel-block-major kernel with staged input tiles sums the same
    split-f16 products as the tap-major kernel in another order: outputs agree to fp32 rounding
    (|d| < 1e-5) on ragged batches, edges included; both are pinned to the oracle by the goldens."""
    from parallelwavegan_amd import configs, synthetic
    from parallelwavegan_amd.hifigan import HiFiGANGenerator
    from parallelwavegan_amd.melgan import MelGANGenerator

    cls_name, params = configs.vocoder_params(cfg)
    m = {"MelGANGenerator": MelGANGenerator, "HiFiGANGenerator": HiFiGANGenerator}[cls_name](**params)
    m.load_state_dict({k: torch.from_numpy(v) for k, v in synthetic.make_module_state_dict(m, seed=6).items()})
    m = m.to(cuda_device)
    eng = m.engine()
    mels = [synthetic.make_mel(f, 80, seed=80 + i) for i, f in enumerate([4, 11, 5])]  # reflect pad 3 < T
    with torch.no_grad():
        eng.set_xtile(False)
        ref = [y.cpu().numpy() for y in m.inference_batch(mels)]
        eng.set_xtile(True)
        got = [y.cpu().numpy() for y in m.inference_batch(mels)]
    for a, b in zip(got, ref):
        assert np.abs(a - b).max() < 1e-5


@pytest.mark.parametrize("cfg", ["hifigan_v1", "mb_melgan_v2", "melgan_v1", "hifigan_v1_causal"])
def test_xtile_dma_staging_bitwise_equal(cfg, built_lib, cuda_device):
    """PWG_CNET_OPT_XT_DMA: x-tile convs with their weight fragments DMA-staged (global_load_lds,
    two LDS buffers, tap groups sized for one or two workgroups per CU) run the same MFMAs in the
    same order as the register-staged kernels: bit-identical, on the measured rule's shapes and on
    every eligible conv, on ragged batches whose utterances are shorter than, equal to and longer
    than one 256-column tile. The wide ConvTranspose phases on the DMA kernel (flag 8, in every arm
    here) sum channel-block-major where the tap-major kernel sums tap-major: the two agree to fp32
    rounding (|d| < 1e-5)."""
    from parallelwavegan_amd import configs, synthetic
    from parallelwavegan_amd.cnet import CnetEngine
    from parallelwavegan_amd.hifigan import HiFiGANGenerator
    from parallelwavegan_amd.melgan import PQMF, MelGANGenerator

    cls_name, params = configs.vocoder_params(cfg)
    m = {"MelGANGenerator": MelGANGenerator, "HiFiGANGenerator": HiFiGANGenerator}[cls_name](**params)
    m.load_state_dict({k: torch.from_numpy(v) for k, v in synthetic.make_module_state_dict(m, seed=7).items()})
    if cfg in configs.VOCODER_PQMF:
        m.pqmf = PQMF(**configs.VOCODER_PQMF[cfg])
    m = m.to(cuda_device)
    eng = m.engine()
    eng.set_narrow(0)  # the default (8-wave) launches themselves, not their small-plan form
    mels = [synthetic.make_mel(f, 80, seed=120 + i) for i, f in enumerate([4, 5, 37, 9, 130])]
    C = CnetEngine
    outs = {}
    with torch.no_grad():
        for mode in (C.XT_DMA_CONVT, C.XT_DMA_CONVT | C.XT_DMA_RULE, C.XT_DMA_CONVT | C.XT_DMA_ALL,
                     C.XT_DMA_CONVT | C.XT_DMA_ALL | C.XT_DMA_FEWEST, 0):
            eng.set_xt_dma(mode)
            outs[mode] = [y.cpu().numpy() for y in m.inference_batch(mels)]
        eng.set_xt_dma(C.XT_DMA_CONVT | C.XT_DMA_RULE)
    ref = outs[C.XT_DMA_CONVT]
    for mode in (9, 10, 14):
        for a, b in zip(outs[mode], ref):
            np.testing.assert_array_equal(a, b)
    for a, b in zip(outs[0], ref):
        assert np.abs(a - b).max() < 1e-5


@pytest.mark.parametrize("cfg", ["hifigan_v1", "melgan_v1", "mb_melgan_v2"])
def test_xcd_tile_order_bitwise_equal(cfg, built_lib, cuda_device):
    """PWG_CNET_OPT_XCD_ORDER only permutes which workgroup computes which (column block, m-group,
    ConvTranspose phase) tile: bit-identical output, with and without the DMA x-tile kernels, on
    a ragged batch whose block counts are not multiples of 8 (the bijection's tail)."""
    from parallelwavegan_amd import configs, synthetic
    from parallelwavegan_amd.hifigan import HiFiGANGenerator
    from parallelwavegan_amd.melgan import PQMF, MelGANGenerator

    cls_name, params = configs.vocoder_params(cfg)
    m = {"MelGANGenerator": MelGANGenerator, "HiFiGANGenerator": HiFiGANGenerator}[cls_name](**params)
    m.load_state_dict({k: torch.from_numpy(v) for k, v in synthetic.make_module_state_dict(m, seed=8).items()})
    if cfg in configs.VOCODER_PQMF:
        m.pqmf = PQMF(**configs.VOCODER_PQMF[cfg])
    m = m.to(cuda_device)
    eng = m.engine()
    eng.set_narrow(0)  # the default (8-wave) launches themselves, not their small-plan form
    mels = [synthetic.make_mel(f, 80, seed=140 + i) for i, f in enumerate([7, 61, 4, 23, 150])]
    with torch.no_grad():
        for dma in (0, 9):
            eng.set_xt_dma(dma)
            outs = []
            for order in (0, 1):
                eng.set_xcd_order(order)
                outs.append([y.cpu().numpy() for y in m.inference_batch(mels)])
            for a, b in zip(*outs):
                np.testing.assert_array_equal(a, b)
        eng.set_xt_dma(9)


@pytest.mark.parametrize("cfg", ["hifigan_v1", "melgan_v1", "mb_melgan_v2", "hifigan_v1_causal", "mb_melgan_v2_causal"])
def test_narrow_launches_bitwise_equal(cfg, built_lib, cuda_device):
    """PWG_CNET_OPT_NARROW (the B = 1 path): x-tile launches with fewer workgroups than CUs run
    1-4-wave, 1-2-m-tile workgroups, and the fused x-tile pairs / stacks whose first conv does run
    as their two ops. Every column sums the same products in the same order, so the output is
    bit-identical to the default launches: narrow off (0), automatic (1: the short utterance alone
    and the ragged batch pick different launches) and forced on every x-tile launch (2), each on
    the DMA-ring kernel (PWG_CNET_OPT_NARROW_DMA 1) and on the narrow x-tile / tap-major ones (0)."""
    from parallelwavegan_amd import configs, synthetic
    from parallelwavegan_amd.hifigan import HiFiGANGenerator
    from parallelwavegan_amd.melgan import PQMF, MelGANGenerator

    cls_name, params = configs.vocoder_params(cfg)
    m = {"MelGANGenerator": MelGANGenerator, "HiFiGANGenerator": HiFiGANGenerator}[cls_name](**params)
    m.load_state_dict({k: torch.from_numpy(v) for k, v in synthetic.make_module_state_dict(m, seed=9).items()})
    if cfg in configs.VOCODER_PQMF:
        m.pqmf = PQMF(**configs.VOCODER_PQMF[cfg])
    m = m.to(cuda_device)
    eng = m.engine()
    mels = [synthetic.make_mel(f, 80, seed=150 + i) for i, f in enumerate([64, 9, 23, 131])]
    # 300 frames alone: launches whose DMA-ring workgroups would need more than one round over the
    # CUs (narrow x-tile kernel, 2 m-tiles per workgroup)
    long = synthetic.make_mel(300, 80, seed=149)
    with torch.no_grad():
        outs = {}
        for mode, dma in ((0, 1), (1, 1), (2, 1), (1, 0), (2, 0)):
            eng.set_narrow(mode)
            eng.set_narrow_dma(dma)
            outs[mode, dma] = ([m.inference(torch.from_numpy(x).to(cuda_device)).cpu().numpy() for x in (mels[0], long)] +
                               [y.cpu().numpy() for y in m.inference_batch(mels)])
        eng.set_narrow(1)
        eng.set_narrow_dma(1)
    # narrow_dma 1: the DMA-ring kernel (x-tile family and, K = 1 mode, the tap-major convs);
    # 0: the DMA-staged narrow x-tile kernel and the narrow tap-major kernel
    for key in ((1, 1), (2, 1), (1, 0), (2, 0)):
        for a, b in zip(outs[key], outs[0, 1]):
            assert np.isfinite(a).all()
            np.testing.assert_array_equal(a, b)


@pytest.mark.parametrize("cfg", ["hifigan_v1", "mb_melgan_v2", "hifigan_v1_causal"])
def test_concurrent_streams_bitwise_equal(cfg, built_lib, cuda_device):
    """PWG_CNET_OPT_STREAMS: independent launches (HiFiGAN's parallel residual blocks) forked onto
    auxiliary streams and joined back with events give the same bits as one stream, for the B = 1
    plan (auto mode) and a ragged batch (forced on); a captured graph of the forked forward too."""
    from parallelwavegan_amd import configs, synthetic
    from parallelwavegan_amd.hifigan import HiFiGANGenerator
    from parallelwavegan_amd.melgan import PQMF, MelGANGenerator

    cls_name, params = configs.vocoder_params(cfg)
    m = {"MelGANGenerator": MelGANGenerator, "HiFiGANGenerator": HiFiGANGenerator}[cls_name](**params)
    m.load_state_dict({k: torch.from_numpy(v) for k, v in synthetic.make_module_state_dict(m, seed=11).items()})
    if cfg in configs.VOCODER_PQMF:
        m.pqmf = PQMF(**configs.VOCODER_PQMF[cfg])
    m = m.to(cuda_device)
    eng = m.engine()
    mels = [synthetic.make_mel(f, 80, seed=170 + i) for i, f in enumerate([64, 9, 23])]
    outs = {}
    with torch.no_grad():
        for mode in (0, 1, 2):
            eng.set_streams(mode)
            outs[mode] = ([m.inference(torch.from_numpy(mels[0]).to(cuda_device)).cpu().numpy()] +
                          [y.cpu().numpy() for y in m.inference_batch(mels)])
        eng.set_streams(1)
        # graph capture of the forked forward (fork / join events become graph edges)
        plan = eng.plan([64])
        mel = torch.from_numpy(mels[0]).to(cuda_device).reshape(-1).contiguous()
        out = torch.empty(plan.out_rows * eng.out_channels, device=cuda_device)
        s = torch.cuda.Stream(cuda_device)
        with torch.cuda.stream(s):
            eng.run(plan, mel, out, stream=s)
            torch.cuda.synchronize()
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, stream=s):
                eng.run(plan, mel, out, stream=s, check=False)
            out.zero_()
            g.replay()
            torch.cuda.synchronize()
        # one plan enqueued on two caller streams back to back (each run forks / joins its own events)
        mel2 = torch.from_numpy(synthetic.make_mel(64, 80, seed=190)).to(cuda_device).reshape(-1).contiguous()
        eng.set_streams(0)
        ref2 = torch.empty_like(out)
        eng.run(plan, mel2, ref2)
        eng.set_streams(1)
        s1, s2 = torch.cuda.Stream(cuda_device), torch.cuda.Stream(cuda_device)
        o1, o2 = torch.empty_like(out), torch.empty_like(out)
        torch.cuda.synchronize()
        for _ in range(3):
            eng.run(plan, mel, o1, stream=s1, check=False)
            eng.run(plan, mel2, o2, stream=s2, check=False)
        torch.cuda.synchronize()
    for mode in (1, 2):
        for a, b in zip(outs[mode], outs[0]):
            assert np.isfinite(a).all()
            np.testing.assert_array_equal(a, b)
    np.testing.assert_array_equal(out.cpu().numpy().reshape(outs[0][0].shape), outs[0][0])
    np.testing.assert_array_equal(o1.cpu().numpy().reshape(outs[0][0].shape), outs[0][0])
    np.testing.assert_array_equal(o2.cpu().numpy(), ref2.cpu().numpy())


@pytest.mark.parametrize("cfg", ["hifigan_v1", "hifigan_v1_causal"])
def test_graph_replay_bitwise_equal(cfg, built_lib, cuda_device):
    """Small plans replay a captured forward (CnetEngine.graphs): same bits as the eager forward,
    for two different inputs through one captured graph, after an option change (re-capture) and
    with the range check reading the graph's own workspace."""
    from parallelwavegan_amd import configs, synthetic
    from parallelwavegan_amd.hifigan import HiFiGANGenerator
    from parallelwavegan_amd.melgan import PQMF, MelGANGenerator

    cls_name, params = configs.vocoder_params(cfg)
    m = {"MelGANGenerator": MelGANGenerator, "HiFiGANGenerator": HiFiGANGenerator}[cls_name](**params)
    m.load_state_dict({k: torch.from_numpy(v) for k, v in synthetic.make_module_state_dict(m, seed=13).items()})
    if cfg in configs.VOCODER_PQMF:
        m.pqmf = PQMF(**configs.VOCODER_PQMF[cfg])
    m = m.to(cuda_device)
    eng = m.engine()
    mels = [torch.from_numpy(synthetic.make_mel(48, 80, seed=200 + i)).to(cuda_device) for i in range(2)]
    eng.GRAPH_AFTER = 2  # (capture on the shape's second run; the default waits for GRAPH_AFTER = 64 runs)
    with torch.no_grad():
        eng.set_graphs(False)
        ref = [m.inference(x).cpu().numpy() for x in mels]
        eng.set_graphs(True)
        got = [m.inference(x).cpu().numpy() for x in mels] + [m.inference(mels[0]).cpu().numpy()]
        n_graphs = len(eng._graphs)
        eng.set_streams(0)  # option change: captured forwards are stale, the next call re-captures
        got.append(m.inference(mels[1]).cpu().numpy())
        eng.set_streams(1)
    assert n_graphs == 1
    for a, b in zip(got, [ref[0], ref[1], ref[0], ref[1]]):
        np.testing.assert_array_equal(a, b)



@pytest.mark.parametrize("cfg", ["hifigan_v1", "mb_melgan_v2", "hifigan_v1_causal"])
def test_descriptor_kernel_writes_the_host_image(cfg, built_lib, cuda_device):
    """Plans are host objects: every pwg_cnet_run starts with pwg_cnet_desc_kernel, which writes the
    plan's device lists into the workspace from the utterance lengths in its arguments. The image
    it writes is the one the host built and checked (pwg_cnet_plan_image), byte for byte, for a
    B = 1 plan, a ragged batch and a batch of more utterances than one descriptor launch holds
    (CN_DESC_UTTS = 64); a workspace full of garbage beforehand changes nothing."""
    from parallelwavegan_amd import configs, synthetic
    from parallelwavegan_amd.hifigan import HiFiGANGenerator
    from parallelwavegan_amd.melgan import PQMF, MelGANGenerator

    cls_name, params = configs.vocoder_params(cfg)
    m = {"MelGANGenerator": MelGANGenerator, "HiFiGANGenerator": HiFiGANGenerator}[cls_name](**params)
    m.load_state_dict({k: torch.from_numpy(v) for k, v in synthetic.make_module_state_dict(m, seed=21).items()})
    if cfg in configs.VOCODER_PQMF:
        m.pqmf = PQMF(**configs.VOCODER_PQMF[cfg])
    m = m.to(cuda_device)
    eng = m.engine()
    rs = np.random.RandomState(5)
    with torch.no_grad():
        for frames in ([37], [9, 130, 17, 64], [int(f) for f in rs.randint(8, 24, 70)]):
            plan = eng.plan(frames)
            mel = torch.from_numpy(rs.standard_normal((sum(frames), 80)).astype(np.float32)).to(cuda_device)
            out = torch.empty(plan.out_rows * eng.out_channels, device=cuda_device)
            ws = torch.full((plan.workspace_bytes,), 0xA5, dtype=torch.uint8, device=cuda_device)
            eng._enqueue(plan, mel.reshape(-1), out, None, None, torch.cuda.current_stream(), ws=ws)
            torch.cuda.synchronize()
            off, img = plan.image()
            dev = ws[off:off + 4 * img.size].cpu().numpy().view(np.int32)
            np.testing.assert_array_equal(dev, img)
            assert np.isfinite(out.cpu().numpy()).all()


@pytest.mark.parametrize("cfg", ["hifigan_v1", "mb_melgan_v2"])
def test_distinct_length_decode_loop(cfg, built_lib, cuda_device):
    """The reference's decode loop (bin/decode.py:236-268): one inference() per utterance, each with
    its own length. Every call builds a new plan on the host; no graph is captured for a length used
    once or repeated a few times (a capture costs 4-26 ms and a replay saves ~0.09 ms: the policy waits
    for GRAPH_AFTER runs of a shape, counted across plan evictions), a length used that often is
    captured and replayed (HiFiGAN); every output is bit-identical to the same utterance decoded with
    graphs off, and to its slice of one ragged batch."""
    from parallelwavegan_amd import configs, synthetic
    from parallelwavegan_amd.hifigan import HiFiGANGenerator
    from parallelwavegan_amd.melgan import PQMF, MelGANGenerator

    cls_name, params = configs.vocoder_params(cfg)
    m = {"MelGANGenerator": MelGANGenerator, "HiFiGANGenerator": HiFiGANGenerator}[cls_name](**params)
    m.load_state_dict({k: torch.from_numpy(v) for k, v in synthetic.make_module_state_dict(m, seed=22).items()})
    if cfg in configs.VOCODER_PQMF:
        m.pqmf = PQMF(**configs.VOCODER_PQMF[cfg])
    m = m.to(cuda_device)
    eng = m.engine()
    lengths = [int(f) for f in np.random.RandomState(3).randint(16, 160, 10)]
    mels = [torch.from_numpy(synthetic.make_mel(f, 80, seed=300 + i)).to(cuda_device) for i, f in enumerate(lengths)]
    with torch.no_grad():
        got = [m.inference(x).cpu().numpy() for x in mels]
        assert len(eng._graphs) == 0
        for _ in range(3):  # a few repeats: still eager
            again = m.inference(mels[0]).cpu().numpy()
        assert len(eng._graphs) == 0
        eng._plans.clear()  # use counts survive plan eviction
        for _ in range(eng.GRAPH_AFTER - 5):
            m.inference(mels[0])
        assert len(eng._graphs) == 0
        again = m.inference(mels[0]).cpu().numpy()  # the GRAPH_AFTER-th run of that length: captured (HiFiGAN)
        third = m.inference(mels[0]).cpu().numpy()  # replayed
        n_graphs = len(eng._graphs)
        eng.set_graphs(False)
        ref = [m.inference(x).cpu().numpy() for x in mels]
        eng.set_graphs(True)
        batch = [y.cpu().numpy() for y in m.inference_batch([x.cpu().numpy() for x in mels])]
    assert n_graphs == (1 if cls_name == "HiFiGANGenerator" else 0)
    for a, b, c in zip(got, ref, batch):
        np.testing.assert_array_equal(a, b)
        np.testing.assert_array_equal(a, c)
    np.testing.assert_array_equal(again, ref[0])
    np.testing.assert_array_equal(third, ref[0])


@pytest.mark.parametrize("cfg", ["mb_melgan_v2", "melgan_v1", "mb_melgan_test"])
def test_fused_stack_chain_bitwise_equal(cfg, built_lib, cuda_device):
    """PWG_CNET_OPT_MSTACK (pwg_mstack.hip): a MelGAN stage's ResidualStack chain as one launch per
    block of output columns, the input tile +- the summed dilations in LDS (reflect-padded edges
    inside the tile), h in registers. Same products, order, splits and epilogues as the two launches
    per stack: bit-identical to mstack off, at B = 1 (short utterances: every block touches an edge;
    T' = 64 and 131) and on a forced ragged batch, also on one stream (workspace slots reused across
    buffers, the chain's input kept live through the fused launch); the chains ran fused (their
    inner ops record no launch)."""
    from parallelwavegan_amd import configs, synthetic
    from parallelwavegan_amd.melgan import PQMF, MelGANGenerator

    _, params = configs.vocoder_params(cfg)
    m = MelGANGenerator(**params)
    m.load_state_dict({k: torch.from_numpy(v) for k, v in synthetic.make_module_state_dict(m, seed=31).items()})
    if cfg in configs.VOCODER_PQMF:
        m.pqmf = PQMF(**configs.VOCODER_PQMF[cfg])
    m = m.to(cuda_device)
    eng = m.engine()
    singles = [synthetic.make_mel(f, 80, seed=400 + f) for f in (64, 9, 131, 5)]
    batch = [synthetic.make_mel(f, 80, seed=410 + i) for i, f in enumerate([5, 40, 17, 64])]
    with torch.no_grad():
        outs = {}
        for mode in (0, 1):
            eng.set_mstack(mode)
            eng.set_timing(True)
            eng.collect_timing()
            outs[mode] = [m.inference(torch.from_numpy(x).to(cuda_device)).cpu().numpy() for x in singles]
            t = eng.collect_timing()
            eng.set_timing(False)
            outs[mode] += [y.cpu().numpy() for y in m.inference_batch(batch)]
            if mode == 1:
                fused = sum(1 for name, _, n in t if n == 0 and "stack" in name)
        # one stream: the plan's workspace slots are reused across buffers (assign_slots(true)), so
        # a chain's input and its output must not share a slot while the fused launch reads halos
        eng.set_mstack(1)
        eng.set_streams(0)
        outs["s0"] = [m.inference(torch.from_numpy(x).to(cuda_device)).cpu().numpy() for x in singles]
        outs["s0"] += [y.cpu().numpy() for y in m.inference_batch(batch)]
        eng.set_streams(1)
    assert fused > 0
    for mode in (1, "s0"):
        for a, b in zip(outs[mode], outs[0]):
            assert np.isfinite(a).all()
            np.testing.assert_array_equal(a, b)


@pytest.mark.parametrize("cfg", ["mb_melgan_v2", "hifigan_v1", "melgan_v1", "hifigan_causal_test"])
def test_presplit_images_bitwise_equal(cfg, built_lib, cuda_device):
    """PWG_CNET_OPT_PRESPLIT: DMA-ring and narrow x-tile launches whose inputs were written by DMA-ring
    or x-tile launches stage the writers' pre-split images (pre-activated, fp16 hi / lo rows) instead
    of converting the fp32 rows in every workgroup and step. The same conversion of the same values, done once: bit-identical
    to presplit off at B = 1 (short utterances: every block touches an edge; zero and reflect padding)
    and on a ragged batch, with fused stack chains on and off."""
    from parallelwavegan_amd import configs, synthetic
    from parallelwavegan_amd.hifigan import HiFiGANGenerator
    from parallelwavegan_amd.melgan import PQMF, MelGANGenerator

    cls, params = configs.vocoder_params(cfg)
    m = {"MelGANGenerator": MelGANGenerator, "HiFiGANGenerator": HiFiGANGenerator}[cls](**params)
    m.load_state_dict({k: torch.from_numpy(v) for k, v in synthetic.make_module_state_dict(m, seed=37).items()})
    if cfg in configs.VOCODER_PQMF:
        m.pqmf = PQMF(**configs.VOCODER_PQMF[cfg])
    m = m.to(cuda_device)
    eng = m.engine()
    # (131 and 300 frames: HiFiGAN's 128- and 64-channel stages on the narrow x-tile kernel, which
    # reads images written by the x-tile kernels' epilogue)
    singles = [synthetic.make_mel(f, 80, seed=500 + f) for f in (64, 9, 131, 5, 300)]
    batch = [synthetic.make_mel(f, 80, seed=510 + i) for i, f in enumerate([5, 40, 17, 64])]
    with torch.no_grad():
        outs = {}
        for ms in (1, 0):
            eng.set_mstack(ms)
            for pre in (0, 1):
                eng.set_presplit(pre)
                outs[ms, pre] = [m.inference(torch.from_numpy(x).to(cuda_device)).cpu().numpy() for x in singles]
                outs[ms, pre] += [y.cpu().numpy() for y in m.inference_batch(batch)]
        eng.set_presplit(1)
        eng.set_mstack(1)
    for ms in (1, 0):
        for a, b in zip(outs[ms, 1], outs[ms, 0]):
            assert np.isfinite(a).all()
            np.testing.assert_array_equal(a, b)


@pytest.mark.parametrize("cfg", ["mb_melgan_v2", "melgan_v1", "mb_melgan_v2_causal"])
def test_rstack_bitwise_equal_on_a_large_batch(cfg, built_lib, cuda_device):
    """PWG_CNET_OPT_RSTACK: the batched ResidualStack kernel (pwg_rstack.hip: persistent workgroups,
    LDS ring of weights and raw rows two steps ahead across tiles -- or, <= 64 channels, the weights
    resident in LDS and only rows in the ring --, rows converted in place, h and x operands in
    registers), both forms, against the x-tile stack kernel on a ragged batch big enough for several
    tiles per workgroup (8 utterances of the bench's LibriTTS lengths, 1-2 rounds over the CUs at
    every stage), reflect and causal padding: bit-identical, and every stack ran on the ring
    kernels (the wide stages' k = 3 conv and 1x1 on pwg_rconv_kernel / pwg_r1x1_kernel, modes 1
    and 2 only; mode 0 keeps the x-tile and tap-major kernels)."""
    from parallelwavegan_amd import configs, synthetic
    from parallelwavegan_amd.melgan import PQMF, MelGANGenerator

    _, params = configs.vocoder_params(cfg)
    m = MelGANGenerator(**params)
    m.load_state_dict({k: torch.from_numpy(v) for k, v in synthetic.make_module_state_dict(m, seed=41).items()})
    if cfg in configs.VOCODER_PQMF:
        m.pqmf = PQMF(**configs.VOCODER_PQMF[cfg])
    m = m.to(cuda_device)
    eng = m.engine()
    lengths = [int(f) for f in synthetic.libritts_lengths(8, seed=5)] + [11, 9]
    mels = [synthetic.make_mel(f, 80, seed=500 + i) for i, f in enumerate(lengths)]
    with torch.no_grad():
        eng.set_rstack(0)
        ref = [y.cpu().numpy() for y in m.inference_batch(mels)]
        eng.set_rstack(2)  # weights streamed at every width
        streamed = [y.cpu().numpy() for y in m.inference_batch(mels)]
        eng.set_rstack(1)  # weights resident at <= 64 channels (the default)
        n0 = _rstack_launches()
        got = [y.cpu().numpy() for y in m.inference_batch(mels)]
    # every ResidualStack of the batch on the ring kernels: <= 96 channels one fused launch per stack,
    # 128-256 channels two (pwg_rconv_kernel + pwg_r1x1_kernel)
    chans = [params["channels"] >> (i + 1) for i in range(len(params["upsample_scales"]))]
    want = sum(params["stacks"] * (1 if c <= 96 else 2) for c in chans)
    assert _rstack_launches() - n0 == want, "the ring stack kernels did not all run"
    for a, b, c in zip(got, ref, streamed):
        assert np.isfinite(a).all()
        np.testing.assert_array_equal(a, b)
        np.testing.assert_array_equal(c, b)


@pytest.mark.parametrize("cfg, frames", [("mb_melgan_v2", 64), ("melgan_v1", 48), ("mb_melgan_test", 40)])
def test_fused_chains_and_presplit_against_oracle(cfg, frames, built_lib, cuda_device):
    """The B = 1 path's own kernels against the float64 oracle (oracle/melgan_numpy.py), not only
    against the executor's other launches: a short utterance with PWG_CNET_OPT_MSTACK 1 (each
    stage's ResidualStack chain as one pwg_mstack.hip launch) and PWG_CNET_OPT_PRESPLIT 1 (DMA-ring
    launches reading pre-split images), both asserted engaged, |d| < 1e-4."""
    from oracle import melgan_numpy
    from parallelwavegan_amd import configs, synthetic
    from parallelwavegan_amd.engine import fold_weight_norm
    from parallelwavegan_amd.melgan import PQMF, MelGANGenerator

    _, params = configs.vocoder_params(cfg)
    m = MelGANGenerator(**params)
    sd = synthetic.make_module_state_dict(m, seed=13)
    m.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()})
    syn = None
    if cfg in configs.VOCODER_PQMF:
        m.pqmf = PQMF(**configs.VOCODER_PQMF[cfg])
        syn = m.pqmf.synthesis_taps()
    m = m.to(cuda_device)
    eng = m.engine()
    eng.set_mstack(1)
    eng.set_presplit(False)
    ws_plain = eng.plan([frames]).workspace_bytes
    eng.set_presplit(True)
    assert eng.plan([frames]).workspace_bytes > ws_plain, "no pre-split images in the B = 1 plan"
    mel = synthetic.make_mel(frames, 80, seed=17)
    with torch.no_grad():
        eng.set_timing(True)
        eng.collect_timing()
        y = m.inference(mel).cpu().numpy()
        t = eng.collect_timing()
        eng.set_timing(False)
    assert sum(1 for name, _, n in t if n == 0 and "stack" in name) > 0, "no fused stack chain ran"
    ref = melgan_numpy.melgan_inference(mel, fold_weight_norm(sd), params, syn)
    assert y.shape == ref.shape
    err = np.abs(y - ref).max()
    assert err < ATOL, f"{cfg}: max|d| = {err:.3e}"


def test_release_stream_then_reuse(built_lib, cuda_device):
    """pwg_cnet_release_stream: a caller stream's auxiliary streams, events and pinned status word
    are freed on request; the next run on that stream builds them again and gives the same bits
    (HiFiGAN v1 at B = 1: concurrent branches on the auxiliary streams)."""
    from parallelwavegan_amd import configs, synthetic
    from parallelwavegan_amd.hifigan import HiFiGANGenerator

    _, params = configs.vocoder_params("hifigan_v1")
    m = HiFiGANGenerator(**params)
    m.load_state_dict({k: torch.from_numpy(v) for k, v in synthetic.make_module_state_dict(m, seed=51).items()})
    m = m.to(cuda_device)
    eng = m.engine()
    mel = torch.from_numpy(synthetic.make_mel(40, 80, seed=52)).to(cuda_device)
    s = torch.cuda.Stream(cuda_device)
    with torch.no_grad(), torch.cuda.stream(s):
        a = m.inference(mel).cpu().numpy()
        eng.release_stream(s)
        b = m.inference(mel).cpu().numpy()
        eng.release_stream(s)
    np.testing.assert_array_equal(a, b)
