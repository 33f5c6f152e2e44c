"""Host side of the conv-network executor (include/pwg_cnet.h) for the MelGAN-family drop-ins:
program lowering, reference-order flattening, fragment packing and argument validation. CPU only:
nothing here touches device memory."""

import numpy as np
import pytest
import torch

from conftest import vocoder_golden_names, vocoder_holder, load_golden
from parallelwavegan_amd import cnet, configs, synthetic
from parallelwavegan_amd.hifigan import HiFiGANGenerator
from parallelwavegan_amd.melgan import PQMF, MelGANGenerator


def _holder(name):
    cls, p = configs.vocoder_params(name)
    return {"MelGANGenerator": MelGANGenerator, "HiFiGANGenerator": HiFiGANGenerator}[cls](**p)


@pytest.mark.parametrize("name", ["mb_melgan_v2", "melgan_v1", "hifigan_v1", "mb_melgan_test", "hifigan_noadd_test",
                                  "mb_melgan_v2_causal", "hifigan_v1_causal", "hifigan_causal_test"])
def test_program_covers_every_weight_and_packs(name, built_lib):
    m = _holder(name)
    if isinstance(m, MelGANGenerator) and m.out_channels > 1:
        m.pqmf = PQMF(m.out_channels)
        P, extra = m.program(True)
    elif isinstance(m, MelGANGenerator):
        P, extra = m.program(False)
    else:
        P, extra = m.program(), {}
    sd = synthetic.make_module_state_dict(m, seed=0)
    from parallelwavegan_amd.engine import fold_weight_norm

    folded = fold_weight_norm(sd)
    # every parameter of the module is consumed exactly once by the program
    assert set(k for k in P.weights if k not in extra) == set(folded)
    eng = cnet.CnetEngine(P, None, host_only=True)
    packed = eng.pack(sd, extra)
    assert packed.shape == (eng.packed_weight_count,)
    assert np.isfinite(packed).all()
    # the fragments hold every weight value (plus zero padding): compare sums of |w|
    _, n_ref = P.offsets()
    flat = P.flatten(sd, extra)
    assert flat.size == n_ref
    # the output is the last buffer with the generator's hop
    hop = m.upsample_factor * (m.pqmf.subbands if isinstance(m, MelGANGenerator) and m.pqmf is not None else 1)
    assert P.rate[-1] == hop


def test_convt_fragment_layout(built_lib):
    """One ConvTranspose1d op: phase r uses taps k_a = (r+p) % s and k_a + s of W (C_in, C_out, 2s)."""
    P = cnet.Program(16)
    out = P.buffer(32, 4)
    P.convt("ct", out, 32, P.src(0, 16, weight="w"), 4, 2, 0, bias="b")
    rs = np.random.RandomState(0)
    w = rs.standard_normal((16, 32, 8)).astype(np.float32)
    b = rs.standard_normal(32).astype(np.float32)
    eng = cnet.CnetEngine(P, None, host_only=True)
    packed = eng.pack({"w": w, "b": b})
    # 2 chunks (taps) x 1 m-tile x 512 floats, fp32 fragments then split-f16 fragments, + bias
    per_phase = 2 * 2 * 1 * 512 + 32
    assert eng.packed_weight_count == 4 * per_phase
    for r in range(4):
        base = r * per_phase
        ka = (r + 2) % 4
        for tap in range(2):
            frag = packed[base + tap * 512: base + (tap + 1) * 512].reshape(2, 64, 4)
            for lane in (0, 5, 33, 63):
                for i in range(8):
                    sub, e = divmod(i, 4)
                    o = lane & 31
                    ch = i + 8 * (lane >> 5)
                    assert frag[sub, lane, e] == w[ch, o, ka + tap * 4]
            # split-f16 fragment of the same chunk: [hi/lo][lane][8 halves], channel 8*(lane>>5) + j
            f16 = packed[base + 1024 + tap * 512: base + 1024 + (tap + 1) * 512].view(np.float16).reshape(2, 64, 8)
            for lane in (0, 5, 33, 63):
                for j in range(8):
                    want = w[8 * (lane >> 5) + j, lane & 31, ka + tap * 4]
                    hi, lo = f16[0, lane, j], f16[1, lane, j]
                    assert hi == np.float16(want)
                    # ~22 significant bits; an fp16-subnormal lo still resolves 2^-25 absolute
                    assert abs(float(hi) + float(lo) - float(want)) <= max(2.0 ** -21 * abs(float(want)), 2.0 ** -25)
        np.testing.assert_array_equal(packed[base + 2048: base + 2080], b)


@pytest.mark.parametrize("bad", ["rate", "channels", "dst", "convt_pad", "causal_convt_pad", "convt_reflect"])
def test_invalid_programs_raise(bad, built_lib):
    P = cnet.Program(16)
    if bad == "rate":
        out = P.buffer(8, 2)
        P.conv("c", out, 8, [P.src(0, 16, weight="w")])
    elif bad == "channels":
        out = P.buffer(8, 1)
        P.conv("c", out, 8, [P.src(0, 32, weight="w")])
    elif bad == "dst":
        out = P.buffer(4, 1)
        P.conv("c", out, 8, [P.src(0, 16, weight="w")])
    elif bad == "convt_pad":
        out = P.buffer(8, 4)
        P.convt("c", out, 8, P.src(0, 16, weight="w"), 4, 1, 0)
    elif bad == "causal_convt_pad":  # the causal (replicate-padded) form has no padding
        out = P.buffer(8, 4)
        P.convt("c", out, 8, P.src(0, 16, weight="w", pad_mode=cnet.PAD_REPLICATE), 4, 2, 0)
    else:
        out = P.buffer(8, 4)
        P.convt("c", out, 8, P.src(0, 16, weight="w", pad_mode=cnet.PAD_REFLECT), 4, 2, 0)
    with pytest.raises((ValueError, NotImplementedError)):
        cnet.CnetEngine(P, None, host_only=True)


def test_causal_lowering(built_lib):
    """CausalConv1d -> pad (K-1)*dil with the pad module's edge mode; CausalConvTranspose1d -> a
    CONVT op with padding 0 and a replicate-padded source (layers/causal_conv.py:12-78)."""
    m = _holder("mb_melgan_causal_test")
    P, _ = m.program(False)
    first = P.ops[0]["srcs"][0]
    assert (first["taps"], first["pad"], first["pad_mode"], first["normalize"]) == (7, 6, cnet.PAD_REFLECT, True)
    convts = [op for op in P.ops if op["kind"] == cnet.CONVT]
    assert convts and all(op["padding"] == 0 and op["srcs"][0]["pad_mode"] == cnet.PAD_REPLICATE for op in convts)
    dil = [op["srcs"][0] for op in P.ops if op["srcs"][0]["dilation"] > 1]
    assert dil and all(s["pad"] == (s["taps"] - 1) * s["dilation"] for s in dil)
    h = _holder("hifigan_causal_test")
    assert all(op["srcs"][0]["pad_mode"] == cnet.PAD_ZERO for op in h.program().ops if op["kind"] == cnet.CONV)


def test_unsupported_modules_raise():
    # a causal conv padded with a non-zero constant has no engine edge mode
    m = MelGANGenerator(**configs.vocoder_params("melgan_causal_test", pad="ConstantPad1d",
                                                 pad_params={"value": 1.0})[1])
    with pytest.raises(NotImplementedError):
        m.program(False)
    with pytest.raises(NotImplementedError):
        MelGANGenerator(**configs.vocoder_params("melgan_test", nonlinear_activation="ELU",
                                                 nonlinear_activation_params={}) [1]).program(False)


def test_cpu_module_fails_loudly(built_lib):
    m = _holder("mb_melgan_test")
    with pytest.raises(RuntimeError):
        m.inference(np.zeros((8, 80), np.float32))


@pytest.mark.parametrize("name", vocoder_golden_names())
def test_fixture_state_dicts_load_into_dropins(name):
    m, params, folded = vocoder_holder(load_golden(name)["meta"])
    assert sum(p.numel() for p in m.parameters()) > 0


def test_plan_past_the_buffer_limit_is_refused(built_lib):
    """pwg_cnet_plan_create refuses a batch whose largest buffer would exceed 2^31 elements
    (int32 row offsets in the kernels, pwg_cnet.hip plan limit) before touching a GPU: HiFiGAN v1's
    32-channel stage at 256x frame rate holds 2^31 / 32 rows, i.e. 262,144 frames."""
    import pytest

    from parallelwavegan_amd import configs
    from parallelwavegan_amd.cnet import CnetEngine
    from parallelwavegan_amd.hifigan import HiFiGANGenerator

    _, params = configs.vocoder_params("hifigan_v1")
    P = HiFiGANGenerator(**params).program()
    eng = CnetEngine(P, None, host_only=True)
    with pytest.raises(NotImplementedError, match="too large"):
        eng.plan([262144])
    with pytest.raises(NotImplementedError, match="too large"):
        eng.plan([131072, 131072])
    with pytest.raises(ValueError):
        eng.plan([0])


@pytest.mark.parametrize("name", ["mb_melgan_v2", "melgan_v1", "hifigan_v1", "mb_melgan_v2_causal",
                                  "hifigan_v1_causal", "hifigan_causal_test"])
def test_host_only_plans_build_and_check_their_block_lists(name, built_lib):
    """pwg_cnet_plan_create on a host-only handle (device -1) runs the whole host side of the plan
    (buffer rows, workspace slots, every phase's block / strip / x-tile lists and their bounds
    check) without a GPU, so the plan builder runs here and under the sanitizers
    (tests/test_host_sanitized.py): ragged batches, the shortest utterances ReflectionPad1d allows, long utterances. A host-
    only plan refuses to run."""
    import ctypes

    from parallelwavegan_amd import _lib
    from parallelwavegan_amd.cnet import CnetEngine

    m = _holder(name)
    if isinstance(m, MelGANGenerator) and m.out_channels > 1:
        m.pqmf = PQMF(m.out_channels)
        P, _ = m.program(True)
    elif isinstance(m, MelGANGenerator):
        P, _ = m.program(False)
    else:
        P = m.program()
    eng = CnetEngine(P, None, host_only=True)
    hop = P.rate[-1]
    for frames in ([8], [9, 8, 10], [64], [80, 1199, 517], [2048] * 4, [9000]):  # MelGAN: reflect pads up to 6
        plan = eng.plan(frames)
        assert plan.out_rows == sum(frames) * hop
        assert plan.workspace_bytes >= 256
    p = eng.plan([16])
    rc = eng._lib.pwg_cnet_run(p._p, ctypes.c_void_p(16), ctypes.c_void_p(16), None, None, ctypes.c_void_p(16),
                               ctypes.c_void_p(256), None)
    assert rc == _lib.PWG_ERR_INVALID
    # launch options on the handle: PWG_CNET_OPT_NARROW (6) takes 0-2, PWG_CNET_OPT_NARROW_DMA (7) 0-1
    # (its mode 2 measured slower and was removed in round 6), PWG_CNET_OPT_RSTACK (11) 0-2
    eng.set_narrow(2)
    eng.set_narrow_dma(False)
    assert eng.plan([64]).out_rows == 64 * hop
    eng.set_narrow_dma(True)
    assert eng._lib.pwg_cnet_set_option(eng._h, 6, 3) == _lib.PWG_ERR_INVALID
    assert eng._lib.pwg_cnet_set_option(eng._h, 7, 2) == _lib.PWG_ERR_INVALID
    assert eng._lib.pwg_cnet_set_option(eng._h, 11, 3) == _lib.PWG_ERR_INVALID
    eng.set_rstack(0)
    eng.set_rstack(2)
    eng.set_rstack(1)
    assert eng.plan([64]).out_rows == 64 * hop


def test_concurrent_schedule_host_only(built_lib):
    """pwg_cnet_plan_schedule on a host-only plan: HiFiGAN v1 at B = 1 (narrow launches) spreads its
    multi-receptive-field branches over the caller's stream and auxiliary ones, the enqueue order is
    a permutation that keeps each stream's launches in program order and starts with the first
    launch; PWG_CNET_OPT_STREAMS 0 and a large plan (no narrow launches) stay on one stream in
    program order."""
    from parallelwavegan_amd.cnet import CnetEngine

    m = _holder("hifigan_v1")
    eng = CnetEngine(m.program(), None, host_only=True)
    launches, order = eng.schedule(eng.plan([64]))
    streams = {st for _, st in launches}
    assert len(streams) >= 3 and streams <= {0, 1, 2, 3}
    assert sorted(order) == list(range(len(launches))) and order[0] == 0
    pos = {L: i for i, L in enumerate(order)}
    for k in streams:
        ls = [L for L, (_, st) in enumerate(launches) if st == k]
        assert [pos[L] for L in ls] == sorted(pos[L] for L in ls)
    assert [ph for ph, _ in launches] == sorted(ph for ph, _ in launches)
    eng.set_streams(0)
    launches0, order0 = eng.schedule(eng.plan([64]))
    assert {st for _, st in launches0} == {0} and order0 == list(range(len(launches0)))
    eng.set_streams(1)
    big, order_big = eng.schedule(eng.plan([4000] * 8))
    assert {st for _, st in big} == {0} and order_big == list(range(len(big)))


@pytest.mark.parametrize("name", ["hifigan_v1", "mb_melgan_v2"])
def test_plan_image_is_host_built_and_cheap(name, built_lib):
    """Plans are host objects (include/pwg_cnet.h): their device lists are an image the descriptor
    kernel writes into the workspace every run. The host image has the segment lists of every
    buffer rate (first row, rows per utterance, back to back) and stays small for B = 1; building a
    plan for 32 distinct lengths (the reference's decode loop, bin/decode.py:236-268) costs host time
    only, well under a millisecond per plan."""
    import time

    from parallelwavegan_amd.cnet import CnetEngine

    m = _holder(name)
    if isinstance(m, MelGANGenerator):
        m.pqmf = PQMF(m.out_channels)
        P, _ = m.program(True)
    else:
        P = m.program()
    eng = CnetEngine(P, None, host_only=True)
    frames = [9, 130, 17]
    plan = eng.plan(frames)
    off, img = plan.image()
    assert off % 256 == 0 and off + 4 * img.size <= plan.workspace_bytes
    # the first list is buffer 0's segments (rate 1: frames)
    np.testing.assert_array_equal(img[:6], [0, 9, 9, 130, 139, 17])
    lens = np.random.RandomState(3).randint(80, 1200, 32)
    t0 = time.perf_counter()
    for f in lens:
        p = CnetEngine.plan(eng, [int(f)])
        assert p.image()[1].size < 64 * 1024
    per_plan_ms = (time.perf_counter() - t0) * 1e3 / len(lens)
    assert per_plan_ms < 5.0, per_plan_ms


def test_fused_stack_chains_in_the_schedule(built_lib):
    """PWG_CNET_OPT_MSTACK: MB-MelGAN v2's ResidualStacks form one chain per upsampling stage (4
    stacks: a k = 3 conv + the two-source 1x1 each). At B = 1, T' = 64 the chains of the 96- and
    48-channel stages run as one launch each (the 192-channel one stays unfused), so the plan's
    launches drop by 2 x (2 x 4 - 1); with the option off, or for a large plan, nothing changes
    (mode 2, every chain, measured slower and was removed in round 6)."""
    from parallelwavegan_amd.cnet import CnetEngine

    m = _holder("mb_melgan_v2")
    m.pqmf = PQMF(m.out_channels)
    P, _ = m.program(True)
    eng = CnetEngine(P, None, host_only=True)
    n_on = len(eng.schedule(eng.plan([64]))[0])
    eng.set_mstack(0)
    n_off = len(eng.schedule(eng.plan([64]))[0])
    assert n_off - n_on == 2 * (2 * 4 - 1), (n_off, n_on)
    big_off = len(eng.schedule(eng.plan([1000] * 8))[0])
    eng.set_mstack(1)
    assert len(eng.schedule(eng.plan([1000] * 8))[0]) == big_off

    from parallelwavegan_amd import _lib
    assert eng._lib.pwg_cnet_set_option(eng._h, 9, 2) == _lib.PWG_ERR_INVALID


@pytest.mark.parametrize("cfg", ["mb_melgan_v2", "hifigan_v1"])
def test_presplit_images_only_for_small_plans(cfg, built_lib):
    """PWG_CNET_OPT_PRESPLIT: a B = 1 plan (DMA-ring launches) reserves workspace for pre-split
    images of the buffers DMA-ring launches read from DMA-ring writers, each rows x channels x 4 B;
    a large batched plan (no narrow launches) reserves none; with the option off, none either."""
    from parallelwavegan_amd.cnet import CnetEngine

    m = _holder(cfg)
    if cfg == "mb_melgan_v2":
        m.pqmf = PQMF(m.out_channels)
        P, _ = m.program(True)
    else:
        P = m.program()
    P = P[0] if isinstance(P, tuple) else P
    eng = CnetEngine(P, None, host_only=True)
    on_small = eng.plan([64]).workspace_bytes
    on_big = eng.plan([1000] * 8).workspace_bytes
    eng.set_presplit(False)
    off_small = eng.plan([64]).workspace_bytes
    off_big = eng.plan([1000] * 8).workspace_bytes
    assert on_small > off_small, (on_small, off_small)
    assert on_big == off_big
    # every image is a multiple of one 64-frame buffer's rows x channels x 4 B (256-aligned)
    assert (on_small - off_small) % 256 == 0
