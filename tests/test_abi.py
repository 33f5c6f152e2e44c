"""The C-ABI library builds, loads and exports every symbol include/pwg.h declares; host-side
logic (config validation -> exception mapping, weight counts, packing) behaves. CPU only: no
call here launches a kernel or touches device memory."""

import ctypes
import os
import re

import numpy as np
import pytest

from conftest import REPO
from parallelwavegan_amd import _lib, configs, synthetic
from parallelwavegan_amd.engine import HostHandle, make_config, ref_weight_keys


def _declared_symbols():
    import glob

    src = "".join(open(p).read() for p in sorted(glob.glob(os.path.join(REPO, "include", "*.h"))))
    return sorted(set(re.findall(r"PWG_API\s+[\w\s\*]+?\b(pwg_\w+)\s*\(", src)))


def test_header_declarations_match_binding_list():
    assert _declared_symbols() == sorted(_lib.EXPORTED_SYMBOLS)


def test_library_exports_every_declared_symbol(built_lib):
    for name in _declared_symbols():
        assert hasattr(built_lib, name), name
        assert ctypes.cast(getattr(built_lib, name), ctypes.c_void_p).value


def test_library_exports_nothing_else(built_lib):
    import subprocess

    out = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True, text=True).stdout
    exported = sorted({ln.split()[-1] for ln in out.splitlines() if " T " in ln})
    assert exported == sorted(_lib.EXPORTED_SYMBOLS)


def test_library_is_gfx950_code_object(built_lib):
    blob = open(_lib.LIB_PATH, "rb").read()
    assert b"gfx950" in blob


def test_abi_version(built_lib):
    assert built_lib.pwg_abi_version() == 2  # 2: PwgConfig.interpolate_mode


@pytest.mark.parametrize("name", ["yesno_debug", "ljspeech_v1", "libritts_v1", "reference_test"])
def test_weight_counts_match_state_dict(built_lib, name):
    params = configs.generator_params(name)
    h = HostHandle(params)
    n = sum(int(np.prod(s)) for _, s in synthetic.parameter_shapes(params))
    assert h.ref_weight_count == n
    keys = [k for k, _ in ref_weight_keys(params) if k is not None]
    assert sorted(keys) == sorted(k for k, _ in synthetic.parameter_shapes(params))


def test_receptive_field_and_upsample_factor(built_lib):
    h = HostHandle(configs.generator_params("ljspeech_v1"))
    assert h.receptive_field_size == 6139  # models/parallel_wavegan.py:197-211, SURVEY a14
    assert h.upsample_factor == 256
    h = HostHandle(configs.generator_params("yesno_debug"))
    assert h.receptive_field_size == 4093  # 2*(2*1023)+1 (SURVEY a14 says 2047: miscount)
    assert HostHandle(configs.generator_params("libritts_v1")).upsample_factor == 300


@pytest.mark.parametrize(
    "override, exc",
    [
        (dict(layers=10, stacks=3), AssertionError),  # parallel_wavegan.py:77
        (dict(kernel_size=4), AssertionError),  # residual_block.py:77
        (dict(in_channels=2), NotImplementedError),
        (dict(gate_channels=512), NotImplementedError),
        (dict(gate_channels=7), ValueError),
        (dict(upsample_net="MelGANGenerator"), NotImplementedError),
        (dict(upsample_params={"upsample_scales": [4], "nonlinear_activation": "ReLU"}), NotImplementedError),
        (dict(upsample_params={"upsample_scales": [4], "freq_axis_kernel_size": 3}), NotImplementedError),
    ],
)
def test_invalid_configs_raise_reference_exceptions(built_lib, override, exc):
    params = configs.generator_params("ljspeech_v1", **override)
    with pytest.raises(exc):
        HostHandle(params)


def _ref_pack_gate(wd, G, R, KS, lane, s, m):
    """Independent restatement of the gate A-fragment element (pwg_kernels.hip, GEMM 1): K rows
    are tap blocks of RP = ceil(R/16)*16 channels, gate rows packed [Za | pad | Zb | pad]."""
    GH = G // 2
    GHPAD = 16 if GH <= 16 else (GH + 31) // 32 * 32
    RP = (R + 15) // 16 * 16
    prow = 32 * m + (lane & 31)
    k = 2 * s + (lane >> 5)
    grow = (prow if prow < GH else None) if prow < GHPAD else (GH + prow - GHPAD if prow - GHPAD < GH else None)
    tap, ch = k // RP, k % RP
    if grow is None or ch >= R:
        return 0.0
    return wd[grow, ch, tap]


@pytest.mark.parametrize("name", ["reference_test", "ljspeech_v1"])
def test_pack_gate_fragments(built_lib, name):
    params = configs.generator_params(name)
    h = HostHandle(params)
    sd = synthetic.make_state_dict(params, seed=0)
    packed = h.pack(sd)
    assert packed.shape == (h.packed_weight_count,)
    assert np.isfinite(packed).all()
    wd = sd["conv_layers.0.conv.weight"]
    G, R, KS = wd.shape
    GH = G // 2
    MT = 1 if GH <= 16 else (GH + 31) // 32 * 32 // 16
    RP = (R + 15) // 16 * 16
    # locate the first layer's first fragment in the image by value, then check all of them
    f = np.asarray([_ref_pack_gate(wd, G, R, KS, lane, 0, 0) for lane in range(64)], np.float32)
    hits = [i for i in range(0, packed.size - 64, 64) if np.array_equal(packed[i:i + 64], f)]
    assert len(hits) == 1
    base = hits[0]
    for s in range(KS * RP // 2):
        for m in range(MT):
            frag = packed[base + (s * MT + m) * 64: base + (s * MT + m + 1) * 64]
            ref = [_ref_pack_gate(wd, G, R, KS, lane, s, m) for lane in range(64)]
            np.testing.assert_array_equal(frag, np.asarray(ref, np.float32))


def test_pack_rejects_missing_weights(built_lib):
    params = configs.generator_params("reference_test")
    sd = synthetic.make_state_dict(params, seed=0)
    del sd["conv_layers.3.conv1x1_aux.weight"]
    with pytest.raises(KeyError):
        HostHandle(params).pack(sd)


def test_weight_norm_state_packs_like_folded(built_lib):
    params = configs.generator_params("reference_test")
    wn = synthetic.make_state_dict(params, seed=0, weight_norm=True)
    from oracle.pwg_numpy import fold_weight_norm

    folded = {k: np.asarray(v, np.float32) for k, v in fold_weight_norm(wn).items()}
    h = HostHandle(params)
    np.testing.assert_allclose(h.pack(wn), h.pack(folded), rtol=2e-7, atol=1e-7)


def test_config_translation():
    cfg = make_config(configs.generator_params("libritts_v1"))
    assert list(cfg.upsample_scales)[: cfg.num_scales] == [4, 5, 3, 5]
    assert cfg.use_conv_in == 1 and cfg.aux_context_window == 2


def test_pack_reports_fp16_pair_range(built_lib):
    """pwg_pack_weights returns PWG_ERR_RANGE (image still complete for the exact-fp32 kernels)
    when a weight of the split-f16 images leaves the fp16 range; in-range weights pack clean."""
    params = configs.generator_params("libritts_v1")
    h = HostHandle(params)
    sd = synthetic.make_state_dict(params, seed=0)
    ok = h.pack(sd)
    assert h.split_range_ok
    sd["conv_layers.3.conv.weight"] = sd["conv_layers.3.conv.weight"].copy()
    sd["conv_layers.3.conv.weight"][5, 7, 1] = 7e4
    bad = h.pack(sd)
    assert not h.split_range_ok
    assert "fp16" in built_lib.pwg_last_error().decode()
    assert np.isfinite(ok).all() and bad.shape == ok.shape


def test_get_option_reports_default_layer_kernel(built_lib):
    for name, kernel in (("libritts_v1", 3), ("yesno_debug", 0), ("reference_test", 0)):
        h = HostHandle(configs.generator_params(name))
        v = ctypes.c_longlong()
        _lib.check(built_lib.pwg_get_option(h._h, _lib.PWG_OPT_LAYER_KERNEL, ctypes.byref(v)))
        assert v.value == kernel, name


def test_sync_options_round_trip_and_validate(built_lib):
    """PWG_OPT_SYNC (grid-synchronised plan limit, >= 0), PWG_OPT_SYNC_ABORT and PWG_OPT_SYNC_TIMEOUT
    (test hooks, 0/1):
    set / get round trip and argument checks, host-only; the error codes map to the Python
    exceptions (PWG_ERR_RERUN -> RerunError)."""
    h = HostHandle(configs.generator_params("ljspeech_v1"))
    v = ctypes.c_longlong()
    for opt, good, bad in ((_lib.PWG_OPT_SYNC, (0, 4096, 1 << 40), (-1,)),
                           (_lib.PWG_OPT_SYNC_ABORT, (0, 1), (2, -1)),
                           (_lib.PWG_OPT_SYNC_TIMEOUT, (0, 1), (2, -1))):
        for val in good:
            _lib.check(built_lib.pwg_set_option(h._h, opt, val))
            _lib.check(built_lib.pwg_get_option(h._h, opt, ctypes.byref(v)))
            assert v.value == val
        for val in bad:
            assert built_lib.pwg_set_option(h._h, opt, val) == _lib.PWG_ERR_INVALID
    assert _lib._ERRORS[_lib.PWG_ERR_RERUN] is _lib.RerunError
    assert issubclass(_lib.RerunError, RuntimeError)


def test_rccl_entry_points_validate_arguments(built_lib):
    """Argument checks of the RCCL entries need no GPU (no communicator is created)."""
    assert built_lib.pwg_rccl_unique_id(None) == _lib.PWG_ERR_INVALID
    comm = ctypes.c_void_p()
    assert built_lib.pwg_rccl_comm_create(2, None, 0, 0, ctypes.byref(comm)) == _lib.PWG_ERR_INVALID
    buf = ctypes.create_string_buffer(_lib.PWG_RCCL_UNIQUE_ID_BYTES)
    assert built_lib.pwg_rccl_comm_create(2, buf, 2, 0, ctypes.byref(comm)) == _lib.PWG_ERR_INVALID
    assert built_lib.pwg_broadcast_weights(None, None, 0, None, None) == _lib.PWG_ERR_INVALID
    assert built_lib.pwg_rccl_comm_destroy(None) == _lib.PWG_OK


def test_interpolate_modes(built_lib):
    """Stretch2d interpolate_mode (layers/upsample.py:43-45, 62-128): "nearest", "nearest-exact" and
    "area" are the same map at integer scales, "bilinear" is linear along time; the handle builds
    and verifies its composite upsampler tables for each (pwg_create fails otherwise). Bilinear at a
    scale that is not a power of two, and other modes, are refused: aten computes the bilinear
    source index in fp32, exact only at power-of-two scales."""
    for cfg, scales in (("ljspeech_v1", [4, 4, 4, 4]), ("reference_test", [8, 2]), ("reference_test", [4, 4])):
        for mode in ("nearest", "nearest-exact", "area", "bilinear"):
            for causal in (False, True):
                p = configs.generator_params(cfg, use_causal_conv=causal,
                                             upsample_params={"upsample_scales": scales, "interpolate_mode": mode})
                h = HostHandle(p)
                assert h.config.interpolate_mode == (1 if mode == "bilinear" else 0)
    with pytest.raises(NotImplementedError, match="power-of-two"):
        HostHandle(configs.generator_params("libritts_v1", upsample_params={"upsample_scales": [4, 5, 3, 5],
                                                                             "interpolate_mode": "bilinear"}))
    for mode in ("bicubic", "linear", "trilinear"):
        with pytest.raises(NotImplementedError):
            HostHandle(configs.generator_params("ljspeech_v1", upsample_params={"upsample_scales": [4, 4, 4, 4],
                                                                                 "interpolate_mode": mode}))


def test_release_stream_entry_points(built_lib):
    """pwg_release_stream / pwg_cnet_release_stream (per-caller-stream resources): a null handle is
    PWG_ERR_INVALID; an unknown stream, and any stream of a host-only conv-network handle, is a no-op."""
    import ctypes

    from parallelwavegan_amd import configs as cfgs
    from parallelwavegan_amd.cnet import CnetEngine
    from parallelwavegan_amd.melgan import MelGANGenerator

    assert built_lib.pwg_release_stream(None, None) == _lib.PWG_ERR_INVALID
    L = built_lib
    L.pwg_cnet_release_stream.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
    assert L.pwg_cnet_release_stream(None, None) == _lib.PWG_ERR_INVALID
    _, p = cfgs.vocoder_params("mb_melgan_test")
    P, _ = MelGANGenerator(**p).program(False)
    eng = CnetEngine(P, None, host_only=True)
    assert L.pwg_cnet_release_stream(eng._h, ctypes.c_void_p(1234)) == _lib.PWG_OK


def test_engine_classes_carry_their_methods():
    """The engines' GPU methods are only exercised by `-m gpu` tests: check here that the classes
    still own them (a module-level def dropped into a class body silently ends the class)."""
    from parallelwavegan_amd.cnet import CnetEngine
    from parallelwavegan_amd.engine import Engine, warm_batch_kernels

    for name in ("load_state_dict", "set_packed", "reserve_workspace", "plan", "workspace", "set_option",
                 "get_option", "run", "run_status", "release_stream"):
        assert callable(getattr(Engine, name, None)), name
    for name in ("load_state_dict", "reserve_workspace", "release_stream", "set_rstack"):
        assert callable(getattr(CnetEngine, name, None)), name
    assert callable(warm_batch_kernels)
