"""Generator configurations of the benchmark recipes (``generator_params`` blocks).

Values are restated from the reference recipe YAMLs:
  yesno_debug  egs/yesno/voc1/conf/parallel_wavegan.v1.debug.yaml:26-44 (fs 8 kHz, hop 256)
  ljspeech_v1  egs/ljspeech/voc1/conf/parallel_wavegan.v1.yaml:28-46   (fs 22.05 kHz, hop 256)
  libritts_v1  egs/libritts/voc1/conf/parallel_wavegan.v1.yaml:28-46   (fs 24 kHz, hop 300)
``reference_test`` is the small generator of the reference unit tests
(test/test_parallel_wavegan.py:31-51) with dropout removed.
"""

import copy

_PWG_V1 = dict(
    in_channels=1,
    out_channels=1,
    kernel_size=3,
    layers=30,
    stacks=3,
    residual_channels=64,
    gate_channels=128,
    skip_channels=64,
    aux_channels=80,
    aux_context_window=2,
    dropout=0.0,
    use_weight_norm=True,
    upsample_net="ConvInUpsampleNetwork",
    upsample_params={"upsample_scales": [4, 4, 4, 4]},
)

GENERATOR_PARAMS = {
    "yesno_debug": dict(
        _PWG_V1,
        layers=20,
        stacks=2,
        residual_channels=16,
        gate_channels=32,
        skip_channels=16,
        aux_context_window=1,
    ),
    "ljspeech_v1": dict(_PWG_V1),
    "libritts_v1": dict(_PWG_V1, upsample_params={"upsample_scales": [4, 5, 3, 5]}),
    "reference_test": dict(
        in_channels=1,
        out_channels=1,
        kernel_size=3,
        layers=6,
        stacks=3,
        residual_channels=8,
        gate_channels=16,
        skip_channels=8,
        aux_channels=10,
        aux_context_window=2,
        dropout=0.0,
        use_weight_norm=True,
        use_causal_conv=False,
        upsample_conditional_features=True,
        upsample_net="ConvInUpsampleNetwork",
        upsample_params={"upsample_scales": [4, 4]},
    ),
}

SAMPLING_RATE = {
    "yesno_debug": 8000,
    "ljspeech_v1": 22050,
    "libritts_v1": 24000,
    "reference_test": 16000,
}


def generator_params(name, **overrides):
    """Deep copy of a recipe's generator_params (the constructor mutates upsample_params,
    models/parallel_wavegan.py:85-107, so callers must never share the dict)."""
    p = copy.deepcopy(GENERATOR_PARAMS[name])
    p.update(copy.deepcopy(overrides))
    return p


# MelGAN-family generators, executed by the conv-network engine.
#   melgan_v1     egs/ljspeech/voc1/conf/melgan.v1.yaml (generator_params)
#   mb_melgan_v2  egs/ljspeech/voc1/conf/multi_band_melgan.v2.yaml:38-48, + PQMF(4) synthesis
#   hifigan_v1    egs/ljspeech/voc1/conf/hifigan.v1.yaml:32-50
# ``*_test`` are reduced shapes for parity fixtures (same code paths, seconds on the oracle).
VOCODER_PARAMS = {
    "melgan_v1": ("MelGANGenerator", dict(in_channels=80, out_channels=1, kernel_size=7, channels=512,
                                          upsample_scales=[8, 8, 2, 2], stack_kernel_size=3, stacks=3,
                                          use_weight_norm=True, use_causal_conv=False)),
    "mb_melgan_v2": ("MelGANGenerator", dict(in_channels=80, out_channels=4, kernel_size=7, channels=384,
                                             upsample_scales=[8, 4, 2], stack_kernel_size=3, stacks=4,
                                             use_weight_norm=True, use_causal_conv=False)),
    "hifigan_v1": ("HiFiGANGenerator", dict(in_channels=80, out_channels=1, channels=512, kernel_size=7,
                                            upsample_scales=[8, 8, 2, 2], upsample_kernel_sizes=[16, 16, 4, 4],
                                            resblock_kernel_sizes=[3, 7, 11],
                                            resblock_dilations=[[1, 3, 5], [1, 3, 5], [1, 3, 5]],
                                            use_additional_convs=True, bias=True,
                                            nonlinear_activation="LeakyReLU",
                                            nonlinear_activation_params={"negative_slope": 0.1},
                                            use_weight_norm=True)),
    "mb_melgan_test": ("MelGANGenerator", dict(in_channels=80, out_channels=4, kernel_size=7, channels=64,
                                               upsample_scales=[4, 2], stack_kernel_size=3, stacks=3,
                                               use_weight_norm=True, use_causal_conv=False)),
    "melgan_test": ("MelGANGenerator", dict(in_channels=80, out_channels=1, kernel_size=7, channels=96,
                                            upsample_scales=[3, 2, 2], stack_kernel_size=3, stacks=2,
                                            use_weight_norm=True, use_causal_conv=False)),
    "hifigan_test": ("HiFiGANGenerator", dict(in_channels=80, out_channels=1, channels=64, kernel_size=7,
                                              upsample_scales=[4, 2], upsample_kernel_sizes=[8, 4],
                                              resblock_kernel_sizes=[3, 5], resblock_dilations=[[1, 3], [1, 2]],
                                              use_additional_convs=True, bias=True,
                                              nonlinear_activation="LeakyReLU",
                                              nonlinear_activation_params={"negative_slope": 0.1},
                                              use_weight_norm=True)),
    "hifigan_noadd_test": ("HiFiGANGenerator", dict(in_channels=80, out_channels=1, channels=32, kernel_size=5,
                                                    upsample_scales=[3], upsample_kernel_sizes=[6],
                                                    resblock_kernel_sizes=[3, 5, 7],
                                                    resblock_dilations=[[1, 3], [1, 2], [2, 1]],
                                                    use_additional_convs=False, bias=True,
                                                    nonlinear_activation="LeakyReLU",
                                                    nonlinear_activation_params={"negative_slope": 0.1},
                                                    use_weight_norm=True)),
}

def _causal(name, **over):
    cls, p = VOCODER_PARAMS[name]
    p = copy.deepcopy(p)
    p.update(use_causal_conv=True, **over)
    return cls, p


# causal variants (models/melgan.py:73-151, models/hifigan.py:83-164, layers/causal_conv.py;
# the reference's causality tests use odd and mixed upsample scales, test/test_hifigan.py:163-196,
# test/test_melgan.py:267-274)
VOCODER_PARAMS.update({
    "melgan_causal_test": _causal("melgan_test"),
    "mb_melgan_causal_test": _causal("mb_melgan_test", upsample_scales=[3, 2]),
    "hifigan_causal_test": _causal("hifigan_test", upsample_scales=[5, 3], upsample_kernel_sizes=[10, 6]),
    "hifigan_noadd_causal_test": _causal("hifigan_noadd_test"),
    "mb_melgan_v2_causal": _causal("mb_melgan_v2"),
    "hifigan_v1_causal": _causal("hifigan_v1"),
    "melgan_v1_causal": _causal("melgan_v1"),
})
VOCODER_PQMF = {"mb_melgan_v2": dict(subbands=4), "mb_melgan_test": dict(subbands=4),
                "mb_melgan_v2_causal": dict(subbands=4), "mb_melgan_causal_test": dict(subbands=4)}
SAMPLING_RATE.update(melgan_v1=22050, mb_melgan_v2=22050, hifigan_v1=22050)


def vocoder_params(name, **overrides):
    """(generator class name, deep-copied generator_params) of a MelGAN-family recipe."""
    cls, p = VOCODER_PARAMS[name]
    p = copy.deepcopy(p)
    p.update(copy.deepcopy(overrides))
    return cls, p
