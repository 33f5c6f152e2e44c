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
