"""Seeded synthetic weights and inputs (there is no network for checkpoints or corpora).

Everything is drawn from ``numpy.random.RandomState`` (legacy MT19937, stream-stable across
numpy versions), so this container, the golden-fixture generator and the GPU box regenerate
bit-identical arrays from the same seeds.

Weights follow the reference initialisation in distribution: kaiming-normal (relu) convs
(layers/residual_block.py:26-30) and FIR taps near 1/(2s+1) (layers/upsample.py:55-59),
perturbed so every tap is distinct (a mirrored or shifted stencil then fails parity). Biases
are small non-zero values so the bias paths are exercised.
"""

import numpy as np


def _upsample_scales(params):
    return list(params.get("upsample_params", {}).get("upsample_scales", [4, 4, 4, 4]))


def parameter_shapes(params):
    """Ordered (state_dict key, shape) of the generator after remove_weight_norm
    (key names of models/parallel_wavegan.py:80-138)."""
    R = params.get("residual_channels", 64)
    G = params.get("gate_channels", 128)
    S = params.get("skip_channels", 64)
    A = params.get("aux_channels", 80)
    K = params.get("kernel_size", 3)
    L = params.get("layers", 30)
    O = params.get("out_channels", 1)
    I = params.get("in_channels", 1)
    w = params.get("aux_context_window", 2)
    causal = params.get("use_causal_conv", False)
    net = params.get("upsample_net", "ConvInUpsampleNetwork")
    bias = params.get("bias", True)
    out = [("first_conv.weight", (R, I, 1)), ("first_conv.bias", (R,))]
    if net == "ConvInUpsampleNetwork":
        kw = w + 1 if causal else 2 * w + 1
        out.append(("upsample_net.conv_in.weight", (A, A, kw)))
        prefix = "upsample_net.upsample.up_layers"
    else:
        prefix = "upsample_net.up_layers"
    for i, s in enumerate(_upsample_scales(params)):
        out.append((f"{prefix}.{2 * i + 1}.weight", (1, 1, 1, 2 * s + 1)))
    for l in range(L):
        p = f"conv_layers.{l}"
        out.append((f"{p}.conv.weight", (G, R, K)))
        if bias:
            out.append((f"{p}.conv.bias", (G,)))
        out.append((f"{p}.conv1x1_aux.weight", (G, A, 1)))
        out.append((f"{p}.conv1x1_out.weight", (R, G // 2, 1)))
        if bias:
            out.append((f"{p}.conv1x1_out.bias", (R,)))
        out.append((f"{p}.conv1x1_skip.weight", (S, G // 2, 1)))
        if bias:
            out.append((f"{p}.conv1x1_skip.bias", (S,)))
    out += [
        ("last_conv_layers.1.weight", (S, S, 1)),
        ("last_conv_layers.1.bias", (S,)),
        ("last_conv_layers.3.weight", (O, S, 1)),
        ("last_conv_layers.3.bias", (O,)),
    ]
    return out


def make_state_dict(params, seed=0, weight_norm=False, bias_std=0.05):
    """Seeded generator weights as a {key: float32 ndarray} dict.

    weight_norm=False: folded weights (keys ``*.weight``), as after remove_weight_norm.
    weight_norm=True: old-style ``*.weight_g`` (O,1,..) / ``*.weight_v`` keys, as saved by a
    training checkpoint (models/parallel_wavegan.py:141-142,187-195); g = ||v|| * U(0.5, 1.5).
    """
    rs = np.random.RandomState(seed)
    sd = {}
    for key, shape in parameter_shapes(params):
        if key.endswith(".bias"):
            sd[key] = (bias_std * rs.standard_normal(shape)).astype(np.float32)
            continue
        if len(shape) == 4:  # FIR taps of the upsampler
            n = shape[-1]
            taps = 1.0 / n + 0.1 / n * rs.standard_normal(shape)
            w = taps.astype(np.float32)
        else:
            fan_in = int(np.prod(shape[1:]))
            w = (np.sqrt(2.0 / fan_in) * rs.standard_normal(shape)).astype(np.float32)
        if weight_norm:
            v = w
            axes = tuple(range(1, v.ndim))
            norm = np.sqrt(np.sum(v.astype(np.float64) ** 2, axis=axes, keepdims=True))
            g = (norm * rs.uniform(0.5, 1.5, size=norm.shape)).astype(np.float32)
            base = key[: -len(".weight")]
            sd[base + ".weight_g"] = g
            sd[base + ".weight_v"] = v
        else:
            sd[key] = w
    return sd


def make_mel(frames, aux_channels=80, seed=1):
    """Normalised log-mel stand-in, (T', aux) frames-major like inference()'s ``c``
    (bin/normalize.py:237-270 makes each band ~N(0,1))."""
    return np.random.RandomState(seed).standard_normal((frames, aux_channels)).astype(np.float32)


def make_noise(samples, seed=2):
    """Explicit input noise ``x`` (T, 1), the distribution of torch.randn in
    models/parallel_wavegan.py:250-253."""
    return np.random.RandomState(seed).standard_normal((samples, 1)).astype(np.float32)


def libritts_lengths(n_utts, seed=3, low=80, high=1200):
    """Utterance lengths in mel frames for the multi-utterance LibriTTS workload
    (RandomState(3).randint(80, 1200))."""
    return np.random.RandomState(seed).randint(low, high, size=n_utts).astype(np.int64)


def make_module_state_dict(module, seed=0, gain=1.0, bias_std=0.05, weight_norm=None):
    """Seeded weights for any generator holder module (MelGAN / HiFiGAN drop-ins): conv weights
    ~ N(0, gain^2 / fan_in) with fan_in = C_in*K (Conv1d) or C_in*2 (ConvTranspose1d, 2 taps per
    output), biases ~ N(0, bias_std^2). Keys follow the module's state dict: with weight norm
    applied, ``weight_v`` = the drawn weight and ``weight_g`` = ||v|| * U(0.5, 1.5) per output
    slice. Buffers (PQMF filters, stats) are left out."""
    import torch

    rs = np.random.RandomState(seed)
    sd = {}
    kinds = {}
    for name, m in module.named_modules():
        if isinstance(m, torch.nn.ConvTranspose1d):
            kinds[name] = ("convt", m.in_channels * 2)
        elif isinstance(m, torch.nn.Conv1d):
            kinds[name] = ("conv", m.in_channels * m.kernel_size[0])
    for key, p in module.named_parameters():
        base, leaf = key.rsplit(".", 1)
        shape = tuple(p.shape)
        if leaf == "bias":
            sd[key] = (bias_std * rs.standard_normal(shape)).astype(np.float32)
        elif leaf in ("weight", "weight_v"):
            fan = kinds[base][1]
            w = (gain / np.sqrt(fan) * rs.standard_normal(shape)).astype(np.float32)
            sd[key] = w
            if leaf == "weight_v":
                axes = tuple(range(1, w.ndim))
                norm = np.sqrt(np.sum(w.astype(np.float64) ** 2, axis=axes, keepdims=True))
                sd[base + ".weight_g"] = (norm * rs.uniform(0.5, 1.5, size=norm.shape)).astype(np.float32)
    return sd
