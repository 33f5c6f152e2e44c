"""CPU oracle (TEST INFRASTRUCTURE ONLY): float64 NumPy restatement of the reference's MelGAN /
multi-band MelGAN + PQMF / HiFiGAN generator forwards, used by tests/ to check the HIP conv-network
executor. Never imported by the product path.

Every function cites the reference code it restates:
  MelGANGenerator     /root/reference/parallel_wavegan/models/melgan.py:17-170, 229-246
  ResidualStack       /root/reference/parallel_wavegan/layers/residual_stack.py:13-85
  PQMF.synthesis      /root/reference/parallel_wavegan/layers/pqmf.py:133-149
  HiFiGANGenerator    /root/reference/parallel_wavegan/models/hifigan.py:23-192, 251-265
  HiFiGANResidualBlock /root/reference/parallel_wavegan/layers/residual_block.py:143-258
  CausalConv1d / CausalConvTranspose1d  /root/reference/parallel_wavegan/layers/causal_conv.py:12-78
    (use_causal_conv=True: models/melgan.py:73-84,101-112,141-151, residual_stack.py:65-80,
    models/hifigan.py:83-88,110-124,153-164, residual_block.py:198-241)
Weights come as a folded state dict {key: ndarray} (weight norm folded, engine.fold_weight_norm).
Arrays are (channels, time) per utterance, like the reference's (B=1, C, T) tensors.
"""

import numpy as np


def lrelu(x, slope):
    return np.where(x > 0, x, x * slope)


def pad1d(x, left, right, mode):
    """torch.nn.ReflectionPad1d / ConstantPad1d(0) / Conv1d zero padding."""
    if left == 0 and right == 0:
        return x
    if mode == "reflect":
        assert left < x.shape[1] and right < x.shape[1], "ReflectionPad1d needs pad < input size"
        return np.pad(x, ((0, 0), (left, right)), mode="reflect")
    return np.pad(x, ((0, 0), (left, right)))


def conv1d(x, w, b, dilation=1):
    """Valid Conv1d: x (C_in, T), w (C_out, C_in, K) -> (C_out, T - (K-1)*dilation)."""
    K = w.shape[2]
    T = x.shape[1] - (K - 1) * dilation
    y = np.zeros((w.shape[0], T))
    for k in range(K):
        y += w[:, :, k] @ x[:, k * dilation:k * dilation + T]
    if b is not None:
        y += b[:, None]
    return y


def conv_transpose1d(x, w, b, stride, padding, output_padding):
    """torch ConvTranspose1d: x (C_in, L), w (C_in, C_out, K):
    out[o, j*s - p + k] += sum_i x[i, j] w[i, o, k]."""
    C_in, L = x.shape
    K = w.shape[2]
    full = (L - 1) * stride + K
    y = np.zeros((w.shape[1], full + output_padding))
    for k in range(K):
        y[:, k:k + (L - 1) * stride + 1:stride] += w[:, :, k].T @ x
    T_out = (L - 1) * stride - 2 * padding + K + output_padding
    y = y[:, padding:padding + T_out]
    if b is not None:
        y = y + b[:, None]
    return y


def causal_conv1d(x, w, b, dilation=1, mode="zero"):
    """layers/causal_conv.py:34-45: pad (K-1)*dilation (the pad module pads both sides, only the
    left part reaches the first T outputs), valid conv, keep the first T outputs."""
    p = (w.shape[2] - 1) * dilation
    if mode == "reflect":
        assert p < x.shape[1], "ReflectionPad1d needs pad < input size"
        xp = np.pad(x, ((0, 0), (p, 0)), mode="reflect")
    elif mode == "replicate":
        xp = np.pad(x, ((0, 0), (p, 0)), mode="edge")
    else:
        xp = np.pad(x, ((0, 0), (p, 0)))
    return conv1d(xp, w, b, dilation)


def causal_conv_transpose1d(x, w, b, stride):
    """layers/causal_conv.py:67-78: ReplicationPad1d((1, 0)), ConvTranspose1d(2s, s), [s:-s]."""
    xp = np.concatenate([x[:, :1], x], axis=1)
    y = conv_transpose1d(xp, w, b, stride, 0, 0)
    return y[:, stride:-stride]


def _g(sd, key):
    v = sd.get(key)
    return None if v is None else np.asarray(v, dtype=np.float64)


def residual_stack(x, sd, prefix, dilation, kernel_size, slope, pad_mode, causal=False):
    """layers/residual_stack.py:75-85: stack(c) + skip_layer(c) (causal stack: :65-80)."""
    if causal:
        h = causal_conv1d(lrelu(x, slope), _g(sd, prefix + ".stack.1.conv.weight"),
                          _g(sd, prefix + ".stack.1.conv.bias"), dilation, pad_mode)
        i1 = 3
    else:
        p = (kernel_size - 1) // 2 * dilation
        h = conv1d(pad1d(lrelu(x, slope), p, p, pad_mode), _g(sd, prefix + ".stack.2.weight"),
                   _g(sd, prefix + ".stack.2.bias"), dilation)
        i1 = 4
    h = conv1d(lrelu(h, slope), _g(sd, prefix + f".stack.{i1}.weight"), _g(sd, prefix + f".stack.{i1}.bias"))
    return h + conv1d(x, _g(sd, prefix + ".skip_layer.weight"), _g(sd, prefix + ".skip_layer.bias"))


def melgan_forward(c, sd, params):
    """models/melgan.py:17-170 with the module indices of its nn.Sequential. c (in, T')."""
    P = dict(in_channels=80, out_channels=1, kernel_size=7, channels=512, upsample_scales=[8, 8, 2, 2],
             stack_kernel_size=3, stacks=3, nonlinear_activation_params={"negative_slope": 0.2},
             pad="ReflectionPad1d", use_final_nonlinear_activation=True, use_causal_conv=False)
    P.update(params)
    slope = P["nonlinear_activation_params"]["negative_slope"]
    mode = {"ReflectionPad1d": "reflect", "ReplicationPad1d": "replicate"}.get(P["pad"], "zero")
    k = P["kernel_size"]
    causal = bool(P["use_causal_conv"])
    c = np.asarray(c, np.float64)
    if causal:  # [CausalConv1d]
        x = causal_conv1d(c, _g(sd, "melgan.0.conv.weight"), _g(sd, "melgan.0.conv.bias"), 1, mode)
        idx = 1
    else:  # [pad, Conv1d]
        x = conv1d(pad1d(c, (k - 1) // 2, (k - 1) // 2, mode), _g(sd, "melgan.1.weight"), _g(sd, "melgan.1.bias"))
        idx = 2
    for s in P["upsample_scales"]:
        idx += 1  # activation
        if causal:
            x = causal_conv_transpose1d(lrelu(x, slope), _g(sd, f"melgan.{idx}.deconv.weight"),
                                        _g(sd, f"melgan.{idx}.deconv.bias"), s)
        else:
            x = conv_transpose1d(lrelu(x, slope), _g(sd, f"melgan.{idx}.weight"), _g(sd, f"melgan.{idx}.bias"), s,
                                 s // 2 + s % 2, s % 2)
        idx += 1
        for j in range(P["stacks"]):
            x = residual_stack(x, sd, f"melgan.{idx}", P["stack_kernel_size"] ** j, P["stack_kernel_size"], slope,
                               mode, causal)
            idx += 1
    if causal:
        idx += 1  # activation
        x = causal_conv1d(lrelu(x, slope), _g(sd, f"melgan.{idx}.conv.weight"), _g(sd, f"melgan.{idx}.conv.bias"),
                          1, mode)
    else:
        idx += 2  # activation, pad
        x = conv1d(pad1d(lrelu(x, slope), (k - 1) // 2, (k - 1) // 2, mode), _g(sd, f"melgan.{idx}.weight"),
                   _g(sd, f"melgan.{idx}.bias"))
    if P["use_final_nonlinear_activation"]:
        x = np.tanh(x)
    return x


def pqmf_synthesis(x, syn):
    """layers/pqmf.py:133-149: conv_transpose1d with updown*S (zero insertion, x S), then the
    (taps+1)-tap synthesis conv with zero padding taps/2. x (S, L), syn (S, taps+1) -> (1, S*L)."""
    S, L = x.shape
    NT = syn.shape[1]
    u = np.zeros((S, S * L))
    u[:, ::S] = S * x
    return conv1d(pad1d(u, NT // 2, NT // 2, "zero"), np.asarray(syn, np.float64)[None], None)


def melgan_inference(c, sd, params, syn=None, mean=None, scale=None):
    """models/melgan.py:229-246: c (T', in) -> (T, 1 or out_channels)."""
    c = np.asarray(c, np.float64)
    if mean is not None:
        c = (c - mean) / scale
    y = melgan_forward(c.T, sd, params)
    if syn is not None:
        y = pqmf_synthesis(y, syn)
    return y.T


def hifigan_forward(c, sd, params):
    """models/hifigan.py:173-192 with HiFiGANResidualBlock (layers/residual_block.py:244-258);
    causal convs (zero padded) when use_causal_conv."""
    P = dict(in_channels=80, out_channels=1, channels=512, kernel_size=7, upsample_scales=(8, 8, 2, 2),
             upsample_kernel_sizes=(16, 16, 4, 4), resblock_kernel_sizes=(3, 7, 11),
             resblock_dilations=[(1, 3, 5), (1, 3, 5), (1, 3, 5)], use_additional_convs=True,
             nonlinear_activation_params={"negative_slope": 0.1}, use_causal_conv=False)
    P.update(params)
    slope = P["nonlinear_activation_params"]["negative_slope"]
    k = P["kernel_size"]
    causal = bool(P["use_causal_conv"])

    def conv(x, key, d=1):  # Conv1d(padding=(K-1)//2*d) or CausalConv1d
        if causal:
            return causal_conv1d(x, _g(sd, key + ".conv.weight"), _g(sd, key + ".conv.bias"), d)
        w = _g(sd, key + ".weight")
        p = (w.shape[2] - 1) // 2 * d
        return conv1d(pad1d(x, p, p, "zero"), w, _g(sd, key + ".bias"), d)

    x = conv(np.asarray(c, np.float64), "input_conv")
    nb = len(P["resblock_kernel_sizes"])
    for i, s in enumerate(P["upsample_scales"]):
        if causal:
            x = causal_conv_transpose1d(lrelu(x, slope), _g(sd, f"upsamples.{i}.1.deconv.weight"),
                                        _g(sd, f"upsamples.{i}.1.deconv.bias"), s)
        else:
            x = conv_transpose1d(lrelu(x, slope), _g(sd, f"upsamples.{i}.1.weight"), _g(sd, f"upsamples.{i}.1.bias"),
                                 s, s // 2 + s % 2, s % 2)
        cs = 0.0
        for j, ks in enumerate(P["resblock_kernel_sizes"]):
            pre = f"blocks.{i * nb + j}"
            xb = x
            for d_i, d in enumerate(P["resblock_dilations"][j]):
                xt = conv(lrelu(xb, slope), f"{pre}.convs1.{d_i}.1", d)
                if P["use_additional_convs"]:
                    xt = conv(lrelu(xt, slope), f"{pre}.convs2.{d_i}.1")
                xb = xt + xb
            cs = cs + xb
        x = cs / nb
    x = conv(lrelu(x, 0.01), "output_conv.1")
    return np.tanh(x)


def hifigan_inference(c, sd, params, mean=None, scale=None):
    """models/hifigan.py:251-265: c (T', in) -> (T, out_channels)."""
    c = np.asarray(c, np.float64)
    if mean is not None:
        c = (c - mean) / scale
    return hifigan_forward(c.T, sd, params).T
