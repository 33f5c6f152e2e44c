"""CPU oracle (TEST INFRASTRUCTURE ONLY): float64 NumPy restatement of the reference's MelGAN /
multi-band MelGAN + PQMF / HiFiGAN generator forwards, used by tests/ to check the HIP conv-network
executor. Never imported by the product path.

Every function cites the reference code it restates:
  MelGANGenerator     /root/reference/parallel_wavegan/models/melgan.py:17-170, 229-246
  ResidualStack       /root/reference/parallel_wavegan/layers/residual_stack.py:13-85
  PQMF.synthesis      /root/reference/parallel_wavegan/layers/pqmf.py:133-149
  HiFiGANGenerator    /root/reference/parallel_wavegan/models/hifigan.py:23-192, 251-265
  HiFiGANResidualBlock /root/reference/parallel_wavegan/layers/residual_block.py:143-258
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


def _g(sd, key):
    v = sd.get(key)
    return None if v is None else np.asarray(v, dtype=np.float64)


def residual_stack(x, sd, prefix, dilation, kernel_size, slope, pad_mode):
    """layers/residual_stack.py:75-85: stack(c) + skip_layer(c)."""
    p = (kernel_size - 1) // 2 * dilation
    h = conv1d(pad1d(lrelu(x, slope), p, p, pad_mode), _g(sd, prefix + ".stack.2.weight"),
               _g(sd, prefix + ".stack.2.bias"), dilation)
    h = conv1d(lrelu(h, slope), _g(sd, prefix + ".stack.4.weight"), _g(sd, prefix + ".stack.4.bias"))
    return h + conv1d(x, _g(sd, prefix + ".skip_layer.weight"), _g(sd, prefix + ".skip_layer.bias"))


def melgan_forward(c, sd, params):
    """models/melgan.py:17-170 with the module indices of its nn.Sequential. c (in, T')."""
    P = dict(in_channels=80, out_channels=1, kernel_size=7, channels=512, upsample_scales=[8, 8, 2, 2],
             stack_kernel_size=3, stacks=3, nonlinear_activation_params={"negative_slope": 0.2},
             pad="ReflectionPad1d", use_final_nonlinear_activation=True)
    P.update(params)
    slope = P["nonlinear_activation_params"]["negative_slope"]
    mode = "reflect" if P["pad"] == "ReflectionPad1d" else "zero"
    k = P["kernel_size"]
    idx = 0
    x = conv1d(pad1d(np.asarray(c, np.float64), (k - 1) // 2, (k - 1) // 2, mode), _g(sd, "melgan.1.weight"),
               _g(sd, "melgan.1.bias"))
    idx = 2
    for s in P["upsample_scales"]:
        idx += 1  # activation
        x = conv_transpose1d(lrelu(x, slope), _g(sd, f"melgan.{idx}.weight"), _g(sd, f"melgan.{idx}.bias"), s,
                             s // 2 + s % 2, s % 2)
        idx += 1
        for j in range(P["stacks"]):
            x = residual_stack(x, sd, f"melgan.{idx}", P["stack_kernel_size"] ** j, P["stack_kernel_size"], slope,
                               mode)
            idx += 1
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
    """models/hifigan.py:173-192 with HiFiGANResidualBlock (layers/residual_block.py:244-258)."""
    P = dict(in_channels=80, out_channels=1, channels=512, kernel_size=7, upsample_scales=(8, 8, 2, 2),
             upsample_kernel_sizes=(16, 16, 4, 4), resblock_kernel_sizes=(3, 7, 11),
             resblock_dilations=[(1, 3, 5), (1, 3, 5), (1, 3, 5)], use_additional_convs=True,
             nonlinear_activation_params={"negative_slope": 0.1})
    P.update(params)
    slope = P["nonlinear_activation_params"]["negative_slope"]
    k = P["kernel_size"]
    x = conv1d(pad1d(np.asarray(c, np.float64), (k - 1) // 2, (k - 1) // 2, "zero"), _g(sd, "input_conv.weight"),
               _g(sd, "input_conv.bias"))
    nb = len(P["resblock_kernel_sizes"])
    for i, s in enumerate(P["upsample_scales"]):
        x = conv_transpose1d(lrelu(x, slope), _g(sd, f"upsamples.{i}.1.weight"), _g(sd, f"upsamples.{i}.1.bias"), s,
                             s // 2 + s % 2, s % 2)
        cs = 0.0
        for j, ks in enumerate(P["resblock_kernel_sizes"]):
            pre = f"blocks.{i * nb + j}"
            xb = x
            for d_i, d in enumerate(P["resblock_dilations"][j]):
                p = (ks - 1) // 2 * d
                xt = conv1d(pad1d(lrelu(xb, slope), p, p, "zero"), _g(sd, f"{pre}.convs1.{d_i}.1.weight"),
                            _g(sd, f"{pre}.convs1.{d_i}.1.bias"), d)
                if P["use_additional_convs"]:
                    p2 = (ks - 1) // 2
                    xt = conv1d(pad1d(lrelu(xt, slope), p2, p2, "zero"), _g(sd, f"{pre}.convs2.{d_i}.1.weight"),
                                _g(sd, f"{pre}.convs2.{d_i}.1.bias"))
                xb = xt + xb
            cs = cs + xb
        x = cs / nb
    x = conv1d(pad1d(lrelu(x, 0.01), (k - 1) // 2, (k - 1) // 2, "zero"), _g(sd, "output_conv.1.weight"),
               _g(sd, "output_conv.1.bias"))
    return np.tanh(x)


def hifigan_inference(c, sd, params, mean=None, scale=None):
    """models/hifigan.py:251-265: c (T', in) -> (T, out_channels)."""
    c = np.asarray(c, np.float64)
    if mean is not None:
        c = (c - mean) / scale
    return hifigan_forward(c.T, sd, params).T
