"""TEST INFRASTRUCTURE ONLY — NumPy restatement of the reference PWG generator forward.

This is the parity checker for the HIP engine, not a product path: only tests/,
__graft_entry__.smoke() and bench.py's cpu_baseline leg may use it.

Pinned against golden vectors produced by the reference itself (tests/golden/make_golden.py
imports /root/reference in the dev container and records its outputs); see
tests/test_oracle_golden.py. Every function cites the reference code it restates
(paths relative to /root/reference/parallel_wavegan).

Arithmetic defaults to float64 so the oracle's own rounding is far below the |d| < 1e-4 bar.
"""

import math

import numpy as np


def _w(sd, key, dtype):
    return np.asarray(sd[key], dtype=dtype)


def fold_weight_norm(sd):
    """W = g * v / ||v||_2 over all dims but 0 (torch weight_norm dim=0, applied by
    models/parallel_wavegan.py:187-195, removed by :175-185)."""
    out = {}
    for k, v in sd.items():
        if k.endswith(".weight_g"):
            continue
        if k.endswith(".weight_v"):
            base = k[: -len(".weight_v")]
            v64 = np.asarray(v, np.float64)
            g64 = np.asarray(sd[base + ".weight_g"], np.float64)
            norm = np.sqrt(np.sum(v64 ** 2, axis=tuple(range(1, v64.ndim)), keepdims=True))
            out[base + ".weight"] = g64 * v64 / norm
        else:
            out[k] = np.asarray(v)
    return out


def conv_in(c, w, causal=False, aux_context_window=0):
    """ConvInUpsampleNetwork.conv_in: Conv1d(A, A, k, bias=False), no padding (valid),
    layers/upsample.py:166-168,192; causal trims the last w outputs (:193).
    c (A, T'+2w) -> (A, T')."""
    A, Tin = c.shape
    k = w.shape[2]
    Tout = Tin - k + 1
    y = np.zeros((w.shape[0], Tout), dtype=c.dtype)
    for j in range(k):
        y += w[:, :, j] @ c[:, j:j + Tout]
    if causal and aux_context_window > 0:
        y = y[:, :-aux_context_window]
    return y


def stretch(c, scale, mode="nearest"):
    """Stretch2d (layers/upsample.py:43-45): F.interpolate(scale_factor=(1, s)) on (B, 1, C, T).
    nearest (and nearest-exact / area at integer scales): out[t] = in[t // s]. bilinear
    (align_corners=False; the channel axis at scale 1 is the identity): aten's linear source index
    src = max((t + 0.5) / s - 0.5, 0), i0 = floor(src), i1 = min(i0 + 1, T - 1),
    out[t] = (1 - l) in[i0] + l in[i1], l = src - i0."""
    if mode in ("nearest", "nearest-exact", "area"):
        return np.repeat(c, scale, axis=1)
    if mode != "bilinear":
        raise NotImplementedError(mode)
    n = c.shape[1]
    t = np.arange(n * scale, dtype=np.float64)
    src = np.maximum((t + 0.5) / scale - 0.5, 0.0)
    i0 = np.floor(src).astype(np.int64)
    i1 = np.minimum(i0 + 1, n - 1)
    lam = (src - i0).astype(c.dtype)
    return (1 - lam) * c[:, i0] + lam * c[:, i1]


def upsample_stage(c, scale, taps, causal=False, mode="nearest"):
    """Stretch2d xs (stretch(); layers/upsample.py:43-45) followed by the
    Conv2d (1, 2s+1) FIR with zero padding (s, s) or causal (2s, 2s) + trim (:97-103,124-125),
    torch cross-correlation: out[t] = sum_k h[k] * up[t + k - pad]."""
    up = stretch(c, scale, mode)
    n = up.shape[1]
    pad = 2 * scale if causal else scale
    upp = np.pad(up, ((0, 0), (pad, pad)))
    kt = taps.size
    nout = n + 2 * pad - kt + 1
    y = np.zeros((c.shape[0], nout), dtype=c.dtype)
    for k in range(kt):
        y += taps[k] * upp[:, k:k + nout]
    return y[:, :n] if causal else y


def upsample_net(c, sd, params, dtype=np.float64):
    """ConvInUpsampleNetwork.forward / UpsampleNetwork.forward (layers/upsample.py:112-128,
    178-194) for one item: c (A, T'+2w) -> (A, T'*H)."""
    causal = params.get("use_causal_conv", False)
    scales = params["upsample_params"]["upsample_scales"]
    if params.get("upsample_net", "ConvInUpsampleNetwork") == "ConvInUpsampleNetwork":
        w = params.get("aux_context_window", 2)
        c = conv_in(c, _w(sd, "upsample_net.conv_in.weight", dtype), causal and w > 0, w)
        prefix = "upsample_net.upsample.up_layers"
    else:
        prefix = "upsample_net.up_layers"
    mode = params["upsample_params"].get("interpolate_mode", "nearest")
    for i, s in enumerate(scales):
        taps = _w(sd, f"{prefix}.{2 * i + 1}.weight", dtype).reshape(-1)
        c = upsample_stage(c, s, taps, causal, mode)
    return c


def residual_block(x, c, sd, l, dilation, kernel_size, causal, dtype):
    """WaveNetResidualBlock.forward (layers/residual_block.py:102-140) for one item.
    x (R, T), c (A, T) -> (x_out (R, T), skip (S, T))."""
    p = f"conv_layers.{l}"
    W = _w(sd, f"{p}.conv.weight", dtype)  # (G, R, K)
    R, T = x.shape
    pad = (kernel_size - 1) * dilation if causal else (kernel_size - 1) // 2 * dilation
    xp = np.pad(x, ((0, 0), (pad, pad)))
    y = np.zeros((W.shape[0], T), dtype=dtype)
    for k in range(kernel_size):
        y += W[:, :, k] @ xp[:, k * dilation:k * dilation + T]
    if f"{p}.conv.bias" in sd:
        y += _w(sd, f"{p}.conv.bias", dtype)[:, None]
    y += _w(sd, f"{p}.conv1x1_aux.weight", dtype)[:, :, 0] @ c
    gh = W.shape[0] // 2
    g = np.tanh(y[:gh]) * (1.0 / (1.0 + np.exp(-y[gh:])))
    s = _w(sd, f"{p}.conv1x1_skip.weight", dtype)[:, :, 0] @ g
    if f"{p}.conv1x1_skip.bias" in sd:
        s += _w(sd, f"{p}.conv1x1_skip.bias", dtype)[:, None]
    o = _w(sd, f"{p}.conv1x1_out.weight", dtype)[:, :, 0] @ g
    if f"{p}.conv1x1_out.bias" in sd:
        o += _w(sd, f"{p}.conv1x1_out.bias", dtype)[:, None]
    return (o + x) * math.sqrt(0.5), s


def forward_one(z, c, sd, params, dtype=np.float64, return_cup=False):
    """ParallelWaveGANGenerator.forward (models/parallel_wavegan.py:144-173) for one item:
    z (T,), c (A, T'+2w) -> y (O, T)."""
    sd = fold_weight_norm(sd)
    z = np.asarray(z, dtype).reshape(-1)
    c = np.asarray(c, dtype)
    cup = upsample_net(c, sd, params, dtype)
    assert cup.shape[1] == z.size  # :158
    x = _w(sd, "first_conv.weight", dtype)[:, 0, 0][:, None] * z[None, :] + _w(sd, "first_conv.bias", dtype)[:, None]
    L = params.get("layers", 30)
    lps = L // params.get("stacks", 3)
    K = params.get("kernel_size", 3)
    causal = params.get("use_causal_conv", False)
    skips = 0
    for l in range(L):
        x, h = residual_block(x, cup, sd, l, 2 ** (l % lps), K, causal, dtype)
        skips = skips + h
    skips = skips * math.sqrt(1.0 / L)  # :166
    h = np.maximum(skips, 0)  # last_conv_layers :131-138
    h = _w(sd, "last_conv_layers.1.weight", dtype)[:, :, 0] @ h + _w(sd, "last_conv_layers.1.bias", dtype)[:, None]
    h = np.maximum(h, 0)
    y = _w(sd, "last_conv_layers.3.weight", dtype)[:, :, 0] @ h + _w(sd, "last_conv_layers.3.bias", dtype)[:, None]
    return (y, cup) if return_cup else y


def forward(z, c, sd, params, dtype=np.float64):
    """Batched forward: z (B, 1, T), c (B, A, T'+2w) -> (B, O, T)."""
    return np.stack([forward_one(z[b, 0], c[b], sd, params, dtype) for b in range(z.shape[0])])


def pad_inference_features(c, params, mean=None, scale=None):
    """inference() preprocessing (models/parallel_wavegan.py:254-262): optional
    (c - mean) / scale, transpose to (A, T'), ReplicationPad1d(aux_context_window)."""
    c = np.asarray(c, np.float64)
    if mean is not None:
        c = (c - np.asarray(mean, np.float64)) / np.asarray(scale, np.float64)
    c = c.T
    w = params.get("aux_context_window", 2)
    if w > 0:
        c = np.concatenate([np.repeat(c[:, :1], w, axis=1), c, np.repeat(c[:, -1:], w, axis=1)], axis=1)
    return c


def inference(c, x, sd, params, mean=None, scale=None, dtype=np.float64, return_cup=False):
    """ParallelWaveGANGenerator.inference with explicit noise (models/parallel_wavegan.py:231-263):
    c (T', A), x (T, 1) -> (T, O)."""
    cp = pad_inference_features(c, params, mean, scale).astype(dtype)
    res = forward_one(np.asarray(x).reshape(-1), cp, sd, params, dtype, return_cup)
    if return_cup:
        return res[0].T, res[1]
    return res.T
