"""Causal convolution holders (layers/causal_conv.py:12-78) for the causal MelGAN / HiFiGAN
drop-ins.

Same sub-module names as the reference (``pad`` + ``conv`` / ``deconv``), so causal checkpoints
load unchanged (``...conv.weight_g``, ``...deconv.weight_v``). They only hold parameters: the
generators lower them to conv-network ops (include/pwg_cnet.h):

* ``CausalConv1d``: pad (K-1)*dil on the left, keep the first T outputs (``:34-45``) = a conv op
  whose source reads rows t - (K-1)*dil + k*dil with the pad module's edge mode;
* ``CausalConvTranspose1d``: ReplicationPad1d((1, 0)), ConvTranspose1d(2s, s), trim s on both
  sides (``:48-78``) = a CONVT op with padding 0 and a replicate-padded source.
"""

import torch

from . import cnet


class CausalConv1d(torch.nn.Module):
    """layers/causal_conv.py:12-45 (parameter holder)."""

    def __init__(self, in_channels, out_channels, kernel_size, dilation=1, bias=True, pad="ConstantPad1d",
                 pad_params={"value": 0.0}):
        super().__init__()
        self.pad = getattr(torch.nn, pad)((kernel_size - 1) * dilation, **pad_params)
        self.conv = torch.nn.Conv1d(in_channels, out_channels, kernel_size, dilation=dilation, bias=bias)

    def forward(self, x):
        raise RuntimeError("parameter holder: the generator runs on the MI355X conv-network engine")


class CausalConvTranspose1d(torch.nn.Module):
    """layers/causal_conv.py:48-78 (parameter holder)."""

    def __init__(self, in_channels, out_channels, kernel_size, stride, bias=True, pad="ReplicationPad1d",
                 pad_params={}):
        super().__init__()
        self.pad = getattr(torch.nn, pad)((1, 0), **pad_params)
        self.deconv = torch.nn.ConvTranspose1d(in_channels, out_channels, kernel_size, stride, bias=bias)
        self.stride = stride

    def forward(self, x):
        raise RuntimeError("parameter holder: the generator runs on the MI355X conv-network engine")


def edge_mode(pad):
    """cnet pad mode of a padding module: ReflectionPad1d, zero ConstantPad1d, ReplicationPad1d."""
    if isinstance(pad, torch.nn.ReflectionPad1d):
        return cnet.PAD_REFLECT
    if isinstance(pad, torch.nn.ReplicationPad1d):
        return cnet.PAD_REPLICATE
    if isinstance(pad, torch.nn.ConstantPad1d) and pad.value == 0.0:
        return cnet.PAD_ZERO
    raise NotImplementedError(f"{type(pad).__name__} padding in a causal conv is not supported by the MI355X engine")


def conv_src(P, buf, channels, m, key, pre_slope=1.0, normalize=False):
    """Source descriptor of a CausalConv1d ``m`` whose state-dict prefix is ``key``."""
    c = m.conv
    k, d = c.kernel_size[0], c.dilation[0]
    if c.stride[0] != 1 or c.groups != 1 or c.padding[0] != 0:
        raise NotImplementedError("strided / grouped / padded conv inside CausalConv1d")
    return P.src(buf, channels, k, d, (k - 1) * d, edge_mode(m.pad), pre_slope, key + ".conv.weight",
                 normalize=normalize)


def convt_src(P, buf, channels, m, key, pre_slope=1.0, normalize=False):
    """(source, stride) of a CausalConvTranspose1d ``m``; the op is a CONVT with padding 0."""
    ct = m.deconv
    s = ct.stride[0]
    if ct.kernel_size[0] != 2 * s or ct.padding[0] != 0 or ct.output_padding[0] != 0:
        raise NotImplementedError("CausalConvTranspose1d must have kernel 2*stride")
    if not isinstance(m.pad, torch.nn.ReplicationPad1d) or tuple(m.pad.padding) != (1, 0):
        raise NotImplementedError("CausalConvTranspose1d needs ReplicationPad1d((1, 0))")
    src = P.src(buf, channels, pre_slope=pre_slope, weight=key + ".deconv.weight", normalize=normalize,
                pad_mode=cnet.PAD_REPLICATE)
    return src, s
