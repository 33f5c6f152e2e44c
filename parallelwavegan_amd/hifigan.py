"""Drop-in ``HiFiGANGenerator`` running on the MI355X conv-network executor (include/pwg_cnet.h).

Mirrors parallel_wavegan.models.HiFiGANGenerator (/root/reference/parallel_wavegan/models/
hifigan.py:23-265) and HiFiGANResidualBlock (layers/residual_block.py:143-258): same constructor
arguments, sub-module names and state-dict keys (input_conv, upsamples.i.1, blocks.j.convs1/2.d.1,
output_conv.1), ``forward(c)``, ``inference(c, normalize_before)``, ``remove_weight_norm``,
``apply_weight_norm``, ``register_stats``.

Lowering of the multi-receptive-field fusion (models/hifigan.py:173-192): block j of stage i is
x <- conv2(lrelu(conv1(lrelu(x)))) + x per dilation, each conv one fused op whose epilogue adds
the residual; the LAST conv of block j also adds the running sum of blocks 0..j-1 (and the last
block divides by num_blocks), so ``cs += block(c); c = cs / num_blocks`` costs no extra pass and
keeps the reference's summation order.
"""

import logging

import numpy as np
import torch

from . import causal, cnet
from .engine import WeightTracker, first_parameter, forget_device
from .melgan import _slope


class HiFiGANResidualBlock(torch.nn.Module):
    """Parameter holder with the layout of layers/residual_block.py:143-243."""

    def __init__(self, kernel_size=3, channels=512, dilations=(1, 3, 5), bias=True, use_additional_convs=True,
                 nonlinear_activation="LeakyReLU", nonlinear_activation_params={"negative_slope": 0.1},
                 use_causal_conv=False):
        super().__init__()
        assert kernel_size % 2 == 1, "Kernel size must be odd number."
        self.use_additional_convs = use_additional_convs
        self.use_causal_conv = bool(use_causal_conv)
        self.kernel_size = kernel_size
        self.dilations = tuple(dilations)
        act = getattr(torch.nn, nonlinear_activation)

        def conv(d):
            if use_causal_conv:  # layers/residual_block.py:198-241
                return causal.CausalConv1d(channels, channels, kernel_size, dilation=d, bias=bias)
            return torch.nn.Conv1d(channels, channels, kernel_size, 1, dilation=d, bias=bias,
                                   padding=(kernel_size - 1) // 2 * d)

        self.convs1 = torch.nn.ModuleList()
        if use_additional_convs:
            self.convs2 = torch.nn.ModuleList()
        for d in dilations:
            self.convs1 += [torch.nn.Sequential(act(**nonlinear_activation_params), conv(d))]
            if use_additional_convs:
                self.convs2 += [torch.nn.Sequential(act(**nonlinear_activation_params), conv(1))]


def _conv_src(P, buf, ch, seq, key, normalize=False):
    """Source descriptor of Sequential(act, Conv1d | CausalConv1d) (zero padding from the conv)."""
    act, conv = seq[0], seq[1]
    if isinstance(conv, causal.CausalConv1d):
        return causal.conv_src(P, buf, ch, conv, key + ".1", _slope(act), normalize=normalize)
    return P.src(buf, ch, conv.kernel_size[0], conv.dilation[0], conv.padding[0], cnet.PAD_ZERO, _slope(act),
                 key + ".1.weight", normalize=normalize)


def _conv_bias(seq, key):
    """State-dict key of the bias of Sequential(act, Conv1d | CausalConv1d) ``key``, or None."""
    conv = seq[1]
    if isinstance(conv, causal.CausalConv1d):
        return key + ".1.conv.bias" if conv.conv.bias is not None else None
    return key + ".1.bias" if conv.bias is not None else None


class HiFiGANGenerator(torch.nn.Module):
    """models/hifigan.py:23-265, executed on the MI355X conv-network engine."""

    def __init__(self, in_channels=80, out_channels=1, channels=512, kernel_size=7, upsample_scales=(8, 8, 2, 2),
                 upsample_kernel_sizes=(16, 16, 4, 4), resblock_kernel_sizes=(3, 7, 11),
                 resblock_dilations=[(1, 3, 5), (1, 3, 5), (1, 3, 5)], use_additional_convs=True, bias=True,
                 nonlinear_activation="LeakyReLU", nonlinear_activation_params={"negative_slope": 0.1},
                 use_causal_conv=False, use_weight_norm=True):
        super().__init__()
        assert kernel_size % 2 == 1, "Kernel size must be odd number."
        assert len(upsample_scales) == len(upsample_kernel_sizes)
        assert len(resblock_dilations) == len(resblock_kernel_sizes)
        self.num_upsamples = len(upsample_kernel_sizes)
        self.num_blocks = len(resblock_kernel_sizes)
        self.use_causal_conv = bool(use_causal_conv)
        self.in_channels, self.out_channels = in_channels, out_channels
        self.upsample_factor = int(np.prod(upsample_scales))
        act = getattr(torch.nn, nonlinear_activation)
        if not use_causal_conv:
            self.input_conv = torch.nn.Conv1d(in_channels, channels, kernel_size, bias=bias,
                                              padding=(kernel_size - 1) // 2)
        else:  # models/hifigan.py:83-88
            self.input_conv = causal.CausalConv1d(in_channels, channels, kernel_size, bias=bias)
        self.upsamples = torch.nn.ModuleList()
        self.blocks = torch.nn.ModuleList()
        for i in range(len(upsample_kernel_sizes)):
            assert upsample_kernel_sizes[i] == 2 * upsample_scales[i]
            s = upsample_scales[i]
            cin, cout = channels // (2 ** i), channels // (2 ** (i + 1))
            if not use_causal_conv:
                up = torch.nn.ConvTranspose1d(cin, cout, upsample_kernel_sizes[i], s, padding=s // 2 + s % 2,
                                              output_padding=s % 2, bias=bias)
            else:  # models/hifigan.py:110-124
                up = causal.CausalConvTranspose1d(cin, cout, upsample_kernel_sizes[i], s, bias=bias)
            self.upsamples += [torch.nn.Sequential(act(**nonlinear_activation_params), up)]
            for j in range(len(resblock_kernel_sizes)):
                self.blocks += [HiFiGANResidualBlock(resblock_kernel_sizes[j], cout, resblock_dilations[j], bias,
                                                     use_additional_convs, nonlinear_activation,
                                                     nonlinear_activation_params, use_causal_conv)]
        cout = channels // (2 ** (i + 1))
        if not use_causal_conv:
            oconv = torch.nn.Conv1d(cout, out_channels, kernel_size, bias=bias, padding=(kernel_size - 1) // 2)
        else:  # models/hifigan.py:153-164
            oconv = causal.CausalConv1d(cout, out_channels, kernel_size, bias=bias)
        self.output_conv = torch.nn.Sequential(
            torch.nn.LeakyReLU(),  # slope 0.01, as the reference (models/hifigan.py:149-152)
            oconv,
            torch.nn.Tanh(),
        )
        if use_weight_norm:
            self.apply_weight_norm()
        self.reset_parameters()
        self._engine = None
        self._weights = WeightTracker()
        self._sig = None

    # ------------------------------------------------------------------ reference API
    def reset_parameters(self):
        """models/hifigan.py:194-207: conv weights ~ N(0, 0.01)."""
        def _reset(m):
            if isinstance(m, (torch.nn.Conv1d, torch.nn.ConvTranspose1d)):
                m.weight.data.normal_(0.0, 0.01)
        self.apply(_reset)

    def remove_weight_norm(self):
        def _remove(m):
            try:
                torch.nn.utils.remove_weight_norm(m)
            except ValueError:
                return
        self.apply(_remove)

    def apply_weight_norm(self):
        def _apply(m):
            if isinstance(m, (torch.nn.Conv1d, torch.nn.ConvTranspose1d)):
                torch.nn.utils.weight_norm(m)
        self.apply(_apply)

    def register_stats(self, stats):
        """models/hifigan.py:233-249 (.npy; .h5 needs h5py, absent here)."""
        assert stats.endswith(".h5") or stats.endswith(".npy")
        if stats.endswith(".h5"):
            import h5py
            with h5py.File(stats, "r") as f:
                mean, scale = f["mean"][()].reshape(-1), f["scale"][()].reshape(-1)
        else:
            arr = np.load(stats)
            mean, scale = arr[0].reshape(-1), arr[1].reshape(-1)
        dev = first_parameter(self).device
        self.register_buffer("mean", torch.from_numpy(np.asarray(mean)).float().to(dev))
        self.register_buffer("scale", torch.from_numpy(np.asarray(scale)).float().to(dev))
        logging.info("Successfully registered stats as buffer.")

    # ------------------------------------------------------------------ lowering
    def program(self):
        P = cnet.Program(self.in_channels)
        ic = self.input_conv
        if isinstance(ic, causal.CausalConv1d):
            ch = ic.conv.out_channels
            cur = P.buffer(ch, 1)
            P.conv("input_conv", cur, ch, [causal.conv_src(P, 0, self.in_channels, ic, "input_conv", normalize=True)],
                   bias="input_conv.conv.bias" if ic.conv.bias is not None else None)
        else:
            ch = ic.out_channels
            cur = P.buffer(ch, 1)
            P.conv("input_conv", cur, ch,
                   [P.src(0, self.in_channels, ic.kernel_size[0], 1, ic.padding[0], cnet.PAD_ZERO, 1.0,
                          "input_conv.weight", normalize=True)],
                   bias="input_conv.bias" if ic.bias is not None else None)
        rate = 1
        for i in range(self.num_upsamples):
            act, ct = self.upsamples[i][0], self.upsamples[i][1]
            key = f"upsamples.{i}.1"
            if isinstance(ct, causal.CausalConvTranspose1d):
                src, s = causal.convt_src(P, cur, ch, ct, key, _slope(act))
                ct, key, padding, output_padding = ct.deconv, key + ".deconv", 0, 0
            else:
                s = ct.stride[0]
                src = P.src(cur, ch, pre_slope=_slope(act), weight=key + ".weight")
                padding, output_padding = ct.padding[0], ct.output_padding[0]
            rate *= s
            up = P.buffer(ct.out_channels, rate)
            P.convt(key, up, ct.out_channels, src, s, padding, output_padding,
                    bias=key + ".bias" if ct.bias is not None else None)
            ch = ct.out_channels
            acc = P.buffer(ch, rate)
            for j in range(self.num_blocks):
                blk = self.blocks[i * self.num_blocks + j]
                bkey = f"blocks.{i * self.num_blocks + j}"
                x = up
                nd = len(blk.convs1)
                for d in range(nd):
                    last = d == nd - 1
                    c1 = blk.convs1[d]
                    k1 = f"{bkey}.convs1.{d}"
                    fin = dict(accumulate=j > 0, out_div=float(self.num_blocks) if j == self.num_blocks - 1 else 1.0)
                    if blk.use_additional_convs:
                        t = P.buffer(ch, rate)
                        P.conv(k1, t, ch, [_conv_src(P, x, ch, c1, k1)], bias=_conv_bias(c1, k1))
                        c2 = blk.convs2[d]
                        k2 = f"{bkey}.convs2.{d}"
                        dst = acc if last else P.buffer(ch, rate)
                        P.conv(k2, dst, ch, [_conv_src(P, t, ch, c2, k2)], bias=_conv_bias(c2, k2), res=x,
                               **(fin if last else {}))
                    else:
                        dst = acc if last else P.buffer(ch, rate)
                        P.conv(k1, dst, ch, [_conv_src(P, x, ch, c1, k1)], bias=_conv_bias(c1, k1), res=x,
                               **(fin if last else {}))
                    x = dst
            cur = acc
        out = P.buffer(self.out_channels, rate)
        P.conv("output_conv.1", out, self.out_channels, [_conv_src(P, cur, ch, self.output_conv, "output_conv")],
               bias=_conv_bias(self.output_conv, "output_conv"), post_act=cnet.ACT_TANH)
        return P

    # ------------------------------------------------------------------ engine plumbing
    def _device(self):
        dev = first_parameter(self).device
        if dev.type != "cuda":
            raise RuntimeError("parallelwavegan_amd.HiFiGANGenerator runs on a ROCm GPU only; move the module "
                               "with .to('cuda') (there is no CPU fallback)")
        return dev

    def _apply(self, fn, *args, **kwargs):
        forget_device(self)
        if getattr(self, "_weights", None) is not None:
            self._weights.invalidate()  # .to() / .cuda() replace parameter storage
        return super()._apply(fn, *args, **kwargs)

    def invalidate_weights(self):
        """Force a re-pack on the next call (after writes through ``p.data`` aliases, which the
        WeightTracker cannot see)."""
        self._weights.invalidate()

    def engine(self):
        dev = self._device()
        if self._engine is None or self._engine.device != dev:
            self._engine = cnet.CnetEngine(self.program(), dev)
            self._weights.invalidate()
        if self._weights.changed(self):
            with torch.no_grad():
                state = {k: v for k, v in self.state_dict().items() if k not in ("mean", "scale")}
                self._engine.load_state_dict(state)
            self._weights.mark_packed()
        return self._engine

    def forward(self, c):
        """models/hifigan.py:173-192: c (B, in_channels, T') -> (B, out_channels, T'*hop)."""
        eng = self.engine()
        dev = eng.device
        if c.dim() != 3 or c.size(1) != self.in_channels:
            raise ValueError(f"forward expects c (B, {self.in_channels}, T')")
        mels = [c[b].to(dev, torch.float32).transpose(0, 1).contiguous() for b in range(c.size(0))]
        return torch.stack([o.transpose(0, 1) for o in eng.infer(mels)], 0)

    def inference(self, c, normalize_before=False):
        """models/hifigan.py:251-265: c (T', in_channels) -> (T'*hop, out_channels)."""
        return self.inference_batch([c], normalize_before)[0]

    def inference_batch(self, cs, normalize_before=False):
        dev = self._device()
        eng = self.engine()
        cs = [torch.as_tensor(c, dtype=torch.float32).to(dev).contiguous() for c in cs]
        for c in cs:
            if c.dim() != 2 or c.size(1) != self.in_channels:
                raise ValueError(f"c must be (T', {self.in_channels})")
        mean = scale = None
        if normalize_before:
            mean, scale = self.mean, self.scale
        return eng.infer(cs, mean, scale)
