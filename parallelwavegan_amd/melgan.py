"""Drop-in ``MelGANGenerator`` (MelGAN, multi-band MelGAN) and ``PQMF`` running on the MI355X
conv-network executor (include/pwg_cnet.h).

Mirrors parallel_wavegan.models.MelGANGenerator (/root/reference/parallel_wavegan/models/
melgan.py:17-257), ResidualStack (layers/residual_stack.py:13-85) and PQMF (layers/pqmf.py:14-149):
same constructor arguments, the same ``melgan`` Sequential indices and therefore the same
state-dict keys (weight-norm ``weight_g``/``weight_v`` included), ``forward(c)``,
``inference(c, normalize_before)`` (with ``self.pqmf`` synthesis when set, as
utils.load_model does for out_channels > 1, utils/utils.py:347-358), ``remove_weight_norm``,
``apply_weight_norm``, ``register_stats``.

The torch modules only HOLD parameters; the forward is lowered to a conv program (one fused MFMA
op per Conv1d / ConvTranspose1d / ResidualStack half) and runs in libpwg_hip.so. A CPU module
raises instead of falling back.
"""

import logging

import numpy as np
import torch

from . import causal, cnet
from .engine import WeightTracker, first_parameter, forget_device


def _kaiser(m, beta):
    """Symmetric Kaiser window, the scipy.signal.windows.kaiser(m, beta) definition."""
    n = np.arange(m, dtype=np.float64)
    alpha = (m - 1) / 2.0
    return np.i0(beta * np.sqrt(1.0 - ((n - alpha) / alpha) ** 2)) / np.i0(float(beta))


def design_prototype_filter(taps=62, cutoff_ratio=0.142, beta=9.0):
    """Kaiser-window prototype low-pass (layers/pqmf.py:14-48): (taps + 1,) float64."""
    assert taps % 2 == 0, "The number of taps mush be even number."
    assert 0.0 < cutoff_ratio < 1.0, "Cutoff ratio must be > 0.0 and < 1.0."
    n = np.arange(taps + 1) - 0.5 * taps
    wc = np.pi * cutoff_ratio
    with np.errstate(invalid="ignore", divide="ignore"):
        h = np.sin(wc * n) / (np.pi * n)
    h[taps // 2] = cutoff_ratio
    return h * _kaiser(taps + 1, beta)


def pqmf_filters(subbands=4, taps=62, cutoff_ratio=0.142, beta=9.0):
    """(analysis, synthesis) cosine-modulated filter banks, float64 (subbands, taps + 1)
    (layers/pqmf.py:72-95)."""
    h = design_prototype_filter(taps, cutoff_ratio, beta)
    n = np.arange(taps + 1) - taps / 2
    ana = np.zeros((subbands, taps + 1))
    syn = np.zeros((subbands, taps + 1))
    for k in range(subbands):
        phase = (2 * k + 1) * (np.pi / (2 * subbands)) * n
        ana[k] = 2 * h * np.cos(phase + (-1) ** k * np.pi / 4)
        syn[k] = 2 * h * np.cos(phase - (-1) ** k * np.pi / 4)
    return ana, syn


class PQMF(torch.nn.Module):
    """PQMF filter bank holder (layers/pqmf.py:51-149). ``synthesis`` is executed by the engine
    as the last op of a MelGANGenerator program; the module keeps the same buffers
    (analysis_filter, synthesis_filter, updown_filter) so state dicts match."""

    def __init__(self, subbands=4, taps=62, cutoff_ratio=0.142, beta=9.0):
        super().__init__()
        ana, syn = pqmf_filters(subbands, taps, cutoff_ratio, beta)
        self.register_buffer("analysis_filter", torch.from_numpy(ana).float().unsqueeze(1))
        self.register_buffer("synthesis_filter", torch.from_numpy(syn).float().unsqueeze(0))
        updown = torch.zeros((subbands, subbands, subbands)).float()
        for k in range(subbands):
            updown[k, k, 0] = 1.0
        self.register_buffer("updown_filter", updown)
        self.subbands = subbands
        self.taps = taps
        self.pad_fn = torch.nn.ConstantPad1d(taps // 2, 0.0)

    def synthesis_taps(self):
        """(subbands, taps + 1) float32 synthesis filters as the engine consumes them."""
        return self.synthesis_filter[0].detach().cpu().numpy().astype(np.float32)


class ResidualStack(torch.nn.Module):
    """Parameter holder with the reference's sub-module layout (layers/residual_stack.py:13-85):
    stack = [act, pad, Conv1d(dilated), act, Conv1d 1x1] ([act, CausalConv1d, act, Conv1d 1x1]
    when causal), skip_layer = Conv1d 1x1."""

    def __init__(self, kernel_size=3, channels=32, dilation=1, bias=True, nonlinear_activation="LeakyReLU",
                 nonlinear_activation_params={"negative_slope": 0.2}, pad="ReflectionPad1d", pad_params={},
                 use_causal_conv=False):
        super().__init__()
        act = getattr(torch.nn, nonlinear_activation)
        if not use_causal_conv:
            assert (kernel_size - 1) % 2 == 0, "Not support even number kernel size."
            self.stack = torch.nn.Sequential(
                act(**nonlinear_activation_params),
                getattr(torch.nn, pad)((kernel_size - 1) // 2 * dilation, **pad_params),
                torch.nn.Conv1d(channels, channels, kernel_size, dilation=dilation, bias=bias),
                act(**nonlinear_activation_params),
                torch.nn.Conv1d(channels, channels, 1, bias=bias),
            )
        else:  # residual_stack.py:65-80
            self.stack = torch.nn.Sequential(
                act(**nonlinear_activation_params),
                causal.CausalConv1d(channels, channels, kernel_size, dilation=dilation, bias=bias, pad=pad,
                                    pad_params=pad_params),
                act(**nonlinear_activation_params),
                torch.nn.Conv1d(channels, channels, 1, bias=bias),
            )
        self.skip_layer = torch.nn.Conv1d(channels, channels, 1, bias=bias)


def _slope(m):
    if isinstance(m, torch.nn.LeakyReLU):
        return float(m.negative_slope)
    if isinstance(m, torch.nn.ReLU):
        return 0.0
    raise NotImplementedError(f"activation {type(m).__name__} is not supported by the MI355X engine")


def _pad_of(m):
    """(pad, mode) of a padding module, None for anything else."""
    if isinstance(m, torch.nn.ReflectionPad1d):
        l, r = m.padding
        if l != r:
            raise NotImplementedError("asymmetric padding")
        return l, cnet.PAD_REFLECT
    if isinstance(m, torch.nn.ConstantPad1d):
        l, r = m.padding
        if l != r or m.value != 0.0:
            raise NotImplementedError("only symmetric zero or reflection padding is supported")
        return l, cnet.PAD_ZERO
    if isinstance(m, torch.nn.ReplicationPad1d):
        raise NotImplementedError("ReplicationPad1d inside the generator is not supported")
    return None


def _bias_key(prefix, conv):
    return prefix + ".bias" if conv.bias is not None else None


class MelGANGenerator(torch.nn.Module):
    """models/melgan.py:17-257, executed on the MI355X conv-network engine."""

    def __init__(self, in_channels=80, out_channels=1, kernel_size=7, channels=512, bias=True,
                 upsample_scales=[8, 8, 2, 2], stack_kernel_size=3, stacks=3, nonlinear_activation="LeakyReLU",
                 nonlinear_activation_params={"negative_slope": 0.2}, pad="ReflectionPad1d", pad_params={},
                 use_final_nonlinear_activation=True, use_weight_norm=True, use_causal_conv=False):
        super().__init__()
        assert channels >= np.prod(upsample_scales)
        assert channels % (2 ** len(upsample_scales)) == 0
        if not use_causal_conv:
            assert (kernel_size - 1) % 2 == 0, "Not support even number kernel size."
        act = getattr(torch.nn, nonlinear_activation)
        padm = getattr(torch.nn, pad)
        if not use_causal_conv:
            mods = [padm((kernel_size - 1) // 2, **pad_params),
                    torch.nn.Conv1d(in_channels, channels, kernel_size, bias=bias)]
        else:  # models/melgan.py:73-84
            mods = [causal.CausalConv1d(in_channels, channels, kernel_size, bias=bias, pad=pad, pad_params=pad_params)]
        ch = channels
        for i, s in enumerate(upsample_scales):
            mods.append(act(**nonlinear_activation_params))
            if not use_causal_conv:
                mods.append(torch.nn.ConvTranspose1d(ch, ch // 2, s * 2, stride=s, padding=s // 2 + s % 2,
                                                     output_padding=s % 2, bias=bias))
            else:
                mods.append(causal.CausalConvTranspose1d(ch, ch // 2, s * 2, stride=s, bias=bias))
            ch //= 2
            for j in range(stacks):
                mods.append(ResidualStack(stack_kernel_size, ch, stack_kernel_size ** j, bias, nonlinear_activation,
                                          nonlinear_activation_params, pad, pad_params, use_causal_conv))
        mods.append(act(**nonlinear_activation_params))
        if not use_causal_conv:
            mods.append(padm((kernel_size - 1) // 2, **pad_params))
            mods.append(torch.nn.Conv1d(ch, out_channels, kernel_size, bias=bias))
        else:
            mods.append(causal.CausalConv1d(ch, out_channels, kernel_size, bias=bias, pad=pad, pad_params=pad_params))
        if use_final_nonlinear_activation:
            mods.append(torch.nn.Tanh())
        self.melgan = torch.nn.Sequential(*mods)
        self.in_channels, self.out_channels = in_channels, out_channels
        self.use_causal_conv = bool(use_causal_conv)
        self.upsample_factor = int(np.prod(upsample_scales))
        if use_weight_norm:
            self.apply_weight_norm()
        self.reset_parameters()
        self.pqmf = None
        self._engines = {}

    # ------------------------------------------------------------------ reference API
    def remove_weight_norm(self):
        """models/melgan.py:172-182."""
        def _remove(m):
            try:
                torch.nn.utils.remove_weight_norm(m)
            except ValueError:
                return
        self.apply(_remove)

    def apply_weight_norm(self):
        """models/melgan.py:184-194."""
        def _apply(m):
            if isinstance(m, (torch.nn.Conv1d, torch.nn.ConvTranspose1d)):
                torch.nn.utils.weight_norm(m)
        self.apply(_apply)

    def reset_parameters(self):
        """models/melgan.py:196-209: conv weights ~ N(0, 0.02)."""
        def _reset(m):
            if isinstance(m, (torch.nn.Conv1d, torch.nn.ConvTranspose1d)):
                m.weight.data.normal_(0.0, 0.02)
        self.apply(_reset)

    def register_stats(self, stats):
        """models/melgan.py:211-227 (.npy; .h5 needs h5py, absent here)."""
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
    def program(self, with_pqmf):
        """The conv program of ``self.melgan`` (+ PQMF synthesis)."""
        P = cnet.Program(self.in_channels)
        cur, cur_ch, rate = 0, self.in_channels, 1
        slope, pad = 1.0, None
        first = True
        for idx, m in enumerate(self.melgan):
            key = f"melgan.{idx}"
            if isinstance(m, (torch.nn.LeakyReLU, torch.nn.ReLU)):
                slope = _slope(m)
            elif _pad_of(m) is not None:
                pad = _pad_of(m)
            elif isinstance(m, torch.nn.Conv1d):
                k, d = m.kernel_size[0], m.dilation[0]
                if pad is None:
                    p, mode = m.padding[0], cnet.PAD_ZERO
                else:
                    p, mode = pad
                    if m.padding[0] != 0:
                        raise NotImplementedError("padding module and conv padding together")
                if m.stride[0] != 1 or m.groups != 1:
                    raise NotImplementedError("strided / grouped conv")
                dst = P.buffer(m.out_channels, rate)
                src = P.src(cur, cur_ch, k, d, p, mode, slope, key + ".weight", normalize=first)
                P.conv(key, dst, m.out_channels, [src], bias=_bias_key(key, m))
                cur, cur_ch, slope, pad, first = dst, m.out_channels, 1.0, None, False
            elif isinstance(m, causal.CausalConv1d):
                if pad is not None:
                    raise NotImplementedError("padding module before a CausalConv1d")
                dst = P.buffer(m.conv.out_channels, rate)
                P.conv(key + ".conv", dst, m.conv.out_channels,
                       [causal.conv_src(P, cur, cur_ch, m, key, slope, normalize=first)],
                       bias=_bias_key(key + ".conv", m.conv))
                cur, cur_ch, slope, first = dst, m.conv.out_channels, 1.0, False
            elif isinstance(m, causal.CausalConvTranspose1d):
                if pad is not None:
                    raise NotImplementedError("padding module before a CausalConvTranspose1d")
                src, s = causal.convt_src(P, cur, cur_ch, m, key, slope, normalize=first)
                rate *= s
                dst = P.buffer(m.deconv.out_channels, rate)
                P.convt(key + ".deconv", dst, m.deconv.out_channels, src, s, 0, 0, bias=_bias_key(key + ".deconv", m.deconv))
                cur, cur_ch, slope, first = dst, m.deconv.out_channels, 1.0, False
            elif isinstance(m, torch.nn.ConvTranspose1d):
                s = m.stride[0]
                if m.kernel_size[0] != 2 * s or pad is not None:
                    raise NotImplementedError("ConvTranspose1d must have kernel 2*stride")
                rate *= s
                dst = P.buffer(m.out_channels, rate)
                src = P.src(cur, cur_ch, pre_slope=slope, weight=key + ".weight", normalize=first)
                P.convt(key, dst, m.out_channels, src, s, m.padding[0], m.output_padding[0], bias=_bias_key(key, m))
                cur, cur_ch, slope, first = dst, m.out_channels, 1.0, False
            elif isinstance(m, ResidualStack):
                if slope != 1.0 or pad is not None:
                    raise NotImplementedError("activation before a ResidualStack")
                h = P.buffer(cur_ch, rate)
                if len(m.stack) == 4:  # causal: [act, CausalConv1d, act, 1x1]
                    a0, cc, a1, c1 = m.stack
                    i1 = 3
                    P.conv(key + ".stack.1.conv", h, cur_ch,
                           [causal.conv_src(P, cur, cur_ch, cc, key + ".stack.1", _slope(a0), normalize=first)],
                           bias=_bias_key(key + ".stack.1.conv", cc.conv))
                else:
                    a0, pd, cd, a1, c1 = m.stack
                    i1 = 4
                    pp, mode = _pad_of(pd)
                    P.conv(key + ".stack.2", h, cur_ch,
                           [P.src(cur, cur_ch, cd.kernel_size[0], cd.dilation[0], pp, mode, _slope(a0),
                                  key + ".stack.2.weight", normalize=first)],
                           bias=_bias_key(key + ".stack.2", cd))
                y = P.buffer(cur_ch, rate)
                # stack(c) + skip_layer(c) as ONE two-source 1x1 op over [lrelu(h); c]
                P.conv(key + f".stack.{i1}+skip_layer", y, cur_ch,
                       [P.src(h, cur_ch, pre_slope=_slope(a1), weight=key + f".stack.{i1}.weight"),
                        P.src(cur, cur_ch, weight=key + ".skip_layer.weight", normalize=first)],
                       bias=_bias_key(key + f".stack.{i1}", c1), bias2=_bias_key(key + ".skip_layer", m.skip_layer))
                cur, first = y, False
            elif isinstance(m, torch.nn.Tanh):
                P.ops[-1]["post_act"] = cnet.ACT_TANH
            else:
                raise NotImplementedError(f"{type(m).__name__} in a MelGAN generator")
        extra = {}
        if with_pqmf:
            if self.pqmf.subbands != cur_ch:
                raise ValueError("PQMF subbands must equal out_channels")
            taps = self.pqmf.synthesis_taps()
            out = P.buffer(1, rate * self.pqmf.subbands)
            P.pqmf("pqmf.synthesis", out, cur, self.pqmf.subbands, "pqmf.synthesis_taps", taps.shape[1])
            extra["pqmf.synthesis_taps"] = taps
        else:
            # the op writing the last buffer defines the output
            if cur != len(P.channels) - 1:
                raise AssertionError("program output is not the last buffer")
        return P, extra

    # ------------------------------------------------------------------ engine plumbing
    def _device(self):
        dev = first_parameter(self).device
        if dev.type != "cuda":
            raise RuntimeError("parallelwavegan_amd.MelGANGenerator runs on a ROCm GPU only; move the module "
                               "with .to('cuda') (there is no CPU fallback)")
        return dev

    def _apply(self, fn, *args, **kwargs):
        forget_device(self)
        for ent in getattr(self, "_engines", {}).values():
            ent[1].invalidate()  # .to() / .cuda() replace parameter storage
        return super()._apply(fn, *args, **kwargs)

    def invalidate_weights(self):
        """Force a re-pack on the next call (after writes through ``p.data`` aliases, which the
        WeightTracker cannot see)."""
        for ent in self._engines.values():
            ent[1].invalidate()

    def engine(self, with_pqmf=None):
        if with_pqmf is None:
            with_pqmf = self.pqmf is not None
        dev = self._device()
        ent = self._engines.get(with_pqmf)
        if ent is None or ent[0].device != dev:
            P, extra = self.program(with_pqmf)
            ent = [cnet.CnetEngine(P, dev), WeightTracker()]
            self._engines[with_pqmf] = ent
        if ent[1].changed(self, (self.pqmf.synthesis_filter,) if with_pqmf else ()):
            _, extra = self.program(with_pqmf)
            with torch.no_grad():
                state = {k: v for k, v in self.state_dict().items() if not k.startswith("pqmf.") and
                         k not in ("mean", "scale")}
                ent[0].load_state_dict(state, extra)
            ent[1].mark_packed()
        return ent[0]

    # ------------------------------------------------------------------ forward paths
    def forward(self, c):
        """models/melgan.py:160-170: c (B, in_channels, T') -> (B, out_channels, T'*hop) (no PQMF)."""
        eng = self.engine(False)
        dev = eng.device
        if c.dim() != 3 or c.size(1) != self.in_channels:
            raise ValueError(f"forward expects c (B, {self.in_channels}, T')")
        B, _, T = c.shape
        mels = [c[b].to(dev, torch.float32).transpose(0, 1).contiguous() for b in range(B)]
        outs = eng.infer(mels)
        return torch.stack([o.transpose(0, 1) for o in outs], 0)

    def inference(self, c, normalize_before=False):
        """models/melgan.py:229-246: c (T', in_channels) -> (T'*hop[*subbands], 1 or out)."""
        return self.inference_batch([c], normalize_before)[0]

    def inference_batch(self, cs, normalize_before=False):
        """Ragged multi-utterance inference in one engine pass (no reference counterpart)."""
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
