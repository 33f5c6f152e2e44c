"""Drop-in ``ParallelWaveGANGenerator`` whose forward runs on the MI355X HIP engine.

Mirrors parallel_wavegan.models.ParallelWaveGANGenerator
(/root/reference/parallel_wavegan/models/parallel_wavegan.py:21-263): same constructor
arguments, same sub-module names and therefore the same state-dict keys (including the
old-style ``weight_g``/``weight_v`` of weight norm), ``forward(z, c)``, ``inference(c, x,
normalize_before)``, ``remove_weight_norm``/``apply_weight_norm``, ``register_stats``,
``receptive_field_size`` and ``upsample_factor``.

The torch Conv modules below only HOLD parameters (so checkpoints load unchanged); they are
never called. Every forward goes through ``libpwg_hip.so``; on a CPU module ``forward`` and
``inference`` raise instead of falling back.
"""

import copy
import logging
import math

import numpy as np
import torch

from . import _lib
from .engine import Engine, WeightTracker, first_parameter, forget_device


def _kaiming_conv1d(*args, **kwargs):
    """torch Conv1d holding parameters with the reference init (layers/residual_block.py:19-30)."""
    m = torch.nn.Conv1d(*args, **kwargs)
    torch.nn.init.kaiming_normal_(m.weight, nonlinearity="relu")
    if m.bias is not None:
        torch.nn.init.constant_(m.bias, 0.0)
    return m


def _fir_conv2d(scale, causal):
    """Conv2d(1,1,(1,2s+1)) FIR holder, init 1/(2s+1) (layers/upsample.py:48-59,97-103)."""
    pad = (0, 2 * scale) if causal else (0, scale)
    m = torch.nn.Conv2d(1, 1, kernel_size=(1, 2 * scale + 1), padding=pad, bias=False)
    m.weight.data.fill_(1.0 / (2 * scale + 1))
    return m


class _Stretch2d(torch.nn.Module):
    """Parameter-free placeholder keeping up_layers indices equal to the reference's
    (Stretch2d at even indices, layers/upsample.py:16-45)."""

    def __init__(self, x_scale, y_scale=1, mode="nearest"):
        super().__init__()
        self.x_scale, self.y_scale, self.mode = x_scale, y_scale, mode


class _UpsampleNetwork(torch.nn.Module):
    """Holder for layers/upsample.py:62-128 parameters."""

    def __init__(self, upsample_scales, use_causal_conv=False, **unused):
        super().__init__()
        self.use_causal_conv = use_causal_conv
        self.up_layers = torch.nn.ModuleList()
        for s in upsample_scales:
            self.up_layers += [_Stretch2d(s), _fir_conv2d(s, use_causal_conv)]


class _ConvInUpsampleNetwork(torch.nn.Module):
    """Holder for layers/upsample.py:131-194 parameters."""

    def __init__(self, upsample_scales, aux_channels=80, aux_context_window=0, use_causal_conv=False, **unused):
        super().__init__()
        self.aux_context_window = aux_context_window
        self.use_causal_conv = use_causal_conv and aux_context_window > 0
        k = aux_context_window + 1 if use_causal_conv else 2 * aux_context_window + 1
        self.conv_in = _kaiming_conv1d(aux_channels, aux_channels, kernel_size=k, bias=False)
        self.upsample = _UpsampleNetwork(upsample_scales, use_causal_conv=use_causal_conv)


class _ResidualBlock(torch.nn.Module):
    """Holder for WaveNetResidualBlock parameters (layers/residual_block.py:43-100)."""

    def __init__(self, kernel_size, residual_channels, gate_channels, skip_channels, aux_channels,
                 dilation, bias, use_causal_conv):
        super().__init__()
        if use_causal_conv:
            padding = (kernel_size - 1) * dilation
        else:
            assert (kernel_size - 1) % 2 == 0, "Not support even number kernel size."
            padding = (kernel_size - 1) // 2 * dilation
        self.dilation = dilation
        self.use_causal_conv = use_causal_conv
        self.conv = _kaiming_conv1d(residual_channels, gate_channels, kernel_size, padding=padding,
                                    dilation=dilation, bias=bias)
        self.conv1x1_aux = _kaiming_conv1d(aux_channels, gate_channels, 1, bias=False)
        self.conv1x1_out = _kaiming_conv1d(gate_channels // 2, residual_channels, 1, bias=bias)
        self.conv1x1_skip = _kaiming_conv1d(gate_channels // 2, skip_channels, 1, bias=bias)


class ParallelWaveGANGenerator(torch.nn.Module):
    """Parallel WaveGAN generator; forward/inference run on the HIP engine."""

    def __init__(
        self,
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
        bias=True,
        use_weight_norm=True,
        use_causal_conv=False,
        upsample_conditional_features=True,
        upsample_net="ConvInUpsampleNetwork",
        upsample_params={"upsample_scales": [4, 4, 4, 4]},
    ):
        super().__init__()
        upsample_params = copy.deepcopy(upsample_params)  # the reference mutates it in place
        self.in_channels = in_channels
        self.out_channels = out_channels
        self.aux_channels = aux_channels
        self.aux_context_window = aux_context_window
        self.layers = layers
        self.stacks = stacks
        self.kernel_size = kernel_size
        assert layers % stacks == 0
        layers_per_stack = layers // stacks
        self._params = dict(
            in_channels=in_channels, out_channels=out_channels, kernel_size=kernel_size, layers=layers,
            stacks=stacks, residual_channels=residual_channels, gate_channels=gate_channels,
            skip_channels=skip_channels, aux_channels=aux_channels, aux_context_window=aux_context_window,
            dropout=dropout, bias=bias, use_causal_conv=use_causal_conv,
            upsample_conditional_features=upsample_conditional_features, upsample_net=upsample_net,
            upsample_params=copy.deepcopy(upsample_params),
        )

        self.first_conv = _kaiming_conv1d(in_channels, residual_channels, 1, bias=True)
        if not upsample_conditional_features:
            raise NotImplementedError("upsample_conditional_features=False is not supported")
        if upsample_net == "ConvInUpsampleNetwork":
            self.upsample_net = _ConvInUpsampleNetwork(
                aux_channels=aux_channels, aux_context_window=aux_context_window,
                use_causal_conv=use_causal_conv, **upsample_params)
        elif upsample_net == "UpsampleNetwork":
            self.upsample_net = _UpsampleNetwork(use_causal_conv=use_causal_conv, **upsample_params)
        else:
            raise NotImplementedError(f"upsample_net={upsample_net!r} is not supported")
        self.upsample_factor = int(np.prod(upsample_params["upsample_scales"]))

        self.conv_layers = torch.nn.ModuleList()
        for layer in range(layers):
            self.conv_layers += [
                _ResidualBlock(kernel_size, residual_channels, gate_channels, skip_channels, aux_channels,
                               2 ** (layer % layers_per_stack), bias, use_causal_conv)
            ]
        self.last_conv_layers = torch.nn.ModuleList([
            torch.nn.ReLU(inplace=True),
            _kaiming_conv1d(skip_channels, skip_channels, 1, bias=True),
            torch.nn.ReLU(inplace=True),
            _kaiming_conv1d(skip_channels, out_channels, 1, bias=True),
        ])
        if use_weight_norm:
            self.apply_weight_norm()
        self._engine = None
        self._weights = WeightTracker()

    # ------------------------------------------------------------------ reference API
    def remove_weight_norm(self):
        """models/parallel_wavegan.py:175-185."""
        def _remove(m):
            try:
                torch.nn.utils.remove_weight_norm(m)
            except ValueError:
                return
        self.apply(_remove)

    def apply_weight_norm(self):
        """models/parallel_wavegan.py:187-195."""
        def _apply(m):
            if isinstance(m, (torch.nn.Conv1d, torch.nn.Conv2d)):
                torch.nn.utils.weight_norm(m)
        self.apply(_apply)

    @staticmethod
    def _get_receptive_field_size(layers, stacks, kernel_size, dilation=lambda x: 2**x):
        assert layers % stacks == 0
        layers_per_cycle = layers // stacks
        dilations = [dilation(i % layers_per_cycle) for i in range(layers)]
        return (kernel_size - 1) * sum(dilations) + 1

    @property
    def receptive_field_size(self):
        return self._get_receptive_field_size(self.layers, self.stacks, self.kernel_size)

    def register_stats(self, stats):
        """models/parallel_wavegan.py:213-229 (.npy; .h5 needs h5py)."""
        assert stats.endswith(".h5") or stats.endswith(".npy")
        if stats.endswith(".h5"):
            import h5py  # noqa: F401  (absent in this image -> ImportError, as the reference)
            with h5py.File(stats, "r") as f:
                mean = f["mean"][()].reshape(-1)
                scale = f["scale"][()].reshape(-1)
        else:
            arr = np.load(stats)
            mean = arr[0].reshape(-1)
            scale = arr[1].reshape(-1)
        dev = first_parameter(self).device
        self.register_buffer("mean", torch.from_numpy(np.asarray(mean)).float().to(dev))
        self.register_buffer("scale", torch.from_numpy(np.asarray(scale)).float().to(dev))
        logging.info("Successfully registered stats as buffer.")

    # ------------------------------------------------------------------ engine plumbing
    def _device(self):
        dev = first_parameter(self).device
        if dev.type != "cuda":
            raise RuntimeError(
                "parallelwavegan_amd.ParallelWaveGANGenerator runs on a ROCm GPU only; move the "
                "module with .to('cuda') (there is no CPU fallback)")
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
        """The HIP engine with this module's current weights packed (re-packed when a
        parameter changes: WeightTracker)."""
        dev = self._device()
        if self._engine is None or self._engine.device != dev:
            self._engine = Engine(self._params, dev)
            self._weights.invalidate()
        if self._weights.changed(self):
            with torch.no_grad():
                state = {k: v for k, v in self.state_dict().items() if k not in ("mean", "scale")}
                self._engine.load_state_dict(state)
            self._weights.mark_packed()
        return self._engine

    # ------------------------------------------------------------------ forward paths
    def forward(self, z, c):
        """Batched forward (models/parallel_wavegan.py:144-173).

        z (B, 1, T) noise, c (B, aux, T' + 2w) context-padded features -> (B, out, T).
        """
        eng = self.engine()
        dev = eng.device
        if z.dim() != 3 or c.dim() != 3 or z.size(0) != c.size(0):
            raise ValueError("forward expects z (B, 1, T) and c (B, aux, T'+2w)")
        if c.size(1) != self.aux_channels:
            raise ValueError(f"c has {c.size(1)} channels, expected {self.aux_channels}")
        frames = c.size(-1) - 2 * self.aux_context_window
        assert frames >= 1 and frames * self.upsample_factor == z.size(-1)  # parallel_wavegan.py:158
        B, T = z.size(0), z.size(-1)
        z = z.to(dev, torch.float32).contiguous()
        c = c.to(dev, torch.float32).contiguous()
        plan = eng.plan([frames] * B, _lib.PWG_LAYOUT_FORWARD)
        out = torch.empty(B, self.out_channels, T, dtype=torch.float32, device=dev)
        eng.run(plan, c, z, out)
        return out

    def inference(self, c=None, x=None, normalize_before=False):
        """Single-utterance inference (models/parallel_wavegan.py:231-263).

        c (T', aux) ndarray/tensor, x (T, 1) or None -> (T, out_channels) on the module device.
        """
        dev = self._device()
        if x is not None:
            if not isinstance(x, torch.Tensor):
                x = torch.tensor(x, dtype=torch.float).to(dev)
            x = x.to(dev, torch.float32)
        else:
            assert c is not None
            # same generator and device hop as the reference (:250-253): CPU randn, then .to()
            x = torch.randn(1, 1, len(c) * self.upsample_factor).to(dev).view(-1, 1)
        if c is None:
            raise NotImplementedError("inference without conditioning features is not supported")
        if not isinstance(c, torch.Tensor):
            c = torch.tensor(c, dtype=torch.float).to(dev)
        c = c.to(dev, torch.float32)
        return self.inference_batch([c], [x], normalize_before)[0]

    def _engine_deferred(self):
        """(engine, refresh): the engine with the weights packed at the last check, and a callable
        that runs the weight check (WeightTracker, ~25-50 us of host time for PWG v1) and re-packs
        when a parameter changed, returning True then. The drop-in calls refresh() after the
        forward is enqueued, so the check overlaps the GPU; a re-pack redoes the forward. Before
        the first pack (or on a new device) the engine is built and checked up front."""
        dev = self._device()
        if self._engine is None or self._engine.device != dev or self._engine.packed is None:
            return self.engine(), None

        def refresh():
            if not self._weights.changed(self):
                return False
            self.engine()
            return True

        return self._engine, refresh

    def inference_batch(self, cs, xs=None, normalize_before=False):
        """Ragged multi-utterance inference in ONE engine pass (no reference counterpart; the
        reference decodes one utterance per call, bin/decode.py:236-268).

        cs: list of (T'_u, aux); xs: list of (T_u, 1) or None (CPU randn per utterance).
        Returns a list of (T_u, out_channels) device tensors.
        """
        eng, refresh = self._engine_deferred()
        dev = eng.device
        cs = [torch.as_tensor(c, dtype=torch.float32).to(dev).contiguous() for c in cs]
        for c in cs:
            if c.dim() != 2 or c.size(1) != self.aux_channels:
                raise ValueError(f"c must be (T', {self.aux_channels})")
        if xs is None:
            xs = [torch.randn(1, 1, c.size(0) * self.upsample_factor).to(dev).view(-1, 1) for c in cs]
        xs = [torch.as_tensor(x, dtype=torch.float32).to(dev).contiguous() for x in xs]
        for c, x in zip(cs, xs):
            assert x.numel() == c.size(0) * self.upsample_factor  # forward's length assert
        mean = scale = None
        if normalize_before:
            mean, scale = self.mean, self.scale  # AttributeError without register_stats, as the reference
        return eng.infer(cs, xs, mean, scale, refresh=refresh)
