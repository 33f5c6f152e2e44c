"""Host-side engine over the C-ABI: config translation, weight flattening/packing, batch plans,
workspace and launch on the caller's current HIP stream.

This module is plumbing around ``libpwg_hip.so``; all generator arithmetic runs in the HIP
kernels. torch is used for device memory and the current stream only.
"""

import ctypes
import logging
import os
import operator
from collections import OrderedDict

import numpy as np
import torch

from . import _lib


def _scales(params):
    return list(params.get("upsample_params", {}).get("upsample_scales", [4, 4, 4, 4]))


def make_config(params):
    """Translate ParallelWaveGANGenerator constructor kwargs (models/parallel_wavegan.py:24-43)
    into a PwgConfig, raising NotImplementedError for options outside the hot path."""
    up = dict(params.get("upsample_params", {"upsample_scales": [4, 4, 4, 4]}))
    if not params.get("upsample_conditional_features", True):
        raise NotImplementedError("upsample_conditional_features=False is not supported")
    net = params.get("upsample_net", "ConvInUpsampleNetwork")
    if net not in ("ConvInUpsampleNetwork", "UpsampleNetwork"):
        raise NotImplementedError(f"upsample_net={net!r} is not supported")
    if up.get("nonlinear_activation") is not None:
        raise NotImplementedError("upsample nonlinear_activation is not supported")
    if up.get("freq_axis_kernel_size", 1) != 1:
        raise NotImplementedError("freq_axis_kernel_size != 1 is not supported")
    mode = up.get("interpolate_mode", "nearest")
    if mode not in INTERPOLATE_MODES:
        raise NotImplementedError(f"interpolate_mode={mode!r} is not supported (nearest, nearest-exact, area, bilinear)")
    scales = list(up.get("upsample_scales", [4, 4, 4, 4]))
    if not 1 <= len(scales) <= _lib.PWG_MAX_SCALES:
        raise NotImplementedError("1..8 upsample scales supported")
    cfg = _lib.PwgConfig()
    cfg.in_channels = int(params.get("in_channels", 1))
    cfg.out_channels = int(params.get("out_channels", 1))
    cfg.kernel_size = int(params.get("kernel_size", 3))
    cfg.layers = int(params.get("layers", 30))
    cfg.stacks = int(params.get("stacks", 3))
    cfg.residual_channels = int(params.get("residual_channels", 64))
    cfg.gate_channels = int(params.get("gate_channels", 128))
    cfg.skip_channels = int(params.get("skip_channels", 64))
    cfg.aux_channels = int(params.get("aux_channels", 80))
    cfg.aux_context_window = int(params.get("aux_context_window", 2))
    cfg.use_causal_conv = int(bool(params.get("use_causal_conv", False)))
    cfg.use_conv_in = int(net == "ConvInUpsampleNetwork")
    cfg.num_scales = len(scales)
    for i, s in enumerate(scales):
        cfg.upsample_scales[i] = int(s)
    cfg.interpolate_mode = INTERPOLATE_MODES[mode]
    return cfg


# Stretch2d modes (layers/upsample.py:43-45) the engine computes: F.interpolate with scale_factor
# (1, s) on (B, 1, C, T); "nearest-exact" and "area" give nearest's map at integer scales, and
# "bilinear" is linear along time (scale 1 along the channel axis is the identity)
INTERPOLATE_MODES = {"nearest": 0, "nearest-exact": 0, "area": 0, "bilinear": 1}


def ref_weight_keys(params):
    """(state-dict key, rows) in the C-ABI's reference order (include/pwg.h,
    pwg_ref_weight_count). key is ``None`` for an absent bias (bias=False), passed as ``rows``
    zeros."""
    L = int(params.get("layers", 30))
    G = int(params.get("gate_channels", 128))
    S = int(params.get("skip_channels", 64))
    R = int(params.get("residual_channels", 64))
    net = params.get("upsample_net", "ConvInUpsampleNetwork")
    bias = params.get("bias", True)
    keys = [("first_conv.weight", 0), ("first_conv.bias", 0)]
    if net == "ConvInUpsampleNetwork":
        keys.append(("upsample_net.conv_in.weight", 0))
        prefix = "upsample_net.upsample.up_layers"
    else:
        prefix = "upsample_net.up_layers"
    for i in range(len(_scales(params))):
        keys.append((f"{prefix}.{2 * i + 1}.weight", 0))
    for l in range(L):
        p = f"conv_layers.{l}"
        keys += [
            (f"{p}.conv.weight", 0),
            (f"{p}.conv.bias" if bias else None, G),
            (f"{p}.conv1x1_aux.weight", 0),
            (f"{p}.conv1x1_skip.weight", 0),
            (f"{p}.conv1x1_skip.bias" if bias else None, S),
            (f"{p}.conv1x1_out.weight", 0),
            (f"{p}.conv1x1_out.bias" if bias else None, R),
        ]
    keys += [
        ("last_conv_layers.1.weight", 0),
        ("last_conv_layers.1.bias", 0),
        ("last_conv_layers.3.weight", 0),
        ("last_conv_layers.3.bias", 0),
    ]
    return keys


def _to_numpy(v):
    return v.detach().cpu().numpy() if torch.is_tensor(v) else np.asarray(v)


def fold_weight_norm(state):
    """{k: ndarray} with weight_g/weight_v pairs folded to ``weight`` = g * v / ||v|| (norm over
    every dim but 0), the torch.nn.utils.weight_norm(dim=0) definition used by
    apply_weight_norm/remove_weight_norm (models/parallel_wavegan.py:175-195). Load-time
    parameter preprocessing, not part of the forward."""
    out = {}
    for k, v in state.items():
        if k.endswith(".weight_g"):
            continue
        if k.endswith(".weight_v"):
            base = k[: -len(".weight_v")]
            g = torch.from_numpy(np.ascontiguousarray(_to_numpy(state[base + ".weight_g"]), np.float32))
            vv = torch.from_numpy(np.ascontiguousarray(_to_numpy(v), np.float32))
            out[base + ".weight"] = torch._weight_norm(vv, g, 0).numpy()
        else:
            out[k] = _to_numpy(v)
    return out


# Bumped whenever any module registers a parameter (module.weight = Parameter(...),
# register_parameter, weight-norm add/remove): invalidates every WeightTracker's parameter list.
_PARAM_REGISTRATIONS = [0]


def _on_parameter_registration(module, name, param):
    _PARAM_REGISTRATIONS[0] += 1


torch.nn.modules.module.register_module_parameter_registration_hook(_on_parameter_registration)


def first_parameter(module):
    """module's first parameter, cached on the module until a parameter registration anywhere (or
    the module's _apply, which the drop-ins route here through ``forget_device``): the drop-ins ask
    for their device on every call, and ``next(module.parameters())`` walks the module tree
    (~20-50 us per call on a 100-module generator)."""
    c = module.__dict__.get("_pwg_first_param")
    if c is None or c[0] != _PARAM_REGISTRATIONS[0]:
        c = (_PARAM_REGISTRATIONS[0], next(module.parameters()))
        module.__dict__["_pwg_first_param"] = c
    return c[1]


def forget_device(module):
    module.__dict__.pop("_pwg_first_param", None)


_DATA_PTR = torch.Tensor.data_ptr
_VERSION = operator.attrgetter("_version")


class WeightTracker:
    """Per-call "do the packed weights still match the module?" check for the drop-in modules.

    The first version re-walked ``module.parameters()`` per call (640 us for PWG v1's 221
    parameters). This keeps the parameter list (re-collected only after a parameter registration
    anywhere or an explicit ``invalidate()``, which the modules call from ``_apply``, i.e.
    ``.to()``/``.cuda()``) and compares each listed tensor's ``(data_ptr, _version)``:
    - ``_version`` catches in-place updates through the parameter itself (load_state_dict's
      ``copy_``, optimizer steps, ``add_`` under no_grad);
    - ``data_ptr`` catches storage replacement, ``p.data = t``, which keeps ``_version``.
    Not detectable without reading the values: an in-place write through the ``.data`` alias
    (``p.data.copy_(t)``, ``p.data.mul_(s)``): ``.data`` is a new tensor with its own version
    counter over the same storage. After such a write call ``invalidate_weights()`` on the module
    (or re-load the state dict). ~25 us per check."""

    def __init__(self):
        self._key = None
        self._params = None
        self._sig = None

    def invalidate(self):
        self._key = None
        self._sig = None

    def _signature(self):
        ps = self._params
        return tuple(map(_DATA_PTR, ps)), tuple(map(_VERSION, ps))

    def changed(self, module, extra=()):
        """extra: tensors outside module.parameters() the packed image also holds (a PQMF
        filter buffer); compared by identity as well as storage and version."""
        key = (_PARAM_REGISTRATIONS[0], id(module), tuple(id(t) for t in extra))
        if key != self._key:
            self._params = list(module.parameters()) + list(extra)
            self._key = key
            self._sig = None
        return self._signature() != self._sig

    def mark_packed(self):
        self._sig = self._signature()


class HostHandle:
    """A pwg handle used for host-only work (packing, shape queries); needs no GPU."""

    def __init__(self, params):
        self._lib = _lib.load()
        self.params = dict(params)
        self.config = make_config(self.params)
        h = ctypes.c_void_p()
        _lib.check(self._lib.pwg_create(ctypes.byref(self.config), 0, ctypes.byref(h)))
        self._h = h
        self.receptive_field_size = self._lib.pwg_receptive_field_size(h)
        self.upsample_factor = self._lib.pwg_upsample_factor(h)
        self.ref_weight_count = self._lib.pwg_ref_weight_count(h)
        self.packed_weight_count = self._lib.pwg_packed_weight_count(h)

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and h.value:
            self._lib.pwg_destroy(h)
            self._h = None

    def flatten_state_dict(self, state):
        """Reference-order flat float32 vector (include/pwg.h) from a state dict."""
        folded = fold_weight_norm(state)
        fill = []
        for k, rows in ref_weight_keys(self.params):
            if k is None:
                fill.append(np.zeros(rows, np.float32))
                continue
            if k not in folded:
                raise KeyError(f"missing generator weight {k!r}")
            fill.append(np.ascontiguousarray(folded[k], dtype=np.float32).reshape(-1))
        flat = np.concatenate(fill).astype(np.float32)
        if flat.size != self.ref_weight_count:
            raise ValueError(f"weight count {flat.size} != expected {self.ref_weight_count}")
        return flat

    def pack(self, state):
        """Host-side packed image (np.float32, pwg_packed_weight_count).

        Sets ``split_range_ok``: False when a weight of the split-f16 images exceeds the fp16 range
        (pwg_pack_weights returned PWG_ERR_RANGE); the image is then complete for the exact-fp32
        layer kernels only."""
        flat = self.flatten_state_dict(state)
        packed = np.empty(self.packed_weight_count, np.float32)
        rc = self._lib.pwg_pack_weights(self._h, flat.ctypes.data, packed.ctypes.data)
        self.split_range_ok = rc != _lib.PWG_ERR_RANGE
        if rc != _lib.PWG_ERR_RANGE:
            _lib.check(rc)
        return packed


class Plan:
    """A planned batch (pwg_plan_create): utterance descriptors uploaded once, reusable for
    every batch of the same lengths."""

    def __init__(self, engine, frames, layout):
        lib = _lib.load()
        self.engine = engine
        self.frames = tuple(int(f) for f in frames)
        self.layout = layout
        arr = (ctypes.c_longlong * len(self.frames))(*self.frames)
        ptr = ctypes.c_void_p()
        _lib.check(lib.pwg_plan_create(engine._h, len(self.frames), arr, layout, ctypes.byref(ptr)))
        self._p = ptr
        self.total_samples = lib.pwg_plan_total_samples(ptr)
        self.padded_samples = lib.pwg_plan_padded_samples(ptr)
        self.workspace_bytes = lib.pwg_plan_workspace_bytes(ptr)
        self._lib = lib

    def __del__(self):
        p = getattr(self, "_p", None)
        if p is not None and p.value:
            self._lib.pwg_plan_destroy(p)
            self._p = None


def warm_batch_kernels(device):
    """The drop-ins' batch path concatenates the utterances' inputs (torch.cat) and slices the
    output: run both once on ``device`` so their first use is not inside a timed call."""
    a = torch.zeros(3, dtype=torch.float32, device=device)
    torch.cat([a[:1], a[1:]])
    torch.cat([a.view(3, 1), a.view(3, 1)], dim=1)


class Engine:
    """One generator configuration on one device.

    ``load_state_dict`` takes a generator state dict (folded or weight-norm form), packs it with
    pwg_pack_weights and uploads the image; ``run`` launches one forward of a plan.
    """

    def __init__(self, params, device):
        self.params = dict(params)
        self.device = torch.device(device)
        if self.device.type != "cuda":
            raise RuntimeError("the PWG engine runs on a ROCm GPU only (no CPU fallback)")
        lib = _lib.load()
        self._lib = lib
        self.config = make_config(self.params)
        h = ctypes.c_void_p()
        idx = self.device.index if self.device.index is not None else torch.cuda.current_device()
        _lib.check(lib.pwg_create(ctypes.byref(self.config), idx, ctypes.byref(h)))
        self._h = h
        self.receptive_field_size = lib.pwg_receptive_field_size(h)
        self.upsample_factor = lib.pwg_upsample_factor(h)
        self.ref_weight_count = lib.pwg_ref_weight_count(h)
        self.packed_weight_count = lib.pwg_packed_weight_count(h)
        self.packed = None
        self._plans = OrderedDict()
        self._workspaces = {}  # one per stream: concurrent runs on different streams never share one
        self.timing_enabled = False
        self.split_range_ok = True
        self.range_reruns = 0  # runs redone on the exact-fp32 kernel after a split-f16 range flag
        self.sync_reruns = 0  # grid-synchronised runs redone per-layer (the GPU was shared)
        # consecutive sync reruns; at SYNC_FAIL_STREAK the engine stops using the synchronised
        # forward for SYNC_RETRY_RUNS runs (a persistently shared GPU would otherwise pay the
        # residency wait, a stream sync and a full per-layer rerun on every call)
        self._sync_streak = 0
        self._sync_saved = None  # the sync plan limit while suspended
        self._sync_retry_in = 0
        self.layer_kernel = self.get_option("layer_kernel")

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and h.value:
            self._plans = OrderedDict()
            self._lib.pwg_destroy(h)
            self._h = None

    # ---------------------------------------------------------------- weights
    flatten_state_dict = HostHandle.flatten_state_dict
    pack = HostHandle.pack

    def load_state_dict(self, state):
        packed = self.pack(state)
        if not self.split_range_ok and self.layer_kernel in (2, 3):
            logging.warning("generator weights exceed the fp16 pair range of the split-f16 layer kernel: "
                            "using the exact-fp32 layer kernel")
            self.set_option("layer_kernel", "persistent")
        self.set_packed(torch.from_numpy(packed).to(self.device))
        return self.packed

    def set_packed(self, packed_dev):
        if packed_dev.device != self.device or packed_dev.dtype != torch.float32:
            raise ValueError("packed weights must be float32 on the engine's device")
        if packed_dev.numel() != self.packed_weight_count or not packed_dev.is_contiguous():
            raise ValueError("packed weight image has the wrong size")
        first = self.packed is None
        self.packed = packed_dev
        if first:
            self.reserve_workspace()

    # Workspace reserved when the weights load (outside any call), so a serving loop's first call at
    # a new batch shape does not pay a fresh device allocation (hipMalloc of a new caching-allocator
    # segment: the B = 16, T' = 64 first call cost 9.3 ms against 2.0 ms steady, round 5). 512 MiB
    # covers ~650 k samples (~27 s of 24 kHz audio) per call at ~820 B per sample; PWG_WORKSPACE_RESERVE_MB
    # overrides (0: none).
    WORKSPACE_RESERVE_MB = 512

    def reserve_workspace(self, nbytes=None, stream=None):
        """Grow ``stream``'s cached workspace to ``nbytes`` now (default: PWG_WORKSPACE_RESERVE_MB
        or WORKSPACE_RESERVE_MB MiB), and run the batch path's concatenation once: torch loads a
        kernel's code object on its first use, and the first ``inference_batch`` paid that (13 ms
        for torch.cat, tools/diag/first_call_b16.py) inside the call."""
        if nbytes is None:
            nbytes = int(os.environ.get("PWG_WORKSPACE_RESERVE_MB", self.WORKSPACE_RESERVE_MB)) << 20
        if nbytes > 0:
            self.workspace(nbytes, stream)
        warm_batch_kernels(self.device)

    # ---------------------------------------------------------------- plans
    def plan(self, frames, layout=_lib.PWG_LAYOUT_INFERENCE):
        key = (tuple(int(f) for f in frames), layout)
        p = self._plans.get(key)
        if p is None:
            p = Plan(self, key[0], layout)
            self._plans[key] = p
            while len(self._plans) > 16:
                self._plans.popitem(last=False)
        else:
            self._plans.move_to_end(key)
        return p

    def workspace(self, nbytes, stream=None):
        """The cached workspace of ``stream`` (default: the current stream), grown to ``nbytes``
        and allocated on that stream, so runs on different streams never share buffers."""
        if stream is None:
            stream = torch.cuda.current_stream(self.device)
        key = stream.cuda_stream
        ws = self._workspaces.get(key)
        if ws is None or ws.numel() < nbytes:
            # grow geometrically (x1.5): a run of growing batch shapes reallocates O(log) times
            grow = int(ws.numel() * 1.5) if ws is not None else 0
            self._workspaces.pop(key, None)
            ws = None
            with torch.cuda.stream(stream):
                ws = torch.empty(max(int(nbytes), grow, 256), dtype=torch.uint8, device=self.device)
            self._workspaces[key] = ws
        return ws

    def release_workspace(self):
        """Drop the cached workspaces (the caching allocator keeps the memory for reuse)."""
        self._workspaces = {}

    def release_stream(self, stream):
        """pwg_release_stream: free the handle's pinned status word for ``stream`` and this engine's
        workspace for it; call before the stream is destroyed when streams are created per request."""
        key = stream.cuda_stream
        self._workspaces.pop(key, None)
        _lib.check(self._lib.pwg_release_stream(self._h, ctypes.c_void_p(key)))

    # ---------------------------------------------------------------- options
    LAYER_KERNELS = {"persistent": 0, "tiled": 1, "split": 2, "split16": 3}

    def set_option(self, option, value):
        """pwg_set_option: option in {"layer_kernel", "waves_per_wg", "wg_per_cu", "fuse_first_conv",
        "pipeline", "half_blocks", "sync"}. "pipeline" (largest padded plan on the layer-pipelined launch, 0 = never)
        applies to plans created afterwards: the cached plans are dropped."""
        opts = self._OPTS
        if option == "layer_kernel" and isinstance(value, str):
            value = self.LAYER_KERNELS[value]
        if option == "layer_kernel" and int(value) in (2, 3) and not self.split_range_ok:
            raise _lib.RangeError("the loaded weights exceed the fp16 pair range of the split-f16 layer kernels")
        _lib.check(self._lib.pwg_set_option(self._h, opts[option], int(value)))
        if option == "layer_kernel":
            self.layer_kernel = int(value)
        if option == "pipeline":
            self._plans = OrderedDict()

    _OPTS = {"layer_kernel": _lib.PWG_OPT_LAYER_KERNEL, "waves_per_wg": _lib.PWG_OPT_WAVES_PER_WG,
             "wg_per_cu": _lib.PWG_OPT_WG_PER_CU, "fuse_first_conv": _lib.PWG_OPT_FUSE_FIRST_CONV,
             "pipeline": _lib.PWG_OPT_PIPELINE, "half_blocks": _lib.PWG_OPT_HALF_BLOCKS,
             "sync": _lib.PWG_OPT_SYNC, "sync_abort": _lib.PWG_OPT_SYNC_ABORT,
             "sync_timeout": _lib.PWG_OPT_SYNC_TIMEOUT}
    SYNC_FAIL_STREAK = 3
    SYNC_RETRY_RUNS = 256

    def get_option(self, option):
        v = ctypes.c_longlong()
        _lib.check(self._lib.pwg_get_option(self._h, self._OPTS[option], ctypes.byref(v)))
        return int(v.value)

    # ---------------------------------------------------------------- timing
    def set_timing(self, enable):
        self.timing_enabled = bool(enable)
        _lib.check(self._lib.pwg_set_timing(self._h, int(enable)))

    def timing_span(self):
        """pwg_timing_span: device ms from the first timed launch's start to the last one's end
        (gaps included); call before collect_timing."""
        v = ctypes.c_double()
        _lib.check(self._lib.pwg_timing_span(self._h, ctypes.byref(v)))
        return v.value

    def collect_timing(self):
        ms = (ctypes.c_double * len(_lib.KERNEL_BUCKETS))()
        n = (ctypes.c_longlong * len(_lib.KERNEL_BUCKETS))()
        _lib.check(self._lib.pwg_timing_collect(self._h, ms, n))
        return {k: (ms[i], n[i]) for i, k in enumerate(_lib.KERNEL_BUCKETS)}

    # ---------------------------------------------------------------- run
    def run(self, plan, mel, noise, out, mean=None, scale=None, stream=None, check=True):
        """Enqueue one forward of ``plan`` on ``stream`` (default: torch's current stream).

        check=True (the drop-in's setting) runs the split-f16 range check after the forward
        (pwg_run_status, one stream synchronisation) and, when a value left the fp16 pair range,
        redoes the forward on the exact-fp32 layer kernel, so the result always holds fp32
        semantics. check=False only enqueues (the bench's timed loop; check afterwards with
        ``run_status``)."""
        if stream is None:
            stream = torch.cuda.current_stream(self.device)
        self._sync_tick()
        self._enqueue(plan, mel, noise, out, mean, scale, stream)
        if check:
            self._range_check(plan, mel, noise, out, mean, scale, stream)
        return out

    def _range_check(self, plan, mel, noise, out, mean, scale, stream):
        """Split-f16 range check of the run just enqueued on ``stream``; a flagged run is redone
        on the exact-fp32 layer kernel. A grid-synchronised run that did not complete
        (PWG_ERR_RERUN: the GPU was shared, or a grid-barrier wait gave up; its output is NaN) is
        redone on the per-layer launches first."""
        if self.layer_kernel not in (2, 3):
            return
        try:
            try:
                self.run_status(plan, stream)
                self._sync_streak = 0
            except _lib.RerunError as e:
                self._enqueue_per_layer(plan, mel, noise, out, mean, scale, stream)
                self._note_sync_rerun(e)
                self.run_status(plan, stream)
        except _lib.RangeError as e:
            logging.warning("%s; rerunning on the exact-fp32 layer kernel", e)
            kernel = self.layer_kernel
            self.set_option("layer_kernel", "persistent")
            try:
                self._enqueue(plan, mel, noise, out, mean, scale, stream)
            finally:
                self.set_option("layer_kernel", kernel)
            self.range_reruns += 1

    def _note_sync_rerun(self, err):
        """Count a PWG_ERR_RERUN; after SYNC_FAIL_STREAK in a row, stop using the synchronised
        forward for SYNC_RETRY_RUNS runs (then try it again)."""
        self.sync_reruns += 1
        self._sync_streak += 1
        if self._sync_streak >= self.SYNC_FAIL_STREAK and self._sync_saved is None:
            logging.warning("%s (%d runs in a row): per-layer launches for the next %d runs",
                            err, self._sync_streak, self.SYNC_RETRY_RUNS)
            self._sync_saved = self.get_option("sync")
            self._sync_retry_in = self.SYNC_RETRY_RUNS
            _lib.check(self._lib.pwg_set_option(self._h, _lib.PWG_OPT_SYNC, 0))

    def _sync_tick(self):
        """Called once per forward a caller asks for (run / infer), never from inside a rerun
        (_enqueue_per_layer saves and restores PWG_OPT_SYNC around its own enqueue): restore the
        synchronised forward after a suspension. One more failure then suspends it again at once."""
        if self._sync_saved is None:
            return
        self._sync_retry_in -= 1
        if self._sync_retry_in <= 0:
            _lib.check(self._lib.pwg_set_option(self._h, _lib.PWG_OPT_SYNC, self._sync_saved))
            self._sync_saved = None
            self._sync_streak = self.SYNC_FAIL_STREAK - 1

    def _enqueue_per_layer(self, plan, mel, noise, out, mean, scale, stream):
        """Redo a run on the per-layer launches: the grid-synchronised forward and the layer
        pipeline off for this one enqueue (set through the C-ABI directly: the cached plans stay)."""
        lib, h = self._lib, self._h
        sync, pipe = self.get_option("sync"), self.get_option("pipeline")
        _lib.check(lib.pwg_set_option(h, _lib.PWG_OPT_SYNC, 0))
        _lib.check(lib.pwg_set_option(h, _lib.PWG_OPT_PIPELINE, 0))
        try:
            self._enqueue(plan, mel, noise, out, mean, scale, stream)
        finally:
            _lib.check(lib.pwg_set_option(h, _lib.PWG_OPT_SYNC, sync))
            _lib.check(lib.pwg_set_option(h, _lib.PWG_OPT_PIPELINE, pipe))

    def run_status(self, plan, stream=None):
        """pwg_run_status of the last run on ``stream``'s workspace: raises _lib.RangeError when the
        split-f16 range flag is set (synchronises the stream)."""
        if stream is None:
            stream = torch.cuda.current_stream(self.device)
        ws = self.workspace(plan.workspace_bytes, stream)
        _lib.check(self._lib.pwg_run_status(plan._p, ws.data_ptr(), stream.cuda_stream))

    def _enqueue(self, plan, mel, noise, out, mean, scale, stream):
        if self.packed is None:
            raise RuntimeError("no weights loaded")
        for name, t in (("mel", mel), ("noise", noise), ("out", out)):
            if t.device != self.device or t.dtype != torch.float32 or not t.is_contiguous():
                raise ValueError(f"{name} must be a contiguous float32 tensor on {self.device}")
        A = self.config.aux_channels
        w = self.config.aux_context_window
        nf = sum(plan.frames)
        want_mel = nf * A if plan.layout == _lib.PWG_LAYOUT_INFERENCE else len(plan.frames) * A * (plan.frames[0] + 2 * w)
        if mel.numel() != want_mel:
            raise ValueError(f"mel has {mel.numel()} elements, plan needs {want_mel}")
        if noise.numel() != plan.total_samples:
            raise ValueError(f"noise has {noise.numel()} elements, plan needs {plan.total_samples}")
        if out.numel() != plan.total_samples * self.config.out_channels:
            raise ValueError("output buffer has the wrong size")
        mp = sp = None
        if mean is not None:
            mean = mean.to(self.device, torch.float32).contiguous()
            scale = scale.to(self.device, torch.float32).contiguous()
            mp, sp = mean.data_ptr(), scale.data_ptr()
        ws = self.workspace(plan.workspace_bytes, stream)
        _lib.check(
            self._lib.pwg_run(
                plan._p,
                self.packed.data_ptr(),
                mel.data_ptr(),
                noise.data_ptr(),
                mp,
                sp,
                out.data_ptr(),
                ws.data_ptr(),
                stream.cuda_stream,
            )
        )
        return out

    def infer(self, mels, noises, mean=None, scale=None, refresh=None):
        """Ragged batch of inference() calls in ONE engine pass.

        mels: list of (T'_u, aux) float32 device tensors; noises: list of (T_u,) or (T_u, 1).
        Returns a list of (T_u, out_channels) tensors (views of one output buffer).
        refresh: optional callable run after the forward is enqueued and before the range check;
        it returns True when it re-packed the weights (the drop-in module's weight check, run while
        the GPU works), and the forward is then enqueued again on the new image.
        """
        frames = [int(m.shape[0]) for m in mels]
        plan = self.plan(frames, _lib.PWG_LAYOUT_INFERENCE)
        mel = torch.cat([m.reshape(-1) for m in mels]) if len(mels) > 1 else mels[0].reshape(-1).contiguous()
        noise = torch.cat([n.reshape(-1) for n in noises]) if len(noises) > 1 else noises[0].reshape(-1).contiguous()
        O = self.config.out_channels
        out = torch.empty(plan.total_samples * O, dtype=torch.float32, device=self.device)
        if refresh is None:
            self.run(plan, mel, noise, out, mean, scale)
        else:
            stream = torch.cuda.current_stream(self.device)
            self._sync_tick()
            self._enqueue(plan, mel, noise, out, mean, scale, stream)
            if refresh():  # the weights changed under the enqueued forward: redo it on the new image
                self._enqueue(plan, mel, noise, out, mean, scale, stream)
            self._range_check(plan, mel, noise, out, mean, scale, stream)
        res, off = [], 0
        H = self.upsample_factor
        for f in frames:
            T = f * H
            res.append(out[off * O:(off + T) * O].view(T, O))
            off += T
        return res


class GraphedRun:
    """One forward of ``plan`` captured as a HIP graph (pwg_graph_create) over static buffers
    owned by this object: refill ``mel`` / ``noise`` (or pass them to ``__call__``), replay the
    whole forward as one submission, read ``out`` (overwritten by the next replay). For repeated
    shapes (fixed-size streaming chunks, a serving loop over one batch shape); ``Engine.run`` is
    the general path. The graph keeps the weights, options and plan of capture time: reloading
    weights into the engine (a new packed image) invalidates it, and __call__ then raises."""

    def __init__(self, engine, plan, mean=None, scale=None):
        if plan.layout != _lib.PWG_LAYOUT_INFERENCE:
            raise ValueError("graphs are captured for the inference layout")
        if engine.packed is None:
            raise RuntimeError("no weights loaded")
        if engine.timing_enabled:
            raise RuntimeError("disable engine timing before capturing a graph")
        dev = engine.device
        self.engine, self.plan = engine, plan
        A, O = engine.config.aux_channels, engine.config.out_channels
        self.mel = torch.zeros(sum(plan.frames) * A, dtype=torch.float32, device=dev)
        self.noise = torch.zeros(plan.total_samples, dtype=torch.float32, device=dev)
        self.out = torch.empty(plan.total_samples * O, dtype=torch.float32, device=dev)
        self.mean = self.scale = None
        if mean is not None:
            self.mean = mean.to(dev, torch.float32).contiguous().clone()
            self.scale = scale.to(dev, torch.float32).contiguous().clone()
        self.ws = torch.empty(max(int(plan.workspace_bytes), 256), dtype=torch.uint8, device=dev)
        self._packed = engine.packed
        self._kernel = engine.layer_kernel
        stream = torch.cuda.Stream(dev)  # capture needs a created stream
        torch.cuda.synchronize(dev)
        g = ctypes.c_void_p()
        _lib.check(engine._lib.pwg_graph_create(
            plan._p, self._packed.data_ptr(), self.mel.data_ptr(), self.noise.data_ptr(),
            self.mean.data_ptr() if self.mean is not None else None,
            self.scale.data_ptr() if self.scale is not None else None,
            self.out.data_ptr(), self.ws.data_ptr(), stream.cuda_stream, ctypes.byref(g)))
        self._g = g
        self._lib = engine._lib

    def __del__(self):
        g = getattr(self, "_g", None)
        if g is not None and g.value:
            self._lib.pwg_graph_destroy(g)
            self._g = None

    def __call__(self, mel=None, noise=None, check=True):
        """Replay on torch's current stream; returns ``out`` (flat, total_samples * out_channels).
        check=True: split-f16 range check (one synchronisation); a flagged replay is redone by
        ``Engine.run`` on the exact-fp32 kernel, as the drop-in does."""
        eng = self.engine
        if eng.packed is not self._packed:
            raise RuntimeError("the engine's weights changed after capture: capture a new GraphedRun")
        if mel is not None:
            self.mel.copy_(mel.reshape(-1))
        if noise is not None:
            self.noise.copy_(noise.reshape(-1))
        stream = torch.cuda.current_stream(eng.device)
        _lib.check(self._lib.pwg_graph_launch(self._g, stream.cuda_stream))
        if check and self._kernel in (2, 3):
            try:
                try:
                    _lib.check(self._lib.pwg_run_status(self.plan._p, self.ws.data_ptr(), stream.cuda_stream))
                except _lib.RerunError:
                    # (the rerun uses the engine's workspace for this stream, so its status is there)
                    eng._enqueue_per_layer(self.plan, self.mel, self.noise, self.out, self.mean, self.scale, stream)
                    eng.sync_reruns += 1
                    eng.run_status(self.plan, stream)
            except _lib.RangeError as e:
                logging.warning("%s; rerunning on the exact-fp32 layer kernel", e)
                kernel = eng.layer_kernel
                eng.set_option("layer_kernel", "persistent")
                try:
                    eng._enqueue(self.plan, self.mel, self.noise, self.out, self.mean, self.scale, stream)
                finally:
                    eng.set_option("layer_kernel", kernel)
                eng.range_reruns += 1
        return self.out

