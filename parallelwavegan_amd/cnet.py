"""ctypes binding of the conv-network executor (include/pwg_cnet.h) and the program builder the
MelGAN-family drop-ins use.

A ``Program`` is a list of fused conv ops over numbered time-major buffers (buffer 0 = the mel
input, the last buffer = the output) plus the reference-order flat weight layout: every op names
its weights by state-dict key, and ``CnetEngine.pack`` flattens a (weight-norm folded) state dict
in that order before the library packs it into MFMA fragments. Nothing here computes: the forward
runs in libpwg_hip.so, and a missing library or a CPU device raises.
"""

import ctypes
import logging
import os
from collections import OrderedDict

import numpy as np
import torch

from . import _lib
from .engine import fold_weight_norm

CONV, CONVT, PQMF = 0, 1, 2
PAD_ZERO, PAD_REFLECT, PAD_REPLICATE = 0, 1, 2
ACT_NONE, ACT_LRELU, ACT_TANH = 0, 1, 2

CNET_SYMBOLS = tuple(n for n in _lib.EXPORTED_SYMBOLS if n.startswith("pwg_cnet_"))


class PwgCnetSrc(ctypes.Structure):
    _fields_ = [
        ("buf", ctypes.c_int),
        ("channels", ctypes.c_int),
        ("taps", ctypes.c_int),
        ("dilation", ctypes.c_int),
        ("pad", ctypes.c_int),
        ("pad_mode", ctypes.c_int),
        ("normalize", ctypes.c_int),
        ("pre_slope", ctypes.c_float),
        ("w_off", ctypes.c_longlong),
    ]


class PwgCnetOp(ctypes.Structure):
    _fields_ = [
        ("kind", ctypes.c_int),
        ("dst", ctypes.c_int),
        ("out_channels", ctypes.c_int),
        ("src", PwgCnetSrc * 2),
        ("b_off", ctypes.c_longlong),
        ("b2_off", ctypes.c_longlong),
        ("res", ctypes.c_int),
        ("accumulate", ctypes.c_int),
        ("out_div", ctypes.c_float),
        ("post_act", ctypes.c_int),
        ("post_slope", ctypes.c_float),
        ("stride", ctypes.c_int),
        ("padding", ctypes.c_int),
        ("output_padding", ctypes.c_int),
    ]


_bound = False


def lib():
    """The loaded library with the cnet prototypes declared."""
    global _bound
    L = _lib.load()
    if not _bound:
        vp, ll = ctypes.c_void_p, ctypes.c_longlong
        L.pwg_cnet_abi_version.restype = ctypes.c_int
        L.pwg_cnet_create.argtypes = [ctypes.POINTER(PwgCnetOp), ctypes.c_int, ctypes.c_int,
                                      ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int), ll,
                                      ctypes.c_int, ctypes.POINTER(vp)]
        L.pwg_cnet_destroy.argtypes = [vp]
        L.pwg_cnet_destroy.restype = None
        L.pwg_cnet_packed_weight_count.argtypes = [vp]
        L.pwg_cnet_packed_weight_count.restype = ll
        L.pwg_cnet_pack_weights.argtypes = [vp, vp, vp]
        L.pwg_cnet_plan_create.argtypes = [vp, ctypes.c_int, ctypes.POINTER(ll), ctypes.POINTER(vp)]
        L.pwg_cnet_plan_destroy.argtypes = [vp]
        L.pwg_cnet_plan_destroy.restype = None
        L.pwg_cnet_plan_image.argtypes = [vp, ctypes.POINTER(ll), ctypes.POINTER(ll), vp, ll]
        L.pwg_cnet_plan_rows.argtypes = [vp, ctypes.c_int]
        L.pwg_cnet_plan_rows.restype = ll
        L.pwg_cnet_plan_workspace_bytes.argtypes = [vp]
        L.pwg_cnet_plan_workspace_bytes.restype = ll
        L.pwg_cnet_run.argtypes = [vp] * 8
        L.pwg_cnet_run_status.argtypes = [vp, vp, vp]
        ip = ctypes.POINTER(ctypes.c_int)
        L.pwg_cnet_plan_schedule.argtypes = [vp, ctypes.c_int, ip, ip, ip, ip]
        L.pwg_cnet_set_timing.argtypes = [vp, ctypes.c_int]
        L.pwg_cnet_set_option.argtypes = [vp, ctypes.c_int, ctypes.c_longlong]
        L.pwg_cnet_timing_collect.argtypes = [vp, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ll)]
        L.pwg_cnet_timing_span.argtypes = [vp, ctypes.POINTER(ctypes.c_double)]
        L.pwg_cnet_release_stream.argtypes = [vp, vp]
        if L.pwg_cnet_abi_version() != 1:
            raise RuntimeError("libpwg_hip cnet ABI version mismatch")
        _bound = True
    return L


class Program:
    """Builder of a conv-network program. Weights are referenced by state-dict key; ``weights``
    keeps the reference order (first use) and sizes."""

    def __init__(self, in_channels):
        self.channels = [int(in_channels)]
        self.rate = [1]
        self.ops = []
        self.names = []
        self.weights = OrderedDict()  # key -> number of floats

    def buffer(self, channels, rate):
        self.channels.append(int(channels))
        self.rate.append(int(rate))
        return len(self.channels) - 1

    def _w(self, key, count):
        if key is None:
            return -1
        if key in self.weights:
            if self.weights[key] != count:
                raise ValueError(f"weight {key} used with two sizes")
        else:
            self.weights[key] = int(count)
        return key

    @staticmethod
    def src(buf, channels, taps=1, dilation=1, pad=0, pad_mode=PAD_ZERO, pre_slope=1.0, weight=None,
            normalize=False):
        return dict(buf=buf, channels=channels, taps=taps, dilation=dilation, pad=pad, pad_mode=pad_mode,
                    pre_slope=pre_slope, weight=weight, normalize=normalize)

    def conv(self, name, dst, out_channels, srcs, bias=None, bias2=None, res=-1, accumulate=False, out_div=1.0,
             post_act=ACT_NONE, post_slope=1.0):
        for s in srcs:
            self._w(s["weight"], out_channels * s["channels"] * s["taps"])
        self._w(bias, out_channels)
        self._w(bias2, out_channels)
        self.ops.append(dict(kind=CONV, dst=dst, out_channels=out_channels, srcs=srcs, bias=bias, bias2=bias2,
                             res=res, accumulate=accumulate, out_div=out_div, post_act=post_act,
                             post_slope=post_slope, stride=1, padding=0, output_padding=0))
        self.names.append(name)

    def convt(self, name, dst, out_channels, src, stride, padding, output_padding, bias=None):
        self._w(src["weight"], src["channels"] * out_channels * 2 * stride)
        self._w(bias, out_channels)
        self.ops.append(dict(kind=CONVT, dst=dst, out_channels=out_channels, srcs=[src], bias=bias, bias2=None,
                             res=-1, accumulate=False, out_div=1.0, post_act=ACT_NONE, post_slope=1.0,
                             stride=stride, padding=padding, output_padding=output_padding))
        self.names.append(name)

    def pqmf(self, name, dst, src_buf, subbands, filt_key, filt_taps):
        self._w(filt_key, subbands * filt_taps)
        src = self.src(src_buf, subbands, weight=filt_key)
        self.ops.append(dict(kind=PQMF, dst=dst, out_channels=1, srcs=[src], bias=None, bias2=None, res=-1,
                             accumulate=False, out_div=1.0, post_act=ACT_NONE, post_slope=1.0, stride=subbands,
                             padding=filt_taps, output_padding=0))
        self.names.append(name)

    # ------------------------------------------------------------------ lowering
    def offsets(self):
        off, o = {}, 0
        for k, n in self.weights.items():
            off[k] = o
            o += n
        return off, o

    def c_ops(self):
        off, _ = self.offsets()
        arr = (PwgCnetOp * len(self.ops))()
        for i, op in enumerate(self.ops):
            c = arr[i]
            c.kind, c.dst, c.out_channels = op["kind"], op["dst"], op["out_channels"]
            for j in range(2):
                s = c.src[j]
                if j < len(op["srcs"]):
                    d = op["srcs"][j]
                    s.buf, s.channels, s.taps, s.dilation = d["buf"], d["channels"], d["taps"], d["dilation"]
                    s.pad, s.pad_mode, s.normalize = d["pad"], d["pad_mode"], int(bool(d["normalize"]))
                    s.pre_slope = d["pre_slope"]
                    s.w_off = off[d["weight"]] if d["weight"] is not None else -1
                else:
                    s.buf = -1
            c.b_off = off[op["bias"]] if op["bias"] is not None else -1
            c.b2_off = off[op["bias2"]] if op["bias2"] is not None else -1
            c.res, c.accumulate, c.out_div = op["res"], int(op["accumulate"]), op["out_div"]
            c.post_act, c.post_slope = op["post_act"], op["post_slope"]
            c.stride, c.padding, c.output_padding = op["stride"], op["padding"], op["output_padding"]
        return arr

    def flatten(self, state, extra=None):
        """Reference-order flat float32 vector from a state dict (+ host-side constants such as
        the PQMF filters in ``extra``)."""
        folded = fold_weight_norm(state)
        if extra:
            folded.update(extra)
        parts = []
        for k, n in self.weights.items():
            if k not in folded:
                raise KeyError(f"missing generator weight {k!r}")
            v = np.ascontiguousarray(folded[k], dtype=np.float32).reshape(-1)
            if v.size != n:
                raise ValueError(f"weight {k!r} has {v.size} values, expected {n}")
            parts.append(v)
        return np.concatenate(parts).astype(np.float32)


class CnetPlan:
    def __init__(self, eng, frames):
        self.eng = eng
        self.frames = tuple(int(f) for f in frames)
        arr = (ctypes.c_longlong * len(self.frames))(*self.frames)
        p = ctypes.c_void_p()
        _lib.check(eng._lib.pwg_cnet_plan_create(eng._h, len(self.frames), arr, ctypes.byref(p)))
        self._p = p
        nb = len(eng.program.channels)
        self.out_rows = eng._lib.pwg_cnet_plan_rows(p, nb - 1)
        self.workspace_bytes = eng._lib.pwg_cnet_plan_workspace_bytes(p)
        self.runs = 0  # forwards run with this plan (CnetEngine captures a graph from the second on)

    def image(self):
        """pwg_cnet_plan_image: (byte offset in the workspace, int32 array) of the device lists
        every run writes there, as the host built and checked them."""
        off, n = ctypes.c_longlong(), ctypes.c_longlong()
        _lib.check(self.eng._lib.pwg_cnet_plan_image(self._p, ctypes.byref(off), ctypes.byref(n), None, 0))
        img = np.zeros(n.value, np.int32)
        _lib.check(self.eng._lib.pwg_cnet_plan_image(self._p, ctypes.byref(off), ctypes.byref(n),
                                                     img.ctypes.data, n.value))
        return off.value, img

    def __del__(self):
        p = getattr(self, "_p", None)
        h = getattr(self.eng, "_h", None)
        # (a plan outliving its engine's handle is leaked, not destroyed: its C struct points at it)
        if p is not None and p.value and h is not None and h.value:
            self.eng._lib.pwg_cnet_plan_destroy(p)
        self._p = None


class CnetEngine:
    """One program on one device: weights packed once, plans cached per utterance-length tuple."""

    def __init__(self, program, device, host_only=False):
        self.program = program
        self.host_only = bool(host_only)
        self.device = torch.device(device) if device is not None else None
        if not host_only and (self.device is None or self.device.type != "cuda"):
            raise RuntimeError("the conv-network engine runs on a ROCm GPU only (no CPU fallback)")
        L = lib()
        self._lib = L
        ops = program.c_ops()
        nb = len(program.channels)
        ch = (ctypes.c_int * nb)(*program.channels)
        rt = (ctypes.c_int * nb)(*program.rate)
        _, n_ref = program.offsets()
        idx = -1  # host-only handle: packing and checked plans, nothing on a GPU (include/pwg_cnet.h)
        if not host_only:
            idx = self.device.index if self.device.index is not None else torch.cuda.current_device()
        h = ctypes.c_void_p()
        _lib.check(L.pwg_cnet_create(ops, len(program.ops), nb, ch, rt, n_ref, idx, ctypes.byref(h)))
        self._h = h
        self.packed_weight_count = L.pwg_cnet_packed_weight_count(h)
        self.packed = None
        self._plans = OrderedDict()
        self._workspaces = {}
        self.split_f16 = True       # PWG_CNET_OPT_SPLIT_F16 (the library default)
        self.graphs = True          # replay captured forwards of small plans (set_graphs)
        # ... of programs with parallel branches (an accumulated sum: HiFiGAN's MRF blocks), the ones
        # PWG_CNET_OPT_STREAMS runs concurrently; a single chain (MelGAN) gains nothing from the graph
        # and pays its input / output copies (MB-MelGAN v2 T' = 64: 0.449 -> 0.466 ms)
        self._branchy = any(op["accumulate"] for op in program.ops)
        self._graphs = OrderedDict()
        self._uses = OrderedDict()  # runs per batch shape (frames tuple), kept across plan evictions
        self._graph_epoch = 0       # bumped by every option change: captured forwards are stale
        self._last_ws = {}          # (plan, stream) -> workspace of its last replayed forward
        self._timing = False
        self.split_range_ok = True  # the loaded weights fit the fp16 pair range
        self.range_reruns = 0       # runs redone in exact fp32 after a split-f16 range flag

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and h.value:
            self._graphs = OrderedDict()  # captured forwards hold plans: release them first
            self._last_ws = {}
            self._plans = OrderedDict()
            self._lib.pwg_cnet_destroy(h)
            self._h = None

    def pack(self, state, extra=None):
        """Host-side packed image. Sets ``split_range_ok``: False when a weight cannot be carried
        as an fp16 pair (pwg_cnet_pack_weights returned PWG_ERR_RANGE); the image is then complete
        for the exact-fp32 mode only."""
        flat = self.program.flatten(state, extra)
        packed = np.empty(self.packed_weight_count, np.float32)
        rc = self._lib.pwg_cnet_pack_weights(self._h, flat.ctypes.data, packed.ctypes.data)
        self.split_range_ok = rc != _lib.PWG_ERR_RANGE
        if rc != _lib.PWG_ERR_RANGE:
            _lib.check(rc)
        return packed

    def load_state_dict(self, state, extra=None):
        packed = self.pack(state, extra)
        if not self.split_range_ok and self.split_f16:
            logging.warning("vocoder weights exceed the fp16 pair range of the split-f16 mode: using exact fp32")
            self._set_split(False)
            self.split_f16 = False
        first = self.packed is None
        self.packed = torch.from_numpy(packed).to(self.device)
        if first and not self.host_only:
            self.reserve_workspace()
        return self.packed

    # Workspace reserved when the weights load (outside any call; see Engine.WORKSPACE_RESERVE_MB):
    # a first call at a new batch shape then pays no device allocation. A MelGAN-family plan needs
    # ~0.5-1.5 KB per output sample; 256 MiB covers B = 16 x T' = 512 of HiFiGAN v1.
    WORKSPACE_RESERVE_MB = 256

    def reserve_workspace(self, nbytes=None, stream=None):
        """Grow ``stream``'s cached workspace to ``nbytes`` (default PWG_CNET_WORKSPACE_RESERVE_MB or
        WORKSPACE_RESERVE_MB MiB) and load the batch path's concatenation kernel."""
        from .engine import warm_batch_kernels

        if nbytes is None:
            nbytes = int(os.environ.get("PWG_CNET_WORKSPACE_RESERVE_MB", self.WORKSPACE_RESERVE_MB)) << 20
        if nbytes > 0:
            self.workspace(nbytes, stream)
        warm_batch_kernels(self.device)

    def plan(self, frames):
        key = tuple(int(f) for f in frames)
        p = self._plans.get(key)
        if p is None:
            p = CnetPlan(self, key)
            self._plans[key] = p
            while len(self._plans) > 16:
                self._plans.popitem(last=False)
        else:
            self._plans.move_to_end(key)
        return p

    def workspace(self, nbytes, stream=None):
        """The cached workspace of ``stream`` (default: the current stream), grown to ``nbytes``
        and allocated on that stream: runs on different streams never share buffers."""
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
        """pwg_cnet_release_stream: free what the handle keeps for ``stream`` (auxiliary streams,
        events, pinned status word) and this engine's workspace and graphs for it; call before the
        stream is destroyed when streams are created per request."""
        key = stream.cuda_stream
        self._workspaces.pop(key, None)
        for gk in [k for k in self._graphs if k[1] == key]:
            self._graphs.pop(gk)
        for wk in [k for k in self._last_ws if k[1] == key]:
            self._last_ws.pop(wk)
        _lib.check(self._lib.pwg_cnet_release_stream(self._h, ctypes.c_void_p(key)))

    @property
    def out_channels(self):
        return self.program.channels[-1]

    @property
    def hop(self):
        return self.program.rate[-1]

    def run(self, plan, mel, out, mean=None, scale=None, stream=None, check=True):
        """Enqueue one forward of ``plan`` on ``stream`` (default: torch's current stream).

        check=True (the drop-ins' setting) reads the split-f16 range status after the forward
        (pwg_cnet_run_status: one stream synchronisation) and, when the output came out non-finite,
        redoes the forward in exact fp32, so the result always holds the reference's fp32
        semantics. check=False only enqueues (the bench's timed loop; ``run_status`` afterwards)."""
        if stream is None:
            stream = torch.cuda.current_stream(self.device)
        ws = None
        key = (id(plan), stream.cuda_stream)
        plan.runs += 1
        uses = self._uses.get(plan.frames, 0) + 1
        self._uses[plan.frames] = uses
        self._uses.move_to_end(plan.frames)
        while len(self._uses) > self.USES_CACHE:
            self._uses.popitem(last=False)
        if self._graph_ok(plan, mean, stream, uses):
            ws = self._replay(plan, mel, out, stream)
            self._last_ws[key] = ws  # run_status reads the captured forward's own workspace
        else:
            self._last_ws.pop(key, None)
            self._enqueue(plan, mel, out, mean, scale, stream)
        if check and self.split_f16:
            try:
                if ws is None:
                    self.run_status(plan, stream)
                else:
                    _lib.check(self._lib.pwg_cnet_run_status(plan._p, ws.data_ptr(), stream.cuda_stream))
            except _lib.RangeError as e:
                logging.warning("%s; rerunning in exact fp32", e)
                self._set_split(False)
                try:
                    self._enqueue(plan, mel, out, mean, scale, stream)
                finally:
                    self._set_split(True)
                self.range_reruns += 1
        return out

    # ------------------------------------------------------------------ captured forwards
    # A small plan's forward is 30-80 latency-bound launches, and with PWG_CNET_OPT_STREAMS its
    # independent launches only overlap if they are queued faster than the GPU runs them: enqueued
    # from the host (~10 us per launch with its events) HiFiGAN v1's B = 1 forward was host-bound
    # (profiles/r04_m). Small plans therefore run as a hipGraph captured once per (plan, caller
    # stream, weights, options) and replayed: input copied into the graph's buffer, replay, output
    # copied out. Same kernels, same arguments: bit-identical to the eager forward.
    # A graph is captured only for a batch shape that has run GRAPH_AFTER times (counted per frames
    # tuple, surviving plan eviction): a capture (eager warm-up, capture, instantiation) costs 4-26 ms
    # and a replay saves ~0.09 ms over the eager forward (HiFiGAN v1 B = 1: 1.67 vs 1.58 ms, DESIGN
    # sec. 11), so it pays back after ~50-300 replays. The reference's decode loop (bin/decode.py:
    # 236-268) repeats a length only occasionally (the 512-utterance RandomState(3) list: 97 repeated
    # lengths, none more than a few times), which under the round-5 policy (capture on a plan's second
    # run) paid captures it never recovered; a serving loop over a fixed shape still gets its graph.
    GRAPH_MAX_FRAMES = 512
    GRAPH_AFTER = 64
    GRAPH_CACHE = 8
    USES_CACHE = 4096

    def set_graphs(self, enable):
        """Replay captured forwards of small plans (default on); off: every forward enqueued."""
        self.graphs = bool(enable)
        self._graphs.clear()

    def _graph_ok(self, plan, mean, stream, uses):
        return (self.graphs and self._branchy and not self._timing and mean is None
                and sum(plan.frames) <= self.GRAPH_MAX_FRAMES and not torch.cuda.is_current_stream_capturing()
                and (uses >= self.GRAPH_AFTER or self._graph_key(plan, stream) in self._graphs))

    def _graph_key(self, plan, stream):
        return (id(plan), stream.cuda_stream, self.packed.data_ptr(), self.split_f16, self._graph_epoch)

    def _replay(self, plan, mel, out, stream):
        key = self._graph_key(plan, stream)
        ent = self._graphs.get(key)
        if ent is None:
            for name, t in (("mel", mel), ("out", out)):
                if t.device != self.device or t.dtype != torch.float32 or not t.is_contiguous():
                    raise ValueError(f"{name} must be a contiguous float32 tensor on {self.device}")
            # the graph's own buffers and workspace: no other run (eager forwards on a pool stream
            # of the same handle value, other graphs) ever writes them
            cs = torch.cuda.Stream(self.device)
            g_mel, g_out = torch.empty_like(mel), torch.empty_like(out)
            g_ws = torch.empty(max(int(plan.workspace_bytes), 256), dtype=torch.uint8, device=self.device)
            cs.wait_stream(stream)
            with torch.cuda.stream(cs):
                g_mel.copy_(mel)
                self._enqueue(plan, g_mel, g_out, None, None, cs, ws=g_ws)  # warm-up
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g, stream=cs, capture_error_mode="thread_local"):
                    self._enqueue(plan, g_mel, g_out, None, None, cs, ws=g_ws)
            stream.wait_stream(cs)
            # (the entry holds the plan, the weights and the workspace the graph's launches point at)
            ent = (g, g_mel, g_out, cs, g_ws, plan, self.packed)
            self._graphs[key] = ent
            while len(self._graphs) > self.GRAPH_CACHE:
                self._graphs.popitem(last=False)
        else:
            self._graphs.move_to_end(key)
        g, g_mel, g_out, cs, ws = ent[:5]
        if mel.numel() != g_mel.numel() or out.numel() != g_out.numel():
            raise ValueError("mel / output buffer has the wrong size for the plan")
        with torch.cuda.stream(stream):
            g_mel.copy_(mel)
            g.replay()
            out.copy_(g_out)
        return ws

    def schedule(self, plan):
        """pwg_cnet_plan_schedule: [(phase, stream)] per launch in program order, and the enqueue
        order (launch indices) -- what ``run`` would enqueue with the current options."""
        n = ctypes.c_int()
        _lib.check(self._lib.pwg_cnet_plan_schedule(plan._p, 0, ctypes.byref(n), None, None, None))
        k = n.value
        ph, st, od = (ctypes.c_int * k)(), (ctypes.c_int * k)(), (ctypes.c_int * k)()
        _lib.check(self._lib.pwg_cnet_plan_schedule(plan._p, k, ctypes.byref(n), ph, st, od))
        return list(zip(ph, st)), list(od)

    def run_status(self, plan, stream=None):
        """pwg_cnet_run_status of the last run on ``stream``'s workspace: raises _lib.RangeError
        when the split-f16 range flag is set (synchronises the stream)."""
        if stream is None:
            stream = torch.cuda.current_stream(self.device)
        ws = self._last_ws.get((id(plan), stream.cuda_stream))
        if ws is None:
            ws = self.workspace(plan.workspace_bytes, stream)
        _lib.check(self._lib.pwg_cnet_run_status(plan._p, ws.data_ptr(), stream.cuda_stream))

    def _enqueue(self, plan, mel, out, mean, scale, stream, ws=None):
        if self.packed is None:
            raise RuntimeError("no weights loaded")
        for name, t in (("mel", mel), ("out", out)):
            if t.device != self.device or t.dtype != torch.float32 or not t.is_contiguous():
                raise ValueError(f"{name} must be a contiguous float32 tensor on {self.device}")
        if mel.numel() != sum(plan.frames) * self.program.channels[0]:
            raise ValueError("mel has the wrong size for the plan")
        if out.numel() != plan.out_rows * self.out_channels:
            raise ValueError("output buffer has the wrong size")
        mp = sp = None
        if mean is not None:
            mean = mean.to(self.device, torch.float32).contiguous()
            scale = scale.to(self.device, torch.float32).contiguous()
            mp, sp = mean.data_ptr(), scale.data_ptr()
        if ws is None:
            ws = self.workspace(plan.workspace_bytes, stream)
        _lib.check(self._lib.pwg_cnet_run(plan._p, self.packed.data_ptr(), mel.data_ptr(), mp, sp, out.data_ptr(),
                                          ws.data_ptr(), stream.cuda_stream))
        return out

    def infer(self, mels, mean=None, scale=None):
        """Ragged batch: list of (T'_u, in_channels) device tensors -> list of (T'_u*hop, out)."""
        frames = [int(m.shape[0]) for m in mels]
        plan = self.plan(frames)
        mel = torch.cat([m.reshape(-1) for m in mels]) if len(mels) > 1 else mels[0].reshape(-1).contiguous()
        O = self.out_channels
        out = torch.empty(plan.out_rows * O, dtype=torch.float32, device=self.device)
        self.run(plan, mel, out, mean, scale)
        res, off = [], 0
        for f in frames:
            T = f * self.hop
            res.append(out[off * O:(off + T) * O].view(T, O))
            off += T
        return res

    def set_timing(self, enable):
        _lib.check(self._lib.pwg_cnet_set_timing(self._h, int(enable)))
        self._timing = bool(enable)  # per-op events: forwards run eagerly while on

    def _set_split(self, enable):
        _lib.check(self._lib.pwg_cnet_set_option(self._h, 0, int(bool(enable))))
        self._graph_epoch += 1

    def set_split_f16(self, enable):
        """pwg_cnet_set_option(PWG_CNET_OPT_SPLIT_F16): fp16-pair operands on the f16 MFMA
        (default) or exact fp32 MFMA. Refused (RangeError) for weights beyond the pair range."""
        if enable and not self.split_range_ok:
            raise _lib.RangeError("the loaded weights exceed the fp16 pair range of the split-f16 mode")
        self._set_split(enable)
        self.split_f16 = bool(enable)

    def set_fuse_pairs(self, enable):
        """pwg_cnet_set_option(PWG_CNET_OPT_FUSE_PAIRS): run conv pairs whose intermediate has no
        other reader (HiFiGAN ResBlock steps) as one kernel, intermediate in LDS (default on,
        split-f16 mode only; bit-identical to the unfused ops)."""
        _lib.check(self._lib.pwg_cnet_set_option(self._h, 1, int(bool(enable))))
        self._graph_epoch += 1

    def set_xtile(self, enable):
        """pwg_cnet_set_option(PWG_CNET_OPT_XTILE): dilated convs channel-block-major with the
        input tile staged once per 16-channel block (default on); off: the tap-major kernel and
        the fused conv pairs."""
        _lib.check(self._lib.pwg_cnet_set_option(self._h, 3, int(bool(enable))))
        self._graph_epoch += 1

    XT_DMA_RULE, XT_DMA_ALL, XT_DMA_FEWEST, XT_DMA_CONVT = 1, 2, 4, 8  # include/pwg_cnet.h flags

    def set_xt_dma(self, mode):
        """pwg_cnet_set_option(PWG_CNET_OPT_XT_DMA) flags: x-tile convs stage their weight fragments
        by DMA (global_load_lds) into two LDS buffers, overlapped with the MFMAs (bit-identical to
        the register-staged kernels): 1 the shapes where that measured faster, 2 every eligible conv,
        4 the fewest tap groups; 8 the wide ConvTranspose phases on that kernel. Default 9."""
        _lib.check(self._lib.pwg_cnet_set_option(self._h, 4, int(mode)))
        self._graph_epoch += 1

    def set_xcd_order(self, enable):
        """pwg_cnet_set_option(PWG_CNET_OPT_XCD_ORDER): the m-groups / ConvTranspose phases of one
        column block run on one XCD back to back, sharing its L2 (default on; same results)."""
        _lib.check(self._lib.pwg_cnet_set_option(self._h, 5, int(bool(enable))))
        self._graph_epoch += 1

    def set_narrow(self, mode):
        """pwg_cnet_set_option(PWG_CNET_OPT_NARROW): small launches of the x-tile family run narrow
        workgroups (1-4 waves, 1-2 m-tiles) spread over every CU: 1 (default) when a launch would
        have fewer workgroups than CUs, 2 always, 0 never. Plan-time: cached plans are dropped.
        Bit-identical."""
        _lib.check(self._lib.pwg_cnet_set_option(self._h, 6, int(mode)))
        self._graph_epoch += 1
        self._plans.clear()

    def set_streams(self, mode):
        """pwg_cnet_set_option(PWG_CNET_OPT_STREAMS): independent launches on auxiliary streams
        for plans with narrow launches (1, default), every plan (2) or never (0). Bit-identical."""
        _lib.check(self._lib.pwg_cnet_set_option(self._h, 8, int(mode)))
        self._graph_epoch += 1

    def set_mstack(self, mode):
        """pwg_cnet_set_option(PWG_CNET_OPT_MSTACK): a MelGAN stage's chain of ResidualStacks as one
        launch (pwg_mstack.hip): 1 (default) when the chain's first conv runs narrow, 2 every chain,
        0 never. Plan-time (cached plans are dropped); bit-identical."""
        _lib.check(self._lib.pwg_cnet_set_option(self._h, 9, int(mode)))
        self._graph_epoch += 1
        self._plans.clear()

    def set_presplit(self, enable):
        """pwg_cnet_set_option(PWG_CNET_OPT_PRESPLIT): DMA-ring launches write pre-split images of
        the buffers other DMA-ring launches read, which stage them as they are (default) or, 0,
        every reader converts its fp32 rows. Plan-time (cached plans are dropped); bit-identical."""
        _lib.check(self._lib.pwg_cnet_set_option(self._h, 10, 1 if enable else 0))
        self._graph_epoch += 1
        self._plans.clear()

    def set_rstack(self, mode):
        """pwg_cnet_set_option(PWG_CNET_OPT_RSTACK): batched fused ResidualStacks of 32-96 channels
        on the persistent LDS-ring kernel (pwg_rstack.hip; 1 = default, weights resident in LDS at
        <= 64 channels; 2 = weights streamed at every width) or, 0, on the x-tile stack kernel.
        Run-time; bit-identical."""
        _lib.check(self._lib.pwg_cnet_set_option(self._h, 11, int(mode)))
        self._graph_epoch += 1

    def set_narrow_dma(self, enable):
        """pwg_cnet_set_option(PWG_CNET_OPT_NARROW_DMA): narrow launches on the DMA-ring kernel
        (default) or, 0, on the narrow x-tile / tap-major kernels. Plan-time (cached plans are
        dropped); bit-identical."""
        _lib.check(self._lib.pwg_cnet_set_option(self._h, 7, 1 if enable else 0))
        self._graph_epoch += 1
        self._plans.clear()

    def set_pair_steps(self, steps):
        """pwg_cnet_set_option(PWG_CNET_OPT_PAIR_STEPS): 128-column tiles per fused-pair
        workgroup, for plans created afterwards (cached plans are dropped)."""
        _lib.check(self._lib.pwg_cnet_set_option(self._h, 2, int(steps)))
        self._graph_epoch += 1
        self._plans.clear()

    def timing_span(self):
        """pwg_cnet_timing_span: device ms from the first timed launch's start to the last one's
        end (concurrent streams counted once); call before collect_timing."""
        v = ctypes.c_double()
        _lib.check(self._lib.pwg_cnet_timing_span(self._h, ctypes.byref(v)))
        return v.value

    def collect_timing(self):
        n = len(self.program.ops)
        ms = (ctypes.c_double * n)()
        cnt = (ctypes.c_longlong * n)()
        _lib.check(self._lib.pwg_cnet_timing_collect(self._h, ms, cnt))
        return [(self.program.names[i], ms[i], cnt[i]) for i in range(n)]
