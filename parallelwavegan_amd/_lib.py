"""ctypes binding of the engine's C-ABI (include/pwg.h) and its in-tree build.

The shared library is built IN-TREE (parallelwavegan_amd/lib/libpwg_hip.so) by ``build()``
with hipcc for gfx950 so it travels with the repository snapshot. There is no fallback: if the
library is missing, ``load()`` raises, and so does every GPU entry point that needs it.

``torch`` must be imported before the library is loaded: torch ships its own
libamdhip64.so.7 and the dynamic loader then resolves our NEEDED entry to that same runtime
(one HIP runtime per process, so torch device pointers and streams are valid here).
"""

import ctypes
import os
import subprocess
import threading

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
REPO_DIR = os.path.dirname(PKG_DIR)
LIB_DIR = os.path.join(PKG_DIR, "lib")
LIB_PATH = os.environ.get("PWG_LIB_PATH") or os.path.join(LIB_DIR, "libpwg_hip.so")
CSRC = [
    os.path.join(PKG_DIR, "csrc", "pwg_kernels.hip"),
    os.path.join(PKG_DIR, "csrc", "pwg_capi.hip"),
    os.path.join(PKG_DIR, "csrc", "pwg_cnet.hip"),
    os.path.join(PKG_DIR, "csrc", "pwg_split.hip"),
    os.path.join(PKG_DIR, "csrc", "pwg_split16.hip"),
    os.path.join(PKG_DIR, "csrc", "pwg_rccl.hip"),
    os.path.join(PKG_DIR, "csrc", "pwg_mstack.hip"),
    os.path.join(PKG_DIR, "csrc", "pwg_rstack.hip"),
]
HEADERS = [
    os.path.join(REPO_DIR, "include", "pwg.h"),
    os.path.join(REPO_DIR, "include", "pwg_cnet.h"),
    os.path.join(PKG_DIR, "csrc", "pwg_internal.h"),
]
OFFLOAD_ARCH = "gfx950"

PWG_OK = 0
PWG_ERR_INVALID = 1
PWG_ERR_ASSERT = 2
PWG_ERR_HIP = 3
PWG_ERR_UNSUPPORTED = 4
PWG_ERR_RANGE = 5
PWG_ERR_RERUN = 6
PWG_RCCL_UNIQUE_ID_BYTES = 128

PWG_LAYOUT_INFERENCE = 0
PWG_LAYOUT_FORWARD = 1

KERNEL_BUCKETS = ("conv_in", "upsample", "first_conv", "residual_layer", "head")
PWG_MAX_SCALES = 8

# Every symbol include/*.h declares (checked by tests/test_abi.py).
EXPORTED_SYMBOLS = (
    "pwg_abi_version",
    "pwg_last_error",
    "pwg_create",
    "pwg_destroy",
    "pwg_receptive_field_size",
    "pwg_upsample_factor",
    "pwg_ref_weight_count",
    "pwg_packed_weight_count",
    "pwg_pack_weights",
    "pwg_plan_create",
    "pwg_plan_destroy",
    "pwg_plan_total_samples",
    "pwg_plan_padded_samples",
    "pwg_plan_workspace_bytes",
    "pwg_run",
    "pwg_run_status",
    "pwg_graph_create",
    "pwg_graph_launch",
    "pwg_graph_destroy",
    "pwg_set_option",
    "pwg_get_option",
    "pwg_set_timing",
    "pwg_release_stream",
    "pwg_timing_collect",
    "pwg_timing_span",
    "pwg_rccl_unique_id",
    "pwg_rccl_comm_create",
    "pwg_rccl_comm_destroy",
    "pwg_broadcast_weights",
    # include/pwg_cnet.h: conv-network executor (MelGAN family)
    "pwg_cnet_abi_version",
    "pwg_cnet_create",
    "pwg_cnet_destroy",
    "pwg_cnet_packed_weight_count",
    "pwg_cnet_pack_weights",
    "pwg_cnet_plan_create",
    "pwg_cnet_plan_destroy",
    "pwg_cnet_plan_image",
    "pwg_cnet_plan_rows",
    "pwg_cnet_plan_workspace_bytes",
    "pwg_cnet_run",
    "pwg_cnet_run_status",
    "pwg_cnet_plan_schedule",
    "pwg_cnet_set_option",
    "pwg_cnet_set_timing",
    "pwg_cnet_timing_collect",
    "pwg_cnet_timing_span",
    "pwg_cnet_release_stream",
    "pwg_rstack_debug_launches",
    "pwg_rstack_debug_probe",
)

PWG_OPT_LAYER_KERNEL = 0
PWG_OPT_WAVES_PER_WG = 1
PWG_OPT_WG_PER_CU = 2
PWG_OPT_FUSE_FIRST_CONV = 3
PWG_OPT_PIPELINE = 4
PWG_OPT_HALF_BLOCKS = 5
PWG_OPT_SYNC = 6
PWG_OPT_SYNC_ABORT = 7
PWG_OPT_SYNC_TIMEOUT = 8


class PwgConfig(ctypes.Structure):
    _fields_ = [
        ("in_channels", ctypes.c_int),
        ("out_channels", ctypes.c_int),
        ("kernel_size", ctypes.c_int),
        ("layers", ctypes.c_int),
        ("stacks", ctypes.c_int),
        ("residual_channels", ctypes.c_int),
        ("gate_channels", ctypes.c_int),
        ("skip_channels", ctypes.c_int),
        ("aux_channels", ctypes.c_int),
        ("aux_context_window", ctypes.c_int),
        ("use_causal_conv", ctypes.c_int),
        ("use_conv_in", ctypes.c_int),
        ("num_scales", ctypes.c_int),
        ("upsample_scales", ctypes.c_int * PWG_MAX_SCALES),
        ("interpolate_mode", ctypes.c_int),
    ]


def _needs_build():
    if not os.path.exists(LIB_PATH):
        return True
    t = os.path.getmtime(LIB_PATH)
    return any(os.path.getmtime(p) > t for p in CSRC + HEADERS)


def _compile_cmd(hipcc, extra_flags):
    return [
        hipcc,
        f"--offload-arch={OFFLOAD_ARCH}",
        "-O3",
        "-std=c++17",
        "-fPIC",
        "-fvisibility=hidden",
        "-mcode-object-version=5",
        # keep the work-queue atomic a plain per-lane op: the optimizer's wave-reduction form
        # waits for the returned value right after issue, which defeats the claim-ahead
        "-mllvm",
        "-amdgpu-atomic-optimizer-strategy=None",
        "-Wall",
    ] + list(extra_flags)


def build(force=False, verbose=False, extra_flags=(), out_path=None, jobs=None, link_flags=()):
    """Compile the HIP kernels + C-ABI into parallelwavegan_amd/lib/libpwg_hip.so (gfx950): one
    hipcc -c per source in parallel (objects under build/<variant>/, rebuilt when a source or
    header is newer), then one link. extra_flags/out_path build A/B measurement variants (e.g.
    -DPWG_STORE_SC1=0) elsewhere."""
    from concurrent.futures import ThreadPoolExecutor

    target = out_path or LIB_PATH
    if not force and out_path is None and (os.environ.get("PWG_NO_BUILD") == "1" or not _needs_build()):
        return LIB_PATH
    os.makedirs(os.path.dirname(target), exist_ok=True)
    hipcc = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
    variant = os.path.splitext(os.path.basename(target))[0]
    objdir = os.path.join(REPO_DIR, "build", variant)
    os.makedirs(objdir, exist_ok=True)
    base = _compile_cmd(hipcc, extra_flags)
    stamp = os.path.join(objdir, "flags.txt")
    flags_txt = " ".join(base)
    stale_flags = not os.path.exists(stamp) or open(stamp).read() != flags_txt
    newest_header = max(os.path.getmtime(h) for h in HEADERS)

    def compile_one(src):
        obj = os.path.join(objdir, os.path.basename(src) + ".o")
        if (not force and not stale_flags and os.path.exists(obj)
                and os.path.getmtime(obj) >= max(os.path.getmtime(src), newest_header)):
            return obj, ""
        tmp = obj + ".tmp.%d" % os.getpid()
        cmd = base + ["-c", "-o", tmp, src]
        res = subprocess.run(cmd, capture_output=True, text=True)
        if res.returncode != 0:
            raise RuntimeError("hipcc failed:\n" + " ".join(cmd) + "\n" + res.stdout + res.stderr)
        os.replace(tmp, obj)
        return obj, res.stdout + res.stderr

    n = jobs or min(len(CSRC), max(1, int(os.environ.get("MAX_JOBS", os.cpu_count() or 1))))
    with ThreadPoolExecutor(max_workers=n) as ex:
        results = list(ex.map(compile_one, CSRC))
    with open(stamp, "w") as f:
        f.write(flags_txt)
    tmp = target + ".tmp.%d" % os.getpid()
    cmd = ([hipcc, f"--offload-arch={OFFLOAD_ARCH}", "-shared", "-fPIC", "-o", tmp] + [o for o, _ in results]
           + list(link_flags) + ["-ldl"])
    res = subprocess.run(cmd, capture_output=True, text=True)
    if res.returncode != 0:
        raise RuntimeError("hipcc link failed:\n" + " ".join(cmd) + "\n" + res.stdout + res.stderr)
    if verbose:
        for _, log in results:
            if log:
                print(log)
    os.replace(tmp, target)
    return target


# Host-side sanitizer build: the C-ABI's host code (config checks, weight
# packing, PWG and conv-network plan builders) under AddressSanitizer + UndefinedBehaviorSanitizer,
# with every uninitialised automatic variable filled with a 0xAA pattern (a field that is never
# assigned then holds a large, deterministic garbage value instead of whatever the stack held,
# which is how an uninitialised OpPhase field once produced a garbage block list and a GPU fault).
# Device code is built unoptimised (-O0: 1 min instead of 3; it never runs) and unsanitised (each
# -fsanitize= only after -Xarch_host): this library is for the host-only tests in this container
# (tests/test_host_sanitized.py), never for a GPU run.
SANITIZE_FLAGS = ["-O1", "-g", "-Xarch_device", "-O0"] + [f for x in ("-fsanitize=address", "-fsanitize=undefined", "-fno-omit-frame-pointer",
                                               "-ftrivial-auto-var-init=pattern") for f in ("-Xarch_host", x)]
SANITIZE_LINK = ["-Xarch_host", "-fsanitize=address", "-Xarch_host", "-fsanitize=undefined", "-shared-libsan"]
SANITIZED_LIB_PATH = os.path.join(REPO_DIR, "build", "sanitized", "libpwg_hip_asan.so")


SANITIZED_SOURCES = ("pwg_capi.hip", "pwg_cnet.hip")  # the host plan builders; the others are launchers


def build_host_sanitized(force=False):
    """Build SANITIZED_LIB_PATH: pwg_capi.hip and pwg_cnet.hip (config checks, packing, plan
    builders) compiled with SANITIZE_FLAGS, linked with the product build's objects of the other
    sources (kernels and their launchers; build() first). Returns the library path."""
    from concurrent.futures import ThreadPoolExecutor

    build()
    objdir = os.path.dirname(SANITIZED_LIB_PATH)
    os.makedirs(objdir, exist_ok=True)
    hipcc = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
    base = _compile_cmd(hipcc, SANITIZE_FLAGS)
    newest = max(os.path.getmtime(f) for f in CSRC + HEADERS)
    if not force and os.path.exists(SANITIZED_LIB_PATH) and os.path.getmtime(SANITIZED_LIB_PATH) >= newest:
        return SANITIZED_LIB_PATH

    def compile_one(src):
        obj = os.path.join(objdir, os.path.basename(src) + ".o")
        res = subprocess.run(base + ["-c", "-o", obj, src], capture_output=True, text=True)
        if res.returncode != 0:
            raise RuntimeError("hipcc (sanitized) failed:\n" + res.stdout + res.stderr)
        return obj

    srcs = [c for c in CSRC if os.path.basename(c) in SANITIZED_SOURCES]
    with ThreadPoolExecutor(max_workers=len(srcs)) as ex:
        objs = list(ex.map(compile_one, srcs))
    product = os.path.join(REPO_DIR, "build", os.path.splitext(os.path.basename(LIB_PATH))[0])
    objs += [os.path.join(product, os.path.basename(c) + ".o") for c in CSRC if os.path.basename(c) not in SANITIZED_SOURCES]
    cmd = ([hipcc, f"--offload-arch={OFFLOAD_ARCH}", "-shared", "-fPIC", "-o", SANITIZED_LIB_PATH] + objs
           + SANITIZE_LINK + ["-ldl"])
    res = subprocess.run(cmd, capture_output=True, text=True)
    if res.returncode != 0:
        raise RuntimeError("hipcc link (sanitized) failed:\n" + res.stdout + res.stderr)
    return SANITIZED_LIB_PATH


def sanitizer_runtime():
    """The ASan runtime to LD_PRELOAD into an uninstrumented python (None if absent)."""
    import glob

    hits = sorted(glob.glob("/opt/rocm/lib/llvm/lib/clang/*/lib/linux/libclang_rt.asan-x86_64.so"))
    return hits[-1] if hits else None


_lib = None
_lock = threading.Lock()


def load():
    """Load the built library (raises if it is missing: no CPU fallback exists)."""
    global _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(
                f"{LIB_PATH} is missing: build it with `python -c 'import __graft_entry__ as g; g.build()'`"
            )
        import torch  # noqa: F401  (bind our NEEDED libamdhip64.so.7 to torch's HIP runtime)

        lib = ctypes.CDLL(LIB_PATH)
        vp = ctypes.c_void_p
        ll = ctypes.c_longlong
        lib.pwg_abi_version.restype = ctypes.c_int
        lib.pwg_last_error.restype = ctypes.c_char_p
        lib.pwg_create.argtypes = [ctypes.POINTER(PwgConfig), ctypes.c_int, ctypes.POINTER(vp)]
        lib.pwg_destroy.argtypes = [vp]
        lib.pwg_destroy.restype = None
        for name in ("pwg_receptive_field_size", "pwg_upsample_factor", "pwg_ref_weight_count",
                     "pwg_packed_weight_count"):
            getattr(lib, name).argtypes = [vp]
            getattr(lib, name).restype = ll
        lib.pwg_pack_weights.argtypes = [vp, vp, vp]
        lib.pwg_plan_create.argtypes = [vp, ctypes.c_int, ctypes.POINTER(ll), ctypes.c_int, ctypes.POINTER(vp)]
        lib.pwg_plan_destroy.argtypes = [vp]
        lib.pwg_plan_destroy.restype = None
        for name in ("pwg_plan_total_samples", "pwg_plan_padded_samples", "pwg_plan_workspace_bytes"):
            getattr(lib, name).argtypes = [vp]
            getattr(lib, name).restype = ll
        lib.pwg_run.argtypes = [vp, vp, vp, vp, vp, vp, vp, vp, vp]
        lib.pwg_run_status.argtypes = [vp, vp, vp]
        lib.pwg_graph_create.argtypes = [vp] * 9 + [ctypes.POINTER(vp)]
        lib.pwg_graph_launch.argtypes = [vp, vp]
        lib.pwg_graph_destroy.argtypes = [vp]
        lib.pwg_graph_destroy.restype = None
        lib.pwg_get_option.argtypes = [vp, ctypes.c_int, ctypes.POINTER(ll)]
        lib.pwg_rccl_unique_id.argtypes = [vp]
        lib.pwg_rccl_comm_create.argtypes = [ctypes.c_int, vp, ctypes.c_int, ctypes.c_int, ctypes.POINTER(vp)]
        lib.pwg_rccl_comm_destroy.argtypes = [vp]
        lib.pwg_broadcast_weights.argtypes = [vp, vp, ctypes.c_int, vp, vp]
        lib.pwg_set_timing.argtypes = [vp, ctypes.c_int]
        lib.pwg_release_stream.argtypes = [vp, vp]
        lib.pwg_set_option.argtypes = [vp, ctypes.c_int, ctypes.c_longlong]
        lib.pwg_timing_collect.argtypes = [vp, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ll)]
        lib.pwg_timing_span.argtypes = [vp, ctypes.POINTER(ctypes.c_double)]
        if lib.pwg_abi_version() != 2:
            raise RuntimeError("libpwg_hip ABI version mismatch")
        _lib = lib
        return lib


class RangeError(ArithmeticError):
    """PWG_ERR_RANGE: a value left the fp16 pair range of the split-f16 kernels."""


class RerunError(RuntimeError):
    """PWG_ERR_RERUN: a grid-synchronised or layer-pipelined forward did not complete (the GPU was
    shared, or a bounded wait gave up); its output is invalid and the run must be redone on the
    per-layer launches."""


_ERRORS = {
    PWG_ERR_RANGE: RangeError,
    PWG_ERR_RERUN: RerunError,
    PWG_ERR_INVALID: ValueError,
    PWG_ERR_ASSERT: AssertionError,
    PWG_ERR_HIP: RuntimeError,
    PWG_ERR_UNSUPPORTED: NotImplementedError,
}


def check(rc):
    """Raise the reference's exception type for a non-zero status (include/pwg.h)."""
    if rc == PWG_OK:
        return
    msg = load().pwg_last_error().decode(errors="replace")
    raise _ERRORS.get(rc, RuntimeError)(msg)
