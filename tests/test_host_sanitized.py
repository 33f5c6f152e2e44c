"""The C-ABI's host code under AddressSanitizer + UndefinedBehaviorSanitizer.

Round 3's one GPU fault came from host code: an OpPhase field the conv-network plan builder never
assigned (pwg_cnet.hip) gave a garbage column step, the block list pointed outside the buffers and
a kernel read an illegal address. Nothing on the CPU side would have caught it. Here the host
plan builders (pwg_capi.hip: config checks, weight packing, PWG plans; pwg_cnet.hip: program
lowering checks, fragment packing, fusion and staging decisions) are rebuilt with ASan, UBSan and
pattern-initialised automatic variables (_lib.build_host_sanitized), and the host-only test files
run against that library in a child python with the ASan runtime preloaded. Any sanitizer report
fails the test. CPU only; the sanitized library never goes to a GPU box."""

import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HOST_TESTS = ["tests/test_cnet_host.py", "tests/test_abi.py"]


def test_host_code_is_clean_under_asan_and_ubsan(built_lib):
    from parallelwavegan_amd import _lib

    rt = _lib.sanitizer_runtime()
    if rt is None:
        pytest.skip("no ASan runtime in this image")
    lib = _lib.build_host_sanitized()
    env = dict(os.environ, LD_PRELOAD=rt, PWG_NO_BUILD="1", PWG_LIB_PATH=lib,
               ASAN_OPTIONS="detect_leaks=0:halt_on_error=1:abort_on_error=0",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
    r = subprocess.run([sys.executable, "-m", "pytest", "-x", "-q", "-m", "not gpu", "-p", "no:cacheprovider"]
                       + HOST_TESTS, cwd=REPO, env=env, capture_output=True, text=True, timeout=900)
    log = r.stdout + r.stderr
    assert "AddressSanitizer" not in log and "runtime error:" not in log, log[-6000:]
    assert r.returncode == 0, log[-6000:]
    assert " passed" in log
