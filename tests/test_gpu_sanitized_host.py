"""GPU: libdm with ASan + UBSan on its host code (tests/native/api_san, built
in-tree on the CPU: `make -C tests/native api_san`), every product call of the
C-ABI on cuda:0 — integrate (host and async inputs), frontiers (sync,
pipelined, dense outputs), row bands with halos, device export + merge
(checked against the single map), checkpoint, LD06 conversion, the atomic
probe.  GPU-side sanitizers are not available on this pool; this covers the
host code that moves every byte in and out."""
import os
import subprocess

import pytest

pytestmark = pytest.mark.gpu
EXE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "native", "api_san")


def test_c_abi_product_calls_under_host_asan():
    if not os.path.exists(EXE):
        pytest.fail("tests/native/api_san not built (make -C tests/native api_san)")
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=0", UBSAN_OPTIONS="print_stacktrace=1")
    r = subprocess.run([EXE, "--gpu"], capture_output=True, text=True, timeout=240, env=env)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert "product calls ok" in r.stdout and "ERROR: AddressSanitizer" not in r.stderr
