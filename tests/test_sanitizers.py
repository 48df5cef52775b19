"""CPU: ASan + UBSan builds.

* the kernel emulation (tests/native/emulate.cpp, from the kernels' geometry
  header csrc/dm_ray.h) and the C oracle, run against each other on seeded
  batches (ragged maps, a band, chunked beams, NaN / 0 / inf ranges) plus an
  oracle frontier pass with halos;
* libdm's host code built with -Xarch_host -fsanitize=address,undefined,
  driven through its C-ABI by a C program (tests/native/api_san.c): here the
  validation and error paths (no GPU); the product calls run on the GPU box
  (tests/test_gpu_sanitized_host.py)."""
import os
import subprocess

import pytest

NATIVE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "native")
ENV = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0", UBSAN_OPTIONS="print_stacktrace=1")


def _build(target):
    subprocess.run(["make", "-s", "-C", NATIVE, target], check=True, timeout=600)


def test_emulation_and_oracle_under_asan_ubsan():
    _build("sanitize_main")
    r = subprocess.run([os.path.join(NATIVE, "sanitize_main")], capture_output=True, text=True, timeout=600,
                       env=ENV)
    assert r.returncode == 0, r.stdout + r.stderr
    assert r.stdout.count(": ok,") == 5 and "ERROR" not in r.stderr


def test_c_abi_error_paths_under_host_asan():
    from conftest import gpu_available

    _build("api_san")
    env = dict(ENV, ASAN_OPTIONS="detect_leaks=0")  # the HIP runtime keeps its allocations
    r = subprocess.run([os.path.join(NATIVE, "api_san")], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "api_san: ok" in r.stdout and "ERROR" not in r.stderr
    if gpu_available():
        pytest.skip("product calls are the GPU test's")
