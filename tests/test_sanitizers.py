"""Sanitizer runs of the native host runtime ("build the C++ runtime with
-fsanitize=thread in a CI job for the host side").

The shared-memory control-plane collectives are exercised by a multi-threaded stress driver whose
ranks share one mapping, under ThreadSanitizer and under AddressSanitizer + UBSan. A report makes
the driver exit non-zero (TSAN: 66) and the test fail with the report.
"""

import shutil
import subprocess

import pytest

from myfyp_amd.ops.build import build_sanitized


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs the host C++ compiler")
@pytest.mark.parametrize("sanitize,iters", [("thread", 1500), ("address,undefined", 3000)])
def test_shm_collective_under_sanitizer(sanitize, iters):
    exe = build_sanitized(sanitize)
    env = {"TSAN_OPTIONS": "halt_on_error=1 second_deadlock_stack=1", "ASAN_OPTIONS": "detect_leaks=1:halt_on_error=1", "UBSAN_OPTIONS": "halt_on_error=1:print_stacktrace=1"}
    res = subprocess.run([exe, "4", str(iters)], capture_output=True, text=True, timeout=240, env=env)
    assert res.returncode == 0, res.stdout[-2000:] + res.stderr[-6000:]
    assert "OK world=4" in res.stdout and "WARNING" not in res.stderr, res.stderr[-4000:]
