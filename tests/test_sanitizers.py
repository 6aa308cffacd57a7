"""Host code under AddressSanitizer + UndefinedBehaviorSanitizer (SURVEY.md
section 5: the reference relies on the JVM; our host side is C/C++, so it runs
instrumented).  Device code is not instrumented -- GPU ASan is not available.

* the C oracle, driven over 1..4 parties with faults and non-canonical words;
* libamphora_hip.so's host side via the C++ mirror test: CPU-only checks here,
  the full KAT + GPU round trip under -m gpu.
"""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))

# HIP's runtime is not instrumented and keeps allocations until exit
_ENV = dict(os.environ, ASAN_OPTIONS="detect_leaks=0:abort_on_error=0",
            UBSAN_OPTIONS="print_stacktrace=1")


@pytest.fixture(scope="module")
def san():
    import build_native
    return build_native.build_sanitized()


def _run(args, timeout, env=_ENV):
    r = subprocess.run(args, capture_output=True, text=True, timeout=timeout, env=env)
    out = r.stdout + r.stderr
    assert r.returncode == 0 and "ERROR: AddressSanitizer" not in out and "runtime error" not in out, out
    return out


def test_oracle_sanitized(san):
    env = dict(_ENV, ASAN_OPTIONS="detect_leaks=1")  # pure C: leaks are ours
    assert "clean" in _run([san["oracle"]], 300, env)


def test_mirror_cpu_sanitized(san):
    assert "0 failures" in _run([san["mirror"], "cpu"], 120)


@pytest.mark.gpu
def test_mirror_gpu_sanitized(san):
    assert "0 failures" in _run([san["mirror"], "gpu"], 600)
