"""The C++ host mirror (include/amphora.hpp) run as a program: host-only
checks on CPU, the reference KATs + a round trip on the GPU."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))


def _bin():
    import build_native
    return build_native.build_cpp_test()


def test_cpp_mirror_cpu():
    r = subprocess.run([_bin(), "cpu"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr


@pytest.mark.gpu
def test_cpp_mirror_gpu():
    r = subprocess.run([_bin(), "gpu"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
