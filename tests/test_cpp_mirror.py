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


@pytest.mark.gpu
def test_c1_native_round_trip():
    """BASELINE config C1 through the C++ mirror: upload + download of a
    ragged word count over two in-process parties (JSON open between party
    threads), secrets back bit-exact (tools/c1_native.cpp)."""
    import build_native
    import json
    r = subprocess.run([build_native.build_c1_native(), "1001", "2"], capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    line = json.loads(r.stdout.strip().splitlines()[-1])
    assert line["bit_exact_round_trip"] is True and line["words"] == 1001


@pytest.mark.gpu
def test_c1_native_three_parties_shared_context():
    """The same flow with three parties (two partner texts per open) whose
    threads all call into one context at once."""
    import build_native
    import json
    r = subprocess.run([build_native.build_c1_native(), "777", "2", "shared", "3"], capture_output=True,
                       text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    line = json.loads(r.stdout.strip().splitlines()[-1])
    assert line["bit_exact_round_trip"] is True and line["parties"] == 3 and line["contexts"] == 1
