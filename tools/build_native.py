"""Build libamphora_hip.so (HIP kernels + C ABI) in-tree for gfx950.

    python tools/build_native.py [--force]     # or __graft_entry__.build()

hipcc cross-compiles without a GPU.  The .so lands next to this file so it
travels with the repo snapshot to the GPU box (it is git-ignored).
"""
from __future__ import annotations

import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HERE = os.path.join(ROOT, "amphora_amd")
CSRC = os.path.join(HERE, "csrc")
LIB = os.path.join(HERE, "libamphora_hip.so")
SOURCES = [os.path.join(CSRC, f) for f in ("kernels.hip", "codec.hip", "exchange.hip", "capi.hip")]
DEPS = SOURCES + [os.path.join(CSRC, f) for f in ("field.hpp", "kernels.hpp", "host_stream.hpp")] + [
    os.path.join(ROOT, "include", "amphora.h")]
ARCH = os.environ.get("AMPH_OFFLOAD_ARCH", "gfx950")


def hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", "hipcc"):
        if cand and (os.path.isabs(cand) and os.path.exists(cand) or not os.path.isabs(cand)):
            return cand
    return "hipcc"


def up_to_date() -> bool:
    if not os.path.exists(LIB):
        return False
    t = os.path.getmtime(LIB)
    return all(os.path.getmtime(d) <= t for d in DEPS)


def build(force: bool = False, verbose: bool = False) -> str:
    if not force and up_to_date():
        return LIB
    cmd = [hipcc(), "--offload-arch=%s" % ARCH, "-O3", "-std=c++17", "-fPIC", "-shared",
           "-mcode-object-version=5", "-Wall", "-I" + os.path.join(ROOT, "include"),
           "-Wl,-rpath,/opt/rocm/lib", "-o", LIB + ".tmp"] + SOURCES
    if verbose:
        print(" ".join(cmd))
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        sys.stderr.write(r.stdout + r.stderr)
        raise RuntimeError("hipcc failed building libamphora_hip.so")
    os.replace(LIB + ".tmp", LIB)
    return LIB


CPP_TEST_SRC = os.path.join(ROOT, "tests", "cpp", "mirror_test.cpp")
CPP_TEST_BIN = os.path.join(ROOT, "tests", "cpp", "mirror_test")


def build_cpp_test(force: bool = False) -> str:
    """The C++ host-mirror test program (include/amphora.hpp) against the .so."""
    deps = [CPP_TEST_SRC, os.path.join(ROOT, "include", "amphora.hpp"), LIB]
    if not force and os.path.exists(CPP_TEST_BIN) and all(
            os.path.getmtime(d) <= os.path.getmtime(CPP_TEST_BIN) for d in deps):
        return CPP_TEST_BIN
    cmd = ["g++", "-std=c++17", "-O2", "-Wall", "-I" + os.path.join(ROOT, "include"), CPP_TEST_SRC,
           "-L" + HERE, "-lamphora_hip", "-Wl,-rpath,$ORIGIN/../../amphora_amd", "-o", CPP_TEST_BIN]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        sys.stderr.write(r.stdout + r.stderr)
        raise RuntimeError("g++ failed building the C++ mirror test")
    return CPP_TEST_BIN


C1_SRC = os.path.join(ROOT, "tools", "c1_native.cpp")
C1_BIN = os.path.join(ROOT, "tools", "c1_native")


def build_c1_native(force: bool = False) -> str:
    """BASELINE config C1 through the C++ mirror (tools/c1_native.cpp)."""
    deps = [C1_SRC, os.path.join(ROOT, "include", "amphora.hpp"), LIB]
    if not force and os.path.exists(C1_BIN) and all(
            os.path.getmtime(d) <= os.path.getmtime(C1_BIN) for d in deps):
        return C1_BIN
    cmd = ["g++", "-std=c++17", "-O2", "-Wall", "-pthread", "-I" + os.path.join(ROOT, "include"), C1_SRC,
           "-L" + HERE, "-lamphora_hip", "-Wl,-rpath,$ORIGIN/../amphora_amd", "-o", C1_BIN]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        sys.stderr.write(r.stdout + r.stderr)
        raise RuntimeError("g++ failed building tools/c1_native")
    return C1_BIN


SAN_DIR = os.path.join(ROOT, "build", "sanitize")
SAN_FLAGS = ["-fsanitize=address", "-fsanitize=undefined", "-fno-sanitize-recover=all",
             "-fno-omit-frame-pointer"]


def build_sanitized(force: bool = False) -> dict:
    """Host-code ASan/UBSan builds: the library with its
    host side instrumented (device code untouched -- GPU ASan is not
    available), the C++ mirror test linked against it, and a driver of the C
    oracle.  Output in build/sanitize/ (git-ignored)."""
    os.makedirs(SAN_DIR, exist_ok=True)
    lib = os.path.join(SAN_DIR, "libamphora_hip.so")
    mirror = os.path.join(SAN_DIR, "mirror_test")
    orc = os.path.join(SAN_DIR, "oracle_sanitize")
    orc_src = os.path.join(ROOT, "tests", "cpp", "oracle_sanitize.c")
    jobs = [
        (lib, DEPS, [hipcc(), "--offload-arch=%s" % ARCH, "-O1", "-g", "-std=c++17", "-fPIC", "-shared",
                     "-mcode-object-version=5", "-I" + os.path.join(ROOT, "include"),
                     "-Wl,-rpath,/opt/rocm/lib", "-o", lib] + SOURCES
         + [x for f in SAN_FLAGS for x in ("-Xarch_host", f)]),
        (mirror, [CPP_TEST_SRC, os.path.join(ROOT, "include", "amphora.hpp"), lib],
         ["/opt/rocm/llvm/bin/clang++", "-std=c++17", "-O1", "-g", "-I" + os.path.join(ROOT, "include"),
          CPP_TEST_SRC, "-L" + SAN_DIR, "-lamphora_hip", "-Wl,-rpath,$ORIGIN", "-o", mirror] + SAN_FLAGS),
        (orc, [orc_src, os.path.join(ROOT, "oracle", "amphora_oracle.c")],
         ["gcc", "-O1", "-g", "-fopenmp", "-Wall", "-Wextra", orc_src, "-o", orc] + SAN_FLAGS),
    ]
    for out, deps, cmd in jobs:
        if not force and os.path.exists(out) and all(os.path.getmtime(d) <= os.path.getmtime(out) for d in deps):
            continue
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            sys.stderr.write(r.stdout + r.stderr)
            raise RuntimeError("sanitizer build failed: %s" % out)
    return {"lib": lib, "mirror": mirror, "oracle": orc}


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
    print(build_cpp_test(force="--force" in sys.argv))
